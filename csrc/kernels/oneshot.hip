// One-shot collectives over peer (HIP IPC) pointers for latency-bound messages — SURVEY §5.8
// design item 5: the per-forward BN buffer broadcast (C4, ~38-212 KB) and tiny gradient buckets,
// where a ring all-reduce's 2(N-1) dependent hops cost more than the bytes.
//
// Every rank owns one workspace (hipMalloc, exported with hipIpcGetMemHandle, mapped by every
// peer):   [0, 2 KB)  flags[rank r][block b]: the epoch peer r's block b last published
//          [2 KB]     error words: {1 + the peer a bounded wait gave up on, that call's epoch}
//          [3 KB)     ctr[block b]: this rank's epoch counter of block b (local only)
//          [4 KB, ..) two data slots of `cap` bytes (epoch parity)
// The grid is FIXED for a communicator (nblocks, from its slot size): every call runs every
// block, blocks whose slice is empty still publish and wait, so all per-block epochs advance in
// lock-step and block b's slot parity always names the same call on every rank.  (With a grid
// sized per message, a block that sat out a small call would reuse a parity a slower peer was
// still reading from the previous call's block b — advisor finding, round 3.)
// One call, per block b over its slice of the message:
//   1. e = ctr[b] + 1; stage the slice into MY slot[e & 1] (broadcast: the source only);
//   2. release at system scope (every wave drains its stores and writes its L2 lines back), then
//      store e into flags[me][b] of every peer — system-scope atomic stores over xGMI;
//   3. one lane per peer polls its flag in MY workspace (relaxed, system scope, s_sleep between
//      polls, bounded by an s_memrealtime deadline), then a system-scope acquire (drops stale
//      L1/L2 lines) and a barrier.  A wait that gives up records {1 + peer, epoch} in the error
//      words and the block SKIPS the data phase (it never consumes a slot it was not handed):
//      the output is left as it was and the host side turns the error words into an exception
//      (parallel/oneshot.py OneShotComm.check, polled by DDP without a host sync);
//   4. read every rank's slot[e & 1] slice straight over xGMI and sum it in rank order (the same
//      order on every rank: bit-identical results), or copy the source's slice;
//   5. ctr[b] = e.
// Two slots make a single publish per call enough: a rank can only start call N+2 (same slot as
// call N) after every peer published call N+1, which each does only after its call-N kernel
// finished reading (in-stream order).  Epochs live in device memory, so a captured hipGraph
// replays correctly; flags only grow, so a peer that is one call ahead (flag e+1) still counts.
#include "common.hpp"

namespace mipipe {

constexpr int kOsMaxRanks = 8;
constexpr int kOsMaxBlocks = 64;
constexpr int kOsFlagOff = 0;
constexpr int kOsErrOff = 2048;
constexpr int kOsCtrOff = 3072;
constexpr int kOsDataOff = 4096;

struct OsPeers {
  char* base[kOsMaxRanks];
};

typedef __attribute__((address_space(1))) unsigned int gu32_t;

// a word of a workspace as a GLOBAL pointer (atomics on global, never flat)
__device__ __forceinline__ gu32_t* g32(char* p) { return (gu32_t*)(p); }

// timeout_ticks: the bounded wait, in ticks of the 100 MHz s_memrealtime clock
template <bool REDUCE>
__global__ __launch_bounds__(256) void oneshot_kernel(OsPeers P, const uint4* in, uint4* out,
                                                      long nvec, int rank, int world, int src,
                                                      float scale, long cap,
                                                      unsigned long long timeout_ticks) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  char* mine = P.base[rank];
  unsigned int* ctr = reinterpret_cast<unsigned int*>(mine + kOsCtrOff) + b;
  __shared__ unsigned int s_e, s_fail;
  if (tid == 0) {
    s_e = *ctr + 1;  // only this block ever touches ctr[b]
    s_fail = 0;
  }
  __syncthreads();
  const unsigned int e = s_e;
  const long slot_off = kOsDataOff + (long)(e & 1u) * cap;
  const long per = (nvec + nb - 1) / nb;
  const long lo = (long)b * per;
  const long hi = lo + per < nvec ? lo + per : nvec;
  if (REDUCE || rank == src) {
    uint4* dst = reinterpret_cast<uint4*>(mine + slot_off);
    for (long i = lo + tid; i < hi; i += 256) dst[i] = in[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every wave: its stores drained + written back
  __syncthreads();
  if (tid < world && tid != rank) {
    gu32_t* f = g32(P.base[tid] + kOsFlagOff) + rank * kOsMaxBlocks + b;
    __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world && tid != rank) {
    gu32_t* f = g32(mine + kOsFlagOff) + tid * kOsMaxBlocks + b;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(g32(mine + kOsErrOff) + 1, e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(g32(mine + kOsErrOff), 1u + (unsigned)tid,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_fail = 1;  // benign race: every writer stores 1
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // drop stale lines before reading peer slots
  __syncthreads();
  if (s_fail) return;  // a peer never published this call: never read its (stale) slot
  if (REDUCE) {
    for (long i = lo + tid; i < hi; i += 256) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < world; ++r) {  // rank order: identical sums on every rank
        const float4 v = reinterpret_cast<const float4*>(P.base[r] + slot_off)[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
      reinterpret_cast<float4*>(out)[i] = acc;
    }
  } else {
    const uint4* s = reinterpret_cast<const uint4*>(P.base[src] + slot_off);
    for (long i = lo + tid; i < hi; i += 256) out[i] = s[i];
  }
  __syncthreads();
  if (tid == 0) *ctr = e;
}

int oneshot_blocks(long cap) {
  long nb = cap / (64 << 10);  // a full slot: >= 64 KB per block
  return (int)(nb < 1 ? 1 : (nb > kOsMaxBlocks ? kOsMaxBlocks : nb));
}

// nbytes % 16 == 0, nbytes <= cap; fp32 sum (times scale) or a byte broadcast from `src`.
// nblocks: the communicator's fixed grid (oneshot_blocks(cap)), the same for every call.
void oneshot_launch(char* const* bases, int rank, int world, const void* in, void* out,
                    long nbytes, bool reduce, int src, float scale, long cap, int nblocks,
                    double timeout_s, hipStream_t st) {
  OsPeers P;
  for (int r = 0; r < kOsMaxRanks; ++r) P.base[r] = r < world ? bases[r] : nullptr;
  const long nvec = nbytes / 16;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);
  const int nb = nblocks < 1 ? 1 : (nblocks > kOsMaxBlocks ? kOsMaxBlocks : nblocks);
  if (reduce)
    hipLaunchKernelGGL(oneshot_kernel<true>, dim3((unsigned)nb), dim3(256), 0, st, P,
                       (const uint4*)in, (uint4*)out, nvec, rank, world, src, scale, cap, ticks);
  else
    hipLaunchKernelGGL(oneshot_kernel<false>, dim3((unsigned)nb), dim3(256), 0, st, P,
                       (const uint4*)in, (uint4*)out, nvec, rank, world, src, scale, cap, ticks);
}

}  // namespace mipipe
