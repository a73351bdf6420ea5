// Probe of ds_pk_add_bf16 semantics on the box: lanes add bf16 values into zeroed LDS words.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  __shared__ unsigned s[64];
  s[threadIdx.x] = 0;
  __syncthreads();
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned*)(s + (threadIdx.x & 7));
  // lane t adds 1.0 (bf16 0x3f80) into the low half if t < 32, 2.0 (0x4000) into the high half otherwise
  const unsigned v = threadIdx.x < 32 ? 0x3f80u : 0x40000000u;
  asm volatile("ds_pk_add_bf16 %0, %1" ::"v"(a), "v"(v) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  out[threadIdx.x] = s[threadIdx.x];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[64];
  hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i) printf("word %d = 0x%08x\n", i, h[i]);
  printf("expected: 0x%08x (lo 4 x 1.0 = 4.0 -> 0x4080, hi 4 x 2.0 = 8.0 -> 0x4100)\n", 0x41004080u);
  return 0;
}
