// Host-side launch API of mipipe's gfx950 kernels (raw pointers + shapes + stream).
// Bound to Python in csrc/bindings.cpp.  Every launcher is graph-capture safe: no
// allocation, no synchronisation (cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mipipe {

// ---- convolution (NHWC activations, weights [Co][KH][KW][Ci]) --------------------------------
struct ConvShape {
  int N, H, W, Ci;   // input
  int Co, KH, KW, stride, pad;
  int Ho, Wo;        // output
  int stride_w = 0;  // horizontal stride when != stride (0: same); fwd / wgrad only
  int pad_w = -1;    // horizontal padding when >= 0 (else pad): Inception 1x7 / 7x1 convs
  bool f32 = false;  // fp32 activations/weights (split-bf16 MFMA main loop) instead of bf16
};

// BatchNorm statistics are accumulated with fp32 atomics into kStatReplicas replica rows of a
// [R][C] slab (spreads contention); the consumer (bn_finalize / bwd finalize) reduces the R rows
// and ZEROES the slab again, so a persistent zero-initialised slab can be reused every step.
// The slab LAYOUT always has kStatReplicas rows; kernels write rows blockIdx % g_stat_rows
// (<= kStatReplicas; the rest stay zero), so the spread is tunable at runtime for sweeps.
// Measured (profiles/r1_stat_rows_probe.jsonl): 64 rows save <= 8 % on the widest statistics
// epilogues but make the per-channel finalize / collect kernels (one thread per channel summing
// every row) 10-35x slower — a net ResNet-50 loss of 30 % — so the layout stays at 16.
constexpr int kStatReplicas = 16;
extern int g_stat_rows;
// Split-K sizing for the atomically-accumulated weight-gradient GEMMs: splits are chosen so
// that tiles * splits ~= this many workgroups (tunable at runtime for sweeps).
extern int g_splitk_target;
// Dense (1x1) conv fwd/dgrad with reduction K <= this use the single-LDS-stage kernels.
extern int g_ns1_max_k;
extern int g_ns1_max_k_gather;  // same for the gathered (im2col / strided dgrad) convs
// Deterministic mode (reference task.py:25-26 cudnn.deterministic): every float reduction runs
// in a fixed order — no float atomics (det.hip); set from Python (mipipe.ops.set_deterministic).
extern int g_deterministic;
// out[c] (+)= sum over P rows of in[p][c] (and in1 -> out1), fixed order.  The partial rows are
// SCRATCH: long sums (P > 256) are done in two levels, the first writing chunk sums in place.
void det_sum_rows(float* in0, float* in1, int P, int C, float* out0, float* out1,
                  bool accumulate, hipStream_t st, float* in2 = nullptr, float* out2 = nullptr);
// First level of a long fixed-order column sum: rows [k*kDetChunkRows, (k+1)*kDetChunkRows) of
// each array summed in place into row k*kDetChunkRows (arrays in order: in2 only with in1).
// Returns the number of chunk rows (every kDetChunkRows-th row) the second level sums.
constexpr int kDetChunkRows = 64;
int det_chunk_sums(float* in0, float* in1, float* in2, int P, int C, hipStream_t st);
// bn_bwd_collect of [2|3][P][C] deterministic partial rows (det_sum_rows' order; rows scratch)
void bn_bwd_collect_rows(float* rows, int P, int C, bool two, float* out_g, float* out_gx,
                         float* out_gx2, float* dgamma, float* dbeta, float* dgamma2,
                         float* dbeta2, const float* gx_div, hipStream_t st);
// out[i] += sum_s ws[s][i] over splits in order.
void splitk_sum(const float* ws, int splits, long n, float* out, hipStream_t st);
// out[m][n] (bf16, row pitch ldc) = sum_s ws[s][m][n] + bias[n] (bias may be null); N % 8 == 0
void splitk_sum_bf16(const float* ws, int splits, long M, int N, const float* bias, void* out,
                     long ldc, hipStream_t st, const void* addend = nullptr);
// the same with an fp32 output (the reference-precision path)
void splitk_sum_f32out(const float* ws, int splits, long M, int N, const float* bias, float* out,
                       long ldc, hipStream_t st, const float* addend = nullptr);
int conv_fwd_stat_rows(const ConvShape& s);
// st_sum / st_sq: zeroed [kStatReplicas][Co] slabs (accumulated into)
// bias / relu: optional per-channel bias and ReLU in the epilogue (convs without BN: VGG, AlexNet)
// cfg: tile config id (conv_common.hpp table; < 0 = heuristic default)
constexpr int kConvTileConfigs = 15;
//  det_rows > 0 (deterministic mode): st_sum / st_sq are [det_rows][Co] partial slabs, one row
//  per M-tile (det_rows = conv_fwd_tiles_m(s, cfg)), written without atomics.
// wflip (Ci*KH*KW*Co elements, w's dtype): when dgrad_preflip_ok(s), trailing blocks of the
// launch also write the tap-flipped weight the stride-1 data-grad reads (conv_dgrad's
// `preflipped`) — no flip kernel in the backward.
// split_ws: fp32 workspace of conv_fwd_split_ws_elems(s, cfg) elements when the plan splits K
void conv_fwd(const void* x, const void* w, void* y, float* st_sum, float* st_sq,
              const float* st_shift, const ConvShape& s, hipStream_t st,
              const float* bias = nullptr, bool relu = false, int cfg = -1, int det_rows = 0,
              void* wflip = nullptr, float* split_ws = nullptr,
              const float* in_scale = nullptr, const float* in_bias = nullptr);
constexpr int kConvBnInMaxK = 1024;  // input channels of a folded-BN forward (LDS table)
inline bool conv_is_dense(const ConvShape& s) {  // 1x1, stride 1, no padding
  return s.KH == 1 && s.KW == 1 && s.stride == 1 && s.pad == 0 && s.pad_w <= 0 &&
         (s.stride_w == 0 || s.stride_w == 1);
}
// in_scale / in_bias (bf16 dense 1x1, Ci <= 1024): x holds y of a BatchNorm + ReLU whose apply is
// FOLDED into this conv — the conv consumes relu(y*in_scale + in_bias) (per input channel),
// transformed after each operand fragment's LDS read; the normalised tensor never exists.
// Conv forward / forward-style data-grad PLANS: tile id + kConvSplitPlan * splits.  A split plan
// (splits >= 2) runs the k-steps in `splits` slices (grid.y) into an fp32 workspace and a finish
// launch sums the slices in slice order (deterministic) and runs the regular epilogue — for the
// small-spatial layers whose tiles alone cannot fill 256 CUs (ResNet-18 32x32 layer 3 / 4: 64-128
// tiles of 36 k-steps each).
constexpr int kConvSplitPlan = 16;
inline int conv_plan_tile(int plan) { return plan < 0 ? plan : plan % kConvSplitPlan; }
inline int conv_plan_splits(int plan) { return plan < kConvSplitPlan ? 1 : plan / kConvSplitPlan; }
// (effective splits, k-steps per split) of nk k-steps under a plan's split request
inline void conv_split_geometry(int nk, int req, int* splits, int* kps) {
  if (req <= 1 || nk < 2) {
    *splits = 1;
    *kps = nk;
    return;
  }
  *kps = (nk + req - 1) / req;
  *splits = (nk + *kps - 1) / *kps;
}
long conv_fwd_split_ws_elems(const ConvShape& s, int cfg);
void conv_tile_dims(int cfg, bool f32, int* bm, int* bn);  // block tile of a plan's tile id
long conv_dgrad_split_ws_elems(const ConvShape& s, int cfg);
// The data-grad of s runs as forward-style parity classes over tap-flipped sub-kernels (see
// conv_dgrad_fwd_style; stride <= 2), so a forward launch can produce those weights.
bool dgrad_preflip_ok(const ConvShape& s);
// The flipped sub-kernels in conv_dgrad's workspace layout: class c holds
// wt[off + (ci*taps + a*nkw + b)*Co + co] = w[co][kh0 + S(nkh-1-a)][kw0 + S(nkw-1-b)][ci];
// blocks: one per (64-ci, 64-co, tap), class c's from b0.
struct FlipClass {
  int kh0, kw0, nkh, nkw;
  long off;
  uint32_t b0;
};
struct FlipPlan {
  FlipClass cls[4];
  int ncls = 0, S = 1;
  uint32_t nblk = 0;
};
void dgrad_flip_plan(const ConvShape& s, FlipPlan& p);
int dgrad_fwd_style_mode();  // MIPIPE_DGRAD_FWD (0 off, 1 non-dense, 2 also dense 1x1)
int conv_fwd_tiles_m(const ConvShape& s, int cfg);
// Optional dgrad epilogue fusions:
//  addend: [N*H*W][Ci] (activation dtype) added to dx (the block input's other gradient, e.g. the residual);
//  bn_*:   the conv input was relu(bn(y)) with a single consumer: dx becomes g = dx*[z > 0] and
//          Σg, Σg·x̂ go to rep rows 0/1 ([3][kStatReplicas][Ci] zeroed slab, see bn_bwd_collect).
struct DgradFusion {
  const void* addend = nullptr;
  const void* bn_y = nullptr;
  const float *bn_mean = nullptr, *bn_invstd = nullptr, *bn_scale = nullptr, *bn_bias = nullptr;
  float* bn_rep = nullptr;
  const void* bn_z = nullptr;  // optional stored relu output: mask = z > 0 (residual blocks)
  const uint8_t* bn_mask = nullptr;  // or that mask as bits ([rows][Ci/8] bytes, bit q = chan q)
  // two-branch block output relu(bn(y) + bn2(y2)): Σg·x̂₂ to rep array 2 (bf16, 1x1 convs)
  const void* bn_y2 = nullptr;
  const float *bn_mean2 = nullptr, *bn_invstd2 = nullptr;
  int det_rows = 0;  // deterministic mode: bn_rep is [2][det_rows][Ci] partials, one row per tile
};
// w_flip: a workspace of Co*KH*KW*Ci elements — when given, every stride-parity class with taps
// runs as a stride-1 FORWARD im2col convolution of dy over its tap-flipped sub-kernel (written
// into the workspace by this call); allocate it only when conv_dgrad_fwd_style(s, ...) holds
// preflipped: w_flip already holds the flipped weight (conv_fwd's wflip, dgrad_preflip_ok(s))
// split_ws: conv_dgrad_split_ws_elems(s, cfg) fp32 elements when the plan splits K (the
// forward-style classes only; the other data-grad kernels ignore the split)
void conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, hipStream_t st,
                const DgradFusion* fz = nullptr, int cfg = -1, void* w_flip = nullptr,
                bool preflipped = false, float* split_ws = nullptr);
bool conv_dgrad_fwd_style(const ConvShape& s, bool dense_too);
int conv_dgrad_tiles_m(const ConvShape& s, int cfg);  // M-tiles over all stride classes
// dw is ACCUMULATED into (split-K fp32 atomics, or a plain read-modify-write when unsplit): pass
// a zeroed buffer, or the parameter's gradient buffer to fuse autograd's accumulation (gradient
// lands directly in the DDP bucket).  splits: > 0 forces the split-K count, -1 = heuristic.
//  ws != nullptr (deterministic mode): [conv_wgrad_splits(s, cfg, splits)][Co*KH*KW*Ci] workspace
//  for the split-K partials, summed into dw in split order.
// BN-backward collect riding in another kernel: block (0,0) of the kernel sums the replica rows
// of a bwd slab that the PREVIOUS kernel filled (the fused dgrad of the same conv), writes
// out[0][C] = Σg, out[1][C] = Σg·x̂, re-zeroes the slab and accumulates dβ += Σg, dγ += Σg·x̂
// (dgamma / dbeta may be null) — the work of a separate bn_bwd_collect launch, whose ~6 us
// standalone cost grows to 10-15 us right after a large kernel (tools/r2/collect_probe.py), hidden
// in the weight-grad kernel that runs between the dgrad and the BN apply anyway.
struct BnCollect {
  float* rep = nullptr;  // [3][kStatReplicas][C] slab; null: nothing to collect
  int C = 0;
  float* out = nullptr;  // [2][C], or [3][C] with `two`
  float *dgamma = nullptr, *dbeta = nullptr;
  // two-branch block output: also Σg·x̂₂ (slab array 2) -> out[2][C]; dγ₂ += Σg·x̂₂, dβ₂ += Σg
  bool two = false;
  float *dgamma2 = nullptr, *dbeta2 = nullptr;
};
// Finishing a workspace split-K GEMM inside the GEMM: every split stores its partial tile to its
// workspace slice, then takes a ticket (one int per output tile, a zeroed self-resetting array);
// the split that arrives last sums the tile's slices in slice order (bit-identical to
// splitk_sum / splitk_sum_bf16) and writes the result — no second kernel, no second pass over
// the slices of tiles that finished early.
struct WsFinish {
  int* ticket = nullptr;   // [tiles] zeroed ints (re-zeroed by the last split); null: off
  void* out = nullptr;     // fp32 accumulate target (out += Σ) or bf16 output
  long ldo = 0;
  const float* bias = nullptr;   // bf16 output: + bias[n]
  const void* addend = nullptr;  // bf16 output: + addend[m][n] (bf16, row pitch N)
  int bf16 = 0;
};
// col: optional collect riding in this launch (see BnCollect)
// in_scale / in_bias: folded input BatchNorm (see conv_fwd; bf16 dense): x holds y and the
// weight-grad reads relu(y*in_scale + in_bias)
void conv_wgrad(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st,
                int cfg = -1, float* ws = nullptr, int splits = -1, const BnCollect* col = nullptr,
                const float* in_scale = nullptr, const float* in_bias = nullptr);
int conv_wgrad_splits(const ConvShape& s, int cfg, int splits = -1);
// 3x3 / stride 1 / pad 1 bf16 weight-grad with the input patch resident in LDS (wgrad3x3.hip):
// partial tiles per split go to ws [splits][Co*9*Ci] and are added to dw in a fixed order
bool conv_wgrad3x3_supported(const ConvShape& s);
int conv_wgrad3x3_splits(const ConvShape& s, int splits_req = -1);
void conv_wgrad3x3(const void* dy, const void* x, float* dw, const ConvShape& s, hipStream_t st,
                   float* ws, int splits, const BnCollect* col = nullptr);
extern bool g_wgrad3x3;  // route supported shapes to conv_wgrad3x3 (default on)

// ---- direct convolution, BatchNorm for any C, k x k average pool (vision.hip) ----------------
struct GConvShape {
  int N, H, W, Ci, Co, KH, KW, sh, sw, ph, pw, groups, Ho, Wo;
};
// act: 0 none, 1 relu, 2 relu6.  Weights [Co][KH][KW][Ci/groups].  f32: activations and
// weights are fp32 (the reference's precision) instead of bf16.
void gconv_fwd(const void* x, const void* w, const float* bias, void* y, const GConvShape& s,
               int act, hipStream_t st, bool f32 = false);
// z (optional): the forward OUTPUT of a fused activation; dy is masked by act'(z)
void gconv_dgrad(const void* dy, const void* w, const void* z, void* dx, const GConvShape& s,
                 int act, hipStream_t st, bool f32 = false);
// dw [Co][KH][KW][Ci/groups] and dbias [Co] (optional) are ACCUMULATED into (fp32 atomics)
void gconv_wgrad(const void* dy, const void* x, const void* z, float* dw, float* dbias,
                 const GConvShape& s, int act, hipStream_t st, bool f32 = false);
// depthwise (groups == Ci == Co, C % 8 == 0, C <= 2048): taps-major weights wt [KH*KW][C];
// dw stays in the parameter layout [C][KH][KW]
void dwconv_fwd(const void* x, const void* wt, const float* bias, void* y, const GConvShape& s,
                int act, hipStream_t st, bool f32 = false);
void dwconv_dgrad(const void* dy, const void* wt, const void* z, void* dx, const GConvShape& s,
                  int act, hipStream_t st, bool f32 = false);
void dwconv_wgrad(const void* dy, const void* x, const void* z, float* dw, float* dbias,
                  const GConvShape& s, int act, hipStream_t st, bool f32 = false);
// psum/psq: zeroed [C] accumulators of Σ(y - shift), Σ(y - shift)²
void chan_stats(const void* y, const float* shift, long M, int C, float* psum, float* psq,
                hipStream_t st, bool f32 = false);
void affine_act(const void* y, const float* scale, const float* bias, void* z, long M, int C,
                int act, hipStream_t st, bool f32 = false);
// out_g / out_gx: zeroed [C] accumulators
void bn_generic_bwd_reduce(const void* dz, const void* z, const void* y, const float* mean,
                           const float* invstd, long M, int C, int act, float* out_g,
                           float* out_gx, hipStream_t st, bool f32 = false);
void bn_generic_bwd_apply(const void* dz, const void* z, const void* y, const float* mean,
                          const float* invstd, const float* gamma, const float* sum_g,
                          const float* sum_gx, long count, long M, int C, int act, void* dy,
                          hipStream_t st, bool f32 = false);
void avgpool2d_fwd(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int k,
                   int stride, int pad, hipStream_t st, bool f32 = false);
void avgpool2d_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo, int k,
                   int stride, int pad, hipStream_t st, bool f32 = false);

// ---- dense GEMM: C[M][N] = op(A) op(B) --------------------------------------------------------
//  a_kc: A stored [M][K] (else [K][M]);  b_kc: B stored [N][K] (else [K][N]).
//  out: 0 = activation-dtype store (bias/act), 1 = fp32 store (bias), 2 = fp32 accumulate into C
//  (split-K atomics when splits > 1, else a non-atomic read-modify-write).
//  f32: A and B are fp32 (split-bf16 main loop); out 0 then stores fp32 (the activation dtype).
//  cfg: tile config id (conv_common.hpp table; -1 = heuristic); splits (out 2): > 0 forces the
//  split-K count (1 = no split), -1 = heuristic.  addend (out 0, A [M][K], B [K][N] only): a
//  [M][ldc] tensor of the output dtype added to the product in the epilogue.
//  ws_split (out 2, splits > 1): C is a [splits][M][ldc] fp32 WORKSPACE; split s stores its
//  partial tile into slice s with plain stores (no atomics; the caller sums the slices in order
//  with splitk_sum) — deterministic, and for small outputs faster than atomics (~1.3 TB/s).
//  fin (with ws_split, N % 4 == 0): the GEMM finishes the sum itself (WsFinish), the caller
//  runs no splitk_sum.
void gemm(const void* A, long lda, bool a_kc, const void* B, long ldb, bool b_kc, void* C,
          long ldc, int M, int N, int K, const float* bias, int act, int out, hipStream_t st,
          bool f32 = false, int cfg = -1, int splits = -1, const void* addend = nullptr,
          bool ws_split = false, const WsFinish* fin = nullptr, void* aux = nullptr,
          const struct TouchRanges* pf = nullptr);
// pf: up to 2 byte ranges (another GEMM's cold operands) that this GEMM's blocks warm into the
// memory-side cache beside their main loop (one load per 64-B line; mipipe/ops/prefetch.py)
//  act 2 (GELU, bf16 output mode 0): C = gelu(A B + bias) and aux = A B + bias (the
//  pre-activation the backward needs), both [M][ldc]
// WsFinish tickets a gemm needs at most: one per output tile of the smallest tile config
inline long gemm_max_tiles(long M, long N) { return ((M + 63) / 64) * ((N + 63) / 64); }
// the split count a ws_split gemm of this K actually uses for `splits` requested
int gemm_ws_splits(int K, int splits);
int default_gemm_cfg(int M, int N, bool f32);

// ---- BatchNorm ------------------------------------------------------------------------------
// Reduce a [P][C] partial slab pair (shifted sums) and finalize: mean, invstd, scale, bias and
// running-stat update.  work: >= 2*64*C floats scratch.
// psum/psq: [P][C] slabs; when zero_after the slabs are re-zeroed (replica slabs).
void bn_finalize(float* psum, float* psq, int P, int C, long count, const float* shift,
                 const float* gamma, const float* beta, float* run_mean, float* run_var,
                 float momentum, float eps, float* mean, float* invstd, float* scale, float* bias,
                 bool zero_after, long long* nbt, hipStream_t st);
// z = act(y*scale + bias [+ r | + r*rscale + rbias])   (M rows of C channels, bf16 or f32)
void bn_act_fwd(const void* y, const float* scale, const float* bias, const void* r,
                const float* rscale, const float* rbias, void* z, long M, int C, bool relu,
                hipStream_t st, bool f32 = false, uint8_t* mask = nullptr);
// sums: out_g[C], out_gx[C], out_gx2[C] (if y2).  rep: zeroed [3][kStatReplicas][C] slab,
// left zeroed on return.
void bn_act_bwd_reduce(const void* dz, const void* z, const void* y, const float* mean,
                       const float* invstd, const void* y2, const float* mean2,
                       const float* invstd2, bool relu, long M, int C, float* out_g,
                       float* out_gx, float* out_gx2, float* rep, float* dgamma, float* dbeta,
                       float* dgamma2, float* dbeta2, hipStream_t st, bool f32 = false,
                       float* det_ws = nullptr, const float* gx_div = nullptr);
// (invstd may be null: 1.  gx_div: out_gx /= gx_div[c] before dγ — with y = z = a post-ReLU BN
// output, mean = β and invstd = null this turns Σg·(z-β) into Σg·x̂, x̂ = (z-β)/γ where z > 0.)
// grid size of the reduce pass: deterministic mode needs det_ws = [3][blocks][C] floats
int bn_bwd_reduce_blocks(long M, int C);
// Sum the replica rows of a bwd slab (filled by a fused dgrad epilogue) into out_g / out_gx,
// re-zero it, optionally accumulate dγ += Σg·x̂, dβ += Σg.
void bn_bwd_collect(float* rep, int C, float* out_g, float* out_gx, float* dgamma, float* dbeta,
                    hipStream_t st);
void bn_act_bwd_apply(const void* dz, const void* z, const void* y, const float* mean,
                      const float* invstd, const float* gamma, const float* sum_g,
                      const float* sum_gx, const void* y2, const float* mean2,
                      const float* invstd2, const float* gamma2, const float* sum_gx2, long count,
                      bool relu, bool want_dres, void* dy, void* dother, long M, int C,
                      hipStream_t st, bool f32 = false);

// ---- pooling ----------------------------------------------------------------------------------
void maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                 int k, int stride, int pad, hipStream_t st, bool f32 = false);
void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int Ho,
                 int Wo, int k, int stride, int pad, hipStream_t st, bool f32 = false);
// Stem fusion (pool.hip): out = maxpool_k,s,p(relu(y*scale + bias)) + window argmax idx, and
// the backward as gathers over the windows (g = Σ dp over windows whose argmax is the pixel and
// whose output is > 0): Σg, Σg·x̂ into the replica slab rep ([3][kStatReplicas][C]; det_rows > 0:
// rep is [2][det_rows][C] partial rows, one per block), then dy = A·g + B·y + C.
// C % 8 == 0 and 256 % (C / 8) == 0.
void pool_bn_fwd(const void* y, const float* scale, const float* bias, void* out, uint8_t* idx,
                 int N, int H, int W, int C, int Ho, int Wo, int k, int stride, int pad,
                 hipStream_t st, bool f32 = false);
int pool_bn_bwd_reduce_blocks(long pixels, int C);
void pool_bn_bwd_reduce(const void* dp, const uint8_t* idx, const void* pout, const void* y,
                        const float* mean, const float* invstd, int N, int H, int W, int C,
                        int Ho, int Wo, int k, int stride, int pad, float* rep, int det_rows,
                        hipStream_t st, bool f32 = false);
void pool_bn_bwd_apply(const void* dp, const uint8_t* idx, const void* pout, const void* y,
                       const float* mean, const float* invstd, const float* gamma,
                       const float* sum_g, const float* sum_gx, long count, void* dy, int N, int H,
                       int W, int C, int Ho, int Wo, int k, int stride, int pad, hipStream_t st,
                       bool f32 = false);
void avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st, bool f32 = false);
void avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st, bool f32 = false);

// ---- loss / optimizer / data -----------------------------------------------------------------
// work: 4 ints (valid-row count) then R floats (per-row losses, summed in a fixed order: the
// loss is bit-reproducible)
void cross_entropy_fwd_bwd(const void* logits, const int64_t* labels, float* loss, void* grad,
                           int R, int V, float smoothing, int64_t ignore_index, int* work,
                           hipStream_t st, bool f32 = false, int valid_cols = 0);
// The training-step split of the same loss: cross_entropy_fwd writes the loss, the valid-row count
// (work[0]) and per-row losses / log-sum-exps (work + 4: [2][R] floats; work holds 4 + 2R ints);
// cross_entropy_bwd then writes grad = (softmax - target) * gout[0] / count from the logits.
void cross_entropy_fwd(const void* logits, const int64_t* labels, float* loss, int R, int V,
                       float smoothing, int64_t ignore_index, int* work, hipStream_t st, bool f32,
                       int Vv);
void cross_entropy_bwd(const void* logits, const int64_t* labels, const int* work,
                       const float* gout, void* grad, int R, int V, float smoothing,
                       int64_t ignore_index, hipStream_t st, bool f32, int Vv);
// *correct += #rows whose first maximal logit is at the label (torch.argmax tie rule)
void top1_correct(const void* logits, const int64_t* labels, int R, int V, int* correct,
                  hipStream_t st, bool f32 = false);
void sgd_step(float* p, const float* g, float* m, void* shadow, long n, float lr, float momentum,
              float dampening, float wd, bool nesterov, bool first, float grad_scale,
              hipStream_t st);
// One-shot collective over peer workspaces (csrc/kernels/oneshot.hip): fp32 sum * scale
// (reduce) or a byte broadcast from `src`; nbytes % 16 == 0, nbytes <= cap.  nblocks: the
// communicator's fixed grid (oneshot_blocks(cap)); timeout_s: the bounded wait for a peer.
constexpr long kOneShotHeaderBytes = 4096;
constexpr long kOneShotErrOffset = 2048;  // two words: {1 + peer, epoch} of a wait that gave up
int oneshot_blocks(long cap);
void oneshot_launch(char* const* bases, int rank, int world, const void* in, void* out,
                    long nbytes, bool reduce, int src, float scale, long cap, int nblocks,
                    double timeout_s, hipStream_t st);
// DDP bf16 wire: wire = bf16(g * scale), g = fp32(wire); n % 8 == 0, 16-B aligned pointers
void grad_pack_bf16(const float* g, void* wire, long n, float scale, hipStream_t st);
void grad_unpack_bf16(const void* wire, float* g, long n, hipStream_t st);
// t_dev (device step counter, may be null): bias corrections 1 - b^t computed in the kernel
void adamw_step(float* p, const float* g, float* m, float* v, void* shadow, long n, float lr,
                float b1, float b2, float eps, float wd, float bc1, float bc2, float grad_scale,
                hipStream_t st, const int* t_dev = nullptr);
void nchw_to_nhwc(const void* x, bool x_is_bf16, void* y, int N, int C, int H, int W, int Cp,
                  hipStream_t st, bool y_f32 = false);
// Stem "super-pixel" packing (C <= 4): y[n][h'][j][p*4 + c] = x[n][c][h'-pad][2j+p-pad] (zero
// outside), h' < Hp, j < Wsp.  A KxK stride-2 conv on x becomes a K x ceil(K/2) conv with
// vertical stride 2 and horizontal stride 1 on 8-channel super-pixels: 16-byte operand rows with
// 3 of 8 lanes padding instead of 5 of 8 (the reduction shrinks from K*K*8 to K*ceil(K/2)*8).
// w (fp32 [Co][C][K][K], strides ws[4]) given: the same launch also writes the packed filter
// wp [Co][K][ceil(K/2)][8] in y's dtype.
void stem_pack(const void* x, bool x_is_bf16, void* y, int N, int C, int H, int W, int pad,
               int Hp, int Wsp, hipStream_t st, bool y_f32 = false, const float* w = nullptr,
               void* wp = nullptr, int Co = 0, int K = 0, const long* ws = nullptr);
// g[co][c][kh][kw] (strides gs[4]) += dwp[co][kh][kw/2][(kw%2)*4 + c] (packed stem filter grad)
void stem_wgrad_unpack(const float* dwp, float* g, int Co, int C, int K, const long* gs,
                       hipStream_t st);
void synthetic_batch(const int64_t* idx, int n, int C, int H, int W, int classes, int seed,
                     void* x, bool bf16_out, int64_t* labels, hipStream_t st);
// Fused ResNet stem on the packed input (stem.hip): conv 7x7/2 (packed K = 224, 64 channels,
// 112 output columns) -> BN -> ReLU -> max-pool 3x3/2/1.
//   stem_fwd_stats : shifted Σ, Σ² of bf16(y) per channel (conv recomputed, y not stored) ->
//                    replica rows (atomics) or, with det_rows = stem_stats_blocks(), one partial
//                    row per block (plain stores)
//   stem_fwd_pool  : y (bf16, for the backward), out = maxpool(bf16(relu(y*scale + bias))),
//                    idx = window tap (0xFF where out is not > 0)
//   stem_bwd_wgrad : dW[64][224] += Σ dy ⊗ x with dy = A·g + B·y + C formed in LDS (g routed from
//                    dp / idx; Σg, Σg·x̂ from pool_bn_bwd_reduce); ws: [stem_wgrad_blocks][64*224]
bool stem_fused_supported(int N, int Ho, int Wo, int Hp, int Wsp, int Co, int Hpool, int Wpool);
int stem_stats_blocks(int N, int Ho);
int stem_wgrad_blocks(int N, int Ho);
void stem_fwd_stats(const void* xp, const void* w, int N, int Ho, int Hp, const float* shift,
                    float* ssum, float* ssq, int R, int det_rows, hipStream_t st);
void stem_fwd_pool(const void* xp, const void* w, int N, int Ho, int Hp, const float* scale,
                   const float* bias, void* out, uint8_t* idx, void* y, hipStream_t st);
void stem_bwd_wgrad(const void* xp, const void* y, int N, int Ho, int Hp, const void* dp,
                    const uint8_t* idx, const float* mean, const float* invstd, const float* gamma,
                    const float* sum_g, const float* sum_gx, long count, float* ws, float* dw,
                    hipStream_t st);

// ---- transformer ops ------------------------------------------------------------------------
// Hash dropout of an operand (the mask of dropout_fwd with the same seed / element index).
struct DropSpec {
  float p;
  uint32_t seed;
  const uint32_t* seed_dev;  // device step counter mixed into the seed (may be null)
};
// drop (may be null): y = LN(dropout(x) + res) — BERT's post-LN residual branch in one pass
void layernorm_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y,
                   void* xsum, float* mean, float* rstd, long rows, int H, float eps,
                   hipStream_t st, const DropSpec* drop = nullptr);
// drop + dxd: also writes dxd = dropout'(dx), the dropped branch's gradient
void layernorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd,
                   const float* gamma, void* dx, float* dgamma, float* dbeta, float* work,
                   long rows, int H, hipStream_t st, void* dxd = nullptr,
                   const DropSpec* drop = nullptr, float* dbias = nullptr);
int layernorm_bwd_blocks(long rows);  // partial rows of layernorm_bwd's work
// LayerNorm kernel family: 0 = the generic one-row-per-wave kernels (16-B chunks, any H % 8 == 0),
// 4 / 8 (default) / 16 = the exact-width kernels (chunk width picked so every lane holds whole
// chunks, DPP wave sums) with that many waves per backward block; the generic kernels still
// serve the widths the exact ones do not cover (and the 8-wide forward).  MIPIPE_LN_MODE.
// Cache warming: one load per 64-B line of each range, nothing written (touch_kernel).
constexpr int kTouchRanges = 4;
struct TouchRanges {
  const uint8_t* ptr[kTouchRanges];
  long bytes[kTouchRanges];
  int count = 0;
};
void touch(const TouchRanges& r, hipStream_t st);
void set_layernorm_mode(int mode);
int get_layernorm_mode();
void gelu_fwd(const void* x, void* y, long n, hipStream_t st);
void gelu_bwd(const void* dy, const void* x, void* dx, long n, hipStream_t st);
// gelu_bwd of a [rows, cols] tensor that also accumulates out[c] += Σ_rows dx[:, c] (the GELU
// Linear's bias gradient); work (deterministic mode): [gelu_bwd_colsum_blocks(rows, cols)][cols]
void gelu_bwd_colsum(const void* dy, const void* x, void* dx, float* out, long rows, int cols,
                     float* work, hipStream_t st);
int gelu_bwd_colsum_blocks(long rows, int cols);
// Fused self-attention, head_dim 64, on the packed projection layout (attention.hip):
//   qkv [B*S][3*H*64] bf16, o [B*S][H*64] bf16, lse [B][H][S] fp32, mask [B][S] additive or null.
// p_drop > 0 applies attention-probability dropout keyed by (seed, b, h, q, k).
extern int g_attn_waves;  // attention block size override (0 auto, 2, 4)
void attention_fwd(const void* qkv, const float* mask, void* o, float* lse, int B, int S, int H,
                   float scale, float p_drop, uint32_t seed, hipStream_t st,
                   const uint32_t* seed_dev = nullptr);
// dqkv [B*S][3*H*64]; delta [B][H][S] and dq_acc [attention_dq_slabs(S)][B*S][H*64] fp32 are
// scratch (deterministic mode: one dQ slab per key block, summed in order; else 1 slab + atomics;
// 0 slabs when S fits one key block: dQ is then stored as bf16 by the backward kernel itself).
int attention_dq_slabs(int S);
bool attention_dq_direct(int S);
void attention_bwd(const void* dout, const void* qkv, const void* o, const float* lse,
                   const float* mask, void* dqkv, float* delta, float* dq_acc, int B, int S,
                   int H, float scale, float p_drop, uint32_t seed, hipStream_t st,
                   const uint32_t* seed_dev = nullptr);
// Elementwise dropout keyed by (seed, element index): y = x * keep / (1 - p); the backward
// recomputes the same keep mask from the seed (no mask tensor).
// seed_dev (device step counter, may be null) is mixed into the seed inside the kernel, so a
// replayed hipGraph draws a fresh mask every step.
void dropout_fwd(const void* x, void* y, long n, float p, uint32_t seed, hipStream_t st,
                 const uint32_t* seed_dev = nullptr);
// partial (tables of <= 8 rows, deterministic mode): [embedding_bwd_small_blocks(n)][rows*H]
// scratch — per-block tables summed in block order instead of float atomics
void embedding_bwd(const void* dy, const int64_t* idx, float* out, long n, int H, int rows,
                   hipStream_t st, float* partial = nullptr);
int embedding_bwd_small_blocks(long n);
// Deterministic scatter-add: out[sorted_ids[i]] += scale * dy[perm[i]], tokens stably sorted by
// id (perm: their positions); one writer per output row, rows summed in position order in
// fixed 64-entry chunks (long runs in parallel, then the chunk partials in order).  ws:
// embedding_bwd_sorted_ws_floats(n, H) floats of scratch.  Negative ids are skipped.
// H % 8 == 0, H <= 2048.
long embedding_bwd_sorted_ws_floats(long n, int H);
void embedding_bwd_sorted(const void* dy, const int64_t* sorted_ids, const int64_t* perm,
                          float* out, float* ws, long n, int H, float scale, hipStream_t st);
// work (deterministic mode, else null): [colsum_blocks(rows, cols)][cols] floats of partials
void colsum_f32(const void* x, bool bf16, float* out, long rows, int cols, float* work,
                hipStream_t st);
int colsum_blocks(long rows, int cols);
extern int g_colsum_row_blocks;
extern int g_nt_store;  // non-temporal activation stores: 1 conv fwd, 2 dgrad, 4 BN passes
extern long g_nt_min_bytes;  // outputs up to this size keep cached stores (MALL-resident)

}  // namespace mipipe
