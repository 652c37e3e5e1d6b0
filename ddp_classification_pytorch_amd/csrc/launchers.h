// Host-side launcher declarations shared by the kernel translation units and
// the PyTorch operator bindings (bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

typedef __bf16 bf16;

namespace dcp {

// tuning switches (in-process A/B experiments, the autotuner's overrides): named slots, tune.h
}  // namespace dcp
#include "tune.h"
namespace dcp {

constexpr int kMaxTaps = 64;

struct TapList {
  int n;
  int dy[kMaxTaps], dx[kMaxTaps], widx[kMaxTaps];
};

// Backward of a training-mode BN + ReLU/identity (+ residual add) fused into the epilogue of
// the stride-1 dgrad that produces the gradient g of the BN layer's OUTPUT:
//   dst = g' = g * act'(y*scale + shift [+ res])   (the activation-masked gradient)
//   part[tile][0][c] = sum g',  part[tile][1][c] = sum g' * (y - mean) * invstd  (per 128-row tile)
// so the separate BN backward reduction pass (re-reading g and y) disappears.
struct BnBwdEpi {
  const bf16* y;        // BN input [M][C]
  const bf16* res;      // residual added before the activation, or nullptr
  const float* scale;   // gamma * invstd
  const float* shift;   // beta - mean * scale
  const float* mean;
  const float* invstd;
  float* part;          // [ceil(M/128)][2][C]
  int act;              // 0 none, 1 ReLU (gradient stored masked), 2 leaky ReLU (stored RAW, summed masked)
  const uint8_t* mask;  // act'(z) > 0 as bits [M][C/8] (bn_act's mask output), or nullptr: recompute z
  float slope;          // leaky slope (act 2)
  // addsrc on the stride-2 subgrid only: [N][add_hc][add_wc][C] holds the gradient of the even
  // (y, x) pixels, zero elsewhere -- a projection block's 1x1 / stride-2 downsample dgrad, deposited
  // compact instead of as a mostly-zero full-size tensor (ops/functional.py StridedGrad)
  int add_s2;
  int add_hc, add_wc;
};

// Eval-mode BN folded into the forward conv's store epilogue (running statistics: model.eval(),
// NESTED's frozen BN): dst = act(acc_bf16 * scale + shift [+ addsrc]) per output channel, so the
// conv output is never written un-normalised and no separate BN-apply pass runs.
struct AffineEpi {
  const float* scale;  // gamma * invstd(running var)
  const float* shift;  // beta - running_mean * scale
  int act;             // 0 none, 1 ReLU, 2 leaky ReLU
  float slope;
};

// stream-ordered device workspace for kernels that need scratch (stream-K partials): bindings.cpp
// registers PyTorch's caching allocator (raw_alloc_with_stream / raw_delete)
using WorkspaceAlloc = void* (*)(size_t bytes, hipStream_t stream);
using WorkspaceFree = void (*)(void* ptr);
void set_workspace_allocator(WorkspaceAlloc alloc, WorkspaceFree free_fn);
// number of problems the tap-GEMM autotuner (g_tune[kAutotune] = 1) has measured in this process
int tap_gemm_tuned_count();
// the tuner's per-problem choices as "key\tchoice" lines, and back (returns entries accepted)
std::string tap_gemm_tune_export();
int tap_gemm_tune_import(const std::string& text);
void launch_tap_gemm(const bf16* src, int N, int Hs, int Ws, int Cs, const bf16* wt, int Co, int T, bf16* dst, int Hd,
                     int Wd, int Hy, int Wy, int ss, int ds, int oy, int ox, const TapList& taps, float* stats,
                     const float* bias, int relu, const bf16* zero, hipStream_t stream, const bf16* addsrc = nullptr,
                     const BnBwdEpi* bnb = nullptr, const AffineEpi* aff = nullptr,
                     const float* pscale = nullptr, const float* pshift = nullptr, int nbias = 0);
// (pscale, pshift: BN + ReLU prologue on the input of a 1x1 stride-1 forward, K5 -- the input is
// the BN's input x and the conv sees bf16(relu(x * pscale[c] + pshift[c])))
// backward of act(c * scale + shift [+ r]) from its output y: g = dy * act'(y) and dc = g * scale
// (g only when want_g: the residual's gradient)
void launch_act_scale_bwd(const bf16* dy, const bf16* y, const float* scale, int64_t M, int C, int act, float slope,
                          bf16* dc, bf16* g, hipStream_t s);
void launch_partial_sum(const float* part, int P, int K, float* out, hipStream_t s);
void launch_partial_sum_bf16(const float* part, int P, int K, bf16* out, hipStream_t s);
// partial-slab split-K weight gradient: dw is fully written when part != nullptr
// (part = wgrad_splits(...) x Co x T*Cs floats); part == nullptr -> fp32 atomics into a zeroed dw
int wgrad_splits(int M, int Co, int ldw, int taps, int num_cu, int* rows_per_split);
// splits (partials) of launch_wgrad for this geometry: the direct 3x3 kernel's where it applies
int wgrad_plan_splits(int N, int Ho, int Wo, int Co, int Hs, int Ws, int Cs, int ss, const TapList& taps,
                      int num_cu);
// wgrad3x3.hip: direct 3x3 / stride-1 / pad-1 weight gradient (0 = not applicable)
int wgrad3x3_splits(int N, int H, int W, int C, int Co, int num_cu);
void launch_wgrad3x3(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Co, float* part, int splits,
                     const bf16* zero, hipStream_t stream, const float* pscale = nullptr,
                     const float* pshift = nullptr);
void launch_split_reduce(const float* part, int splits, int n, float* out, hipStream_t stream);
void launch_wgrad(const bf16* dy, int N, int Ho, int Wo, int Co, const bf16* src, int Hs, int Ws, int Cs, int ss,
                  const TapList& taps, float* dw, float* part, const bf16* zero, int num_cu, hipStream_t stream,
                  const float* pscale = nullptr, const float* pshift = nullptr);
// frag: gconv_frag_elems(...) bf16 workspace (MFMA path; may be null -> direct kernels)
// stats (optional, [gconv_fwd_stat_blocks(M)][3][Co]): BN partials of y from the MFMA kernel's epilogue;
// returns whether they were written (false: the direct fallback kernel ran)
bool launch_grouped_conv_fwd(const bf16* x, const bf16* w, bf16* y, bf16* frag, int N, int H, int W, int C, int Ho,
                             int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s,
                             float* stats = nullptr);
int gconv_fwd_stat_blocks(int M);
void launch_grouped_conv_dgrad(const bf16* dy, const bf16* w, bf16* dx, bf16* frag, int N, int H, int W, int C,
                               int Ho, int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s);
// dw is fully written; part = workspace of gconv_mfma_wgrad_splits(...) x Co*KH*KW*(C/G) floats
void launch_grouped_conv_wgrad(const bf16* dy, const bf16* x, float* dw, float* part, int splits, const bf16* zero,
                               int N, int H, int W, int C, int Ho, int Wo, int Co, int G, int KH, int KW, int stride,
                               int pad, hipStream_t s);
// MFMA super-group kernels (gconv.hip); return false for shapes they do not cover
int gconv_frag_elems(int C, int G, int KH, int KW);
bool launch_gconv_mfma_fwd(const bf16* x, const bf16* w, bf16* y, bf16* frag, int N, int H, int W, int C, int Ho,
                           int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s,
                           float* stats = nullptr);
// fused ReLU-BN backward reduction for the grouped dgrad (z: BN input; part: [gconv_fwd_stat_blocks(M)][2][C])
struct GconvBnBwd {
  const bf16* z;
  const float *scale, *shift, *mean, *invstd;
  float* part;
};
bool launch_gconv_mfma_dgrad(const bf16* dy, const bf16* w, bf16* dx, bf16* frag, int N, int H, int W, int C, int Ho,
                             int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s,
                             const GconvBnBwd* bn = nullptr);
int gconv_mfma_wgrad_splits(int N, int Ho, int Wo, int C, int G);
int gconv_fallback_wgrad_splits(int M, int nw);  // part rows the direct fallback needs
bool launch_gconv_mfma_wgrad(const bf16* dy, const bf16* x, float* dw, float* part, int splits, const bf16* zero,
                             int N, int H, int W, int C, int Ho, int Wo, int Co, int G, int KH, int KW, int stride,
                             int pad, hipStream_t s);

int bn_stats_partials(int M, int C, bool from_slabs);
void launch_bn_stats(const bf16* x, const float* slabs, int M, int C, float* part, float* out, hipStream_t s);
// iabn_eps >= 0 (the finalize launchers): InplaceABN's |gamma| + iabn_eps as the weight, 1 / it into rgamma
void launch_bn_stats_finalize(const bf16* x, const float* slabs, int M, int C, float* part, float eps,
                              const float* gamma, const float* beta, float* mean, float* invstd, float* scale,
                              float* shift, float* rm, float* rv, float momentum, hipStream_t s, float iabn_eps = -1.f,
                              float* rgamma = nullptr);
// BN statistics from ready first-level partials [P][3][C] (e.g. the stem kernel's)
// two-level merge of many partials: chunks of 128 rows (0 = merge directly), and the first level
int bn_partial_chunks(int P);
void launch_bn_partial_chunk(const float* part, int P, int C, float* tmp, hipStream_t s);
void launch_bn_merge(const float* part, int P, int C, float* out, hipStream_t s);
void launch_bn_merge_finalize(const float* part, int P, int C, float eps, const float* gamma, const float* beta,
                              float* mean, float* invstd, float* scale, float* shift, float* rm, float* rv,
                              float momentum, hipStream_t s, float iabn_eps = -1.f, float* rgamma = nullptr);
// stem.hip: the space-to-depth stem conv [N][H][W][16] x [64][4][4][16] -> [N][H][W][64]
bool stem_fwd_supported(int H, int W, int C, int Co, int KH, int KW);
int stem_fwd_blocks(int N, int H);
void launch_stem_fwd(const bf16* x, const bf16* w, bf16* y, float* part, const bf16* zero, int N, int H, int W,
                     hipStream_t s);
// fused stem backward (BN + ReLU + 3x3/2 max pool + weight gradient): part [blocks][part_floats];
// reduce it over blocks (launch_split_reduce) -> tot, then sums [2][64] and dw [64][256]
bool stem_bwd_supported(int H, int W, int C, int Ho, int Wo);
int stem_bwd_blocks(int N, int H, int num_cu);
int stem_bwd_part_floats();
void launch_stem_bwd(const bf16* z, const bf16* x16, const bf16* dy, const uint8_t* idx, const float* scale,
                     const float* shift, const float* mean, int act, int N, int H, int W, int nblocks, float* part,
                     hipStream_t s);
void launch_stem_bwd_sums(const float* tot, const float* invstd, float* sums, hipStream_t s);
void launch_stem_bwd_dw(const float* tot, const float* sums, const float* scale, const float* invstd, float inv_count,
                        float* dw, hipStream_t s);
int colsum_partials(int M);
void launch_colsum(const bf16* x, int M, int C, float* part, float* out, hipStream_t s);
void launch_bn_finalize(const float* st, int W, int C, float eps, const float* gamma, const float* beta, float* mean,
                        float* invstd, float* scale, float* shift, float* rm, float* rv, float momentum,
                        hipStream_t s, float iabn_eps = -1.f, float* rgamma = nullptr);
void launch_bn_eval_coeff(int C, float eps, const float* gamma, const float* beta, const float* rm, const float* rv,
                          float* mean, float* invstd, float* scale, float* shift, hipStream_t s);
void launch_bn_act_fwd(const bf16* x, const bf16* res, const float* scale, const float* shift, bf16* y, size_t numel,
                       int C, int act, float slope, hipStream_t s, uint8_t* mask = nullptr,
                       const float* rscale = nullptr, const float* rshift = nullptr);
void launch_bn2_bwd_elemt(const bf16* dy, const bf16* x, const bf16* r, const float* scale, const float* mean,
                          const float* invstd, const float* sums, const float* rscale, const float* rmean,
                          const float* rinvstd, const float* rsums, float inv_count, size_t numel, int C, bf16* dx,
                          bf16* dr, hipStream_t s);
int bn_bwd_reduce_blocks(int M, int C);
void launch_bn_bwd_reduce(const bf16* dy, const bf16* x, const bf16* res, const float* scale, const float* shift,
                          const float* mean, const float* invstd, int M, int C, int act, float slope, float* partials,
                          float* out, hipStream_t s, int inv = 0);
// inv = 1: InplaceABN backward -- x is the layer OUTPUT y (act invertible: none / leaky), mean /
// invstd are beta / 1/gamma, and the pre-activation is recovered in registers
// dg != nullptr (with sums): also dg = sign(graw) * sums[1] -- InplaceABN's raw-weight gradient
void launch_bn_bwd_elemt(const bf16* dy, const bf16* x, const bf16* res, const float* scale, const float* shift,
                         const float* mean, const float* invstd, const float* sums, float inv_count, size_t numel,
                         int C, int act, float slope, bf16* dx, bf16* dres, hipStream_t s, int inv = 0,
                         const float* graw = nullptr, float* dg = nullptr);

void launch_maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo, int k,
                        int s, int p, hipStream_t st, const float* scale = nullptr, const float* shift = nullptr,
                        int act = 0);
// backward of BN(+act) -> max pool: dx == nullptr -> reduction pass (part: maxpool_bn_bwd_blocks() x 2 x C
// scratch, sums_out [2][C]); else the elementwise pass with the global `sums`
int maxpool_bn_bwd_blocks();
void launch_maxpool_bn_bwd(const bf16* dy, const uint8_t* idx, const bf16* x, int N, int H, int W, int C, int Ho,
                           int Wo, int k, int s, int p, const float* scale, const float* shift, const float* mean,
                           const float* invstd, int act, float* part, float* sums_out, const float* sums,
                           float inv_count, bf16* dx, hipStream_t st);
void launch_maxpool_bwd(const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st);
// two-level reductions over HW per (n, c) (gap_fwd, chan_scale_bwd): row splits S; the
// part workspace holds S x N x C floats
int hw_splits(int N, int HW, int C);
void launch_gap_fwd(const bf16* x, bf16* y, float* part, int N, int HW, int C, hipStream_t st);
void launch_gap_bwd(const bf16* dy, bf16* dx, int N, int HW, int C, hipStream_t st, const bf16* add = nullptr);
void launch_s2d(const bf16* x, bf16* y, int N, int H, int W, int C, int b, int inverse, hipStream_t st);

void launch_xent_fwd(const void* logits, bool is_bf16, int B, int ld, int C, const int64_t* labels, float* loss,
                     int* rank, float smoothing, hipStream_t s);
void launch_metric_accum(double* acc, const float* loss, int nloss, float loss_scale, const int* rank, int nrows,
                         hipStream_t s);
void launch_xent_bwd(const void* logits, bool in_bf16, int B, int ld, int C, const int64_t* labels,
                     const float* grad_out, float scale, float smoothing, void* dlogits, int ldo, bool out_bf16,
                     hipStream_t s);
void launch_log_softmax_fwd(const void* x, bool is_bf16, int B, int ld, int C, float* y, hipStream_t s);
void launch_log_softmax_bwd(const float* y, const float* dy, int B, int C, int ldo, void* dx, bool out_bf16,
                            hipStream_t s);
void launch_l2norm_rows(const void* x, bool is_bf16, int R, int Rout, int D, int ldo, bf16* y, float* inv_norm, float eps,
                        hipStream_t s);
void launch_l2norm_bwd(const void* dy, bool dy_bf16, int ldd, const bf16* y, int ldy, const float* inv_norm, int R,
                       int D, void* dx, bool out_bf16, hipStream_t s);
void launch_transpose2d(const bf16* x, bf16* y, int R, int C, hipStream_t s);
void launch_arcface_fwd(const bf16* cosv, int B, int ld, int C, const int64_t* labels, float s, float cos_m,
                        float sin_m, float th, float mm, int easy, float* out_logits, float* loss, int* rank,
                        float* lab_dphi, hipStream_t st);
void launch_arcface_bwd(const bf16* cosv, int B, int ld, int C, const int64_t* labels, float s, float cos_m,
                        float sin_m, float th, float mm, int easy, const float* lab_dphi, const float* grad_out,
                        float scale, bf16* dcos, hipStream_t st);

struct MTEntry {
  float* p;
  float* g;
  float* s1;
  float* s2;
  bf16* shadow;
  int64_t n;
};
struct SgdHyper {
  float lr, momentum, dampening, wd, grad_scale;
  int nesterov, first;
};
struct AdamHyper {
  float lr, beta1, beta2, eps, wd, grad_scale, bc1, bc2;
  int decoupled;
  const int* step_dev;  // optional device step count: bc1/bc2 computed in-kernel from it
};
// mode: bit 0 = source bf16, bit 1 = destination bf16 (MTEntry.p = destination, .g = source)
void launch_mt_copy(const MTEntry* tab, const int2* chunks, int nchunks, float scale, int mode, hipStream_t s);
void launch_mt_sgd(const MTEntry* tab, const int2* chunks, int nchunks, SgdHyper h, hipStream_t s);
void launch_mt_adam(const MTEntry* tab, const int2* chunks, int nchunks, AdamHyper h, hipStream_t s);
void launch_cdr_threshold(const MTEntry* tab, const int2* chunks, int nchunks, uint32_t* state, uint32_t* hist,
                          hipStream_t s);
void launch_cdr_mask(const MTEntry* tab, const int2* chunks, int nchunks, const uint32_t* state, float clip,
                     hipStream_t s);

// local training BN: statistics finalize (from conv slabs [R][2][C], R <= bn_direct_slabs(), or
// partials [P][3][C]) + BN / act (+ residual, + mask bits) in one launch; sync: 3 zeroed uint32 counters
// reserved for this stream (re-armed by every launch; sync[2] != 0 after a spin timeout)
int bn_direct_slabs();
void launch_bn_fin_act(const bf16* x, const bf16* res, const float* src, int nsrc, int partials, int M, int C,
                       float eps, const float* gamma, const float* beta, float* mean, float* invstd, float* scale,
                       float* shift, float* rm, float* rv, float momentum, float iabn_eps, float* rgamma, bf16* y,
                       uint8_t* mask, int act, float slope, uint32_t* sync, hipStream_t s);

// direct 3x3 / s1 / p1 conv, 64 -> 64 channels (conv3x3.hip); part: [blocks][3][64] (n, mean, M2) or null
bool conv3x3_c64_supported(int H, int W, int C, int Co);
int conv3x3_c64_blocks(int N, int H, int W, int num_cu);
void launch_conv3x3_c64(const bf16* x, const bf16* w, bf16* y, float* part, const bf16* zero, int N, int H, int W,
                        int blocks, hipStream_t stream, const float* pscale = nullptr, const float* pshift = nullptr,
                        int wflip = 0);

// host int64 table -> device through kernel arguments (graph-capture safe, see misc.hip)
void launch_table_fill(const int64_t* host, int64_t n, int64_t* out, hipStream_t s);
void launch_weight_prep(const float* w, int Co, int T, int Ci, int Co_pad, bf16* wb, bf16* wt, hipStream_t s);
// entries: packed {w, wb, wt, Co, T, Ci_src, Ci, Cp, tci, tco, pad} (56 B each); blocks: int2 (entry, tile)
void launch_mt_weight_prep(const void* entries, const void* blocks, int nblocks, hipStream_t s);
void launch_to_nhwc(const void* src, int is_u8, int nchw, int N, int C, int H, int W, int Cp, float in_scale,
                    const float* mean, const float* stdv, bf16* dst, hipStream_t s);
// space-to-depth input: block 2 (ResNet s2d stem) dst [N][H/2][W/2][16], channel (py*2+px)*4 + c (c < 3
// real); block 4 (TResNet SpaceToDepth(4)) dst [N][H/4][W/4][48], channel (py*4+px)*3 + c
void launch_to_nhwc_s2d(const void* src, int is_u8, int nchw, int N, int C, int H, int W, float in_scale,
                        const float* mean, const float* stdv, bf16* dst, hipStream_t s, int block = 2);
// shard-loader augmentation: meta [B][8] = {byte offset, H, W, y0, x0, h, w, flip} -> out [B][Ho][Wo][3]
void launch_crop_resize(const uint8_t* src, const int64_t* meta, int B, int Ho, int Wo, uint8_t* out, hipStream_t s);
void launch_act_bwd(const bf16* dy, const bf16* y, bf16* dx, size_t numel, int act, hipStream_t s);
void launch_prefix_mask(const bf16* x, bf16* y, int B, int D, const int* keep, hipStream_t s);
// Philox dropout (misc.hip): y = x * keep / (1 - p); keep from (seed, *offset_ptr, element index);
// `used` (optional) receives the offset the launch drew with (for the mask-regenerating backward)
// InplaceABN effective weight: geff = |g| + eps, rg = 1 / geff; backward out = d * sign(g)
void launch_iabn_gamma(const float* g, float eps, float* geff, float* rg, int C, hipStream_t s);
void launch_sign_mul(const float* d, const float* g, float* out, int C, hipStream_t s);
void launch_dropout(const void* x, void* y, size_t n, int is_bf16, float p, uint64_t seed, const int64_t* offset_ptr,
                    int64_t* used, hipStream_t s);
// adaptive average pool NHWC [N,H,W,C] -> [N,OH,OW,C]; backward = true: dy [N,OH,OW,C] -> dx [N,H,W,C]
void launch_adaptive_avg(const bf16* src, bf16* dst, int N, int H, int W, int C, int OH, int OW, bool backward,
                         hipStream_t s);
void launch_nested_eval_scalar(const float* feat, const float* W, const int64_t* labels, int B, int D, int C,
                               int* counts, hipStream_t s);
// workspace bytes of launch_nested_eval (label score chains + per-class-block rank counts)
// weight-stationary persistent 1x1 stride-1 forward GEMM (conv_ws.hip): src [M][K], wt [Co][ldw] -> dst [M][Co]
// (+ per-128-row slab BN statistics); K in {64, 128, 256}, Co % 128 == 0; false = unsupported
bool conv1x1_ws_supported(int K, int Co, long M);
bool launch_conv1x1_ws(const bf16* src, const bf16* wt, int ldw, bf16* dst, float* stats, const bf16* zero, int M,
                       int K, int Co, hipStream_t st);
// store-decoupled persistent 1x1 stride-1 forward GEMM (conv1x1_ps.hip): loader waves fill an LDS-DMA
// ring, consumer waves store straight from the accumulators; same contract as launch_conv1x1_ws
// (ablate: conv1x1_ps.hip PsParams; timing experiments only); cw: consumer waves, 4 or 8
bool conv1x1_ps_supported(int K, int Co, long M);
bool launch_conv1x1_ps(const bf16* src, const bf16* wt, int ldw, bf16* dst, float* stats, const bf16* zero, int M,
                       int K, int Co, int ablate, int cw, hipStream_t st);
// Fused ArcFace head (arcface.hip): no [B, C] tensor.  xn [Bp][Dp] / wn [Cp][Dp] normalised bf16
// (zero padding rows), Bp % 64 == Cp % 64 == 0, Dp in {128, 256}, (128 + Bp / 64) KB of LDS for
// the dW kernel at Dp = 256; false = unsupported shape.
bool launch_arcface_l2norm_t(const void* x, bool is_bf16, int R, int D, int Rp, int Dp, bf16* y, bf16* yT, float* inv,
                             float eps, hipStream_t st);
int arcface_fused_fwd_splits(int Bp, int Cp);
int arcface_fused_dx_splits(int Bp, int Cp);
bool launch_arcface_fused_fwd(const bf16* xn, const bf16* wn, const int64_t* labels, int B, int Bp, int C, int Cp,
                              int Dp, float s, float m, int easy, float* lab, float* part, float* loss, int* rank,
                              float* lse, hipStream_t st);
bool launch_arcface_fused_dx(const bf16* xn, const bf16* wn, const bf16* wnT, const int64_t* labels, int B, int Bp,
                             int C, int Cp, int Dp, int D, float s, const float* lab, const float* lse,
                             const float* gout, float scale, const float* inv_x, float* part, void* dx, bool dx_bf16,
                             hipStream_t st);
int arcface_fused_dw_splits(int Bp, int Cp);
bool launch_arcface_fused_dw(const bf16* xn, const bf16* xnT, const bf16* wn, const int64_t* labels, int B, int Bp,
                             int C, int Cp, int Dp, int D, float s, const float* lab, const float* lse,
                             const float* gout, float scale, const float* inv_w, float* part, float* dw,
                             hipStream_t st);
// SyncBN peer-memory exchange (peer.hip): gather (mode 0, dst [world][n]) or rank-ordered sum
// (mode 1, dst [n]) of n floats through the IPC-mapped mailboxes `boxes` ([world] base addresses);
// a rank missing for timeout_ms sets *err and poisons dst with NaN (this and every later exchange)
bool launch_peer_exchange(const float* src, int n, float* dst, const int64_t* boxes, int* epoch, int rank, int world,
                          int slot, int mode, int* err, int timeout_ms, hipStream_t s);
size_t nested_eval_workspace(int B, int D, int C);
void launch_nested_eval(const float* feat, const float* W, const int64_t* labels, int B, int D, int C, int* counts,
                        void* ws, hipStream_t s);

void launch_dwconv_fwd(const bf16* x, const float* w, bf16* y, int N, int H, int W, int C, int Ho, int Wo, int k,
                       int s, int p, int reflect, hipStream_t st);
void launch_dwconv_bwd(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C, int Ho, int Wo, int k,
                       int s, int p, int reflect, hipStream_t st);
void launch_chan_scale_fwd(const bf16* x, const bf16* g, const bf16* res, bf16* y, int N, int HW, int C, int relu,
                           hipStream_t st);
// squeeze-excitation gate of a small batch, one MFMA workgroup per direction (extra.hip): p [N,C],
// W1 [>=R rows, C], W2 [>=C rows, R] bf16 forward; their transposes W1^T [C][ld1t], W2^T [R][ld2t] backward
bool se_gate_supported(int N, int C, int R);
void launch_se_gate_fwd(const bf16* p, const bf16* w1, const float* b1, const bf16* w2, const float* b2, bf16* h,
                        bf16* g, int N, int C, int R, hipStream_t st);
void launch_se_gate_bwd(const bf16* dg, const bf16* g, const bf16* h, const bf16* p, const bf16* w1t, int ld1t,
                        const bf16* w2t, int ld2t, float* dw1, float* db1, float* dw2, float* db2, bf16* dp, int N,
                        int C, int R, hipStream_t st);
void launch_chan_scale_bwd(const bf16* dy, const bf16* x, const bf16* g, const bf16* res, bf16* dx, bf16* dg, float* part,
                           bf16* dres, int N, int HW, int C, int relu, hipStream_t st);

// stem weight 7x7/2 [Co][7][7][C<=4] <-> space-to-depth 4x4 [Co][4][4][16] (misc.hip)
void launch_s2d_weight(const float* w7, int Co, int C, float* w16, hipStream_t s);
void launch_s2d_weight_bwd(const float* g16, int Co, int C, float* g7, hipStream_t s);

}  // namespace dcp
