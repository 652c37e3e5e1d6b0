// Kernels for the non-ResNet model families:
//   * grouped convolution fallback (shapes the MFMA super-group kernels of
//     gconv.hip do not cover): direct NHWC kernels, 8 channels per thread;
//   * depthwise k x k filter with reflect padding (TResNet anti-aliased
//     downsampling "blur pool", timm tresnet);
//   * per-(sample, channel) scaling for squeeze-and-excitation (K22).
#include <algorithm>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

// ---------------------------------------------------------------------------
// grouped conv. w: [Co][KH][KW][Cg] (Cg = C/G input channels per group)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gconv_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                        bf16* __restrict__ y, int N, int H, int W, int C, int Ho,
                                                        int Wo, int Co, int G, int KH, int KW, int s, int p) {
  const int Cg = C / G, Cog = Co / G;
  const int cpo = Co >> 3;  // 8 output channels per thread (Cog % 8 == 0 or Cog >= 8 multiple)
  const size_t total = (size_t)N * Ho * Wo * cpo;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int oc = (int)(i % cpo) * 8;
    size_t pix = i / cpo;
    const int wo = (int)(pix % Wo);
    pix /= Wo;
    const int ho = (int)(pix % Ho);
    const int n = (int)(pix / Ho);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int hi = ho * s - p + kh;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int wi = wo * s - p + kw;
        if ((unsigned)wi >= (unsigned)W) continue;
        const bf16* xp = x + (((size_t)n * H + hi) * W + wi) * C;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int co = oc + q;
          const int g = co / Cog;
          const bf16* wp = w + (((size_t)co * KH + kh) * KW + kw) * Cg;
          const bf16* xg = xp + g * Cg;
          float a = 0.f;
          for (int c = 0; c < Cg; ++c) a += bf2f(xg[c]) * bf2f(wp[c]);
          acc[q] += a;
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(y + i * 8) = o;
  }
}

__global__ void __launch_bounds__(256) gconv_dgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w,
                                                          bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                          int Wo, int Co, int G, int KH, int KW, int s, int p) {
  const int Cg = C / G, Cog = Co / G;
  const int cpi = C >> 3;
  const size_t total = (size_t)N * H * W * cpi;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ic = (int)(i % cpi) * 8;
    size_t pix = i / cpi;
    const int wi = (int)(pix % W);
    pix /= W;
    const int hi = (int)(pix % H);
    const int n = (int)(pix / H);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int th = hi + p - kh;
      if (th < 0 || th % s) continue;
      const int ho = th / s;
      if (ho >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = wi + p - kw;
        if (tw < 0 || tw % s) continue;
        const int wo = tw / s;
        if (wo >= Wo) continue;
        const bf16* gp = dy + (((size_t)n * Ho + ho) * Wo + wo) * Co;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int ci = ic + q;
          const int g = ci / Cg, cig = ci - g * Cg;
          float a = 0.f;
          for (int j = 0; j < Cog; ++j) {
            const int co = g * Cog + j;
            a += bf2f(gp[co]) * bf2f(w[(((size_t)co * KH + kh) * KW + kw) * Cg + cig]);
          }
          acc[q] += a;
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(dx + i * 8) = o;
  }
}

// dW[co][kh][kw][cig]: one thread per weight element, workgroup-split over rows; split y writes
// its partial to out + y * nw (reduced by split_reduce -- deterministic, no float atomics)
__global__ void __launch_bounds__(256) gconv_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                          float* __restrict__ out, int N, int H, int W, int C, int Ho,
                                                          int Wo, int Co, int G, int KH, int KW, int s, int p,
                                                          int rows_per_split) {
  const int Cg = C / G, Cog = Co / G;
  const int nw = Co * KH * KW * Cg;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nw) return;
  const int cig = e % Cg;
  int t = e / Cg;
  const int kw = t % KW;
  t /= KW;
  const int kh = t % KH;
  const int co = t / KH;
  const int ci = (co / Cog) * Cg + cig;
  const int M = N * Ho * Wo;
  const int m0 = blockIdx.y * rows_per_split, m1 = min(M, m0 + rows_per_split);
  float acc = 0.f;
  for (int m = m0; m < m1; ++m) {
    const int wo = m % Wo;
    const int q = m / Wo;
    const int ho = q % Ho, n = q / Ho;
    const int hi = ho * s - p + kh, wi = wo * s - p + kw;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) continue;
    acc += bf2f(dy[(size_t)m * Co + co]) * bf2f(x[(((size_t)n * H + hi) * W + wi) * C + ci]);
  }
  out[(size_t)blockIdx.y * nw + e] = acc;
}

// ---------------------------------------------------------------------------
// depthwise k x k filter shared by all channels (blur pool), stride s, pad p
// ---------------------------------------------------------------------------
__device__ __forceinline__ int refl(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

__global__ void __launch_bounds__(256) dwconv_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ f,
                                                         bf16* __restrict__ y, int N, int H, int W, int C, int Ho,
                                                         int Wo, int k, int s, int p, int reflect) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * Ho * Wo * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    size_t pix = i / cpr;
    const int wo = (int)(pix % Wo);
    pix /= Wo;
    const int ho = (int)(pix % Ho);
    const int n = (int)(pix / Ho);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    for (int kh = 0; kh < k; ++kh) {
      int hi = ho * s - p + kh;
      if (reflect) hi = refl(hi, H);
      else if ((unsigned)hi >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        int wi = wo * s - p + kw;
        if (reflect) wi = refl(wi, W);
        else if ((unsigned)wi >= (unsigned)W) continue;
        const float fv = f[kh * k + kw];
        const bf16x8 v = *(const bf16x8*)(x + (((size_t)n * H + hi) * W + wi) * C + ch * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += fv * bf2f(v[q]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(y + i * 8) = o;
  }
}

// backward = scatter of the forward taps; done as a gather over output pixels whose
// (possibly reflected) tap lands on this input pixel
__global__ void __launch_bounds__(256) dwconv_bwd_kernel(const bf16* __restrict__ dy, const float* __restrict__ f,
                                                         bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                         int Wo, int k, int s, int p, int reflect) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * H * W * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    size_t pix = i / cpr;
    const int wi = (int)(pix % W);
    pix /= W;
    const int hi = (int)(pix % H);
    const int n = (int)(pix / H);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    // candidate output rows: any ho whose window (after reflection) touches hi
    // (reflection folds taps near an edge back inside; widen the range there)
    int ho_lo = max(0, (hi + p - k + 1) / s - 1), ho_hi = min(Ho - 1, (hi + p) / s + 1);
    int wo_lo = max(0, (wi + p - k + 1) / s - 1), wo_hi = min(Wo - 1, (wi + p) / s + 1);
    if (reflect) {
      if (hi <= k) ho_lo = 0;
      if (hi >= H - 1 - k) ho_hi = Ho - 1;
      if (wi <= k) wo_lo = 0;
      if (wi >= W - 1 - k) wo_hi = Wo - 1;
    }
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      for (int kh = 0; kh < k; ++kh) {
        int h = ho * s - p + kh;
        if (reflect) h = refl(h, H);
        if (h != hi) continue;
        for (int wo = wo_lo; wo <= wo_hi; ++wo) {
          for (int kw = 0; kw < k; ++kw) {
            int ww = wo * s - p + kw;
            if (reflect) ww = refl(ww, W);
            if (ww != wi) continue;
            const float fv = f[kh * k + kw];
            const bf16x8 g = *(const bf16x8*)(dy + (((size_t)n * Ho + ho) * Wo + wo) * C + ch * 8);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] += fv * bf2f(g[q]);
          }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(dx + i * 8) = o;
  }
}

// ---------------------------------------------------------------------------
// squeeze-and-excitation apply, optionally fused with the block's residual add
// and ReLU:  y[n][hw][c] = act(x[n][hw][c] * g[n][c] (+ res[n][hw][c]))
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) chan_scale_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ g,
                                                             const bf16* __restrict__ res, bf16* __restrict__ y,
                                                             int N, int HW, int C, int relu) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * HW * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    const size_t n = i / cpr / HW;
    const bf16x8 v = *(const bf16x8*)(x + i * 8);
    const bf16x8 s = *(const bf16x8*)(g + n * C + ch * 8);
    bf16x8 r;
    if (res) r = *(const bf16x8*)(res + i * 8);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float z = bf2f(v[q]) * bf2f(s[q]);
      if (res) z += bf2f(r[q]);
      if (relu) z = fmaxf(z, 0.f);
      o[q] = f2bf(z);
    }
    *(bf16x8*)(y + i * 8) = o;
  }
}

// dz = dy * relu'(z);  dx = dz * g ; dg[n][c] = sum_hw dz*x ; dres = dz  (z recomputed from x,
// g, res).  Workgroup (n, s) covers rows [HW s / S, HW (s+1) / S) of image n, 256 / (C/8) rows
// per pass, and writes its dg partial part[s][n][C] (summed by launch_partial_sum): the early
// SE layers (56x56, 64 channels) have few (n, chunk) pairs but many rows.
__global__ void __launch_bounds__(256) chan_scale_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                             const bf16* __restrict__ g, const bf16* __restrict__ res,
                                                             bf16* __restrict__ dx, float* __restrict__ part,
                                                             bf16* __restrict__ dres, int N, int HW, int C,
                                                             int relu) {
  const int n = blockIdx.x, s = blockIdx.y, S = gridDim.y;
  const int cpr = C >> 3, rpp = 256 / cpr;
  const int slot = threadIdx.x / cpr, ch = threadIdx.x - slot * cpr;
  const int r0 = (int)((long long)HW * s / S), r1 = (int)((long long)HW * (s + 1) / S);
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (slot < rpp) {
    const bf16x8 sv = *(const bf16x8*)(g + (size_t)n * C + ch * 8);
    float sc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) sc[q] = bf2f(sv[q]);
    for (int t = r0 + slot; t < r1; t += rpp) {
      const size_t o = ((size_t)n * HW + t) * C + ch * 8;
      const bf16x8 gv = *(const bf16x8*)(dy + o);
      const bf16x8 xv = *(const bf16x8*)(x + o);
      bf16x8 rv;
      if (res) rv = *(const bf16x8*)(res + o);
      bf16x8 d, dz8;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float dz = bf2f(gv[q]);
        if (relu) {
          float z = bf2f(xv[q]) * sc[q];
          if (res) z += bf2f(rv[q]);
          dz = z > 0.f ? dz : 0.f;
        }
        acc[q] += dz * bf2f(xv[q]);
        d[q] = f2bf(dz * sc[q]);
        dz8[q] = f2bf(dz);
      }
      *(bf16x8*)(dx + o) = d;
      if (dres) *(bf16x8*)(dres + o) = dz8;
    }
  }
  __shared__ float red[256 * 8];
#pragma unroll
  for (int q = 0; q < 8; ++q) red[threadIdx.x * 8 + q] = acc[q];
  __syncthreads();
  if (slot == 0) {
    for (int k = 1; k < rpp; ++k)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += red[(k * cpr + ch) * 8 + q];
#pragma unroll
    for (int q = 0; q < 8; ++q) part[((size_t)s * N + n) * C + ch * 8 + q] = acc[q];
  }
}

// ---------------------------------------------------------------------------
static inline int grid_of(size_t n) {
  size_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

bool launch_grouped_conv_fwd(const bf16* x, const bf16* w, bf16* y, bf16* frag, int N, int H, int W, int C, int Ho,
                             int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s, float* stats) {
  if (launch_gconv_mfma_fwd(x, w, y, frag, N, H, W, C, Ho, Wo, Co, G, KH, KW, stride, pad, s, stats))
    return stats != nullptr;
  const size_t total = (size_t)N * Ho * Wo * (Co / 8);
  hipLaunchKernelGGL(gconv_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, s, x, w, y, N, H, W, C, Ho, Wo, Co, G, KH,
                     KW, stride, pad);
  return false;
}
void launch_grouped_conv_dgrad(const bf16* dy, const bf16* w, bf16* dx, bf16* frag, int N, int H, int W, int C,
                               int Ho, int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s) {
  if (launch_gconv_mfma_dgrad(dy, w, dx, frag, N, H, W, C, Ho, Wo, Co, G, KH, KW, stride, pad, s)) return;
  const size_t total = (size_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(gconv_dgrad_kernel, dim3(grid_of(total)), dim3(256), 0, s, dy, w, dx, N, H, W, C, Ho, Wo, Co, G,
                     KH, KW, stride, pad);
}
void launch_grouped_conv_wgrad(const bf16* dy, const bf16* x, float* dw, float* part, int splits, const bf16* zero,
                               int N, int H, int W, int C, int Ho, int Wo, int Co, int G, int KH, int KW, int stride,
                               int pad, hipStream_t s) {
  if (launch_gconv_mfma_wgrad(dy, x, dw, part, splits, zero, N, H, W, C, Ho, Wo, Co, G, KH, KW, stride, pad, s)) return;
  const int M = N * Ho * Wo;
  const int nw = Co * KH * KW * (C / G);
  const int nsplit = gconv_fallback_wgrad_splits(M, nw);
  const int rps = (M + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(gconv_wgrad_kernel, dim3((nw + 255) / 256, nsplit), dim3(256), 0, s, dy, x,
                     nsplit == 1 ? dw : part, N, H, W, C, Ho, Wo, Co, G, KH, KW, stride, pad, rps);
  if (nsplit > 1) launch_split_reduce(part, nsplit, nw, dw, s);
}
// row splits of the direct fallback: ~2048 workgroups, at most 64 (one split_reduce pass), one
// when the weight count is not a multiple of 4 (the float4 reduction)
int gconv_fallback_wgrad_splits(int M, int nw) {
  if (nw % 4) return 1;
  int nsplit = 2048 / ((nw + 255) / 256);
  nsplit = std::min(std::max(nsplit, 1), 64);
  return std::max(1, std::min(nsplit, (M + 63) / 64));
}
void launch_dwconv_fwd(const bf16* x, const float* w, bf16* y, int N, int H, int W, int C, int Ho, int Wo, int k,
                       int s, int p, int reflect, hipStream_t st) {
  const size_t total = (size_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(dwconv_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, st, x, w, y, N, H, W, C, Ho, Wo, k, s, p,
                     reflect);
}
void launch_dwconv_bwd(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C, int Ho, int Wo, int k,
                       int s, int p, int reflect, hipStream_t st) {
  const size_t total = (size_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(dwconv_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, st, dy, w, dx, N, H, W, C, Ho, Wo, k, s,
                     p, reflect);
}
void launch_chan_scale_fwd(const bf16* x, const bf16* g, const bf16* res, bf16* y, int N, int HW, int C, int relu,
                           hipStream_t st) {
  const size_t total = (size_t)N * HW * (C / 8);
  hipLaunchKernelGGL(chan_scale_fwd_kernel, dim3(grid_of(total)), dim3(256), 0, st, x, g, res, y, N, HW, C, relu);
}
void launch_chan_scale_bwd(const bf16* dy, const bf16* x, const bf16* g, const bf16* res, bf16* dx, bf16* dg,
                           float* part, bf16* dres, int N, int HW, int C, int relu, hipStream_t st) {
  const int S = hw_splits(N, HW, C);
  hipLaunchKernelGGL(chan_scale_bwd_kernel, dim3(N, S), dim3(256), 0, st, dy, x, g, res, dx, part, dres, N, HW, C,
                     relu);
  launch_partial_sum_bf16(part, S, N * C, dg, st);  // the gate's gradient in its own dtype: no cast pass
}

// ---------------------------------------------------------------------------
// Squeeze-excitation gate of a SMALL batch, one workgroup per direction, every product on MFMA
// (TResNet-M at the reference's batch 16: 18 gates per step, each a [N, C] x [C, R] and a [N, R] x [R, C]
// product with N = 16, C <= 256, R <= 128, that ran as two GEMM launches forward and ~10 small launches
// backward: sigmoid' and ReLU' passes, two data-gradient GEMMs, two weight-gradient GEMMs + reductions,
// two bias column sums).  The roundings follow that chain: h, g, d2 = dg g (1 - g), dh (then
// d1 = dh [h > 0]) and dp are bf16; weight and bias gradients fp32.
//   forward : h = relu(p W1^T + b1), g = sigmoid(h W2^T + b2)        (p [N,C], W1 [R,C], W2 [C,R])
//   backward: dW2 = d2^T h, db2 = sum_n d2, dh = d2 W2, d1 = dh [h > 0],
//             dW1 = d1^T p, db1 = sum_n d1, dp = d1 W1
// Batch rows are padded to 32 in LDS (zero rows): the n-sums of the weight gradients are one 32-deep
// MFMA k-step.  16 waves take the 16 x 16 output tiles round-robin.
// v_mfma_f32_16x16x32_bf16 operands: A lane l = row (l & 15), k 8 (l >> 4) .. + 7; B the same with
// column (l & 15); D lane l = column (l & 15), rows 4 (l >> 4) .. + 3.
constexpr int kSeN = 32, kSeMaxC = 256, kSeMaxR = 128;

bool se_gate_supported(int N, int C, int R) {
  return N >= 1 && N <= kSeN && C % 32 == 0 && R % 32 == 0 && C <= kSeMaxC && R <= kSeMaxR;
}

namespace {
// D (16 x 16) += A[m0 .. m0+15][0 .. K) x B[n0 .. n0+15][0 .. K)^T, both k-contiguous rows (LDS or global),
// K <= 256: every k-step's fragments are loaded before the MFMA chain (one load round trip per tile
// instead of one per k-step -- the weight fragments come from L2)
__device__ __forceinline__ f32x4 se_mma(const bf16* A, int lda, const bf16* B, int ldb, int K, int lane) {
  const int r = lane & 15, kq = 8 * (lane >> 4);
  constexpr int KS = kSeMaxC / 32;
  bf16x8 a[KS], b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    if (s * 32 < K) {
      a[s] = *(const bf16x8*)(A + r * lda + s * 32 + kq);
      b[s] = *(const bf16x8*)(B + r * ldb + s * 32 + kq);
    }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
    if (s * 32 < K) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b[s], acc, 0, 0, 0);
  return acc;
}
}  // namespace

__global__ void __launch_bounds__(1024) se_gate_fwd_kernel(const bf16* __restrict__ p, const bf16* __restrict__ w1,
                                                          const float* __restrict__ b1, const bf16* __restrict__ w2,
                                                          const float* __restrict__ b2, bf16* __restrict__ h,
                                                          bf16* __restrict__ g, int N, int C, int R) {
  constexpr int LP = kSeMaxC + 8, LH = kSeMaxR + 8;  // row pitches (16-byte skew)
  __shared__ __attribute__((aligned(16))) bf16 sp[kSeN * LP];
  __shared__ __attribute__((aligned(16))) bf16 sh[kSeN * LH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = (N + 15) / 16;
  for (int i = tid; i < 16 * nb * (C / 8); i += blockDim.x) {
    const int n = i / (C / 8), c = (i - n * (C / 8)) * 8;
    *(bf16x8*)(sp + n * LP + c) = n < N ? *(const bf16x8*)(p + (size_t)n * C + c) : bf16x8{};
  }
  __syncthreads();
  // h^T tiles: D[r][n] = W1[r][:] . p[n][:]
  for (int t = wave; t < (R / 16) * nb; t += 16) {
    const int rt = t % (R / 16), nt = t / (R / 16);
    const f32x4 acc = se_mma(w1 + (size_t)rt * 16 * C, C, sp + nt * 16 * LP, LP, C, lane);
    const int n = nt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rt * 16 + 4 * (lane >> 4) + q;
      const bf16 hb = f2bf(fmaxf(acc[q] + (b1 ? b1[r] : 0.f), 0.f));
      sh[n * LH + r] = hb;
      if (n < N) h[(size_t)n * R + r] = hb;
    }
  }
  __syncthreads();
  // g^T tiles: D[c][n] = W2[c][:] . h[n][:]
  for (int t = wave; t < (C / 16) * nb; t += 16) {
    const int ct = t % (C / 16), nt = t / (C / 16);
    const f32x4 acc = se_mma(w2 + (size_t)ct * 16 * R, R, sh + nt * 16 * LH, LH, R, lane);
    const int n = nt * 16 + (lane & 15);
    if (n < N)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = ct * 16 + 4 * (lane >> 4) + q;
        g[(size_t)n * C + c] = f2bf(1.f / (1.f + __expf(-(acc[q] + (b2 ? b2[c] : 0.f)))));
      }
  }
}

// w1t = W1^T [C][ld1t], w2t = W2^T [R][ld2t] (the transposed prepared weights)
__global__ void __launch_bounds__(1024) se_gate_bwd_kernel(const bf16* __restrict__ dg, const bf16* __restrict__ g,
                                                          const bf16* __restrict__ h, const bf16* __restrict__ p,
                                                          const bf16* __restrict__ w1t, int ld1t,
                                                          const bf16* __restrict__ w2t, int ld2t,
                                                          float* __restrict__ dw1, float* __restrict__ db1,
                                                          float* __restrict__ dw2, float* __restrict__ db2,
                                                          bf16* __restrict__ dp, int N, int C, int R) {
  constexpr int LC = kSeMaxC + 8, LR = kSeMaxR + 8, LN = kSeN + 8;
  __shared__ __attribute__((aligned(16))) bf16 sd2[kSeN * LC];    // d2 [n][c]
  __shared__ __attribute__((aligned(16))) bf16 sd2t[kSeMaxC * LN];  // d2^T [c][n]
  __shared__ __attribute__((aligned(16))) bf16 spt[kSeMaxC * LN];   // p^T [c][n]
  __shared__ __attribute__((aligned(16))) bf16 sht[kSeMaxR * LN];   // h^T [r][n]
  __shared__ __attribute__((aligned(16))) bf16 sd1[kSeN * LR];    // d1 [n][r]
  __shared__ __attribute__((aligned(16))) bf16 sd1t[kSeMaxR * LN];  // d1^T [r][n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = (N + 15) / 16;
  for (int i = tid; i < kSeN * C; i += blockDim.x) {
    const int n = i / C, c = i - n * C;
    bf16 d = f2bf(0.f), pv = f2bf(0.f);
    if (n < N) {
      const float gv = bf2f(g[(size_t)n * C + c]);
      d = f2bf(bf2f(dg[(size_t)n * C + c]) * gv * (1.f - gv));
      pv = p[(size_t)n * C + c];
    }
    sd2[n * LC + c] = d;
    sd2t[c * LN + n] = d;
    spt[c * LN + n] = pv;
  }
  for (int i = tid; i < kSeN * R; i += blockDim.x) {
    const int n = i / R, r = i - n * R;
    sht[r * LN + n] = n < N ? h[(size_t)n * R + r] : f2bf(0.f);
  }
  __syncthreads();
  // dW2 [c][r] = sum_n d2^T[c][n] h^T[r][n]: one 32-deep k-step per tile
  for (int t = wave; t < (C / 16) * (R / 16); t += 16) {
    const int ct = t / (R / 16), rt = t - ct * (R / 16);
    const f32x4 acc = se_mma(sd2t + ct * 16 * LN, LN, sht + rt * 16 * LN, LN, kSeN, lane);
    const int r = rt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) dw2[(size_t)(ct * 16 + 4 * (lane >> 4) + q) * R + r] = acc[q];
  }
  for (int c = tid; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < N; ++n) a += bf2f(sd2t[c * LN + n]);
    db2[c] = a;
  }
  // dh [n][r] = d2[n][:] . W2^T[r][:] -> d1 = bf16(dh) [h > 0]
  for (int t = wave; t < nb * (R / 16); t += 16) {
    const int nt = t / (R / 16), rt = t - nt * (R / 16);
    const f32x4 acc = se_mma(sd2 + nt * 16 * LC, LC, w2t + (size_t)rt * 16 * ld2t, ld2t, C, lane);
    const int r = rt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nt * 16 + 4 * (lane >> 4) + q;
      const bf16 d = (n < N && bf2f(sht[r * LN + n]) > 0.f) ? f2bf(acc[q]) : f2bf(0.f);
      sd1[n * LR + r] = d;
      sd1t[r * LN + n] = d;
    }
  }
  // rows n in [16 nb, 32) of d1^T: zero (the dW1 k-step reads all 32)
  for (int i = tid; i < (kSeN - 16 * nb) * R; i += blockDim.x) {
    const int n = 16 * nb + i / R, r = i % R;
    sd1t[r * LN + n] = f2bf(0.f);
  }
  __syncthreads();
  // dW1 [r][c] = sum_n d1^T[r][n] p^T[c][n]
  for (int t = wave; t < (R / 16) * (C / 16); t += 16) {
    const int rt = t / (C / 16), ct = t - rt * (C / 16);
    const f32x4 acc = se_mma(sd1t + rt * 16 * LN, LN, spt + ct * 16 * LN, LN, kSeN, lane);
    const int c = ct * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) dw1[(size_t)(rt * 16 + 4 * (lane >> 4) + q) * C + c] = acc[q];
  }
  for (int r = tid; r < R; r += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < N; ++n) a += bf2f(sd1t[r * LN + n]);
    db1[r] = a;
  }
  // dp [n][c] = d1[n][:] . W1^T[c][:]
  for (int t = wave; t < nb * (C / 16); t += 16) {
    const int nt = t / (C / 16), ct = t - nt * (C / 16);
    const f32x4 acc = se_mma(sd1 + nt * 16 * LR, LR, w1t + (size_t)ct * 16 * ld1t, ld1t, R, lane);
    const int c = ct * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nt * 16 + 4 * (lane >> 4) + q;
      if (n < N) dp[(size_t)n * C + c] = f2bf(acc[q]);
    }
  }
}

void launch_se_gate_fwd(const bf16* p, const bf16* w1, const float* b1, const bf16* w2, const float* b2, bf16* h,
                        bf16* g, int N, int C, int R, hipStream_t st) {
  hipLaunchKernelGGL(se_gate_fwd_kernel, dim3(1), dim3(1024), 0, st, p, w1, b1, w2, b2, h, g, N, C, R);
}

void launch_se_gate_bwd(const bf16* dg, const bf16* g, const bf16* h, const bf16* p, const bf16* w1t, int ld1t,
                        const bf16* w2t, int ld2t, float* dw1, float* db1, float* dw2, float* db2, bf16* dp, int N,
                        int C, int R, hipStream_t st) {
  hipLaunchKernelGGL(se_gate_bwd_kernel, dim3(1), dim3(1024), 0, st, dg, g, h, p, w1t, ld1t, w2t, ld2t, dw1, db1, dw2,
                     db2, dp, N, C, R);
}

}  // namespace dcp
