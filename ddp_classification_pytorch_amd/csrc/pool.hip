// Pooling and small layout kernels, NHWC bf16.
//
// Replaces the ATen max-pool (stem, NESTED/model/imagenet_resnet.py:111),
// average pool (:116 AvgPool2d(7) / torchvision AdaptiveAvgPool2d) and
// TResNet's SpaceToDepth stem (timm).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.cuh"
#include "pool_gather.cuh"
#include "launchers.h"

namespace dcp {

// 32-bit decode of a flat (pixel, 8-channel chunk) index i = ((n*H + y)*W + x)*cpr + ch with
// magic-number divisions (64-bit integer division is emulated on the GPU and dominated these
// memory-bound kernels); chunk indices < 2^31 are checked on the host, element offsets are
// 64-bit (the R101 b3072 stem pool output is 2.47e9 elements)
struct PixDiv {
  FastDiv cpr, w, h;
  __device__ __forceinline__ void decode(uint32_t i, int& ch, int& x, int& y, int& n) const {
    const uint32_t pix = fdiv(i, cpr);
    ch = (int)(i - pix * cpr.d);
    const uint32_t q = fdiv(pix, w);
    x = (int)(pix - q * w.d);
    const uint32_t nn = fdiv(q, h);
    y = (int)(q - nn * h.d);
    n = (int)nn;
  }
};

static inline PixDiv make_pixdiv(int cpr, int W, int H) {
  return PixDiv{make_fastdiv(cpr), make_fastdiv(W), make_fastdiv(H)};
}

// max pool k x k / stride s / pad p; 8 channels per thread; argmax as window index
// With `scale` != nullptr the input is a BN layer's INPUT and every window element is first
// mapped through bf16(act(x*scale + shift)) (act: 0 none, 1 ReLU): the stem's BN-apply + ReLU
// fused into the pool, so the full-resolution activation is never written (it is recomputed
// from x in the backward, maxpool_bn_bwd_kernel).
// KK/SS/PP > 0: compile-time window geometry (the ResNet stem's 3x3/2 pad 1: divisions by the
// stride become shifts); 0: runtime k, s, p
template <int KK, int SS, int PP>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                          int Ho, int Wo, int k_, int s_, int p_,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int act, PixDiv dv) {
  const int k = KK ? KK : k_, s = SS ? SS : s_, p = KK ? PP : p_;
  const int cpr = C >> 3;
  const uint32_t total = (uint32_t)N * Ho * Wo * cpr;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int ch, wo, ho, n;
    dv.decode(i, ch, wo, ho, n);
    float best[8], sc[8], sh[8];
    uint8_t bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      bi[q] = 0;
      sc[q] = scale ? scale[ch * 8 + q] : 1.f;
      sh[q] = scale ? shift[ch * 8 + q] : 0.f;
    }
    if constexpr (KK > 0) {
      // compile-time window: all KK*KK loads issued up front from clamped addresses, taps
      // outside the image masked afterwards (a branch per tap serialised the loads)
      bf16x8 v[KK * KK];
      bool ok[KK * KK];
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int kw = 0; kw < KK; ++kw) {
          const int hi = ho * SS - PP + kh, wi = wo * SS - PP + kw;
          ok[kh * KK + kw] = ((unsigned)hi < (unsigned)H) & ((unsigned)wi < (unsigned)W);
          const int hc = min(max(hi, 0), H - 1), wc = min(max(wi, 0), W - 1);
          v[kh * KK + kw] = *(const bf16x8*)(x + (size_t)((uint32_t)(n * H + hc) * W + wc) * C + ch * 8);
        }
#pragma unroll
      for (int t = 0; t < KK * KK; ++t)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float f = bf2f(v[t][q]);
          if (scale) {
            f = f * sc[q] + sh[q];
            if (act == 1) f = fmaxf(f, 0.f);
            f = bf2f(f2bf(f));  // the bf16 activation the unfused BN kernel would have stored
          }
          const bool take = ok[t] & (f > best[q]);  // first maximum in window order, as below
          best[q] = take ? f : best[q];
          bi[q] = take ? (uint8_t)t : bi[q];
        }
    } else {
      for (int kh = 0; kh < k; ++kh) {
        const int hi = ho * s - p + kh;
        if ((unsigned)hi >= (unsigned)H) continue;
        for (int kw = 0; kw < k; ++kw) {
          const int wi = wo * s - p + kw;
          if ((unsigned)wi >= (unsigned)W) continue;
          const bf16x8 v = *(const bf16x8*)(x + (size_t)((uint32_t)(n * H + hi) * W + wi) * C + ch * 8);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float f = bf2f(v[q]);
            if (scale) {
              f = f * sc[q] + sh[q];
              if (act == 1) f = fmaxf(f, 0.f);
              f = bf2f(f2bf(f));  // the bf16 activation the unfused BN kernel would have stored
            }
            if (f > best[q]) {
              best[q] = f;
              bi[q] = (uint8_t)(kh * k + kw);
            }
          }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(best[q]);
    *(bf16x8*)(y + (size_t)i * 8) = o;
    if (idx) {
      uint64_t packed = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) packed |= (uint64_t)bi[q] << (8 * q);
      *(uint64_t*)(idx + (size_t)i * 8) = packed;
    }
  }
}

// gather form of the max-pool backward: every input pixel sums the output
// gradients whose window argmax points at it (deterministic, no atomics)
template <int KK, int SS, int PP>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                          int Wo, int k_, int s_, int p_, PixDiv dv) {
  const int k = KK ? KK : k_, s = SS ? SS : s_, p = KK ? PP : p_;
  const int cpr = C >> 3;
  const uint32_t total = (uint32_t)N * H * W * cpr;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int ch, wi, hi, n;
    dv.decode(i, ch, wi, hi, n);
    float acc[8];
    gather_pool_grad<KK, SS, PP>(dy, idx, n, hi, wi, Ho, Wo, C, ch, k, s, p, acc);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(dx + (size_t)i * 8) = o;
  }
}

// Backward of BN(+act) followed by the max pool, from the pooled gradient dy and the window
// argmax: every input pixel gathers its gradient g from the <= ceil(k/s)^2 windows whose argmax
// points at it, masks it with act'(x*scale + shift), then
//   PASS 0: per-workgroup partial (sum g', sum g' * (x - mean) * invstd)  -> part[block][2][C]
//   PASS 1: dx = a*g' + b*x + c with the BN coefficients folded from the global sums
// (the unfused chain wrote the full-resolution pool gradient and read it twice).
// Requires 256 % (C/8) == 0 so each thread keeps one 8-channel chunk for the whole grid stride.
template <int PASS, int KK, int SS, int PP>
__global__ void __launch_bounds__(256) maxpool_bn_bwd_kernel(const bf16* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx,
                                                             const bf16* __restrict__ x, int N, int H, int W, int C,
                                                             int Ho, int Wo, int k_, int s_, int p_,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, int act,
                                                             const float* __restrict__ sums, float inv_count,
                                                             float* __restrict__ part, bf16* __restrict__ dx,
                                                             PixDiv dv) {
  const int k = KK ? KK : k_, s = SS ? SS : s_, p = KK ? PP : p_;
  const int cpr = C >> 3;
  const int ch = threadIdx.x % cpr;
  float sc[8], sh[8], mu[8], ca[8], cb[8], cc[8], s1[8], s2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = ch * 8 + q;
    sc[q] = scale[c];
    sh[q] = shift[c];
    mu[q] = mean[c];
    s1[q] = s2[q] = 0.f;
    if (PASS == 1) {
      const float is = invstd[c];
      const float a2 = sums[c] * inv_count, a3 = sums[C + c] * inv_count * is;
      ca[q] = sc[q];
      cb[q] = -sc[q] * a3;
      cc[q] = -sc[q] * a2 + sc[q] * a3 * mu[q];
    }
  }
  const uint32_t total = (uint32_t)N * H * W * cpr;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int chd, wi, hi, n;
    dv.decode(i, chd, wi, hi, n);
    float g[8];
    const bf16x8 xv = *(const bf16x8*)(x + (size_t)i * 8);
    gather_pool_grad<KK, SS, PP>(dy, idx, n, hi, wi, Ho, Wo, C, ch, k, s, p, g);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float xf = bf2f(xv[q]);
      float gq = bf2f(f2bf(g[q]));  // the bf16 pool gradient of the unfused chain
      if (act == 1 && !(xf * sc[q] + sh[q] > 0.f)) gq = 0.f;
      if (PASS == 0) {
        s1[q] += gq;
        s2[q] += gq * (xf - mu[q]);
      } else {
        o[q] = f2bf(ca[q] * gq + cb[q] * xf + cc[q]);
      }
    }
    if (PASS == 1) *(bf16x8*)(dx + (size_t)i * 8) = o;
  }
  if (PASS == 0) {
    __shared__ float red[2][256][8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[0][threadIdx.x][q] = s1[q];
      red[1][threadIdx.x][q] = s2[q] * invstd[ch * 8 + q];
    }
    __syncthreads();
    if ((int)threadIdx.x < cpr * 8 * 2) {
      const int which = threadIdx.x / (cpr * 8), c = threadIdx.x % (cpr * 8);
      const int cch = c >> 3, q = c & 7;
      float t = 0.f;
      for (int r = cch; r < 256; r += cpr) t += red[which][r][q];
      part[((size_t)blockIdx.x * 2 + which) * C + c] = t;
    }
  }
}

// global average pool [N][HW][C] -> [N][C] (bf16 out, fp32 accumulate), two levels so that
// early, large-HW layers (TResNet's SE blocks at 56x56 / 64 channels) spread over the chip:
// workgroup (n, s) sums rows [HW s / S, HW (s+1) / S) of image n -> part[s][n][C]; then
// gap_final sums the S partials of each (n, c).  C <= 2048 (one 8-channel chunk per thread).
__device__ __forceinline__ void rows_sum8(const bf16* __restrict__ base, int r0, int r1, int rpp, int C, float* acc) {
  int r = r0;
  for (; r + 3 * rpp < r1; r += 4 * rpp) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(base + (size_t)(r + u * rpp) * C);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[u][q]);
  }
  for (; r < r1; r += rpp) {
    const bf16x8 v = *(const bf16x8*)(base + (size_t)r * C);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[q]);
  }
}

__global__ void __launch_bounds__(256) gap_partial_kernel(const bf16* __restrict__ x, float* __restrict__ part, int N,
                                                          int HW, int C) {
  const int n = blockIdx.x, s = blockIdx.y, S = gridDim.y;
  const int cpr = C >> 3, rpp = 256 / cpr;
  const int slot = threadIdx.x / cpr, ch = threadIdx.x - slot * cpr;
  const int r0 = (int)((long long)HW * s / S), r1 = (int)((long long)HW * (s + 1) / S);
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (slot < rpp) rows_sum8(x + (size_t)n * HW * C + ch * 8, r0 + slot, r1, rpp, C, acc);
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

__global__ void __launch_bounds__(256) gap_final_kernel(const float* __restrict__ part, bf16* __restrict__ y, int NC,
                                                        int S, float inv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NC) return;
  float t = 0.f;
  for (int s = 0; s < S; ++s) t += part[(size_t)s * NC + i];
  y[i] = f2bf(t * inv);
}

// dx = broadcast(dy / HW) (+ add: the other consumers' gradient of the pooled tensor, e.g. a
// squeeze-excitation block's channel-scale dgrad -- summed here instead of by an extra add pass)
__global__ void __launch_bounds__(256) gap_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N,
                                                      int HW, int C, const bf16* __restrict__ add) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * HW * cpr;
  const float inv = 1.f / HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    const size_t n = i / cpr / HW;
    const bf16x8 g = *(const bf16x8*)(dy + n * C + ch * 8);
    bf16x8 o;
    if (add) {
      const bf16x8 a = *(const bf16x8*)(add + i * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(fmaf(bf2f(g[q]), inv, bf2f(a[q])));
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(bf2f(g[q]) * inv);
    }
    *(bf16x8*)(dx + i * 8) = o;
  }
}

// space-to-depth (block b): [N][H][W][C] -> [N][H/b][W/b][b*b*C], channel order (bh, bw, c)
__global__ void __launch_bounds__(256) s2d_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H,
                                                  int W, int C, int b, int inverse) {
  const int Ho = H / b, Wo = W / b;
  const size_t total = (size_t)N * H * W * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const int ho = h / b, bh = h - ho * b, wo = w / b, bw = w - wo * b;
    const size_t o = (((size_t)n * Ho + ho) * Wo + wo) * (b * b * C) + (bh * b + bw) * C + c;
    if (inverse)
      y[i] = x[o];
    else
      y[o] = x[i];
  }
}

// one (pixel, 8-channel chunk) per thread: the memory-bound passes reach HBM rate only with
// the whole tensor's loads spread over many short-lived waves (see bn.hip ew_grid)
static inline int ew_grid2(size_t n) {
  size_t g = (n + 255) / 256;
  if (g > (1u << 20)) g = 1u << 20;
  if (g < 1) g = 1;
  return (int)g;
}

static void check_flat(size_t elems) {
  if (elems / 8 >= (1ull << 31)) {
    fprintf(stderr, "pool kernels: tensor of %zu elements exceeds the 2^31 8-channel-chunk index range\n", elems);
    abort();
  }
}

void launch_maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo, int k,
                        int s, int p, hipStream_t st, const float* scale, const float* shift, int act) {
  const size_t total = (size_t)N * Ho * Wo * (C / 8);
  check_flat((size_t)N * H * W * C);
  check_flat((size_t)N * Ho * Wo * C);
  const PixDiv dv = make_pixdiv(C / 8, Wo, Ho);
  if (k == 3 && s == 2 && p == 1)
    hipLaunchKernelGGL((maxpool_fwd_kernel<3, 2, 1>), dim3(ew_grid2(total)), dim3(256), 0, st, x, y, idx, N, H, W, C,
                       Ho, Wo, k, s, p, scale, shift, act, dv);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<0, 0, 0>), dim3(ew_grid2(total)), dim3(256), 0, st, x, y, idx, N, H, W, C,
                       Ho, Wo, k, s, p, scale, shift, act, dv);
}

int maxpool_bn_bwd_blocks() { return 8192; }

void launch_maxpool_bn_bwd(const bf16* dy, const uint8_t* idx, const bf16* x, int N, int H, int W, int C, int Ho,
                           int Wo, int k, int s, int p, const float* scale, const float* shift, const float* mean,
                           const float* invstd, int act, float* part, float* sums_out, const float* sums,
                           float inv_count, bf16* dx, hipStream_t st) {
  const size_t total = (size_t)N * H * W * (C / 8);
  check_flat((size_t)N * H * W * C);
  const PixDiv dv = make_pixdiv(C / 8, W, H);
  const bool stem = k == 3 && s == 2 && p == 1;
  if (dx == nullptr) {
    const int g = maxpool_bn_bwd_blocks();
    if (stem)
      hipLaunchKernelGGL((maxpool_bn_bwd_kernel<0, 3, 2, 1>), dim3(g), dim3(256), 0, st, dy, idx, x, N, H, W, C, Ho,
                         Wo, k, s, p, scale, shift, mean, invstd, act, nullptr, 0.f, part, nullptr, dv);
    else
      hipLaunchKernelGGL((maxpool_bn_bwd_kernel<0, 0, 0, 0>), dim3(g), dim3(256), 0, st, dy, idx, x, N, H, W, C, Ho,
                         Wo, k, s, p, scale, shift, mean, invstd, act, nullptr, 0.f, part, nullptr, dv);
    launch_partial_sum(part, g, 2 * C, sums_out, st);
  } else {
    // grid-stride over 8192 workgroups: the windows' overlapping dy / argmax reads stay in the
    // L2 of the XCD walking them (a one-shot grid measured 583 -> 747 us on the R50 stem)
    const int g = std::min(ew_grid2(total), 8192);
    if (stem)
      hipLaunchKernelGGL((maxpool_bn_bwd_kernel<1, 3, 2, 1>), dim3(g), dim3(256), 0, st, dy, idx, x, N,
                         H, W, C, Ho, Wo, k, s, p, scale, shift, mean, invstd, act, sums, inv_count, nullptr, dx, dv);
    else
      hipLaunchKernelGGL((maxpool_bn_bwd_kernel<1, 0, 0, 0>), dim3(g), dim3(256), 0, st, dy, idx, x, N,
                         H, W, C, Ho, Wo, k, s, p, scale, shift, mean, invstd, act, sums, inv_count, nullptr, dx, dv);
  }
}

void launch_maxpool_bwd(const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st) {
  const size_t total = (size_t)N * H * W * (C / 8);
  check_flat((size_t)N * H * W * C);
  const PixDiv dv = make_pixdiv(C / 8, W, H);
  if (k == 3 && s == 2 && p == 1)
    hipLaunchKernelGGL((maxpool_bwd_kernel<3, 2, 1>), dim3(ew_grid2(total)), dim3(256), 0, st, dy, idx, dx, N, H, W,
                       C, Ho, Wo, k, s, p, dv);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<0, 0, 0>), dim3(ew_grid2(total)), dim3(256), 0, st, dy, idx, dx, N, H, W,
                       C, Ho, Wo, k, s, p, dv);
}

// row splits per image of the two-level per-(n, c) reductions over HW: ~2048 workgroups in
// total, at least 4 passes of rows each
int hw_splits(int N, int HW, int C) {
  const int rpp = 256 / (C / 8);
  int S = (2048 + N - 1) / N;
  S = std::min(S, std::max(1, HW / (4 * rpp)));
  return std::max(1, std::min(S, 64));
}

void launch_gap_fwd(const bf16* x, bf16* y, float* part, int N, int HW, int C, hipStream_t st) {
  const int S = hw_splits(N, HW, C);
  hipLaunchKernelGGL(gap_partial_kernel, dim3(N, S), dim3(256), 0, st, x, part, N, HW, C);
  hipLaunchKernelGGL(gap_final_kernel, dim3((N * C + 255) / 256), dim3(256), 0, st, part, y, N * C, S, 1.f / HW);
}

void launch_gap_bwd(const bf16* dy, bf16* dx, int N, int HW, int C, hipStream_t st, const bf16* add) {
  const size_t total = (size_t)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, dy, dx, N, HW, C, add);
}

void launch_s2d(const bf16* x, bf16* y, int N, int H, int W, int C, int b, int inverse, hipStream_t st) {
  const size_t total = (size_t)N * H * W * C;
  hipLaunchKernelGGL(s2d_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, x, y, N, H, W, C, b, inverse);
}


// ---------------------------------------------------------------------------
// Adaptive average pool NHWC -> [N, OH, OW, C] (torchvision VGG's AdaptiveAvgPool2d((7, 7)),
// NESTED/model/vgg.py:48): output cell (oh, ow) averages rows [floor(oh H / OH), ceil((oh+1) H / OH))
// and the same for columns.  Backward: each input pixel gathers the cells whose window holds it.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int ad_start(int o, int I, int O) { return (o * I) / O; }
__device__ __forceinline__ int ad_end(int o, int I, int O) { return ((o + 1) * I + O - 1) / O; }

__global__ void __launch_bounds__(256) adaptive_avg_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                               int H, int W, int C, int OH, int OW) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * OH * OW * cpr;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int ch = (int)(i % cpr);
    size_t t = i / cpr;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    const int h0 = ad_start(oh, H, OH), h1 = ad_end(oh, H, OH), w0 = ad_start(ow, W, OW), w1 = ad_end(ow, W, OW);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        const bf16x8 v = *(const bf16x8*)(x + (((size_t)n * H + h) * W + w) * C + ch * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
      }
    const float inv = 1.f / (float)((h1 - h0) * (w1 - w0));
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e] * inv);
    *(bf16x8*)(y + (((size_t)n * OH + oh) * OW + ow) * C + ch * 8) = o;
  }
}

__global__ void __launch_bounds__(256) adaptive_avg_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                               int N, int H, int W, int C, int OH, int OW) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * H * W * cpr;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int ch = (int)(i % cpr);
    size_t t = i / cpr;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // cells whose window holds row h: oh in [floor(h OH / H) - 1, ...] -- scan the (few) candidates
    const int oh_lo = max(0, (h * OH) / H - 1), oh_hi = min(OH - 1, ((h + 1) * OH) / H + 1);
    const int ow_lo = max(0, (w * OW) / W - 1), ow_hi = min(OW - 1, ((w + 1) * OW) / W + 1);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int h0 = ad_start(oh, H, OH), h1 = ad_end(oh, H, OH);
      if (h < h0 || h >= h1) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int w0 = ad_start(ow, W, OW), w1 = ad_end(ow, W, OW);
        if (w < w0 || w >= w1) continue;
        const float inv = 1.f / (float)((h1 - h0) * (w1 - w0));
        const bf16x8 g = *(const bf16x8*)(dy + (((size_t)n * OH + oh) * OW + ow) * C + ch * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(g[e]) * inv;
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    *(bf16x8*)(dx + i * 8) = o;
  }
}

void launch_adaptive_avg(const bf16* src, bf16* dst, int N, int H, int W, int C, int OH, int OW, bool backward,
                         hipStream_t s) {
  const size_t total = (size_t)N * (backward ? H * W : OH * OW) * (C / 8);
  size_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (backward)
    hipLaunchKernelGGL(adaptive_avg_bwd_kernel, dim3((int)g), dim3(256), 0, s, src, dst, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(adaptive_avg_fwd_kernel, dim3((int)g), dim3(256), 0, s, src, dst, N, H, W, C, OH, OW);
}

}  // namespace dcp
