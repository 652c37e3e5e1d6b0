// Pooling and small layout kernels, NHWC bf16.
//
// Replaces the ATen max-pool (stem, NESTED/model/imagenet_resnet.py:111),
// average pool (:116 AvgPool2d(7) / torchvision AdaptiveAvgPool2d) and
// TResNet's SpaceToDepth stem (timm).
#include "common.cuh"
#include "launchers.h"

namespace dcp {

// max pool k x k / stride s / pad p; 8 channels per thread; argmax as window index
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                          int Ho, int Wo, int k, int s, int p) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * Ho * Wo * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    size_t pix = i / cpr;
    const int wo = (int)(pix % Wo);
    pix /= Wo;
    const int ho = (int)(pix % Ho);
    const int n = (int)(pix / Ho);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      bi[q] = 0;
    }
    for (int kh = 0; kh < k; ++kh) {
      const int hi = ho * s - p + kh;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int wi = wo * s - p + kw;
        if ((unsigned)wi >= (unsigned)W) continue;
        const bf16x8 v = *(const bf16x8*)(x + (((size_t)n * H + hi) * W + wi) * C + ch * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float f = bf2f(v[q]);
          if (f > best[q]) {
            best[q] = f;
            bi[q] = (uint8_t)(kh * k + kw);
          }
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(best[q]);
    *(bf16x8*)(y + i * 8) = o;
    if (idx) {
      uint64_t packed = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) packed |= (uint64_t)bi[q] << (8 * q);
      *(uint64_t*)(idx + i * 8) = packed;
    }
  }
}

// gather form of the max-pool backward: every input pixel sums the output
// gradients whose window argmax points at it (deterministic, no atomics)
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          bf16* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                          int Wo, int k, int s, int p) {
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
    // ho*s - p <= hi <= ho*s - p + k - 1
    const int ho_lo = max(0, (hi + p - k + s) / s);  // ceil((hi+p-k+1)/s) for non-negative numerators
    const int ho_hi = min(Ho - 1, (hi + p) / s);
    const int wo_lo = max(0, (wi + p - k + s) / s);
    const int wo_hi = min(Wo - 1, (wi + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = hi - (ho * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = wi - (wo * s - p);
        if (kw < 0 || kw >= k) continue;
        const size_t o = (((size_t)n * Ho + ho) * Wo + wo) * C + ch * 8;
        const uint64_t packed = *(const uint64_t*)(idx + o);
        const bf16x8 g = *(const bf16x8*)(dy + o);
        const uint8_t want = (uint8_t)(kh * k + kw);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (((packed >> (8 * q)) & 0xff) == want) acc[q] += bf2f(g[q]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(bf16x8*)(dx + i * 8) = o;
  }
}

// global average pool [N][HW][C] -> [N][C] (bf16 out, fp32 accumulate)
__global__ void __launch_bounds__(256) gap_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                      int HW, int C) {
  const int cpr = C >> 3;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * cpr) return;
  const int n = i / cpr, ch = i - n * cpr;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  const bf16* base = x + (size_t)n * HW * C + ch * 8;
  for (int t = 0; t < HW; ++t) {
    const bf16x8 v = *(const bf16x8*)(base + (size_t)t * C);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[q]);
  }
  const float inv = 1.f / HW;
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q] * inv);
  *(bf16x8*)(y + (size_t)n * C + ch * 8) = o;
}

__global__ void __launch_bounds__(256) gap_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int N,
                                                      int HW, int C) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * HW * cpr;
  const float inv = 1.f / HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cpr);
    const size_t n = i / cpr / HW;
    const bf16x8 g = *(const bf16x8*)(dy + n * C + ch * 8);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(bf2f(g[q]) * inv);
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

static inline int ew_grid2(size_t n) {
  size_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_maxpool_fwd(const bf16* x, bf16* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo, int k,
                        int s, int p, hipStream_t st) {
  const size_t total = (size_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, x, y, idx, N, H, W, C, Ho, Wo, k,
                     s, p);
}

void launch_maxpool_bwd(const bf16* dy, const uint8_t* idx, bf16* dx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st) {
  const size_t total = (size_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, dy, idx, dx, N, H, W, C, Ho, Wo,
                     k, s, p);
}

void launch_gap_fwd(const bf16* x, bf16* y, int N, int HW, int C, hipStream_t st) {
  const int n = N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, st, x, y, N, HW, C);
}

void launch_gap_bwd(const bf16* dy, bf16* dx, int N, int HW, int C, hipStream_t st) {
  const size_t total = (size_t)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, dy, dx, N, HW, C);
}

void launch_s2d(const bf16* x, bf16* y, int N, int H, int W, int C, int b, int inverse, hipStream_t st) {
  const size_t total = (size_t)N * H * W * C;
  hipLaunchKernelGGL(s2d_kernel, dim3(ew_grid2(total)), dim3(256), 0, st, x, y, N, H, W, C, b, inverse);
}

}  // namespace dcp
