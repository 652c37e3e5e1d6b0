// Fused multi-tensor optimizer steps and the CDR critical-parameter gradient
// mask.
//
// * SGD (momentum, dampening, weight decay, nesterov) and Adam/AdamW replace
//   torch.optim.SGD/Adam used at BASELINE/main.py:153, ARCFACE/arc_main.py:249-253,
//   CDR/main.py:339, NESTED/train.py:386-392, PLC/utils.py:237 (SURVEY.md
//   §2.5 K14/K15). One launch updates every parameter: a device table lists
//   (param, grad, state, bf16 shadow) per tensor and a chunk table maps
//   workgroups to 4096-element slices.  The step optionally refreshes the
//   bf16 compute copy of each weight, so the forward pass reads weights that
//   the optimizer already converted.
// * CDR (CDR/main.py:186-204): threshold = k-th largest |g*w| over all 2-D/4-D
//   parameters, found by a 4-pass 8-bit radix select over the float bit
//   patterns (non-negative floats order like their uint32 bits) without
//   materialising the 25.6M-element concatenation or sorting it; then
//   g *= (|g*w| >= thr) * clip in place.
#include "common.cuh"
#include "launchers.h"

namespace dcp {


constexpr int kChunk = 4096;


__global__ void __launch_bounds__(256) mt_sgd_kernel(const MTEntry* __restrict__ tab, const int2* __restrict__ chunks,
                                                     SgdHyper h) {
  const int2 ck = chunks[blockIdx.x];
  const MTEntry e = tab[ck.x];
  const int64_t base = (int64_t)ck.y * kChunk;
  const int64_t end = min(e.n, base + kChunk);
  // 16-byte path (uniform per chunk): the 4-byte loop kept one 4-byte load per lane and tensor in
  // flight per iteration (96 us for ResNet-50's 25.6M parameters, ~5.3 TB/s); the per-element math
  // is the same, so both paths give identical results.  Bucket views at odd offsets take the scalar
  // loop.
  const uintptr_t mis = ((uintptr_t)(e.p + base) | (uintptr_t)(e.g + base) |
                         (h.momentum != 0.f ? (uintptr_t)(e.s1 + base) : 0)) & 15u;
  const uintptr_t smis = e.shadow ? ((uintptr_t)(e.shadow + base) & 7u) : 0;
  if (mis == 0 && smis == 0 && ((end - base) & 3) == 0) {
    const int64_t n4 = (end - base) >> 2;
    float4* p4 = (float4*)(e.p + base);
    const float4* g4 = (const float4*)(e.g + base);
    float4* s4 = (float4*)(e.s1 + base);
#pragma unroll 4
    for (int64_t j = threadIdx.x; j < n4; j += blockDim.x) {
      float gv[4], pv[4], bv[4];
      *(float4*)gv = g4[j];
      *(float4*)pv = p4[j];
      const bool mom = h.momentum != 0.f;
      if (mom && !h.first) *(float4*)bv = s4[j];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float g = gv[u] * h.grad_scale;
        if (h.wd != 0.f) g += h.wd * pv[u];
        if (mom) {
          const float b = h.first ? g : h.momentum * bv[u] + (1.f - h.dampening) * g;
          bv[u] = b;
          g = h.nesterov ? g + h.momentum * b : b;
        }
        pv[u] -= h.lr * g;
      }
      if (mom) s4[j] = *(float4*)bv;
      p4[j] = *(float4*)pv;
      if (e.shadow) {
        bf16x4 sv;
#pragma unroll
        for (int u = 0; u < 4; ++u) sv[u] = f2bf(pv[u]);
        *(bf16x4*)(e.shadow + base + 4 * j) = sv;
      }
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    float g = e.g[i] * h.grad_scale;
    float p = e.p[i];
    if (h.wd != 0.f) g += h.wd * p;
    if (h.momentum != 0.f) {
      float b;
      if (h.first)
        b = g;
      else
        b = h.momentum * e.s1[i] + (1.f - h.dampening) * g;
      e.s1[i] = b;
      g = h.nesterov ? g + h.momentum * b : b;
    }
    p -= h.lr * g;
    e.p[i] = p;
    if (e.shadow) e.shadow[i] = f2bf(p);
  }
}


__global__ void __launch_bounds__(256) mt_adam_kernel(const MTEntry* __restrict__ tab, const int2* __restrict__ chunks,
                                                      AdamHyper h) {
  const int2 ck = chunks[blockIdx.x];
  const MTEntry e = tab[ck.x];
  const int64_t base = (int64_t)ck.y * kChunk;
  const int64_t end = min(e.n, base + kChunk);
  float bc1 = h.bc1, bc2 = h.bc2;
  if (h.step_dev) {  // 1 - beta^t without the cancellation of 1 - powf
    const float t = (float)*h.step_dev;
    bc1 = -expm1f(t * logf(h.beta1));
    bc2 = -expm1f(t * logf(h.beta2));
  }
  const float rbc2 = 1.f / sqrtf(bc2);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    float g = e.g[i] * h.grad_scale;
    float p = e.p[i];
    if (h.wd != 0.f) {
      if (h.decoupled)
        p *= 1.f - h.lr * h.wd;
      else
        g += h.wd * p;
    }
    const float m = h.beta1 * e.s1[i] + (1.f - h.beta1) * g;
    const float v = h.beta2 * e.s2[i] + (1.f - h.beta2) * g * g;
    e.s1[i] = m;
    e.s2[i] = v;
    const float denom = sqrtf(v) * rbc2 + h.eps;
    p -= (h.lr / bc1) * m / denom;
    e.p[i] = p;
    if (e.shadow) e.shadow[i] = f2bf(p);
  }
}

// ---------------------------------------------------------------------------
// CDR radix select.  state: [0] prefix bits, [1] prefix mask, [2] k remaining
// (1-based rank among elements matching the prefix), [3] threshold bits.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cdr_hist_kernel(const MTEntry* __restrict__ tab, const int2* __restrict__ chunks,
                                                       const uint32_t* __restrict__ state, int shift,
                                                       uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[256];
  lh[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t prefix = state[0], pmask = state[1];
  const int2 ck = chunks[blockIdx.x];
  const MTEntry e = tab[ck.x];
  const int64_t base = (int64_t)ck.y * kChunk;
  const int64_t end = min(e.n, base + kChunk);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    const float v = fabsf(e.g[i] * e.p[i]);
    const uint32_t u = __float_as_uint(v);
    if ((u & pmask) == prefix) atomicAdd(&lh[(u >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}

// single workgroup: walk bins from the top, find the bin holding the k-th largest
__global__ void cdr_select_kernel(uint32_t* __restrict__ state, uint32_t* __restrict__ hist, int shift) {
  if (threadIdx.x == 0) {
    uint32_t k = state[2];
    int b = 255;
    for (; b > 0; --b) {
      const uint32_t c = hist[b];
      if (c >= k) break;
      k -= c;
    }
    state[0] |= (uint32_t)b << shift;
    state[1] |= 255u << shift;
    state[2] = k;
    if (shift == 0) state[3] = state[0];
  }
  __syncthreads();
  hist[threadIdx.x] = 0;  // ready for the next pass (blockDim = 256)
}

__global__ void __launch_bounds__(256) cdr_mask_kernel(const MTEntry* __restrict__ tab, const int2* __restrict__ chunks,
                                                       const uint32_t* __restrict__ state, float clip) {
  const float thr = __uint_as_float(state[3]);
  const int2 ck = chunks[blockIdx.x];
  const MTEntry e = tab[ck.x];
  const int64_t base = (int64_t)ck.y * kChunk;
  const int64_t end = min(e.n, base + kChunk);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    const float g = e.g[i];
    const float v = fabsf(g * e.p[i]);
    e.g[i] = (v >= thr) ? g * clip : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Multi-tensor scaled copy: dst_t[i] = src_t[i] * scale for every table entry (MTEntry.p = dst,
// MTEntry.g = src, raw pointers; SRC_BF16 / DST_BF16 pick the element types).  The gradient
// bucket engine (parallel/reducer.py) packs a bucket's parameter gradients into its flat
// all-reduce buffer with one launch (pre-divided by the world size; optionally rounded to bf16
// for a half-size all-reduce) and, for a bf16 bucket, unpacks the reduced values into the fp32
// gradient views in one launch.
template <bool SRC_BF16, bool DST_BF16>
__global__ void __launch_bounds__(256) mt_copy_kernel(const MTEntry* __restrict__ tab, const int2* __restrict__ chunks,
                                                      float scale) {
  const int2 ck = chunks[blockIdx.x];
  const MTEntry e = tab[ck.x];
  const int64_t base = (int64_t)ck.y * kChunk;
  const int64_t end = min(e.n, base + kChunk);
  const void* src = (const void*)e.g;
  void* dst = (void*)e.p;
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    const float v = (SRC_BF16 ? bf2f(((const bf16*)src)[i]) : ((const float*)src)[i]) * scale;
    if (DST_BF16)
      ((bf16*)dst)[i] = f2bf(v);
    else
      ((float*)dst)[i] = v;
  }
}

void launch_mt_copy(const MTEntry* tab, const int2* chunks, int nchunks, float scale, int mode, hipStream_t s) {
  if (!nchunks) return;
  switch (mode & 3) {
    case 0: hipLaunchKernelGGL((mt_copy_kernel<false, false>), dim3(nchunks), dim3(256), 0, s, tab, chunks, scale); break;
    case 1: hipLaunchKernelGGL((mt_copy_kernel<true, false>), dim3(nchunks), dim3(256), 0, s, tab, chunks, scale); break;
    case 2: hipLaunchKernelGGL((mt_copy_kernel<false, true>), dim3(nchunks), dim3(256), 0, s, tab, chunks, scale); break;
    default: hipLaunchKernelGGL((mt_copy_kernel<true, true>), dim3(nchunks), dim3(256), 0, s, tab, chunks, scale); break;
  }
}

void launch_mt_sgd(const MTEntry* tab, const int2* chunks, int nchunks, SgdHyper h, hipStream_t s) {
  if (nchunks) hipLaunchKernelGGL(mt_sgd_kernel, dim3(nchunks), dim3(256), 0, s, tab, chunks, h);
}
void launch_mt_adam(const MTEntry* tab, const int2* chunks, int nchunks, AdamHyper h, hipStream_t s) {
  if (nchunks) hipLaunchKernelGGL(mt_adam_kernel, dim3(nchunks), dim3(256), 0, s, tab, chunks, h);
}
void launch_cdr_threshold(const MTEntry* tab, const int2* chunks, int nchunks, uint32_t* state, uint32_t* hist,
                          hipStream_t s) {
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(cdr_hist_kernel, dim3(nchunks), dim3(256), 0, s, tab, chunks, state, shift, hist);
    hipLaunchKernelGGL(cdr_select_kernel, dim3(1), dim3(256), 0, s, state, hist, shift);
  }
}
void launch_cdr_mask(const MTEntry* tab, const int2* chunks, int nchunks, const uint32_t* state, float clip,
                     hipStream_t s) {
  if (nchunks) hipLaunchKernelGGL(cdr_mask_kernel, dim3(nchunks), dim3(256), 0, s, tab, chunks, state, clip);
}

}  // namespace dcp
