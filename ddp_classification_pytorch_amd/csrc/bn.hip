// BatchNorm (training / eval / frozen), fused activation and residual add,
// NHWC bf16 activations with fp32 statistics.
//
// Replaces the ATen BatchNorm / SyncBatchNorm CUDA kernels the reference uses
// through nn.BatchNorm2d + convert_sync_batchnorm (BASELINE/main.py:148,
// ARCFACE/arc_main.py:239; SURVEY.md §2.2 X5, kernels K4-K7) and the
// InplaceABN BN+leaky-ReLU of timm's TResNet (X3, K21).
//
// Statistics are carried as (count, mean, M2) and combined with Chan's
// parallel-variance formula at every level, never as (sum, sumsq): deep
// ResNets feed BN inputs whose mean is large against their spread (post-ReLU
// inputs to 1x1 convs) and E[x^2]-E[x]^2 in fp32 loses the variance.
// Pipeline per BN layer (training):
//   conv epilogue    -> per-128-row slab (mean, M2)                 (conv_igemm.hip)
//   bn_slab_partial  -> per-split (n, mean, M2) partials  } bn_stats -> [1][3][C]
//   bn_merge         -> one (n, mean, M2) per channel     }   (SyncBN: all_gather -> [W][3][C])
//   bn_finalize      -> merge W entries; mean, invstd, scale, shift; running-stat update
//   bn_act_fwd       -> y = act(x*scale + shift [+ residual])
// backward:
//   bn_bwd_reduce    -> per-workgroup partial (sum dz, sum dz*xhat) -> partial_sum -> [2][C]
//                       (+ all_reduce for SyncBN)
//   bn_bwd_elemt     -> dx (and d(residual) = dz)
// The activation mask is recomputed from x (and the residual) instead of
// saving the post-activation tensor.
#include <type_traits>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2 };

__device__ __forceinline__ float act_f(float z, int act, float slope) {
  if (act == ACT_RELU) return fmaxf(z, 0.f);
  if (act == ACT_LEAKY) return z >= 0.f ? z : z * slope;
  return z;
}
__device__ __forceinline__ float act_d(float z, int act, float slope) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_LEAKY) return z >= 0.f ? 1.f : slope;
  return 1.f;
}

// pre-activation from the activation output (invertible activations only: identity, leaky ReLU)
__device__ __forceinline__ float act_inv(float y, int act, float slope) {
  return (act == 2 && y < 0.f) ? y / slope : y;
}

// Chan et al. pairwise merge of (n, mean, M2) accumulators
struct Welford {
  float n, mean, m2;
  __device__ __forceinline__ void merge(float nb, float meanb, float m2b) {
    if (nb <= 0.f) return;
    const float nt = n + nb;
    const float d = meanb - mean;
    const float f = nb / nt;
    mean += d * f;
    m2 += m2b + d * d * n * f;
    n = nt;
  }
};

// conv slabs [R][2][C] = per-128-row slab (mean, M2); slab r holds min(128, M-128r) rows.
// out[blockIdx.y][3][C] = (n, mean, M2) over this split's slabs (<= kSlabsPerSplit: 4 waves x
// 16 merges, each wave's loads issued four slabs ahead of its merge chain).
constexpr int kSlabsPerSplit = 64;
__global__ void __launch_bounds__(256) bn_slab_partial_kernel(const float* __restrict__ slabs, int R, int M, int C,
                                                              int tiles_per_split, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * tiles_per_split;
  const int r1 = min(R, r0 + tiles_per_split);
  Welford a{0.f, 0.f, 0.f};
  if (c < C) {
    int r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      float mb[4], m2b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        mb[u] = slabs[((size_t)(r + 4 * u) * 2 + 0) * C + c];
        m2b[u] = slabs[((size_t)(r + 4 * u) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) a.merge((float)min(128, M - 128 * (r + 4 * u)), mb[u], m2b[u]);
    }
    for (; r < r1; r += 4) {
      const float nb = (float)min(128, M - 128 * r);
      a.merge(nb, slabs[((size_t)r * 2 + 0) * C + c], slabs[((size_t)r * 2 + 1) * C + c]);
    }
  }
  __shared__ float red[3][4][64];
  red[0][w][lane] = a.n;
  red[1][w][lane] = a.mean;
  red[2][w][lane] = a.m2;
  __syncthreads();
  if (w == 0 && c < C) {
    for (int k = 1; k < 4; ++k) a.merge(red[0][k][lane], red[1][k][lane], red[2][k][lane]);
    out[((size_t)blockIdx.y * 3 + 0) * C + c] = a.n;
    out[((size_t)blockIdx.y * 3 + 1) * C + c] = a.mean;
    out[((size_t)blockIdx.y * 3 + 2) * C + c] = a.m2;
  }
}

// raw activations [M][C] -> out[blockIdx][3][C] (n, mean, M2).  Each thread
// accumulates sums shifted by its first observed value (a per-channel
// estimate of the mean), converts to (n, mean, M2), then the workgroup's row
// slots are merged with Chan's formula.
__global__ void __launch_bounds__(256) chan_welford_partial_kernel(const bf16* __restrict__ x, int M, int C,
                                                                   float* __restrict__ out) {
  const int cpr = C >> 3, rpi = 256 / cpr;
  const int slot = threadIdx.x / cpr, ch = threadIdx.x - slot * cpr, c0 = ch * 8;
  float n = 0.f, sh[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[k] = s1[k] = s2[k] = 0.f;
  const int first = blockIdx.x * rpi + slot;
  if (slot < rpi && first < M) {
    const bf16x8 v0 = *(const bf16x8*)(x + (size_t)first * C + c0);
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[k] = bf2f(v0[k]);
    for (int m = first; m < M; m += gridDim.x * rpi) {
      const bf16x8 v = *(const bf16x8*)(x + (size_t)m * C + c0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = bf2f(v[k]) - sh[k];
        s1[k] += d;
        s2[k] += d * d;
      }
      n += 1.f;
    }
  }
  extern __shared__ float shm[];  // [3][256][8]
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float mean = n > 0.f ? sh[k] + s1[k] / n : 0.f;
    const float m2 = n > 0.f ? fmaxf(s2[k] - s1[k] * s1[k] / n, 0.f) : 0.f;
    shm[threadIdx.x * 8 + k] = n;
    shm[2048 + threadIdx.x * 8 + k] = mean;
    shm[4096 + threadIdx.x * 8 + k] = m2;
  }
  __syncthreads();
  if (slot == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      Welford a{0.f, 0.f, 0.f};
      for (int sl = 0; sl < rpi; ++sl) {
        const int t = (sl * cpr + ch) * 8 + k;
        a.merge(shm[t], shm[2048 + t], shm[4096 + t]);
      }
      out[((size_t)blockIdx.x * 3 + 0) * C + c0 + k] = a.n;
      out[((size_t)blockIdx.x * 3 + 1) * C + c0 + k] = a.mean;
      out[((size_t)blockIdx.x * 3 + 2) * C + c0 + k] = a.m2;
    }
  }
}

// partials [P][3][C] -> (n, mean, M2) of channel blockIdx.x*64 + lane, complete in wave 0;
// one workgroup (NW waves splitting P) per 64 channels
constexpr int kMergeWaves = 16;
constexpr int kPartialChunk = 128;
template <int NW = kMergeWaves>
__device__ __forceinline__ Welford merge_partials(const float* __restrict__ part, int P, int C, int cb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * 64 + lane;
  Welford a{0.f, 0.f, 0.f};
  if (c < C) {
    int p = w;
    for (; p + 3 * NW < P; p += 4 * NW) {
      float v[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 3; ++q) v[u][q] = part[((size_t)(p + u * NW) * 3 + q) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) a.merge(v[u][0], v[u][1], v[u][2]);
    }
    for (; p < P; p += NW)
      a.merge(part[((size_t)p * 3 + 0) * C + c], part[((size_t)p * 3 + 1) * C + c],
              part[((size_t)p * 3 + 2) * C + c]);
  }
  __shared__ float red[3][NW][64];
  red[0][w][lane] = a.n;
  red[1][w][lane] = a.mean;
  red[2][w][lane] = a.m2;
  __syncthreads();
  if (w == 0)
    for (int k = 1; k < NW; ++k) a.merge(red[0][k][lane], red[1][k][lane], red[2][k][lane]);
  return a;
}

// conv slabs [R][2][C] (per-128-row (mean, M2), slab r holds min(128, M - 128 r) rows) merged
// straight into (n, mean, M2) of channel cb * kSlabCh + (lane & 15), complete in lanes 0-15 of wave 0 --
// the one-level path for R <= kDirectSlabs (small activations: no bn_slab_partial launch, whose per-launch
// cost dominated the statistics of every layer at batch 32-128).  16 channels per workgroup, so a
// 64-channel layer's slabs spread over four CUs (one workgroup read all 400 KB of a batch-32 stage-1
// layer's slabs at its CU's L2 -> LDS rate: 15 us): 64 row streams (4 per wave, 16 lanes = 16
// consecutive channels = 64 contiguous bytes per slab row), 8 slabs' loads in flight per stream, then a
// two-level fixed-order combine of the streams (deterministic).
constexpr int kDirectSlabs = 1024;
constexpr int kSlabCh = 16;
__device__ __forceinline__ Welford merge_slabs(const float* __restrict__ slabs, int R, int M, int C, int cb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * kSlabCh + (lane & 15);
  const int rs = (lane >> 4) + 4 * w;  // row stream 0 .. 63
  Welford a{0.f, 0.f, 0.f};
  if (c < C) {
    int r = rs;
    for (; r + 7 * 64 < R; r += 8 * 64) {
      float mb[8], m2b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        mb[u] = slabs[((size_t)(r + u * 64) * 2 + 0) * C + c];
        m2b[u] = slabs[((size_t)(r + u * 64) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a.merge((float)min(128, M - 128 * (r + u * 64)), mb[u], m2b[u]);
    }
    for (; r < R; r += 64)
      a.merge((float)min(128, M - 128 * r), slabs[((size_t)r * 2 + 0) * C + c], slabs[((size_t)r * 2 + 1) * C + c]);
  }
  __shared__ float red[3][64][kSlabCh];
  const int ch = lane & 15;
  red[0][rs][ch] = a.n;
  red[1][rs][ch] = a.mean;
  red[2][rs][ch] = a.m2;
  __syncthreads();
  if (rs < 8) {  // streams rs, rs + 8, .. rs + 56
    Welford b{0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) b.merge(red[0][rs + 8 * k][ch], red[1][rs + 8 * k][ch], red[2][rs + 8 * k][ch]);
    a = b;
  }
  __syncthreads();
  if (rs < 8) {
    red[0][rs][ch] = a.n;
    red[1][rs][ch] = a.mean;
    red[2][rs][ch] = a.m2;
  }
  __syncthreads();
  if (rs == 0) {
    Welford b{0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) b.merge(red[0][k][ch], red[1][k][ch], red[2][k][ch]);
    a = b;
  }
  return a;
}

// slabs [R][2][C] -> out [3][C] (R <= kDirectSlabs)
__global__ void __launch_bounds__(64 * kMergeWaves) bn_slab_merge_kernel(const float* __restrict__ slabs, int R, int M,
                                                                         int C, float* __restrict__ out) {
  const Welford a = merge_slabs(slabs, R, M, C, blockIdx.x);
  const int c = blockIdx.x * kSlabCh + (threadIdx.x & 63);
  if (threadIdx.x < kSlabCh && c < C) {
    out[c] = a.n;
    out[C + c] = a.mean;
    out[2 * C + c] = a.m2;
  }
}

// partials [P][3][C] -> out [3][C]
__global__ void __launch_bounds__(64 * kMergeWaves) bn_merge_kernel(const float* __restrict__ part, int P, int C,
                                                       float* __restrict__ out) {
  const Welford a = merge_partials(part, P, C, blockIdx.x);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((threadIdx.x >> 6) == 0 && c < C) {
    out[c] = a.n;
    out[C + c] = a.mean;
    out[2 * C + c] = a.m2;
  }
}

// first level of a two-level partial merge: chunk blockIdx.y of kPartialChunk partial rows ->
// tmp [chunks][3][C].  One workgroup merging thousands of partials (the stem conv's 7,168 at batch
// 1024) ran 143 us on one CU; chunks of 128 spread it over the chip.
__global__ void __launch_bounds__(64 * kMergeWaves) bn_partial_chunk_kernel(const float* __restrict__ part, int P,
                                                                            int C, float* __restrict__ out) {
  const int r0 = blockIdx.y * kPartialChunk;
  const Welford a = merge_partials(part + (size_t)r0 * 3 * C, min(kPartialChunk, P - r0), C, blockIdx.x);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((threadIdx.x >> 6) == 0 && c < C) {
    out[((size_t)blockIdx.y * 3 + 0) * C + c] = a.n;
    out[((size_t)blockIdx.y * 3 + 1) * C + c] = a.mean;
    out[((size_t)blockIdx.y * 3 + 2) * C + c] = a.m2;
  }
}

int bn_partial_chunks(int P) { return P > 2 * kPartialChunk ? (P + kPartialChunk - 1) / kPartialChunk : 0; }

void launch_bn_partial_chunk(const float* part, int P, int C, float* tmp, hipStream_t s) {
  hipLaunchKernelGGL(bn_partial_chunk_kernel, dim3((C + 63) / 64, bn_partial_chunks(P)), dim3(64 * kMergeWaves), 0,
                     s, part, P, C, tmp);
}

// merged (n, mean, M2) of channel c -> mean, invstd, scale, shift (+ running stats)
// iabn_eps >= 0: InplaceABN's effective weight |gamma| + iabn_eps (and its reciprocal into rgamma) -- the
// separate iabn_gamma launch of every layer folded in (its gradient's sign: bn_bwd_elemt's dg output)
// WT: scale / shift stored write-through (agent-scope atomic stores) for readers in other workgroups
// of the same launch (bn_fin_act_kernel)
template <bool WT = false>
__device__ __forceinline__ void finalize_channel(const Welford& a, int c, float eps, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float* __restrict__ mean,
                                                 float* __restrict__ invstd, float* __restrict__ scale,
                                                 float* __restrict__ shift, float* __restrict__ run_mean,
                                                 float* __restrict__ run_var, float momentum, float iabn_eps,
                                                 float* __restrict__ rgamma) {
  const float var = a.n > 0.f ? a.m2 / a.n : 0.f;
  const float is = rsqrtf(var + eps);
  mean[c] = a.mean;
  invstd[c] = is;
  float g = gamma ? gamma[c] : 1.f;
  if (iabn_eps >= 0.f) {
    g = fabsf(g) + iabn_eps;
    if (rgamma) rgamma[c] = 1.f / g;
  }
  const float b = beta ? beta[c] : 0.f;
  if (WT) {
    __hip_atomic_store(scale + c, g * is, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(shift + c, b - a.mean * g * is, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    scale[c] = g * is;
    shift[c] = b - a.mean * g * is;
  }
  if (run_mean) {
    const float unb = a.n > 1.f ? a.m2 / (a.n - 1.f) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * a.mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// local BN (one rank): partials [P][3][C] -> mean, invstd, scale, shift in one launch
// (bn_merge + bn_finalize with W = 1; bit-identical to the two-kernel path)
__global__ void __launch_bounds__(64 * kMergeWaves) bn_merge_finalize_kernel(
    const float* __restrict__ part, int P, int C, float eps, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ scale,
    float* __restrict__ shift, float* __restrict__ run_mean, float* __restrict__ run_var, float momentum, float iabn_eps,
    float* __restrict__ rgamma) {
  const Welford m = merge_partials(part, P, C, blockIdx.x);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  Welford a{0.f, 0.f, 0.f};
  a.merge(m.n, m.mean, m.m2);  // the W = 1 merge of bn_finalize_kernel
  finalize_channel(a, c, eps, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, momentum, iabn_eps, rgamma);
}

// local BN from the conv slabs in one launch (R <= kDirectSlabs): merge + finalize; the same
// merge order as bn_slab_merge_kernel, so SyncBN at world size 1 stays bit-identical
__global__ void __launch_bounds__(64 * kMergeWaves) bn_slab_finalize_kernel(
    const float* __restrict__ slabs, int R, int M, int C, float eps, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ scale,
    float* __restrict__ shift, float* __restrict__ run_mean, float* __restrict__ run_var, float momentum, float iabn_eps,
    float* __restrict__ rgamma) {
  const Welford m = merge_slabs(slabs, R, M, C, blockIdx.x);
  const int c = blockIdx.x * kSlabCh + (threadIdx.x & 63);
  if (threadIdx.x >= kSlabCh || c >= C) return;
  Welford a{0.f, 0.f, 0.f};
  a.merge(m.n, m.mean, m.m2);  // the W = 1 merge of bn_finalize_kernel
  finalize_channel(a, c, eps, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, momentum, iabn_eps, rgamma);
}


// [P][K] -> [K] column sums; one workgroup per 64 columns, 4 waves x 4-deep unroll over P
template <typename OUT = float>
__global__ void __launch_bounds__(256) partial_sum_kernel(const float* __restrict__ part, int P, int K,
                                                          OUT* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (k < K) {
    int p = w;
    // 16 loads in flight per wave (a small batch's BN sums reduce ~800 partials: load round trips,
    // not adds, set the time); each accumulator still adds its rows in the same order
    for (; p + 60 < P; p += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = part[(size_t)(p + 4 * u) * K + k];
#pragma unroll
      for (int u = 0; u < 16; u += 4) {
        s0 += v[u];
        s1 += v[u + 1];
        s2 += v[u + 2];
        s3 += v[u + 3];
      }
    }
    for (; p + 12 < P; p += 16) {
      s0 += part[(size_t)p * K + k];
      s1 += part[(size_t)(p + 4) * K + k];
      s2 += part[(size_t)(p + 8) * K + k];
      s3 += part[(size_t)(p + 12) * K + k];
    }
    for (; p < P; p += 4) s0 += part[(size_t)p * K + k];
  }
  __shared__ float red[4][64];
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && k < K) {
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if constexpr (std::is_same<OUT, float>::value) out[k] = t;
    else out[k] = f2bf(t);  // (round to nearest even, as a torch .to(bfloat16) of the fp32 sum)
  }
}

// stats [W][3][C] (one (n, mean, M2) per rank) -> mean, invstd, scale, shift (+ running stats)
__global__ void bn_finalize_kernel(const float* __restrict__ st, int W, int C, float eps,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ mean, float* __restrict__ invstd,
                                   float* __restrict__ scale, float* __restrict__ shift,
                                   float* __restrict__ run_mean, float* __restrict__ run_var,
                                   float momentum, float iabn_eps, float* __restrict__ rgamma) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  Welford a{0.f, 0.f, 0.f};
  for (int w = 0; w < W; ++w)
    a.merge(st[((size_t)w * 3 + 0) * C + c], st[((size_t)w * 3 + 1) * C + c], st[((size_t)w * 3 + 2) * C + c]);
  finalize_channel(a, c, eps, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, momentum, iabn_eps, rgamma);
}

// eval / frozen BN: scale = gamma / sqrt(var + eps), shift = beta - mean*scale
__global__ void bn_eval_coeff_kernel(int C, float eps, const float* __restrict__ gamma,
                                     const float* __restrict__ beta, const float* __restrict__ rm,
                                     const float* __restrict__ rv, float* __restrict__ mean,
                                     float* __restrict__ invstd, float* __restrict__ scale,
                                     float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  mean[c] = rm[c];
  invstd[c] = is;
  scale[c] = g * is;
  shift[c] = b - rm[c] * g * is;
}

// plain column sums of [M][C] -> per-workgroup partials out[blockIdx][C]
__global__ void __launch_bounds__(256) colsum_partial_kernel(const bf16* __restrict__ x, int M, int C,
                                                             float* __restrict__ out) {
  const int cbase = blockIdx.y * 2048;
  const int Cw = min(2048, C - cbase);
  const int cpr = Cw >> 3, rpi = 256 / cpr;
  const int slot = threadIdx.x / cpr, ch = threadIdx.x - slot * cpr;
  float s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = 0.f;
  if (slot < rpi)
    for (int m = blockIdx.x * rpi + slot; m < M; m += gridDim.x * rpi) {
      const bf16x8 v = *(const bf16x8*)(x + (size_t)m * C + cbase + ch * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) s1[k] += bf2f(v[k]);
    }
  __shared__ float sh[2048];
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = s1[k];
  __syncthreads();
  if (slot == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = 0.f;
      for (int sl = 0; sl < rpi; ++sl) t += sh[(sl * cpr + ch) * 8 + k];
      out[(size_t)blockIdx.x * C + cbase + ch * 8 + k] = t;
    }
}

// ---------------------------------------------------------------------------
// Row-tiled elementwise kernels.  A workgroup of 256 threads covers `rpi` rows
// x C channels per pass; each thread owns ONE fixed 8-channel chunk, so its
// per-channel coefficients live in registers for the whole kernel, and walks
// rows with a 4-deep unroll so 4 independent 16-byte loads per operand are in
// flight (the kernels are HBM-bound; memory-level parallelism is the lever).
// ---------------------------------------------------------------------------
struct RowTile {
  int cpr, rpi, slot, ch, c0;
  __device__ RowTile(int C, int tid) {
    cpr = C >> 3;
    rpi = 256 / cpr;
    slot = tid / cpr;
    ch = tid - slot * cpr;
    c0 = ch * 8;
  }
  __device__ explicit RowTile(int C) : RowTile(C, threadIdx.x) {}
};

__device__ __forceinline__ void load8(const float* __restrict__ p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// the rows of one (virtual) 256-thread workgroup vb of VG: y = act(x*sc + sh [+ res*rsc + rsh])
template <int ACT, bool RES>
__device__ __forceinline__ void bn_act_rows(const RowTile& t, int vb, int VG, const bf16* __restrict__ x,
                                            const bf16* __restrict__ res, const float* sc, const float* sh,
                                            const float* rsc, const float* rsh, bf16* __restrict__ y, int M, int C,
                                            float slope, int nt, uint8_t* __restrict__ mask) {
  const int step = VG * t.rpi;
  int m = vb * t.rpi + t.slot;
  constexpr int U = 4;
  for (; m + (U - 1) * step < M; m += U * step) {
    bf16x8 v[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)(m + u * step) * C + t.c0;
      v[u] = *(const bf16x8*)(x + off);
      if (RES) r[u] = *(const bf16x8*)(res + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bf16x8 o;
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = bf2f(v[u][k]) * sc[k] + sh[k];
        if (RES) z += bf2f(r[u][k]) * rsc[k] + rsh[k];
        bits |= (z > 0.f ? 1u : 0u) << k;
        o[k] = f2bf(act_f(z, ACT, slope));
      }
      if (nt) __builtin_nontemporal_store(o, (bf16x8*)(y + (size_t)(m + u * step) * C + t.c0));
      else *(bf16x8*)(y + (size_t)(m + u * step) * C + t.c0) = o;
      if (mask) mask[(size_t)(m + u * step) * t.cpr + t.ch] = (uint8_t)bits;
    }
  }
  for (; m < M; m += step) {
    const size_t off = (size_t)m * C + t.c0;
    const bf16x8 v = *(const bf16x8*)(x + off);
    bf16x8 r;
    if (RES) r = *(const bf16x8*)(res + off);
    bf16x8 o;
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = bf2f(v[k]) * sc[k] + sh[k];
      if (RES) z += bf2f(r[k]) * rsc[k] + rsh[k];
      bits |= (z > 0.f ? 1u : 0u) << k;
      o[k] = f2bf(act_f(z, ACT, slope));
    }
    *(bf16x8*)(y + off) = o;
    if (mask) mask[(size_t)m * t.cpr + t.ch] = (uint8_t)bits;
  }
}

template <int ACT, bool RES>
__global__ void __launch_bounds__(256) bn_act_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, bf16* __restrict__ y,
                                                         int M, int C, float slope, int nt,
                                                         uint8_t* __restrict__ mask,
                                                         const float* __restrict__ rscale,
                                                         const float* __restrict__ rshift) {
  // mask != nullptr: also store act'(z) > 0 as one bit per element ([M][C/8] bytes), so the
  // backward of a BN + residual + ReLU layer reads 1/16 of the residual's bytes for its mask.
  // rscale != nullptr: the residual is itself a raw BN input (a projection shortcut's conv
  // output) normalised on the fly, res * rscale + rshift -- its BN never writes an activation.
  const RowTile t(C);
  if (t.slot >= t.rpi) return;
  float sc[8], sh[8], rsc[8], rsh[8];
  load8(scale + t.c0, sc);
  load8(shift + t.c0, sh);
  if (RES && rscale) {
    load8(rscale + t.c0, rsc);
    load8(rshift + t.c0, rsh);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) rsc[k] = 1.f, rsh[k] = 0.f;
  }
  bn_act_rows<ACT, RES>(t, blockIdx.x, gridDim.x, x, res, sc, sh, rsc, rsh, y, M, C, slope, nt, mask);
}

// ---------------------------------------------------------------------------
// Local training-mode BN: statistics finalize + BN / act (+ residual) apply in ONE launch.  At small
// batch every BN layer was two dependent launches of a few us each (bn_slab_finalize on one to 32
// workgroups, then bn_act_fwd) -- pure launch latency.
// Workgroups 0 .. nfin-1, dispatched first and waiting on nothing before they publish, merge the
// statistics of 64 channels each with the code and order of bn_slab_finalize / bn_merge_finalize
// (bit-identical coefficients), store scale / shift WRITE-THROUGH (agent-scope atomic stores: no
// release fence, whose L2 write-back stalled the ticket reductions of round 3), drain their stores
// and count themselves in sync[0].  Every workgroup waits for the nfin arrivals (bounded spin: a
// timeout sets sync[2] and is reported by the host), reads its coefficients coherently and runs
// bn_act_fwd's math as 4 virtual 256-thread workgroups; the last workgroup through resets sync[0..1]
// for the next launch (stream-ordered: graph-replay safe).
struct FinActParams {
  const bf16* x;
  const bf16* res;
  const float* src;  // conv slabs [R][2][C] (partials == 0) or partials [P][3][C]
  int nsrc, partials, M, C, nfin;
  float eps, momentum, iabn_eps, slope;
  const float* gamma;
  const float* beta;
  float* mean;
  float* invstd;
  float* scale;
  float* shift;
  float* run_mean;
  float* run_var;
  float* rgamma;
  bf16* y;
  uint8_t* mask;
  uint32_t* sync;  // [0] finalize arrivals, [1] workgroups through, [2] spin timeouts
};

template <int ACT, bool RES>
__global__ void __launch_bounds__(1024) bn_fin_act_kernel(const FinActParams p) {
  if ((int)blockIdx.x < p.nfin) {
    const Welford m = p.partials ? merge_partials(p.src, p.nsrc, p.C, blockIdx.x)
                                 : merge_slabs(p.src, p.nsrc, p.M, p.C, blockIdx.x);
    const int cpb = p.partials ? 64 : kSlabCh;  // channels per finalize workgroup
    const int c = blockIdx.x * cpb + (threadIdx.x & 63);
    if ((int)threadIdx.x < cpb && c < p.C) {
      Welford a{0.f, 0.f, 0.f};
      a.merge(m.n, m.mean, m.m2);  // the W = 1 merge of bn_finalize_kernel
      finalize_channel<true>(a, c, p.eps, p.gamma, p.beta, p.mean, p.invstd, p.scale, p.shift, p.run_mean,
                             p.run_var, p.momentum, p.iabn_eps, p.rgamma);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(p.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    // one poller per workgroup, ~1 us apart: hundreds of workgroups hammering the counter's memory
    // channel would slow the finalize workgroups' own slab loads
    uint32_t spins = 0;
    while (__hip_atomic_load(p.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)p.nfin) {
      if (++spins > (1u << 22)) {
        __hip_atomic_store(p.sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(32);
    }
  }
  __syncthreads();
  // scale / shift staged once per workgroup: one coherent (sc1, past any stale L2 line of the reused
  // allocation) 16-byte load per thread at most, then LDS reads -- per-thread coherent loads of
  // 16 coefficients cost ~9 us per layer at batch 32
  __shared__ f32x4 coef[2 * 2048 / 4];
  {
    const int n4 = p.C / 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.scale, (short)0, p.C * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(p.shift, (short)0, p.C * 4, 0x00020000);
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
      coef[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, 16 /* sc1 */));
      coef[n4 + i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, i * 16, 0, 16));
    }
  }
  __syncthreads();
  const RowTile t(p.C, threadIdx.x & 255);
  float sc[8], sh[8], one[8], zero[8];
  const float* cf = (const float*)coef;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = cf[t.c0 + k];
    sh[k] = cf[p.C + t.c0 + k];
    one[k] = 1.f;
    zero[k] = 0.f;
  }
  if (threadIdx.x == 0) {
    // every workgroup counted here has passed the wait: the last one re-arms the counters
    const uint32_t done = __hip_atomic_fetch_add(p.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(p.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (t.slot >= t.rpi) return;
  bn_act_rows<ACT, RES>(t, blockIdx.x * 4 + (threadIdx.x >> 8), gridDim.x * 4, p.x, p.res, sc, sh, one, zero, p.y,
                        p.M, p.C, p.slope, 0, p.mask);
}

// sums over rows of dz = dy*act'(z) and dz*xhat -> per-workgroup partials out[blockIdx][2][C]
// (deterministic; summed by partial_sum_kernel -- no contended atomics)
template <int ACT, bool RES>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int M, int C,
                                                            float slope, float* __restrict__ out, int inv) {
  // inv (InplaceABN backward, X3/K21): x holds the layer's OUTPUT y = act(z); z = act^-1(y) is
  // recovered in registers and mean / invstd carry beta / 1/gamma, so xhat = (z - beta) / gamma --
  // the BN input itself is never stored
  const RowTile t(C);
  float s1[8], s2[8], sc[8], sh[8], mu[8], is[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
  load8(scale + t.c0, sc);
  load8(shift + t.c0, sh);
  load8(mean + t.c0, mu);
  load8(invstd + t.c0, is);
  if (t.slot < t.rpi) {
    const int step = gridDim.x * t.rpi;
    int m = blockIdx.x * t.rpi + t.slot;
    constexpr int U = 4;
    for (; m + (U - 1) * step < M; m += U * step) {
      bf16x8 g[U], v[U], r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t off = (size_t)(m + u * step) * C + t.c0;
        g[u] = *(const bf16x8*)(dy + off);
        v[u] = *(const bf16x8*)(x + off);
        if (RES) r[u] = *(const bf16x8*)(res + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float xv = bf2f(v[u][k]);
          float z = xv * sc[k] + sh[k];
          if (RES) z += bf2f(r[u][k]);
          if (inv) xv = z = act_inv(bf2f(v[u][k]), ACT, slope);
          const float dz = bf2f(g[u][k]) * act_d(z, ACT, slope);
          s1[k] += dz;
          s2[k] += dz * (xv - mu[k]);
        }
    }
    for (; m < M; m += step) {
      const size_t off = (size_t)m * C + t.c0;
      const bf16x8 g = *(const bf16x8*)(dy + off);
      const bf16x8 v = *(const bf16x8*)(x + off);
      bf16x8 r;
      if (RES) r = *(const bf16x8*)(res + off);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float xv = bf2f(v[k]);
        float z = xv * sc[k] + sh[k];
        if (RES) z += bf2f(r[k]);
        if (inv) xv = z = act_inv(bf2f(v[k]), ACT, slope);
        const float dz = bf2f(g[k]) * act_d(z, ACT, slope);
        s1[k] += dz;
        s2[k] += dz * (xv - mu[k]);
      }
    }
  }
  extern __shared__ float sh_red[];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh_red[threadIdx.x * 8 + k] = s1[k];
    sh_red[2048 + threadIdx.x * 8 + k] = s2[k] * is[k];
  }
  __syncthreads();
  if (t.slot == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t1 = 0.f, t2 = 0.f;
      for (int s = 0; s < t.rpi; ++s) {
        t1 += sh_red[(s * t.cpr + t.ch) * 8 + k];
        t2 += sh_red[2048 + (s * t.cpr + t.ch) * 8 + k];
      }
      out[((size_t)blockIdx.x * 2 + 0) * C + t.c0 + k] = t1;
      out[((size_t)blockIdx.x * 2 + 1) * C + t.c0 + k] = t2;
    }
  }
}

// dx = scale*(dz - sum_dz/count - xhat*sum_dzxhat/count)  [sums != nullptr]
//    = a*dz + b*x + c  with per-channel a, b, c folded once per thread
// dx = scale*dz                                            [eval / frozen BN]
// dres = dz (if dres != nullptr)
template <int ACT, bool RES>
__global__ void __launch_bounds__(256) bn_bwd_elemt_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                           const bf16* __restrict__ res,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ sums, float inv_count, int M,
                                                           int C, float slope, bf16* __restrict__ dx,
                                                           bf16* __restrict__ dres, int inv,
                                                           const float* __restrict__ graw, float* __restrict__ dg) {
  // inv: InplaceABN backward from the output y (see bn_bwd_reduce_kernel); mean / invstd = beta /
  // 1/gamma, scale = the true gamma * invstd
  const RowTile t(C);
  if (t.slot >= t.rpi) return;
  if (dg != nullptr && blockIdx.x == 0 && t.slot == 0) {
    // InplaceABN's weight gradient: d(|g| + eps)/dg = sign(g) times the effective weight's gradient
    // (sums row 1, this rank's) -- the separate sign_mul launch of every layer folded in.  A
    // workgroup's row slot 0 covers every channel (C <= 2048: C / 8 <= 256 threads).
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = graw[t.c0 + k], d = sums[C + t.c0 + k];
      dg[t.c0 + k] = v > 0.f ? d : (v < 0.f ? -d : 0.f);
    }
  }
  float sc[8], sh[8], ca[8], cb[8], cc[8];
  load8(scale + t.c0, sc);
  load8(shift + t.c0, sh);
  if (sums) {
    float mu[8], is[8], k2[8], k3[8];
    load8(mean + t.c0, mu);
    load8(invstd + t.c0, is);
    load8(sums + t.c0, k2);
    load8(sums + C + t.c0, k3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a2 = k2[k] * inv_count, a3 = k3[k] * inv_count * is[k];
      ca[k] = sc[k];
      cb[k] = -sc[k] * a3;
      cc[k] = -sc[k] * a2 + sc[k] * a3 * mu[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ca[k] = sc[k];
      cb[k] = 0.f;
      cc[k] = 0.f;
    }
  }
  const int step = gridDim.x * t.rpi;
  int m = blockIdx.x * t.rpi + t.slot;
  constexpr int U = 4;
  auto body = [&](const bf16x8& g, const bf16x8& v, const bf16x8& r, size_t off) {
    bf16x8 o, od;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float xv = bf2f(v[k]);
      float z = xv * sc[k] + sh[k];
      if (RES) z += bf2f(r[k]);
      if (inv) xv = z = act_inv(bf2f(v[k]), ACT, slope);
      const float dz = bf2f(g[k]) * act_d(z, ACT, slope);
      od[k] = f2bf(dz);
      o[k] = f2bf(ca[k] * dz + cb[k] * xv + cc[k]);
    }
    *(bf16x8*)(dx + off) = o;
    if (dres) *(bf16x8*)(dres + off) = od;
  };
  for (; m + (U - 1) * step < M; m += U * step) {
    bf16x8 g[U], v[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)(m + u * step) * C + t.c0;
      g[u] = *(const bf16x8*)(dy + off);
      v[u] = *(const bf16x8*)(x + off);
      if (RES) r[u] = *(const bf16x8*)(res + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(g[u], v[u], r[u], (size_t)(m + u * step) * C + t.c0);
  }
  for (; m < M; m += step) {
    const size_t off = (size_t)m * C + t.c0;
    const bf16x8 g = *(const bf16x8*)(dy + off);
    const bf16x8 v = *(const bf16x8*)(x + off);
    bf16x8 r;
    if (RES) r = *(const bf16x8*)(res + off);
    body(g, v, r, off);
  }
}


// Both BN backwards of a projection block's output (act(BN(x) + BN_r(r)), see bn2_act_mask)
// in one pass over the already-masked gradient g: dx = BN'(g, x), dr = BN_r'(g, r).  One read of
// g instead of two.  Coefficients per channel: d = ca*g + cb*v + cc (training statistics).
__device__ inline void bn_bwd_coeff8(const float* scale, const float* mean, const float* invstd, const float* sums,
                                     int C, int c0, float inv_count, float* ca, float* cb, float* cc) {
  float sc[8], mu[8], is[8], k2[8], k3[8];
  load8(scale + c0, sc);
  load8(mean + c0, mu);
  load8(invstd + c0, is);
  load8(sums + c0, k2);
  load8(sums + C + c0, k3);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float a2 = k2[k] * inv_count, a3 = k3[k] * inv_count * is[k];
    ca[k] = sc[k];
    cb[k] = -sc[k] * a3;
    cc[k] = -sc[k] * a2 + sc[k] * a3 * mu[k];
  }
}

__global__ void __launch_bounds__(256) bn2_bwd_elemt_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ r, const float* __restrict__ scale,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ sums,
                                                            const float* __restrict__ rscale,
                                                            const float* __restrict__ rmean,
                                                            const float* __restrict__ rinvstd,
                                                            const float* __restrict__ rsums, float inv_count, int M,
                                                            int C, bf16* __restrict__ dx, bf16* __restrict__ dr) {
  const RowTile t(C);
  if (t.slot >= t.rpi) return;
  float ca[8], cb[8], cc[8], ra[8], rb[8], rc[8];
  bn_bwd_coeff8(scale, mean, invstd, sums, C, t.c0, inv_count, ca, cb, cc);
  bn_bwd_coeff8(rscale, rmean, rinvstd, rsums, C, t.c0, inv_count, ra, rb, rc);
  const int step = gridDim.x * t.rpi;
  int m = blockIdx.x * t.rpi + t.slot;
  constexpr int U = 4;
  auto body = [&](const bf16x8& g, const bf16x8& v, const bf16x8& w, size_t off) {
    bf16x8 o, orr;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gv = bf2f(g[k]);
      o[k] = f2bf(ca[k] * gv + cb[k] * bf2f(v[k]) + cc[k]);
      orr[k] = f2bf(ra[k] * gv + rb[k] * bf2f(w[k]) + rc[k]);
    }
    *(bf16x8*)(dx + off) = o;
    *(bf16x8*)(dr + off) = orr;
  };
  for (; m + (U - 1) * step < M; m += U * step) {
    bf16x8 g[U], v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)(m + u * step) * C + t.c0;
      g[u] = *(const bf16x8*)(dy + off);
      v[u] = *(const bf16x8*)(x + off);
      w[u] = *(const bf16x8*)(r + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(g[u], v[u], w[u], (size_t)(m + u * step) * C + t.c0);
  }
  for (; m < M; m += step) {
    const size_t off = (size_t)m * C + t.c0;
    body(*(const bf16x8*)(dy + off), *(const bf16x8*)(x + off), *(const bf16x8*)(r + off), off);
  }
}

// ---------------------------------------------------------------------------
int bn_stats_partials(int M, int C, bool from_slabs) {
  if (from_slabs) {
    const int R = (M + 127) / 128;
    int splits = (R + kSlabsPerSplit - 1) / kSlabsPerSplit;
    return splits > 4096 ? 4096 : (splits < 1 ? 1 : splits);
  }
  const int rpi = 256 / (C / 8);
  int g = (M + rpi * 32 - 1) / (rpi * 32);
  return g > 256 ? 256 : (g < 1 ? 1 : g);
}

// first level of the statistics: part[P][3][C] from the conv slabs or the raw activations
static int launch_stat_partials(const bf16* x, const float* slabs, int M, int C, float* part, hipStream_t s) {
  const int P = bn_stats_partials(M, C, slabs != nullptr);
  if (slabs) {
    const int R = (M + 127) / 128;
    const int tps = (R + P - 1) / P;
    hipLaunchKernelGGL(bn_slab_partial_kernel, dim3((C + 63) / 64, P), dim3(256), 0, s, slabs, R, M, C, tps, part);
  } else {
    hipLaunchKernelGGL(chan_welford_partial_kernel, dim3(P), dim3(256), 3 * 2048 * 4, s, x, M, C, part);
  }
  return P;
}

// part: bn_stats_partials(...) x 3 x C scratch; out [3][C]
void launch_bn_stats(const bf16* x, const float* slabs, int M, int C, float* part, float* out, hipStream_t s) {
  const int R = (M + 127) / 128;
  if (slabs && R <= kDirectSlabs) {
    hipLaunchKernelGGL(bn_slab_merge_kernel, dim3((C + kSlabCh - 1) / kSlabCh), dim3(64 * kMergeWaves), 0, s, slabs,
                       R, M, C, out);
    return;
  }
  const int P = launch_stat_partials(x, slabs, M, C, part, s);
  hipLaunchKernelGGL(bn_merge_kernel, dim3((C + 63) / 64), dim3(64 * kMergeWaves), 0, s, part, P, C, out);
}

void launch_bn_stats_finalize(const bf16* x, const float* slabs, int M, int C, float* part, float eps,
                              const float* gamma, const float* beta, float* mean, float* invstd, float* scale,
                              float* shift, float* rm, float* rv, float momentum, hipStream_t s, float iabn_eps,
                              float* rgamma) {
  const int R = (M + 127) / 128;
  if (slabs && R <= kDirectSlabs) {
    hipLaunchKernelGGL(bn_slab_finalize_kernel, dim3((C + kSlabCh - 1) / kSlabCh), dim3(64 * kMergeWaves), 0, s,
                       slabs, R, M, C, eps, gamma, beta, mean, invstd, scale, shift, rm, rv, momentum, iabn_eps,
                       rgamma);
    return;
  }
  const int P = launch_stat_partials(x, slabs, M, C, part, s);
  hipLaunchKernelGGL(bn_merge_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kMergeWaves), 0, s, part, P, C, eps, gamma, beta,
                     mean, invstd, scale, shift, rm, rv, momentum, iabn_eps, rgamma);
}

void launch_bn_merge(const float* part, int P, int C, float* out, hipStream_t s) {
  hipLaunchKernelGGL(bn_merge_kernel, dim3((C + 63) / 64), dim3(64 * kMergeWaves), 0, s, part, P, C, out);
}

void launch_bn_merge_finalize(const float* part, int P, int C, float eps, const float* gamma, const float* beta,
                              float* mean, float* invstd, float* scale, float* shift, float* rm, float* rv,
                              float momentum, hipStream_t s, float iabn_eps, float* rgamma) {
  hipLaunchKernelGGL(bn_merge_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kMergeWaves), 0, s, part, P, C, eps,
                     gamma, beta, mean, invstd, scale, shift, rm, rv, momentum, iabn_eps, rgamma);
}

void launch_partial_sum(const float* part, int P, int K, float* out, hipStream_t s) {
  hipLaunchKernelGGL(partial_sum_kernel<float>, dim3((K + 63) / 64), dim3(256), 0, s, part, P, K, out);
}

void launch_partial_sum_bf16(const float* part, int P, int K, bf16* out, hipStream_t s) {
  hipLaunchKernelGGL(partial_sum_kernel<bf16>, dim3((K + 63) / 64), dim3(256), 0, s, part, P, K, out);
}

// ~16 rows per workgroup (at most 128 partials): a linear layer's bias gradient over a 1024-row
// batch with 1000 columns ran as 4 latency-bound workgroups (42 us) at 256 rows each
int colsum_partials(int M) {
  int g = (M + 15) / 16;
  return g > 128 ? 128 : (g < 1 ? 1 : g);
}

void launch_colsum(const bf16* x, int M, int C, float* part, float* out, hipStream_t s) {
  const int P = colsum_partials(M);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(P, (C + 2047) / 2048), dim3(256), 0, s, x, M, C, part);
  hipLaunchKernelGGL(partial_sum_kernel<float>, dim3((C + 63) / 64), dim3(256), 0, s, part, P, C, out);
}

void launch_bn_finalize(const float* st, int W, int C, float eps, const float* gamma, const float* beta, float* mean,
                        float* invstd, float* scale, float* shift, float* rm, float* rv, float momentum,
                        hipStream_t s, float iabn_eps, float* rgamma) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, st, W, C, eps, gamma, beta, mean,
                     invstd, scale, shift, rm, rv, momentum, iabn_eps, rgamma);
}

void launch_bn_eval_coeff(int C, float eps, const float* gamma, const float* beta, const float* rm,
                          const float* rv, float* mean, float* invstd, float* scale, float* shift,
                          hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, eps, gamma, beta, rm, rv,
                     mean, invstd, scale, shift);
}

static inline int rows_grid(int M, int C, int rows_per_thread, int cap) {
  const int rpi = 256 / (C / 8);
  long g = ((long)M + (long)rpi * rows_per_thread - 1) / ((long)rpi * rows_per_thread);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

#define DCP_ACT_RES_DISPATCH(KERNEL, GRID, SHMEM, STREAM, RESPTR, ACTV, ...)                        \
  do {                                                                                              \
    const bool has_res = (RESPTR) != nullptr;                                                       \
    if (ACTV == ACT_RELU) {                                                                         \
      if (has_res)                                                                                  \
        hipLaunchKernelGGL((KERNEL<ACT_RELU, true>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__);  \
      else                                                                                          \
        hipLaunchKernelGGL((KERNEL<ACT_RELU, false>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__); \
    } else if (ACTV == ACT_LEAKY) {                                                                 \
      if (has_res)                                                                                  \
        hipLaunchKernelGGL((KERNEL<ACT_LEAKY, true>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__); \
      else                                                                                          \
        hipLaunchKernelGGL((KERNEL<ACT_LEAKY, false>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__);\
    } else {                                                                                        \
      if (has_res)                                                                                  \
        hipLaunchKernelGGL((KERNEL<ACT_NONE, true>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__);  \
      else                                                                                          \
        hipLaunchKernelGGL((KERNEL<ACT_NONE, false>), GRID, dim3(256), SHMEM, STREAM, __VA_ARGS__); \
    }                                                                                               \
  } while (0)

// Elementwise grid: two rows per thread and no practical cap on the workgroup count.  Measured
// on the R50 b512 stage-1/2 tensors (tools/ew_bench.py): 5.7-6.0 TB/s against 4.5 TB/s for a
// 4096-workgroup grid-stride loop over 8 rows per thread -- HBM wants the whole tensor's loads
// spread over many short-lived waves.  g_tune[kEwGridCap] / [10] override cap / rows (A/B only).
static inline dim3 ew_grid(int M, int C) {
  // 4 rows per thread where that still leaves >= 2048 workgroups (8 per CU): R50 b1024 +0.4 % over
  // 2 (same box, 4 pairs; 8 rows -0.6 %, 1 row -5 %: profiles/r3/ew_rows_ab.txt); small tensors 2
  const int cap = g_tune[kEwGridCap] > 0 ? g_tune[kEwGridCap] : (1 << 20);
  if (g_tune[kEwRows] > 0) return dim3(rows_grid(M, C, g_tune[kEwRows], cap));
  const int g4 = rows_grid(M, C, 4, cap);
  return dim3(g4 >= 2048 ? g4 : rows_grid(M, C, 2, cap));
}

void launch_bn_act_fwd(const bf16* x, const bf16* res, const float* scale, const float* shift, bf16* y,
                       size_t numel, int C, int act, float slope, hipStream_t s, uint8_t* mask,
                       const float* rscale, const float* rshift) {
  const int M = (int)(numel / C);
  const dim3 grid = ew_grid(M, C);
  DCP_ACT_RES_DISPATCH(bn_act_fwd_kernel, grid, 0, s, res, act, x, res, scale, shift, y, M, C, slope, g_tune[kBnActVariant],
                       mask, rscale, rshift);
}

void launch_bn_fin_act(const bf16* x, const bf16* res, const float* src, int nsrc, int partials, int M, int C,
                       float eps, const float* gamma, const float* beta, float* mean, float* invstd, float* scale,
                       float* shift, float* rm, float* rv, float momentum, float iabn_eps, float* rgamma, bf16* y,
                       uint8_t* mask, int act, float slope, uint32_t* sync, hipStream_t s) {
  FinActParams p;
  p.x = x; p.res = res; p.src = src; p.nsrc = nsrc; p.partials = partials; p.M = M; p.C = C;
  p.nfin = partials ? (C + 63) / 64 : (C + kSlabCh - 1) / kSlabCh;
  p.eps = eps; p.momentum = momentum; p.iabn_eps = iabn_eps; p.slope = slope;
  p.gamma = gamma; p.beta = beta; p.mean = mean; p.invstd = invstd; p.scale = scale; p.shift = shift;
  p.run_mean = rm; p.run_var = rv; p.rgamma = rgamma; p.y = y; p.mask = mask; p.sync = sync;
  // the apply grid of bn_act_fwd in 1024-thread workgroups (4 virtual 256-thread ones each)
  const int g = std::max(p.nfin, (int)((ew_grid(M, C).x + 3) / 4));
  const dim3 grid(g);
  if (act == ACT_RELU) {
    if (res) hipLaunchKernelGGL((bn_fin_act_kernel<ACT_RELU, true>), grid, dim3(1024), 0, s, p);
    else hipLaunchKernelGGL((bn_fin_act_kernel<ACT_RELU, false>), grid, dim3(1024), 0, s, p);
  } else if (act == ACT_LEAKY) {
    if (res) hipLaunchKernelGGL((bn_fin_act_kernel<ACT_LEAKY, true>), grid, dim3(1024), 0, s, p);
    else hipLaunchKernelGGL((bn_fin_act_kernel<ACT_LEAKY, false>), grid, dim3(1024), 0, s, p);
  } else {
    if (res) hipLaunchKernelGGL((bn_fin_act_kernel<ACT_NONE, true>), grid, dim3(1024), 0, s, p);
    else hipLaunchKernelGGL((bn_fin_act_kernel<ACT_NONE, false>), grid, dim3(1024), 0, s, p);
  }
}

int bn_direct_slabs() { return kDirectSlabs; }

// g_tune[kBnBwdCap] overrides the workgroup cap (A/B only: 256 and 1024 measured 0.5-1.2 % slower end to end
// at b1024, profiles/r3/ew_rows_ab.txt)
// 32 rows per thread where the cap binds (large activations); smaller ones spread over up to the cap's
// workgroups at >= 4 rows per thread: at batch 16 a TResNet-M layer's reduction ran as ~49 workgroups of
// 32 serial rows, 20 us of latency for a few MB (36 such layers per step)
int bn_bwd_reduce_blocks(int M, int C) {
  const int cap = g_tune[kBnBwdCap] > 0 ? g_tune[kBnBwdCap] : 512;
  const int g = rows_grid(M, C, 32, cap);
  return g < cap ? rows_grid(M, C, 4, cap) : g;
}

// partials must hold bn_bwd_reduce_blocks(M, C) x 2 x C floats; out [2][C]
void launch_bn_bwd_reduce(const bf16* dy, const bf16* x, const bf16* res, const float* scale, const float* shift,
                          const float* mean, const float* invstd, int M, int C, int act, float slope, float* partials,
                          float* out, hipStream_t s, int inv) {
  const int g = bn_bwd_reduce_blocks(M, C);
  DCP_ACT_RES_DISPATCH(bn_bwd_reduce_kernel, dim3(g), 2 * 2048 * 4, s, res, act, dy, x, res, scale, shift, mean,
                       invstd, M, C, slope, partials, inv);
  hipLaunchKernelGGL(partial_sum_kernel<float>, dim3((2 * C + 63) / 64), dim3(256), 0, s, partials, g, 2 * C, out);
}

void launch_bn_bwd_elemt(const bf16* dy, const bf16* x, const bf16* res, const float* scale, const float* shift,
                         const float* mean, const float* invstd, const float* sums, float inv_count, size_t numel,
                         int C, int act, float slope, bf16* dx, bf16* dres, hipStream_t s, int inv, const float* graw,
                         float* dg) {
  const int M = (int)(numel / C);
  const dim3 grid = ew_grid(M, C);
  DCP_ACT_RES_DISPATCH(bn_bwd_elemt_kernel, grid, 0, s, res, act, dy, x, res, scale, shift, mean, invstd, sums,
                       inv_count, M, C, slope, dx, dres, inv, graw, dg);
}


void launch_bn2_bwd_elemt(const bf16* dy, const bf16* x, const bf16* r, const float* scale, const float* mean,
                          const float* invstd, const float* sums, const float* rscale, const float* rmean,
                          const float* rinvstd, const float* rsums, float inv_count, size_t numel, int C, bf16* dx,
                          bf16* dr, hipStream_t s) {
  const int M = (int)(numel / C);
  hipLaunchKernelGGL(bn2_bwd_elemt_kernel, ew_grid(M, C), dim3(256), 0, s, dy, x, r, scale, mean, invstd, sums,
                     rscale, rmean, rinvstd, rsums, inv_count, M, C, dx, dr);
}

// Backward of the folded eval-mode BN (launchers.h AffineEpi) from its bf16 output y:
// g = dy * act'(y) (act' of the pre-activation: y keeps its sign), dc = g * scale per channel.
// G: also store g (the gradient of the residual added before the activation).
template <int ACT, bool G>
__global__ void __launch_bounds__(256) act_scale_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                            const float* __restrict__ scale, int M, int C, float slope,
                                                            bf16* __restrict__ dc, bf16* __restrict__ g) {
  const RowTile t(C);
  if (t.slot >= t.rpi) return;
  float sc[8];
  load8(scale + t.c0, sc);
  const int step = gridDim.x * t.rpi;
  for (int m = blockIdx.x * t.rpi + t.slot; m < M; m += step) {
    const size_t off = (size_t)m * C + t.c0;
    const bf16x8 d = *(const bf16x8*)(dy + off);
    const bf16x8 v = ACT ? *(const bf16x8*)(y + off) : bf16x8{};
    bf16x8 oc, og;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gk = bf2f(d[k]);
      if (ACT == 1 && !(bf2f(v[k]) > 0.f)) gk = 0.f;
      if (ACT == 2 && !(bf2f(v[k]) >= 0.f)) gk *= slope;
      og[k] = f2bf(gk);
      oc[k] = f2bf(gk * sc[k]);
    }
    *(bf16x8*)(dc + off) = oc;
    if (G) *(bf16x8*)(g + off) = og;
  }
}

void launch_act_scale_bwd(const bf16* dy, const bf16* y, const float* scale, int64_t M, int C, int act, float slope,
                          bf16* dc, bf16* g, hipStream_t s) {
  const dim3 grid = ew_grid((int)M, C);
#define DCP_ASB(A_)                                                                                          \
  if (g) hipLaunchKernelGGL((act_scale_bwd_kernel<A_, true>), grid, dim3(256), 0, s, dy, y, scale, (int)M, C, \
                            slope, dc, g);                                                                   \
  else hipLaunchKernelGGL((act_scale_bwd_kernel<A_, false>), grid, dim3(256), 0, s, dy, y, scale, (int)M, C,  \
                          slope, dc, g);
  if (act == 1) { DCP_ASB(1) }
  else if (act == 2) { DCP_ASB(2) }
  else { DCP_ASB(0) }
#undef DCP_ASB
}

}  // namespace dcp
