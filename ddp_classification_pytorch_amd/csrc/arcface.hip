// Fused ArcFace head (ArcMarginProduct + softmax cross-entropy), nothing [B, C] in memory.
//
// Reference: ARCFACE/arc_main.py:130-176 (ArcMarginProduct: cosine of the L2-normalised feature and
// class-weight rows, additive angular margin on the label column, scale s) and :245
// (nn.CrossEntropyLoss over those logits); SURVEY.md §2.5 K13.  The unfused path (loss.hip +
// the MFMA linear kernels) writes the bf16 cosine matrix [B, C] and its gradient [B, C] and reads
// each back twice; at 100k classes and batch 1024 that is 400 MB per step.  Here:
//
//   forward   arc_label_kernel        per row: cos(x_r, w_{y_r}) (fp32 dot of the bf16 operands),
//                                     target logit t_r = s * phi, d phi / d cos
//             arc_rows_kernel<0>      (row block x class split) workgroups stream 64-class tiles of
//                                     the normalised weights through LDS; the cosine tile is an MFMA
//                                     result in registers (v_mfma_f32_16x16x32_bf16, x fragments held
//                                     in VGPRs for the whole kernel); each lane keeps an online
//                                     log-sum-exp (max, scaled sum) and the label-rank count of the
//                                     margin logits for its row -> per-split partials [S][B]
//             arc_fwd_finalize        merges the splits: loss_r = lse_r - t_r, rank_r, lse_r saved
//   backward  arc_rows_kernel<1>      recomputes each cosine tile, forms
//                                     dcos = g s (softmax - onehot) (x dphi at the label) in registers
//                                     and feeds it straight into a second MFMA against the transposed
//                                     weight tile: dxn partials [S][B][D] (a few class splits)
//             arc_norm_bwd_kernel     sums the dxn splits and applies the L2-normalisation backward
//             arc_dw_kernel           one workgroup per 64-class block over ALL rows: recomputed
//                                     cosine tile (x tiles through LDS, the block's weight fragments
//                                     in VGPRs), dcos, MFMA against the transposed x tile -> the
//                                     block's complete dwn in registers, the normalisation backward
//                                     applied in the epilogue (cross-lane dot) -> dW written once.
//
// The dcos register tile becomes the next MFMA's B operand without any data movement: its
// accumulator layout (lane holds 4 consecutive rows of one column) is read as a 32-deep k-fragment
// whose k order is a fixed permutation, and the A operand is loaded in the same permuted order.
// Deterministic: every sum has a fixed order (no atomics).
#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {

constexpr int kArcTile = 64;  // classes (rows) per staged tile

struct ArcParams {
  const bf16* xn;    // [Bp][Dp] normalised features (rows >= B zero)
  const bf16* xnT;   // [Dp][Bp]
  const bf16* wn;    // [Cp][Dp] normalised class weights (rows >= C zero)
  const bf16* wnT;   // [Dp][Cp]
  const int64_t* labels;  // [B]
  const float* lab;  // [Bp][2]: target logit s * phi, d phi / d cos (0, 0 for an invalid row)
  const float* lse;  // [Bp] (backward)
  const float* gout; // [1] upstream gradient of the mean loss (backward)
  float* part;       // split partials
  float scale;       // 1 / B (mean reduction)
  int B, Bp, C, Cp, Dp, S, tps;
  float s;
};

// margin (ARCFACE/arc_main.py:157-176), guarded at cos = +-1
__device__ __forceinline__ void arc_margin(float c, float cos_m, float sin_m, float th, float mm, int easy, float& phi,
                                           float& dphi) {
  c = fminf(fmaxf(c, -1.f), 1.f);
  const float sn = sqrtf(fminf(fmaxf(1.f - c * c, 0.f), 1.f));
  const float p = c * cos_m - sn * sin_m;
  const float dp = cos_m + (sn > 1e-6f ? sin_m * c / sn : 0.f);
  if (easy) {
    phi = c > 0.f ? p : c;
    dphi = c > 0.f ? dp : 1.f;
  } else {
    phi = c > th ? p : c - mm;
    dphi = c > th ? dp : 1.f;
  }
}

// byte offset of 16-byte chunk c of row r in a row-major [rows][Dp] bf16 tile, XOR-swizzled
// (16 consecutive rows at one chunk -> 16 distinct bank groups for the fragment reads)
__device__ __forceinline__ uint32_t rm_off(uint32_t r, uint32_t c, uint32_t Dp) {
  return r * Dp * 2u + ((c ^ (r & 15u)) << 4);
}
// byte offset of 8-byte half h of chunk c of row d in a [Dp][64] bf16 tile (128-byte rows)
__device__ __forceinline__ uint32_t tr_off(uint32_t d, uint32_t c, uint32_t h) {
  return d * 128u + ((c ^ (d & 7u)) << 4) + (h << 3);
}

// LDS-DMA versions of the two stagings (one 16-byte global_load_lds per lane and instruction, the
// lane's data landing at base + 16 lane: the swizzle is applied on the source side).  Untracked: the
// caller waits vmcnt(0) + barrier before reading the tile.  4 waves share the tile.
template <int DP>
__device__ __forceinline__ void dma_rm(char* T, const bf16* g, int r0, int w, int lane) {
  constexpr int CPR = DP / 8, RPB = 64 / CPR, NI = kArcTile / RPB / 4;  // rows per 1 KB block; blocks per wave
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int blk = w * NI + i;
    const int r = blk * RPB + lane / CPR, pos = lane % CPR;
    const int c = pos ^ (r & 15);
    dma16(g + (size_t)(r0 + r) * DP + c * 8, T + blk * 1024);
  }
}
template <int DP>
__device__ __forceinline__ void dma_tr(char* T, const bf16* g, int c0, int ld, int w, int lane) {
  constexpr int NI = DP / 8 / 4;  // 8 rows (128 B each) per 1 KB block
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int blk = w * NI + i;
    const int d = blk * 8 + lane / 8, pos = lane % 8;
    const int c = pos ^ (d & 7);
    dma16(g + (size_t)d * ld + c0 + c * 8, T + blk * 1024);
  }
}

// the 8 bf16 of a permuted 32-deep k-fragment from a transposed tile: k slots 8q..8q+3 <- columns
// 32 kk + 4q .. +3, slots 8q+4..8q+7 <- columns 32 kk + 16 + 4q .. +3 (the accumulator layout of
// two 16-wide MFMA results, read as one k-fragment)
__device__ __forceinline__ bf16x8 tr_frag(const char* T, uint32_t d, int kk, uint32_t q) {
  const uint32_t lo = 32u * kk + 4u * q, hi = lo + 16u;  // column indices (bf16)
  const bf16x4 a = *LDS_PTR(const bf16x4, T + tr_off(d, lo >> 3, (lo >> 2) & 1u));
  const bf16x4 b = *LDS_PTR(const bf16x4, T + tr_off(d, hi >> 3, (hi >> 2) & 1u));
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

}  // namespace

// rows of x [R][D] (fp32 or bf16) -> normalised bf16 rows y [Rp][Dp] AND their transpose yT [Dp][Rp]
// (zero padding in both dimensions), inverse norms [Rp]: the operands of the fused head in one pass
// (a separate transpose launch per operand cost as much as the normalisation).  One workgroup per
// 64 rows; each wave normalises 16 rows, the tile is transposed through LDS.
template <typename T, int DP>
__global__ void __launch_bounds__(256) arc_l2norm_t_kernel(const T* __restrict__ x, int R, int D, int Rp,
                                                           bf16* __restrict__ y, bf16* __restrict__ yT,
                                                           float* __restrict__ inv_norm, float eps) {
  constexpr int EPL = DP / 64;  // elements per lane of a row
  __shared__ __attribute__((aligned(16))) bf16 tile[64][DP + 8];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.x * 64;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int rl = w * 16 + k, r = r0 + rl;
    float v[EPL];
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int j = lane * EPL + e;
      v[e] = (r < R && j < D) ? (float)x[(size_t)r * D + j] : 0.f;
      ss += v[e] * v[e];
    }
    ss = wave_sum(ss);
    const float iv = r < R ? 1.f / fmaxf(sqrtf(ss), eps) : 0.f;
    if (lane == 0) inv_norm[r] = iv;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const bf16 b = f2bf(v[e] * iv);
      tile[rl][lane * EPL + e] = b;
      y[(size_t)r * DP + lane * EPL + e] = b;
    }
  }
  __syncthreads();
  // yT rows d: the 64 columns r0 .. r0 + 63 (128 contiguous bytes); a thread writes 8 columns
  for (int e = threadIdx.x; e < DP * 8; e += 256) {
    const int d = e >> 3, c = (e & 7) * 8;
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = tile[c + k][d];
    *(bf16x8*)(yT + (size_t)d * Rp + r0 + c) = o;
  }
}

// per row: target logit and margin derivative (one wave per row)
__global__ void __launch_bounds__(256) arc_label_kernel(const bf16* __restrict__ xn, const bf16* __restrict__ wn,
                                                        const int64_t* __restrict__ labels, int B, int Bp, int C,
                                                        int Dp, float s, float cos_m, float sin_m, float th, float mm,
                                                        int easy, float* __restrict__ lab) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= Bp) return;
  const int y = r < B ? (int)labels[r] : -1;
  const bool valid = y >= 0 && y < C;
  float acc = 0.f;
  if (valid)
    for (int j = lane; j < Dp; j += 64) acc += bf2f(xn[(size_t)r * Dp + j]) * bf2f(wn[(size_t)y * Dp + j]);
  acc = wave_sum(acc);
  if (lane == 0) {
    float phi = 0.f, dphi = 0.f;
    if (valid) arc_margin(acc, cos_m, sin_m, th, mm, easy, phi, dphi);
    lab[2 * r] = valid ? s * phi : 0.f;
    lab[2 * r + 1] = valid ? dphi : 0.f;
  }
}

// MODE 0: forward partials (max, scaled sum, rank count) per (split, row);
// MODE 1: dxn partials [S][Bp][Dp].  Grid (Bp / 64, S); 4 waves x 16 rows.
template <int KS, int MODE>
__global__ void __launch_bounds__(256, 2) arc_rows_kernel(const ArcParams p) {
  constexpr int DP = KS * 32, DF = DP / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // two buffers of [64 classes][DP] swizzled (+ [DP][64 classes] for MODE 1), LDS-DMA double buffered
  constexpr int BUF = kArcTile * DP * 2 * (MODE == 1 ? 2 : 1);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = lane >> 4, l15 = lane & 15;
  // XCD-aware (row block, split) of this workgroup: workgroups are dispatched round-robin over the 8
  // XCDs, so the ones sharing an XCD (and its L2) take the SAME class splits for all row blocks --
  // each XCD streams 1/8 of the weight tiles instead of all of them
  int rb = blockIdx.x, split = blockIdx.y;
  {
    const int RB = gridDim.x, S = gridDim.y, L = blockIdx.x + blockIdx.y * RB;
    if ((S & 7) == 0) {
      const int xcd = L & 7, idx = L >> 3;
      split = xcd * (S >> 3) + idx / RB;
      rb = idx % RB;
    }
  }
  const int row = rb * 64 + w * 16 + (int)l15;
  // this lane's x fragments (n = row), the whole feature dimension, in VGPRs
  bf16x8 xf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) xf[ks] = *(const bf16x8*)(p.xn + (size_t)row * DP + ks * 32 + q * 8);
  const int y = row < p.B ? (int)p.labels[row] : -1;
  const bool valid = y >= 0 && y < p.C;
  const float t = p.lab[2 * row], dphi = p.lab[2 * row + 1];
  float lse = 0.f, gs = 0.f;
  if constexpr (MODE == 1) {
    lse = p.lse[row];
    gs = valid ? p.gout[0] * p.scale * p.s : 0.f;
  }
  float run_m = -INFINITY, run_s = 0.f, cnt = 0.f;
  f32x4 dacc[MODE == 1 ? DF : 1];
  if constexpr (MODE == 1)
#pragma unroll
    for (int f = 0; f < DF; ++f) dacc[f] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ntiles = p.Cp / kArcTile;
  const int t0 = split * p.tps, t1 = min(ntiles, t0 + p.tps);
  auto stage = [&](int tile, int b) {
    char* Wb = smem + b * BUF;
    dma_rm<DP>(Wb, p.wn, tile * kArcTile, w, lane);
    if constexpr (MODE == 1) dma_tr<DP>(Wb + kArcTile * DP * 2, p.wnT, tile * kArcTile, p.Cp, w, lane);
  };
  if (t0 < t1) stage(t0, 0);
  for (int tile = t0; tile < t1; ++tile) {
    const int c0 = tile * kArcTile, b = (tile - t0) & 1;
    const char* Wt = smem + b * BUF;
    const char* WT = Wt + kArcTile * DP * 2;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // this tile landed for every wave; the other buffer's reads are done
    asm volatile("" ::: "memory");
    if (tile + 1 < t1) stage(tile + 1, b ^ 1);
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 a = *LDS_PTR(const bf16x8, Wt + rm_off(16 * j + l15, ks * 4 + q, DP));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xf[ks], acc[j], 0, 0, 0);
      }
    // lane: cos of classes c0 + 16 j + 4 q + i (i = 0..3) for its row
    if constexpr (MODE == 0) {
      float v[16];
      float tmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cls = c0 + 16 * j + 4 * (int)q + i;
          const bool on = cls < p.C;
          const float x = cls == y ? t : p.s * acc[j][i];
          v[4 * j + i] = on ? x : -INFINITY;
          tmax = fmaxf(tmax, v[4 * j + i]);
          cnt += (on && cls != y && x > t) ? 1.f : 0.f;
        }
      const float m_new = fmaxf(run_m, tmax);
      if (m_new > -INFINITY) {
        float sum = run_m > -INFINITY ? run_s * __expf(run_m - m_new) : 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) sum += __expf(v[k] - m_new);
        run_s = sum;
        run_m = m_new;
      }
    } else {
      bf16x8 dfr[2];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cls = c0 + 16 * j + 4 * (int)q + i;
          const bool lab_col = cls == y;
          const float x = lab_col ? t : p.s * acc[j][i];
          const float pr = __expf(x - lse);
          const float d0 = gs * (pr - (lab_col ? 1.f : 0.f)) * (lab_col ? dphi : 1.f);
          const float d = (valid && cls < p.C) ? d0 : 0.f;  // (a select: padding rows carry no lse)
          dfr[j >> 1][(j & 1) * 4 + i] = f2bf(d);
        }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < DF; ++f) {
          const bf16x8 a = tr_frag(WT, 16u * f + l15, kk, q);
          dacc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, dfr[kk], dacc[f], 0, 0, 0);
        }
    }
  }
  if constexpr (MODE == 0) {
    // the 4 lanes of a row (l15, + 16, + 32, + 48): merge (max, sum) and counts
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float om = __shfl_xor(run_m, o, 64), os = __shfl_xor(run_s, o, 64), oc = __shfl_xor(cnt, o, 64);
      const float m_new = fmaxf(run_m, om);
      float sum = 0.f;
      if (m_new > -INFINITY) {
        sum = (run_m > -INFINITY ? run_s * __expf(run_m - m_new) : 0.f) +
              (om > -INFINITY ? os * __expf(om - m_new) : 0.f);
      }
      run_m = m_new;
      run_s = sum;
      cnt += oc;
    }
    if (q == 0) {
      float* o = p.part + ((size_t)split * p.Bp + row) * 4;
      *(f32x4*)o = f32x4{run_m, run_s, cnt, 0.f};
    }
  } else {
    // lane holds dxn[row][16 f + 4 q + i]
    float* o = p.part + ((size_t)split * p.Bp + row) * DP + 4 * q;
#pragma unroll
    for (int f = 0; f < DF; ++f) *(f32x4*)(o + 16 * f) = dacc[f];
  }
}

// merge the forward splits per row: loss, label rank, lse (saved for the backward)
__global__ void __launch_bounds__(256) arc_fwd_finalize_kernel(const float* __restrict__ part, int S, int B, int Bp,
                                                               int C, const int64_t* __restrict__ labels,
                                                               const float* __restrict__ lab,
                                                               float* __restrict__ loss, int* __restrict__ rank,
                                                               float* __restrict__ lse) {
  // one wave per row, one lane per split (S <= 64): the split loads go out together, the merge is a
  // wave reduction (a thread-per-row loop over 64 splits was a 22 us latency chain)
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= Bp) return;
  if (r >= B) {  // padding rows: a defined lse for the backward kernels (their gradient is zero)
    if (lane == 0) lse[r] = 0.f;
    return;
  }
  f32x4 v = f32x4{-INFINITY, 0.f, 0.f, 0.f};
  if (lane < S) v = *(const f32x4*)(part + ((size_t)lane * Bp + r) * 4);
  const float M = wave_max(v[0]);
  const float sum = wave_sum(v[0] > -INFINITY ? v[1] * __expf(v[0] - M) : 0.f);
  const float cnt = wave_sum(v[2]);
  if (lane == 0) {
    const float l = M + __logf(sum);
    const int y = (int)labels[r];
    const bool valid = y >= 0 && y < C;
    lse[r] = l;
    loss[r] = valid ? l - lab[2 * r] : 0.f;
    if (rank) rank[r] = (int)cnt;
  }
}

// rows r < R: g = sum_s part[s][r][:D] (fp32), out[r] = inv[r] * (g - y[r] <g, y[r]>)  (the backward of
// y = x / |x|), out fp32 or bf16 [R][D]
template <typename TO>
__global__ void __launch_bounds__(256) arc_norm_bwd_kernel(const float* __restrict__ part, int S, size_t sstride,
                                                           const bf16* __restrict__ y, int Dp, int D,
                                                           const float* __restrict__ inv, TO* __restrict__ out) {
  __shared__ float red[16];
  const int r = blockIdx.x;
  float dot = 0.f;
  float g[2] = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = threadIdx.x + 256 * k;
    if (j < D) {
      // the split partials' loads issued together (up to 16 in flight), summed in split order
      float a = 0.f;
      for (int s0 = 0; s0 < S; s0 += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = s0 + u < S ? part[(s0 + u) * sstride + (size_t)r * Dp + j] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) a += v[u];
      }
      g[k] = a;
      dot += a * bf2f(y[(size_t)r * Dp + j]);
    }
  }
  dot = block_sum(dot, red);
  const float iv = inv[r];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = threadIdx.x + 256 * k;
    if (j < D) out[(size_t)r * D + j] = (TO)(iv * (g[k] - bf2f(y[(size_t)r * Dp + j]) * dot));
  }
}

// dW: one workgroup per 64-class block over every row; 4 waves x 16 classes.  Writes
// dw[c][:D] = inv_w[c] (dwn - wn <dwn, wn>) for c < C (fp32).
// With p.S > 1 row splits (grid.y), each split writes its dwn partial to p.part [S][Cp][DP] instead
// and arc_norm_bwd_kernel sums the splits and applies the normalisation backward (small C: the
// 64-class blocks alone leave most CUs idle).
template <int KS>
__global__ void __launch_bounds__(256, 2) arc_dw_kernel(const ArcParams p, const float* __restrict__ inv_w,
                                                        int D, float* __restrict__ dw) {
  constexpr int DP = KS * 32, DF = DP / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // two buffers of ([64 rows][DP] swizzled, [DP][64 rows]), LDS-DMA double buffered, then the
  // per-row (label, t, dphi, lse) of every row, staged once
  constexpr int BUF = kArcTile * DP * 2 * 2;
  float* info = (float*)(smem + 2 * BUF);  // [Bp][4]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = lane >> 4, l15 = lane & 15;
  const int cls = blockIdx.x * 64 + w * 16 + (int)l15;
  bf16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) wf[ks] = *(const bf16x8*)(p.wn + (size_t)cls * DP + ks * 32 + q * 8);
  const float g0 = p.gout[0] * p.scale * p.s;
  f32x4 dacc[DF];
#pragma unroll
  for (int f = 0; f < DF; ++f) dacc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int r = tid; r < p.Bp; r += 256) {
    const int y = r < p.B ? (int)p.labels[r] : -1;
    const bool valid = y >= 0 && y < p.C;
    *LDS_PTR(f32x4, info + r * 4) = f32x4{valid ? (float)y : -1.f, p.lab[2 * r], p.lab[2 * r + 1], p.lse[r]};
  }
  auto stage = [&](int r0, int b) {
    char* Xb = smem + b * BUF;
    dma_rm<DP>(Xb, p.xn, r0, w, lane);
    dma_tr<DP>(Xb + kArcTile * DP * 2, p.xnT, r0, p.Bp, w, lane);
  };
  // this split's row tiles
  const int nrt = p.Bp / kArcTile, rps = (nrt + p.S - 1) / p.S;
  const int rt0 = blockIdx.y * rps, rt1 = min(nrt, rt0 + rps);
  const int rbeg = rt0 * kArcTile, rend = rt1 * kArcTile;
  if (rbeg < rend) stage(rbeg, 0);
  for (int r0 = rbeg; r0 < rend; r0 += kArcTile) {
    const int b = ((r0 - rbeg) / kArcTile) & 1;
    const char* Xt = smem + b * BUF;
    const char* XT = Xt + kArcTile * DP * 2;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // this row tile landed for every wave; the other buffer is free
    asm volatile("" ::: "memory");
    if (r0 + kArcTile < rend) stage(r0 + kArcTile, b ^ 1);
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 a = *LDS_PTR(const bf16x8, Xt + rm_off(16 * j + l15, ks * 4 + q, DP));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc[j], 0, 0, 0);
      }
    // lane: cos of rows r0 + 16 j + 4 q + i for class cls
    bf16x8 dfr[2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 16 * j + 4 * (int)q + i;
        const f32x4 in = *LDS_PTR(const f32x4, info + (r0 + rl) * 4);
        const bool lab_col = (float)cls == in[0];
        const float x = lab_col ? in[1] : p.s * acc[j][i];
        const float pr = __expf(x - in[3]);
        const float d0 = g0 * (pr - (lab_col ? 1.f : 0.f)) * (lab_col ? in[2] : 1.f);
        const float d = (in[0] >= 0.f && cls < p.C) ? d0 : 0.f;
        dfr[j >> 1][(j & 1) * 4 + i] = f2bf(d);
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < DF; ++f) {
        const bf16x8 a = tr_frag(XT, 16u * f + l15, kk, q);
        dacc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, dfr[kk], dacc[f], 0, 0, 0);
      }
  }
  if (p.S > 1) {  // a row split's partial: summed and normalised by arc_norm_bwd_kernel
    float* o = p.part + ((size_t)blockIdx.y * p.Cp + cls) * DP + 4 * q;
#pragma unroll
    for (int f = 0; f < DF; ++f) *(f32x4*)(o + 16 * f) = dacc[f];
    return;
  }
  // lane holds dwn[cls][16 f + 4 q + i]; the normalisation backward needs <dwn, wn> per class:
  // the 4 lanes of a class (q = 0..3) hold disjoint dimensions
  float dot = 0.f;
#pragma unroll
  for (int f = 0; f < DF; ++f) {
    const bf16x4 wv = *(const bf16x4*)(p.wn + (size_t)cls * DP + 16 * f + 4 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) dot += dacc[f][i] * bf2f(wv[i]);
  }
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);
  if (cls >= p.C) return;
  const float iv = inv_w[cls];
#pragma unroll
  for (int f = 0; f < DF; ++f) {
    const bf16x4 wv = *(const bf16x4*)(p.wn + (size_t)cls * DP + 16 * f + 4 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 16 * f + 4 * (int)q + i;
      if (j < D) dw[(size_t)cls * D + j] = iv * (dacc[f][i] - bf2f(wv[i]) * dot);
    }
  }
}

// ---------------------------------------------------------------------------
namespace {
int arc_splits(int blocks, int ntiles, int target, int cap) {
  int s = (target + blocks - 1) / std::max(1, blocks);
  s = std::max(1, std::min(s, std::min(ntiles, cap)));
  return s;
}
template <int KS>
void set_lds(const void* f, size_t bytes) {
  (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
}  // namespace

bool launch_arcface_l2norm_t(const void* x, bool is_bf16, int R, int D, int Rp, int Dp, bf16* y, bf16* yT, float* inv,
                             float eps, hipStream_t st) {
  if (Rp % 64 || Rp < R || D > Dp || !(Dp == 128 || Dp == 256)) return false;
#define ARC_NT(T_, DP_) \
  hipLaunchKernelGGL((arc_l2norm_t_kernel<T_, DP_>), dim3(Rp / 64), dim3(256), 0, st, (const T_*)x, R, D, Rp, y, yT, inv, eps);
  if (is_bf16) {
    if (Dp == 128) { ARC_NT(bf16, 128) } else { ARC_NT(bf16, 256) }
  } else {
    if (Dp == 128) { ARC_NT(float, 128) } else { ARC_NT(float, 256) }
  }
#undef ARC_NT
  return true;
}

int arcface_fused_fwd_splits(int Bp, int Cp) {
  const int s = arc_splits(Bp / 64, Cp / kArcTile, 1024, 64);
  return s >= 8 ? s / 8 * 8 : s;
}
int arcface_fused_dx_splits(int Bp, int Cp) {
  const int s = arc_splits(Bp / 64, Cp / kArcTile, 256, 16);
  return s >= 8 ? s / 8 * 8 : s;  // multiples of 8: the XCD-aware split mapping
}

bool launch_arcface_fused_fwd(const bf16* xn, const bf16* wn, const int64_t* labels, int B, int Bp, int C, int Cp,
                              int Dp, float s, float m, int easy, float* lab, float* part, float* loss, int* rank,
                              float* lse, hipStream_t st) {
  if (Bp % 64 || Cp % kArcTile || !(Dp == 128 || Dp == 256)) return false;
  const float cm = cosf(m), sm = sinf(m), th = cosf(3.14159265358979f - m), mm = sinf(3.14159265358979f - m) * m;
  hipLaunchKernelGGL(arc_label_kernel, dim3(Bp / 4), dim3(256), 0, st, xn, wn, labels, B, Bp, C, Dp, s, cm, sm, th, mm,
                     easy, lab);
  ArcParams p{};
  p.xn = xn; p.wn = wn; p.labels = labels; p.lab = lab; p.part = part;
  p.B = B; p.Bp = Bp; p.C = C; p.Cp = Cp; p.Dp = Dp; p.s = s;
  p.S = arcface_fused_fwd_splits(Bp, Cp);
  p.tps = (Cp / kArcTile + p.S - 1) / p.S;
  const size_t lds = (size_t)kArcTile * Dp * 2 * 2;
  const dim3 grid(Bp / 64, p.S);
#define ARC_FWD(KS_)                                                                                   \
  set_lds<KS_>((const void*)arc_rows_kernel<KS_, 0>, lds);                                            \
  hipLaunchKernelGGL((arc_rows_kernel<KS_, 0>), grid, dim3(256), lds, st, p);
  if (Dp == 128) { ARC_FWD(4) } else { ARC_FWD(8) }
#undef ARC_FWD
  hipLaunchKernelGGL(arc_fwd_finalize_kernel, dim3(Bp / 4), dim3(256), 0, st, part, p.S, B, Bp, C, labels,
                     lab, loss, rank, lse);
  return true;
}

bool launch_arcface_fused_dx(const bf16* xn, const bf16* wn, const bf16* wnT, const int64_t* labels, int B, int Bp,
                             int C, int Cp, int Dp, int D, float s, const float* lab, const float* lse,
                             const float* gout, float scale, const float* inv_x, float* part, void* dx, bool dx_bf16,
                             hipStream_t st) {
  if (Bp % 64 || Cp % kArcTile || !(Dp == 128 || Dp == 256) || D > Dp) return false;
  ArcParams p{};
  p.xn = xn; p.wn = wn; p.wnT = wnT; p.labels = labels; p.lab = lab; p.lse = lse; p.gout = gout; p.part = part;
  p.scale = scale; p.B = B; p.Bp = Bp; p.C = C; p.Cp = Cp; p.Dp = Dp; p.s = s;
  p.S = arcface_fused_dx_splits(Bp, Cp);
  p.tps = (Cp / kArcTile + p.S - 1) / p.S;
  const size_t lds = (size_t)kArcTile * Dp * 2 * 2 * 2;
  const dim3 grid(Bp / 64, p.S);
#define ARC_DX(KS_)                                                                                    \
  set_lds<KS_>((const void*)arc_rows_kernel<KS_, 1>, lds);                                            \
  hipLaunchKernelGGL((arc_rows_kernel<KS_, 1>), grid, dim3(256), lds, st, p);
  if (Dp == 128) { ARC_DX(4) } else { ARC_DX(8) }
#undef ARC_DX
  const size_t ss = (size_t)Bp * Dp;
  if (dx_bf16)
    hipLaunchKernelGGL(arc_norm_bwd_kernel<bf16>, dim3(B), dim3(256), 0, st, part, p.S, ss, xn, Dp, D, inv_x,
                       (bf16*)dx);
  else
    hipLaunchKernelGGL(arc_norm_bwd_kernel<float>, dim3(B), dim3(256), 0, st, part, p.S, ss, xn, Dp, D, inv_x,
                       (float*)dx);
  return true;
}

int arcface_fused_dw_splits(int Bp, int Cp) {
  // row splits only when the class blocks leave most CUs idle (each split adds a [Cp][Dp] fp32 partial)
  const int blocks = Cp / 64;
  // (one workgroup per CU: a grid past 256 leaves a partly idle second round)
  return std::max(1, std::min(std::min(4, Bp / 64), 256 / std::max(1, blocks)));
}

bool launch_arcface_fused_dw(const bf16* xn, const bf16* xnT, const bf16* wn, const int64_t* labels, int B, int Bp,
                             int C, int Cp, int Dp, int D, float s, const float* lab, const float* lse,
                             const float* gout, float scale, const float* inv_w, float* part, float* dw,
                             hipStream_t st) {
  if (Bp % 64 || Cp % kArcTile || !(Dp == 128 || Dp == 256) || D > Dp) return false;
  ArcParams p{};
  p.xn = xn; p.xnT = xnT; p.wn = wn; p.labels = labels; p.lab = lab; p.lse = lse; p.gout = gout;
  p.scale = scale; p.B = B; p.Bp = Bp; p.C = C; p.Cp = Cp; p.Dp = Dp; p.s = s;
  p.S = arcface_fused_dw_splits(Bp, Cp);
  p.part = part;
  if (p.S > 1 && part == nullptr) return false;
  const size_t lds = (size_t)kArcTile * Dp * 2 * 2 * 2 + (size_t)Bp * 16;
  if (lds > 160 * 1024) return false;
#define ARC_DW(KS_)                                                                                    \
  set_lds<KS_>((const void*)arc_dw_kernel<KS_>, lds);                                                 \
  hipLaunchKernelGGL((arc_dw_kernel<KS_>), dim3(Cp / 64, p.S), dim3(256), lds, st, p, inv_w, D, dw);
  if (Dp == 128) { ARC_DW(4) } else { ARC_DW(8) }
#undef ARC_DW
  if (p.S > 1)
    hipLaunchKernelGGL(arc_norm_bwd_kernel<float>, dim3(C), dim3(256), 0, st, part, p.S, (size_t)Cp * Dp, wn, Dp, D,
                       inv_w, dw);
  return true;
}

}  // namespace dcp
