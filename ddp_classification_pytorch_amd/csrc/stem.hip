// Forward of the ResNet stem convolution in its space-to-depth form, as a dedicated kernel.
//
// The 7x7 / stride-2 / pad-3 stem conv of torchvision's resnet50 (BASELINE/main.py builds it
// through models.resnet50; SURVEY.md §2 kernel K1) runs as a 4x4 / stride-1 conv over the
// 2x2 space-to-depth input, [N][H][W][16] -> [N][H][W][64], padded 2 top/left and 1
// bottom/right (ops/functional.py stem_s2d_weight).  The generic implicit GEMM
// (conv_igemm.hip) stages every input pixel once per tap -- 16 times -- through LDS.  Here a
// workgroup owns a strip of kStemRows output rows of one image:
//  * the 64 x 256 weight is held in registers (16 MFMA A-fragments per lane), loaded once;
//  * input rows stream through an LDS ring of kSlots row slots by LDS-DMA, two rows per step,
//    one step ahead of the MFMAs.  A slot keeps the two 8-channel halves of the 16 input
//    channels in separate planes of 16-byte pixels with a 128-pixel pitch, which puts the
//    16 lanes of every B-fragment read on 16 distinct 16-byte bank groups;
//  * a wave computes 32 output channels of one whole output row per step (W/16 MFMA tiles
//    per 16-channel group), stages the bf16 row pair in LDS for 16-byte coalesced stores and
//    accumulates shifted per-channel sums of the fp32 accumulators,
//    turned into (n, mean, M2) and merged per workgroup into part[block][3][64] -- the first
//    level of the BatchNorm statistics (bn.hip), so bn_stats / bn_stats_finalize skip the
//    slab pass.
#include <algorithm>

#include <type_traits>

#include "common.cuh"
#include "launchers.h"
#include "pool_gather.cuh"

namespace dcp {

namespace {
constexpr int kPlanePx = 128;                  // pixels per channel-half plane (>= W + 4)
constexpr int kSlotBytes = 2 * kPlanePx * 16;  // one input row: two planes, 4 KB
constexpr int kSlots = 8;                      // ring of input rows (5 in use + 2 in flight)
constexpr int kStemRows = 16;                  // output rows per workgroup
constexpr int kStemCo = 64, kStemK = 256;      // output channels, 4 x 4 taps x 16 channels

struct StemParams {
  const bf16* x;     // [N][H][W][16]
  const bf16* w;     // [64][4][4][16]
  bf16* y;           // [N][H][W][64]
  float* part;       // [blocks][3][64] (n, mean, M2) or nullptr
  const bf16* zero;  // 16 zero bytes (out-of-image rows)
  int H, bpi;        // rows, workgroups per image
};

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
}  // namespace

// W output columns in NSUB 16-pixel MFMA tiles (W a multiple of 8: the last tile of a W = 56 row --
// the 112 px ArcFace input -- is half valid; its other lanes compute unused columns, skipped in
// the stores and the statistics)
template <int NSUB, int W = NSUB * 16>
__global__ void __launch_bounds__(256, 2) stem_fwd_kernel(StemParams p) {
  constexpr bool PART = W != NSUB * 16;
  constexpr int NST = PART ? (16 * W - 192 + 255) / 256 : NSUB;  // 16-byte stores per step, last wave
  static_assert(W + 4 <= kPlanePx, "row does not fit a plane");
  static_assert(W % 8 == 0 && W > 16 * (NSUB - 1) && W <= 16 * NSUB, "W in the last tile");
  // [kSlots * kSlotBytes ring][2 * W * 128 B output staging of one row pair]
  extern __shared__ __attribute__((aligned(16))) char ring[];
  char* stage = ring + kSlots * kSlotBytes;
  __shared__ float xch[3][kStemCo];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave & 1, rp = wave >> 1;  // channel half (32 co), row of the step pair
  const int H = p.H;
  const int n = blockIdx.x / p.bpi;
  const int r0 = (blockIdx.x - n * p.bpi) * kStemRows;
  const int r1 = min(H, r0 + kStemRows);
  const uint32_t l16 = lane & 15, kq = lane >> 4;

  // weights -> A fragments: wf[j][s] = w[co][32 s + 8 kq .. +8], co = (2 cg + j) * 16 + l16
  bf16x8 wf[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      wf[j][s] = *(const bf16x8*)(p.w + (size_t)((2 * cg + j) * 16 + l16) * kStemK + s * 32 + kq * 8);

  // padding pixels 0, 1, W+2, W+3 of both planes of every slot (LDS-DMA never writes them)
  if (tid < kSlots * 2 * 4) {
    const int q = tid & 3, px = q < 2 ? q : W + q;
    *(u32x4*)(ring + (tid >> 3) * kSlotBytes + ((tid >> 2) & 1) * (kPlanePx * 16) + px * 16) = u32x4{0, 0, 0, 0};
  }

  // input row ir -> its slot; wave (plane wave>>1, columns (wave&1)*64 + lane), one DMA per row
  const int lq = wave >> 1;
  const int lpx = (wave & 1) * 64 + lane;
  auto load_row = [&](int ir) {
    char* dst = ring + ((ir + kSlots) & (kSlots - 1)) * kSlotBytes + lq * (kPlanePx * 16) + (2 + (wave & 1) * 64) * 16;
    const bf16* g = (unsigned)ir < (unsigned)H ? p.x + ((size_t)(n * H + ir) * W + lpx) * 16 + lq * 8 : p.zero;
    if (lpx < W) dma16(g, dst);
  };
#pragma unroll
  for (int d = -2; d <= 2; ++d) load_row(r0 + d);

  // statistics: per lane and channel, sums of (v - K) and (v - K)^2 over the lane's pixels with
  // K = the lane's first value of the channel (c = 4 j + r; scalar fp32: packed fp32 beside
  // MFMAs costs more than it saves)
  float shf[8], s1[8], s2[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) shf[c] = s1[c] = s2[c] = 0.f;

  const int nsteps = (r1 - r0) >> 1;
  for (int st = 0; st < nsteps; ++st) {
    const int y0 = r0 + 2 * st;
    // rows y0-2 .. y0+2 landed: they were issued before the previous step's NSUB output stores
    // per lane (vmcnt counts loads, stores and LDS-DMA together, in issue order).  After the
    // barrier every wave is done with the previous step's ring slots and staging reads.
    if (st == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // also publishes the zeroed padding
    } else {
      // (PART: the last store instruction has no lanes in the upper waves, which then issued
      // NST stores -- the fewest of any wave; a smaller count only waits longer)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (st + 1 < nsteps) {
      load_row(y0 + 3);
      load_row(y0 + 4);
    }

    const int yy = y0 + rp;
    f32x4 acc[2][NSUB];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < NSUB; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      // k-step s: tap row ty = s/2, tap columns tx = 2 (s&1) + kq/2, channel half kq&1
      const int ir = yy + (s >> 1) - 2;
      const char* base = ring + ((ir + kSlots) & (kSlots - 1)) * kSlotBytes + (kq & 1) * (kPlanePx * 16) +
                         (l16 + (s & 1) * 2 + (kq >> 1)) * 16;
      bf16x8 af[NSUB];
#pragma unroll
      for (int i = 0; i < NSUB; ++i) af[i] = *(const bf16x8*)(base + i * 256);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < NSUB; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], af[i], acc[j][i], 0, 0, 0);
    }

    // epilogue: lane holds co = (2 cg + j) * 16 + 4 kq + r of pixel i * 16 + l16.  The row pair
    // is contiguous in memory (2 W pixels x 128 B): staged in LDS in that order, 8-byte slots
    // of a pixel XOR-swizzled by the pixel index (conflict-free 8-byte writes), then written
    // by every thread as 16-byte stores, 4 KB per workgroup instruction (8-byte stores from
    // the accumulators are store-issue bound).
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < NSUB; ++i) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[j][i][r]);
        const uint32_t px = rp * W + i * 16 + l16;
        const uint32_t slot = (((2 * cg + j) * 4 + kq) ^ (px & 15));
        if (!PART || i * 16 + (int)l16 < W) *(bf16x4*)(stage + px * 128 + slot * 8) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // not __syncthreads: keep the loads in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16* ydst = p.y + (size_t)(n * H + y0) * W * kStemCo;
#pragma unroll
    for (int k = 0; k < NSUB; ++k) {
      const uint32_t q = k * 256 + tid, px = q >> 3, c = q & 7, sw = px & 15;
      if (PART && q >= 16u * W) break;  // 2 W pixels x 8 chunks
      u32x4 v = *(const u32x4*)(stage + px * 128 + ((c ^ (sw >> 1)) << 4));
      if (sw & 1) v = u32x4{v[2], v[3], v[0], v[1]};
      *(u32x4*)(ydst + (size_t)q * 8) = v;
    }
    if (p.part) {
      if (st == 0)
#pragma unroll
        for (int c = 0; c < 8; ++c) shf[c] = acc[c >> 2][0][c & 3];
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int i = 0; i < NSUB; ++i) {
          if (PART && i == NSUB - 1 && (int)l16 >= W - 16 * (NSUB - 1)) continue;
          const float d = acc[c >> 2][i][c & 3] - shf[c];
          s1[c] += d;
          s2[c] = fmaf(d, d, s2[c]);
        }
    }
  }

  if (p.part) {
    // lane (n, mean, M2) per channel, merged over the 16 lanes of the pixel group (equal counts),
    // then across the two row waves of each channel half through LDS
    // lanes of a partial last tile hold one column fewer: count-weighted merges (PART)
    const int lane_cols = (PART && (int)l16 >= W - 16 * (NSUB - 1)) ? NSUB - 1 : NSUB;
    float n = (float)(lane_cols * nsteps), mean[8], m2[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float a1 = s1[c], a2 = s2[c];
      mean[c] = shf[c] + a1 / n;
      m2[c] = fmaxf(a2 - a1 * a1 / n, 0.f);
    }
    auto level = [&](auto partner) {
      if constexpr (PART) {
        const float nb = partner(n), nt = n + nb, f = nb / nt;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float mb = partner(mean[c]), m2b = partner(m2[c]);
          const float d = mb - mean[c];
          mean[c] += d * f;
          m2[c] += m2b + d * d * n * f;
        }
        n = nt;
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float mb = partner(mean[c]), m2b = partner(m2[c]);
          const float d = mb - mean[c];
          mean[c] += 0.5f * d;
          m2[c] += m2b + d * d * (0.5f * n);
        }
        n *= 2.f;
      }
    };
    level([](float v) { return dpp_f<0x128>(v); });
    level([](float v) { return dpp_f<0x124>(v); });
    level([](float v) { return dpp_f<0x4E>(v); });
    level([](float v) { return dpp_f<0xB1>(v); });
    if (rp == 1 && l16 == 0)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int co = (2 * cg + (c >> 2)) * 16 + kq * 4 + (c & 3);
        xch[0][co] = n;
        xch[1][co] = mean[c];
        xch[2][co] = m2[c];
      }
    __syncthreads();
    if (rp == 0 && l16 == 0)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int co = (2 * cg + (c >> 2)) * 16 + kq * 4 + (c & 3);
        const float nbb = xch[0][co], nt = n + nbb;
        float mu = mean[c], q = m2[c];
        if (nbb > 0.f) {
          const float d = xch[1][co] - mu, f = nbb / nt;
          mu += d * f;
          q += xch[2][co] + d * d * n * f;
        }
        float* out = p.part + (size_t)blockIdx.x * 3 * kStemCo + co;
        out[0] = nt;
        out[kStemCo] = mu;
        out[2 * kStemCo] = q;
      }
  }
}

// ---------------------------------------------------------------------------
// Fused stem backward: BN(+ReLU) backward + 3x3/2 max-pool backward + the stem weight gradient in
// ONE pass over the stem output, without the BN statistics first.
//
// The weight gradient is linear in the conv-output gradient dz, and training-mode BN backward is
// dz = sc (g' - a2 - a3 (z - mu)) with per-channel a2 = mean(g'), a3 = mean(g' xhat) invstd, where
// g' is the pooled gradient gathered to the pixel and masked by relu'(z sc + sh).  So
//   dW[co][k] = sc[co] (G1[co][k] - a3[co] G2[co][k] - a2[co] G3[k])
//   G1 = sum_px g'[px][co] X[px][k],  G2 = sum_px (z - mu)[px][co] X[px][k],  G3 = sum_px X[px][k]
// (X: the space-to-depth input patch of k = (ty, tx, c)) -- all three, and the BN sums
// (sum g', sum g' (z - mu)), accumulate in the same pass; stem_bwd_finalize applies the
// coefficients once the (possibly all-reduced) sums are known.  This replaces the two
// maxpool_bn_bwd passes, the full-resolution dz tensor and the stem weight-gradient GEMM.
//
// Workgroup: a contiguous range of output rows (n, y).  Per row:
//  phase E: every (pixel, 8-channel chunk) gathers g' and writes g' and z - mu (bf16) into two
//    LDS images [128 px][64 ch] (128-byte rows, chunks XOR-swizzled by row bits 1..2; two sets
//    by row parity, so phase E of the next row runs beside phase M of this one);
//  phase M: wave w owns tap row ty = w & 3 and one A image: D[64][64] += A^T B over the row's
//    pixels in k-steps of 32, A = g' or z - mu (4 x 16 ch) and B = the input row y + w - 2 of an LDS
//    ring shifted by tx -- both read with ds_read_b64_tr_b16, the 32 pixels of a k-step
//    assigned to (k group, half) so that every read covers 8 consecutive rows (conflict free);
//    G3 = sum X is summed from the same B fragments with plain adds.
//  Input rows stream through a ring of 8 row slots (+ a zero slot) by LDS-DMA, two rows ahead.
namespace {
constexpr int kSbRing = 132;                 // ring row pixels: 2 pad + W (<= 112) + pad
constexpr int kSbSlot = kSbRing * 32;        // 16 bf16 channels per pixel
constexpr int kSbRows = 129;                 // G rows: 64 g', 64 z - mu, 1 (G3 = sum X)
constexpr int kSbPart = kSbRows * 256 + 128;  // + local BN sums [2][64]

struct StemBwdParams {
  const bf16* z;       // stem conv output = BN input [N][H][W][64]
  const bf16* x16;     // stem input [N][H][W][16]
  const bf16* dy;      // pooled gradient [N][Ho][Wo][64]
  const uint8_t* idx;  // window argmax [N][Ho][Wo][64]
  const float* scale;  // BN scale / shift (the ReLU mask), mean (centering)
  const float* shift;
  const float* mean;
  float* part;         // [blocks][kSbPart]
  int N, H, Ho, Wo, act, rpb;  // rpb: output rows per workgroup
  int ablate;                  // A/B timing only (g_tune[kStemAblate]): 1 no MFMA phase, 2 no gather phase
};

typedef short s16x4 __attribute__((ext_vector_type(4)));  // the 16x16x16 bf16 MFMA operand type

__device__ __forceinline__ uint32_t sb_aoff(uint32_t r, uint32_t col) {
  return r * 128u + (((col >> 3) ^ (((r >> 1) & 3u) << 1)) << 4) + (col & 7) * 2;
}
// 16-byte LDS-DMA per lane (lane-linear destination from the wave-uniform base), issued as
// inline asm: the compiler then does not track it, so LDS reads are not made to wait for it
// (it cannot tell ring slots apart and would drain vmcnt, operand prefetches included).  The
// caller guarantees the data has landed before it is read (see the interval schedule).  M0 is
// saved and restored around the DMA (the instruction captures it at issue).
__device__ __forceinline__ void sb_dma16(const void* g, const char* lds) {
  const uint32_t a = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, lds));
  uint32_t saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(g), "s"(a)
      : "memory");
}
__device__ __forceinline__ bf16x8 sb_tr(const char* a, const char* b) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, b));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
}  // namespace

template <int W>  // output columns (a multiple of 8)
// one workgroup of 8 waves per CU (two per SIMD, so the gather phase's dependent VALU chains
// and the MFMAs of one wave hide behind the other's): wave w owns tap row ty = w & 3 and the g'
// (w < 4) or the z - mu image (w >= 4): 16 accumulator tiles
__global__ void __launch_bounds__(512, 1) stem_bwd_kernel(StemBwdParams p) {
  constexpr int NKS = (W + 31) / 32;
  constexpr bool kTail16 = W - (NKS - 1) * 32 <= 16;  // last k-step on 16-deep MFMAs
  static_assert(W + 4 <= kSbRing && NKS * 32 <= 128, "row does not fit");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // A images, double-buffered by row parity: set b at smem + b * 32 KB = {g' [128 px][64],
  // z - mu [128 px][64]}
  char* ring = smem + 65536;  // 8 row slots + the zero slot (index 8)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H;
  const int g0 = blockIdx.x * p.rpb, g1 = min(p.N * H, g0 + p.rpb);

  // zero: the k-padding rows W..127 of all four A images, every ring slot's padding pixels and
  // the whole zero slot (LDS-DMA only ever writes pixels 2 .. W+1 of slots 0..7)
  for (int i = tid; i < (128 - W) * 8 * 4; i += 512) {
    const int img = i / ((128 - W) * 8), j = i - img * ((128 - W) * 8);
    *(u32x4*)(smem + img * 16384 + (W + j / 8) * 128 + (j & 7) * 16) = u32x4{0, 0, 0, 0};
  }
  for (int i = tid; i < 9 * kSbSlot / 16; i += 512) {
    const int slot = i / (kSbSlot / 16), px = (i - slot * (kSbSlot / 16)) >> 1;
    if (slot == 8 || px < 2 || px >= W + 2) *(u32x4*)(ring + (size_t)i * 16) = u32x4{0, 0, 0, 0};
  }
  // LDS-DMA of input row yy of image n (global row G = n H + yy) into slot G & 7 (waves 0..3)
  auto load_row = [&](int n, int yy) {
    if (yy < 0 || yy >= H) return;
    const int G = n * H + yy;
    const int e = wave * 64 + lane;  // 16-byte piece of the row: W * 2 pieces
    char* dst = ring + (G & 7) * kSbSlot + 64 + wave * 1024;
    if (e < W * 2) sb_dma16(p.x16 + (size_t)G * W * 16 + e * 8, dst);
  };
  // the input rows output row gg adds to those of gg - 1: rows 0 and 1 of a new image, else y + 1
  auto load_new_rows = [&](int gg) {
    const int nn = gg / H, yy = gg - nn * H;
    if (yy == 0) {
      load_row(nn, 0);
      load_row(nn, 1);
    } else {
      load_row(nn, yy + 1);
    }
  };
  auto slot_of = [&](int n, int yy) -> const char* {
    return ring + ((yy < 0 || yy >= H) ? 8 : ((n * H + yy) & 7)) * kSbSlot;
  };

  // BN constants (scale, shift, mean) staged in LDS and re-read per item (24 registers fewer
  // across the MFMA phase); a thread's items all have channel chunk c8 = tid & 7
  float* bnc = (float*)(ring + 9 * kSbSlot);
  if (tid < 192) bnc[tid] = (tid < 64 ? p.scale : tid < 128 ? p.shift : p.mean)[tid & 63];
  const int c8 = tid & 7;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;

  const uint32_t l16 = lane & 15, kq = lane >> 4, q = l16 >> 2, pp = lane & 3;
  const int ty = wave & 3, half = wave >> 2;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // G3 = sum X: an MFMA of a ones A-fragment (k-padding pixels 0) with the B fragments -- every
  // row of the 16 x 16 result is the column sum (the VALU adds it replaced were a quarter of the
  // kernel's VALU work, which sets its time)
  f32x4 g3[4];
#pragma unroll
  for (int tx = 0; tx < 4; ++tx) g3[tx] = f32x4{0.f, 0.f, 0.f, 0.f};

  // phase-E operands of a row, loaded a barrier interval ahead (their HBM latency overlaps the
  // previous interval's MFMAs).  An item is a pixel pair (2j, 2j + 1) x an 8-channel chunk: pixel
  // 2j lies in pooled column j only, pixel 2j + 1 in columns j and j + 1 (3x3 / 2 / pad 1), and
  // an even output row in pooled row y / 2 only -- so an item loads 2 (even row) or 4 (odd row)
  // windows' argmax bytes and pooled gradients instead of 4 per pixel
  constexpr int NIT = (W * 4 + 511) / 512;
  bf16x8 zv[NIT][2], gv[NIT][2][2];
  uint64_t pk[NIT][2][2];
  auto load_items = [&](int gg) {
    const int nn = gg / H, yy = gg - nn * H;
    const bf16* zrow = p.z + (size_t)gg * W * 64;
    const int h0 = yy >> 1, h1 = min((yy + 1) >> 1, p.Ho - 1);  // even rows: h1 = h0 (masked)
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      // unpredicated (lanes past the row reload its last item): a masked load would merge into the
      // live registers through a copy, which waits for the load
      const int i = min(tid + 512 * k, W * 4 - 1);
      {
        const int pr = i >> 3;
        zv[k][0] = *(const bf16x8*)(zrow + (2 * pr) * 64 + c8 * 8);
        zv[k][1] = *(const bf16x8*)(zrow + (2 * pr + 1) * 64 + c8 * 8);
        const int wc1 = min(pr + 1, p.Wo - 1);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const uint32_t o = ((uint32_t)(nn * p.Ho + (r ? h1 : h0)) * p.Wo + (c ? wc1 : pr)) * 64 + c8 * 8;
            pk[k][r][c] = *(const uint64_t*)(p.idx + o);
            gv[k][r][c] = *(const bf16x8*)(p.dy + o);
          }
      }
    }
  };
  // ---- phase E of row gg: g' and z - mu into the A images of set gg & 1 (same masking, order
  // of the window sum and rounding as gather_pool_grad + maxpool_bn_bwd) ----
  // ROW1: the row lies in two pooled rows (odd y, not the last): a uniform branch per row, so an
  // even row's items test 1 (even pixel) + 2 (odd pixel) windows instead of 2 + 4
  auto phase_e_rows = [&](int gg, auto row1_tag) {
    constexpr bool row1 = decltype(row1_tag)::value;
    const int y = gg - (gg / H) * H;
    const int h0 = y >> 1, h1 = (y + 1) >> 1;
    char* ag = smem + (gg & 1) * 32768;
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int i = tid + 512 * k;
      if (i < W * 4) {
        const int pr = i >> 3;
        float sc[8], sh[8], mu[8];
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          *(float4*)&sc[e] = *(const float4*)&bnc[c8 * 8 + e];
          *(float4*)&sh[e] = *(const float4*)&bnc[64 + c8 * 8 + e];
          *(float4*)&mu[e] = *(const float4*)&bnc[128 + c8 * 8 + e];
        }
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const int px = 2 * pr + sp;
          bool ok[2][2];
          uint32_t want[2][2];
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const int ho = r ? h1 : h0, wo = pr + c;
              ok[r][c] = ((r == 0) | row1) & ((c == 0) | ((sp == 1) & (pr + 1 < p.Wo)));
              want[r][c] = (uint32_t)((y - (ho * 2 - 1)) * 3 + (px - (wo * 2 - 1)));
            }
          bf16x8 go, zo;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float gsum = 0.f;  // branch-free: selects, no divergent blocks around the loads' uses
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                const uint32_t b = (uint32_t)(pk[k][r][c] >> (8 * e)) & 0xffu;
                const bool hit = ok[r][c] & (b == want[r][c]);  // non-short-circuit: a select
                gsum += hit ? bf2f(gv[k][r][c][e]) : 0.f;
              }
            const float zf = bf2f(zv[k][sp][e]);
            float gq = bf2f(f2bf(gsum));  // the bf16 pool gradient of the unfused chain
            if (p.act == 1 && !(zf * sc[e] + sh[e] > 0.f)) gq = 0.f;
            const float zc = zf - mu[e];
            s1[e] += gq;
            s2[e] += gq * zc;
            go[e] = f2bf(gq);
            zo[e] = f2bf(zc);
          }
          const uint32_t o = px * 128u + ((c8 ^ (((px >> 1) & 3u) << 1)) << 4);
          *(bf16x8*)(ag + o) = go;
          *(bf16x8*)(ag + 16384 + o) = zo;
        }
      }
    }
  };
  auto phase_e = [&](int gg) {
    const int y = gg - (gg / H) * H;
    const int h0 = y >> 1, h1 = (y + 1) >> 1;
    if ((h1 != h0) & (h1 < p.Ho))
      phase_e_rows(gg, std::true_type{});
    else
      phase_e_rows(gg, std::false_type{});
  };
  // ---- phase M of row gg: this wave's A image of set gg & 1 against input row y + ty - 2 ----
  auto phase_m = [&](int gg) {
    const int n = gg / H, y = gg - n * H;
    const char* brow = slot_of(n, y + ty - 2);
    const char* aimg = smem + (gg & 1) * 32768 + half * 16384;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (kTail16 && ks == NKS - 1) {
        // last k-step with <= 16 valid pixel rows (W = 112: rows 96..111): 16-deep MFMAs over those
        // rows only, one transposed read per operand (lane group kq holds rows kq&1, kq>>1 of the
        // 4-row quads 0..3, the same rows for A and B; the output layout is the 16x16x32 one)
        const uint32_t rt = ks * 32 + (kq & 1) * 4 + (kq >> 1) * 8;
        bf16x4 bt[4];
#pragma unroll
        for (int tx = 0; tx < 4; ++tx)
          bt[tx] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, brow + (rt + q + tx) * 32 + pp * 8));
        if (half == 0) {
          bf16x4 one;
#pragma unroll
          for (int j = 0; j < 4; ++j) one[j] = f2bf(rt + j < (uint32_t)W ? 1.f : 0.f);
#pragma unroll
          for (int tx = 0; tx < 4; ++tx)
            g3[tx] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, one),
                                                               __builtin_bit_cast(s16x4, bt[tx]), g3[tx], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x4 af =
              __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, aimg + sb_aoff(rt + q, i * 16 + pp * 4)));
#pragma unroll
          for (int tx = 0; tx < 4; ++tx)
            acc[i][tx] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, af),
                                                                   __builtin_bit_cast(s16x4, bt[tx]), acc[i][tx], 0, 0, 0);
        }
        continue;
      }
      const uint32_t base = ks * 32 + (kq >> 1) * 16 + (kq & 1) * 4;
      const uint32_t ra = base + q, rb = base + 8 + q;  // this lane's pixel rows (k 0-3 / 4-7)
      bf16x8 bf[4];
#pragma unroll
      for (int tx = 0; tx < 4; ++tx)
        bf[tx] = sb_tr(brow + (ra + tx) * 32 + pp * 8, brow + (rb + tx) * 32 + pp * 8);
      if (half == 0) {  // wave-uniform: G3 = sum X on the matrix pipe, A = 1 on the row's W pixels
        bf16x8 one;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          one[j] = f2bf(base + j < (uint32_t)W ? 1.f : 0.f);
          one[4 + j] = f2bf(base + 8 + j < (uint32_t)W ? 1.f : 0.f);
        }
#pragma unroll
        for (int tx = 0; tx < 4; ++tx) g3[tx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(one, bf[tx], g3[tx], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t col = i * 16 + pp * 4;
        const bf16x8 af = sb_tr(aimg + sb_aoff(ra, col), aimg + sb_aoff(rb, col));
#pragma unroll
        for (int tx = 0; tx < 4; ++tx)
          acc[i][tx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[tx], acc[i][tx], 0, 0, 0);
      }
    }
  };

  // Barrier interval t runs phase E of row t + 1 and phase M of row t (A sets by parity), so the
  // two waves of a SIMD overlap VALU and MFMA: waves 0..3 (which also issue the ring loads) run E
  // first, waves 4..7 run M first.  Interval t issues the new input rows of row t + 3, then the
  // gather operands of row t + 2.  Waves 0..3 wait for those operands in phase E of interval t + 1
  // (vmcnt retires in issue order), so the rows have landed before the barrier ahead of M(t + 3);
  // in use or in flight are at most input rows G - 2 .. G + 4 (7 of the 8 slots).
  // Raw barriers: __syncthreads() would also drain vmcnt.
  if (g0 < g1) {
    const int n = g0 / H, y = g0 - n * H;
#pragma unroll
    for (int d = -2; d <= 1; ++d) load_row(n, y + d);
    if (g0 + 1 < g1) load_new_rows(g0 + 1);
    if (g0 + 2 < g1) load_new_rows(g0 + 2);
    load_items(g0);
  }
  // zero fill + BN constants published; the untracked ring DMA of the first three rows landed
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int t = g0 - 1; t < g1; ++t) {
    const bool doE = t + 1 < g1, doM = t >= g0, doL = t + 2 < g1;
    // The operand loads have ONE unconditional site for every wave (a clamped row at the end):
    // loads in wave-dependent or conditional blocks merge into the loop-carried registers through
    // copies, and a copy of a loading register waits for the load (no prefetch left).  The ring
    // DMA of the rows of output row t + 3 (untracked, sb_dma16) follows them; waves 0..3 drain it
    // after phase E of the next interval, two barriers before M(t + 3) reads the rows.
    if (half != 0 && doM && p.ablate != 1) phase_m(t);
    if (doE && p.ablate != 2) phase_e(t + 1);
    // waves 0..3: the previous interval's ring DMA (behind the operands E just consumed) landed
    if (half == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    load_items(min(t + 2, g1 - 1));
    if (half == 0 && t + 3 < g1) load_new_rows(t + 3);
    if (half == 0 && doM && p.ablate != 1) phase_m(t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // ---- partials: G rows (g' 0..63, z - mu 64..127, G3 128) x 256 columns, then BN sums ----
  float* part = p.part + (size_t)blockIdx.x * kSbPart;
  const int col = ty * 64 + (int)l16;  // + tx * 16: column (ty, tx, c = l16)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int tx = 0; tx < 4; ++tx)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        part[(half * 64 + i * 16 + (int)kq * 4 + r) * 256 + col + tx * 16] = acc[i][tx][r];
  if (half == 0 && kq == 0)  // row 0 of the result (lanes 0..15, register 0)
#pragma unroll
    for (int tx = 0; tx < 4; ++tx) part[128 * 256 + col + tx * 16] = g3[tx][0];
  float* red = (float*)smem;  // [2][512][8] (the A images are free)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[tid * 8 + e] = s1[e];
    red[4096 + tid * 8 + e] = s2[e];
  }
  __syncthreads();
  if (tid < 128) {
    const int which = tid >> 6, ch = tid & 63;
    float t = 0.f;
    for (int u = ch >> 3; u < 512; u += 8) t += red[which * 4096 + u * 8 + (ch & 7)];
    part[kSbRows * 256 + which * 64 + ch] = t;
  }
}

// sums [2][64] = (sum g', sum g' xhat) from the reduced partial
__global__ void stem_bwd_sums_kernel(const float* __restrict__ tot, const float* __restrict__ invstd,
                                     float* __restrict__ sums) {
  const int t = threadIdx.x;
  if (t < 128) sums[t] = tot[kSbRows * 256 + t] * (t >= 64 ? invstd[t - 64] : 1.f);
}

// dW[co][k] = sc (G1 - a3 G2 - a2 G3), a2 = sum g' / n, a3 = (sum g' xhat) / n * invstd
__global__ void stem_bwd_dw_kernel(const float* __restrict__ tot, const float* __restrict__ sums,
                                   const float* __restrict__ scale, const float* __restrict__ invstd, float inv_count,
                                   float* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 256) return;
  const int co = i >> 8, k = i & 255;
  const float a2 = sums[co] * inv_count, a3 = sums[64 + co] * inv_count * invstd[co];
  dw[i] = scale[co] * (tot[co * 256 + k] - a3 * tot[(64 + co) * 256 + k] - a2 * tot[128 * 256 + k]);
}

bool stem_bwd_supported(int H, int W, int C, int Ho, int Wo) {
  return C == kStemCo && H % 2 == 0 && (W % 16 == 0 || W == 56) && W >= 16 && W + 4 <= kSbRing && Ho == H / 2 &&
         Wo == W / 2;
}
int stem_bwd_blocks(int N, int H, int num_cu) { return std::min(N * H, num_cu); }
int stem_bwd_part_floats() { return kSbPart; }

void launch_stem_bwd(const bf16* z, const bf16* x16, const bf16* dy, const uint8_t* idx, const float* scale,
                     const float* shift, const float* mean, int act, int N, int H, int W, int nblocks, float* part,
                     hipStream_t s) {
  StemBwdParams p{z, x16, dy, idx, scale, shift, mean, part, N, H, H / 2, W / 2, act, 0};
  p.rpb = (N * H + nblocks - 1) / nblocks;
  p.ablate = g_tune[kStemAblate];
  constexpr int lds = 65536 + 9 * kSbSlot + 768;
  switch (W) {
#define DCP_STEMB(W_)                                                                                  \
  case W_:                                                                                             \
    (void)hipFuncSetAttribute((const void*)stem_bwd_kernel<W_>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
    hipLaunchKernelGGL(stem_bwd_kernel<W_>, dim3(nblocks), dim3(512), lds, s, p);                      \
    break;
    DCP_STEMB(16) DCP_STEMB(32) DCP_STEMB(48) DCP_STEMB(56) DCP_STEMB(64) DCP_STEMB(80) DCP_STEMB(96) DCP_STEMB(112)
#undef DCP_STEMB
    default: break;
  }
}

void launch_stem_bwd_sums(const float* tot, const float* invstd, float* sums, hipStream_t s) {
  hipLaunchKernelGGL(stem_bwd_sums_kernel, dim3(1), dim3(128), 0, s, tot, invstd, sums);
}

void launch_stem_bwd_dw(const float* tot, const float* sums, const float* scale, const float* invstd, float inv_count,
                        float* dw, hipStream_t s) {
  hipLaunchKernelGGL(stem_bwd_dw_kernel, dim3(64), dim3(256), 0, s, tot, sums, scale, invstd, inv_count, dw);
}

int stem_fwd_blocks(int N, int H) { return N * ((H + kStemRows - 1) / kStemRows); }

bool stem_fwd_supported(int H, int W, int C, int Co, int KH, int KW) {
  return C == 16 && Co == kStemCo && KH == 4 && KW == 4 && H % 2 == 0 && H > 0 && (W % 16 == 0 || W == 56) &&
         W >= 16 && W + 4 <= kPlanePx;
}

void launch_stem_fwd(const bf16* x, const bf16* w, bf16* y, float* part, const bf16* zero, int N, int H, int W,
                     hipStream_t s) {
  StemParams p{x, w, y, part, zero, H, (H + kStemRows - 1) / kStemRows};
  const dim3 grid(stem_fwd_blocks(N, H)), block(256);
  if (W == 56) {  // the 112 px input (ArcFace): 3.5 tiles per row
    hipLaunchKernelGGL((stem_fwd_kernel<4, 56>), grid, block, kSlots * kSlotBytes + 4 * 16 * 256, s, p);
    return;
  }
  switch (W / 16) {
#define DCP_STEM(NS_) \
  case NS_: hipLaunchKernelGGL(stem_fwd_kernel<NS_>, grid, block, kSlots * kSlotBytes + NS_ * 16 * 256, s, p); break;
    DCP_STEM(1) DCP_STEM(2) DCP_STEM(3) DCP_STEM(4) DCP_STEM(5) DCP_STEM(6) DCP_STEM(7)
#undef DCP_STEM
    default: break;
  }
}

}  // namespace dcp
