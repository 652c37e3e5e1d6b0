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

template <int NSUB>  // W = 16 * NSUB output columns
__global__ void __launch_bounds__(256, 2) stem_fwd_kernel(StemParams p) {
  constexpr int W = NSUB * 16;
  static_assert(W + 4 <= kPlanePx, "row does not fit a plane");
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
    if (lpx < W) __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(void, dst), 16, 0, 0);
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
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSUB) : "memory");
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
        *(bf16x4*)(stage + px * 128 + slot * 8) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // not __syncthreads: keep the loads in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16* ydst = p.y + (size_t)(n * H + y0) * W * kStemCo;
#pragma unroll
    for (int k = 0; k < NSUB; ++k) {
      const uint32_t q = k * 256 + tid, px = q >> 3, c = q & 7, sw = px & 15;
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
          const float d = acc[c >> 2][i][c & 3] - shf[c];
          s1[c] += d;
          s2[c] = fmaf(d, d, s2[c]);
        }
    }
  }

  if (p.part) {
    // lane (n, mean, M2) per channel, merged over the 16 lanes of the pixel group (equal counts),
    // then across the two row waves of each channel half through LDS
    float n = (float)(NSUB * nsteps), mean[8], m2[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float a1 = s1[c], a2 = s2[c];
      mean[c] = shf[c] + a1 / n;
      m2[c] = fmaxf(a2 - a1 * a1 / n, 0.f);
    }
    auto level = [&](auto partner) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float mb = partner(mean[c]), m2b = partner(m2[c]);
        const float d = mb - mean[c];
        mean[c] += 0.5f * d;
        m2[c] += m2b + d * d * (0.5f * n);
      }
      n *= 2.f;
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
//    LDS images [128 px][64 ch] (128-byte rows, chunks XOR-swizzled by row bits 1..2);
//  phase M: wave w owns tap row ty = w: D[128][64] += A^T B over the row's pixels in k-steps of
//    32, A = {g' (4 x 16 ch), z - mu (4 x 16 ch)} and B = the input row y + w - 2 of an LDS
//    ring shifted by tx -- both read with ds_read_b64_tr_b16, the 32 pixels of a k-step
//    assigned to (k group, half) so that every read covers 8 consecutive rows (conflict free);
//    G3 = sum X is summed from the same B fragments with plain adds.
//  Input rows stream through a ring of 8 row slots (+ a zero slot) by LDS-DMA, one row ahead.
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
};

__device__ __forceinline__ uint32_t sb_aoff(uint32_t r, uint32_t col) {
  return r * 128u + (((col >> 3) ^ (((r >> 1) & 3u) << 1)) << 4) + (col & 7) * 2;
}
__device__ __forceinline__ bf16x8 sb_tr(const char* a, const char* b) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, b));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
}  // namespace

template <int NSUB>  // W = 16 NSUB output columns
// one workgroup per CU: the 36 accumulator tiles (144 registers) stay live across the gather
// phase, so the kernel takes the full 512-register file (accumulators in AGPRs, no spills)
__global__ void __launch_bounds__(256, 1) stem_bwd_kernel(StemBwdParams p) {
  constexpr int W = NSUB * 16, NKS = (W + 31) / 32;
  static_assert(W + 4 <= kSbRing && NKS * 32 <= 128, "row does not fit");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ag = smem;                 // [128 px][64] g'
  char* Az = smem + 16384;         // [128 px][64] z - mu
  char* ring = smem + 32768;       // 8 row slots + the zero slot (index 8)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H;
  const int g0 = blockIdx.x * p.rpb, g1 = min(p.N * H, g0 + p.rpb);

  // zero: the k-padding rows W..127 of both A images, every ring slot's padding pixels and the
  // whole zero slot (LDS-DMA only ever writes pixels 2 .. W+1 of slots 0..7)
  for (int i = tid; i < (128 - W) * 8 * 2; i += 256) {
    const int img = i / ((128 - W) * 8), j = i - img * ((128 - W) * 8);
    *(u32x4*)(smem + img * 16384 + (W + j / 8) * 128 + (j & 7) * 16) = u32x4{0, 0, 0, 0};
  }
  for (int i = tid; i < 9 * kSbSlot / 16; i += 256) {
    const int slot = i / (kSbSlot / 16), px = (i - slot * (kSbSlot / 16)) >> 1;
    if (slot == 8 || px < 2 || px >= W + 2) *(u32x4*)(ring + (size_t)i * 16) = u32x4{0, 0, 0, 0};
  }
  // LDS-DMA of input row yy of image n (global row G = n H + yy) into slot G & 7
  auto load_row = [&](int n, int yy) {
    if (yy < 0 || yy >= H) return;
    const int G = n * H + yy;
    const int e = wave * 64 + lane;  // 16-byte piece of the row: W * 2 pieces
    char* dst = ring + (G & 7) * kSbSlot + 64 + wave * 1024;
    if (e < W * 2)
      __builtin_amdgcn_global_load_lds((const void*)(p.x16 + (size_t)G * W * 16 + e * 8), LDS_PTR(void, dst), 16, 0, 0);
  };
  auto slot_of = [&](int n, int yy) -> const char* {
    return ring + ((yy < 0 || yy >= H) ? 8 : ((n * H + yy) & 7)) * kSbSlot;
  };

  // per-thread BN constants of its channel chunk (chunk = tid & 7 for every item of the thread)
  const int c8 = tid & 7;
  float sc[8], sh[8], mu[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = p.scale[c8 * 8 + e];
    sh[e] = p.shift[c8 * 8 + e];
    mu[e] = p.mean[c8 * 8 + e];
    s1[e] = s2[e] = 0.f;
  }

  const uint32_t l16 = lane & 15, kq = lane >> 4, q = l16 >> 2, pp = lane & 3;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float g3[4] = {0.f, 0.f, 0.f, 0.f};  // G3 = sum X: plain adds of the B fragments (VALU, beside MFMAs)

  if (g0 < g1) {
    const int n = g0 / H, y = g0 - n * H;
#pragma unroll
    for (int d = -2; d <= 1; ++d) load_row(n, y + d);
  }
  // phase-E operands of a row, loaded one row ahead (the gathers' HBM latency then overlaps the
  // previous row's MFMAs): per item the conv output chunk and the 2 x 2 candidate windows'
  // argmax bytes and pooled gradients (3x3 / 2 / pad 1 geometry)
  constexpr int NIT = (W * 8 + 255) / 256;
  bf16x8 zv[NIT], gv[NIT][4];
  uint64_t pk[NIT][4];
  auto load_items = [&](int gg) {
    const int nn = gg / H, yy = gg - nn * H;
    const bf16* zrow = p.z + (size_t)gg * W * 64;
    const int h0 = yy >> 1, h1 = min((yy + 1) >> 1, p.Ho - 1);
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int i = tid + 256 * k;
      if (i < W * 8) {
        const int px = i >> 3;
        zv[k] = *(const bf16x8*)(zrow + px * 64 + c8 * 8);
        const int w0 = px >> 1, w1 = min((px + 1) >> 1, p.Wo - 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t o = ((uint32_t)(nn * p.Ho + ((c >> 1) ? h1 : h0)) * p.Wo + ((c & 1) ? w1 : w0)) * 64 + c8 * 8;
          pk[k][c] = *(const uint64_t*)(p.idx + o);
          gv[k][c] = *(const bf16x8*)(p.dy + o);
        }
      }
    }
  };
  if (g0 < g1) load_items(g0);
  for (int g = g0; g < g1; ++g) {
    const int n = g / H, y = g - n * H;
    // ---- phase E: g' and z - mu of this row into the A images (same masking and rounding as
    // gather_pool_grad + maxpool_bn_bwd) ----
    {
      const int h0 = y >> 1, h1 = (y + 1) >> 1;
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int i = tid + 256 * k;
        if (i < W * 8) {
          const int px = i >> 3;
          const int w0 = px >> 1, w1 = (px + 1) >> 1;
          bool ok[4];
          uint32_t want[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int ho = (c >> 1) ? h1 : h0, wo = (c & 1) ? w1 : w0;
            ok[c] = (ho < p.Ho) & (wo < p.Wo) & (((c >> 1) == 0) | (h1 != h0)) & (((c & 1) == 0) | (w1 != w0));
            want[c] = (uint32_t)((y - (ho * 2 - 1)) * 3 + (px - (wo * 2 - 1)));
          }
          bf16x8 go, zo;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float gsum = 0.f;  // branch-free: selects, no divergent blocks around the loads' uses
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const uint32_t b = (uint32_t)(pk[k][c] >> (8 * e)) & 0xffu;
              const bool hit = ok[c] & (b == want[c]);  // non-short-circuit: a select, no branch
              gsum += hit ? bf2f(gv[k][c][e]) : 0.f;
            }
            const float zf = bf2f(zv[k][e]);
            float gq = bf2f(f2bf(gsum));  // the bf16 pool gradient of the unfused chain
            if (p.act == 1 && !(zf * sc[e] + sh[e] > 0.f)) gq = 0.f;
            const float zc = zf - mu[e];
            s1[e] += gq;
            s2[e] += gq * zc;
            go[e] = f2bf(gq);
            zo[e] = f2bf(zc);
          }
          const uint32_t o = px * 128u + ((c8 ^ (((px >> 1) & 3u) << 1)) << 4);
          *(bf16x8*)(Ag + o) = go;
          *(bf16x8*)(Az + o) = zo;
        }
      }
    }
    // Next row's operands, issued after this row's were consumed (phase E's waits then never
    // cover fresh loads): the input row(s) the next output row adds -- y + 2, or rows 0 and 1
    // of the next image -- and its gather operands.  The ring rows of THIS row were issued one
    // row earlier, before the operands phase E just consumed, so (vmcnt retires in issue
    // order) they have landed.  A raw barrier: __syncthreads() would also drain vmcnt.
    if (g + 1 < g1) {
      if (y + 1 < H) {
        load_row(n, y + 2);
      } else {
        load_row(n + 1, 0);
        load_row(n + 1, 1);
      }
      load_items(g + 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // ---- phase M ----
    const char* brow = slot_of(n, y + wave - 2);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const uint32_t base = ks * 32 + (kq >> 1) * 16 + (kq & 1) * 4;
      const uint32_t ra = base + q, rb = base + 8 + q;  // this lane's pixel rows (k 0-3 / 4-7)
      bf16x8 bf[4];
#pragma unroll
      for (int tx = 0; tx < 4; ++tx)
        bf[tx] = sb_tr(brow + (ra + tx) * 32 + pp * 8, brow + (rb + tx) * 32 + pp * 8);
#pragma unroll
      for (int tx = 0; tx < 4; ++tx)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          g3[tx] += (base + j < (uint32_t)W) ? bf2f(bf[tx][j]) : 0.f;
          g3[tx] += (base + 8 + j < (uint32_t)W) ? bf2f(bf[tx][4 + j]) : 0.f;
        }
      // A tiles one at a time (register pressure: 32 accumulator tiles are live)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const char* img = i < 4 ? Ag : Az;
        const uint32_t col = (i & 3) * 16 + pp * 4;
        const bf16x8 af = sb_tr(img + sb_aoff(ra, col), img + sb_aoff(rb, col));
#pragma unroll
        for (int tx = 0; tx < 4; ++tx)
          acc[i][tx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[tx], acc[i][tx], 0, 0, 0);
      }
    }
    // A images and this row's ring slots are free (raw barrier: keep the prefetches in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // ---- partials: G rows (g' 0..63, z - mu 64..127, G3 128) x 256 columns, then BN sums ----
  float* part = p.part + (size_t)blockIdx.x * kSbPart;
  const int col = wave * 64 + (int)l16;  // + tx * 16: column (ty = wave, tx, c = l16)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int tx = 0; tx < 4; ++tx)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(i * 16 + (int)kq * 4 + r) * 256 + col + tx * 16] = acc[i][tx][r];
#pragma unroll
  for (int tx = 0; tx < 4; ++tx) {
    float t = g3[tx];
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (kq == 0) part[128 * 256 + col + tx * 16] = t;
  }
  float* red = (float*)smem;  // [2][256][8] (the A images are free)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[tid * 8 + e] = s1[e];
    red[2048 + tid * 8 + e] = s2[e];
  }
  __syncthreads();
  if (tid < 128) {
    const int which = tid >> 6, ch = tid & 63;
    float t = 0.f;
    for (int u = ch >> 3; u < 256; u += 8) t += red[which * 2048 + u * 8 + (ch & 7)];
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
  return C == kStemCo && H % 2 == 0 && W % 16 == 0 && W >= 16 && W + 4 <= kSbRing && Ho == H / 2 && Wo == W / 2;
}
int stem_bwd_blocks(int N, int H, int num_cu) { return std::min(N * H, num_cu); }
int stem_bwd_part_floats() { return kSbPart; }

void launch_stem_bwd(const bf16* z, const bf16* x16, const bf16* dy, const uint8_t* idx, const float* scale,
                     const float* shift, const float* mean, int act, int N, int H, int W, int nblocks, float* part,
                     hipStream_t s) {
  StemBwdParams p{z, x16, dy, idx, scale, shift, mean, part, N, H, H / 2, W / 2, act, 0};
  p.rpb = (N * H + nblocks - 1) / nblocks;
  constexpr int lds = 32768 + 9 * kSbSlot;
  switch (W / 16) {
#define DCP_STEMB(NS_)                                                                                  \
  case NS_:                                                                                             \
    hipFuncSetAttribute((const void*)stem_bwd_kernel<NS_>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
    hipLaunchKernelGGL(stem_bwd_kernel<NS_>, dim3(nblocks), dim3(256), lds, s, p);                      \
    break;
    DCP_STEMB(1) DCP_STEMB(2) DCP_STEMB(3) DCP_STEMB(4) DCP_STEMB(5) DCP_STEMB(6) DCP_STEMB(7)
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
  return C == 16 && Co == kStemCo && KH == 4 && KW == 4 && H % 2 == 0 && H > 0 && W % 16 == 0 && W >= 16 &&
         W + 4 <= kPlanePx;
}

void launch_stem_fwd(const bf16* x, const bf16* w, bf16* y, float* part, const bf16* zero, int N, int H, int W,
                     hipStream_t s) {
  StemParams p{x, w, y, part, zero, H, (H + kStemRows - 1) / kStemRows};
  const dim3 grid(stem_fwd_blocks(N, H)), block(256);
  switch (W / 16) {
#define DCP_STEM(NS_) \
  case NS_: hipLaunchKernelGGL(stem_fwd_kernel<NS_>, grid, block, kSlots * kSlotBytes + NS_ * 16 * 256, s, p); break;
    DCP_STEM(1) DCP_STEM(2) DCP_STEM(3) DCP_STEM(4) DCP_STEM(5) DCP_STEM(6) DCP_STEM(7)
#undef DCP_STEM
    default: break;
  }
}

}  // namespace dcp
