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
#include "common.cuh"
#include "launchers.h"

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
