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
//    per 16-channel group), stores bf16 straight from the accumulators (8 bytes per lane per
//    tile) and folds the row into per-channel (n, mean, M2) statistics, merged per workgroup
//    into part[block][3][64] -- the first level of the BatchNorm statistics (bn.hip), so
//    bn_stats / bn_stats_finalize skip the slab pass.
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
// sum over the 16 lanes of a DPP row, result in every lane of the row
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0x128>(v);  // row_ror:8
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}
}  // namespace

template <int NSUB>  // W = 16 * NSUB output columns
__global__ void __launch_bounds__(256, 2) stem_fwd_kernel(StemParams p) {
  constexpr int W = NSUB * 16;
  static_assert(W + 4 <= kPlanePx, "row does not fit a plane");
  extern __shared__ __attribute__((aligned(16))) char ring[];  // kSlots * kSlotBytes
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

  float sn = 0.f, smean[8], sm2[8];  // this wave's running statistics of channels (j, r)
#pragma unroll
  for (int c = 0; c < 8; ++c) smean[c] = sm2[c] = 0.f;

  const int nsteps = (r1 - r0) >> 1;
  for (int st = 0; st < nsteps; ++st) {
    const int y0 = r0 + 2 * st;
    // rows y0-2 .. y0+2 landed (issued before the previous step's 2*NSUB stores); the slots
    // the next prefetch overwrites were last read in the previous step
    if (st == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // also publishes the zeroed padding
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NSUB) : "memory");
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

    // epilogue: lane holds co = (2 cg + j) * 16 + 4 kq + r of pixel i * 16 + l16
    bf16* yrow = p.y + (size_t)(n * H + yy) * W * kStemCo + (2 * cg) * 16 + kq * 4;
    bf16x4 o[2][NSUB];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < NSUB; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[j][i][r] = f2bf(acc[j][i][r]);
        *(bf16x4*)(yrow + (size_t)(i * 16 + l16) * kStemCo + j * 16) = o[j][i];
      }
    if (p.part) {
      // this row's (W, mean, M2) per channel (of the stored bf16 values), merged into the
      // wave's running statistics with Chan's formula
      const float nb = (float)W, f = nb / (sn + nb), cross = sn * f;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s1 = 0.f;
#pragma unroll
          for (int i = 0; i < NSUB; ++i) s1 += bf2f(o[j][i][r]);
          const float mb = row16_sum(s1) * (1.f / (float)W);
          float s2 = 0.f;
#pragma unroll
          for (int i = 0; i < NSUB; ++i) {
            const float d = bf2f(o[j][i][r]) - mb;
            s2 += d * d;
          }
          const float m2b = row16_sum(s2);
          const int c = j * 4 + r;
          const float d = mb - smean[c];
          smean[c] += d * f;
          sm2[c] += m2b + d * d * cross;
        }
      sn += nb;
    }
  }

  if (p.part) {
    // merge the two row waves of each channel half; lanes l16 == 0 hold their group's channels
    if (rp == 1 && l16 == 0)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int co = (2 * cg + (c >> 2)) * 16 + kq * 4 + (c & 3);
        xch[0][co] = sn;
        xch[1][co] = smean[c];
        xch[2][co] = sm2[c];
      }
    __syncthreads();
    if (rp == 0 && l16 == 0)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int co = (2 * cg + (c >> 2)) * 16 + kq * 4 + (c & 3);
        const float nbb = xch[0][co], nt = sn + nbb;
        float mean = smean[c], m2 = sm2[c];
        if (nbb > 0.f) {
          const float d = xch[1][co] - mean, f = nbb / nt;
          mean += d * f;
          m2 += xch[2][co] + d * d * sn * f;
        }
        float* out = p.part + (size_t)blockIdx.x * 3 * kStemCo + co;
        out[0] = nt;
        out[kStemCo] = mean;
        out[2 * kStemCo] = m2;
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
  case NS_: hipLaunchKernelGGL(stem_fwd_kernel<NS_>, grid, block, kSlots * kSlotBytes, s, p); break;
    DCP_STEM(1) DCP_STEM(2) DCP_STEM(3) DCP_STEM(4) DCP_STEM(5) DCP_STEM(6) DCP_STEM(7)
#undef DCP_STEM
    default: break;
  }
}

}  // namespace dcp
