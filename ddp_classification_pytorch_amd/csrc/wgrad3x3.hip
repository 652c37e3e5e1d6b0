// Direct weight gradient of the 3x3 / stride-1 / pad-1 convolutions (ResNet bottleneck conv2,
// BasicBlock convs).
//
// The implicit-GEMM weight gradient (conv_igemm.hip) gathers an im2col image per k-tile: every
// input pixel is fetched nine times, once per tap, and the 64-channel layers ran latency-bound
// on those gathers (~0.3 PFLOP/s).  Here a workgroup owns one (64 output channels x 64 input
// channels) block of dW for all nine taps and walks a contiguous range of row strips (R rows of
// one image):
//  * the strip's input rows with a one-pixel halo -- (R+2) x (W+2) pixels x 64 channels, zero
//    outside the image, rows padded to an even pitch -- and its R x W output-gradient pixels
//    are staged once in LDS by LDS-DMA; pixel rows are 128 bytes with the 16-byte chunks
//    XOR-swizzled by bits 1 and 3 of the pixel's column (window) or index (gradient), so the
//    ds_read_b64_tr_b16 fragment reads are bank-conflict free and the nine taps' addresses are
//    three per-lane offsets plus uniform row steps;
//  * the GEMM runs over the strip's pixels (k = 32 pixels per step): the dY^T fragments
//    (A, 4 x 16 channels) are read once per step and each tap's input fragment (B) is the same
//    pixel set shifted by (ky, kx) inside the staged window -- no re-fetch from L2;
//  * 8 waves, one workgroup per CU with two strip buffers: strip s+1 is fetched while strip s
//    is computed.  Wave w accumulates dW[64 co][9 taps][16 ci (w & 3)] over the even or odd
//    k-steps (w >> 2) of all its strips in registers (36 MFMA tiles), then stores one fp32
//    partial slice -- two per workgroup -- reduced deterministically by launch_split_reduce.
#include <algorithm>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {
constexpr int kW3MaxBuf = 80 * 1024;  // one of the two strip buffers (160 KB: one workgroup per CU)

struct W3Params {
  const bf16* dy;    // [N][H][W][Co]
  const bf16* x;     // [N][H][W][C]
  float* part;       // [2 splits][Co][9][C] (or dW itself when there is one slice)
  const bf16* zero;  // >= 16 zero bytes
  int H, W, C, Co;
  int R, spi;        // rows per strip, strips per image
  int strips, sps;   // strips in total, strips per split
  int xq, xbytes;    // 16-byte chunks of the input window image; its LDS bytes
  int buf;           // bytes per strip buffer (window + output-gradient pixels)
  int nib;           // 64-channel input blocks
  int Wq;            // window row pitch in pixels: W + 2 rounded up to even (the swizzle's parity)
  int ablate;        // tuning experiments only (g_tune[kAblate]): 1 = no strip prefetch, 2 = no MFMA loop
  FastDiv div_wq, div_w, div_spi;
  // BN prologue (the forward's conv3x3_c64 PRO): x is a BN's input, the GEMM operand
  // relu(x * pscale[c] + pshift[c]), recomputed once per staged window element; nullptr: off
  const float* pscale;
  const float* pshift;
};

// pixel-row swizzle of the 128-byte-row images (as swz128tr in conv_igemm.hip)
__device__ __forceinline__ uint32_t w3_g(uint32_t P) { return (((P >> 1) & 1u) | (((P >> 3) & 1u) << 1)) << 1; }
__device__ __forceinline__ uint32_t w3_off(uint32_t P, uint32_t col) {
  return P * 128u + (((col >> 3) ^ w3_g(P)) << 4) + (col & 7) * 2;
}
// 16x16x32 operand fragment over pixel rows Pa (k 0..3 of the lane's block) and Pb (k 4..7),
// channel columns col .. col+3 of the lane (transposed by ds_read_b64_tr_b16)
__device__ __forceinline__ bf16x8 w3_frag(const char* img, uint32_t Pa, uint32_t Pb, uint32_t col) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + w3_off(Pa, col)));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + w3_off(Pb, col)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
}  // namespace

__global__ void __launch_bounds__(512, 1) wgrad3x3_kernel(const W3Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // two strip buffers

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave & 3, half = wave >> 2;  // 16-channel input subtile, k-step parity
  const int pairs = (p.Co >> 6) * p.nib;
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / pairs, pr = lid - split * pairs;
  const int co0 = (pr / p.nib) * 64, ci0 = (pr % p.nib) * 64;
  const int s_begin = split * p.sps, s_end = min(p.strips, s_begin + p.sps);
  const int H = p.H, W = p.W, Wq = p.Wq;

  // strip s -> buffer b: its input window -- chunk qq = LDS pixel qq/8 = (rr, xx) -- and its
  // output-gradient pixels (rows past the strip read zeros: those k rows contribute nothing)
  auto load_strip = [&](int s, int b) {
    char* ximg = smem + b * p.buf;
    char* dimg = ximg + p.xbytes;
    const int n = fdiv(s, p.div_spi);
    const int y0 = (s - n * p.spi) * p.R;
    const int rows = min(p.R, H - y0), npix = rows * W;
    for (int qq = tid; qq < p.xq; qq += 512) {
      const uint32_t P = qq >> 3;
      const uint32_t rr = fdiv(P, p.div_wq), xx = P - rr * Wq;
      const int yy = y0 - 1 + (int)rr, xi = (int)xx - 1;
      const bool ok = (int)rr < rows + 2 && yy >= 0 && yy < H && xi >= 0 && xi < W;
      const uint32_t c = (qq & 7) ^ w3_g(xx);
      const bf16* g = ok ? p.x + ((size_t)(n * H + yy) * W + xi) * p.C + ci0 + c * 8 : p.zero;
      dma16(g, ximg + (qq - lane) * 16);
    }
    const int dq = ((npix + 31) >> 5) * 256;
    for (int qq = tid; qq < dq; qq += 512) {
      const uint32_t P = qq >> 3;
      const uint32_t r = fdiv(P, p.div_w), xpx = P - r * W;
      const uint32_t c = (qq & 7) ^ w3_g(P);
      const bf16* g = (int)P < npix ? p.dy + ((size_t)(n * H + y0 + r) * W + xpx) * p.Co + co0 + c * 8 : p.zero;
      dma16(g, dimg + (qq - lane) * 16);
    }
  };

  const uint32_t q = (lane & 15) >> 2, pp = lane & 3, kq = lane >> 4;
  f32x4 acc[4][9];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (s_begin < s_end) load_strip(s_begin, 0);
  for (int s = s_begin; s < s_end; ++s) {
    const int b = (s - s_begin) & 1;
    // strip s landed in buffer b (own DMA drained, then the barrier); every wave is done with
    // buffer b^1 (strip s-1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (p.pscale != nullptr) {
      // BN + ReLU once per staged in-image window element, before the next strip's DMA is issued
      // (the per-channel coefficients are ordinary loads: a compiler-counted wait behind an
      // untracked DMA would drain it); the zero halo stays zero
      char* xw = smem + b * p.buf;
      const int n = fdiv(s, p.div_spi);
      const int y0 = (s - n * p.spi) * p.R;
      const int rows = min(p.R, H - y0);
      for (int qq = tid; qq < p.xq; qq += 512) {
        const uint32_t P = qq >> 3;
        const uint32_t rr = fdiv(P, p.div_wq), xx = P - rr * Wq;
        const int yy = y0 - 1 + (int)rr, xi = (int)xx - 1;
        if ((int)rr < rows + 2 && yy >= 0 && yy < H && xi >= 0 && xi < W) {
          const int c0 = ci0 + (int)(((qq & 7) ^ w3_g(xx)) * 8);
          float sc[8], sh[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            sc[e] = p.pscale[c0 + e];
            sh[e] = p.pshift[c0 + e];
          }
          bf16x8 v = *LDS_PTR(bf16x8, xw + qq * 16);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf(bf2f(v[e]) * sc[e] + sh[e], 0.f));  // as bn_act_fwd_kernel
          *LDS_PTR(bf16x8, xw + qq * 16) = v;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (s + 1 < s_end && !(p.ablate & 1)) load_strip(s + 1, b ^ 1);
    const char* ximg = smem + b * p.buf;
    const char* dimg = ximg + p.xbytes;
    const int n = fdiv(s, p.div_spi);
    const int y0 = (s - n * p.spi) * p.R;
    const int npix = min(p.R, H - y0) * W;
    const int nks = (npix + 31) >> 5;
    for (int ks = half; ks < ((p.ablate & 2) ? 0 : nks); ks += 2) {
      const uint32_t pa = ks * 32 + 8 * kq + q, pb = pa + 4;  // the lane's two pixel rows
      bf16x8 af[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) af[c] = w3_frag(dimg, pa, pb, c * 16 + pp * 4);
      // window byte offsets of the lane's pixels for taps (0, kx): the swizzle depends on the
      // window column only, so the three tap rows ky add a uniform ky * Wq * 128.  Pixels past
      // the strip read window pixels of row 0 -- finite values against their zero A rows.
      const uint32_t ra = (int)pa < npix ? fdiv(pa, p.div_w) : 0u, rb = (int)pb < npix ? fdiv(pb, p.div_w) : 0u;
      const uint32_t xa = (int)pa < npix ? pa - ra * W : 0u, xb = (int)pb < npix ? pb - rb * W : 0u;
      const uint32_t cc = (wq * 16 + pp * 4) >> 3, e = (pp & 1) * 8;
      uint32_t oa[3], ob[3];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        oa[kx] = (ra * Wq + xa + kx) * 128u + ((cc ^ w3_g(xa + kx)) << 4) + e;
        ob[kx] = (rb * Wq + xb + kx) * 128u + ((cc ^ w3_g(xb + kx)) << 4) + e;
      }
      const uint32_t rowb = (uint32_t)Wq * 128u;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint32_t dky = (t / 3) * rowb;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, ximg + oa[t % 3] + dky));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, ximg + ob[t % 3] + dky));
        const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[c], bf, acc[c][t], 0, 0, 0);
      }
    }
  }

  // D[co][ci]: lane holds co = 16 c + 4 kq + r, ci = 16 wq + (lane & 15); one slice per half
  const int ci = ci0 + wq * 16 + (lane & 15);
  const size_t slice = (size_t)split * 2 + half;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + c * 16 + kq * 4 + r;
        p.part[((slice * p.Co + co) * 9 + t) * p.C + ci] = acc[c][t][r];
      }
}

// ---------------------------------------------------------------------------
static int w3_pitch(int W) { return (W + 3) & ~1; }

static int w3_buf(int R, int W) {
  const int xb = ((R + 2) * w3_pitch(W) * 128 + 1023) / 1024 * 1024;
  return xb + ((R * W + 31) / 32) * 32 * 128;
}

// rows per strip: about 256 pixels, the strips of an image equal, a buffer within kW3MaxBuf
static int w3_rows(int H, int W) {
  int R = std::min(H, std::max(1, 256 / W));
  while (R > 1 && w3_buf(R, W) > kW3MaxBuf) --R;
  if (w3_buf(R, W) > kW3MaxBuf) return 0;
  const int nstrip = (H + R - 1) / R;
  return (H + nstrip - 1) / nstrip;
}

// partial slices (2 per workgroup) of the direct kernel, 0 where it does not apply: 64-channel
// blocks, at most 2 x 2 of them (wider layers keep the 256-tile implicit GEMM, which measured
// faster there)
int wgrad3x3_splits(int N, int H, int W, int C, int Co, int num_cu) {
  if (g_tune[kWg3x3] == 1 || C % 64 != 0 || Co % 64 != 0 || H < 1 || W < 1) return 0;
  const int pairs = (Co / 64) * (C / 64);
  if (pairs > 4 && g_tune[kWg3x3] != 2) return 0;
  const int R = w3_rows(H, W);
  if (R == 0) return 0;
  const int strips = N * ((H + R - 1) / R);
  int splits = std::max(1, std::min(strips, num_cu / pairs));
  if (g_tune[kWgSplitCap] > 1) splits = std::max(1, std::min(splits, g_tune[kWgSplitCap] / 2));  // cap on the slices (2 per split)
  const int sps = (strips + splits - 1) / splits;
  return 2 * ((strips + sps - 1) / sps);
}

void launch_wgrad3x3(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Co, float* part, int slices,
                     const bf16* zero, hipStream_t stream, const float* pscale, const float* pshift) {
  W3Params p;
  p.dy = dy; p.x = x; p.part = part; p.zero = zero;
  p.pscale = pscale; p.pshift = pshift;
  p.H = H; p.W = W; p.C = C; p.Co = Co;
  p.R = w3_rows(H, W);
  p.spi = (H + p.R - 1) / p.R;
  p.strips = N * p.spi;
  const int splits = slices / 2;
  p.sps = (p.strips + splits - 1) / splits;
  p.Wq = w3_pitch(W);
  p.xq = (p.R + 2) * p.Wq * 8;
  p.xbytes = (p.xq * 16 + 1023) / 1024 * 1024;
  p.buf = w3_buf(p.R, W);
  p.nib = C / 64;
  p.div_wq = make_fastdiv(p.Wq);
  p.ablate = g_tune[kAblate];
  p.div_w = make_fastdiv(W);
  p.div_spi = make_fastdiv(p.spi);
  const int lds = 2 * p.buf;
  static int attr = 0;
  if (lds > attr) {
    hipFuncSetAttribute((const void*)wgrad3x3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kW3MaxBuf);
    attr = 2 * kW3MaxBuf;
  }
  const int grid = splits * (Co / 64) * (C / 64);
  hipLaunchKernelGGL(wgrad3x3_kernel, dim3(grid), dim3(512), lds, stream, p);
}

}  // namespace dcp
