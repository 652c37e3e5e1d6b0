// Direct 3x3 / stride-1 / pad-1 forward convolution for 64 -> 64 channels (ResNet-50 layer1
// conv2, ResNet-18/34 layer1), with the BN statistics of the output as per-workgroup
// (n, mean, M2) partials (SURVEY.md §2.5 K1 + K4).
//
// The implicit GEMM (conv_igemm.hip) stages an im2col A tile per tap: every input pixel is
// fetched into LDS nine times and, with only 64 output channels per tile, each staged byte
// feeds few MACs -- these layers ran at ~0.45 PFLOP/s.  Here:
//  * the weights (9 taps x 64 x 64 bf16) live in VGPRs for the whole kernel: wave w holds the
//    B fragments of output channels 32*(w&1) .. +31 for all taps (36 x 16 bytes per lane);
//  * a workgroup walks a contiguous range of row strips (R output rows of one image); the
//    strip's input window -- (R+2) x (W+8) pixels x 128 bytes, zero outside the image -- is
//    staged ONCE in LDS by LDS-DMA, 16-byte chunks XOR-swizzled by the window pixel's low
//    three bits so the ds_read_b128 fragment reads of 8 consecutive pixels hit 8 different
//    bank groups; the nine taps are the same fragments at shifted window pixels;
//  * per 16-pixel subtile a wave issues 18 fragment reads and 36 MFMAs (16x16x32 bf16, two
//    output-channel subtiles); waves 0/1 and 2/3 split the subtiles by parity and process two
//    at a time (four independent accumulator chains);
//  * the epilogue rounds to bf16, accumulates shifted per-channel sums of the rounded values
//    (the numbers the BN normalises) and stores each lane's 4 channels straight from the
//    accumulators (c3_tile_direct, weights as the MFMA A operand; g_tune[kC3Epilogue] = 2: the older
//    per-wave LDS staging tile); the next strip's window streams in behind this strip's
//    MFMAs (8 waves, two window buffers; g_tune[kC3Variant] = 1 / 2: 4-wave variants, not faster);
//  * the window DMA is untracked (dma16), so the fragment prefetch gets exact lgkmcnt waits.
//    Timing ablations (g_tune[kAblate]) at b1024: no stores 251 us, no window loads 232, neither 210,
//    full 284 -- the MFMA loop itself, not memory, is the bound (~45 % of MFMA peak).
#include <algorithm>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {
constexpr int kC3WinMax = 48 * 1024;        // single window buffer: bytes per workgroup
constexpr int kC3WinBuf2 = 35 * 1024;       // each of two window buffers (two workgroups per CU)
constexpr int kC3Stage = 4 * 32 * 64;       // per-wave 32 px x 32 ch bf16 staging tiles (4 waves)
constexpr int kC3WinDirect = 72 * 1024;     // each of two window buffers, direct epilogue (no staging)

struct C3Params {
  const bf16* x;     // [N][H][W][64]
  const bf16* w;     // [64][9][64]
  bf16* y;           // [N][H][W][64]
  float* part;       // [gridDim.x][3][64] (n, mean, M2) or nullptr
  const bf16* zero;  // >= 16 zero bytes
  int H, W;
  int R, spi;        // rows per strip, strips per image
  int strips, sps;   // strips in total, strips per workgroup
  int Wp, xq;        // window pitch (c3_pitch) and its 16-byte chunk count
  int wbytes, nbuf;  // bytes per window buffer (1 KB aligned), window buffers (1 or 2)
  int ablate;        // timing ablations (g_tune[kAblate], direct epilogue only): 1 no stores, 2 no window loads
  int sched;         // g_tune[kC3Variant] = 3: s_setprio 1 for the upper wave half; 4: upper half out of phase
  FastDiv div_wp, div_w, div_spi;
  // BN prologue (K5 on the 3x3 consumer): the input is a training-mode BN's INPUT, used as
  // relu(x * pscale[c] + pshift[c]) -- applied ONCE per staged window element (each feeds nine
  // taps), so the BN + ReLU output of the producing layer is never written.  nullptr: off.
  const float* pscale;
  const float* pshift;
  // 1: read tap 8 - t of w for tap t (the spatially flipped weight of the data gradient, read in
  // place: no flipped copy per call)
  int wflip;
};

__device__ __forceinline__ uint32_t c3_addr(uint32_t wpix, uint32_t c) {
  return wpix * 128u + ((c ^ (wpix & 7u)) << 4);
}
}  // namespace

// relu(v * sc + sh) of the 8 bf16 channels of one 16-byte LDS chunk, in place
__device__ __forceinline__ void bn_relu_chunk_lds(char* at, const float (&sc)[8], const float (&sh)[8]) {
  bf16x8 v = *LDS_PTR(bf16x8, at);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf(bf2f(v[e]) * sc[e] + sh[e], 0.f));  // as bn_act_fwd_kernel
  *LDS_PTR(bf16x8, at) = v;
}

// NU (1 or 2) 16-pixel subtiles s0, s0 + 2 of the staged strip: 9 taps x 2 k-halves x NU
// fragment reads, 36 NU MFMAs, then the bf16 epilogue (statistics, staged 32-byte row stores).
// Staging rows (pixels) are 64 B = 4 chunks of 16 B, chunk XOR-swizzled by (row >> 2) & 3: the
// ds_read_b128 lane groups of the read-back then hit 16 distinct slots (the 2-byte writes stay
// at most 2-way, which costs nothing extra).
template <int NU>
__device__ __forceinline__ void c3_tile(const C3Params& p, const char* win, char* stage, const bf16x8 (&bw)[9][2][2],
                                        int s0, int du, int npix, size_t ybase, int ch, int lane, float (&K)[2],
                                        float (&s1)[2], float (&s2)[2], float& cnt, bool& have_k) {
  const uint32_t lr = lane & 15, lg = lane >> 4;
  const int W = p.W, Wp = p.Wp;
  uint32_t base[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const uint32_t pix = min((s0 + du * u) * 16 + (int)lr, npix - 1);  // past the strip: clamped
    const uint32_t r = fdiv(pix, p.div_w), xp = pix - r * W;
    base[u] = r * Wp + xp;
  }
  f32x4 acc[NU][2];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[u][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 18 (tap, k-half) steps, software-pipelined: the fragments of step i+1 are read from LDS
  // before the MFMAs of step i, so the LDS latency hides behind the previous step's MFMAs
  auto frag = [&](int st, int u) {
    const int t = st >> 1, h = st & 1;
    return *LDS_PTR(bf16x8, win + c3_addr(base[u] + (t / 3) * Wp + (t % 3), 4 * h + lg));
  };
  bf16x8 a[2][NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) a[0][u] = frag(0, u);
#pragma unroll
  for (int st = 0; st < 18; ++st) {
    if (st + 1 < 18)
#pragma unroll
      for (int u = 0; u < NU; ++u) a[(st + 1) & 1][u] = frag(st + 1, u);
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[u][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st & 1][u], bw[st >> 1][st & 1][n], acc[u][n], 0, 0, 0);
  }
  // epilogue: D[pixel 16 sub + 4 lg + i][co 32 ch + 16 n + lr]
  if (!have_k) {  // per-wave statistics shift: the wave's first output (a valid pixel)
#pragma unroll
    for (int n = 0; n < 2; ++n) K[n] = __shfl(bf2f(f2bf(acc[0][n][0])), (int)lr, 64);
    have_k = true;
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = u * 16 + 4 * (int)lg + i;
      const bool valid = (s0 + du * u) * 16 + 4 * (int)lg + i < npix;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const bf16 v = f2bf(acc[u][n][i]);
        const float d = valid ? bf2f(v) - K[n] : 0.f;
        s1[n] += d;
        s2[n] = fmaf(d, d, s2[n]);
        const uint32_t cc = (uint32_t)(2 * n + (lr >> 3)) ^ lg;  // (row >> 2) & 3 == lg
        *LDS_PTR(bf16, stage + row * 64 + cc * 16 + (lr & 7) * 2) = v;
      }
      cnt += valid ? 1.f : 0.f;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's staging writes are done
  __builtin_amdgcn_wave_barrier();
  {
    const int u = lane >> 5, pr = (lane >> 1) & 15, half = lane & 1;
    const int row = u * 16 + pr, q = (pr >> 2) & 3;
    const int pix = (s0 + du * u) * 16 + pr;
    bf16x8 v0, v1;
    if (u < NU) {
      v0 = *LDS_PTR(bf16x8, stage + row * 64 + (((2 * half) ^ q) << 4));
      v1 = *LDS_PTR(bf16x8, stage + row * 64 + (((2 * half + 1) ^ q) << 4));
    }
    if (u < NU && pix < npix) {
      bf16* dst = p.y + ybase + (size_t)pix * 64 + 32 * ch + 16 * half;
      *(bf16x8*)dst = v0;
      *(bf16x8*)(dst + 8) = v1;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before the next writes
  __builtin_amdgcn_wave_barrier();
}

// Same tile with the MFMA operands swapped (weights as A, window as B): the accumulator then
// holds D[co 32 ch + 16 n + 4 lg + i][pixel 16 sub + lr], i.e. each lane owns 4 consecutive
// output channels of one pixel and stores them as one 8-byte piece straight from registers --
// no LDS staging round trip, no wave barriers.  Statistics are per (lane group, i) channel and
// reduced across the 16 pixel lanes at the end.  The default: 2-7 % faster than the staged
// epilogue at b1024 (profiles/r4/conv3x3_direct_epilogue_ab.txt); bit-identical outputs, BN
// statistics equal up to fp32 summation order.  g_tune[kC3Epilogue] = 2 selects the staged epilogue.
template <int NU>
__device__ __forceinline__ void c3_tile_direct(const C3Params& p, const char* win, const bf16x8 (&bw)[9][2][2], int s0,
                                               int du, int npix, size_t ybase, int ch, int lane, float (&K)[2][4],
                                               float (&s1)[2][4], float (&s2)[2][4], float& cnt, bool& have_k) {
  const uint32_t lr = lane & 15, lg = lane >> 4;
  const int W = p.W, Wp = p.Wp;
  uint32_t base[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const uint32_t pix = min((s0 + du * u) * 16 + (int)lr, npix - 1);
    const uint32_t r = fdiv(pix, p.div_w), xp = pix - r * W;
    base[u] = r * Wp + xp;
  }
  f32x4 acc[NU][2];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[u][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto frag = [&](int st, int u) {
    const int t = st >> 1, h = st & 1;
    return *LDS_PTR(bf16x8, win + c3_addr(base[u] + (t / 3) * Wp + (t % 3), 4 * h + lg));
  };
  // fragments are read PD steps ahead (ring of PD + 1); the schedule-group barriers keep the
  // scheduler from sinking the reads next to their MFMAs (that exposes the LDS latency per step)
  constexpr int PD = 2;
  bf16x8 a[PD + 1][NU];
#pragma unroll
  for (int st = 0; st < PD; ++st)
#pragma unroll
    for (int u = 0; u < NU; ++u) a[st][u] = frag(st, u);
#pragma unroll
  for (int st = 0; st < 18; ++st) {
    if (st + PD < 18)
#pragma unroll
      for (int u = 0; u < NU; ++u) a[(st + PD) % (PD + 1)][u] = frag(st + PD, u);
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[u][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[st >> 1][st & 1][n], a[st % (PD + 1)][u], acc[u][n],
                                                            0, 0, 0);
    if (st + PD < 18) __builtin_amdgcn_sched_group_barrier(0x100, NU, 0);  // this step's reads, then
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * NU, 0);                // its MFMAs
  }
  if (!have_k) {  // shift: the wave's first output pixel (lane lr = 0 of the lane group)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) K[n][i] = __shfl(bf2f(f2bf(acc[0][n][i])), (int)lg * 16, 64);
    have_k = true;
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int pix = (s0 + du * u) * 16 + (int)lr;
    const bool valid = pix < npix;
    bf16* dst = p.y + ybase + (size_t)pix * 64 + 32 * ch + 4 * lg;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = f2bf(acc[u][n][i]);
        const float d = valid ? bf2f(v[i]) - K[n][i] : 0.f;
        s1[n][i] += d;
        s2[n][i] = fmaf(d, d, s2[n][i]);
      }
      if (valid && !(p.ablate & 1)) *(bf16x4*)(dst + 16 * n) = v;
    }
    cnt += valid ? 1.f : 0.f;
  }
}

// NW waves per workgroup: wave w owns output-channel half w & 1 and pixel group w >> 1 (NW / 2
// groups split a strip's 16-pixel subtiles); NW = 4 runs two workgroups per CU, NW = 8 one.
template <int NW, bool DE>
__global__ void __launch_bounds__(64 * NW, 8 / NW) conv3x3_c64_kernel(const C3Params p) {
  constexpr int NPG = NW / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ch = wave & 1, pg = wave >> 1;
  char* stage = smem + p.nbuf * p.wbytes + wave * (32 * 64);
  const int H = p.H, W = p.W, Wp = p.Wp;
  const uint32_t lr = lane & 15, lg = lane >> 4;

  // B fragments: lane holds co = 32 ch + 16 n + lr, ci = 32 h + 8 lg .. +7 of tap t
  bf16x8 bw[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bw[t][h][n] =
            *(const bf16x8*)(p.w + ((size_t)(32 * ch + 16 * n + lr) * 9 + (p.wflip ? 8 - t : t)) * 64 + 32 * h + 8 * lg);

  if (p.sched == 3 && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // BN prologue: a thread's window chunks all hold the same 8 channels -- chunk qq = tid + k * 64 NW
  // keeps qq & 7 and (qq >> 3) & 7, so its channel chunk (qq & 7) ^ (pixel & 7) is fixed
  const bool pro = p.pscale != nullptr;
  float psc[8], psh[8];
  if (pro) {
    const int pc = ((tid & 7) ^ ((tid >> 3) & 7)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      psc[e] = p.pscale[pc + e];
      psh[e] = p.pshift[pc + e];
    }
  }
  float K[2] = {0.f, 0.f}, s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, cnt = 0.f;
  float K4[DE ? 2 : 1][4] = {}, t1[DE ? 2 : 1][4] = {}, t2[DE ? 2 : 1][4] = {};
  bool have_k = false;
  const int s_begin = blockIdx.x * p.sps, s_end = min(p.strips, s_begin + p.sps);

  // strip s's input window -> window buffer b (LDS-DMA; zero page outside the image)
  auto load_strip = [&](int s, int b) {
    if (DE && (p.ablate & 2) && s != s_begin) return;
    char* wb = smem + b * p.wbytes;
    const int n_img = fdiv(s, p.div_spi);
    const int y0 = (s - n_img * p.spi) * p.R;
    for (int qq = tid; qq < p.xq; qq += 64 * NW) {
      const uint32_t P = qq >> 3;
      const uint32_t rr = fdiv(P, p.div_wp), xx = P - rr * Wp;
      const int yy = y0 - 1 + (int)rr, xi = (int)xx - 1;
      const bool ok = yy >= 0 && yy < H && xi >= 0 && xi < W;
      const uint32_t c = (qq & 7) ^ (P & 7u);
      const bf16* g = ok ? p.x + ((size_t)(n_img * H + yy) * W + xi) * 64 + c * 8 : p.zero;
      dma16(g, wb + (qq - lane) * 16);
    }
  };
  if (p.nbuf == 2 && s_begin < s_end) load_strip(s_begin, 0);
  for (int s = s_begin; s < s_end; ++s) {
    const int n_img = fdiv(s, p.div_spi);
    const int y0 = (s - n_img * p.spi) * p.R;
    const int rows = min(p.R, H - y0), npix = rows * W;
    const int b = p.nbuf == 2 ? (s - s_begin) & 1 : 0;
    if (p.nbuf == 1) {
      __syncthreads();  // every wave is done with the previous strip's window
      load_strip(s, 0);
    }
    // strip s landed (own DMA drained, then the barrier); with two buffers every wave is also
    // done with buffer b^1 (strip s-1), which now receives strip s+1 behind this strip's MFMAs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (p.nbuf == 2 && s + 1 < s_end) load_strip(s + 1, b ^ 1);
    if (pro) {
      // BN + ReLU once per staged in-image element (the zero halo / padding stays zero: the conv
      // pads the BN OUTPUT), then a raw barrier: the next strip's DMA stays in flight
      char* wb = smem + b * p.wbytes;
      for (int qq = tid; qq < p.xq; qq += 64 * NW) {
        const uint32_t P = qq >> 3;
        const uint32_t rr = fdiv(P, p.div_wp), xx = P - rr * Wp;
        const int yy = y0 - 1 + (int)rr, xi = (int)xx - 1;
        if (yy >= 0 && yy < H && xi >= 0 && xi < W) bn_relu_chunk_lds(wb + qq * 16, psc, psh);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    const char* win = smem + b * p.wbytes;

    const int nsub = (npix + 15) >> 4;
    const size_t ybase = ((size_t)(n_img * H + y0) * W) * 64;
    // sched = 4: the upper wave half (sharing each SIMD with a lower-half wave) walks its
    // subtiles in reverse, so the two waves of a SIMD are out of phase (one reads / stores while
    // the other runs MFMAs) instead of in lockstep
    const bool rev = p.sched == 4 && wave >= NW / 2 && pg < nsub;
    const int s_last = pg < nsub ? pg + 2 * NPG * ((nsub - 1 - pg) / (2 * NPG)) : pg;
    for (int it = pg; it < nsub; it += 2 * NPG) {
      const int s0 = rev ? s_last - (it - pg) : it;
      if constexpr (DE) {
        if (s0 + NPG < nsub)
          c3_tile_direct<2>(p, win, bw, s0, NPG, npix, ybase, ch, lane, K4, t1, t2, cnt, have_k);
        else
          c3_tile_direct<1>(p, win, bw, s0, NPG, npix, ybase, ch, lane, K4, t1, t2, cnt, have_k);
      } else {
        if (s0 + NPG < nsub)
          c3_tile<2>(p, win, stage, bw, s0, NPG, npix, ybase, ch, lane, K, s1, s2, cnt, have_k);
        else  // odd tail: one subtile, no wasted MFMAs
          c3_tile<1>(p, win, stage, bw, s0, NPG, npix, ybase, ch, lane, K, s1, s2, cnt, have_k);
      }
    }
  }
  if (!p.part) return;

  if constexpr (DE) {
    // direct epilogue: lanes lr (pixels) share channel 32 ch + 16 n + 4 lg + i -> reduce across them
#pragma unroll
    for (int off = 1; off < 16; off *= 2) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          t1[n][i] += __shfl_xor(t1[n][i], off, 64);
          t2[n][i] += __shfl_xor(t2[n][i], off, 64);
        }
      cnt += __shfl_xor(cnt, off, 64);
    }
    __syncthreads();
    float* sc = (float*)smem;
    if (lr == 0)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* e = sc + ((wave * 2 + n) * 16 + 4 * lg + i) * 4;
          e[0] = cnt;
          e[1] = K4[n][i];
          e[2] = t1[n][i];
          e[3] = t2[n][i];
        }
  } else {
    // per-wave channel sums: lanes lr share a channel across the 4 lane groups
#pragma unroll
    for (int off = 16; off < 64; off *= 2) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        s1[n] += __shfl_xor(s1[n], off, 64);
        s2[n] += __shfl_xor(s2[n], off, 64);
      }
      cnt += __shfl_xor(cnt, off, 64);
    }
    __syncthreads();  // window / staging no longer read: reuse as scratch
    float* sc = (float*)smem;  // [NW waves][2 n][16][4]: cnt, K, s1, s2
    if (lg == 0)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float* e = sc + ((wave * 2 + n) * 16 + lr) * 4;
        e[0] = cnt;
        e[1] = K[n];
        e[2] = s1[n];
        e[3] = s2[n];
      }
  }
  __syncthreads();
  const float* sc = (const float*)smem;
  if (tid < 64) {  // channel c = tid: waves (c >> 5) + 2 q hold it, n = (c >> 4) & 1
    const int c = tid, cw = c >> 5, n = (c >> 4) & 1, l = c & 15;
    float nt = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int q = 0; q < NPG; ++q) {
      const float* e = sc + (((cw + 2 * q) * 2 + n) * 16 + l) * 4;
      const float nb = e[0];
      if (nb <= 0.f) continue;
      const float mb = e[1] + e[2] / nb, m2b = fmaxf(e[3] - e[2] * e[2] / nb, 0.f);
      const float ntot = nt + nb, delta = mb - mean;
      mean += delta * nb / ntot;
      m2 += m2b + delta * delta * nt * nb / ntot;
      nt = ntot;
    }
    float* o = p.part + (size_t)blockIdx.x * 3 * 64;
    o[c] = nt;
    o[64 + c] = mean;
    o[128 + c] = m2;
  }
}

// ---------------------------------------------------------------------------
// variants (g_tune[kC3Variant]): 0 = 8 waves, one workgroup per CU, double-buffered windows (the next
// strip streams in behind this strip's MFMAs); 1 = 4 waves, two workgroups per CU, one window
// each; 2 = 4 waves, two double-buffered smaller windows
struct C3Cfg {
  int nw, nbuf, budget;  // waves, window buffers, bytes per window buffer
};
static C3Cfg c3_cfg() {
  if (g_tune[kC3Variant] == 1) return {4, 1, kC3WinMax};
  if (g_tune[kC3Variant] == 2) return {4, 2, kC3WinBuf2};
  if (g_tune[kC3Epilogue] != 2)  // direct epilogue: no staging tiles, the LDS goes to taller windows
    return {8, 2, g_tune[kC3WindowKB] > 0 ? std::min(g_tune[kC3WindowKB], 78) * 1024 : kC3WinDirect};
  return {8, 2, kC3WinMax};
}

// window pitch: W + 8 pixels (>= the 2 halo columns, and Wp - W = 0 mod 8 keeps the 16-B chunk
// swizzle residues consecutive across an output-row wrap inside a 16-pixel subtile)
static int c3_pitch(int W) { return W + 8; }

static int c3_rows(int H, int W) {
  const int Wp = c3_pitch(W);
  int R = c3_cfg().budget / (Wp * 128) - 2;
  R = std::min(R, H);
  if (R < 1) return 0;
  const int spi = (H + R - 1) / R;  // equal strips per image
  return (H + spi - 1) / spi;
}

bool conv3x3_c64_supported(int H, int W, int C, int Co) {
  return g_tune[kC3Off] != 1 && C == 64 && Co == 64 && H >= 1 && W >= 1 && c3_rows(H, W) > 0;
}

int conv3x3_c64_blocks(int N, int H, int W, int num_cu) {
  const int R = c3_rows(H, W);
  const int strips = N * ((H + R - 1) / R);
  const int target = std::max(1, num_cu * 8 / c3_cfg().nw);
  const int sps = (strips + target - 1) / target;
  return (strips + sps - 1) / sps;
}

void launch_conv3x3_c64(const bf16* x, const bf16* w, bf16* y, float* part, const bf16* zero, int N, int H, int W,
                        int blocks, hipStream_t stream, const float* pscale, const float* pshift, int wflip) {
  const C3Cfg cfg = c3_cfg();
  C3Params p;
  p.x = x; p.w = w; p.y = y; p.part = part; p.zero = zero;
  p.pscale = pscale; p.pshift = pshift;
  p.wflip = wflip;
  p.H = H; p.W = W;
  p.ablate = g_tune[kAblate];
  p.sched = g_tune[kC3Variant];
  p.R = c3_rows(H, W);
  p.spi = (H + p.R - 1) / p.R;
  p.strips = N * p.spi;
  p.sps = (p.strips + blocks - 1) / blocks;
  p.Wp = c3_pitch(W);
  p.xq = (p.R + 2) * p.Wp * 8;
  p.nbuf = cfg.nbuf;
  p.wbytes = (p.xq * 16 + 1023) / 1024 * 1024;
  p.div_wp = make_fastdiv(p.Wp);
  p.div_w = make_fastdiv(W);
  p.div_spi = make_fastdiv(p.spi);
  const bool de = g_tune[kC3Epilogue] != 2;
  const int lds = p.nbuf * p.wbytes + (de ? 0 : cfg.nw * 32 * 64);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3x3_c64_kernel<4, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * kC3WinBuf2 + 2048 + kC3Stage);
    (void)hipFuncSetAttribute((const void*)conv3x3_c64_kernel<4, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * kC3WinBuf2 + 2048 + kC3Stage);
    (void)hipFuncSetAttribute((const void*)conv3x3_c64_kernel<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * kC3WinMax + 2048 + 2 * kC3Stage);
    (void)hipFuncSetAttribute((const void*)conv3x3_c64_kernel<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * 78 * 1024 + 2048);
    attr = true;
  }
  if (cfg.nw == 8) {
    if (de)
      hipLaunchKernelGGL((conv3x3_c64_kernel<8, true>), dim3(blocks), dim3(512), lds, stream, p);
    else
      hipLaunchKernelGGL((conv3x3_c64_kernel<8, false>), dim3(blocks), dim3(512), lds, stream, p);
  } else {
    if (de)
      hipLaunchKernelGGL((conv3x3_c64_kernel<4, true>), dim3(blocks), dim3(256), lds, stream, p);
    else
      hipLaunchKernelGGL((conv3x3_c64_kernel<4, false>), dim3(blocks), dim3(256), lds, stream, p);
  }
}

}  // namespace dcp
