// Grouped convolution on the matrix cores (ResNeXt-50 32x4d, BASELINE.json
// config 4; reference: torchvision resnext50_32x4d as
// built by BASELINE/train.py `--model`).
//
// The group widths of ResNeXt (CG = 4, 8, 16, 32 channels) are far below an
// MFMA tile, so channels are processed in "super-groups" of SG = 16 or 32
// channels (SG a multiple of CG).  Inside a super-group the grouped conv is a
// dense SG x (T*SG) GEMM whose weight is block-diagonal: the zero blocks cost
// MFMA issue slots (cheap: the op is memory-bound) but let every operand be a
// plain 16x16x32 bf16 fragment.
//
// One workgroup = 256 consecutive destination pixels (linear n,y,x order) of
// one super-group (gconv_gather_kernel) or of several (gconv_gather_multi_kernel:
// per-pixel setup done once, super-groups streamed through an LDS ring).  The
// source rows those pixels touch (a contiguous range of global rows n*Hs+h) are
// staged once in LDS with 16-byte loads, so every tap re-reads LDS instead of
// L2.  Pixel index 0 of the LDS image is a zero pixel that out-of-range taps
// point at ("pad, don't mask").
//
//   fwd  : dst = y  [N,Ho,Wo,C], src = x  rows  y*s + (kh-p)
//   dgrad: dst = dx [N,H,W,C],   src = dy rows (y + (p-kh)) / s when divisible
//   wgrad: A = dy^T and B = gathered x, both read with ds_read_b64_tr_b16 from
//          LDS images [pixel][SG]; per-split partials reduced deterministically.
#include <map>
#include <mutex>
#include <tuple>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {

constexpr int GP = 256;  // destination pixels per workgroup / wgrad chunk
constexpr int GT = 9;    // max taps

struct GconvParams {
  const bf16* src;  // gathered image [N][Hs][Ws][C]
  const bf16* w;    // [C][T][CG] grouped weight (bf16)
  bf16* dst;        // fwd / dgrad output [N][Hd][Wd][C]
  const bf16* dy;   // wgrad: [N][Hd][Wd][C]
  float* part;      // wgrad: [splits][C][T][CG]
  float* stats;     // fwd (optional): BN partials [pixel blocks][3][C] = (n, mean, M2) of the output
  // dgrad (optional) fused backward of the ReLU BN that produced the conv input: dst receives the
  // masked gradient g = dx * [z*scale + shift > 0] and bnsum[pixel block][2][C] its per-tile
  // (sum g, sum g * (z - mean) * invstd)
  const bf16* bnz;
  const float *bn_scale, *bn_shift, *bn_mean, *bn_invstd;
  float* bnsum;
  const bf16* wfrag;  // fwd/dgrad: fragment-ordered block-diagonal weight (gconv_frag_kernel)
  const bf16* zero;   // >= 16 bytes of zeros (global)
  int nbuf;           // wgrad: 2 = double-buffered chunks
  int ablate;         // multi kernel timing ablations (g_tune ablate): 1 = loads only, 2 = no loads, 4 = no stores
  int spw, nbuf_g, bufb_g;  // fwd/dgrad multi kernel: super-groups per workgroup, LDS ring buffers, bytes each
  int Hs, Ws, Hd, Wd, C, CG, T;
  int ss, sd;       // src row = (dst_row*ss + oh) / sd, sd in {1, 2}
  int M;            // N*Hd*Wd
  int nsg, ntiles;  // super-groups, total tiles (pixel blocks x nsg)
  int rows_per_split, bufb;  // wgrad: pixels per split, LDS bytes per chunk buffer
  int ohmin, ohmax;
  FastDiv div_wd, div_hd;
  int8_t oh[GT + 1], ow[GT + 1];
};

__device__ __forceinline__ int floor_sd(int v, int sd) { return sd == 1 ? v : (v >> 1); }

// contiguous global-row range [R_lo, R_lo + NR) of src rows touched by dst pixels [m0, m1]
__device__ __forceinline__ void halo_rows(const GconvParams& p, int m0, int m1, int& R_lo, int& NR) {
  const uint32_t q0 = fdiv((uint32_t)m0, p.div_wd), q1 = fdiv((uint32_t)m1, p.div_wd);
  const int n0 = (int)fdiv(q0, p.div_hd), n1 = (int)fdiv(q1, p.div_hd);
  const int y0 = (int)q0 - n0 * p.Hd, y1 = (int)q1 - n1 * p.Hd;
  const int rlo = max(0, floor_sd(y0 * p.ss + p.ohmin, p.sd));
  const int rhi = min(p.Hs - 1, floor_sd(y1 * p.ss + p.ohmax, p.sd));
  R_lo = n0 * p.Hs + rlo;
  NR = n1 * p.Hs + rhi - R_lo + 1;
}

// stage NR*Ws pixels x SG channels of super-group sg at LDS pixel 1.. with
// LDS-DMA (global_load_lds: lane data lands at wave base + 16*lane, and the
// image is laid out in exactly the enumeration order); zero pixel at 0.
template <int SG>
__device__ __forceinline__ void stage_halo(const GconvParams& p, char* img, int sg, int R_lo, int NR) {
  constexpr int CH = SG / 8;
  const int total = NR * p.Ws * CH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bf16* base = p.src + (size_t)R_lo * p.Ws * p.C + sg * SG;
  for (int e0 = wave * 64; e0 < total; e0 += 256) {
    const int e = e0 + lane;
    if (e < total)
      dma16((base + (size_t)(e / CH) * p.C + (e % CH) * 8), img + SG * 2 + e0 * 16);
  }
}

template <int SG>
__device__ __forceinline__ void zero_pixel(char* img) {
  if (threadIdx.x < SG / 8) *(bf16x8*)(img + threadIdx.x * 16) = bf16x8{};
}

struct PixGeo {
  int rb;   // (n*Hs - R_lo) : row base relative to the halo
  int yy, xx;
  bool ok;
};

__device__ __forceinline__ PixGeo pix_geo(const GconvParams& p, int m, int R_lo) {
  PixGeo g;
  g.ok = m < p.M;
  const uint32_t mm = g.ok ? (uint32_t)m : 0u;
  const uint32_t q = fdiv(mm, p.div_wd);
  const int x = (int)(mm - q * p.Wd);
  const int n = (int)fdiv(q, p.div_hd);
  const int y = (int)q - n * p.Hd;
  g.rb = n * p.Hs - R_lo;
  g.yy = y * p.ss;
  g.xx = x * p.ss;
  return g;
}

// LDS pixel index of tap (oh, ow) for a destination pixel, 0 = zero pixel
__device__ __forceinline__ int tap_idx(const GconvParams& p, const PixGeo& g, int oh, int ow, bool tap_ok) {
  int h = g.yy + oh, w = g.xx + ow;
  bool ok = g.ok && tap_ok;
  if (p.sd != 1) {
    ok = ok && (((h | w) & 1) == 0);
    h >>= 1;
    w >>= 1;
  }
  ok = ok && (unsigned)h < (unsigned)p.Hs && (unsigned)w < (unsigned)p.Ws;
  return ok ? 1 + (g.rb + h) * p.Ws + w : 0;
}

// A fragment of the block-diagonal dense weight: 8 k-values (tap t, channels c0..c0+7)
// of row `row`.  DGRAD=false: row = output channel, k channel = input channel;
// DGRAD=true: row = input channel, k channel = output channel.
template <int SG, bool DGRAD>
__device__ __forceinline__ bf16x8 w_frag(const GconvParams& p, int sg, int row, int t, int c0) {
  bf16x8 v{};
  if (t >= p.T) return v;
  const int T = p.T, CG = p.CG;
  const int grow = row / CG;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    if (c / CG != grow) continue;
    const int co = DGRAD ? c : row;   // output channel (local)
    const int ci = DGRAD ? row : c;   // input channel (local)
    v[e] = p.w[((size_t)(sg * SG + co) * T + t) * CG + (ci % CG)];
  }
  return v;
}

// ---------------------------------------------------------------------------
// fwd / dgrad: D[row = channel][col = pixel] = W_bd[row][k] * B[k][pixel]
// ---------------------------------------------------------------------------
// DPP data movement inside a row of 16 lanes (VALU, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ float gdpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, true));
}
// sum over the 16 lanes of a row, every lane of the row receiving the same total: row_ror 8 is
// xor 8, row_ror 4 on the then period-8 pattern is xor 4, the quad permutations xor 2 and xor 1
__device__ __forceinline__ float row16_sum(float v) {
  v += gdpp<0x128>(v);
  v += gdpp<0x124>(v);
  v += gdpp<0x4E>(v);
  v += gdpp<0xB1>(v);
  return v;
}

__device__ __forceinline__ bf16x4 cvt_bf16x4(f32x4 v) { return __builtin_convertvector(v, bf16x4); }

// BN statistics of the forward tile (256 pixels x SG channels) from the bf16-rounded outputs ob:
// per-wave shifted sums (shift = the row's first lane's first output of each channel, broadcast
// with row_newbcast), the 16 lanes of one channel group summed with DPP, the four waves merged
// with Chan's formula -> (n, mean, M2) of the tile's channels in partial row pb (the [P][3][C]
// layout bn_stats / bn_stats_finalize merge).
template <int SG, int NRT, int CPT>
__device__ __forceinline__ void gconv_tile_stats(const GconvParams& p, const bf16x4 (&ob)[NRT][CPT], float* sc,
                                                 bool lead_sync, int m0, int sg, int pb, int wave, int lane) {
  const int wbase = m0 + wave * 64;
  float K[NRT][4], s1[NRT][4], s2[NRT][4];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      K[rt][r] = gdpp<0x150>(bf2f(ob[rt][0][r]));  // row_newbcast:0
      s1[rt][r] = s2[rt][r] = 0.f;
    }
#pragma unroll
  for (int ct = 0; ct < CPT; ++ct) {
    const bool valid = wbase + ct * 16 + (lane & 15) < p.M;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = valid ? bf2f(ob[rt][ct][r]) - K[rt][r] : 0.f;
        s1[rt][r] += d;
        s2[rt][r] = fmaf(d, d, s2[rt][r]);
      }
  }
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[rt][r] = row16_sum(s1[rt][r]);
      s2[rt][r] = row16_sum(s2[rt][r]);
    }
  const float cnt = (float)min(max(p.M - wbase, 0), 64);  // valid pixels of the wave
  if (lead_sync) __syncthreads();  // scratch aliases the staged halo image: every wave must be done with it
  // sc: [4 waves][SG channels][4]: cnt, K, s1, s2
  if ((lane & 15) == 0)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* e = sc + (wave * SG + rt * 16 + (lane >> 4) * 4 + r) * 4;
        e[0] = cnt;
        e[1] = K[rt][r];
        e[2] = s1[rt][r];
        e[3] = s2[rt][r];
      }
  __syncthreads();
  if (threadIdx.x < SG) {
    const int c = threadIdx.x;
    float nt = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* e = sc + (w * SG + c) * 4;
      const float nb = e[0];
      if (nb <= 0.f) continue;
      const float rnb = __builtin_amdgcn_rcpf(nb);
      const float mb = e[1] + e[2] * rnb, m2b = fmaxf(e[3] - e[2] * e[2] * rnb, 0.f);
      const float ntot = nt + nb, delta = mb - mean, f = nb * __builtin_amdgcn_rcpf(ntot);
      mean += delta * f;
      m2 += m2b + delta * delta * nt * f;
      nt = ntot;
    }
    float* o = p.stats + (size_t)pb * 3 * p.C + sg * SG + c;
    o[0] = nt;
    o[p.C] = mean;
    o[2 * p.C] = m2;
  }
}

// dgrad epilogue fused with the producing BN(+ReLU)'s backward reduction: store the masked
// gradient and the tile's per-channel (sum g, sum g * xhat) -- the BN backward is then left with
// its elementwise pass (no reduction pass re-reading g and z).
template <int SG, int NRT, int CPT>
__device__ __forceinline__ void gconv_dgrad_bn_epilogue(const GconvParams& p, const f32x4 (&acc)[NRT][CPT],
                                                        float* xs, bool lead_sync, int m0, int sg, int pb,
                                                        int wave, int lane) {
  float sc[NRT][4], sh[NRT][4], mu[NRT][4], is[NRT][4], sg1[NRT][4], sg2[NRT][4];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = sg * SG + rt * 16 + (lane >> 4) * 4 + r;
      sc[rt][r] = p.bn_scale[c];
      sh[rt][r] = p.bn_shift[c];
      mu[rt][r] = p.bn_mean[c];
      is[rt][r] = p.bn_invstd[c];
      sg1[rt][r] = sg2[rt][r] = 0.f;
    }
#pragma unroll
  for (int ct = 0; ct < CPT; ++ct) {
    const int m = m0 + wave * 64 + ct * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
      const size_t off = (size_t)m * p.C + sg * SG + rt * 16 + (lane >> 4) * 4;
      const bf16x4 z = *(const bf16x4*)(p.bnz + off);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float zf = bf2f(z[r]);
        const bf16 gb = f2bf(zf * sc[rt][r] + sh[rt][r] > 0.f ? acc[rt][ct][r] : 0.f);
        o[r] = gb;
        const float g = bf2f(gb);
        sg1[rt][r] += g;
        sg2[rt][r] = fmaf(g, (zf - mu[rt][r]) * is[rt][r], sg2[rt][r]);
      }
      *(bf16x4*)(p.dst + off) = o;
    }
  }
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sg1[rt][r] = row16_sum(sg1[rt][r]);
      sg2[rt][r] = row16_sum(sg2[rt][r]);
    }
  if (lead_sync) __syncthreads();  // scratch aliases the staged image: every wave must be done with it
  // xs: [4 waves][2][SG]
  if ((lane & 15) == 0)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = rt * 16 + (lane >> 4) * 4 + r;
        xs[(wave * 2 + 0) * SG + c] = sg1[rt][r];
        xs[(wave * 2 + 1) * SG + c] = sg2[rt][r];
      }
  __syncthreads();
  if (threadIdx.x < 2 * SG) {
    const int k = threadIdx.x / SG, c = threadIdx.x % SG;
    const float t = (xs[(0 * 2 + k) * SG + c] + xs[(1 * 2 + k) * SG + c]) +
                    (xs[(2 * 2 + k) * SG + c] + xs[(3 * 2 + k) * SG + c]);
    p.bnsum[((size_t)pb * 2 + k) * p.C + sg * SG + c] = t;
  }
}

template <int SG, bool DGRAD>
__global__ void __launch_bounds__(256) gconv_gather_kernel(const GconvParams p) {
  constexpr int NRT = SG / 16;                 // 16-row tiles of the output channels
  constexpr int TPS = SG == 16 ? 2 : 1;        // taps per k-step (32 k per MFMA)
  constexpr int NST = (GT + TPS - 1) / TPS;    // max k-steps
  constexpr int CPT = 4;                       // 16-pixel column tiles per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = (int)xcd_remap(blockIdx.x, p.ntiles);
  const int sg = tile % p.nsg, pb = tile / p.nsg;
  const int m0 = pb * GP, m1 = min(p.M, m0 + GP) - 1;
  int R_lo, NR;
  halo_rows(p, m0, m1, R_lo, NR);
  stage_halo<SG>(p, smem, sg, R_lo, NR);
  zero_pixel<SG>(smem);

  const int kc = lane >> 4;                    // k-chunk of 8 within the 32-wide k-step
  const int chunk = SG == 16 ? (kc & 1) : kc;  // 16-byte chunk of the source pixel
  const int nst = (p.T + TPS - 1) / TPS;

  // lane-private tap list + weight fragments (registers for the whole block)
  int8_t toh[NST], tow[NST];
  bool tok[NST];
  bf16x8 a[NST][NRT];
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    const int t0 = st * TPS;
    const int t = SG == 16 ? ((kc >> 1) ? t0 + 1 : t0) : t0;
    toh[st] = SG == 16 ? ((kc >> 1) ? p.oh[t0 + 1] : p.oh[t0]) : p.oh[t0];
    tow[st] = SG == 16 ? ((kc >> 1) ? p.ow[t0 + 1] : p.ow[t0]) : p.ow[t0];
    tok[st] = t < p.T;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
      a[st][rt] = st < nst ? *(const bf16x8*)(p.wfrag + ((size_t)((sg * nst + st) * NRT + rt) * 64 + lane) * 8)
                           : bf16x8{};
  }

  PixGeo g[CPT];
#pragma unroll
  for (int ct = 0; ct < CPT; ++ct) g[ct] = pix_geo(p, m0 + wave * 64 + ct * 16 + (lane & 15), R_lo);

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[NRT][CPT];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CPT; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // forward: every k-step runs -- past the kernel's taps (st >= nst) the fragments are zero and
  // the taps point at the zero pixel, so the products vanish, and a uniform branch around them cut
  // the accumulators' live ranges into pieces shuttled through AGPRs (fwd 163 -> 154 us on the
  // 1024-channel stride-2 shape); the data gradient keeps the branch (without it its 32-channel
  // variant measured 449 -> 568 us, gconv_oldkernel_ab.txt)
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    if (DGRAD && st >= nst) continue;  // uniform
    bf16x8 b[CPT];
#pragma unroll
    for (int ct = 0; ct < CPT; ++ct) {
      const int idx = tap_idx(p, g[ct], toh[st], tow[st], tok[st]);
      b[ct] = *LDS_PTR(bf16x8, smem + idx * (SG * 2) + chunk * 16);
    }
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CPT; ++ct)
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st][rt], b[ct], acc[rt][ct], 0, 0, 0);
  }

  if constexpr (DGRAD) {
    if (p.bnz) {
      gconv_dgrad_bn_epilogue<SG, NRT, CPT>(p, acc, (float*)smem, true, m0, sg, pb, wave, lane);
      return;
    }
  }
  // lane holds pixel column lane&15, channels (lane>>4)*4 .. +3 of each row tile
  bf16x4 ob[NRT][CPT];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CPT; ++ct) ob[rt][ct] = cvt_bf16x4(acc[rt][ct]);
#pragma unroll
  for (int ct = 0; ct < CPT; ++ct) {
    const int m = m0 + wave * 64 + ct * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
      *(bf16x4*)(p.dst + (size_t)m * p.C + sg * SG + rt * 16 + (lane >> 4) * 4) = ob[rt][ct];
  }
  if constexpr (!DGRAD) {
    if (p.stats) gconv_tile_stats<SG, NRT, CPT>(p, ob, (float*)smem, true, m0, sg, pb, wave, lane);
  }
}

// gconv_dgrad_bn_epilogue with z and the BN coefficients read from the LDS-staged copies
// (zl: [GP][SG] bf16 of this super-group, cl: [scale | shift | mean | invstd][SG] fp32)
template <int SG, int NRT, int CPT>
__device__ __forceinline__ void gconv_dgrad_bn_epilogue_lds(const GconvParams& p, const f32x4 (&acc)[NRT][CPT],
                                                            const char* zl, const float* cl, float* xs, int m0,
                                                            int sg, int pb, int wave, int lane) {
  float sc[NRT][4], sh[NRT][4], mu[NRT][4], is[NRT][4], sg1[NRT][4], sg2[NRT][4];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt) {
    const int c = rt * 16 + (lane >> 4) * 4;
    const f32x4 a = *LDS_PTR(f32x4, cl + c), b = *LDS_PTR(f32x4, cl + SG + c);
    const f32x4 m = *LDS_PTR(f32x4, cl + 2 * SG + c), v = *LDS_PTR(f32x4, cl + 3 * SG + c);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[rt][r] = a[r];
      sh[rt][r] = b[r];
      mu[rt][r] = m[r];
      is[rt][r] = v[r];
      sg1[rt][r] = sg2[rt][r] = 0.f;
    }
  }
#pragma unroll
  for (int ct = 0; ct < CPT; ++ct) {
    const int pl = wave * 64 + ct * 16 + (lane & 15);
    const int m = m0 + pl;
    if (m >= p.M) continue;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
      const int cl4 = rt * 16 + (lane >> 4) * 4;
      const bf16x4 z = *LDS_PTR(bf16x4, zl + (pl * SG + cl4) * 2);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float zf = bf2f(z[r]);
        const bf16 gb = f2bf(zf * sc[rt][r] + sh[rt][r] > 0.f ? acc[rt][ct][r] : 0.f);
        o[r] = gb;
        const float g = bf2f(gb);
        sg1[rt][r] += g;
        sg2[rt][r] = fmaf(g, (zf - mu[rt][r]) * is[rt][r], sg2[rt][r]);
      }
      if (p.ablate != 4) *(bf16x4*)(p.dst + (size_t)m * p.C + sg * SG + cl4) = o;
    }
  }
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sg1[rt][r] = row16_sum(sg1[rt][r]);
      sg2[rt][r] = row16_sum(sg2[rt][r]);
    }
  // xs: [4 waves][2][SG] (the caller's loop barrier orders it against the previous reader)
  if ((lane & 15) == 0)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = rt * 16 + (lane >> 4) * 4 + r;
        xs[(wave * 2 + 0) * SG + c] = sg1[rt][r];
        xs[(wave * 2 + 1) * SG + c] = sg2[rt][r];
      }
  __syncthreads();
  if (threadIdx.x < 2 * SG) {
    const int k = threadIdx.x / SG, c = threadIdx.x % SG;
    const float t = (xs[(0 * 2 + k) * SG + c] + xs[(1 * 2 + k) * SG + c]) +
                    (xs[(2 * 2 + k) * SG + c] + xs[(3 * 2 + k) * SG + c]);
    p.bnsum[((size_t)pb * 2 + k) * p.C + sg * SG + c] = t;
  }
}

// s_waitcnt vmcnt(n') for the largest n' <= n from a short ladder (n is wave-uniform at run time;
// waiting until at most n' <= n operations are outstanding is at least as strict as n)
__device__ __forceinline__ void wait_vmcnt_atmost(int n) {
  if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// fwd / dgrad, SPW super-groups per workgroup (p.spw; the pixel block's super-groups
// sg0 .. sg0+spw-1).  The one-super-group kernel above spends most of its vector-ALU issue on
// per-block setup -- pixel geometry, 20 tap indices per lane, halo bounds -- that does not depend
// on the super-group: here it is done once and reused.  The super-groups' halo images and weight
// fragments stream through a ring of p.nbuf_g LDS buffers (LDS-DMA): a buffer is refilled with
// super-group i + nbuf as soon as every wave has finished computing on super-group i, so every
// buffer but the one being computed on has loads in flight (the one-super-group kernel keeps its
// whole LDS image in flight the same way, through occupancy).  Buffer layout:
// [weight fragments: NST*NRT*64 x 16 B][zero pixel][halo].
template <int SG, bool DGRAD>
__global__ void __launch_bounds__(256) gconv_gather_multi_kernel(const GconvParams p) {
  constexpr int NRT = SG / 16;
  constexpr int TPS = SG == 16 ? 2 : 1;
  constexpr int NST = (GT + TPS - 1) / TPS;
  constexpr int CPT = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = (int)xcd_remap(blockIdx.x, p.ntiles);
  const int nsgb = (p.nsg + p.spw - 1) / p.spw;
  const int sgb = tile % nsgb, pb = tile / nsgb;
  const int sg0 = sgb * p.spw, nsp = min(p.spw, p.nsg - sg0);
  const int m0 = pb * GP, m1 = min(p.M, m0 + GP) - 1;
  const bool full = m0 + GP <= p.M;
  int R_lo, NR;
  halo_rows(p, m0, m1, R_lo, NR);
  const int nfr = NST * NRT * 64;  // 16-byte weight fragments per super-group
  const int fragb = nfr * 16;
  // dgrad fused with the BN backward: the super-group's z tile [GP][SG] and its four coefficient
  // vectors [4][SG] are staged with the halo (no global loads in the loop: the compiler cannot
  // count the untracked LDS-DMA, so any wait it placed for a global load would drain the ring)
  const bool bnst = DGRAD && p.bnz != nullptr;
  const int zo = fragb, co = zo + GP * SG * 2;
  const int imgo = bnst ? co + 4 * SG * 4 : fragb;
  const int nb = p.nbuf_g;
  float* const scratch = (float*)(smem + nb * p.bufb_g);
  // vector-memory instructions this wave issues per staged super-group (the same for every
  // super-group of the block): one per 256-element round it takes part in
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int nhalo = NR * p.Ws * (SG / 8);
  const int per_stage = (nfr - wv * 64 + 255) / 256 + max(0, (nhalo - wv * 64 + 255) / 256) +
                        (bnst ? (GP * SG / 8) / 256 + 1 : 0);

  auto bufp = [&](int i) { return smem + (i % nb) * p.bufb_g; };
  auto stage = [&](int i) {
    if (p.ablate == 2) return;
    char* buf = bufp(i);
    const char* wsrc = (const char*)(p.wfrag + (size_t)(sg0 + i) * nfr * 8);
    for (int e0 = wave * 64; e0 < nfr; e0 += 256) {
      const int e = e0 + lane;
      if (e < nfr) dma16(wsrc + (size_t)e * 16, buf + e0 * 16);
    }
    if (bnst) {
      constexpr int CH = SG / 8;
#pragma unroll
      for (int e0 = wave * 64; e0 < GP * CH; e0 += 256) {
        const int e = e0 + lane;
        const int m = min(m0 + e / CH, m1);  // rows past the image: any valid row (not stored)
        dma16(p.bnz + (size_t)m * p.C + (sg0 + i) * SG + (e % CH) * 8, buf + zo + e0 * 16);
      }
      // [scale | shift | mean | invstd] x SG floats: wave w stages vector w (a wave-uniform pointer
      // choice stays in scalar registers; a per-lane one reads the kernel arguments from memory)
      const float* src = wv == 0 ? p.bn_scale : wv == 1 ? p.bn_shift : wv == 2 ? p.bn_mean : p.bn_invstd;
      if (lane < SG / 4) dma16(src + (sg0 + i) * SG + lane * 4, buf + co + wv * SG * 4);
    }
    stage_halo<SG>(p, buf + imgo, sg0 + i, R_lo, NR);
  };
  for (int i = 0; i < min(nb, nsp); ++i) {
    stage(i);
    zero_pixel<SG>(bufp(i) + imgo);
  }

  // per-lane LDS byte offsets of every (k-step, pixel column) operand, shared by all super-groups
  const int kc = lane >> 4;
  const int chunk = SG == 16 ? (kc & 1) : kc;
  int off[NST][CPT];
  {
    PixGeo g[CPT];
#pragma unroll
    for (int ct = 0; ct < CPT; ++ct) g[ct] = pix_geo(p, m0 + wave * 64 + ct * 16 + (lane & 15), R_lo);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const int t0 = st * TPS;
      const int t = SG == 16 ? t0 + (kc >> 1) : t0;
      // select between the two (scalar) taps rather than index the kernel arguments per lane: a
      // per-lane index becomes a global load whose wait would also drain the prologue's DMA
      const int oh0 = __builtin_amdgcn_readfirstlane(p.oh[t0]), ow0 = __builtin_amdgcn_readfirstlane(p.ow[t0]);
      const int oh1 = __builtin_amdgcn_readfirstlane(p.oh[t0 + 1]), ow1 = __builtin_amdgcn_readfirstlane(p.ow[t0 + 1]);
      const int oh = (SG == 16 && (kc >> 1)) ? oh1 : oh0;
      const int ow = (SG == 16 && (kc >> 1)) ? ow1 : ow0;
#pragma unroll
      for (int ct = 0; ct < CPT; ++ct) off[st][ct] = imgo + tap_idx(p, g[ct], oh, ow, t < p.T) * (SG * 2) + chunk * 16;
    }
  }

  for (int i = 0; i < nsp; ++i) {
    // super-group i's loads are complete once at most the younger operations are outstanding:
    // the stages issued after it (up to nb - 1 of them) and, in a full block after the first
    // iteration, the previous epilogue's CPT*NRT output stores (issued after every stage so far;
    // a ragged block may skip stores, so it does not count them)
    const int younger = p.ablate == 2 ? 0 : (min(nsp - 1, i + nb - 1) - i) * per_stage + ((i > 0 && full && p.ablate == 0) ? CPT * NRT : 0);
    wait_vmcnt_atmost(younger);
    __syncthreads();
    const int sg = sg0 + i;
    const char* cur = bufp(i);
    if (p.ablate == 1) {
      if (i + nb < nsp) {
        __syncthreads();
        stage(i + nb);
      }
      continue;
    }

    f32x4 acc[NRT][CPT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CPT; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NST; ++st) {  // 3x3 only (host-checked): nst == NST, no partial k-step loop
      bf16x8 a[NRT], b[CPT];
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) a[rt] = *LDS_PTR(bf16x8, cur + ((st * NRT + rt) * 64 + lane) * 16);
#pragma unroll
      for (int ct = 0; ct < CPT; ++ct) b[ct] = *LDS_PTR(bf16x8, cur + off[st][ct]);
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CPT; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt], b[ct], acc[rt][ct], 0, 0, 0);
    }
    if constexpr (DGRAD) {
      if (bnst) {
        // the epilogue reads this buffer's z and coefficients; its internal barrier follows the
        // last such read, so the refill goes after it
        gconv_dgrad_bn_epilogue_lds<SG, NRT, CPT>(p, acc, cur + zo, (const float*)(cur + co), scratch, m0, sg, pb,
                                                  wave, lane);
        if (i + nb < nsp) stage(i + nb);
        continue;
      }
    }
    if (i + nb < nsp) {
      __syncthreads();  // every wave is done reading buffer i % nb: refill it
      stage(i + nb);
    }
    bf16x4 ob[NRT][CPT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CPT; ++ct) ob[rt][ct] = cvt_bf16x4(acc[rt][ct]);
#pragma unroll
    for (int ct = 0; ct < CPT; ++ct) {
      const int m = m0 + wave * 64 + ct * 16 + (lane & 15);
      if (m >= p.M) continue;
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
        if (p.ablate != 4) *(bf16x4*)(p.dst + (size_t)m * p.C + sg * SG + rt * 16 + (lane >> 4) * 4) = ob[rt][ct];
    }
    if constexpr (!DGRAD) {
      if (p.stats) gconv_tile_stats<SG, NRT, CPT>(p, ob, scratch, false, m0, sg, pb, wave, lane);
    }
  }
}

// fragment-ordered block-diagonal weight: [sg][st][rt][lane][8]
template <int SG, bool DGRAD>
__global__ void gconv_frag_kernel(const GconvParams p, bf16* __restrict__ out) {
  constexpr int NRT = SG / 16;
  constexpr int TPS = SG == 16 ? 2 : 1;
  const int nst = (p.T + TPS - 1) / TPS;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.nsg * nst * NRT * 64) return;
  const int lane = i & 63, rt = (i >> 6) % NRT, st = ((i >> 6) / NRT) % nst, sg = ((i >> 6) / NRT) / nst;
  const int kc = lane >> 4;
  const int t = st * TPS + (SG == 16 ? (kc >> 1) : 0);
  const int chunk = SG == 16 ? (kc & 1) : kc;
  *(bf16x8*)(out + (size_t)i * 8) = w_frag<SG, DGRAD>(p, sg, rt * 16 + (lane & 15), t, chunk * 8);
}

// 8 consecutive rows (k) x 16 columns of a [row][SG] bf16 LDS image, transposed:
// lane (l&15) receives column col0 + (l&15); rows are given per lane (ra: rows 0-3, rb: 4-7)
__device__ __forceinline__ bf16x8 tr8(const char* img_a, const char* img_b, int lane) {
  (void)lane;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img_a));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img_b));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// ---------------------------------------------------------------------------
// wgrad: D[j][t, c] = sum_m dy[m][j] * x[src(m,t)][c] per super-group
// ---------------------------------------------------------------------------
// bit t (t = kh*3 + kw) set where tap t of a 3x3 stride-1-gather (sd == 1) hits the image
__device__ __forceinline__ uint32_t tap_mask33(const GconvParams& p, const PixGeo& g) {
  uint32_t cm = 0, m = 0;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) cm |= ((unsigned)(g.xx + p.ow[kw]) < (unsigned)p.Ws ? 1u : 0u) << kw;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) m |= (unsigned)(g.yy + p.oh[kh * 3]) < (unsigned)p.Hs ? cm << (3 * kh) : 0u;
  return g.ok ? m : 0u;
}

template <int SG, bool K33>
__global__ void __launch_bounds__(256) gconv_wgrad_kernel(const GconvParams p) {
  constexpr int NRT = SG / 16;
  constexpr int NTG = NRT * NRT;          // tile groups (row tile x column half), 9 taps each
  constexpr int KSPLIT = 4 / NTG;         // waves sharing one tile group split the k-steps
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CH = SG / 8;
  constexpr int DYB = GP * SG * 2;        // dy image [GP][SG] at the start of each buffer

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = (int)xcd_remap(blockIdx.x, p.ntiles);
  const int sg = tile % p.nsg, split = tile / p.nsg;
  const int tg = wave % NTG, kslot = wave / NTG;
  const int rt = tg % NRT, chh = tg / NRT;
  const int q = (lane & 15) >> 2, pp = lane & 3;
  const int mstart = split * p.rows_per_split;
  const int mend = min(p.M, mstart + p.rows_per_split);
  const int nchunks = (mend - mstart + GP - 1) / GP;
  const int bufb = p.bufb;

  bool tok[GT];
  int8_t toh[GT], tow[GT];
  int toff[GT];  // K33: LDS byte offset of tap t's source pixel from tap (0, 0)'s reference
#pragma unroll
  for (int t = 0; t < GT; ++t) {
    tok[t] = t < p.T;
    toh[t] = p.oh[t];
    tow[t] = p.ow[t];
    toff[t] = __builtin_amdgcn_readfirstlane((p.oh[t] * p.Ws + p.ow[t]) * (SG * 2));
  }

  // LDS-DMA of one chunk (dy rows + source halo) into buffer `buf`
  auto issue = [&](int m0c, char* buf) -> int {
    const int m1c = min(mend, m0c + GP) - 1;
    int R_lo, NR;
    halo_rows(p, m0c, m1c, R_lo, NR);
    stage_halo<SG>(p, buf + DYB, sg, R_lo, NR);
#pragma unroll
    for (int e0 = wave * 64; e0 < GP * CH; e0 += 256) {
      const int e = e0 + lane;
      const int m = m0c + e / CH;
      const bf16* g = m <= m1c ? p.dy + (size_t)m * p.C + sg * SG + (e % CH) * 8 : p.zero;
      dma16(g, buf + e0 * 16);
    }
    return R_lo;
  };

  f32x4 acc[GT];
#pragma unroll
  for (int t = 0; t < GT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  zero_pixel<SG>(smem + DYB);
  if (p.nbuf == 2) zero_pixel<SG>(smem + bufb + DYB);
  int R_cur = issue(mstart, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int ci = 0; ci < nchunks; ++ci) {
    const int m0 = mstart + ci * GP;
    const int m1 = min(mend, m0 + GP) - 1;
    char* cur = smem + (p.nbuf == 2 ? (ci & 1) * bufb : 0);
    int R_next = 0;
    if (p.nbuf == 2 && ci + 1 < nchunks) R_next = issue(m0 + GP, smem + ((ci + 1) & 1) * bufb);
    const char* dyimg = cur;
    const char* img = cur + DYB;
    for (int ks = kslot; ks < GP / 32; ks += KSPLIT) {
      const int ra = ks * 32 + 8 * (lane >> 4) + q, rb = ra + 4;
      const int col = rt * 16 + 4 * pp;
      const bf16x8 af = tr8(dyimg + ra * (SG * 2) + col * 2, dyimg + rb * (SG * 2) + col * 2, lane);
      const PixGeo ga = pix_geo(p, m0 + ra, R_cur);
      const PixGeo gb = pix_geo(p, m0 + rb, R_cur);
      const bool oka = m0 + ra <= m1, okb = m0 + rb <= m1;
      const int bcol = (chh * 16 + 4 * pp) * 2;
      if constexpr (K33) {
        // 3x3: the source pixel of tap t is base + toff[t] (uniform offsets), valid where bit t
        // of a per-pixel mask is set -- built once from three row and three column tests instead
        // of nine full bounds checks and index products per pixel
        const uint32_t ma = oka ? tap_mask33(p, ga) : 0u, mb = okb ? tap_mask33(p, gb) : 0u;
        const int ba = (1 + (ga.rb + ga.yy) * p.Ws + ga.xx) * (SG * 2) + bcol;
        const int bb = (1 + (gb.rb + gb.yy) * p.Ws + gb.xx) * (SG * 2) + bcol;
#pragma unroll
        for (int t = 0; t < GT; ++t) {
          const int ia = (ma >> t) & 1u ? ba + toff[t] : bcol;
          const int ib = (mb >> t) & 1u ? bb + toff[t] : bcol;
          const bf16x8 bf = tr8(img + ia, img + ib, lane);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[t], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < GT; ++t) {
          if (t >= p.T) continue;  // uniform
          const int ia = oka ? tap_idx(p, ga, toh[t], tow[t], tok[t]) : 0;
          const int ib = okb ? tap_idx(p, gb, toh[t], tow[t], tok[t]) : 0;
          const bf16x8 bf = tr8(img + ia * (SG * 2) + bcol, img + ib * (SG * 2) + bcol, lane);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[t], 0, 0, 0);
        }
      }
    }
    if (p.nbuf == 1 && ci + 1 < nchunks) {
      __syncthreads();
      R_next = issue(m0 + GP, smem);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    R_cur = R_next;
  }

  // D tile (row tile rt, column half chh, tap t): lane holds column c = chh*16 + (lane&15),
  // rows j = rt*16 + (lane>>4)*4 + r.  Waves that split the k-steps are summed in LDS.
  float* part = p.part + (size_t)split * p.C * p.T * p.CG;
  const int c = chh * 16 + (lane & 15);
  if (KSPLIT > 1) {
    float* red = (float*)smem;  // [KSPLIT][GT][64][4]
#pragma unroll
    for (int t = 0; t < GT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((kslot * GT + t) * 64 + lane) * 4 + r] = acc[t][r];
    __syncthreads();
    if (kslot != 0) return;
#pragma unroll
    for (int t = 0; t < GT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
        for (int k = 0; k < KSPLIT; ++k) s += red[((k * GT + t) * 64 + lane) * 4 + r];
        acc[t][r] = s;
      }
  }
#pragma unroll
  for (int t = 0; t < GT; ++t) {
    if (t >= p.T) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = rt * 16 + (lane >> 4) * 4 + r;
      if (j / p.CG != c / p.CG) continue;
      part[((size_t)(sg * SG + j) * p.T + t) * p.CG + (c % p.CG)] = acc[t][r];
    }
  }
}

__global__ void partial_reduce_kernel(const float* __restrict__ part, int splits, int n, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  int k = 0;
  for (; k + 4 <= splits; k += 4)
    s += (part[(size_t)k * n + i] + part[(size_t)(k + 1) * n + i]) +
         (part[(size_t)(k + 2) * n + i] + part[(size_t)(k + 3) * n + i]);
  for (; k < splits; ++k) s += part[(size_t)k * n + i];
  out[i] = s;
}

// --- host side ------------------------------------------------------------
int pick_sg(int C, int CG) {
  if (CG <= 16 && 16 % CG == 0 && C % 16 == 0) return 16;
  if (CG == 32 && C % 32 == 0) return 32;
  return 0;
}

// weight-gradient super-group: pick_sg's, or 32 channels with g_tune[kGconvSG] = 32 (A/B only: the
// 32-channel block-diagonal tiles measured 8% slower on ResNeXt-50, 8.6k vs 9.4k img/s at b512)
int wgrad_sg(int C, int CG) {
  const int base = pick_sg(C, CG);
  if (base != 0 && g_tune[kGconvSG] == 32 && CG <= 32 && 32 % CG == 0 && C % 32 == 0) return 32;
  return base;
}

GconvParams make_params(int Hs, int Ws, int Hd, int Wd, int N, int C, int CG, int KH, int KW, int ss, int sd,
                        const int* oh, const int* ow) {
  GconvParams p{};
  p.Hs = Hs;
  p.Ws = Ws;
  p.Hd = Hd;
  p.Wd = Wd;
  p.C = C;
  p.CG = CG;
  p.T = KH * KW;
  p.ss = ss;
  p.sd = sd;
  p.M = N * Hd * Wd;
  p.div_wd = make_fastdiv(Wd);
  p.div_hd = make_fastdiv(Hd);
  p.ohmin = 1 << 30;
  p.ohmax = -(1 << 30);
  for (int t = 0; t <= GT; ++t) {
    p.oh[t] = t < p.T ? (int8_t)oh[t] : 0;
    p.ow[t] = t < p.T ? (int8_t)ow[t] : 0;
  }
  for (int t = 0; t < p.T; ++t) {
    p.ohmin = std::min(p.ohmin, oh[t]);
    p.ohmax = std::max(p.ohmax, oh[t]);
  }
  return p;
}

// exact max halo rows over all 256-pixel blocks (cached per geometry)
int max_halo_rows(const GconvParams& p, int N) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int, int>, int> cache;
  const auto key = std::make_tuple(N, p.Hs, p.Ws, p.Hd, p.Wd, p.ss, p.sd, p.ohmin, p.ohmax);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  auto fl = [&](int v) { return p.sd == 1 ? v : (v >= 0 ? v / 2 : -((-v + 1) / 2)); };
  int best = 1;
  for (int m0 = 0; m0 < p.M; m0 += GP) {
    const int m1 = std::min(p.M, m0 + GP) - 1;
    const int q0 = m0 / p.Wd, q1 = m1 / p.Wd;
    const int n0 = q0 / p.Hd, n1 = q1 / p.Hd;
    const int y0 = q0 - n0 * p.Hd, y1 = q1 - n1 * p.Hd;
    const int rlo = std::max(0, fl(y0 * p.ss + p.ohmin));
    const int rhi = std::min(p.Hs - 1, fl(y1 * p.ss + p.ohmax));
    best = std::max(best, n1 * p.Hs + rhi - (n0 * p.Hs + rlo) + 1);
  }
  cache[key] = best;
  return best;
}

template <typename K>
void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024) hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

constexpr size_t kMaxLds = 160 * 1024;

template <int SG, bool DGRAD>
bool launch_gather(GconvParams p, int N, bf16* frag, hipStream_t s) {
  constexpr int TPS = SG == 16 ? 2 : 1;
  p.nsg = p.C / SG;
  const int npb = (p.M + GP - 1) / GP;
  p.ntiles = npb * p.nsg;
  const size_t lds = (size_t)(1 + max_halo_rows(p, N) * p.Ws) * SG * 2;
  if (lds > kMaxLds) return false;
  const int nfrag = p.nsg * ((p.T + TPS - 1) / TPS) * (SG / 16) * 64;
  hipLaunchKernelGGL((gconv_frag_kernel<SG, DGRAD>), dim3((nfrag + 255) / 256), dim3(256), 0, s, p, frag);
  p.wfrag = frag;
  // super-groups per workgroup (g_tune gconv_spw = spw, or 10 * spw + LDS ring buffers).  Default
  // (tools/conv_bench.py --grouped --cfgs, b1024, profiles/r5/gconv_spw_ab_b1024.txt): two 16-channel
  // super-groups with a two-stage ring where the source is read at stride 1 (-21 % fwd, -16 % dgrad
  // over ResNeXt-50's grouped convs); one per workgroup for the stride-2 forward (its doubled halo
  // halves the occupancy of the ring) and for 32-channel super-groups (twice the fragments and
  // accumulators; no gain measured)
  int spw = g_tune[kGconvSpw], nbuf = 2;
  const bool multi1 = spw >= 10 && spw / 10 == 1;  // 11: the multi kernel with one super-group (A/B)
  if (spw >= 10) {
    nbuf = std::max(2, spw % 10);
    spw /= 10;
  }
  if (spw <= 0) spw = (SG == 16 && p.ss == 1 && (size_t)npb * ((p.nsg + 1) / 2) >= 512) ? 2 : 1;
  spw = std::min(spw, p.nsg);
  if ((spw > 1 || multi1) && p.T == GT) {
    const size_t fragb = (size_t)(nfrag / p.nsg) * 16;
    const size_t bnb = (DGRAD && p.bnz) ? (size_t)GP * SG * 2 + 4 * SG * 4 : 0;
    const size_t bufb = (fragb + bnb + lds + 15) / 16 * 16;
    nbuf = std::min(nbuf, spw);
    const size_t total = nbuf * bufb + 4 * SG * 16;
    if (total <= kMaxLds) {
      p.spw = spw;
      p.nbuf_g = nbuf;
      p.ablate = g_tune[kAblate];
      p.bufb_g = (int)bufb;
      p.ntiles = npb * ((p.nsg + spw - 1) / spw);
      allow_lds(gconv_gather_multi_kernel<SG, DGRAD>, total);
      hipLaunchKernelGGL((gconv_gather_multi_kernel<SG, DGRAD>), dim3(p.ntiles), dim3(256), total, s, p);
      return true;
    }
  }
  allow_lds(gconv_gather_kernel<SG, DGRAD>, lds);
  hipLaunchKernelGGL((gconv_gather_kernel<SG, DGRAD>), dim3(p.ntiles), dim3(256), lds, s, p);
  return true;
}

}  // namespace

int gconv_frag_elems(int C, int G, int KH, int KW) {
  const int SG = pick_sg(C, C / G);
  if (SG == 0 || KH * KW > GT) return 0;
  const int TPS = SG == 16 ? 2 : 1;
  return (C / SG) * ((KH * KW + TPS - 1) / TPS) * (SG / 16) * 64 * 8;
}

int gconv_fwd_stat_blocks(int M) { return (M + GP - 1) / GP; }

bool launch_gconv_mfma_fwd(const bf16* x, const bf16* w, bf16* y, bf16* frag, int N, int H, int W, int C, int Ho,
                           int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s,
                           float* stats) {
  const int CG = C / G;
  const int SG = pick_sg(C, CG);
  if (SG == 0 || Co != C || KH * KW > GT || frag == nullptr) return false;
  int oh[GT], ow[GT];
  for (int t = 0; t < KH * KW; ++t) {
    oh[t] = t / KW - pad;
    ow[t] = t % KW - pad;
  }
  GconvParams p = make_params(H, W, Ho, Wo, N, C, CG, KH, KW, stride, 1, oh, ow);
  p.src = x;
  p.w = w;
  p.dst = y;
  p.stats = stats;
  return SG == 16 ? launch_gather<16, false>(p, N, frag, s) : launch_gather<32, false>(p, N, frag, s);
}

bool launch_gconv_mfma_dgrad(const bf16* dy, const bf16* w, bf16* dx, bf16* frag, int N, int H, int W, int C, int Ho,
                             int Wo, int Co, int G, int KH, int KW, int stride, int pad, hipStream_t s,
                             const GconvBnBwd* bn) {
  const int CG = C / G;
  const int SG = pick_sg(C, CG);
  if (SG == 0 || Co != C || KH * KW > GT || stride > 2 || frag == nullptr) return false;
  int oh[GT], ow[GT];
  for (int t = 0; t < KH * KW; ++t) {
    oh[t] = pad - t / KW;
    ow[t] = pad - t % KW;
  }
  GconvParams p = make_params(Ho, Wo, H, W, N, C, CG, KH, KW, 1, stride, oh, ow);
  p.src = dy;
  p.w = w;
  p.dst = dx;
  if (bn) {
    p.bnz = bn->z;
    p.bn_scale = bn->scale;
    p.bn_shift = bn->shift;
    p.bn_mean = bn->mean;
    p.bn_invstd = bn->invstd;
    p.bnsum = bn->part;
  }
  return SG == 16 ? launch_gather<16, true>(p, N, frag, s) : launch_gather<32, true>(p, N, frag, s);
}

int gconv_mfma_wgrad_splits(int N, int Ho, int Wo, int C, int G) {
  const int SG = wgrad_sg(C, C / G);
  if (SG == 0) return 0;
  const int M = N * Ho * Wo;
  const int nsg = C / SG;
  const int chunks = (M + GP - 1) / GP;
  int splits = std::max(1, 2048 / nsg);
  splits = std::min(splits, chunks);
  const int cps = (chunks + splits - 1) / splits;  // chunks per split
  return (chunks + cps - 1) / cps;
}

bool launch_gconv_mfma_wgrad(const bf16* dy, const bf16* x, float* dw, float* part, int splits, const bf16* zero,
                             int N, int H, int W, int C, int Ho, int Wo, int Co, int G, int KH, int KW, int stride,
                             int pad, hipStream_t s) {
  const int CG = C / G;
  const int SG = wgrad_sg(C, CG);
  if (SG == 0 || Co != C || KH * KW > GT || splits <= 0) return false;
  int oh[GT], ow[GT];
  for (int t = 0; t < KH * KW; ++t) {
    oh[t] = t / KW - pad;
    ow[t] = t % KW - pad;
  }
  GconvParams p = make_params(H, W, Ho, Wo, N, C, CG, KH, KW, stride, 1, oh, ow);
  p.src = x;
  p.dy = dy;
  p.part = part;
  p.zero = zero;
  p.nsg = C / SG;
  const int chunks = (p.M + GP - 1) / GP;
  const int cps = (chunks + splits - 1) / splits;
  p.rows_per_split = cps * GP;  // chunk starts stay multiples of GP (the halo bound's blocks)
  p.ntiles = splits * p.nsg;
  const size_t bufb = ((size_t)GP * SG * 2 + (size_t)(1 + max_halo_rows(p, N) * p.Ws) * SG * 2 + 15) / 16 * 16;
  const size_t red = (size_t)(4 / ((SG / 16) * (SG / 16))) * GT * 64 * 4 * 4;
  p.bufb = (int)bufb;
  p.nbuf = (2 * bufb <= kMaxLds && cps > 1) ? 2 : 1;
  const size_t lds = std::max(p.nbuf * bufb, red);
  if (lds > kMaxLds) return false;
  const bool k33 = KH == 3 && KW == 3 && g_tune[kGconvSG] != 1;  // gconv_sg=1: the general tap path (A/B)
  auto launch = [&](auto kernel) {
    allow_lds(kernel, lds);
    hipLaunchKernelGGL(kernel, dim3(p.ntiles), dim3(256), lds, s, p);
  };
  if (SG == 16)
    k33 ? launch(gconv_wgrad_kernel<16, true>) : launch(gconv_wgrad_kernel<16, false>);
  else
    k33 ? launch(gconv_wgrad_kernel<32, true>) : launch(gconv_wgrad_kernel<32, false>);
  const int n = C * KH * KW * CG;
  hipLaunchKernelGGL(partial_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, splits, n, dw);
  return true;
}

}  // namespace dcp
