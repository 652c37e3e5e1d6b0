// MFMA implicit-GEMM convolution for gfx950 (CDNA4), NHWC bf16, fp32 accumulate.
//
// Replaces the cuDNN convolutions the reference gets implicitly from
// torchvision/timm ResNets (kernels K1/K2/K3;
// reference model code: NESTED/model/imagenet_resnet.py:27,68-73,107,134).
//
// One "tap GEMM" kernel covers forward and data-gradient passes:
//
//   dst[n, y*ds+oy, x*ds+ox, co] = sum_t sum_c src[n, y*ss+dy_t, x*ss+dx_t, c] * wt[co, widx_t, c]
//
//   * forward, stride s, pad p:  ss = s, dy_t = kh - p, ds = 1, widx_t = kh*KW+kw
//   * dgrad, stride 1:           src = dY, wt = W^T ([Ci][T][Co]), dy_t = p - kh
//   * dgrad, stride 2:           one launch per output parity class (sub-pixel
//                                decomposition), ds = 2, only the taps whose
//                                parity matches; a class with no taps writes 0.
//
// GEMM view: rows m = (n, y, x) of the output grid, columns = output
// channels, K = taps x channels in 8-channel (16-byte) chunks.  Tiles are
// staged global->LDS with `global_load_lds_dwordx4` (LDS-DMA, no VGPR
// round trip); out-of-bounds / padding taps point the lane at a zero page so
// the gather needs no branches.  The weight-gradient kernels issue it untracked
// (dma16, common.cuh: exact lgkmcnt waits for their fragment prefetch, 10-15 %
// faster); the forward / data-gradient families keep the compiler-tracked builtin
// (dma16_tracked), which measured 1 % faster for them (profiles/r4/dma_untracked_ab.txt).  LDS rows are XOR-swizzled on the source
// address so the MFMA fragment reads (`ds_read_b128`) are bank-conflict free.
// The MFMA is v_mfma_f32_16x16x32_bf16 with the weight as the A operand, so
// each lane ends up owning 4 consecutive output channels of one pixel
// (8-byte stores) and per-channel BN statistics reduce with 4 shuffles.
//
// The weight-gradient kernel computes dW[co][t][c] = sum_m dY[m][co] * im2col(X)[m][t,c]
// with both operands m-major in memory; its LDS images are [m][...] rows read
// with the gfx950 transpose read `ds_read_b64_tr_b16`, split-K over m with
// fp32 atomics into the (zeroed) gradient.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

int g_tune[kTuneSlots] = {0};
// stream-ordered device workspace (the framework registers PyTorch's caching allocator: capture-safe,
// freed blocks reused only by later work on the same stream)
static WorkspaceAlloc g_ws_alloc = nullptr;
static WorkspaceFree g_ws_free = nullptr;
void set_workspace_allocator(WorkspaceAlloc a, WorkspaceFree f) {
  g_ws_alloc = a;
  g_ws_free = f;
}

struct TapGemmParams {
  const bf16* src;   // [N][Hs][Ws][Cs]
  const bf16* wt;    // [Co][T][Cs]
  bf16* dst;         // [N][Hd][Wd][Co]
  float* stats;      // [ceil(M/128)][2][Co] per-128-row slab (mean, M2) or nullptr
  const bf16* zero;  // >= 16 bytes of zeros
  int Hs, Ws, Cs;
  int Hy, Wy, ss;
  int Hd, Wd, ds, oy, ox;
  int Co, T, M;
  int ntaps, cpt, nkt, ldw;
  int relu;          // fused activation on the stored output: 0 none, 1 ReLU, 2 sigmoid (linear heads)
  const float* bias; // optional per-output-channel bias (linear heads)
  int nbias;         // bias entries (channels past it add 0: an unpadded bias of a padded GEMM)
  const bf16* addsrc;  // optional: added to the stored output (same layout as dst; fused residual-gradient sum)
  FastDiv div_wy, div_hy, div_cpt;
  // per tap: dy (int8) | dx (int8) << 8 | weight tap index << 16.  Dword entries so a
  // wave-uniform lookup is one s_load_dword (byte arrays compile to vector loads, whose
  // vmcnt wait would drain the LDS-DMA ring).
  int tap[kMaxTaps];
  int ablate;  // tuning experiments only: 1 = no staging in the k-loop, 2 = no MFMA, 4 = no epilogue (big tile)
  int cvar;    // tuning experiments only: compute-loop variant
  // EPI 3 (stride-1 dgrad): backward of the BN(+ReLU)(+residual) layer that produced this
  // conv's input, fused into the epilogue (see launchers.h BnBwdEpi)
  BnBwdEpi bnb;
  // EPI 0: eval-mode BN folded into the store (launchers.h AffineEpi); fscale == nullptr: off
  const float* fscale;
  const float* fshift;
  int fact;
  float fslope;
  // PRO (1x1 / stride-1 FAST shapes): the A operand is a training-mode BN's INPUT, normalised
  // and ReLU'd in registers between the LDS fragment read and the MFMA,
  // a = bf16(relu(x * pscale[c] + pshift[c])) -- the BN + ReLU output is never written (K5)
  const float* pscale;
  const float* pshift;
  int persist;  // big tile: 1 = persistent workgroups (g_tune[kTgBigPersist])
  // big tile, stream-K (sk_ws != nullptr): the grid's workgroups split the tiles' k-steps evenly;
  // a tile cut between workgroups g and g+1 is finished by g, which adds g+1's fp32 partial
  // (slot g+1 of sk_ws, published by sk_flags[g+1]) before the epilogue.  Flags zeroed per launch.
  f32x4* sk_ws;
  uint32_t* sk_flags;
  int sk_on;  // host side: stream-K requested for this launch (launch_big allocates sk_ws / sk_flags)
  int sk_unit;  // stream-K range granularity in k-steps (divides nkt)
  // 128-row kernel split-K (short grids with deep k-loops: small batches).  kmode 1: workgroup
  // (x, y) runs k-tiles [nkt y / ksplit, nkt (y+1) / ksplit) of tile x and stores its raw fp32
  // accumulators to kp; kmode 2: workgroup x sums tile x's ksplit slices in slice order and runs the
  // epilogue (every EPI) on them.  0: off.
  // slices are cut in 64-deep k units (k64 of them), so every tile width / k depth sums the same slices
  f32x4* kp;
  int ksplit, kmode, k64;
};

__device__ __forceinline__ int tap_dy(int v) { return (int)(int8_t)(v & 0xff); }
__device__ __forceinline__ int tap_dx(int v) { return (int)(int8_t)((v >> 8) & 0xff); }
__device__ __forceinline__ int tap_w(int v) { return (v >> 16) & 0xffff; }

// byte offset of logical 16B chunk `c` of row `r` in a 128-byte-row image
__device__ __forceinline__ uint32_t swz128(uint32_t r, uint32_t c) {
  return r * 128u + ((c ^ ((r >> 1) & 7u)) << 4);
}
// k-tile images of BK bf16 per row: 128-byte rows (BK = 64) or 64-byte rows (BK = 32); the
// XOR of the chunk with row bits 1.. makes the 16x16x32 fragment reads (ds_read_b128, 16-lane
// groups over 16 rows) bank-conflict free in both
template <int BK>
__device__ __forceinline__ uint32_t swz_chunk(uint32_t r) {
  return BK == 64 ? ((r >> 1) & 7u) : ((r >> 1) & 3u);
}
template <int BK>
__device__ __forceinline__ uint32_t swzk(uint32_t r, uint32_t c) {
  return r * (BK * 2u) + ((c ^ swz_chunk<BK>(r)) << 4);
}

// Epilogue image E[rows][BN] bf16: 16-byte chunks XOR-swizzled by row>>1, and the two 8-byte
// halves of a chunk swapped on odd rows, so the accumulator writes (ds_write_b64, 16 lanes = 16
// consecutive rows of one 8-byte half) hit 16 distinct bank slots and the row-chunk reads
// (ds_read_b128) stay conflict free.  eimg_off8: byte offset of the 4 channels cl..cl+3 of row pl.
template <int NCH>
__device__ __forceinline__ uint32_t eimg_off8(uint32_t pl, uint32_t cl) {
  return pl * (NCH * 16) + (((cl >> 3) ^ ((pl >> 1) & (NCH - 1))) << 4) + ((((cl >> 2) & 1) ^ (pl & 1)) << 3);
}
// the 8 channels of chunk c of row pl, in channel order
template <int NCH>
__device__ __forceinline__ bf16x8 eimg_chunk(const char* E, uint32_t pl, uint32_t c) {
  const bf16x8 v = *LDS_PTR(const bf16x8, E + pl * (NCH * 16) + ((c ^ ((pl >> 1) & (NCH - 1))) << 4));
  return (pl & 1) ? bf16x8{v[4], v[5], v[6], v[7], v[0], v[1], v[2], v[3]} : v;
}

// (mean, M2) per channel of the 128-row slab of the LDS output image E (bf16-rounded outputs),
// for BM = 128: thread (chunk c = tid % NCH, row group g = tid / NCH) reads whole 16-byte row
// chunks (8 channels) of rows g, g + G, ...; sums of (v - K) and (v - K)^2 with K = the slab's
// row 0 (one shift per channel for every thread, so the partial sums add) -> wave shuffles ->
// LDS behind row 7 of the image -> one thread per channel.  Replaces 64 two-byte reads and a
// two-pass per thread (tile_stats) with 8 (BN = 128) or 4 (BN = 64) chunk reads.
// vv: this thread's image chunks (chunk tid % NCH of rows tid / NCH + G k), already in registers
// from the store pass (tg_image_store reads exactly these) -- the image is not read twice
template <int BN>
__device__ __forceinline__ void tile_stats128_vv(const TapGemmParams& p, char* E, int m0, int n0, int tid,
                                                 const bf16x8 (&vv)[128 / (256 / (BN / 8))]) {
  constexpr int NCH = BN / 8, G = 256 / NCH, RPT = 128 / G, RB = BN * 2;
  const int c = tid % NCH, g = tid / NCH, lane = tid & 63, wave = tid >> 6;
  const int nvalid = min(128, p.M - m0);
  float K[8], s1[8], s2[8];
  {
    const bf16x8 v = eimg_chunk<NCH>(E, 0, c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      K[e] = bf2f(v[e]);
      s1[e] = s2[e] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k)
    if (g + G * k < nvalid)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = bf2f(vv[k][e]) - K[e];
        s1[e] += d;
        s2[e] = fmaf(d, d, s2[e]);
      }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] = xor_sum_from<NCH>(s1[e]);
    s2[e] = xor_sum_from<NCH>(s2[e]);
  }
  __syncthreads();  // every image read (stores, rows above) is done: rows 8.. become scratch
  float* xch = (float*)(E + 8 * RB);  // [4 waves][2][BN]
  if (lane < NCH)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xch[(wave * 2 + 0) * BN + c * 8 + e] = s1[e];
      xch[(wave * 2 + 1) * BN + c * 8 + e] = s2[e];
    }
  __syncthreads();
  // (nvalid <= 0: a 128-row quadrant of a 256-row tile past M -- no slab to write)
  if (tid < BN && n0 + tid < p.Co && nvalid > 0) {
    float S1 = 0.f, S2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      S1 += xch[(w * 2 + 0) * BN + tid];
      S2 += xch[(w * 2 + 1) * BN + tid];
    }
    const float k0 = bf2f(eimg_chunk<NCH>(E, 0, tid >> 3)[tid & 7]);
    const float n = (float)nvalid;
    const size_t rb = (size_t)(m0 / 128);
    p.stats[(rb * 2 + 0) * p.Co + n0 + tid] = k0 + S1 / n;
    p.stats[(rb * 2 + 1) * p.Co + n0 + tid] = fmaxf(S2 - S1 * S1 / n, 0.f);
  }
}

// vmcnt(n) with a wave-uniform runtime n in [0, 31] (a scalar branch to an immediate wait)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int BN, int EPI>
__device__ __forceinline__ void tg_image_store(const TapGemmParams& p, char* E, int m0, int n0, int tid);

// Store epilogue of the 4-wave 128-row tap GEMMs (EPI 0: bf16 store, optionally folding an
// eval-mode BN and adding addsrc; EPI 1: + the per-128-row BN statistics).  Entered after a
// barrier with no loads in flight; the accumulators go through the LDS image E.
template <int BN, int EPI>
__device__ __forceinline__ void tg_store_epilogue(const TapGemmParams& p, const f32x4 (&acc)[BN / 32][4], char* smem,
                                                  int m0, int n0, int tid, int lane, int wm, int wn) {
  constexpr int BM = 128, TN = BN / 32;
  // ---- epilogue through LDS: the k-loop ended with a barrier and no loads in flight ----
  // tile image E[BM pixels][BN channels] bf16, 16-byte chunks XOR-swizzled by (pixel>>1)
  constexpr int NCH = BN / 8;
  char* E = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t pl = wm * 64 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const uint32_t cl = wn * (BN / 2) + j * 16 + (lane >> 4) * 4;
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[j][i][r]);
      const uint32_t off = eimg_off8<NCH>(pl, cl);
      *LDS_PTR(bf16x4, E + off) = o;
    }
  }
  __syncthreads();
  tg_image_store<BN, EPI>(p, E, m0, n0, tid);
}

// The image -> global half of the store epilogue, for 256 threads over one [128][BN] image E
// (tg_store_epilogue, and per 128 x 128 quadrant in tap_gemm_big_kernel): coalesced 16-byte
// stores, the optional eval-BN fold / add source, then (EPI 1) the slab's BN statistics.
template <int BN, int EPI>
__device__ __forceinline__ void tg_image_store(const TapGemmParams& p, char* E, int m0, int n0, int tid) {
  constexpr int BM = 128, NCH = BN / 8;
  // coalesced 16-byte stores: a pass covers 256/NCH pixel rows x all BN channels.  All the
  // thread's image chunks are read first, so its stores issue back to back instead of each
  // waiting for its own LDS read.
  {
    constexpr int R = 256 / NCH;
    const int c = tid % NCH, pr0 = tid / NCH;
    const bool cok = n0 + c * 8 < p.Co;
    float fsc[8], fsh[8];
    const bool fold = EPI == 0 && p.fscale != nullptr;
    if (fold) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        fsc[e] = cok ? p.fscale[n0 + c * 8 + e] : 0.f;
        fsh[e] = cok ? p.fshift[n0 + c * 8 + e] : 0.f;
      }
    }
    bf16x8 vv[BM / R];
#pragma unroll
    for (int k = 0; k < BM / R; ++k) vv[k] = eimg_chunk<NCH>(E, pr0 + k * R, c);
#pragma unroll
    for (int k = 0; k < BM / R; ++k) {
      const int pl = pr0 + k * R;
      const int m = m0 + pl;
      const bf16x8 v = vv[k];
      if (m < p.M && cok) {
        size_t drow;  // element offsets pass 2^32 at large batch (56x56x256 rows: N > 5,350)
        if (p.ds == 1) {
          drow = (size_t)m * (size_t)p.Co;
        } else {
          const uint32_t q = fdiv(m, p.div_wy);
          const uint32_t x = m - q * p.Wy;
          const uint32_t n = fdiv(q, p.div_hy);
          const uint32_t y = q - n * p.Hy;
          drow = (size_t)((n * p.Hd + y * p.ds + p.oy) * p.Wd + x * p.ds + p.ox) * (size_t)p.Co;
        }
        bf16x8 o = v;
        if (fold) {
          // the bf16 conv output through the unfused BN-apply's fp32 math (bn_act_fwd_kernel)
          bf16x8 a{};
          if (p.addsrc) a = *(const bf16x8*)(p.addsrc + drow + n0 + c * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float t = bf2f(v[e]) * fsc[e] + fsh[e];
            if (p.addsrc) t += bf2f(a[e]);
            if (p.fact == 1) t = fmaxf(t, 0.f);
            else if (p.fact == 2) t = t >= 0.f ? t : t * p.fslope;
            o[e] = f2bf(t);
          }
        } else if (p.addsrc) {
          const bf16x8 a = *(const bf16x8*)(p.addsrc + drow + n0 + c * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(v[e]) + bf2f(a[e]));
        }
        *(bf16x8*)(p.dst + drow + n0 + c * 8) = o;
      }
    }
    // the statistics of the bf16 outputs, from the chunks this pass already holds
    if constexpr (EPI == 1) tile_stats128_vv<BN>(p, E, m0, n0, tid, vv);
  }
}

// EPI: 0 = bf16 store, 1 = store + per-64-row BN statistics, 2 = bias / activation (linear heads)
// FAST: Cs % 64 == 0, one tap per 64-deep k-tile
// NS: LDS stages.  NS = 2: double buffer, vmcnt(0) + barrier per k-tile (several blocks per
// CU hide the latency).  NS > 2 (FAST only): a ring whose LDS-DMA loads stay in flight across
// the raw s_barrier, drained by a counted vmcnt -- for deep-K shapes at one block per CU.
// three waves per SIMD: the fused BN-backward epilogue otherwise lands one register past the
// 168-register step and halves to two workgroups per CU
template <int BN, int EPI, bool FAST, int NS = 2, int BK = 64, bool PRO = false, bool KS = false>
__global__ void __launch_bounds__(256, 3)
tap_gemm_kernel(const TapGemmParams p) {
  static_assert(NS == 2 || FAST, "the LDS ring needs the one-tap-per-k-tile path");
  static_assert(!PRO || (FAST && NS == 2 && EPI < 2), "the BN prologue: FAST double-buffered forward only");
  static_assert(BK == 64 || BK == 32, "k-tile depth");
  constexpr int BM = 128;                 // pixel rows per block
  constexpr int ROWB = BK * 2;            // bytes per image row (BK bf16)
  constexpr int CH = BK / 8;              // 16-byte chunks per row
  constexpr int RPI = 64 / CH;            // image rows per LDS-DMA wave instruction
  constexpr int AI = BM / (4 * RPI);      // A-image LDS-DMA instructions per thread per k-tile
  constexpr int A_BYTES = BM * ROWB;
  constexpr int B_BYTES = BN * ROWB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int TN = BN / 32;             // 16-wide co subtiles per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // wave-uniform in an SGPR: the LDS-DMA destinations derived from it need no readfirstlane
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const uint32_t ntn = (p.Co + BN - 1) / BN;
  const uint32_t ntm = (p.M + BM - 1) / BM;
  const uint32_t bid = xcd_remap(blockIdx.x, ntm * ntn);
  const uint32_t tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- FAST path: per-slot source pointers and tap-validity masks, computed once ----
  // A k-tile's load is then ptr + a wave-uniform tap offset, selected against the zero page
  // by one mask bit: ~3 vector instructions per LDS-DMA instead of ~12 (the k-loop was
  // vector-issue bound on this address arithmetic).  Rows past M / channels past Co read a
  // clamped valid row: their outputs are never stored nor counted in the statistics.
  const bf16* fa_ptr[AI];
  uint32_t fa_vm[AI];
  const bf16* fb_ptr[BN / (4 * RPI)];
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = (wave * AI + i) * RPI + lane / CH;
      const uint32_t mm = (uint32_t)min(m0 + r, p.M - 1);
      const uint32_t q = fdiv(mm, p.div_wy);
      const uint32_t x = mm - q * p.Wy;
      const uint32_t n = fdiv(q, p.div_hy);
      const uint32_t y = q - n * p.Hy;
      const int ys = y * p.ss, xs = x * p.ss;
      fa_ptr[i] = p.src + ((size_t)n * p.Hs * p.Ws + (size_t)ys * p.Ws + xs) * p.Cs +
                  ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
      uint32_t vm = 0;
      for (int t = 0; t < p.ntaps; ++t) {
        const int tv = p.tap[t];
        const int hi = ys + tap_dy(tv), wi = xs + tap_dx(tv);
        vm |= ((unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws) ? (1u << t) : 0u;
      }
      fa_vm[i] = vm;
    }
#pragma unroll
    for (int i = 0; i < BN / (4 * RPI); ++i) {
      const int r = (wave * (BN / (4 * RPI)) + i) * RPI + lane / CH;
      fb_ptr[i] = p.wt + (size_t)min(n0 + r, p.Co - 1) * p.ldw + ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
    }
  }

  // ---- per-thread A-load rows (AI glds per k-tile) ----
  uint32_t a_pix[AI];   // n*Hs*Ws
  int a_ys[AI], a_xs[AI];
  uint32_t a_chunk[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wave * AI + i) * RPI + lane / CH;
    const int m = m0 + r;
    a_ok[i] = m < p.M;
    const uint32_t mm = a_ok[i] ? m : 0;
    const uint32_t q = fdiv(mm, p.div_wy);
    const uint32_t x = mm - q * p.Wy;
    const uint32_t n = fdiv(q, p.div_hy);
    const uint32_t y = q - n * p.Hy;
    a_pix[i] = n * (uint32_t)(p.Hs * p.Ws);
    a_ys[i] = y * p.ss;
    a_xs[i] = x * p.ss;
    a_chunk[i] = (lane % CH) ^ swz_chunk<BK>(r);
  }
  // ---- per-thread B-load rows ----
  constexpr int BI = BN / (4 * RPI);  // glds per thread for B
  uint32_t b_row[BI];
  uint32_t b_chunk[BI];
  bool b_ok[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (wave * BI + i) * RPI + lane / CH;
    b_ok[i] = (n0 + r) < p.Co;
    b_row[i] = (uint32_t)(n0 + r) * p.ldw;
    b_chunk[i] = (lane % CH) ^ swz_chunk<BK>(r);
  }

  const int tiles_per_tap = p.cpt / CH;
  const int kc_total = p.ntaps * p.cpt;
  // Narrow-channel path: a lane's tap index varies per lane, and a per-lane lookup in the
  // kernel arguments is a vector memory load whose wait would drain the LDS-DMA ring every
  // k-tile.  The table is copied once into LDS behind the stages instead (lgkm counter).
  const int* tap_lds = (const int*)(smem + NS * STAGE);
  if constexpr (!FAST) {
    if (tid < p.ntaps) *LDS_PTR(int, smem + NS * STAGE + tid * 4) = p.tap[tid];
    __syncthreads();
  }
  // PRO: the per-channel (scale, shift) table behind the stages the k-loop uses, fp32 [2][Cs]
  // (one tap: k-tile kt covers channels kt*BK ..); made visible by the barrier after stage 0
  float* pro_tbl = (float*)(smem + min(NS, max(p.nkt, 1)) * STAGE);
  if constexpr (PRO) {
    for (int i = tid; i < p.Cs; i += 256) {
      pro_tbl[i] = p.pscale[i];
      pro_tbl[p.Cs + i] = p.pshift[i];
    }
  }

  auto stage = [&](int kt, int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
    if constexpr (FAST) {
      const int t = kt / tiles_per_tap;
      const int cbase = (kt - t * tiles_per_tap) * BK;
      const int tv = p.tap[t];
      const long aoff = (long)(tap_dy(tv) * p.Ws + tap_dx(tv)) * p.Cs + cbase;  // wave-uniform
      const long boff = (long)tap_w(tv) * p.Cs + cbase;
      const uint32_t tbit = 1u << t;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bf16* g = (fa_vm[i] & tbit) ? fa_ptr[i] + aoff : p.zero;
        dma16_tracked(g, As + (wave * AI + i) * 1024);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i)
        dma16_tracked((fb_ptr[i] + boff), Bs + (wave * BI + i) * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int kc = kt * CH + a_chunk[i];
        const int t = fdiv(kc, p.div_cpt);
        const int ci0 = (kc - t * p.cpt) * 8;
        bool ok = a_ok[i] && kc < kc_total;
        const int tv = *LDS_PTR(const int, tap_lds + (ok ? t : 0));
        const int hi = a_ys[i] + tap_dy(tv), wi = a_xs[i] + tap_dx(tv);
        ok = ok && (unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws;
        const bf16* g = ok ? p.src + (size_t)(a_pix[i] + hi * p.Ws + wi) * p.Cs + ci0 : p.zero;
        dma16_tracked(g, As + (wave * AI + i) * 1024);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const int kc = kt * CH + b_chunk[i];
        const int t = fdiv(kc, p.div_cpt);
        const int ci0 = (kc - t * p.cpt) * 8;
        const bool ok = b_ok[i] && kc < kc_total;
        const bf16* g =
            ok ? p.wt + b_row[i] + (uint32_t)tap_w(*LDS_PTR(const int, tap_lds + t)) * p.Cs + ci0 : p.zero;
        dma16_tracked(g, Bs + (wave * BI + i) * 1024);
      }
    }
  };

  f32x4 acc[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this workgroup's k-tiles [kb, kb + nkt) (split-K slice; none in the reduce launch)
  int kb = 0, nkt = p.nkt;
  if constexpr (KS) {  // (a separate instantiation: the split paths cost the others registers)
    if (p.kmode == 1) {
      constexpr int U = 64 / BK;  // k-tiles per 64-deep unit
      kb = (int)((long)p.k64 * blockIdx.y / p.ksplit) * U;
      nkt = min(p.nkt, (int)((long)p.k64 * (blockIdx.y + 1) / p.ksplit) * U) - kb;
    } else {
      nkt = 0;
    }
  }
  auto compute = [&](const char* As, const char* Bs, int kt) {
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const uint32_t c = s * 4 + (lane >> 4);
      bf16x8 wf[TN], af[4];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const uint32_t r = wn * (BN / 2) + j * 16 + (lane & 15);
        wf[j] = *(const bf16x8*)(Bs + swzk<BK>(r, c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t r = wm * 64 + i * 16 + (lane & 15);
        af[i] = *(const bf16x8*)(As + swzk<BK>(r, c));
      }
      if constexpr (PRO) {
        // the lane's 8 channels of this k-step: kt*BK + 8c .. +7 (fragment elements in order)
        const float* t = pro_tbl + kt * BK + c * 8;
        const f32x4 s0 = *LDS_PTR(const f32x4, t), s1 = *LDS_PTR(const f32x4, t + 4);
        const f32x4 h0 = *LDS_PTR(const f32x4, t + p.Cs), h1 = *LDS_PTR(const f32x4, t + p.Cs + 4);
        const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) af[i][e] = f2bf(fmaxf(bf2f(af[i][e]) * sc[e] + sh[e], 0.f));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
    }
  };
  if constexpr (NS == 2) {
    if (nkt > 0) {
      stage(kb, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int kt = 0; kt < nkt; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nkt && !(p.ablate & 1)) stage(kb + kt + 1, buf ^ 1);
      const char* As = smem + buf * STAGE;
      if (!(p.ablate & 2)) compute(As, As + A_BYTES, kb + kt);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    constexpr int LPT = AI + BI;  // LDS-DMA instructions per thread per k-tile
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
      if (i < nkt) stage(kb + i, i);
    for (int kt = 0; kt < nkt; ++kt) {
      // tiles issued after kt: kt+1 .. min(kt+NS-2, nkt-1)
      wait_vmcnt(LPT * min(NS - 2, nkt - 1 - kt));
      __builtin_amdgcn_s_barrier();  // tile kt landed for every wave; tile kt-1's slot is free
      asm volatile("" ::: "memory");
      if (kt + NS - 1 < nkt) stage(kb + kt + NS - 1, (kt + NS - 1) % NS);
      const char* As = smem + (kt % NS) * STAGE;
      compute(As, As + A_BYTES, kb + kt);
    }
    __syncthreads();
  }
  if constexpr (KS) {
   if (p.kmode == 1) {
    // split-K slice: raw accumulators, [slice][tile][j][i][thread] (16 bytes per lane, coalesced)
    f32x4* o = p.kp + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (TN * 4 * 256) + tid;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[(j * 4 + i) * 256] = acc[j][i];
    return;
   }
   // kmode 2: the slices of this tile in slice order (deterministic), one accumulator at a time (a
   // slice-outer loop keeps every slice's loads live at once and spills), then the epilogue below
    const f32x4* q = p.kp + (size_t)blockIdx.x * (TN * 4 * 256) + tid;
    const size_t sstride = (size_t)gridDim.x * (TN * 4 * 256);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4* qq = q + (j * 4 + i) * 256;
        f32x4 t = qq[0];
#pragma unroll 1
        for (int sl = 1; sl < p.ksplit; ++sl) t += qq[sl * sstride];
        acc[j][i] = t;
      }
  }

  if constexpr (EPI == 3 || EPI == 4) {
    // ---- dgrad + fused BN backward (stride 1: dst rows == GEMM rows) ----
    // EPI 4: the activation mask comes as bits (bn_act_mask) instead of being recomputed from
    // the BN input and the residual -- no residual rows, no scale/shift registers.
    constexpr bool MASKED = EPI == 4;
    constexpr int RB = BN * 2, NCH = BN / 8, R = 256 / NCH, RPT = BM / R;
    char* E = smem;
    const int c = tid % NCH, pr0 = tid / NCH;
    const int cg = n0 + c * 8;
    const bool cok = cg < p.Co;
    // accumulators -> LDS image first: the MFMA accumulators are dead before any epilogue row
    // is loaded, which keeps the register peak (and so the occupancy) at the k-loop's
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t pl = wm * 64 + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const uint32_t cl = wn * (BN / 2) + j * 16 + (lane >> 4) * 4;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[j][i][r]);
        const uint32_t off = eimg_off8<NCH>(pl, cl);
        *LDS_PTR(bf16x4, E + off) = o;
      }
    }
    // The HBM-bound part is this thread's BN-input / residual / add-source rows, loaded in
    // batches of RBATCH rows (the first batch in flight across the LDS barrier).
    constexpr int RBATCH = RPT >= 4 ? 4 : RPT;
    const bool has_res = !MASKED && p.bnb.res != nullptr, has_add = p.addsrc != nullptr;
    float sc[8], sh[8], mu[8], s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      if (!MASKED) {
        sc[e] = cok ? p.bnb.scale[cg + e] : 0.f;
        sh[e] = cok ? p.bnb.shift[cg + e] : 0.f;
      }
      mu[e] = cok ? p.bnb.mean[cg + e] : 0.f;
    }
#pragma unroll
    for (int b = 0; b < RPT / RBATCH; ++b) {
      bf16x8 yv[RBATCH], rv[RBATCH], av[RBATCH];
      uint32_t mk[RBATCH];
#pragma unroll
      for (int q = 0; q < RBATCH; ++q) {
        const int m = m0 + pr0 + (b * RBATCH + q) * R;
        const bool ok = m < p.M && cok;
        const size_t off = (size_t)(ok ? m : 0) * p.Co + (cok ? cg : 0);
        yv[q] = ok ? *(const bf16x8*)(p.bnb.y + off) : bf16x8{};
        if (has_res) rv[q] = ok ? *(const bf16x8*)(p.bnb.res + off) : bf16x8{};
        if (has_add) {
          if (p.bnb.add_s2 == 0) {
            av[q] = ok ? *(const bf16x8*)(p.addsrc + off) : bf16x8{};
          } else {
            // compact stride-2 add source: only even (y, x) pixels carry a gradient
            const uint32_t mm = ok ? (uint32_t)m : 0u;
            const uint32_t qq = fdiv(mm, p.div_wy);
            const uint32_t xx = mm - qq * p.Wy;
            const uint32_t nn = fdiv(qq, p.div_hy);
            const uint32_t yy = qq - nn * p.Hy;
            const bool on = ok && !(yy & 1u) && !(xx & 1u);
            const size_t co = ((size_t)(nn * p.bnb.add_hc + (yy >> 1)) * p.bnb.add_wc + (xx >> 1)) * p.Co + cg;
            av[q] = on ? *(const bf16x8*)(p.addsrc + co) : bf16x8{};
          }
        }
        if (MASKED) mk[q] = ok ? p.bnb.mask[off >> 3] : 0u;
      }
      if (b == 0) __syncthreads();
#pragma unroll
      for (int q = 0; q < RBATCH; ++q) {
        const int pl = pr0 + (b * RBATCH + q) * R;
        const int m = m0 + pl;
        if (m < p.M && cok) {
          const bf16x8 v = eimg_chunk<NCH>(E, pl, c);
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float g = bf2f(v[e]);
            if (has_add) g = bf2f(f2bf(g + bf2f(av[q][e])));  // the rounding of the unfused add
            const float yf = bf2f(yv[q][e]);
            float gd = 1.f;  // act'(z) for the leaky sums (the stored gradient stays raw)
            if (MASKED) {
              if (p.bnb.act == 1 && !((mk[q] >> e) & 1u)) g = 0.f;
            } else {
              float z = yf * sc[e] + sh[e];
              if (has_res) z += bf2f(rv[q][e]);
              if (p.bnb.act == 1 && !(z > 0.f)) g = 0.f;
              if (p.bnb.act == 2 && !(z >= 0.f)) gd = p.bnb.slope;  // act_d's leaky convention (bn.hip)
            }
            o[e] = f2bf(g);
            const float gr = bf2f(o[e]) * gd;
            s1[e] += gr;
            s2[e] += gr * (yf - mu[e]);
          }
          *(bf16x8*)(p.dst + (size_t)m * p.Co + cg) = o;
        }
      }
    }
    // per-tile channel sums: fixed-order reduction over the R row groups (deterministic), in
    // the LDS image's space once every thread has read its rows (keeps the workgroup at 32 KB).
    // Layout [which][e][R x NCH (+4 pad)]: the writes (fixed e, consecutive threads = consecutive
    // chunks) and the column reads (32 lanes = 4 chunks x 8 elements) are both bank-conflict free.
    constexpr int SE = R * NCH + 4;
    float* red = (float*)smem;  // [2][8][SE]
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(0 * 8 + e) * SE + pr0 * NCH + c] = s1[e];
      red[(1 * 8 + e) * SE + pr0 * NCH + c] = s2[e];
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int which = tid / BN, ch = tid - which * BN;
      if (n0 + ch < p.Co) {
        const float* col = red + (which * 8 + (ch & 7)) * SE + (ch >> 3);
        float t = 0.f;
#pragma unroll 4
        for (int r = 0; r < R; ++r) t += col[r * NCH];
        if (which) t *= p.bnb.invstd[n0 + ch];
        p.bnb.part[((size_t)tm * 2 + which) * p.Co + n0 + ch] = t;
      }
    }
    return;
  }

  if constexpr (EPI != 2) {
    tg_store_epilogue<BN, EPI>(p, acc, smem, m0, n0, tid, lane, wm, wn);
    return;
  }

  // ---- register epilogue (linear heads): bias / activation, 8-byte stores ----
  const int co_lane = n0 + wn * (BN / 2) + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    const bool mok = m < p.M;
    size_t drow = 0;
    if (mok) {
      const uint32_t q = fdiv(m, p.div_wy);
      const uint32_t x = m - q * p.Wy;
      const uint32_t n = fdiv(q, p.div_hy);
      const uint32_t y = q - n * p.Hy;
      drow = (size_t)((n * p.Hd + y * p.ds + p.oy) * p.Wd + x * p.ds + p.ox) * (size_t)p.Co;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = co_lane + j * 16;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = acc[j][i][r];
        if (p.bias) t += (co + r < p.nbias) ? p.bias[co + r] : 0.f;
        if (p.relu == 1) t = fmaxf(t, 0.f);
        else if (p.relu == 2) t = 1.f / (1.f + __expf(-t));
        v[r] = t;
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
      if (mok && co < p.Co) *(bf16x4*)(p.dst + drow + co) = o;
    }
  }
}

// ---------------------------------------------------------------------------
// Big-tile tap GEMM: WM x WN waves, each owning 128 pixel rows x 64 output channels (8 x 4
// accumulator fragments: 12 fragment reads feed 32 MFMAs per 32-deep k-step, against 8 for 16
// in the 4-wave kernel); workgroup tile BM = 128 WM x BN = 64 WN, e.g. 256 x 256 at 8 waves,
// one workgroup per CU.  The 128-row kernels above run at the ceiling of their structure (two
// barriers' worth of exposed load latency per k-step, 2-3 workgroups per CU: ~900 TF/s on the
// deep-K shapes, cdna_hip_programming.md §5 ladder) and move 32 KB of LDS-DMA per 2 MFLOP; this
// one moves 32 KB per 4.2 MFLOP (256 x 256 x 32) and keeps NS-2 k-tiles of LDS-DMA in flight
// across every raw s_barrier (NS-slot ring of 32-deep k-tiles, counted vmcnt, never 0 in the
// loop; the slot re-staged after barrier kt is the one every wave finished reading before it).
// FAST shapes (Cs % 64 == 0, one tap per k-tile), plain / statistics epilogue (+ eval-BN fold /
// add source): the accumulators go to a whole-tile LDS image cut into 128 x 128 quadrants, which
// the 256-thread groups store through tg_image_store (the 4-wave kernel's epilogue).
// ---------------------------------------------------------------------------
// (CFW: 16-channel accumulator fragments per wave; the 4-wave 256 x 256 tile at CFW = 8 measured
// slower on every R50 shape, profiles/r4/big4_tile_ab_b1024.txt, and was removed)
template <int WM, int WN, int NS, int EPI, int CFW = 4>
__global__ void __launch_bounds__(64 * WM * WN, 2)
tap_gemm_big_kernel(const TapGemmParams p) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BM = 128 * WM, BN = 16 * CFW * WN, BK = 32;
  constexpr int ROWB = BK * 2, CH = BK / 8, RPI = 64 / CH;  // 64-byte rows, 16 rows per LDS-DMA
  constexpr int AI = BM / (NW * RPI), BI = BN / (NW * RPI), LPT = AI + BI;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int QN = BN / 128, NQ = WM * QN, NG = NT / 256, QPG = NQ / NG;  // epilogue quadrants
  static_assert(AI >= 1 && BI >= 1 && AI * NW * RPI == BM && BI * NW * RPI == BN, "LDS-DMA split");
  static_assert(BN % 128 == 0 && NT % 256 == 0 && NQ % NG == 0 && NS >= 3, "tile geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const uint32_t ntn = (p.Co + BN - 1) / BN, ntm = (p.M + BM - 1) / BM;
  const uint32_t bid = xcd_remap(blockIdx.x, ntm * ntn);
  const uint32_t tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // per-slot source pointers + tap-validity masks (as tap_gemm_kernel's FAST path); rows past M
  // and channels past Co read a clamped valid row and are never stored or counted
  const bf16* fa_ptr[AI];
  uint32_t fa_vm[AI];
  const bf16* fb_ptr[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wave * AI + i) * RPI + lane / CH;
    const uint32_t mm = (uint32_t)min(m0 + r, p.M - 1);
    const uint32_t q = fdiv(mm, p.div_wy);
    const uint32_t x = mm - q * p.Wy;
    const uint32_t n = fdiv(q, p.div_hy);
    const uint32_t y = q - n * p.Hy;
    const int ys = y * p.ss, xs = x * p.ss;
    fa_ptr[i] = p.src + ((size_t)n * p.Hs * p.Ws + (size_t)ys * p.Ws + xs) * p.Cs + ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
    uint32_t vm = 0;
    for (int t = 0; t < p.ntaps; ++t) {
      const int tv = p.tap[t];
      const int hi = ys + tap_dy(tv), wi = xs + tap_dx(tv);
      vm |= ((unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws) ? (1u << t) : 0u;
    }
    fa_vm[i] = vm;
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (wave * BI + i) * RPI + lane / CH;
    fb_ptr[i] = p.wt + (size_t)min(n0 + r, p.Co - 1) * p.ldw + ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
  }
  const int tiles_per_tap = p.cpt / CH;
  auto stage = [&](int kt, int slot) {
    char* As = smem + slot * STAGE;
    char* Bs = As + A_BYTES;
    const int t = kt / tiles_per_tap;
    const int cbase = (kt - t * tiles_per_tap) * BK;
    const int tv = p.tap[t];
    const long aoff = (long)(tap_dy(tv) * p.Ws + tap_dx(tv)) * p.Cs + cbase;  // wave-uniform
    const long boff = (long)tap_w(tv) * p.Cs + cbase;
    const uint32_t tbit = 1u << t;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bf16* g = (fa_vm[i] & tbit) ? fa_ptr[i] + aoff : p.zero;
      dma16_tracked(g, As + (wave * AI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i)
      dma16_tracked((fb_ptr[i] + boff), Bs + (wave * BI + i) * 1024);
  };

  f32x4 acc[CFW][8];  // [16-channel fragment][16-pixel fragment]
#pragma unroll
  for (int j = 0; j < CFW; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = p.nkt;
  const uint32_t c = lane >> 4;
  bf16x8 wf[CFW], af[8];
  auto frag_w = [&](int slot) {
    const char* Bs = smem + slot * STAGE + A_BYTES;
#pragma unroll
    for (int j = 0; j < CFW; ++j)
      wf[j] = *(const bf16x8*)(Bs + swzk<BK>(wn * (16 * CFW) + j * 16 + (lane & 15), c));
  };
  auto frag_a = [&](int slot, int i0) {
    const char* As = smem + slot * STAGE;
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i) af[i] = *(const bf16x8*)(As + swzk<BK>(wm * 128 + i * 16 + (lane & 15), c));
  };
  auto mfma_half = [&](int i0) {
#pragma unroll
    for (int j = 0; j < CFW; ++j)
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
  };
  // raw barrier: this wave's fragment reads retired first (WAR on the slot re-staged after it);
  // the counted vmcnt before it is the RAW wait -- no vmcnt(0), the ring stays in flight
  auto ring_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nkt) stage(i, i);
  if (WM == 2 && p.cvar == 3 && nkt > 0) {
    // Ping-pong (g_tune[kTgBigCvar] = 3): the two row halves of the tile are two wave groups
    // (waves 0-3: pixel rows 0-127, waves 4-7: 128-255), and the waves of a workgroup sit on the
    // four SIMDs one from each group.  Group 1 runs one segment behind group 0, so in every
    // interval between two workgroup barriers one wave of each SIMD runs its MFMA segment
    // (k-tile kt's 32 MFMAs from registers) while its partner runs a load segment (the next
    // k-tile's 12 fragment reads and its share of a later k-tile's LDS-DMA): the matrix pipe
    // alternates between the two instead of idling through a common read phase.
    // Synchronisation, counting workgroup barriers b (group 0 loads k-tile kt in (2kt, 2kt+1),
    // computes it in (2kt+1, 2kt+2); group 1 one interval later):
    //   RAW -- every wave retires its own DMA of k-tile kt (counted vmcnt) before barrier 2kt:
    //   group 0 at the end of its compute segment kt-1, group 1 at the end of its load segment kt-1;
    //   WAR -- k-tile kt's slot is last read in (2kt+1, 2kt+2) (each reader waits lgkmcnt(0)
    //   before its next barrier) and is restaged (k-tile kt+NS) in load segments after 2kt+2.
    // Each group passes the same number of barriers: group 1 one extra at the start, group 0 one
    // extra at the end.
    const int grp = wm;
    auto pp_barrier = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    // The load segment issues its LDS-DMA first and its fragment reads behind it, so the DMA's
    // address work overlaps the reads' latency.  The tap table sits in one VGPR (lane t = tap t,
    // read with v_readlane) and the (tap, channel) of the next k-tile to stage advances with
    // scalar selects: a scalar-memory tap lookup would make the compiler wait lgkmcnt(0) -- for the
    // fragment reads too -- before every DMA.
    const int tap_lane = lane < p.ntaps ? p.tap[lane] : 0;
    int st_t = (NS - 1) / tiles_per_tap, st_c = ((NS - 1) - st_t * tiles_per_tap) * BK;
    auto stage_next = [&](int slot) {
      char* As = smem + slot * STAGE;
      char* Bs = As + A_BYTES;
      const int tv = __builtin_amdgcn_readlane(tap_lane, st_t);
      const long aoff = (long)(tap_dy(tv) * p.Ws + tap_dx(tv)) * p.Cs + st_c;  // wave-uniform
      const long boff = (long)tap_w(tv) * p.Cs + st_c;
      const uint32_t tbit = 1u << st_t;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bf16* g = (fa_vm[i] & tbit) ? fa_ptr[i] + aoff : p.zero;
        dma16_tracked(g, As + (wave * AI + i) * 1024);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i) dma16_tracked((fb_ptr[i] + boff), Bs + (wave * BI + i) * 1024);
      st_c += BK;
      const bool wrap = st_c >= p.Cs;
      st_t += wrap ? 1 : 0;
      st_c = wrap ? 0 : st_c;
    };
    wait_vmcnt(LPT * min(NS - 2, nkt - 1));  // k-tile 0 (this wave's share)
    pp_barrier();                            // ... every wave's
    if (grp == 1) pp_barrier();
    for (int kt = 0; kt < nkt; ++kt) {
      const int slot = kt % NS;
      if (kt + NS - 1 < nkt && !(p.ablate & 1)) stage_next((kt + NS - 1) % NS);
      __builtin_amdgcn_sched_barrier(0);
      frag_w(slot);
      frag_a(slot, 0);
      frag_a(slot, 4);
      __builtin_amdgcn_sched_barrier(0);
      if (grp == 1 && kt + 1 < nkt) wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
      if (!(p.ablate & 2)) {  // timing ablations (g_tune[kAblate]): 1 no LDS-DMA, 2 no MFMA
        mfma_half(0);
        mfma_half(4);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (grp == 0 && kt + 1 < nkt) wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));
      pp_barrier();
    }
    if (grp == 0) pp_barrier();
  } else if (p.cvar == 2) {
    // g_tune[kTgBigCvar] = 2 (A/B only): fragments read after the barrier, all 32 MFMAs behind them
    for (int kt = 0; kt < nkt; ++kt) {
      wait_vmcnt(LPT * min(NS - 2, nkt - 1 - kt));  // k-tile kt landed (this wave's share)
      ring_barrier();  // ... for every wave; slot kt-1 is free
      if (kt + NS - 1 < nkt) stage(kt + NS - 1, (kt + NS - 1) % NS);
      frag_w(kt % NS);
      frag_a(kt % NS, 0);
      frag_a(kt % NS, 4);
      mfma_half(0);
      mfma_half(4);
    }
  } else if (nkt > 0) {
    // default: the fragments of k-tile kt+1 are read across the barrier, behind the MFMAs of k-tile
    // kt -- pixel fragments 0..3 after its first half, the rest after its second half (measured
    // 2-4 % faster than reading them after the barrier: profiles/r3/big_tile_ab_b1024_pipelined.txt)
    wait_vmcnt(LPT * min(NS - 2, nkt - 1));
    ring_barrier();
    if (NS - 1 < nkt) stage(NS - 1, NS - 1);
    frag_w(0);
    frag_a(0, 0);
    frag_a(0, 4);
    for (int kt = 0; kt < nkt; ++kt) {
      const int nx = (kt + 1) % NS;
      mfma_half(0);
      if (kt + 1 < nkt) {
        wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));  // k-tile kt+1 landed (this wave's share)
        ring_barrier();  // ... for every wave; every read of slot kt retired: re-stage it
        if (kt + NS < nkt) stage(kt + NS, kt % NS);
        frag_a(nx, 0);
      }
      mfma_half(4);
      if (kt + 1 < nkt) {
        frag_w(nx);
        frag_a(nx, 4);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (p.ablate & 4) return;  // timing ablation: no epilogue

  // ---- epilogue: quadrant (h, qc) = pixels h*128.., channels qc*128.. at smem + (h*QN + qc) * 32 KB ----
  {
    char* Q = smem + (wm * QN + (wn * 16 * CFW) / 128) * 32768;
    const uint32_t cb = (wn * 16 * CFW) % 128;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t pl = i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < CFW; ++j) {
        const uint32_t cl = cb + j * 16 + (lane >> 4) * 4;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[j][i][r]);
        *LDS_PTR(bf16x4, Q + eimg_off8<16>(pl, cl)) = o;
      }
    }
  }
  __syncthreads();
  // group g (threads 256g ..) stores quadrants g*QPG ..; every group passes the same barriers
  // (tile_stats128_vv's), so the quadrant loop stays uniform
  const int g = tid >> 8, gtid = tid & 255;
#pragma unroll
  for (int k = 0; k < QPG; ++k) {
    const int q = g * QPG + k;
    tg_image_store<128, EPI>(p, smem + q * 32768, m0 + (q / QN) * 128, n0 + (q % QN) * 128, gtid);
  }
}

// The same tile as a loop over work segments: persistent workgroups (tg_big_persist) or stream-K
// (p.sk_ws).  A separate kernel because the loop's carried scalars cost ~50 SGPRs spilled to VGPR
// lanes, and every attempt to fold the one-tile kernel above into it (opaque per-tile parameter
// pointers, laundered lane index) either spilled or copied the parameters to scratch and ran the
// big tile 2.5x slower (d4d972e: 512-channel 7x7 3x3 220 -> 645 us).
template <int WM, int WN, int NS, int EPI, int CFW = 4>
__global__ void __launch_bounds__(64 * WM * WN, 2)
tap_gemm_big_loop_kernel(const TapGemmParams p0) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BM = 128 * WM, BN = 16 * CFW * WN, BK = 32;
  constexpr int ROWB = BK * 2, CH = BK / 8, RPI = 64 / CH;  // 64-byte rows, 16 rows per LDS-DMA
  constexpr int AI = BM / (NW * RPI), BI = BN / (NW * RPI), LPT = AI + BI;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int QN = BN / 128, NQ = WM * QN, NG = NT / 256, QPG = NQ / NG;  // epilogue quadrants
  static_assert(AI >= 1 && BI >= 1 && AI * NW * RPI == BM && BI * NW * RPI == BN, "LDS-DMA split");
  static_assert(BN % 128 == 0 && NT % 256 == 0 && NQ % NG == 0 && NS >= 3, "tile geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const uint32_t ntn = (p0.Co + BN - 1) / BN, ntm = (p0.M + BM - 1) / BM;
  // tg_big_persist = 1: one workgroup per CU walks tiles blockIdx.x, + gridDim.x, ... (the same
  // XCD-contiguous tile order as one launch per tile): the epilogue's global stores drain while
  // the next tile's ring fills, and no workgroup is re-dispatched per tile
  const uint32_t ntiles = ntm * ntn;
  const uint32_t tstep = p0.persist ? gridDim.x : ntiles;
  // Stream-K (p.sk_ws set; one workgroup per CU slot, ntiles >= gridDim.x): the ntiles x nkt
  // k-steps are cut into gridDim.x equal contiguous ranges, so every workgroup does the same
  // MFMA work and no tail round of partly idle CUs remains (784 256 x 256 tiles on 256 CUs were
  // 4 rounds for 3.06 rounds of work).  A range covers whole tiles plus at most a tail piece of the
  // tile where it begins (k-steps kb..nkt: published as an fp32 partial, then the next segment) and
  // a head piece of the tile where it ends (k-steps 0..ke: the partial of the next workgroup added,
  // then the tile's normal epilogue).  The tail piece is this workgroup's FIRST segment and the head
  // piece its LAST, so the partial is waited for only after a whole range of work.
  const bool sk = p0.sk_ws != nullptr;
  const int nkt_all = p0.nkt;
  // (32-bit: the host checks ntiles x nkt < 2^31; a 64-bit division here costs ~20 SGPRs)
  uint32_t sk_it = 0, sk_end = 0;
  if (sk) {
    // range boundaries on multiples of sk_unit k-steps (a divisor of nkt): every workgroup starts
    // at one of nkt / sk_unit k positions, so the workgroups of an XCD stream the same few weight
    // slices at a time (unquantised ranges start at every k and the whole weight matrix competes
    // for the XCD's L2: no gain at all on the 4.7 MB 512-channel 3x3)
    const uint32_t u = (uint32_t)p0.sk_unit;
    const uint64_t U = (uint64_t)ntiles * ((uint32_t)nkt_all / u);
    sk_it = (uint32_t)(blockIdx.x * U / gridDim.x) * u;
    sk_end = (uint32_t)((blockIdx.x + 1) * U / gridDim.x) * u;
  }
  uint32_t next_tile = blockIdx.x;
  for (;;) {
    uint32_t tile;
    int kb, ke;
    if (sk) {
      if (sk_it >= sk_end) break;
      tile = sk_it / (uint32_t)nkt_all;
      kb = (int)(sk_it - tile * (uint32_t)nkt_all);
      ke = min(nkt_all, kb + (int)(sk_end - sk_it));
      sk_it += (uint32_t)(ke - kb);
    } else {
      if (next_tile >= ntiles) break;
      tile = next_tile;
      kb = 0;
      ke = nkt_all;
      next_tile += tstep;
    }
    // The parameters re-read per tile from the kernel-argument segment (scalar loads) through an
    // opaque constant-address-space pointer, into a local copy the compiler splits into scalars:
    // nothing derived from them is carried across the loop (held across it, they spilled ~60
    // SGPRs to VGPR lanes: 190 v_readlane in the kernel).  Laundering the address of the by-value
    // argument instead copies the whole struct into per-lane scratch.  The tap table, indexed
    // dynamically, is read through the pointer (pk->tap[t]), never from the copy.
    typedef const __attribute__((address_space(4))) TapGemmParams* KArgPtr;
    KArgPtr pk4 = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(pk4));
    const TapGemmParams* pk = (const TapGemmParams*)pk4;  // (address space inferred back: scalar loads)
    const TapGemmParams p = *pk;
    // the k-loop's scalars, read once per tile and pinned in registers: an asm result cannot be
    // re-loaded from the argument segment inside the k-loop, where each scalar load's lgkmcnt wait
    // would also drain the LDS fragment reads
    int kWs = p.Ws, kCs = p.Cs, kabl = p.ablate;
    const bf16* kzero = p.zero;
    asm volatile("" : "+s"(kWs), "+s"(kCs), "+s"(kabl), "+s"(kzero));
    // the lane index likewise: every lane-derived LDS / global offset is recomputed per tile
    // instead of being hoisted and held in VGPRs through the k-loop
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    // (stream-K: a workgroup's consecutive tiles are neighbours already -- one XCD's L2 sees them)
    const uint32_t bid = sk ? tile : xcd_remap(tile, ntiles);
    const uint32_t tn = bid % ntn, tm = bid / ntn;
    const int m0 = tm * BM, n0 = tn * BN;

    // per-slot source pointers + tap-validity masks (as tap_gemm_kernel's FAST path); rows past M
    // and channels past Co read a clamped valid row and are never stored or counted
    const bf16* fa_ptr[AI];
    uint32_t fa_vm[AI];
    const bf16* fb_ptr[BI];
  #pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = (wave * AI + i) * RPI + lane / CH;
      const uint32_t mm = (uint32_t)min(m0 + r, p.M - 1);
      const uint32_t q = fdiv(mm, p.div_wy);
      const uint32_t x = mm - q * p.Wy;
      const uint32_t n = fdiv(q, p.div_hy);
      const uint32_t y = q - n * p.Hy;
      const int ys = y * p.ss, xs = x * p.ss;
      fa_ptr[i] = p.src + ((size_t)n * p.Hs * p.Ws + (size_t)ys * p.Ws + xs) * p.Cs + ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
      uint32_t vm = 0;
      for (int t = 0; t < p.ntaps; ++t) {
        const int tv = pk->tap[t];
        const int hi = ys + tap_dy(tv), wi = xs + tap_dx(tv);
        vm |= ((unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws) ? (1u << t) : 0u;
      }
      fa_vm[i] = vm;
    }
  #pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int r = (wave * BI + i) * RPI + lane / CH;
      fb_ptr[i] = p.wt + (size_t)min(n0 + r, p.Co - 1) * p.ldw + ((lane % CH) ^ swz_chunk<BK>(r)) * 8;
    }
    const int tiles_per_tap = p.cpt / CH;
    // k-steps kb .. ke-1 of the tile; the loops below count kt from 0 (= k-step kb)
    auto stage = [&](int kt, int slot) {
      char* As = smem + slot * STAGE;
      char* Bs = As + A_BYTES;
      const int ka = kb + kt;
      const int t = ka / tiles_per_tap;
      const int cbase = (ka - t * tiles_per_tap) * BK;
      const int tv = pk->tap[t];
      const long aoff = (long)(tap_dy(tv) * kWs + tap_dx(tv)) * kCs + cbase;  // wave-uniform
      const long boff = (long)tap_w(tv) * kCs + cbase;
      const uint32_t tbit = 1u << t;
  #pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bf16* g = (fa_vm[i] & tbit) ? fa_ptr[i] + aoff : kzero;
        dma16_tracked(g, As + (wave * AI + i) * 1024);
      }
  #pragma unroll
      for (int i = 0; i < BI; ++i)
        dma16_tracked((fb_ptr[i] + boff), Bs + (wave * BI + i) * 1024);
    };

    f32x4 acc[CFW][8];  // [16-channel fragment][16-pixel fragment]
  #pragma unroll
    for (int j = 0; j < CFW; ++j)
  #pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nkt = ke - kb;
    const uint32_t c = lane >> 4;
    bf16x8 wf[CFW], af[8];
    auto frag_w = [&](int slot) {
      const char* Bs = smem + slot * STAGE + A_BYTES;
  #pragma unroll
      for (int j = 0; j < CFW; ++j)
        wf[j] = *(const bf16x8*)(Bs + swzk<BK>(wn * (16 * CFW) + j * 16 + (lane & 15), c));
    };
    auto frag_a = [&](int slot, int i0) {
      const char* As = smem + slot * STAGE;
  #pragma unroll
      for (int i = i0; i < i0 + 4; ++i) af[i] = *(const bf16x8*)(As + swzk<BK>(wm * 128 + i * 16 + (lane & 15), c));
    };
    auto mfma_half = [&](int i0) {
  #pragma unroll
      for (int j = 0; j < CFW; ++j)
  #pragma unroll
        for (int i = i0; i < i0 + 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
    };
    // raw barrier: this wave's fragment reads retired first (WAR on the slot re-staged after it);
    // the counted vmcnt before it is the RAW wait -- no vmcnt(0), the ring stays in flight
    auto ring_barrier = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
  #pragma unroll
    for (int i = 0; i < NS - 1; ++i)
      if (i < nkt) stage(i, i);
    if (WM == 2 && p.cvar >= 3 && nkt > 0) {
      // Ping-pong (g_tune[kTgBigCvar] = 3): the two row halves of the tile are two wave groups
      // (waves 0-3: pixel rows 0-127, waves 4-7: 128-255), and the waves of a workgroup sit on the
      // four SIMDs one from each group.  Group 1 runs one segment behind group 0, so in every
      // interval between two workgroup barriers one wave of each SIMD runs its MFMA segment
      // (k-tile kt's 32 MFMAs from registers) while its partner runs a load segment (the next
      // k-tile's 12 fragment reads and its share of a later k-tile's LDS-DMA): the matrix pipe
      // alternates between the two instead of idling through a common read phase.
      // Synchronisation, counting workgroup barriers b (group 0 loads k-tile kt in (2kt, 2kt+1),
      // computes it in (2kt+1, 2kt+2); group 1 one interval later):
      //   RAW -- every wave retires its own DMA of k-tile kt (counted vmcnt) before barrier 2kt:
      //   group 0 at the end of its compute segment kt-1, group 1 at the end of its load segment kt-1;
      //   WAR -- k-tile kt's slot is last read in (2kt+1, 2kt+2) (each reader waits lgkmcnt(0)
      //   before its next barrier) and is restaged (k-tile kt+NS) in load segments after 2kt+2.
      // Each group passes the same number of barriers: group 1 one extra at the start, group 0 one
      // extra at the end.
      const int grp = wm;
      auto pp_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      };
      // The load segment issues its LDS-DMA first and its fragment reads behind it, so the DMA's
      // address work overlaps the reads' latency.  The tap table sits in one VGPR (lane t = tap t,
      // read with v_readlane) and the (tap, channel) of the next k-tile to stage advances with
      // scalar selects: a scalar-memory tap lookup would make the compiler wait lgkmcnt(0) -- for the
      // fragment reads too -- before every DMA.
      const int tap_lane = lane < p.ntaps ? pk->tap[lane] : 0;
      int st_t = (kb + NS - 1) / tiles_per_tap, st_c = ((kb + NS - 1) - st_t * tiles_per_tap) * BK;
      auto stage_next = [&](int slot) {
        char* As = smem + slot * STAGE;
        char* Bs = As + A_BYTES;
        const int tv = __builtin_amdgcn_readlane(tap_lane, st_t);
        const long aoff = (long)(tap_dy(tv) * kWs + tap_dx(tv)) * kCs + st_c;  // wave-uniform
        const long boff = (long)tap_w(tv) * kCs + st_c;
        const uint32_t tbit = 1u << st_t;
  #pragma unroll
        for (int i = 0; i < AI; ++i) {
          const bf16* g = (fa_vm[i] & tbit) ? fa_ptr[i] + aoff : kzero;
          dma16_tracked(g, As + (wave * AI + i) * 1024);
        }
  #pragma unroll
        for (int i = 0; i < BI; ++i) dma16_tracked((fb_ptr[i] + boff), Bs + (wave * BI + i) * 1024);
        st_c += BK;
        const bool wrap = st_c >= kCs;
        st_t += wrap ? 1 : 0;
        st_c = wrap ? 0 : st_c;
      };
      wait_vmcnt(LPT * min(NS - 2, nkt - 1));  // k-tile 0 (this wave's share)
      pp_barrier();                            // ... every wave's
      if (grp == 1) pp_barrier();
      for (int kt = 0; kt < nkt; ++kt) {
        const int slot = kt % NS;
        if (kt + NS - 1 < nkt && !(kabl & 1)) stage_next((kt + NS - 1) % NS);
        __builtin_amdgcn_sched_barrier(0);
        frag_w(slot);
        frag_a(slot, 0);
        frag_a(slot, 4);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 1 && kt + 1 < nkt) wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));
        pp_barrier();
        __builtin_amdgcn_s_setprio(1);
        if (!(kabl & 2)) {  // timing ablations (g_tune[kAblate]): 1 no LDS-DMA, 2 no MFMA
          mfma_half(0);
          mfma_half(4);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0 && kt + 1 < nkt) wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));
        pp_barrier();
      }
      if (grp == 0) pp_barrier();
    } else if (p.cvar == 2) {
      // g_tune[kTgBigCvar] = 2 (A/B only): fragments read after the barrier, all 32 MFMAs behind them
      for (int kt = 0; kt < nkt; ++kt) {
        wait_vmcnt(LPT * min(NS - 2, nkt - 1 - kt));  // k-tile kt landed (this wave's share)
        ring_barrier();  // ... for every wave; slot kt-1 is free
        if (kt + NS - 1 < nkt) stage(kt + NS - 1, (kt + NS - 1) % NS);
        frag_w(kt % NS);
        frag_a(kt % NS, 0);
        frag_a(kt % NS, 4);
        mfma_half(0);
        mfma_half(4);
      }
    } else if (nkt > 0) {
      // default: the fragments of k-tile kt+1 are read across the barrier, behind the MFMAs of k-tile
      // kt -- pixel fragments 0..3 after its first half, the rest after its second half (measured
      // 2-4 % faster than reading them after the barrier: profiles/r3/big_tile_ab_b1024_pipelined.txt)
      wait_vmcnt(LPT * min(NS - 2, nkt - 1));
      ring_barrier();
      if (NS - 1 < nkt) stage(NS - 1, NS - 1);
      frag_w(0);
      frag_a(0, 0);
      frag_a(0, 4);
      for (int kt = 0; kt < nkt; ++kt) {
        const int nx = (kt + 1) % NS;
        mfma_half(0);
        if (kt + 1 < nkt) {
          wait_vmcnt(LPT * min(NS - 2, nkt - 2 - kt));  // k-tile kt+1 landed (this wave's share)
          ring_barrier();  // ... for every wave; every read of slot kt retired: re-stage it
          if (kt + NS < nkt) stage(kt + NS, kt % NS);
          frag_a(nx, 0);
        }
        mfma_half(4);
        if (kt + 1 < nkt) {
          frag_w(nx);
          frag_a(nx, 4);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (sk && kb > 0) {
      // the tail piece of a tile that workgroup blockIdx.x - 1 finishes: publish the fp32 partial
      // in register order (slot blockIdx.x; lane-contiguous 16-byte stores, 1 KB per instruction)
      // WRITE-THROUGH (sc1): no release fence, whose L2 write-back stalled every workgroup at the
      // start of its range; every storing wave drained, a barrier, then one lane's flag
      // (Guideline 16 R1)
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.sk_ws + ((size_t)blockIdx.x * NW + wave) * (CFW * 8 * 64)), (short)0, 0x7fffffff, 0x00020000);
  #pragma unroll
      for (int j = 0; j < CFW; ++j)
  #pragma unroll
        for (int i = 0; i < 8; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j][i]), rs,
                                                 ((j * 8 + i) * 64 + lane) * 16, 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(p.sk_flags + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const f32x4* skp = nullptr;  // the partial to add in the epilogue (head piece of a cut tile)
    if (sk && ke < nkt_all) {
      // the head piece: wait for workgroup blockIdx.x + 1's partial of the same tile (published at
      // the start of its range, so normally long done), one agent-scope acquire, add it
      if (tid == 0) {
        // bounded spin (the grid is at most one workgroup per CU slot, and the publisher waits on
        // nothing before publishing, so it only has to become resident)
        for (uint32_t spins = 0;
             __hip_atomic_load(p.sk_flags + blockIdx.x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
             spins < (1u << 26);
             ++spins)
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      skp = p.sk_ws + ((size_t)(blockIdx.x + 1) * NW + wave) * (CFW * 8 * 64) + lane;
    }
    if (p.ablate & 4) continue;  // timing ablation: no epilogue

    // ---- epilogue: quadrant (h, qc) = pixels h*128.., channels qc*128.. at smem + (h*QN + qc) * 32 KB ----
    {
      char* Q = smem + (wm * QN + (wn * 16 * CFW) / 128) * 32768;
      const uint32_t cb = (wn * 16 * CFW) % 128;
  #pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t pl = i * 16 + (lane & 15);
  #pragma unroll
        for (int j = 0; j < CFW; ++j) {
          const uint32_t cl = cb + j * 16 + (lane >> 4) * 4;
          f32x4 a = acc[j][i];
          if (skp != nullptr) a += skp[(j * 8 + i) * 64];  // fp32 partial, before the one rounding
          bf16x4 o;
  #pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(a[r]);
          *LDS_PTR(bf16x4, Q + eimg_off8<16>(pl, cl)) = o;
        }
      }
    }
    __syncthreads();
    // group g (threads 256g ..) stores quadrants g*QPG ..; every group passes the same barriers
    // (tile_stats128_vv's), so the quadrant loop stays uniform
    const int g = tid >> 8, gtid = tid & 255;
  #pragma unroll
    for (int k = 0; k < QPG; ++k) {
      const int q = g * QPG + k;
      tg_image_store<128, EPI>(p, smem + q * 32768, m0 + (q / QN) * 128, n0 + (q % QN) * 128, gtid);
    }
    __syncthreads();  // every image read retired before the ring is refilled
  }
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
struct WgradParams {
  const bf16* dy;    // [M][Co]
  const bf16* src;   // [N][Hs][Ws][Cs]
  float* dw;         // [Co][T*Cs] fp32, accumulated atomically (part == nullptr)
  float* part;       // [splits][Co][T*Cs] fp32 per-split partials (plain stores), or nullptr
  const bf16* zero;
  int Hs, Ws, Cs, Ho, Wo, ss;
  int Co, M, ldw;    // ldw = T*Cs
  int cpt, kc_total, rows_per_split;
  int ablate;  // tuning experiments only: 8 = skip the atomic flush
  int direct;  // 1x1 stride-1 (no padding): the input pixel of GEMM row m is m
  // PRO (direct only): the input is a BN's input x, used as relu(x * pscale[c] + pshift[c]) (K5)
  const float* pscale;
  const float* pshift;
  FastDiv div_wo, div_ho, div_cpt;
  int8_t dy_t[kMaxTaps], dx_t[kMaxTaps];
};

// byte offset of logical 16B chunk c of row r in a 256-byte-row image read
// with ds_read_b64_tr_b16 (4-row blocks per 16-lane group)
__device__ __forceinline__ uint32_t swz256(uint32_t r, uint32_t c) {
  return r * 256u + ((c ^ (((r & 3u) << 1) | (((r >> 3) & 1u) << 3))) << 4);
}

__device__ __forceinline__ bf16x8 tr_frag(const char* img, uint32_t row0, uint32_t col0, int lane) {
  // rows row0 .. row0+7 (two 4-row transposed blocks), columns col0 .. col0+15
  const uint32_t q = (lane & 15) >> 2, pp = lane & 3;
  const uint32_t col = col0 + pp * 4;
  const uint32_t r1 = row0 + q, r2 = row0 + 4 + q;
  const uint32_t o1 = swz256(r1, col >> 3) + (col & 7) * 2;
  const uint32_t o2 = swz256(r2, col >> 3) + (col & 7) * 2;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o1));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o2));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// BK = pixel rows per k-tile (64, or 32: half the LDS, twice the workgroups per CU)
// PRO: the B (input) fragments hold one channel per lane (column lane & 15 of the 16-wide
// subtile), so the BN prologue is one (scale, shift) register pair per subtile for the whole
// kernel.  Zero-page rows turn into relu(shift) but meet zero dY rows.
__device__ __forceinline__ void pro_frag(bf16x8& f, float sc, float sh) {
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = f2bf(fmaxf(bf2f(f[e]) * sc + sh, 0.f));
}

template <int BK, bool PRO = false>
__global__ void __launch_bounds__(256, 3)
wgrad_kernel(const WgradParams p) {
  constexpr int IMG = BK * 256;   // BK rows x 128 bf16
  constexpr int STAGE = 2 * IMG;
  constexpr int SL = BK / 16;     // LDS-DMA instructions per thread per image
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = (p.Co + 127) / 128;
  const int ntn = (p.ldw + 127) / 128;
  // 1-D grid over (split, tile): consecutive logical ids -- the tiles of one split, which
  // share its dY rows and input pixels -- land on the same XCD (one L2), so each XCD
  // streams its own contiguous range of rows from HBM once
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t split = lid / (ntm * ntn), tile = lid % (ntm * ntn);
  const int tn = tile % ntn, tmi = tile / ntn;
  const int co0 = tmi * 128, kcol0 = tn * 128;
  const int mstart = split * p.rows_per_split;
  const int mend = min(p.M, mstart + p.rows_per_split);
  const int nkt = (mend - mstart + BK - 1) / BK;

  // per-thread load slots: SL per image; wave instruction i covers rows (wave*SL+i)*4 .. +3
  uint32_t a_col[SL];
  bool a_cok[SL];
  int b_dy[SL], b_dx[SL];
  uint32_t b_ci[SL];
  bool b_cok[SL];
#pragma unroll
  for (int i = 0; i < SL; ++i) {
    const uint32_t r = (wave * SL + i) * 4 + (lane >> 4);
    const uint32_t c = (lane & 15) ^ (((r & 3u) << 1) | (((r >> 3) & 1u) << 3));
    a_col[i] = co0 + c * 8;
    a_cok[i] = (int)a_col[i] < p.Co;
    const int kc = kcol0 / 8 + c;
    b_cok[i] = kc < p.kc_total;
    const int t = b_cok[i] ? (int)fdiv(kc, p.div_cpt) : 0;
    b_ci[i] = (kc - t * p.cpt) * 8;
    b_dy[i] = p.dy_t[t];
    b_dx[i] = p.dx_t[t];
  }

  auto stage = [&](int kt, int buf) {
    char* Ai = smem + buf * STAGE;
    char* Bi = Ai + IMG;
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      const int r = (wave * SL + i) * 4 + (lane >> 4);
      const int m = mstart + kt * BK + r;
      const bool mok = m < mend;
      const bf16* ga = (mok && a_cok[i]) ? p.dy + (size_t)m * p.Co + a_col[i] : p.zero;
      dma16(ga, Ai + (wave * SL + i) * 1024);
      const bf16* gb;
      if (p.direct) {  // 1x1 stride 1: input pixel m is GEMM row m (no decode)
        gb = (mok && b_cok[i]) ? p.src + (size_t)m * p.Cs + b_ci[i] : p.zero;
      } else {
        const uint32_t mm = mok ? m : 0;
        const uint32_t q = fdiv(mm, p.div_wo);
        const uint32_t x = mm - q * p.Wo;
        const uint32_t n = fdiv(q, p.div_ho);
        const uint32_t y = q - n * p.Ho;
        const int hi = (int)y * p.ss + b_dy[i], wi = (int)x * p.ss + b_dx[i];
        const bool ok = mok && b_cok[i] && (unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws;
        gb = ok ? p.src + ((size_t)(n * p.Hs + hi) * p.Ws + wi) * p.Cs + b_ci[i] : p.zero;
      }
      dma16(gb, Bi + (wave * SL + i) * 1024);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float psc[4], psh[4];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = min(kcol0 + wn * 64 + j * 16 + (lane & 15), p.Cs - 1);
      psc[j] = p.pscale[c];
      psh[j] = p.pshift[c];
    }
  }

  if (nkt > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) stage(kt + 1, buf ^ 1);
    const char* Ai = smem + buf * STAGE;
    const char* Bi = Ai + IMG;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const uint32_t row0 = s * 32 + 8 * (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr_frag(Ai, row0, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = tr_frag(Bi, row0, wn * 64 + j * 16, lane);
      if constexpr (PRO)
#pragma unroll
        for (int j = 0; j < 4; ++j) pro_frag(bfr[j], psc[j], psh[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nkt == 0) return;

  // D[co][kcol]: lane holds rows (lane>>4)*4+r, column lane&15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kcol = kcol0 + wn * 64 + j * 16 + (lane & 15);
      if (kcol >= p.ldw) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (co < p.Co && !(p.ablate & 8)) {
          if (p.part) p.part[((size_t)split * p.Co + co) * p.ldw + kcol] = acc[i][j][r];
          else unsafeAtomicAdd(p.dw + (size_t)co * p.ldw + kcol, acc[i][j][r]);
        }
      }
    }
  }
}

// 256 x 256 weight-gradient tile (8 waves, each 64 co x 128 cols): half the LDS-DMA
// and transposed-read instructions per MFMA of the 128 x 128 kernel above; images are
// [64 pixels][256 bf16] (512-byte rows) with the same 32-byte-piece XOR swizzle.
__device__ __forceinline__ uint32_t swz512(uint32_t r, uint32_t c) {
  return r * 512u + ((c ^ (((r & 3u) << 1) | (((r >> 3) & 1u) << 3))) << 4);
}

__device__ __forceinline__ bf16x8 tr_frag512(const char* img, uint32_t row0, uint32_t col0, int lane) {
  const uint32_t q = (lane & 15) >> 2, pp = lane & 3;
  const uint32_t col = col0 + pp * 4;
  const uint32_t o1 = swz512(row0 + q, col >> 3) + (col & 7) * 2;
  const uint32_t o2 = swz512(row0 + 4 + q, col >> 3) + (col & 7) * 2;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o1));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o2));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <bool PRO = false>
__global__ void __launch_bounds__(512)
wgrad256_kernel(const WgradParams p) {
  constexpr int BK = 64;
  constexpr int IMG = BK * 512;   // 64 rows x 256 bf16
  constexpr int STAGE = 2 * IMG;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;   // 64-co group, 128-col group
  const int ntm = (p.Co + 255) / 256;
  const int ntn = (p.ldw + 255) / 256;
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);  // see wgrad_kernel
  const uint32_t split = lid / (ntm * ntn), tile = lid % (ntm * ntn);
  const int tn = tile % ntn, tmi = tile / ntn;
  const int co0 = tmi * 256, kcol0 = tn * 256;
  const int mstart = split * p.rows_per_split;
  const int mend = min(p.M, mstart + p.rows_per_split);
  const int nkt = (mend - mstart + BK - 1) / BK;

  // load slots: 4 per image per thread; wave instruction i covers rows (wave*4+i)*2 .. +1
  uint32_t a_col[4];
  bool a_cok[4];
  int b_dy[4], b_dx[4];
  uint32_t b_ci[4];
  bool b_cok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t r = (wave * 4 + i) * 2 + (lane >> 5);
    const uint32_t c = (lane & 31) ^ (((r & 3u) << 1) | (((r >> 3) & 1u) << 3));
    a_col[i] = co0 + c * 8;
    a_cok[i] = (int)a_col[i] < p.Co;
    const int kc = kcol0 / 8 + c;
    b_cok[i] = kc < p.kc_total;
    const int t = b_cok[i] ? (int)fdiv(kc, p.div_cpt) : 0;
    b_ci[i] = (kc - t * p.cpt) * 8;
    b_dy[i] = p.dy_t[t];
    b_dx[i] = p.dx_t[t];
  }

  auto stage = [&](int kt, int buf) {
    char* Ai = smem + buf * STAGE;
    char* Bi = Ai + IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave * 4 + i) * 2 + (lane >> 5);
      const int m = mstart + kt * BK + r;
      const bool mok = m < mend;
      const bf16* ga = (mok && a_cok[i]) ? p.dy + (size_t)m * p.Co + a_col[i] : p.zero;
      dma16(ga, Ai + (wave * 4 + i) * 1024);
      const bf16* gb;
      if (p.direct) {  // 1x1 stride 1: input pixel m is GEMM row m (no decode)
        gb = (mok && b_cok[i]) ? p.src + (size_t)m * p.Cs + b_ci[i] : p.zero;
      } else {
        const uint32_t mm = mok ? m : 0;
        const uint32_t q = fdiv(mm, p.div_wo);
        const uint32_t x = mm - q * p.Wo;
        const uint32_t n = fdiv(q, p.div_ho);
        const uint32_t y = q - n * p.Ho;
        const int hi = (int)y * p.ss + b_dy[i], wi = (int)x * p.ss + b_dx[i];
        const bool ok = mok && b_cok[i] && (unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws;
        gb = ok ? p.src + ((size_t)(n * p.Hs + hi) * p.Ws + wi) * p.Cs + b_ci[i] : p.zero;
      }
      dma16(gb, Bi + (wave * 4 + i) * 1024);
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // PRO: (scale, shift) pairs in LDS behind the two stages -- 16 more registers per lane would
  // spill this 254-register kernel; read back per k-step (visible after the first barrier)
  float* pro_tbl = (float*)(smem + 2 * STAGE);
  if constexpr (PRO) {
    for (int i = tid; i < p.Cs; i += 512) {
      pro_tbl[2 * i] = p.pscale[i];
      pro_tbl[2 * i + 1] = p.pshift[i];
    }
  }

  if (nkt > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) stage(kt + 1, buf ^ 1);
    const char* Ai = smem + buf * STAGE;
    const char* Bi = Ai + IMG;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t row0 = s * 32 + 8 * (lane >> 4);
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr_frag512(Ai, row0, wm * 64 + i * 16, lane);
      if constexpr (PRO) {
        // input fragments in two halves of 4 (the transform's temporaries fit beside them)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bf16x8 bh[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * h + jj;
            bh[jj] = tr_frag512(Bi, row0, wn * 128 + j * 16, lane);
            const int c = min(kcol0 + wn * 128 + j * 16 + (lane & 15), p.Cs - 1);
            const f32x2 t = *LDS_PTR(const f32x2, pro_tbl + 2 * c);
            pro_frag(bh[jj], t[0], t[1]);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              acc[i][4 * h + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bh[jj], acc[i][4 * h + jj], 0, 0, 0);
        }
      } else {
        bf16x8 bfr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bfr[j] = tr_frag512(Bi, row0, wn * 128 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nkt == 0) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kcol = kcol0 + wn * 128 + j * 16 + (lane & 15);
      if (kcol >= p.ldw) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (co < p.Co) {
          if (p.part) p.part[((size_t)split * p.Co + co) * p.ldw + kcol] = acc[i][j][r];
          else unsafeAtomicAdd(p.dw + (size_t)co * p.ldw + kcol, acc[i][j][r]);
        }
      }
    }
  }
}

// 64 x 256 weight-gradient tile for Co <= 64 (the stem, stage-1 layers): the 128-row tiles
// above leave half of every MFMA on zero rows there.  4 waves, each 64 co x 64 cols; the dY
// image is [64 pixels][64 co] (128-byte rows), the im2col image [64 pixels][256 cols].
// 128-byte rows put two rows in each 256-byte bank window, so the 32-byte pieces a
// ds_read_b64_tr_b16 half-wave reads from rows {r..r+3, r+8..r+11} are spread by XOR-ing
// the piece index with row bits 1 and 3 (conflict-free; chunk pairs stay adjacent).
__device__ __forceinline__ uint32_t swz128tr(uint32_t r, uint32_t c) {
  return r * 128u + ((c ^ ((((r >> 1) & 1u) | (((r >> 3) & 1u) << 1)) << 1)) << 4);
}

__device__ __forceinline__ bf16x8 tr_frag128(const char* img, uint32_t row0, uint32_t col0, int lane) {
  const uint32_t q = (lane & 15) >> 2, pp = lane & 3;
  const uint32_t col = col0 + pp * 4;
  const uint32_t o1 = swz128tr(row0 + q, col >> 3) + (col & 7) * 2;
  const uint32_t o2 = swz128tr(row0 + 4 + q, col >> 3) + (col & 7) * 2;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o1));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + o2));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// NJ: 16-column subtiles per wave -- tiles of 64 NJ columns (4: 256; 3: 192, which covers the
// 576 columns of a 3x3 conv over 64 channels in three full tiles instead of 2.25 tiles of 256).
// The im2col image keeps its 512-byte row pitch; chunks past the tile are never loaded.
template <int BK, int NJ>
__global__ void __launch_bounds__(256, 3)
wgrad64_kernel(const WgradParams p) {
  constexpr int TW = 64 * NJ;     // columns per tile
  constexpr int IMGA = BK * 128;  // BK pixels x 64 co
  constexpr int IMGB = BK * 512;  // BK pixels x (256-column pitch)
  constexpr int STAGE = IMGA + IMGB;
  constexpr int SA = BK / 32, SB = BK / 8;  // LDS-DMA instructions per thread: dY / im2col image
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (p.ldw + TW - 1) / TW;
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);  // see wgrad_kernel
  const uint32_t split = lid / ntn;
  const int tn = lid % ntn;
  const int kcol0 = tn * TW;
  const int mstart = split * p.rows_per_split;
  const int mend = min(p.M, mstart + p.rows_per_split);
  const int nkt = (mend - mstart + BK - 1) / BK;

  // dY image: SA LDS-DMA instructions per thread, instruction i covers rows (wave*SA+i)*8 .. +7
  uint32_t a_col[SA];
  bool a_cok[SA];
#pragma unroll
  for (int i = 0; i < SA; ++i) {
    const uint32_t r = (wave * SA + i) * 8 + (lane >> 3);
    const uint32_t c = (lane & 7) ^ ((((r >> 1) & 1u) | (((r >> 3) & 1u) << 1)) << 1);
    a_col[i] = c * 8;
    a_cok[i] = (int)a_col[i] < p.Co;
  }
  // im2col image: SB instructions per thread, instruction i covers rows (wave*SB+i)*2 .. +1
  int b_dy[SB], b_dx[SB];
  uint32_t b_ci[SB];
  bool b_cok[SB], b_in[SB];
#pragma unroll
  for (int i = 0; i < SB; ++i) {
    const uint32_t r = (wave * SB + i) * 2 + (lane >> 5);
    const uint32_t c = (lane & 31) ^ (((r & 3u) << 1) | (((r >> 3) & 1u) << 3));
    const int kc = kcol0 / 8 + c;
    b_in[i] = c < 8 * NJ;
    b_cok[i] = b_in[i] && kc < p.kc_total;
    const int t = b_cok[i] ? (int)fdiv(kc, p.div_cpt) : 0;
    b_ci[i] = (kc - t * p.cpt) * 8;
    b_dy[i] = p.dy_t[t];
    b_dx[i] = p.dx_t[t];
  }

  auto stage = [&](int kt, int buf) {
    char* Ai = smem + buf * STAGE;
    char* Bi = Ai + IMGA;
#pragma unroll
    for (int i = 0; i < SA; ++i) {
      const int r = (wave * SA + i) * 8 + (lane >> 3);
      const int m = mstart + kt * BK + r;
      const bf16* ga = (m < mend && a_cok[i]) ? p.dy + (size_t)m * p.Co + a_col[i] : p.zero;
      dma16(ga, Ai + (wave * SA + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int r = (wave * SB + i) * 2 + (lane >> 5);
      const int m = mstart + kt * BK + r;
      const bool mok = m < mend;
      const bf16* gb;
      if (p.direct) {  // 1x1 stride 1: input pixel m is GEMM row m (no decode)
        gb = (mok && b_cok[i]) ? p.src + (size_t)m * p.Cs + b_ci[i] : p.zero;
      } else {
        const uint32_t mm = mok ? m : 0;
        const uint32_t q = fdiv(mm, p.div_wo);
        const uint32_t x = mm - q * p.Wo;
        const uint32_t n = fdiv(q, p.div_ho);
        const uint32_t y = q - n * p.Ho;
        const int hi = (int)y * p.ss + b_dy[i], wi = (int)x * p.ss + b_dx[i];
        const bool ok = mok && b_cok[i] && (unsigned)hi < (unsigned)p.Hs && (unsigned)wi < (unsigned)p.Ws;
        gb = ok ? p.src + ((size_t)(n * p.Hs + hi) * p.Ws + wi) * p.Cs + b_ci[i] : p.zero;
      }
      if (NJ == 4 || b_in[i])
        dma16(gb, Bi + (wave * SB + i) * 1024);
    }
  };

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nkt > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) stage(kt + 1, buf ^ 1);
    const char* Ai = smem + buf * STAGE;
    const char* Bi = Ai + IMGA;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const uint32_t row0 = s * 32 + 8 * (lane >> 4);
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr_frag128(Ai, row0, i * 16, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = tr_frag512(Bi, row0, wave * 16 * NJ + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nkt == 0) return;

#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int kcol = kcol0 + wave * 16 * NJ + j * 16 + (lane & 15);
      if (kcol >= p.ldw) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + (lane >> 4) * 4 + r;
        if (co < p.Co) {
          if (p.part) p.part[((size_t)split * p.Co + co) * p.ldw + kcol] = acc[i][j][r];
          else unsafeAtomicAdd(p.dw + (size_t)co * p.ldw + kcol, acc[i][j][r]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
template <int BN, int EPI, bool FAST, int NS, int BK = 64, bool PRO = false>
static void launch_tg(TapGemmParams p, int grid, hipStream_t stream) {
  p.nkt = (p.ntaps * p.cpt + BK / 8 - 1) / (BK / 8);
  // LDS: the stages the k-loop actually uses (short-K shapes -- 1x1 convs with 64 input
  // channels -- need one, which lets more workgroups share a CU) or the epilogue image
  const size_t stage = (size_t)(128 + BN) * BK * 2;
  const size_t full = (size_t)NS * stage;
  size_t epi = 0;
  if (EPI == 0) epi = (size_t)128 * 2 * BN;
  if (EPI == 1) epi = (size_t)128 * 2 * BN;  // tile_stats128_vv keeps its scratch inside the image
  // image, then the sums' [2][8][256 + 4] fp32 in its space
  if (EPI == 3 || EPI == 4) epi = std::max((size_t)128 * 2 * BN, (size_t)2 * 8 * 260 * 4);
  size_t lds = std::max((size_t)std::min(NS, std::max(p.nkt, 1)) * stage, epi);
  if (!FAST) lds = std::max(lds, full + kMaxTaps * sizeof(int));  // LDS tap table behind the stages
  // BN-prologue (scale, shift) table behind the stages in use
  if (PRO) lds = std::max(lds, (size_t)std::min(NS, std::max(p.nkt, 1)) * stage + (size_t)p.Cs * 2 * sizeof(float));
  if (full > 64 * 1024) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)tap_gemm_kernel<BN, EPI, FAST, NS, BK, PRO>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)full);
      if constexpr (BN == 64 && FAST && !PRO && NS <= 3)
        (void)hipFuncSetAttribute((const void*)tap_gemm_kernel<BN, EPI, FAST, NS, BK, PRO, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)full);
      attr = true;
    }
  }
  p.kmode = 0;
  p.kp = nullptr;
  // split-K (tg_split_slices): the 64-channel FAST tiles with <= 3 stages, the configurations the
  // short grids it applies to run (the heuristic picks 64-channel tiles there)
  if constexpr (BN == 64 && FAST && !PRO && NS <= 3) {
    if (p.ksplit > 1 && g_ws_alloc != nullptr) {
      const size_t bytes = (size_t)p.ksplit * grid * (BN / 32) * 4 * 256 * sizeof(f32x4);
      void* ws = g_ws_alloc(bytes, stream);
      if (ws != nullptr) {
        p.kp = (f32x4*)ws;
        p.kmode = 1;
        hipLaunchKernelGGL((tap_gemm_kernel<BN, EPI, FAST, NS, BK, PRO, true>), dim3(grid, p.ksplit), dim3(256), lds,
                           stream, p);
        p.kmode = 2;
        hipLaunchKernelGGL((tap_gemm_kernel<BN, EPI, FAST, NS, BK, PRO, true>), dim3(grid), dim3(256), lds, stream, p);
        g_ws_free(ws);  // stream-ordered: reused only by later work on this stream
        return;
      }
    }
  }
  hipLaunchKernelGGL((tap_gemm_kernel<BN, EPI, FAST, NS, BK, PRO>), dim3(grid), dim3(256), lds, stream, p);
}

template <int WM, int WN, int NS, int CFW = 4>
static void launch_big(TapGemmParams p, int epi, hipStream_t stream) {
  // the 8-wave tile runs the ping-pong schedule by default (tg_big_cvar: 1 = the lockstep
  // schedule, 2 = fragments read after the barrier, 3 = ping-pong); 3-6 % faster on the R50
  // shapes the 256 x 256 tile takes (profiles/r5/pingpong_ab_b1024.txt)
  if (WM * WN == 8) p.cvar = p.cvar == 0 ? 3 : (p.cvar == 1 ? 0 : p.cvar);
  else if (p.cvar == 1) p.cvar = 0;
  constexpr int BM = 128 * WM, BN = 16 * CFW * WN;
  constexpr size_t lds = std::max((size_t)NS * (BM + BN) * 64, (size_t)WM * (BN / 128) * 32768);
  const int tiles = ((p.M + BM - 1) / BM) * ((p.Co + BN - 1) / BN);
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  int grid = p.persist ? std::min(tiles, ncu) : tiles;
  // stream-K: one workgroup per CU slot (LDS-limited: 1 per CU for 256 x 256, 2 for 256 x 128), at
  // most one tile's worth of ranges per workgroup boundary -> needs tiles >= slots
  p.sk_ws = nullptr;
  p.sk_flags = nullptr;
  void* ws = nullptr;
  const int per_cu = std::max(1, (int)(160 * 1024 / lds));
  const int slots = p.sk_on >= 3 ? std::min(p.sk_on, ncu * per_cu) : ncu * per_cu;
  // range granularity: the divisor u >= 8 of nkt (or nkt itself) that minimises the longest range,
  // ceil(tiles * nkt / u / slots) * u k-steps; every range must still cover a whole tile's k-steps
  // (a tile is then cut between at most two workgroups)
  p.sk_unit = 0;
  if (p.sk_on && tiles >= slots && (long)tiles * p.nkt < (1l << 31)) {
    long best = -1;
    for (int u = 1; u <= p.nkt; ++u) {
      if (p.nkt % u != 0 || (u < 8 && u != p.nkt)) continue;
      const long U = (long)tiles * (p.nkt / u);
      if ((U / slots) * u < p.nkt) continue;
      const long longest = (U + slots - 1) / slots * u;
      if (best < 0 || longest <= best) {
        best = longest;
        p.sk_unit = u;
      }
    }
  }
  if (p.sk_unit > 0 && g_ws_alloc != nullptr) {
    const size_t flag_bytes = ((size_t)slots * 4 + 255) / 256 * 256;
    const size_t part_bytes = (size_t)slots * (64 * WM * WN) * CFW * 8 * 16;  // per lane: CFW x 8 f32x4
    ws = g_ws_alloc(flag_bytes + part_bytes, stream);
    if (ws != nullptr) {
      p.sk_flags = (uint32_t*)ws;
      p.sk_ws = (f32x4*)((char*)ws + flag_bytes);
      (void)hipMemsetAsync(ws, 0, flag_bytes, stream);
      grid = slots;
    }
  }
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)tap_gemm_big_kernel<WM, WN, NS, 0, CFW>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)tap_gemm_big_kernel<WM, WN, NS, 1, CFW>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)tap_gemm_big_loop_kernel<WM, WN, NS, 0, CFW>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)tap_gemm_big_loop_kernel<WM, WN, NS, 1, CFW>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const bool loop = p.persist || p.sk_ws != nullptr;
  const dim3 blk(64 * WM * WN);
  if (epi == 1) {
    if (loop) hipLaunchKernelGGL((tap_gemm_big_loop_kernel<WM, WN, NS, 1, CFW>), dim3(grid), blk, lds, stream, p);
    else hipLaunchKernelGGL((tap_gemm_big_kernel<WM, WN, NS, 1, CFW>), dim3(grid), blk, lds, stream, p);
  } else {
    if (loop) hipLaunchKernelGGL((tap_gemm_big_loop_kernel<WM, WN, NS, 0, CFW>), dim3(grid), blk, lds, stream, p);
    else hipLaunchKernelGGL((tap_gemm_big_kernel<WM, WN, NS, 0, CFW>), dim3(grid), blk, lds, stream, p);
  }
  if (ws != nullptr) g_ws_free(ws);  // stream-ordered: reused only by later work on this stream
}

// 0 = the 128-row kernels, 1 = 256 x 256 big tile, 2 = 256 x 128 big tile.  mode = g_tune[kTgBig]
// (0 = this heuristic).  Per-shape A/B at b1024 (profiles/r3/big_tile_ab_b1024_pipelined.txt): the
// big tiles win where the 128-row kernels' grid is short or their k-loop is exposed, and lose on
// the 1x1 stride-1 shapes and the 256-channel 3x3s (784 256 x 256 tiles = 3.06 rounds of 256 CUs):
//   * stride-2 data-gradient parity classes (ds = 2), 256 x 128: 128 ch 3x3 581 -> 497 us,
//     256 ch 3x3 374 -> 348, 1x1 1024 -> 2048 377 -> 323;
//   * 3x3 with 128 output channels, 256 x 128: 28x28 fwd 307 -> 285, dgrad 288 -> 274, the
//     stride-2 fwd 369 -> 349;
//   * 3x3 with >= 512 output channels (the 7x7 outputs), 256 x 256: 257 -> 247 fwd, 253 -> 244 dgrad.
// Only where the big-tile grid still fills the chip (>= 256 tiles): at batch 32 the 7x7 3x3
// convs are 14 256 x 256 tiles (122 us against the 128-row kernel's 52-workgroup grid).
static int big_tile_pick(int mode, int M, int Co, int ntaps, int ds) {
  if (mode == 2) return 0;
  if (mode == 1) return Co >= 256 ? 1 : 2;
  if (mode == 3) return 2;
  int pick = 0;
  if (ds == 2) pick = 2;
  else if (ntaps == 9 && Co == 128) pick = 2;
  else if (ntaps == 9 && Co >= 512) pick = 1;
  const long tiles = (long)((M + 255) / 256) * ((Co + (pick == 1 ? 255 : 127)) / (pick == 1 ? 256 : 128));
  return pick != 0 && tiles >= 256 ? pick : 0;
}

// Split-K of the 128-row kernels: a grid under half a round of 256 CUs with a deep k-loop -- at batch
// 16-32 the 7x7 3x3 convs (104 workgroups x 72 k-tiles), the deep-K 1x1 convs of stage 4 and the
// linear heads run one long latency-bound k-loop per workgroup.  ksplit slices of >= 8 64-deep units
// (~2 rounds of workgroups), then one reduce launch sums the slices in order and runs the epilogue.
// (Measured: grids < 256 tiles and ~3 rounds 1.5 % slower at R50 b32; < 512 and slices of 4 units 8 %
// slower -- profiles/r6/split_k_width_ab_s37_s38.txt.)
// Decided on canonical 64-channel tiles and 64-deep units, so every 128-row configuration (tile
// width, k depth, stages) sums the same slices: the autotuner's candidates stay bitwise equal (the
// big tiles, which do not split, are not candidates where this applies).
// g_tune[kTgSplitK]: 2 off, >= 3 exactly that many slices (A/B), 0 the heuristic.
static int tg_split_slices(int M, int Co, int K) {
  if (g_tune[kTgSplitK] == 2) return 0;
  const int k64 = (K + 63) / 64;
  const long grid_c = (long)((M + 127) / 128) * ((Co + 63) / 64);
  int ks = 0;
  if (g_tune[kTgSplitK] >= 3) ks = g_tune[kTgSplitK];
  else if (g_tune[kTgSplitK] == 1) {  // (A/B) one round of slices
    if (grid_c < 128 && k64 >= 16) ks = (int)std::min<long>(k64 / 8, (256 + grid_c - 1) / grid_c);
  } else if (grid_c < 128 && k64 >= 16) ks = (int)std::min<long>(k64 / 8, (512 + grid_c - 1) / grid_c);
  if (ks > k64) ks = k64;
  return ks >= 2 ? ks : 0;
}

static void tap_gemm_impl(const bf16* src, int N, int Hs, int Ws, int Cs,
                          const bf16* wt, int Co, int T,
                          bf16* dst, int Hd, int Wd, int Hy, int Wy, int ss, int ds, int oy, int ox,
                          const TapList& taps, float* stats, const float* bias, int relu,
                          const bf16* zero, hipStream_t stream, const bf16* addsrc, const BnBwdEpi* bnb,
                          const AffineEpi* aff, const float* pscale, const float* pshift, int nbias) {
  TapGemmParams p;
  p.pscale = pscale;
  p.pshift = pshift;
  p.src = src; p.wt = wt; p.dst = dst; p.stats = stats; p.zero = zero; p.addsrc = addsrc;
  p.fscale = aff ? aff->scale : nullptr;
  p.fshift = aff ? aff->shift : nullptr;
  p.fact = aff ? aff->act : 0;
  p.fslope = aff ? aff->slope : 0.f;
  if (aff != nullptr && (stats != nullptr || bias != nullptr || relu != 0 || bnb != nullptr)) {
    fprintf(stderr, "launch_tap_gemm: the folded BN epilogue is a plain forward store\n");
    abort();
  }
  p.bnb = bnb ? *bnb : BnBwdEpi{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0.f, 0, 0, 0};
  p.Hs = Hs; p.Ws = Ws; p.Cs = Cs;
  p.Hy = Hy; p.Wy = Wy; p.ss = ss;
  p.Hd = Hd; p.Wd = Wd; p.ds = ds; p.oy = oy; p.ox = ox;
  p.Co = Co; p.T = T; p.M = N * Hy * Wy;
  p.ntaps = taps.n; p.cpt = Cs / 8; p.ldw = T * Cs;
  p.nkt = (taps.n * p.cpt + 7) / 8;
  p.relu = relu; p.bias = bias; p.nbias = (nbias > 0 && nbias < Co) ? nbias : Co;
  p.div_wy = make_fastdiv(Wy); p.div_hy = make_fastdiv(Hy); p.div_cpt = make_fastdiv(p.cpt);
  for (int i = 0; i < taps.n; ++i)
    p.tap[i] = (taps.dy[i] & 0xff) | ((taps.dx[i] & 0xff) << 8) | ((taps.widx[i] & 0xffff) << 16);
  if (p.M == 0) return;
  const int ntm = (p.M + 127) / 128;
  int epi = (bias != nullptr || relu != 0) ? 2 : (stats != nullptr ? 1 : 0);
  if (bnb != nullptr) {
    if (ds != 1 || Hd != Hy || Wd != Wy || stats != nullptr || bias != nullptr || relu != 0) {
      fprintf(stderr, "launch_tap_gemm: fused BN backward needs a plain stride-1 dgrad\n");
      abort();
    }
    epi = bnb->mask != nullptr ? 4 : 3;
  }
  const bool fast = (p.cpt & 7) == 0 && taps.n <= 32;  // FAST: 32-bit tap-validity masks
  // config: BN (64/128 output channels per tile) and NS (LDS stages); g_tune overrides the
  // heuristic (tuning experiments only)
  const int env_bn = g_tune[kTgTileN], env_ns = g_tune[kTgStages];
  p.ablate = g_tune[kAblate];
  p.cvar = g_tune[kTgBigCvar];
  p.persist = g_tune[kTgBigPersist];
  // (values >= 3: stream-K over exactly that many workgroups -- tests on small shapes)
  p.sk_on = g_tune[kTgBigSK] == 1 ? 1 : (g_tune[kTgBigSK] >= 3 ? g_tune[kTgBigSK] : 0);
  p.sk_ws = nullptr;
  p.sk_flags = nullptr;
  p.ksplit = tg_split_slices(p.M, Co, taps.n * Cs);  // (the 128-row kernels; tile widths 64 / 128 / 256)
  p.k64 = (taps.n * Cs + 63) / 64;
  p.kp = nullptr;
  p.kmode = 0;
  int bn = Co <= 64 ? 64 : 128, ns = 2;
  // a short grid (< 1.5 rounds of 256 CUs at 128-channel tiles: batch 32-128 from stage 2 on, the
  // stride-2 parity classes, the linear heads) takes 64-channel tiles, twice the workgroups: the
  // per-shape autotuner (DCP_AUTOTUNE) picked them on every such ResNet-50 shape at batch 32
  // (4,616 -> 4,939 img/s), e.g. the 7x7 512-channel 3x3 convs 52 -> 104 workgroups
  if (bn == 128 && fast && (long)ntm * ((Co + 127) / 128) < 384) bn = 64;
  if (env_bn > 0 && fast) bn = env_bn;
  if (env_ns > 0 && fast) ns = env_ns;
  if (!fast) ns = 2;
  // 1x1 shapes with K <= 1024 and 128-channel tiles: 32-deep k-tiles, double-buffered (32 KB of
  // LDS: four workgroups per CU) beat the 64-deep double buffer (two per CU) by 5-25 % and the
  // 32-deep 3-stage ring by 2-12 %; 3x3 and deep-K shapes keep 64-deep tiles (tools/conv_bench.py
  // --cfgs "1=2;8=32,1=3;8=32" per-shape A/B).  g_tune[kTgKDepth] = 32 forces 32-deep tiles (with [1]),
  // 64 disables the heuristic.
  // narrow-channel (non-FAST) shapes -- the space-to-depth stem -- take 32-deep tiles double-
  // buffered only (their taps are looked up per lane; g_tune[kNarrowKDepth] = 32 / 64 selects, A/B)
  bool bk32 = (fast && g_tune[kTgKDepth] == 32 && ns >= 2 && ns <= 4) || (!fast && g_tune[kNarrowKDepth] == 32);
  // (K = 64, one 64-deep k-tile, measured faster with the 64-deep tile: 487 vs 511 us on the R50
  // stage-1 expansion at b1024, tools/fwd_epi_bench.py)
  if (fast && env_ns == 0 && g_tune[kTgKDepth] != 64 && taps.n == 1 && Cs > 64 && Cs <= 1024 && bn == 128) bk32 = true;
  // big-tile kernel (tap_gemm_big_kernel): FAST, plain / statistics epilogue, >= 128 output
  // channels.  g_tune[kTgBig]: 1 = on wherever it applies (256 x 256 for Co >= 256, else 256 x 128),
  // 3 = 256 x 128 only, 2 = off, 0 = heuristic (big_tile_pick)
  // weight-stationary persistent kernel (conv_ws.hip) for plain 1x1 stride-1 GEMMs with K <= 256:
  // g_tune[kTgWs] = 1 on wherever it applies (the autotuner's candidate), 2 off, 0 = heuristic (off)
  const bool plain1x1 = fast && (epi == 0 || epi == 1) && taps.n == 1 && taps.dy[0] == 0 && taps.dx[0] == 0 &&
                        taps.widx[0] == 0 && ss == 1 && ds == 1 && oy == 0 && ox == 0 && Hd == Hy && Wd == Wy &&
                        Hs == Hy && Ws == Wy && T == 1 && addsrc == nullptr && aff == nullptr && bnb == nullptr &&
                        pscale == nullptr && bias == nullptr && relu == 0;
  if (g_tune[kTgWs] == 1 && plain1x1 && conv1x1_ws_supported(Cs, Co, p.M)) {
    if (p.ablate == 0 && launch_conv1x1_ws(src, wt, T * Cs, dst, stats, zero, p.M, Cs, Co, stream)) return;
  }
  // store-decoupled loader / consumer 1x1 kernel (conv1x1_ps.hip): g_tune[kTgPs] = 1 on wherever it
  // applies with 4 consumer waves, 3 with 8 (autotuner candidates), 2 off, 0 = heuristic (off)
  if ((g_tune[kTgPs] == 1 || g_tune[kTgPs] == 3) && plain1x1 && conv1x1_ps_supported(Cs, Co, p.M)) {
    if (launch_conv1x1_ps(src, wt, T * Cs, dst, stats, zero, p.M, Cs, Co, p.ablate, g_tune[kTgPs] == 3 ? 8 : 4,
                          stream))
      return;
  }
  const bool big_ok = fast && taps.n > 0 && (epi == 0 || epi == 1) && bnb == nullptr && pscale == nullptr &&
                      Co >= 128;
  const int big = big_ok ? big_tile_pick(g_tune[kTgBig], p.M, Co, taps.n, ds) : 0;
  if (big != 0) {
    p.nkt = taps.n * p.cpt / 4;  // 32-deep k-tiles (cpt % 8 == 0 on FAST shapes)
    if (big == 1 && g_tune[kTgBigStages] == 5) launch_big<2, 4, 5>(p, epi, stream);
    else if (big == 1) launch_big<2, 4, 4>(p, epi, stream);
    else launch_big<2, 2, 3>(p, epi, stream);
    return;
  }
  // 256-channel tiles (g_tune[kTgTileN] = 256, A/B and autotuner): each wave 64 rows x 128 channels, the
  // A tile read once per 256 output channels -- for the short-K expansion 1x1 convs, whose A reads
  // are half of their bytes at 128-channel tiles.  Plain / statistics epilogue only.
  if (bn == 256 && !(fast && (epi == 0 || epi == 1) && pscale == nullptr && Co > 128)) bn = 128;
  if (bn == 256) {
    // (32-deep k-tiles only: the 64-deep variant spills at the 168-register cap)
    const int grid256 = ntm * ((Co + 255) / 256);
    if (epi == 1) launch_tg<256, 1, true, 2, 32>(p, grid256, stream);
    else launch_tg<256, 0, true, 2, 32>(p, grid256, stream);
    return;
  }
  const int grid = ntm * ((Co + bn - 1) / bn);
  if (pscale != nullptr) {
    // BN prologue on the A operand: 1x1 / stride-1 / FAST, plain or statistics epilogue,
    // double-buffered (the per-channel table is indexed by k-tile)
    if (!(fast && taps.n == 1 && taps.dy[0] == 0 && taps.dx[0] == 0 && ss == 1 && ds == 1 && (epi == 0 || epi == 1) &&
          addsrc == nullptr && aff == nullptr && bnb == nullptr)) {
      fprintf(stderr, "launch_tap_gemm: the BN prologue needs a plain 1x1 stride-1 forward with C %% 64 == 0\n");
      abort();
    }
#define DCP_TG_PRO(BN_)                                                                      \
  if (epi == 1) {                                                                            \
    if (bk32) launch_tg<BN_, 1, true, 2, 32, true>(p, grid, stream);                        \
    else launch_tg<BN_, 1, true, 2, 64, true>(p, grid, stream);                             \
  } else {                                                                                   \
    if (bk32) launch_tg<BN_, 0, true, 2, 32, true>(p, grid, stream);                        \
    else launch_tg<BN_, 0, true, 2, 64, true>(p, grid, stream);                             \
  }
    if (bn == 64) { DCP_TG_PRO(64) } else { DCP_TG_PRO(128) }
#undef DCP_TG_PRO
    return;
  }
#define DCP_TG_NS(BN_, EPI_, FAST_)                                                    \
  if (bk32 && ns == 2) launch_tg<BN_, EPI_, FAST_, 2, 32>(p, grid, stream);             \
  else if (bk32 && ns == 3) launch_tg<BN_, EPI_, (FAST_ || true), 3, 32>(p, grid, stream);  \
  else if (bk32 && ns == 4) launch_tg<BN_, EPI_, (FAST_ || true), 4, 32>(p, grid, stream); \
  else if (ns == 2) launch_tg<BN_, EPI_, FAST_, 2>(p, grid, stream);                   \
  else if (ns == 3) launch_tg<BN_, EPI_, (FAST_ || true), 3>(p, grid, stream);          \
  else launch_tg<BN_, EPI_, (FAST_ || true), 4>(p, grid, stream);
#define DCP_TG_EPI(BN_, FAST_)                     \
  if (epi == 0) { DCP_TG_NS(BN_, 0, FAST_) }       \
  else if (epi == 1) { DCP_TG_NS(BN_, 1, FAST_) }  \
  else if (epi == 3) { DCP_TG_NS(BN_, 3, FAST_) }  \
  else if (epi == 4) { DCP_TG_NS(BN_, 4, FAST_) }  \
  else { DCP_TG_NS(BN_, 2, FAST_) }
  if (bn == 64) {
    if (fast) { DCP_TG_EPI(64, true) } else { DCP_TG_EPI(64, false) }
  } else {
    if (fast) { DCP_TG_EPI(128, true) } else { DCP_TG_EPI(128, false) }
  }
#undef DCP_TG_EPI
#undef DCP_TG_NS
}

// ---------------------------------------------------------------------------
// Per-shape autotuning of the forward / data-gradient GEMM configuration (g_tune[kAutotune] = 1, set
// from DCP_AUTOTUNE=1 by the Python layer; the cudnn.benchmark of this library).  The first call
// of every distinct problem (geometry, channels, taps, epilogue) outside a stream capture times
// the candidate configurations -- the heuristic's choice, 64- vs 32-deep k-tiles, a 3-stage
// ring, 64-channel tiles, the 256 x 128 / 256 x 256 big tiles -- on the real operands (every
// candidate overwrites the same outputs with the same values: each is a pure function of its
// inputs), keeps the fastest and replays it for every later call, captured steps included.
// Every candidate accumulates each output in the same k order, so the conv outputs do not depend
// on the choice; the fused BN statistics / sums of a 64-channel tile add a slab's rows in another
// order (fp32 rounding).  Off by default (the default path is bit-reproducible run to run).
// ---------------------------------------------------------------------------
struct TgCfg {
  int bn, ns, bk, big, cvar, sk, ws, ps;  // tg_tile_n, tg_stages, tg_kdepth, tg_big, tg_big_cvar, tg_big_sk, tg_ws, tg_ps overrides (0 = the heuristic's)
};
static const TgCfg kTgCfgs[] = {
    {0, 0, 0, 0},   // heuristic
    {0, 0, 64, 2},  // 64-deep k-tiles, no big tile
    {0, 2, 32, 2},  // 32-deep k-tiles, double buffer
    {0, 3, 64, 2},  // 3-stage ring of 64-deep k-tiles
    {64, 0, 0, 2},  // 64-channel tiles
    {64, 2, 32, 2}, // 64-channel tiles, 32-deep k-tiles
    {64, 3, 64, 2}, // 64-channel tiles, 3-stage ring
    {0, 4, 64, 2},  // 4-stage ring of 64-deep k-tiles
    {0, 0, 0, 3},   // 256 x 128 big tile
    {0, 0, 0, 1},   // 256 x 256 big tile (Co >= 256)
    {256, 2, 32, 2},  // 256-channel tiles, 32-deep k-tiles (2-3 % on two R50 shapes: profiles/r4/bn256_tile_ab_b1024.txt)
    {0, 0, 0, 1, 1},  // 256 x 256 big tile, lockstep schedule (the ping-pong one is the tile's default)
    {0, 0, 0, 1, 0, 1},  // 256 x 256 big tile, stream-K
    {0, 0, 0, 3, 0, 1},  // 256 x 128 big tile, stream-K
    {0, 0, 0, 2, 0, 0, 0, 1},  // store-decoupled loader / consumer 1x1 kernel (plain 1x1 stride-1, K <= 256)
    {0, 0, 0, 2, 0, 0, 0, 3},  // the same with 8 consumer waves
    // (the weight-stationary persistent 1x1 kernel, g_tune[kTgWs] = 1, is not a candidate: 26-53 %
    // slower on every R50 short-K shape, profiles/r6/ws_1x1_ab_b1024.txt)
    // (the 4-wave 256 x 256 tile, g_tune[kTgBig] = 4, is not a candidate: slower on every R50 shape,
    // profiles/r4/big4_tile_ab_b1024.txt)
};
static std::mutex g_tg_mu;
static std::unordered_map<std::string, int> g_tg_choice;

struct TuneOverride {
  static constexpr int kSlots[8] = {kTgTileN, kTgStages, kTgKDepth, kTgBig, kTgBigCvar, kTgBigSK, kTgWs, kTgPs};
  int saved[8];
  explicit TuneOverride(const TgCfg& c) {
    const int v[8] = {c.bn, c.ns, c.bk, c.big, c.cvar, c.sk, c.ws, c.ps};
    for (int i = 0; i < 8; ++i) {
      saved[i] = g_tune[kSlots[i]];
      g_tune[kSlots[i]] = v[i];
    }
  }
  ~TuneOverride() {
    for (int i = 0; i < 8; ++i) g_tune[kSlots[i]] = saved[i];
  }
};

int tap_gemm_tuned_count() {
  std::lock_guard<std::mutex> lk(g_tg_mu);
  return (int)g_tg_choice.size();
}

// The tuner's decisions as text ("<key>\t<choice>\n" per problem) and back: a tuning cache that
// makes a later process run exactly the kernels an earlier one measured (DCP_TUNE_CACHE, _ext.py) --
// reproducible kernel choices run to run, and profiles without tuning dispatches.  Keys never
// contain tabs or newlines; entries whose choice is out of this build's candidate range are skipped.
std::string tap_gemm_tune_export() {
  std::lock_guard<std::mutex> lk(g_tg_mu);
  std::string out;
  for (const auto& kv : g_tg_choice) out += kv.first + "\t" + std::to_string(kv.second) + "\n";
  return out;
}

int tap_gemm_tune_import(const std::string& text) {
  const int ncfg = (int)(sizeof(kTgCfgs) / sizeof(kTgCfgs[0]));
  std::lock_guard<std::mutex> lk(g_tg_mu);
  int n = 0;
  size_t pos = 0;
  while (pos < text.size()) {
    size_t nl = text.find('\n', pos);
    if (nl == std::string::npos) nl = text.size();
    const std::string line = text.substr(pos, nl - pos);
    pos = nl + 1;
    const size_t tab = line.rfind('\t');
    if (tab == std::string::npos || tab == 0) continue;
    const int c = atoi(line.c_str() + tab + 1);
    if (c < 0 || c >= ncfg) continue;
    g_tg_choice[line.substr(0, tab)] = c;
    ++n;
  }
  return n;
}

void launch_tap_gemm(const bf16* src, int N, int Hs, int Ws, int Cs,
                     const bf16* wt, int Co, int T,
                     bf16* dst, int Hd, int Wd, int Hy, int Wy, int ss, int ds, int oy, int ox,
                     const TapList& taps, float* stats, const float* bias, int relu,
                     const bf16* zero, hipStream_t stream, const bf16* addsrc, const BnBwdEpi* bnb,
                     const AffineEpi* aff, const float* pscale, const float* pshift, int nbias) {
  auto run = [&]() {
    tap_gemm_impl(src, N, Hs, Ws, Cs, wt, Co, T, dst, Hd, Wd, Hy, Wy, ss, ds, oy, ox, taps, stats, bias, relu, zero,
                  stream, addsrc, bnb, aff, pscale, pshift, nbias);
  };
  const bool fast = (Cs % 64) == 0 && taps.n <= 32;
  // only the FAST shapes have alternatives; A/B overrides set by hand win over the tuner
  // (an add source aliasing the output would accumulate over the timing runs: never tuned)
  if (g_tune[kAutotune] != 1 || !fast || pscale != nullptr || g_tune[kTgTileN] || g_tune[kTgStages] || g_tune[kTgKDepth] || g_tune[kTgBig] || g_tune[kTgBigSK] || g_tune[kTgWs] || g_tune[kTgPs] ||
      (long)N * Hy * Wy == 0 || (addsrc != nullptr && addsrc == dst)) {
    run();
    return;
  }
  char kb[512];
  int len = snprintf(kb, sizeof(kb), "%d %d %d %d %d %d %d %d %d %d %d %d %d %d %d|%d%d%d%d%d%d|", N, Hs, Ws, Cs, Co,
                     T, Hd, Wd, Hy, Wy, ss, ds, oy, ox, taps.n, stats != nullptr, bias != nullptr, relu,
                     addsrc != nullptr, bnb ? (bnb->mask ? 2 : 1) : 0, aff != nullptr);
  for (int i = 0; i < taps.n && len < (int)sizeof(kb) - 16; ++i)
    len += snprintf(kb + len, sizeof(kb) - len, "%d,%d,%d;", taps.dy[i], taps.dx[i], taps.widx[i]);
  const std::string key(kb);
  int choice = -1;
  {
    std::lock_guard<std::mutex> lk(g_tg_mu);
    auto it = g_tg_choice.find(key);
    if (it != g_tg_choice.end()) choice = it->second;
  }
  if (choice < 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      run();  // no timing inside a capture: the heuristic (tuned on the eager warm-up steps)
      return;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f, t_heur = 1e30f;
    choice = 0;
    const bool big_ok = bnb == nullptr && aff == nullptr && bias == nullptr && relu == 0 && Co >= 128;
    // where the 128-row kernels split K, the (unsplit) big tiles would sum another way: not candidates
    const bool ksplit = tg_split_slices(N * Hy * Wy, Co, taps.n * Cs) >= 2;
    for (int c = 0; c < (int)(sizeof(kTgCfgs) / sizeof(kTgCfgs[0])); ++c) {
      const TgCfg& cfg = kTgCfgs[c];
      // (those that would not split: big tiles, 128 / 256-channel tiles, the 4-stage ring)
      if (ksplit && (cfg.big == 1 || cfg.big == 3 || cfg.bn == 128 || cfg.bn == 256 || cfg.ns == 4 ||
                     cfg.ws == 1 || cfg.ps != 0))
        continue;
      if (cfg.big == 3 && !big_ok) continue;
      if (cfg.big == 1 && !(big_ok && Co >= 256)) continue;  // (the ping-pong candidate too)
      if (cfg.bn == 256 && !(Co > 128 && bnb == nullptr && bias == nullptr && relu == 0)) continue;
      if (cfg.bn == 64 && Co <= 64 && cfg.ns == 0) continue;  // the heuristic's tile already
      if (cfg.ws == 1 && !(taps.n == 1 && taps.dy[0] == 0 && taps.dx[0] == 0 && ss == 1 && ds == 1 && Hd == Hy &&
                           Wd == Wy && Hs == Hy && Ws == Wy && T == 1 && addsrc == nullptr && aff == nullptr &&
                           bnb == nullptr && bias == nullptr && relu == 0 &&
                           conv1x1_ws_supported(Cs, Co, (long)N * Hy * Wy)))
        continue;  // (the candidate would time the heuristic again)
      if (cfg.ps != 0 && !(taps.n == 1 && taps.dy[0] == 0 && taps.dx[0] == 0 && ss == 1 && ds == 1 && Hd == Hy &&
                           Wd == Wy && Hs == Hy && Ws == Wy && T == 1 && addsrc == nullptr && aff == nullptr &&
                           bnb == nullptr && bias == nullptr && relu == 0 &&
                           conv1x1_ps_supported(Cs, Co, (long)N * Hy * Wy)))
        continue;
      TuneOverride ov(cfg);
      run();  // warm
      float t = 1e30f;
      for (int r = 0; r < 3; ++r) {
        hipEventRecord(e0, stream);
        run();
        hipEventRecord(e1, stream);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        t = std::min(t, ms);
      }
      if (c == 0) {
        t_heur = best = t;
      } else if (t < best && t < 0.98f * t_heur) {  // must beat the heuristic by 2 % to replace it
        best = t;
        choice = c;
      }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    {
      std::lock_guard<std::mutex> lk(g_tg_mu);
      g_tg_choice[key] = choice;
    }
    if (getenv("DCP_AUTOTUNE_LOG"))
      fprintf(stderr, "[dcp-autotune] tap_gemm %s -> cfg %d (%.1f us)\n", key.c_str(), choice, best * 1e3f);
  }
  TuneOverride ov(kTgCfgs[choice]);
  run();  // the outputs of the call itself (the tuning runs already wrote the same values)
}

// Deterministic split-K reduction, two levels: a workgroup sums a chunk of up to 64
// splits for 64 float4 columns (4 sub-lanes per column, 16 independent loads each,
// fixed-order LDS combine), then one pass adds the <= ceil(splits/64) chunk sums.
__global__ void __launch_bounds__(256) split_reduce1_kernel(const float4* __restrict__ part, int splits, int n4,
                                                            float4* __restrict__ out) {
  __shared__ float4 red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  const int k0 = blockIdx.y * 64;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n4) {
#pragma unroll 4
    for (int k = k0 + sub; k < min(splits, k0 + 64); k += 4) {
      const float4 v = part[(size_t)k * n4 + col];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && col < n4) {
    float4 t = red[0][threadIdx.x];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float4 v = red[q][threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    out[(size_t)blockIdx.y * n4 + col] = t;
  }
}

// One launch for a narrow reduction (few columns, up to a few thousand splits: the BN-backward sums
// of a small batch's dgrad epilogue, 2C columns over one partial row per 128-pixel tile): a
// 1024-thread workgroup per 16 float4 columns -- 64 row streams (4 per wave), 8 loads in flight each,
// then a fixed-order two-level combine of the streams in LDS: deterministic, no second launch.  (64
// columns per workgroup left a 256-channel layer's sums on two CUs, each reading ~800 KB at batch 32.)
__global__ void __launch_bounds__(1024) split_reduce_rows_kernel(const float4* __restrict__ part, int splits, int n4,
                                                                 float4* __restrict__ out) {
  __shared__ float4 red[64][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cl = lane & 15, rs = (lane >> 4) + 4 * w;  // column in the workgroup's 16, row stream 0 .. 63
  const int col = blockIdx.x * 16 + cl;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n4) {
    int k = rs;
    for (; k + 7 * 64 < splits; k += 8 * 64) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(k + 64 * u) * n4 + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
      }
    }
    for (; k < splits; k += 64) {
      const float4 v = part[(size_t)k * n4 + col];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[rs][cl] = s;
  __syncthreads();
  if (rs < 8) {  // streams rs, rs + 8, .. rs + 56
    float4 t = red[rs][cl];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      const float4 v = red[rs + 8 * q][cl];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    s = t;
  }
  __syncthreads();
  if (rs < 8) red[rs][cl] = s;
  __syncthreads();
  if (rs == 0 && col < n4) {
    float4 t = red[0][cl];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      const float4 v = red[q][cl];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    out[col] = t;
  }
}

// out[i] = sum_k part[k][i]; n % 4 == 0.  part must hold splits*n + ceil(splits/64)*n floats
// when splits > 64 (the chunk sums are written behind the partials).
void launch_split_reduce(const float* part, int splits, int n, float* out, hipStream_t stream) {
  const int n4 = n / 4;
  const int chunks = (splits + 63) / 64;
  if (chunks == 1) {
    hipLaunchKernelGGL(split_reduce1_kernel, dim3((n4 + 63) / 64, 1), dim3(256), 0, stream, (const float4*)part,
                       splits, n4, (float4*)out);
    return;
  }
  // narrow and not too deep (a small batch's BN-backward sums: 2C <= 4096 columns, <= 2048 tiles):
  // one launch of the row-parallel kernel instead of two latency-bound ones; g_tune[kRowReduce] = 2 off,
  // > 2: the depth limit (A/B)
  const int row_max = g_tune[kRowReduce] > 2 ? g_tune[kRowReduce] : 2048;
  // (wide and deep -- 1,024-channel BN sums over 1,568 tile rows at batch 1024 -- is ~12 MB on
  // n4 / 64 = 8 workgroups, 28 us; the two-level pair spreads it over the chip)
  const bool rows_ok = n4 <= 256 || (size_t)splits * n4 <= (size_t)512 * 1024;
  if (n4 <= 1024 && splits <= row_max && rows_ok && g_tune[kRowReduce] != 2) {
    hipLaunchKernelGGL(split_reduce_rows_kernel, dim3((n4 + 15) / 16), dim3(1024), 0, stream, (const float4*)part,
                       splits, n4, (float4*)out);
    return;
  }
  float* tmp = const_cast<float*>(part) + (size_t)splits * n;
  hipLaunchKernelGGL(split_reduce1_kernel, dim3((n4 + 63) / 64, chunks), dim3(256), 0, stream, (const float4*)part,
                     splits, n4, (float4*)tmp);
  // second level: 4 waves per 64 columns split the chunk rows (a thread-per-column loop over
  // ~200 chunk rows left narrow reductions -- BN sums of 2C columns -- latency bound)
  launch_partial_sum(tmp, chunks, n, out, stream);
}

// split-K plan of the weight-gradient GEMM, >= 256 rows per split: ~2 blocks per CU for
// 1x1 convs / linears (fewer, longer splits: less partial-slab traffic), ~4 for k x k
// (measured per shape with tools/conv_bench.py --cfgs "5=2,5=4")
static bool wgrad_big(int Co, int ldw) { return g_tune[kWgTileMode] != 2 && Co >= 256 && ldw >= 256; }
// 64-row tiles: Co <= 64 with enough columns to fill 256-wide tiles at least half
static bool wgrad_narrow(int Co, int ldw) { return g_tune[kWgTileMode] != 3 && Co <= 64 && ldw >= 128; }

// 16-column subtiles per wave of the narrow kernel: 192-column tiles where they pad less
static int wgrad_nj(int ldw) {
  if (g_tune[kWgCols] == 4 || g_tune[kWgCols] == 3) return g_tune[kWgCols];
  return ((ldw + 191) / 192) * 3 < ((ldw + 255) / 256) * 4 ? 3 : 4;
}

static int wgrad_tiles(int Co, int ldw) {
  if (wgrad_narrow(Co, ldw)) return (ldw + 64 * wgrad_nj(ldw) - 1) / (64 * wgrad_nj(ldw));
  const int bt = wgrad_big(Co, ldw) ? 256 : 128;
  return ((Co + bt - 1) / bt) * ((ldw + bt - 1) / bt);
}

int wgrad_splits(int M, int Co, int ldw, int taps, int num_cu, int* rows_per_split) {
  const bool big = wgrad_big(Co, ldw);
  const int tiles = wgrad_tiles(Co, ldw);
  const int per_cu = (big || wgrad_narrow(Co, ldw)) ? (big ? 1 : 2) : (taps == 1 ? 2 : 4);
  const int target = (g_tune[kWgSplitsPerCu] > 0 ? g_tune[kWgSplitsPerCu] : per_cu) * num_cu;
  // floor: a grid just past a whole number of resident rounds leaves a tail round of one block
  int splits = target / tiles;
  int max_splits = (M + 255) / 256;
  if (splits > max_splits) splits = max_splits;
  // g_tune[kWgSplitCap] > 0: at most that many splits (64: the one-level reduction, no second launch --
  // small batches, where every launch counts; an autotuner candidate)
  if (g_tune[kWgSplitCap] > 0 && splits > g_tune[kWgSplitCap]) splits = g_tune[kWgSplitCap];
  if (splits < 1) splits = 1;
  int rps = (M + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  splits = (M + rps - 1) / rps;
  if (rows_per_split) *rows_per_split = rps;
  return splits;
}

// the 3x3 / stride-1 / pad-1 same-size geometry of wgrad3x3.hip (taps in fwd_taps order)
static bool is_3x3_same(int Ho, int Wo, int Hs, int Ws, int ss, const TapList& taps) {
  if (taps.n != 9 || ss != 1 || Hs != Ho || Ws != Wo) return false;
  for (int i = 0; i < 9; ++i)
    if (taps.dy[i] != i / 3 - 1 || taps.dx[i] != i % 3 - 1) return false;
  return true;
}

int wgrad_plan_splits(int N, int Ho, int Wo, int Co, int Hs, int Ws, int Cs, int ss, const TapList& taps,
                      int num_cu) {
  if (is_3x3_same(Ho, Wo, Hs, Ws, ss, taps)) {
    const int s3 = wgrad3x3_splits(N, Ho, Wo, Cs, Co, num_cu);
    if (s3 > 0) return s3;
  }
  return wgrad_splits(N * Ho * Wo, Co, taps.n * Cs, taps.n, num_cu, nullptr);
}

void launch_wgrad(const bf16* dy, int N, int Ho, int Wo, int Co,
                  const bf16* src, int Hs, int Ws, int Cs, int ss,
                  const TapList& taps, float* dw, float* part, const bf16* zero, int num_cu, hipStream_t stream,
                  const float* pscale, const float* pshift) {
  WgradParams p;
  p.dy = dy; p.src = src; p.dw = dw; p.zero = zero;
  p.pscale = pscale; p.pshift = pshift;
  const bool pro = pscale != nullptr;
  p.Hs = Hs; p.Ws = Ws; p.Cs = Cs; p.Ho = Ho; p.Wo = Wo; p.ss = ss;
  p.Co = Co; p.M = N * Ho * Wo; p.ldw = taps.n * Cs;
  p.cpt = Cs / 8; p.kc_total = taps.n * p.cpt;
  p.div_wo = make_fastdiv(Wo); p.div_ho = make_fastdiv(Ho); p.div_cpt = make_fastdiv(p.cpt);
  for (int i = 0; i < taps.n; ++i) {
    p.dy_t[i] = (int8_t)taps.dy[i];
    p.dx_t[i] = (int8_t)taps.dx[i];
  }
  if (is_3x3_same(Ho, Wo, Hs, Ws, ss, taps)) {
    const int s3 = wgrad3x3_splits(N, Ho, Wo, Cs, Co, num_cu);
    if (s3 > 0) {
      // part holds wgrad_plan_splits(...) = s3 partial slices (the caller sized it by that plan);
      // a BN prologue is recomputed on the staged window (the 3x3 consumer's K5)
      launch_wgrad3x3(dy, src, N, Ho, Wo, Cs, Co, part, s3, zero, stream, pscale, pshift);
      launch_split_reduce(part, s3, Co * 9 * Cs, dw, stream);
      return;
    }
  }
  p.direct = (taps.n == 1 && taps.dy[0] == 0 && taps.dx[0] == 0 && ss == 1 && Hs == Ho && Ws == Wo) ? 1 : 0;
  const bool big = wgrad_big(Co, p.ldw);
  const bool narrow = wgrad_narrow(Co, p.ldw);
  if (pro && (!p.direct || narrow)) {  // (the 64-row kernel has no prologue)
    fprintf(stderr, "launch_wgrad: the BN prologue needs a 1x1 stride-1 conv with Co > 64 or Cs < 128\n");
    abort();
  }
  const int tiles = wgrad_tiles(Co, p.ldw);
  p.ablate = g_tune[kAblate];
  if (g_tune[kWgFlushAblate] == 1) part = nullptr;  // A/B timing of the atomic flush only (dw not zeroed)
  int rps = 0;
  const int splits = wgrad_splits(p.M, Co, p.ldw, taps.n, num_cu, &rps);
  p.rows_per_split = rps;
  // partials: plain stores + one deterministic reduce (memory-side float atomics cost
  // ~1/4 of the kernel); a single split writes the gradient directly
  p.part = (part != nullptr && splits > 1) ? part : nullptr;
  if (splits == 1) {
    p.part = dw;  // split 0 stores straight into dw
  }
  // 32 pixel rows per k-tile (g_tune[kWgRows] = 32): half the LDS of the 64-row tiles
  const bool wbk32 = g_tune[kWgRows] == 32;
  if (narrow) {
    const int nj = wgrad_nj(p.ldw);
    if (wbk32 && nj == 4)
      hipLaunchKernelGGL((wgrad64_kernel<32, 4>), dim3(tiles * splits), dim3(256), 2 * 32 * (128 + 512), stream, p);
    else if (wbk32)
      hipLaunchKernelGGL((wgrad64_kernel<32, 3>), dim3(tiles * splits), dim3(256), 2 * 32 * (128 + 512), stream, p);
    else if (nj == 4)
      hipLaunchKernelGGL((wgrad64_kernel<64, 4>), dim3(tiles * splits), dim3(256), 2 * 64 * (128 + 512), stream, p);
    else
      hipLaunchKernelGGL((wgrad64_kernel<64, 3>), dim3(tiles * splits), dim3(256), 2 * 64 * (128 + 512), stream, p);
  } else if (big) {
    constexpr int lds = 4 * 64 * 512;
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)wgrad256_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr = true;
    }
    static bool attr_pro = false;
    if (pro && !attr_pro) {  // + the (scale, shift) table of up to 2048 channels
      hipFuncSetAttribute((const void*)wgrad256_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          lds + 8 * 2048);
      attr_pro = true;
    }
    if (pro)
      hipLaunchKernelGGL(wgrad256_kernel<true>, dim3(tiles * splits), dim3(512), lds + 8 * Cs, stream, p);
    else hipLaunchKernelGGL(wgrad256_kernel<false>, dim3(tiles * splits), dim3(512), lds, stream, p);
  } else if (pro) {
    if (wbk32) hipLaunchKernelGGL((wgrad_kernel<32, true>), dim3(tiles * splits), dim3(256), 4 * 32 * 256, stream, p);
    else hipLaunchKernelGGL((wgrad_kernel<64, true>), dim3(tiles * splits), dim3(256), 4 * 64 * 256, stream, p);
  } else {
    if (wbk32) hipLaunchKernelGGL(wgrad_kernel<32>, dim3(tiles * splits), dim3(256), 4 * 32 * 256, stream, p);
    else hipLaunchKernelGGL(wgrad_kernel<64>, dim3(tiles * splits), dim3(256), 4 * 64 * 256, stream, p);
  }
  if (part != nullptr && splits > 1) launch_split_reduce(part, splits, Co * p.ldw, dw, stream);
}

}  // namespace dcp
