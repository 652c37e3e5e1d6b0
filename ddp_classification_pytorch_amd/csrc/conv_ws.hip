// Weight-stationary persistent GEMM for the short-K 1x1 stride-1 convolutions (forward, plain or
// BN-statistics epilogue): the expansion convs of every ResNet bottleneck (64 -> 256, 128 -> 512,
// 256 -> 1024 channels; reference NESTED/model/imagenet_resnet.py:82-97, Bottleneck conv3).
//
// Those GEMMs (M = N*H*W pixels, K = 64..256 input channels, N = 4K output channels) move 4x more
// bytes out than in and do little math per byte: the tap-GEMM tiles spend most of their time on a
// per-tile prologue (address setup, the first k-tile's load round trip) and a store epilogue that
// nothing overlaps (profiles/r5/ablations_r6k_b1024.txt: 256 -> 1024 14x14, 226 us, 117 us without
// its epilogue; the epilogue alone ran at ~2.7 TB/s).  This kernel is built around the stores:
//
//   * one workgroup per CU (8 waves, 2 per SIMD) stays resident and walks a list of 256-row tiles
//     of ONE 128-channel output column block; that block's weights [128][K] are loaded into LDS
//     once and stay there (64 KB at K = 256);
//   * the activation rows stream through an LDS-DMA ring of 32-deep k-steps that runs ACROSS tile
//     boundaries: while tile i's last k-steps and its epilogue run, tile i+1's first k-steps are
//     already in flight -- there is no per-tile prologue bubble;
//   * the epilogue stores straight from the accumulators (16-byte buffer stores: the weight rows
//     are permuted in LDS so a lane's two 16-wide MFMA results are 8 consecutive output channels),
//     and nothing waits for those stores: the ring's counted vmcnt waits skip over them (the
//     number of stores issued after each k-step's DMA is known exactly), so tile i's stores drain
//     under tile i+1's MFMAs.  Rows past M are dropped by the buffer resource's range check (no
//     branch, so every wave issues the same number of memory instructions);
//   * BN statistics (per-128-row slab (mean, M2) of the bf16 outputs, the layout every consumer
//     reads) from the registers: shifted sums, DPP row reductions, a Chan merge of the two 64-row
//     halves through a small LDS exchange read after the next ring barrier;
//   * XCD-aware work split: the workgroups that share one XCD (and its L2) take the SAME row tiles
//     for all column blocks, so an activation tile is fetched from HBM once per XCD.
#include <algorithm>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {

constexpr int kWsBM = 256, kWsBN = 128, kWsThreads = 512, kWsSlot = kWsBM * 64;  // ring slot: 256 rows x 32 k

struct WsParams {
  const bf16* src;   // [M][K]
  const bf16* wt;    // [Co][ldw]
  bf16* dst;         // [M][Co]
  float* stats;      // [ceil(M/128)][2][Co] or nullptr
  const bf16* zero;  // >= 16 zero bytes
  int M, Co, ldw;
  int ntm, ntn;      // 256-row tiles, 128-channel column blocks
  int xcd_map, nper; // 1: XCD-aware split (gridDim % 8 == 0, nper = gridDim / 8, nper % ntn == 0)
};

// weights [128][K] in LDS: row length 2K bytes, 16-byte chunks XOR-swizzled (conflict-free
// fragment reads: 16 consecutive rows at one chunk)
template <int K>
__device__ __forceinline__ uint32_t ws_woff(uint32_t r, uint32_t c) {
  if constexpr (K >= 128) return r * (K * 2u) + ((c ^ (r & 15u)) << 4);
  else return r * (K * 2u) + ((c ^ ((r >> 1) & 7u)) << 4);
}
// ring slot: 64-byte rows, chunk XOR (r >> 1) & 3 (the tap GEMMs' 32-deep layout)
__device__ __forceinline__ uint32_t ws_aoff(uint32_t r, uint32_t c) { return r * 64u + ((c ^ ((r >> 1) & 3u)) << 4); }

// number of t in [0, x] with t % nk == nk - 1 (x may be negative)
template <int NK>
__device__ __forceinline__ int ends_upto(int x) {
  return x >= NK - 1 ? (x - (NK - 1)) / NK + 1 : 0;
}

}  // namespace

template <int K, int NSLOT, bool STATS>
__global__ void __launch_bounds__(kWsThreads, 1) conv1x1_ws_kernel(const WsParams p) {
  constexpr int NK = K / 32, P = NSLOT - 1, LPT = 2, ST = 8;
  constexpr int WBYTES = kWsBN * K * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Wl = smem;
  char* ring = smem + WBYTES;
  float* xch = (float*)(ring + NSLOT * kWsSlot);  // [8 waves][64 ch][2] (mean, M2)
  float* xn = xch + 8 * 64 * 2;                   // [8] rows per wave half
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const uint32_t q = lane >> 4, l15 = lane & 15;

  // ---- work: one column block, a strided list of row tiles ----
  int tn, gidx, NG;
  if (p.xcd_map) {
    const int xcd = blockIdx.x & 7, l = blockIdx.x >> 3;
    tn = l % p.ntn;
    const int gper = p.nper / p.ntn;
    gidx = xcd * gper + l / p.ntn;
    NG = 8 * gper;
  } else {
    tn = blockIdx.x % p.ntn;
    gidx = blockIdx.x / p.ntn;
    NG = gridDim.x / p.ntn;
  }
  const int ntiles = gidx < p.ntm ? (p.ntm - 1 - gidx) / NG + 1 : 0;
  if (ntiles == 0) return;  // (uniform over the workgroup)
  const int S = ntiles * NK;
  const int n0 = tn * kWsBN;

  // ---- weights of the column block -> LDS, rows permuted: LDS row 64h + 16j + m holds channel
  // 64h + 32(j >> 1) + 8(m >> 2) + 4(j & 1) + (m & 3), so the accumulator rows a lane owns in
  // fragments j = 2p, 2p + 1 are the 8 consecutive channels 32p + 8q .. + 7 of its half ----
  for (int e = tid; e < kWsBN * (K / 8); e += kWsThreads) {
    const int r = e / (K / 8), c = e - r * (K / 8);
    const int h = r >> 6, j = (r >> 4) & 3, m = r & 15;
    const int ch = 64 * h + 32 * (j >> 1) + 8 * (m >> 2) + 4 * (j & 1) + (m & 3);
    *LDS_PTR(bf16x8, Wl + ws_woff<K>(r, c)) = *(const bf16x8*)(p.wt + (size_t)(n0 + ch) * p.ldw + c * 8);
  }

  // ---- LDS-DMA of k-step s of the stream into its ring slot (2 instructions per lane) ----
  int a_row[LPT];
  uint32_t a_chk[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    a_row[i] = (w * LPT + i) * 16 + lane / 4;
    a_chk[i] = (uint32_t)(lane % 4) ^ (((uint32_t)a_row[i] >> 1) & 3u);
  }
  auto dma = [&](int s) {
    const int it = s / NK, kk = s - it * NK;
    const int m0 = (gidx + it * NG) * kWsBM;
    char* slot = ring + (s % NSLOT) * kWsSlot;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int m = m0 + a_row[i];
      const bf16* g = m < p.M ? p.src + (size_t)m * K + kk * 32 + a_chk[i] * 8 : p.zero;
      dma16(g, slot + (w * LPT + i) * 1024);  // untracked: the counted waits below order it
    }
  };
#pragma unroll
  for (int s = 0; s < P; ++s)
    if (s < S) dma(s);

  f32x4 acc[4][4];  // [16-channel fragment j][16-row fragment i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  bool stats_pending = false;
  int pend_slab = 0, pend_nrec = 0;
  for (int s = 0; s < S; ++s) {
    // ---- wait for this wave's share of DMA(s): the ops issued after it are known exactly ----
    {
      const int n_dma = min(s + P - 1, S - 1) - s;
      const int lo = max(0, s - P);
      const int e_cnt = ends_upto<NK>(s - 1) - ends_upto<NK>(lo - 1);
      int f_cnt = 0;
      if (STATS && (wm & 1) == 0) f_cnt = ends_upto<NK>(s - 2) - ends_upto<NK>(max(0, s - P - 1) - 1);
      wait_vmcnt_wide(min(63, n_dma * LPT + e_cnt * ST + f_cnt * 2));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot s-1 retired
    __builtin_amdgcn_s_barrier();                         // DMA(s) landed for every wave; slot s-1 free
    asm volatile("" ::: "memory");
    if (s + P < S) dma(s + P);
    if (STATS && stats_pending) {
      stats_pending = false;
      if ((wm & 1) == 0) {
        // even waves: merge the partner half (wave w + 2) into this one, 64 channels, one per lane
        const float na = xn[w], nb = xn[w + 2];
        const float ma = xch[(w * 64 + lane) * 2], m2a = xch[(w * 64 + lane) * 2 + 1];
        const float mb = xch[((w + 2) * 64 + lane) * 2], m2b = xch[((w + 2) * 64 + lane) * 2 + 1];
        const float n = na + nb;
        const float delta = mb - ma;
        const float mean = n > 0.f ? ma + delta * (nb / n) : 0.f;
        const float m2 = n > 0.f ? m2a + m2b + delta * delta * (na * nb / n) : 0.f;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.stats + (size_t)pend_slab * 2 * p.Co), (short)0, pend_nrec, 0x00020000);
        const int col = n0 + wn * 64 + lane;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mean), rs, col * 4, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m2), rs, (p.Co + col) * 4, 0, 0);
      }
    }
    // ---- MFMAs of k-step s ----
    const int it = s / NK, kk = s - it * NK;
    const char* slot = ring + (s % NSLOT) * kWsSlot;
    bf16x8 wf[4], af[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *LDS_PTR(const bf16x8, Wl + ws_woff<K>(wn * 64 + 16 * j + l15, kk * 4 + q));
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *LDS_PTR(const bf16x8, slot + ws_aoff(wm * 64 + 16 * i + l15, q));
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
    if (kk != NK - 1) continue;

    // ---- epilogue of tile it: 8 x 16-byte stores per lane, straight from the accumulators ----
    const int m0 = (gidx + it * NG) * kWsBM;
    const int nvalid = min(kWsBM, p.M - m0);
    __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.dst + (size_t)m0 * p.Co), (short)0, nvalid * p.Co * 2, 0x00020000);
    bf16x8 o[2][4];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[pp][i][r] = f2bf(acc[2 * pp][i][r]);
          o[pp][i][4 + r] = f2bf(acc[2 * pp + 1][i][r]);
        }
        const int row = wm * 64 + 16 * i + (int)l15;
        const int col = n0 + wn * 64 + 32 * pp + 8 * (int)q;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o[pp][i]), rd, (row * p.Co + col) * 2, 0, 0);
      }
    if constexpr (STATS) {
      // per-wave (64 rows) shifted sums of the bf16 outputs: shift = the half's first row
      const int nw = max(0, min(64, nvalid - wm * 64));
      float s1[2][8], s2[2][8];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float k0 = __shfl(bf2f(o[pp][0][e]), (int)(lane & 48), 64);
          float a1 = 0.f, a2 = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool ok = 16 * i + (int)l15 < nw;
            const float d = ok ? bf2f(o[pp][i][e]) - k0 : 0.f;
            a1 += d;
            a2 = fmaf(d, d, a2);
          }
          // sum over the 16 lanes of the row (DPP row rotations: every lane gets the total)
          a1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a1), 0x128, 0xf, 0xf, true));
          a2 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a2), 0x128, 0xf, 0xf, true));
          a1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a1), 0x124, 0xf, 0xf, true));
          a2 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a2), 0x124, 0xf, 0xf, true));
          a1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a1), 0x122, 0xf, 0xf, true));
          a2 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a2), 0x122, 0xf, 0xf, true));
          a1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a1), 0x121, 0xf, 0xf, true));
          a2 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a2), 0x121, 0xf, 0xf, true));
          const float nf = (float)nw;
          s1[pp][e] = nw > 0 ? k0 + a1 / nf : 0.f;                     // mean
          s2[pp][e] = nw > 0 ? fmaxf(a2 - a1 * a1 / nf, 0.f) : 0.f;    // M2
        }
      if (l15 == 0) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int c = 32 * pp + 8 * (int)q + e;
            *LDS_PTR(f32x2, xch + (w * 64 + c) * 2) = f32x2{s1[pp][e], s2[pp][e]};
          }
      }
      if (lane == 0) xn[w] = (float)nw;
      stats_pending = true;
      pend_slab = m0 / 128 + (wm >> 1);
      pend_nrec = (nvalid > (wm >> 1) * 128) ? 2 * p.Co * 4 : 0;  // a slab past M: nothing to write
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (STATS && stats_pending) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if ((wm & 1) == 0) {
      const float na = xn[w], nb = xn[w + 2];
      const float ma = xch[(w * 64 + lane) * 2], m2a = xch[(w * 64 + lane) * 2 + 1];
      const float mb = xch[((w + 2) * 64 + lane) * 2], m2b = xch[((w + 2) * 64 + lane) * 2 + 1];
      const float n = na + nb;
      const float delta = mb - ma;
      const float mean = n > 0.f ? ma + delta * (nb / n) : 0.f;
      const float m2 = n > 0.f ? m2a + m2b + delta * delta * (na * nb / n) : 0.f;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.stats + (size_t)pend_slab * 2 * p.Co), (short)0, pend_nrec, 0x00020000);
      const int col = n0 + wn * 64 + lane;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mean), rs, col * 4, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m2), rs, (p.Co + col) * 4, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------
bool conv1x1_ws_supported(int K, int Co, long M) {
  return (K == 64 || K == 128 || K == 256) && Co % kWsBN == 0 && M > 0 && (long)kWsBM * Co * 2 < (1l << 31);
}

template <int K, int NSLOT, bool STATS>
static void launch_ws(const WsParams& p, int grid, hipStream_t st) {
  constexpr size_t lds = (size_t)kWsBN * K * 2 + (size_t)NSLOT * kWsSlot + (8 * 64 * 2 + 8) * 4;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv1x1_ws_kernel<K, NSLOT, STATS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_ws_kernel<K, NSLOT, STATS>), dim3(grid), dim3(kWsThreads), lds, st, p);
}

bool launch_conv1x1_ws(const bf16* src, const bf16* wt, int ldw, bf16* dst, float* stats, const bf16* zero, int M,
                       int K, int Co, hipStream_t st) {
  if (!conv1x1_ws_supported(K, Co, M)) return false;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  WsParams p;
  p.src = src; p.wt = wt; p.dst = dst; p.stats = stats; p.zero = zero;
  p.M = M; p.Co = Co; p.ldw = ldw;
  p.ntm = (M + kWsBM - 1) / kWsBM;
  p.ntn = Co / kWsBN;
  // one workgroup per CU; no more workgroups than (column block, row tile) pairs
  int grid = std::min(ncu, p.ntm * p.ntn);
  const int nper = grid / 8;
  p.xcd_map = (grid % 8 == 0 && nper % p.ntn == 0 && nper >= p.ntn) ? 1 : 0;
  p.nper = nper;
  if (!p.xcd_map) grid = std::max(p.ntn, grid / p.ntn * p.ntn);
  const bool s = stats != nullptr;
  if (K == 256) {
    if (s) launch_ws<256, 4, true>(p, grid, st); else launch_ws<256, 4, false>(p, grid, st);
  } else if (K == 128) {
    if (s) launch_ws<128, 6, true>(p, grid, st); else launch_ws<128, 6, false>(p, grid, st);
  } else {
    if (s) launch_ws<64, 6, true>(p, grid, st); else launch_ws<64, 6, false>(p, grid, st);
  }
  return true;
}

}  // namespace dcp
