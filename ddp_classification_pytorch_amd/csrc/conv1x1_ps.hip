// Store-decoupled persistent 1x1 GEMM for the short-K stride-1 convolutions (forward, plain or
// BN-statistics epilogue): the expansion convs of every ResNet bottleneck (64 -> 256, 128 -> 512,
// 256 -> 1024 channels; reference NESTED/model/imagenet_resnet.py:82-97, Bottleneck conv3), whose
// outputs are 4x their inputs.
//
// Why the earlier designs stall (profiles/r6/pmc_conv_kernels_s1.txt, ws_pmc_s3.txt): a wave's
// s_waitcnt vmcnt counts loads, stores and LDS-DMA together in issue order, so a wave that stores a
// tile and then waits for its next LDS-DMA waits for its own stores to reach memory.  The 128-row tap
// GEMM ends every tile that way (the workgroup exits behind its stores; the next one starts cold:
// 20 % MFMA busy, 2 TB/s of writes on 256 -> 1024 14x14), and the weight-stationary kernel
// (conv_ws.hip) waits on its stores at the first k-step of every tile (5-14 % MFMA busy, 2 TB/s).
//
// Here the roles are split inside one 512-thread workgroup per CU (two waves per SIMD):
//   * 4 LOADER waves only issue LDS-DMA (untracked, global_load_lds_dwordx4) into a ring of 32-deep
//     k-steps of 256 activation rows that runs across tile boundaries, and wait on their own vmcnt
//     (DMA only) before each ring barrier -- NS-1 k-steps stay in flight;
//   * 4 CONSUMER waves (128 rows x 64 channels each, 32 MFMA 16x16x32 per k-step) read fragments from
//     the ring and from the column block's weights, which stay resident in LDS for the whole launch,
//     and store their tile straight from the accumulators.  They never issue a load, so nothing ever
//     waits for their stores: tile i's stores drain under tile i+1's MFMAs.
// The weight rows are permuted in LDS so a lane's accumulators hold 8 consecutive output channels
// per pair of fragments (16-byte stores, 64 contiguous bytes per row per instruction).  A consumer
// wave owns exactly one 128-row statistics slab of its 64 channels, so the BN statistics ((mean, M2)
// of the bf16 outputs, the layout every consumer reads) come from its registers: shifted sums, DPP
// row reductions, no LDS exchange.  Work split: one 128-channel column block per workgroup, a
// strided list of 256-row tiles; the workgroups of an XCD take the same row tiles for all column
// blocks, so an activation tile is fetched from HBM once per XCD.
#include <algorithm>
#include <type_traits>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {

constexpr int kPsBM = 256, kPsBN = 128, kPsSlot = kPsBM * 64;  // ring slot: 256 rows x 32 k

struct PsParams {
  const bf16* src;   // [M][K]
  const bf16* wt;    // [Co][ldw]
  bf16* dst;         // [M][Co]
  float* stats;      // [ceil(M/128)][2][Co] or nullptr
  const bf16* zero;  // >= 16 zero bytes
  int M, Co, ldw;
  int ntm, ntn;      // 256-row tiles, 128-channel column blocks
  int xcd_map, nper; // 1: XCD-aware split (gridDim % 8 == 0, nper = gridDim / 8, nper % ntn == 0)
  int ablate;        // timing ablations: 1 = no LDS-DMA, 2 = no MFMA, 4 = no stores, 8 = no statistics math,
                     // 16 = no ring barriers (with 1 only: timing of everything else)
};

// weights [128][K] in LDS: 2K-byte rows, 16-byte chunks XOR-swizzled (conflict-free fragment reads)
template <int K>
__device__ __forceinline__ uint32_t ps_woff(uint32_t r, uint32_t c) {
  if constexpr (K >= 128) return r * (K * 2u) + ((c ^ (r & 15u)) << 4);
  else return r * (K * 2u) + ((c ^ ((r >> 1) & 7u)) << 4);
}
// ring slot: 64-byte rows, chunk XOR (r >> 1) & 3 (the tap GEMMs' 32-deep layout)
__device__ __forceinline__ uint32_t ps_aoff(uint32_t r, uint32_t c) { return r * 64u + ((c ^ ((r >> 1) & 3u)) << 4); }

// A buffer resource from wave-uniform values, made provably scalar: built from values the compiler's
// divergence analysis cannot see are uniform, the resource lands in VGPRs and every buffer store
// becomes a readfirstlane waterfall loop (the first build of this kernel: 20 loops per tile)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int nrec) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
}

// sum over the 16 lanes of a DPP row; every lane of the row gets the total
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, true));
  return v;
}

}  // namespace

// CW consumer waves: 4 (one per SIMD, 128 rows x 64 channels each) or 8 (two per SIMD, 128 rows x 32
// channels each: a partner wave covers each wave's LDS and dependency latency); 4 loader waves either way
template <int K, int NS, bool STATS, int CW>
__global__ void __launch_bounds__((CW + 4) * 64, 1) conv1x1_ps_kernel(const PsParams p) {
  constexpr int NT = (CW + 4) * 64;
  constexpr int NK = K / 32, P = NS - 1, LPT = 4;  // LDS-DMA instructions per loader wave per k-step
  constexpr int WNW = CW / 2, CWID = kPsBN / WNW, JF = CWID / 16;  // waves across the channels, their width
  constexpr int WBYTES = kPsBN * K * 2;
  static_assert(NS >= 3 && LPT * (P - 1) <= 63, "ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Wl = smem;
  char* ring = smem + WBYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

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
  const int n0 = tn * kPsBN;

  // ---- the column block's weights -> LDS, rows permuted: LDS row CWID h + 16j + m holds channel
  // CWID h + 32(j >> 1) + 8(m >> 2) + 4(j & 1) + (m & 3), so the accumulator rows a lane owns in
  // fragments j = 2t, 2t + 1 are the 8 consecutive channels 32t + 8(lane >> 4) .. + 7 of wave h's slice ----
  for (int e = tid; e < kPsBN * (K / 8); e += NT) {
    const int r = e / (K / 8), c = e - r * (K / 8);
    const int h = r / CWID, j = (r % CWID) >> 4, m = r & 15;
    const int ch = CWID * h + 32 * (j >> 1) + 8 * (m >> 2) + 4 * (j & 1) + (m & 3);
    *LDS_PTR(bf16x8, Wl + ps_woff<K>(r, c)) = *(const bf16x8*)(p.wt + (size_t)(n0 + ch) * p.ldw + c * 8);
  }
  __syncthreads();

  if (w >= CW) {
    // =============================== loader waves ===============================
    const int lw = w - CW;
    int a_row[LPT];
    uint32_t a_chk[LPT];
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      a_row[i] = (lw * LPT + i) * 16 + lane / 4;
      a_chk[i] = (uint32_t)(lane % 4) ^ (((uint32_t)a_row[i] >> 1) & 3u);
    }
    auto dma = [&](int s) {
      const int it = s / NK, kk = s - it * NK;
      const int m0 = (gidx + it * NG) * kPsBM;
      char* slot = ring + (s % NS) * kPsSlot;
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int m = m0 + a_row[i];
        const bf16* g = m < p.M ? p.src + (size_t)m * K + kk * 32 + a_chk[i] * 8 : p.zero;
        if (!(p.ablate & 1)) dma16(g, slot + (lw * LPT + i) * 1024);  // untracked: the counted waits order it
      }
    };
#pragma unroll
    for (int s = 0; s < P; ++s)
      if (s < S) dma(s);
    for (int s = 0; s < S; ++s) {
      // this wave's share of k-step s landed: only DMA is in this wave's counter
      if (p.ablate & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else wait_vmcnt_wide(LPT * min(P - 1, S - 1 - s));
      if (!(p.ablate & 16)) __builtin_amdgcn_s_barrier();  // k-step s landed for every loader; slot s-1 read by every consumer
      asm volatile("" ::: "memory");
      if (s + P < S) dma(s + P);  // into slot (s + P) % NS == (s - 1) % NS
    }
    return;
  }

  // =============================== consumer waves ===============================
  const int wm = w / WNW, wn = w % WNW;
  const uint32_t q = lane >> 4, l15 = lane & 15;
  f32x4 acc[JF][8];  // [16-channel fragment j][16-row fragment i]
  bf16x8 wf[JF], af[8];
  auto read_w = [&](int s) {
#pragma unroll
    for (int j = 0; j < JF; ++j)
      wf[j] = *LDS_PTR(const bf16x8, Wl + ps_woff<K>(wn * CWID + 16 * j + l15, (s % NK) * 4 + q));
  };
  auto read_a = [&](int s, int i) {
    af[i] = *LDS_PTR(const bf16x8, ring + (s % NS) * kPsSlot + ps_aoff(wm * 128 + 16 * i + l15, q));
  };
  auto ring_barrier = [&]() {
    if (!(p.ablate & 16)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto epilogue = [&](int it) {
    // ---- epilogue of tile it: this wave's 128 rows (one statistics slab) x 64 channels ----
    const int mw = (gidx + it * NG) * kPsBM + wm * 128;
    const int nvalid = max(0, min(128, p.M - mw));
    // rows past M dropped by the buffer's range check (no branch: every lane issues the same stores)
    const __amdgpu_buffer_rsrc_t rd = uniform_rsrc(p.dst + (size_t)mw * p.Co, (p.ablate & 4) ? 0 : nvalid * p.Co * 2);
    const int colb = n0 + wn * CWID + 8 * (int)q;  // + 32 t: this lane's 8 channels of 32-channel group t
    // statistics of the bf16 outputs, shifted by the slab's row 0 (lane 16q of this row group), on
    // packed fp32 pairs (v_pk_add / v_pk_fma: two channels per instruction).  Rows past M are not
    // masked: their A rows are the zero page, so their outputs are exactly 0 and contribute
    // d = -k0, d^2 = k0^2 each -- removed in closed form after the row reduction.
    const bool stats = STATS && !(p.ablate & 8);
    const float inv_n = nvalid > 0 ? 1.f / (float)nvalid : 0.f;
    const float npad = (float)(128 - nvalid);  // zero rows counted in the sums
    // lane 16q writes the statistics of the 16 channels of its row group; the other lanes' offsets lie
    // past the range (the resource stays wave-uniform); a slab past M writes nothing
    const __amdgpu_buffer_rsrc_t rs =
        uniform_rsrc(p.stats + (size_t)(mw / 128) * 2 * p.Co, (nvalid > 0 && !(p.ablate & 4)) ? 2 * p.Co * 4 : 0);
    const int loff = l15 == 0 ? 0 : (1 << 30);
    // one 32-channel group t at a time: its accumulators die as its rows are stored, and only one
    // group's statistics registers are live
#pragma unroll
    for (int t = 0; t < JF / 2; ++t) {
      f32x2 k0[4], s1[4], s2[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bf16x8 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = f2bf(acc[2 * t][i][r]);
          o[4 + r] = f2bf(acc[2 * t + 1][i][r]);
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rd,
                                               ((16 * i + (int)l15) * p.Co + colb + 32 * t) * 2, 0, 0);
        if (stats) {
          const u32x4 u = __builtin_bit_cast(u32x4, o);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // channels 2e, 2e + 1 of the chunk: bf16 -> fp32 is a shift / a mask
            const f32x2 v{__uint_as_float(u[e] << 16), __uint_as_float(u[e] & 0xffff0000u)};
            if (i == 0) {
              const uint32_t u0 = (uint32_t)__shfl((int)u[e], (int)(lane & 48), 64);
              k0[e] = f32x2{__uint_as_float(u0 << 16), __uint_as_float(u0 & 0xffff0000u)};
              s1[e] = s2[e] = f32x2{0.f, 0.f};
            }
            const f32x2 d = v - k0[e];
            s1[e] += d;
            s2[e] = __builtin_elementwise_fma(d, d, s2[e]);
          }
        }
      }
      if (stats) {
        float mean[8], m2[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float kk0 = k0[e >> 1][e & 1];
          float a1 = row16_sum(s1[e >> 1][e & 1]), a2 = row16_sum(s2[e >> 1][e & 1]);
          a1 = fmaf(npad, kk0, a1);         // - sum over the zero rows of (0 - k0)
          a2 = fmaf(-npad * kk0, kk0, a2);  // - sum over the zero rows of k0^2
          mean[e] = nvalid > 0 ? fmaf(a1, inv_n, kk0) : 0.f;
          m2[e] = nvalid > 0 ? fmaxf(a2 - a1 * a1 * inv_n, 0.f) : 0.f;
        }
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const f32x4 mv{mean[4 * hh], mean[4 * hh + 1], mean[4 * hh + 2], mean[4 * hh + 3]};
          const f32x4 qv{m2[4 * hh], m2[4 * hh + 1], m2[4 * hh + 2], m2[4 * hh + 3]};
          const int col = colb + 32 * t + 4 * hh;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, mv), rs, loff + col * 4, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, qv), rs, loff + (p.Co + col) * 4, 0, 0);
        }
      }
    }
  };
  auto mfmas = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < JF; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[j][i], 0, 0, 0);
  };
  auto read_all = [&](int s) {
    read_w(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) read_a(s, i);
  };
#pragma unroll
  for (int j = 0; j < JF; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  ring_barrier();  // ring barrier 0: k-step 0 landed
  read_all(0);
  // k-step s: once its fragments are in registers this wave is done with slot s, so it passes ring
  // barrier s+1 BEFORE its MFMAs (the loaders refill slot s behind it); each row fragment i of k-step
  // s+1 is read into the registers of row fragment i of k-step s right behind that fragment's last
  // MFMA, the weight fragments after the last row (one fragment set: the MFMAs of k-step s cover the
  // reads of k-step s+1).  At a tile's last k-step the next fragments are read after the epilogue.
  auto kstep = [&](int s) {
    const int it = s / NK, kk = s - it * NK;
    const bool last = kk == NK - 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool pre = s + 1 < S && !last;
    if (pre) ring_barrier();
    // the next k-step's reads issue behind this one's MFMAs (which read their operands at issue) and
    // land while the matrix pipe drains them
    if (!(p.ablate & 2)) mfmas();
    if (pre) read_all(s + 1);
    if (last) {
      epilogue(it);
#pragma unroll
      for (int j = 0; j < JF; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (s + 1 < S) {
        ring_barrier();
        read_all(s + 1);
      }
    }
  };
  for (int s = 0; s < S; ++s) kstep(s);
}

// ---------------------------------------------------------------------------
bool conv1x1_ps_supported(int K, int Co, long M) {
  return (K == 64 || K == 128 || K == 256) && Co % kPsBN == 0 && M > 0 && (long)kPsBM * Co * 2 < (1l << 31) &&
         M * (long)Co < (1l << 40);
}

template <int K, int NS, bool STATS, int CW>
static void launch_ps1(const PsParams& p, int grid, hipStream_t st) {
  constexpr size_t lds = (size_t)kPsBN * K * 2 + (size_t)NS * kPsSlot;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv1x1_ps_kernel<K, NS, STATS, CW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_ps_kernel<K, NS, STATS, CW>), dim3(grid), dim3((CW + 4) * 64), lds, st, p);
}
template <int K, int NS, bool STATS>
static void launch_ps(const PsParams& p, int cw, int grid, hipStream_t st) {
  if (cw == 8) launch_ps1<K, NS, STATS, 8>(p, grid, st);
  else launch_ps1<K, NS, STATS, 4>(p, grid, st);
}

bool launch_conv1x1_ps(const bf16* src, const bf16* wt, int ldw, bf16* dst, float* stats, const bf16* zero, int M,
                       int K, int Co, int ablate, int cw, hipStream_t st) {
  if (!conv1x1_ps_supported(K, Co, M)) return false;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  PsParams p;
  p.src = src; p.wt = wt; p.dst = dst; p.stats = stats; p.zero = zero;
  p.M = M; p.Co = Co; p.ldw = ldw; p.ablate = ablate;
  p.ntm = (M + kPsBM - 1) / kPsBM;
  p.ntn = Co / kPsBN;
  // one workgroup per CU; no more workgroups than (column block, row tile) pairs
  int grid = std::min(ncu, p.ntm * p.ntn);
  const int nper = grid / 8;
  p.xcd_map = (grid % 8 == 0 && nper % p.ntn == 0 && nper >= p.ntn) ? 1 : 0;
  p.nper = nper;
  if (!p.xcd_map) grid = std::max(p.ntn, grid / p.ntn * p.ntn);
  const bool s = stats != nullptr;
  // ring depth: the LDS the resident weights leave (144 KB in all: one workgroup per CU either way)
  if (K == 256) {
    if (s) launch_ps<256, 5, true>(p, cw, grid, st); else launch_ps<256, 5, false>(p, cw, grid, st);
  } else if (K == 128) {
    if (s) launch_ps<128, 7, true>(p, cw, grid, st); else launch_ps<128, 7, false>(p, cw, grid, st);
  } else {
    if (s) launch_ps<64, 8, true>(p, cw, grid, st); else launch_ps<64, 8, false>(p, cw, grid, st);
  }
  return true;
}

}  // namespace dcp
