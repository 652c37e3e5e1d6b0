// Max-pool backward gather shared by pool.hip (max-pool / BN + max-pool backward) and stem.hip
// (the fused stem backward).
#pragma once
#include "common.cuh"

namespace dcp {

// Sum of the pooled gradients whose window argmax is input pixel (n, hi, wi), 8 channels.
// ho*s - p <= hi <= ho*s - p + k - 1.  The stem geometry (3x3 / 2 / pad 1) has at most 2 x 2
// candidate windows: all four argmax and gradient loads are issued together from clamped
// addresses, duplicates and out-of-range windows masked (no per-window branches).
template <int KK, int SS, int PP>
__device__ __forceinline__ void gather_pool_grad(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx, int n,
                                                 int hi, int wi, int Ho, int Wo, int C, int ch, int k, int s, int p,
                                                 float* g) {
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] = 0.f;
  if constexpr (KK == 3 && SS == 2 && PP == 1) {
    const int h0 = hi >> 1, h1 = (hi + 1) >> 1;  // candidate windows ho in {h0, h1} (equal for even hi)
    const int w0 = wi >> 1, w1 = (wi + 1) >> 1;
    uint64_t pk[4];
    bf16x8 gv[4];
    bool ok[4];
    uint8_t want[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int ho = (c >> 1) ? h1 : h0, wo = (c & 1) ? w1 : w0;
      ok[c] = ho < Ho && wo < Wo && ((c >> 1) == 0 || h1 != h0) && ((c & 1) == 0 || w1 != w0);
      want[c] = (uint8_t)((hi - (ho * 2 - 1)) * 3 + (wi - (wo * 2 - 1)));
      const size_t o = (size_t)((uint32_t)(n * Ho + min(ho, Ho - 1)) * Wo + min(wo, Wo - 1)) * C + ch * 8;
      pk[c] = *(const uint64_t*)(idx + o);
      gv[c] = *(const bf16x8*)(dy + o);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (ok[c] && ((pk[c] >> (8 * q)) & 0xff) == want[c]) g[q] += bf2f(gv[c][q]);
  } else {
    const int ho_lo = max(0, (hi + p - k + s) / s);  // ceil((hi+p-k+1)/s) for non-negative numerators
    const int ho_hi = min(Ho - 1, (hi + p) / s);
    const int wo_lo = max(0, (wi + p - k + s) / s);
    const int wo_hi = min(Wo - 1, (wi + p) / s);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = hi - (ho * s - p);
      if (kh < 0 || kh >= k) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = wi - (wo * s - p);
        if (kw < 0 || kw >= k) continue;
        const size_t o = (size_t)((uint32_t)(n * Ho + ho) * Wo + wo) * C + ch * 8;
        const uint64_t packed = *(const uint64_t*)(idx + o);
        const bf16x8 gw = *(const bf16x8*)(dy + o);
        const uint8_t w = (uint8_t)(kh * k + kw);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (((packed >> (8 * q)) & 0xff) == w) g[q] += bf2f(gw[q]);
      }
    }
  }
}

}  // namespace dcp
