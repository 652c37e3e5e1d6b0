// Small-batch linear backward in ONE launch: the squeeze-excitation MLPs and classifier heads at the
// reference's per-GPU batches of 16-64 (TResNet-M's SE blocks, BASELINE/main.py:29-30; the MLP head,
// BASELINE/main.py:135-149).  At those batches every piece of a linear layer's backward is a few
// microseconds of launch-bound work, and the general path runs up to seven launches per layer:
// act_bwd, the data-gradient GEMM, the weight-gradient GEMM (+ its split-K reduce), and the bias
// column sums (partials + their sum).  TResNet-M at batch 16 runs 37 such layers per step.
//
// Here one grid covers all three outputs of y = act(x W^T + b):
//   g      = bf16(dy * act'(y))                    (act_bwd's rounding: the same operand values)
//   dW     = g^T x        [out][K] fp32            tiles of 64 x 64, K-loop over the N <= 64 rows
//   db     = sum_n g      [out]    fp32            by the dW tiles of the first K column
//   dx     = g W          [N][K]   bf16            tiles of N x 64, a loop over 64-wide chunks of out
// Workgroups [0, ntA) are dW / db tiles, [ntA, ntA + ntB) dx tiles.  fp32 FMA on the VALU in a fixed
// order (deterministic): with N <= 64 the weight gradient is 64 MACs per output and the data gradient
// N x 64 outputs per tile -- the matrix cores would idle on the operand loads anyway.
#include "common.cuh"
#include "launchers.h"

namespace dcp {

namespace {

constexpr int kLsMaxN = 64;

struct LinBwdParams {
  const bf16* dy;  // [N][ldd], the first `out` columns used
  const bf16* y;   // [N][ldd] act output (act != 0)
  const bf16* x;   // [N][K]
  const bf16* wt;  // [K][ldw] bf16 transposed weight (columns >= out unused)
  bf16* dx;        // [N][K] or nullptr
  float* dw;       // [out][K] or nullptr
  float* db;       // [out] or nullptr
  int N, K, out, ldd, ldw, act;
  int nto, ntkA, ntA, ntk;  // dW tiles: nto (out / 64) x ntkA (K / 64, 1 when only db); dx tiles: ntk
};

__device__ __forceinline__ float act_grad(float g, float yv, int act) {
  const float d = act == 2 ? yv * (1.f - yv) : (act == 1 ? (yv > 0.f ? 1.f : 0.f) : 1.f);
  return act ? bf2f(f2bf(g * d)) : g;
}

}  // namespace

__global__ void __launch_bounds__(256) linear_bwd_small_kernel(const LinBwdParams p) {
  __shared__ float gs[kLsMaxN][64];   // g rows of this workgroup's 64 outputs
  __shared__ float xs[kLsMaxN * 64];  // dW tiles: x rows [n][64];  dx tiles: W^T chunk [o][64 (k)]
  const int tid = threadIdx.x;
  const int N = p.N;
  if ((int)blockIdx.x < p.ntA) {
    // ---- dW tile (o0, k0) [+ db when k0 == 0] ----
    const int o0 = (blockIdx.x / p.ntkA) * 64, k0 = (blockIdx.x % p.ntkA) * 64;
    for (int i = tid; i < N * 64; i += 256) {
      const int n = i >> 6, c = i & 63, o = o0 + c, k = k0 + c;
      float g = 0.f;
      if (o < p.out) g = act_grad(bf2f(p.dy[(size_t)n * p.ldd + o]), p.act ? bf2f(p.y[(size_t)n * p.ldd + o]) : 0.f, p.act);
      gs[n][c] = g;
      xs[n * 64 + c] = (p.dw != nullptr && k < p.K) ? bf2f(p.x[(size_t)n * p.K + k]) : 0.f;
    }
    __syncthreads();
    const int ol = tid >> 2, kl = (tid & 3) * 16;
    const int o = o0 + ol;
    if (p.dw != nullptr) {
      float acc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      for (int n = 0; n < N; ++n) {
        const float g = gs[n][ol];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(g, xs[n * 64 + kl + j], acc[j]);
      }
      if (o < p.out) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (k0 + kl + j < p.K) p.dw[(size_t)o * p.K + k0 + kl + j] = acc[j];
      }
    }
    if (p.db != nullptr && k0 == 0 && (tid & 3) == 0 && o < p.out) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += gs[n][ol];
      p.db[o] = s;
    }
    return;
  }
  // ---- dx tile: columns k0 .. k0+63 of all N rows ----
  const int k0 = ((int)blockIdx.x - p.ntA) * 64;
  const int kl = tid & 63, ng = tid >> 6;  // this thread: column kl, rows ng, ng + 4, ...
  float acc[kLsMaxN / 4];
#pragma unroll
  for (int r = 0; r < kLsMaxN / 4; ++r) acc[r] = 0.f;
  for (int o0 = 0; o0 < p.out; o0 += 64) {
    __syncthreads();  // the previous chunk's reads retired
    for (int i = tid; i < N * 64; i += 256) {
      const int n = i >> 6, c = i & 63, o = o0 + c;
      float g = 0.f;
      if (o < p.out) g = act_grad(bf2f(p.dy[(size_t)n * p.ldd + o]), p.act ? bf2f(p.y[(size_t)n * p.ldd + o]) : 0.f, p.act);
      gs[n][c] = g;
    }
    for (int i = tid; i < 64 * 64; i += 256) {
      const int kk = i >> 6, c = i & 63, o = o0 + c, k = k0 + kk;  // W^T row k, 64 consecutive o
      xs[c * 64 + kk] = (o < p.out && k < p.K) ? bf2f(p.wt[(size_t)k * p.ldw + o]) : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int c = 0; c < 64; ++c) {
      const float wv = xs[c * 64 + kl];
#pragma unroll
      for (int r = 0; r < kLsMaxN / 4; ++r)
        if (ng + 4 * r < N) acc[r] = fmaf(gs[ng + 4 * r][c], wv, acc[r]);
    }
  }
  if (k0 + kl < p.K) {
#pragma unroll
    for (int r = 0; r < kLsMaxN / 4; ++r)
      if (ng + 4 * r < N) p.dx[(size_t)(ng + 4 * r) * p.K + k0 + kl] = f2bf(acc[r]);
  }
}

bool linear_bwd_small_supported(int N, int K, int out) { return N >= 1 && N <= kLsMaxN && K >= 1 && out >= 1; }

bool launch_linear_bwd_small(const bf16* dy, const bf16* y, const bf16* x, const bf16* wt, bf16* dx, float* dw,
                             float* db, int N, int K, int out, int ldd, int ldw, int act, hipStream_t st) {
  if (!linear_bwd_small_supported(N, K, out) || (dx == nullptr && dw == nullptr && db == nullptr)) return false;
  LinBwdParams p;
  p.dy = dy; p.y = y; p.x = x; p.wt = wt; p.dx = dx; p.dw = dw; p.db = db;
  p.N = N; p.K = K; p.out = out; p.ldd = ldd; p.ldw = ldw; p.act = act;
  p.nto = (out + 63) / 64;
  p.ntk = (K + 63) / 64;
  p.ntkA = dw != nullptr ? p.ntk : 1;
  p.ntA = (dw != nullptr || db != nullptr) ? p.nto * p.ntkA : 0;
  const int grid = p.ntA + (dx != nullptr ? p.ntk : 0);
  hipLaunchKernelGGL(linear_bwd_small_kernel, dim3(grid), dim3(256), 0, st, p);
  return true;
}

}  // namespace dcp
