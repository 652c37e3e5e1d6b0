// Row-wise classification-loss kernels: softmax cross-entropy (+ label rank
// for top-k accuracy in the same pass), log-softmax, ArcFace additive
// angular margin head.
//
// Replaces nn.CrossEntropyLoss (BASELINE/main.py:152, ARCFACE/arc_main.py:245,
// CDR/main.py:243, NESTED/train.py:385), nn.LogSoftmax (ARCFACE/arc_main.py:230,
// CDR/main.py:336), the top-1/top-3 helpers (BASELINE/main.py:156-168,199-209,
// NESTED/utils.py:32-46) and ArcMarginProduct (ARCFACE/arc_main.py:130-176);
// SURVEY.md §2.5 K11, K12, K13, K16.
#include "common.cuh"
#include "launchers.h"

namespace dcp {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return (float)*p; }

// One workgroup per row. logits [B][ld] (bf16 or fp32), C valid classes.
// loss[b] = logsumexp(x) - x[label]; rank[b] = #{j : x_j > x_label}
template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, int ld, int C,
                                                       const int64_t* __restrict__ labels, float* __restrict__ loss,
                                                       int* __restrict__ rank, float smoothing) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const T* row = logits + (size_t)b * ld;
  const int lab = (int)labels[b];
  const float xl = (lab >= 0 && lab < C) ? ldf(row + lab) : 0.f;
  float mx = -INFINITY;
  int cnt = 0;
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const float v = ldf(row + j);
    mx = fmaxf(mx, v);
    cnt += v > xl;
  }
  mx = block_max(mx, red);
  float se = 0.f, sx = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const float v = ldf(row + j);
    se += __expf(v - mx);
    sx += v;
  }
  se = block_sum(se, red);
  sx = block_sum(sx, red);
  const float c = block_sum((float)cnt, red);
  if (threadIdx.x == 0) {
    const float lse = mx + __logf(se);
    float l = lse - xl;
    if (smoothing > 0.f) l = (1.f - smoothing) * l + smoothing * (lse - sx / C);
    loss[b] = (lab >= 0 && lab < C) ? l : 0.f;
    if (rank) rank[b] = (int)c;
  }
}

// dlogits = g * (softmax(x) - onehot) ; g = grad_out[0] * scale ; pad columns -> 0
template <typename T, typename TO>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, int ld, int C,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ grad_out, float scale,
                                                       float smoothing, TO* __restrict__ dlogits, int ldo) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const T* row = logits + (size_t)b * ld;
  const int lab = (int)labels[b];
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < C; j += blockDim.x) mx = fmaxf(mx, ldf(row + j));
  mx = block_max(mx, red);
  float se = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) se += __expf(ldf(row + j) - mx);
  se = block_sum(se, red);
  const float inv = 1.f / se;
  const bool valid = lab >= 0 && lab < C;
  const float g = valid ? grad_out[0] * scale : 0.f;
  TO* drow = dlogits + (size_t)b * ldo;
  for (int j = threadIdx.x; j < ldo; j += blockDim.x) {
    float d = 0.f;
    if (j < C) {
      const float pj = __expf(ldf(row + j) - mx) * inv;
      const float tgt = (1.f - smoothing) * (j == lab ? 1.f : 0.f) + smoothing / C;
      d = g * (pj - tgt);
    }
    drow[j] = (TO)d;
  }
}

// log-softmax fwd (fp32 out) and bwd: dx = dy - softmax * sum(dy)
template <typename T>
__global__ void __launch_bounds__(256) log_softmax_fwd_kernel(const T* __restrict__ x, int ld, int C,
                                                              float* __restrict__ y) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const T* row = x + (size_t)b * ld;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < C; j += blockDim.x) mx = fmaxf(mx, ldf(row + j));
  mx = block_max(mx, red);
  float se = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) se += __expf(ldf(row + j) - mx);
  se = block_sum(se, red);
  const float lse = mx + __logf(se);
  for (int j = threadIdx.x; j < C; j += blockDim.x) y[(size_t)b * C + j] = ldf(row + j) - lse;
}

template <typename TO>
__global__ void __launch_bounds__(256) log_softmax_bwd_kernel(const float* __restrict__ y,
                                                              const float* __restrict__ dy, int C, int ldo,
                                                              TO* __restrict__ dx) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  float s = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) s += dy[(size_t)b * C + j];
  s = block_sum(s, red);
  for (int j = threadIdx.x; j < ldo; j += blockDim.x) {
    float d = 0.f;
    if (j < C) d = dy[(size_t)b * C + j] - __expf(y[(size_t)b * C + j]) * s;
    dx[(size_t)b * ldo + j] = (TO)d;
  }
}

// ---------------------------------------------------------------------------
// ArcFace (additive angular margin), ARCFACE/arc_main.py:130-176.
//   cos = <x/|x|, w_j/|w_j|> ; sin = sqrt(clamp(1-cos^2, 0, 1))
//   phi = cos*cos_m - sin*sin_m ; easy: phi = cos>0 ? phi : cos ; hard: cos>th ? phi : cos-mm
//   out_j = s * (j == label ? phi : cos)
// The cosine GEMM runs on our MFMA tap-GEMM kernel over L2-normalised bf16
// operands; these kernels do the normalisation and the fused margin +
// softmax-CE with its backward through the margin (guarding cos = +-1).
// ---------------------------------------------------------------------------

// rows of x [R][D] (fp32 or bf16) -> bf16 normalised rows [Rout][ldo] (zero-padded in both
// dimensions, Rout >= R), inverse norms [Rout]
template <typename T>
__global__ void __launch_bounds__(256) l2norm_rows_kernel(const T* __restrict__ x, int R, int D, int ldo,
                                                          bf16* __restrict__ y, float* __restrict__ inv_norm,
                                                          float eps) {
  __shared__ float red[16];
  const int r = blockIdx.x;
  if (r >= R) {  // padding rows of the GEMM operand (R rounded up to the tile): zero, inverse norm 0
    for (int j = threadIdx.x; j < ldo; j += blockDim.x) y[(size_t)r * ldo + j] = f2bf(0.f);
    if (threadIdx.x == 0) inv_norm[r] = 0.f;
    return;
  }
  const T* row = x + (size_t)r * D;
  float s = 0.f;
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    const float v = ldf(row + j);
    s += v * v;
  }
  s = block_sum(s, red);
  const float inv = 1.f / fmaxf(sqrtf(s), eps);
  if (threadIdx.x == 0) inv_norm[r] = inv;
  for (int j = threadIdx.x; j < ldo; j += blockDim.x) y[(size_t)r * ldo + j] = f2bf(j < D ? ldf(row + j) * inv : 0.f);
}

// cos [B][ld] (bf16 from the GEMM) -> margin logits (fp32 [B][C]) + CE loss + rank + dcos (bf16 [B][ld])
__global__ void __launch_bounds__(256) arcface_fwd_kernel(const bf16* __restrict__ cosv, int ld, int C,
                                                          const int64_t* __restrict__ labels, float s,
                                                          float cos_m, float sin_m, float th, float mm,
                                                          int easy_margin, float* __restrict__ out_logits,
                                                          float* __restrict__ loss, int* __restrict__ rank,
                                                          float* __restrict__ lab_dphi) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const bf16* row = cosv + (size_t)b * ld;
  const int lab = (int)labels[b];
  const bool valid = lab >= 0 && lab < C;
  float phi = 0.f, dphi = 0.f;
  if (valid) {
    float c = fminf(fmaxf(bf2f(row[lab]), -1.f), 1.f);
    const float sn = sqrtf(fminf(fmaxf(1.f - c * c, 0.f), 1.f));
    const float p = c * cos_m - sn * sin_m;
    // d phi / d cos = cos_m + sin_m * cos / sin (sin -> 0 guarded)
    const float dp = cos_m + (sn > 1e-6f ? sin_m * c / sn : 0.f);
    if (easy_margin) {
      phi = c > 0.f ? p : c;
      dphi = c > 0.f ? dp : 1.f;
    } else {
      phi = c > th ? p : c - mm;
      dphi = c > th ? dp : 1.f;
    }
  }
  const float xl = s * phi;
  float mx = -INFINITY;
  int cnt = 0;
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const float v = (j == lab) ? xl : s * bf2f(row[j]);
    if (out_logits) out_logits[(size_t)b * C + j] = v;
    mx = fmaxf(mx, v);
    cnt += v > xl;
  }
  mx = block_max(mx, red);
  float se = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const float v = (j == lab) ? xl : s * bf2f(row[j]);
    se += __expf(v - mx);
  }
  se = block_sum(se, red);
  const float c = block_sum((float)cnt, red);
  if (threadIdx.x == 0) {
    loss[b] = valid ? mx + __logf(se) - xl : 0.f;
    if (rank) rank[b] = (int)c;
    lab_dphi[b] = dphi;
  }
}

// dcos_j = g * s * (p_j - onehot_j) * (j == label ? dphi : 1)
__global__ void __launch_bounds__(256) arcface_bwd_kernel(const bf16* __restrict__ cosv, int ld, int C,
                                                          const int64_t* __restrict__ labels, float s,
                                                          float cos_m, float sin_m, float th, float mm,
                                                          int easy_margin, const float* __restrict__ lab_dphi,
                                                          const float* __restrict__ grad_out, float scale,
                                                          bf16* __restrict__ dcos) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const bf16* row = cosv + (size_t)b * ld;
  const int lab = (int)labels[b];
  const bool valid = lab >= 0 && lab < C;
  float phi = 0.f;
  if (valid) {
    float c = fminf(fmaxf(bf2f(row[lab]), -1.f), 1.f);
    const float sn = sqrtf(fminf(fmaxf(1.f - c * c, 0.f), 1.f));
    const float p = c * cos_m - sn * sin_m;
    phi = easy_margin ? (c > 0.f ? p : c) : (c > th ? p : c - mm);
  }
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < C; j += blockDim.x) mx = fmaxf(mx, (j == lab) ? s * phi : s * bf2f(row[j]));
  mx = block_max(mx, red);
  float se = 0.f;
  for (int j = threadIdx.x; j < C; j += blockDim.x) se += __expf(((j == lab) ? s * phi : s * bf2f(row[j])) - mx);
  se = block_sum(se, red);
  const float inv = 1.f / se;
  const float g = valid ? grad_out[0] * scale : 0.f;
  for (int j = threadIdx.x; j < ld; j += blockDim.x) {
    float d = 0.f;
    if (j < C) {
      const float v = (j == lab) ? s * phi : s * bf2f(row[j]);
      const float pj = __expf(v - mx) * inv;
      d = g * s * (pj - (j == lab ? 1.f : 0.f)) * (j == lab ? lab_dphi[b] : 1.f);
    }
    dcos[(size_t)b * ld + j] = f2bf(d);
  }
}

// backward through y = x/|x| :  dx = inv * (dy - y * <dy, y>)   (dy bf16 [R][ldd], y bf16 [R][ldy])
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) l2norm_bwd_kernel(const TI* __restrict__ dy, int ldd,
                                                         const bf16* __restrict__ y, int ldy,
                                                         const float* __restrict__ inv_norm, int D,
                                                         TO* __restrict__ dx) {
  __shared__ float red[16];
  const int r = blockIdx.x;
  float dot = 0.f;
  for (int j = threadIdx.x; j < D; j += blockDim.x) dot += ldf(dy + (size_t)r * ldd + j) * bf2f(y[(size_t)r * ldy + j]);
  dot = block_sum(dot, red);
  const float inv = inv_norm[r];
  for (int j = threadIdx.x; j < D; j += blockDim.x)
    dx[(size_t)r * D + j] = (TO)(inv * (ldf(dy + (size_t)r * ldd + j) - bf2f(y[(size_t)r * ldy + j]) * dot));
}

// ---------------------------------------------------------------------------
void launch_xent_fwd(const void* logits, bool is_bf16, int B, int ld, int C, const int64_t* labels, float* loss,
                     int* rank, float smoothing, hipStream_t s) {
  if (is_bf16)
    hipLaunchKernelGGL(xent_fwd_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)logits, ld, C, labels, loss,
                       rank, smoothing);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)logits, ld, C, labels, loss,
                       rank, smoothing);
}

void launch_xent_bwd(const void* logits, bool in_bf16, int B, int ld, int C, const int64_t* labels,
                     const float* grad_out, float scale, float smoothing, void* dlogits, int ldo, bool out_bf16,
                     hipStream_t s) {
  if (in_bf16 && out_bf16)
    hipLaunchKernelGGL((xent_bwd_kernel<bf16, bf16>), dim3(B), dim3(256), 0, s, (const bf16*)logits, ld, C, labels,
                       grad_out, scale, smoothing, (bf16*)dlogits, ldo);
  else if (in_bf16)
    hipLaunchKernelGGL((xent_bwd_kernel<bf16, float>), dim3(B), dim3(256), 0, s, (const bf16*)logits, ld, C,
                       labels, grad_out, scale, smoothing, (float*)dlogits, ldo);
  else if (out_bf16)
    hipLaunchKernelGGL((xent_bwd_kernel<float, bf16>), dim3(B), dim3(256), 0, s, (const float*)logits, ld, C,
                       labels, grad_out, scale, smoothing, (bf16*)dlogits, ldo);
  else
    hipLaunchKernelGGL((xent_bwd_kernel<float, float>), dim3(B), dim3(256), 0, s, (const float*)logits, ld, C,
                       labels, grad_out, scale, smoothing, (float*)dlogits, ldo);
}

void launch_log_softmax_fwd(const void* x, bool is_bf16, int B, int ld, int C, float* y, hipStream_t s) {
  if (is_bf16)
    hipLaunchKernelGGL(log_softmax_fwd_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)x, ld, C, y);
  else
    hipLaunchKernelGGL(log_softmax_fwd_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)x, ld, C, y);
}

void launch_log_softmax_bwd(const float* y, const float* dy, int B, int C, int ldo, void* dx, bool out_bf16,
                            hipStream_t s) {
  if (out_bf16)
    hipLaunchKernelGGL(log_softmax_bwd_kernel<bf16>, dim3(B), dim3(256), 0, s, y, dy, C, ldo, (bf16*)dx);
  else
    hipLaunchKernelGGL(log_softmax_bwd_kernel<float>, dim3(B), dim3(256), 0, s, y, dy, C, ldo, (float*)dx);
}

void launch_l2norm_rows(const void* x, bool is_bf16, int R, int Rout, int D, int ldo, bf16* y, float* inv_norm,
                        float eps, hipStream_t s) {
  if (is_bf16)
    hipLaunchKernelGGL(l2norm_rows_kernel<bf16>, dim3(Rout), dim3(256), 0, s, (const bf16*)x, R, D, ldo, y, inv_norm,
                       eps);
  else
    hipLaunchKernelGGL(l2norm_rows_kernel<float>, dim3(Rout), dim3(256), 0, s, (const float*)x, R, D, ldo, y,
                       inv_norm, eps);
}

void launch_l2norm_bwd(const void* dy, bool dy_bf16, int ldd, const bf16* y, int ldy, const float* inv_norm, int R,
                       int D, void* dx, bool out_bf16, hipStream_t s) {
  if (dy_bf16 && out_bf16)
    hipLaunchKernelGGL((l2norm_bwd_kernel<bf16, bf16>), dim3(R), dim3(256), 0, s, (const bf16*)dy, ldd, y, ldy,
                       inv_norm, D, (bf16*)dx);
  else if (dy_bf16)
    hipLaunchKernelGGL((l2norm_bwd_kernel<bf16, float>), dim3(R), dim3(256), 0, s, (const bf16*)dy, ldd, y, ldy,
                       inv_norm, D, (float*)dx);
  else if (out_bf16)
    hipLaunchKernelGGL((l2norm_bwd_kernel<float, bf16>), dim3(R), dim3(256), 0, s, (const float*)dy, ldd, y, ldy,
                       inv_norm, D, (bf16*)dx);
  else
    hipLaunchKernelGGL((l2norm_bwd_kernel<float, float>), dim3(R), dim3(256), 0, s, (const float*)dy, ldd, y, ldy,
                       inv_norm, D, (float*)dx);
}

void launch_arcface_fwd(const bf16* cosv, int B, int ld, int C, const int64_t* labels, float s, float cos_m,
                        float sin_m, float th, float mm, int easy, float* out_logits, float* loss, int* rank,
                        float* lab_dphi, hipStream_t st) {
  hipLaunchKernelGGL(arcface_fwd_kernel, dim3(B), dim3(256), 0, st, cosv, ld, C, labels, s, cos_m, sin_m, th, mm,
                     easy, out_logits, loss, rank, lab_dphi);
}

void launch_arcface_bwd(const bf16* cosv, int B, int ld, int C, const int64_t* labels, float s, float cos_m,
                        float sin_m, float th, float mm, int easy, const float* lab_dphi, const float* grad_out,
                        float scale, bf16* dcos, hipStream_t st) {
  hipLaunchKernelGGL(arcface_bwd_kernel, dim3(B), dim3(256), 0, st, cosv, ld, C, labels, s, cos_m, sin_m, th, mm,
                     easy, lab_dphi, grad_out, scale, dcos);
}

// Training / validation metric accumulation in one launch (replaces the per-step compare / sum /
// cast / stack / add chain and the host->device count copy of the loops): with one workgroup,
//   acc[0] += loss_scale * sum(loss[0 .. nloss)),  acc[1] += #{rank[i] < 1},  acc[2] += #{rank[i] < 3},
//   acc[3] += nrows        (i < nrows; acc fp64, the count a kernel argument -- no host copy)
__global__ void __launch_bounds__(256) metric_accum_kernel(double* __restrict__ acc, const float* __restrict__ loss,
                                                           int nloss, float loss_scale, const int* __restrict__ rank,
                                                           int nrows) {
  __shared__ float red[16];
  float ls = 0.f, t1 = 0.f, t3 = 0.f;
  for (int i = threadIdx.x; i < nloss; i += blockDim.x) ls += loss[i];
  for (int i = threadIdx.x; i < nrows; i += blockDim.x) {
    const int r = rank[i];
    t1 += r < 1 ? 1.f : 0.f;
    t3 += r < 3 ? 1.f : 0.f;
  }
  ls = block_sum(ls, red);
  t1 = block_sum(t1, red);
  t3 = block_sum(t3, red);
  if (threadIdx.x == 0) {
    acc[0] += (double)ls * (double)loss_scale;
    acc[1] += (double)t1;
    acc[2] += (double)t3;
    acc[3] += (double)nrows;
  }
}

void launch_metric_accum(double* acc, const float* loss, int nloss, float loss_scale, const int* rank, int nrows,
                         hipStream_t s) {
  metric_accum_kernel<<<1, 256, 0, s>>>(acc, loss, nloss, loss_scale, rank, nrows);
}

}  // namespace dcp
