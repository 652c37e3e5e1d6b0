// PyTorch operator registrations (namespace `dcp`) for the gfx950 kernels.
//
// Every op takes device tensors, checks shapes/dtypes on the host (a wrong
// shape must never reach a kernel), and launches on the current HIP stream so
// it composes with autograd, torch.distributed (RCCL) and HIP graph capture.
// No allocation-free variants are needed: the PyTorch caching allocator
// serves every output.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <torch/library.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "launchers.h"

using at::Tensor;
using std::optional;

namespace {

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be fp32")
#define CHECK_ACT(t) \
  do {               \
    CHECK_DEV(t);    \
    CHECK_CONTIG(t); \
    CHECK_BF16(t);   \
  } while (0)

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// kernel scratch from PyTorch's caching allocator: stream-ordered reuse, and a HIP-graph capture
// takes it from the graph's private pool (registered once at library load)
struct WorkspaceRegistration {
  WorkspaceRegistration() {
    dcp::set_workspace_allocator(
        [](size_t n, hipStream_t s) -> void* { return c10::hip::HIPCachingAllocator::raw_alloc_with_stream(n, s); },
        [](void* p) { c10::hip::HIPCachingAllocator::raw_delete(p); });
  }
} g_workspace_registration;

// fork / join events of the parity-class streams (conv_dgrad stride 2), one set per device; reused
// call after call (an event re-recorded after every wait on it was issued, stream-ordered)
hipEvent_t parity_event(int i) {
  static std::mutex mu;
  static std::unordered_map<int, std::vector<hipEvent_t>> pool;
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto& v = pool[dev];
  while ((int)v.size() <= i) {
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    v.push_back(e);
  }
  return v[i];
}

const bf16* bp(const Tensor& t) { return reinterpret_cast<const bf16*>(t.data_ptr()); }
bf16* bpm(Tensor& t) { return reinterpret_cast<bf16*>(t.data_ptr()); }
const float* fp(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }
float* fpm(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }

// 256 zero bytes per device: the source of every out-of-bounds implicit-GEMM lane
const bf16* zero_page(int dev) {
  static std::mutex mu;
  static std::vector<void*> pages(64, nullptr);
  std::lock_guard<std::mutex> g(mu);
  if (!pages[dev]) {
    void* p = nullptr;
    TORCH_CHECK(hipMalloc(&p, 256) == hipSuccess, "zero page alloc failed");
    TORCH_CHECK(hipMemset(p, 0, 256) == hipSuccess, "zero page memset failed");
    pages[dev] = p;
  }
  return reinterpret_cast<const bf16*>(pages[dev]);
}

int num_cus(int dev) {
  static std::vector<int> cache(64, 0);
  if (!cache[dev]) {
    hipDeviceProp_t prop;
    TORCH_CHECK(hipGetDeviceProperties(&prop, dev) == hipSuccess);
    cache[dev] = prop.multiProcessorCount;
  }
  return cache[dev];
}

at::TensorOptions bf16_like(const Tensor& t) { return t.options().dtype(at::kBFloat16); }
at::TensorOptions f32_like(const Tensor& t) { return t.options().dtype(at::kFloat); }

// ---------------------------------------------------------------------------
// convolution
// ---------------------------------------------------------------------------
dcp::TapList fwd_taps(int KH, int KW, int pad) {
  dcp::TapList t;
  t.n = KH * KW;
  TORCH_CHECK(t.n <= dcp::kMaxTaps, "kernel too large");
  for (int kh = 0; kh < KH; ++kh)
    for (int kw = 0; kw < KW; ++kw) {
      const int i = kh * KW + kw;
      t.dy[i] = kh - pad;
      t.dx[i] = kw - pad;
      t.widx[i] = i;
    }
  return t;
}

// x [N,H,W,C] bf16, w [Co,KH,KW,C] bf16 -> y [N,Ho,Wo,Co], stats slabs [ceil(M/128),2,Co]
std::tuple<Tensor, Tensor> conv_fwd(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad, bool stats) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv_fwd expects NHWC input and [Co,KH,KW,Ci] weight");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(w.size(3) == C, "weight Ci mismatch");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "conv_fwd needs C and Co multiples of 8");
  TORCH_CHECK(KH * KW <= dcp::kMaxTaps && pad <= 100 && KH <= 100, "unsupported conv geometry");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty conv output");
  // GEMM rows (pixels) index as int; element offsets are 64-bit (large per-GPU batches pass 2^32
  // elements: tests/test_large_batch_gpu.py)
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31) && (int64_t)N * Ho * Wo < (1ll << 31), "conv_fwd: too many pixels");
  auto y = at::empty({N, Ho, Wo, Co}, bf16_like(x));
  const int M = N * Ho * Wo;
  if (stride == 1 && pad == 1 && KH == 3 && KW == 3 && dcp::conv3x3_c64_supported(H, W, C, Co)) {
    // direct 64 -> 64 channel 3x3 kernel (conv3x3.hip); statistics as (n, mean, M2) partials
    const int blocks = dcp::conv3x3_c64_blocks(N, H, W, num_cus(x.get_device()));
    Tensor part = stats ? at::empty({blocks, 3, Co}, f32_like(x)) : at::empty({0}, f32_like(x));
    dcp::launch_conv3x3_c64(bp(x), bp(w), bpm(y), stats ? part.data_ptr<float>() : nullptr, zero_page(x.get_device()),
                            N, H, W, blocks, cur_stream());
    return {y, part};
  }
  Tensor slabs;
  if (stats)
    slabs = at::empty({(M + 127) / 128, 2, Co}, f32_like(x));
  else
    slabs = at::empty({0}, f32_like(x));
  const auto taps = fwd_taps(KH, KW, pad);
  dcp::launch_tap_gemm(bp(x), N, H, W, C, bp(w), Co, KH * KW, bpm(y), Ho, Wo, Ho, Wo, stride, 1, 0, 0, taps,
                       stats ? slabs.data_ptr<float>() : nullptr, nullptr, 0, zero_page(x.get_device()),
                       cur_stream());
  return {y, slabs};
}

// forward conv with an eval-mode BN folded into the store: y = act(conv(x) * scale + shift [+ res])
// (scale / shift per output channel, fp32; the BN of running statistics, AffineEpi in launchers.h)
Tensor conv_fwd_affine(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad, const Tensor& scale,
                       const Tensor& shift, int64_t act, double slope, const optional<Tensor>& res) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv_fwd_affine expects NHWC input and [Co,KH,KW,Ci] weight");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(w.size(3) == C && C % 8 == 0 && Co % 8 == 0, "conv_fwd_affine channels");
  TORCH_CHECK(KH * KW <= dcp::kMaxTaps && pad <= 100 && KH <= 100, "unsupported conv geometry");
  TORCH_CHECK(act >= 0 && act <= 2, "conv_fwd_affine: act must be none, ReLU or leaky ReLU");
  for (const Tensor* t : {&scale, &shift}) {
    CHECK_DEV(*t);
    CHECK_F32(*t);
    CHECK_CONTIG(*t);
    TORCH_CHECK(t->numel() == Co, "conv_fwd_affine: per-channel vector size");
  }
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty conv output");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31) && (int64_t)N * Ho * Wo < (1ll << 31), "conv_fwd_affine: too many pixels");
  auto y = at::empty({N, Ho, Wo, Co}, bf16_like(x));
  const bf16* resp = nullptr;
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == y.sizes(), "conv_fwd_affine residual shape");
    resp = bp(*res);
  }
  const auto taps = fwd_taps(KH, KW, pad);
  dcp::AffineEpi aff{scale.data_ptr<float>(), shift.data_ptr<float>(), (int)act, (float)slope};
  dcp::launch_tap_gemm(bp(x), N, H, W, C, bp(w), Co, KH * KW, bpm(y), Ho, Wo, Ho, Wo, stride, 1, 0, 0, taps, nullptr,
                       nullptr, 0, zero_page(x.get_device()), cur_stream(), resp, nullptr, &aff);
  return y;
}

void check_pro_vec(const Tensor& t, int C, const char* what) {
  CHECK_DEV(t);
  CHECK_F32(t);
  CHECK_CONTIG(t);
  TORCH_CHECK(t.numel() == C, what, ": per-input-channel vector size");
}

// 1x1 stride-1 conv of relu(x * scale + shift) with that BN + ReLU applied to the A operand in
// registers (K5 prologue; x is the BN's input, the normalised activation is never written).
// -> (y, BN statistics slabs of y or empty), as conv_fwd
std::tuple<Tensor, Tensor> conv_fwd_pro(const Tensor& x, const Tensor& w, const Tensor& scale, const Tensor& shift,
                                        bool stats) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(1) == 1 && w.size(2) == 1, "conv_fwd_pro: 1x1 NHWC conv");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Co = w.size(0);
  TORCH_CHECK(w.size(3) == C && C % 64 == 0 && Co % 8 == 0, "conv_fwd_pro: C % 64 == 0, Co % 8 == 0");
  check_pro_vec(scale, C, "conv_fwd_pro scale");
  check_pro_vec(shift, C, "conv_fwd_pro shift");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "conv_fwd_pro: too many pixels");
  auto y = at::empty({N, H, W, Co}, bf16_like(x));
  const int M = N * H * W;
  Tensor slabs = stats ? at::empty({(M + 127) / 128, 2, Co}, f32_like(x)) : at::empty({0}, f32_like(x));
  const auto taps = fwd_taps(1, 1, 0);
  dcp::launch_tap_gemm(bp(x), N, H, W, C, bp(w), Co, 1, bpm(y), H, W, H, W, 1, 1, 0, 0, taps,
                       stats ? slabs.data_ptr<float>() : nullptr, nullptr, 0, zero_page(x.get_device()), cur_stream(),
                       nullptr, nullptr, nullptr, scale.data_ptr<float>(), shift.data_ptr<float>());
  return {y, slabs};
}

// weight gradient of conv_fwd_pro: dW = dY^T relu(x * scale + shift), the input recomputed in the
// B-fragment registers
Tensor conv_wgrad_pro(const Tensor& dy, const Tensor& x, const Tensor& scale, const Tensor& shift) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = dy.size(0), H = dy.size(1), W = dy.size(2), Co = dy.size(3), C = x.size(3);
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == H && x.size(2) == W, "conv_wgrad_pro: 1x1 geometry");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0 && C <= 2048 && !(Co <= 64 && C >= 128), "conv_wgrad_pro: channel layout");
  check_pro_vec(scale, C, "conv_wgrad_pro scale");
  check_pro_vec(shift, C, "conv_wgrad_pro shift");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "conv_wgrad_pro: too many pixels");
  auto dw = at::empty({Co, 1, 1, C}, f32_like(dy));
  const auto taps = fwd_taps(1, 1, 0);
  const int ncu = num_cus(dy.get_device());
  const int splits = dcp::wgrad_plan_splits(N, H, W, Co, H, W, C, 1, taps, ncu);
  auto part = at::empty({splits > 1 ? (int64_t)(splits + (splits + 63) / 64) * dw.numel() : 4}, f32_like(dy));
  dcp::launch_wgrad(bp(dy), N, H, W, Co, bp(x), H, W, C, 1, taps, dw.data_ptr<float>(), part.data_ptr<float>(),
                    zero_page(dy.get_device()), ncu, cur_stream(), scale.data_ptr<float>(), shift.data_ptr<float>());
  return dw;
}

// conv3x3(relu(x * scale + shift)) for the 64 -> 64 channel stride-1 3x3 (the direct kernel's BN
// prologue, K5 on a 3x3 consumer): the BN + ReLU is applied once per staged window element
std::tuple<Tensor, Tensor> conv3x3_fwd_pro(const Tensor& x, const Tensor& w, const Tensor& scale, const Tensor& shift,
                                           bool stats) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Co = w.size(0);
  TORCH_CHECK(w.dim() == 4 && w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C, "conv3x3_fwd_pro: [Co,3,3,C]");
  TORCH_CHECK(dcp::conv3x3_c64_supported(H, W, C, Co), "conv3x3_fwd_pro: the direct 64-channel 3x3 geometry only");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "conv3x3_fwd_pro: too many pixels");
  check_pro_vec(scale, C, "conv3x3_fwd_pro scale");
  check_pro_vec(shift, C, "conv3x3_fwd_pro shift");
  auto y = at::empty({N, H, W, Co}, bf16_like(x));
  const int blocks = dcp::conv3x3_c64_blocks(N, H, W, num_cus(x.get_device()));
  Tensor part = stats ? at::empty({blocks, 3, Co}, f32_like(x)) : at::empty({0}, f32_like(x));
  dcp::launch_conv3x3_c64(bp(x), bp(w), bpm(y), stats ? part.data_ptr<float>() : nullptr, zero_page(x.get_device()),
                          N, H, W, blocks, cur_stream(), scale.data_ptr<float>(), shift.data_ptr<float>());
  return {y, part};
}

// weight gradient of conv3x3_fwd_pro: the direct 3x3 weight gradient recomputing relu(x * scale +
// shift) on its staged windows
Tensor conv3x3_wgrad_pro(const Tensor& dy, const Tensor& x, const Tensor& scale, const Tensor& shift) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = dy.size(0), H = dy.size(1), W = dy.size(2), Co = dy.size(3), C = x.size(3);
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == H && x.size(2) == W, "conv3x3_wgrad_pro: geometry");
  check_pro_vec(scale, C, "conv3x3_wgrad_pro scale");
  check_pro_vec(shift, C, "conv3x3_wgrad_pro shift");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "conv3x3_wgrad_pro: too many pixels");
  const int ncu = num_cus(dy.get_device());
  const int s3 = dcp::wgrad3x3_splits(N, H, W, C, Co, ncu);
  TORCH_CHECK(s3 > 0, "conv3x3_wgrad_pro: the direct 3x3 weight-gradient geometry only");
  auto dw = at::empty({Co, 3, 3, C}, f32_like(dy));
  const auto taps = fwd_taps(3, 3, 1);
  auto part = at::empty({(int64_t)(s3 + (s3 + 63) / 64) * dw.numel()}, f32_like(dy));
  dcp::launch_wgrad(bp(dy), N, H, W, Co, bp(x), H, W, C, 1, taps, dw.data_ptr<float>(), part.data_ptr<float>(),
                    zero_page(dy.get_device()), ncu, cur_stream(), scale.data_ptr<float>(), shift.data_ptr<float>());
  return dw;
}

// the direct 3x3 kernels' BN prologue applies (a bottleneck's bn1 -> conv2 at 64 channels)
bool conv3x3_pro_fits(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co) {
  return dcp::conv3x3_c64_supported(H, W, C, Co) && dcp::wgrad3x3_splits(N, H, W, C, Co, 256) > 0;
}

// backward of act(c * scale + shift [+ r]) from its output y: (dc = g * scale, g = dy * act'(y) or empty)
std::tuple<Tensor, Tensor> act_scale_bwd(const Tensor& dy, const Tensor& y, const Tensor& scale, int64_t act,
                                         double slope, bool want_g) {
  CHECK_ACT(dy);
  CHECK_ACT(y);
  TORCH_CHECK(dy.sizes() == y.sizes() && dy.dim() >= 2, "act_scale_bwd shapes");
  const int C = y.size(-1);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "act_scale_bwd: C/8 must divide 256");
  CHECK_DEV(scale);
  CHECK_F32(scale);
  TORCH_CHECK(scale.is_contiguous() && scale.numel() == C, "act_scale_bwd: scale [C]");
  auto dc = at::empty_like(dy);
  Tensor g = want_g ? at::empty_like(dy) : at::empty({0}, dy.options());
  const int64_t M = dy.numel() / C;
  TORCH_CHECK(M < (1ll << 31), "act_scale_bwd: too many rows");
  dcp::launch_act_scale_bwd(bp(dy), bp(y), scale.data_ptr<float>(), M, C, (int)act, (float)slope, bpm(dc),
                            want_g ? bpm(g) : nullptr, cur_stream());
  return {dc, g};
}

// Philox dropout: (y, used) -- `offset` int64[1] device call counter (bumped here after the launch,
// graph-capturable), `used` int64[1] receives the counter value the mask was drawn with
// InplaceABN effective weight and its reciprocal: (|g| + eps, 1 / (|g| + eps))
std::tuple<Tensor, Tensor> iabn_gamma(const Tensor& g, double eps) {
  CHECK_DEV(g);
  CHECK_F32(g);
  CHECK_CONTIG(g);
  auto geff = at::empty_like(g), rg = at::empty_like(g);
  dcp::launch_iabn_gamma(g.data_ptr<float>(), (float)eps, geff.data_ptr<float>(), rg.data_ptr<float>(), g.numel(),
                         cur_stream());
  return {geff, rg};
}

// d * sign(g) (the gradient of |g| + eps)
Tensor sign_mul(const Tensor& d, const Tensor& g) {
  CHECK_DEV(d);
  CHECK_F32(d);
  CHECK_F32(g);
  TORCH_CHECK(d.is_contiguous() && g.is_contiguous() && d.numel() == g.numel(), "sign_mul shapes");
  auto out = at::empty_like(d);
  dcp::launch_sign_mul(d.data_ptr<float>(), g.data_ptr<float>(), out.data_ptr<float>(), d.numel(), cur_stream());
  return out;
}

std::tuple<Tensor, Tensor> dropout_fwd(const Tensor& x, double p, int64_t seed, const Tensor& offset) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "dropout: bf16 or fp32");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout: p in [0, 1)");
  CHECK_DEV(offset);
  TORCH_CHECK(offset.scalar_type() == at::kLong && offset.numel() == 1, "dropout: offset int64[1]");
  auto y = at::empty_like(x);
  auto used = at::empty({1}, offset.options());
  dcp::launch_dropout(x.data_ptr(), y.data_ptr(), x.numel(), x.scalar_type() == at::kBFloat16, (float)p,
                      (uint64_t)seed, offset.data_ptr<int64_t>(), used.data_ptr<int64_t>(), cur_stream());
  offset.add_(1);
  return {y, used};
}

// the same mask (same seed and the forward's `used` offset) applied to the gradient
Tensor dropout_bwd(const Tensor& dy, double p, int64_t seed, const Tensor& used) {
  CHECK_DEV(dy);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat, "dropout: bf16 or fp32");
  TORCH_CHECK(used.scalar_type() == at::kLong && used.numel() == 1 && used.is_cuda(), "dropout: used int64[1]");
  auto g = dy.contiguous();
  auto dx = at::empty_like(g);
  dcp::launch_dropout(g.data_ptr(), dx.data_ptr(), g.numel(), g.scalar_type() == at::kBFloat16, (float)p,
                      (uint64_t)seed, used.data_ptr<int64_t>(), nullptr, cur_stream());
  return dx;
}

// adaptive average pool NHWC x [N,H,W,C] -> [N,OH,OW,C]
Tensor adaptive_avg_pool(const Tensor& x, int64_t OH, int64_t OW) {
  CHECK_ACT(x);
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0 && OH > 0 && OW > 0, "adaptive_avg_pool shapes");
  auto y = at::empty({x.size(0), OH, OW, x.size(3)}, x.options());
  dcp::launch_adaptive_avg(bp(x), bpm(y), x.size(0), x.size(1), x.size(2), x.size(3), OH, OW, false, cur_stream());
  return y;
}

Tensor adaptive_avg_pool_bwd(const Tensor& dy, int64_t H, int64_t W) {
  CHECK_ACT(dy);
  TORCH_CHECK(dy.dim() == 4 && dy.size(3) % 8 == 0 && H > 0 && W > 0, "adaptive_avg_pool_bwd shapes");
  auto dx = at::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  dcp::launch_adaptive_avg(bp(dy), bpm(dx), dy.size(0), H, W, dy.size(3), dy.size(1), dy.size(2), true, cur_stream());
  return dx;
}

// forward with an explicit output grid (asymmetric padding: output (oy, ox) reads input rows
// oy*stride + kh - pad, columns ox*stride + kw - pad; out-of-range taps read zeros)
std::tuple<Tensor, Tensor> conv_fwd_geo(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad, int64_t Ho,
                                        int64_t Wo, bool stats) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(3) == x.size(3), "conv_fwd_geo shapes");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0 && KH * KW <= dcp::kMaxTaps && pad >= 0 && pad < 64, "conv_fwd_geo geometry");
  TORCH_CHECK(Ho > 0 && Wo > 0 && (Ho - 1) * stride - pad < H && (Wo - 1) * stride - pad < W, "conv_fwd_geo grid");
  auto y = at::empty({N, Ho, Wo, Co}, bf16_like(x));
  const int M = N * Ho * Wo;
  Tensor slabs = stats ? at::empty({(M + 127) / 128, 2, Co}, f32_like(x)) : at::empty({0}, f32_like(x));
  const auto taps = fwd_taps(KH, KW, pad);
  dcp::launch_tap_gemm(bp(x), N, H, W, C, bp(w), Co, KH * KW, bpm(y), Ho, Wo, Ho, Wo, stride, 1, 0, 0, taps,
                       stats ? slabs.data_ptr<float>() : nullptr, nullptr, 0, zero_page(x.get_device()),
                       cur_stream());
  return {y, slabs};
}

// the space-to-depth ResNet stem: x [N,H,W,16], w [64,4,4,16] -> y [N,H,W,64] (4x4 / stride 1,
// pad 2 top/left, 1 bottom/right).  Statistics come as first-level BN partials [P,3,64]
// (n, mean, M2) from the dedicated kernel (stem.hip), or as conv slabs when the geometry
// falls back to the implicit GEMM; bn_stats / bn_stats_finalize accept either.
std::tuple<Tensor, Tensor> stem_fwd(const Tensor& x, const Tensor& w, bool stats) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(3) == x.size(3), "stem_fwd shapes");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  if (!dcp::stem_fwd_supported(H, W, C, w.size(0), w.size(1), w.size(2)))
    return conv_fwd_geo(x, w, 1, 2, H, W, stats);
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "stem_fwd: too many pixels");  // 64-bit row offsets
  auto y = at::empty({N, H, W, 64}, bf16_like(x));
  Tensor part = stats ? at::empty({dcp::stem_fwd_blocks(N, H), 3, 64}, f32_like(x)) : at::empty({0}, f32_like(x));
  dcp::launch_stem_fwd(bp(x), bp(w), bpm(y), stats ? part.data_ptr<float>() : nullptr, zero_page(x.get_device()), N,
                       H, W, cur_stream());
  return {y, part};
}

// Fused backward of the s2d stem conv + BN(+ReLU) + 3x3/2 max pool (stem.hip): from the pooled
// gradient, its argmax, the conv output z (BN input) and the stem input x16 -> (tot, sums):
// tot = the block-reduced [G1 (64 x 256), G2 (64 x 256), G3 (256), local sums] and sums [2,64] =
// (sum g', sum g' xhat).  stem_bwd_dw turns tot and the (all-reduced) sums into dW.
bool stem_bwd_fusable(const Tensor& z) {
  return z.dim() == 4 && dcp::stem_bwd_supported(z.size(1), z.size(2), z.size(3), z.size(1) / 2, z.size(2) / 2);
}

std::tuple<Tensor, Tensor> stem_bn_pool_bwd(const Tensor& dy, const Tensor& idx, const Tensor& z, const Tensor& x16,
                                            const Tensor& scale, const Tensor& shift, const Tensor& mean,
                                            const Tensor& invstd, int64_t act) {
  CHECK_ACT(dy);
  CHECK_ACT(z);
  CHECK_ACT(x16);
  const int N = z.size(0), H = z.size(1), W = z.size(2);
  TORCH_CHECK(stem_bwd_fusable(z) && x16.dim() == 4 && x16.size(0) == N && x16.size(1) == H && x16.size(2) == W &&
                  x16.size(3) == 16 && dy.size(1) == H / 2 && dy.size(2) == W / 2 && dy.size(3) == 64 &&
                  idx.numel() == dy.numel() && idx.scalar_type() == at::kByte,
              "stem_bn_pool_bwd shapes");
  // full-resolution rows are addressed with 64-bit offsets, the pooled tensors with 32-bit ones
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31) && (int64_t)N * (H / 2) * (W / 2) * 64 < (1ll << 32),
              "stem_bn_pool_bwd: tensor too large");
  const int nb = dcp::stem_bwd_blocks(N, H, num_cus(z.get_device()));
  const int pf = dcp::stem_bwd_part_floats();
  auto part = at::empty({(int64_t)(nb + (nb + 63) / 64) * pf}, f32_like(z));
  auto tot = at::empty({pf}, f32_like(z));
  auto sums = at::empty({2, 64}, f32_like(z));
  dcp::launch_stem_bwd(bp(z), bp(x16), bp(dy), idx.data_ptr<uint8_t>(), scale.data_ptr<float>(),
                       shift.data_ptr<float>(), mean.data_ptr<float>(), (int)act, N, H, W, nb, part.data_ptr<float>(),
                       cur_stream());
  dcp::launch_split_reduce(part.data_ptr<float>(), nb, pf, tot.data_ptr<float>(), cur_stream());
  dcp::launch_stem_bwd_sums(tot.data_ptr<float>(), invstd.data_ptr<float>(), sums.data_ptr<float>(), cur_stream());
  return {tot, sums};
}

Tensor stem_bwd_dw(const Tensor& tot, const Tensor& sums, const Tensor& scale, const Tensor& invstd, double count) {
  TORCH_CHECK(tot.numel() == dcp::stem_bwd_part_floats() && sums.numel() == 128, "stem_bwd_dw shapes");
  auto dw = at::empty({64, 4, 4, 16}, tot.options());
  dcp::launch_stem_bwd_dw(tot.data_ptr<float>(), sums.data_ptr<float>(), scale.data_ptr<float>(),
                          invstd.data_ptr<float>(), (float)(1.0 / count), dw.data_ptr<float>(), cur_stream());
  return dw;
}

// dy [N,Ho,Wo,Co], wt [C,KH,KW,Co] (transposed weight) -> dx [N,H,W,C]
Tensor conv_dgrad(const Tensor& dy, const Tensor& wt, int64_t H, int64_t W, int64_t stride, int64_t pad,
                  const optional<Tensor>& add) {
  CHECK_ACT(dy);
  CHECK_ACT(wt);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int C = wt.size(0), KH = wt.size(1), KW = wt.size(2);
  TORCH_CHECK(wt.size(3) == Co, "transposed weight Co mismatch");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "conv_dgrad needs channel multiples of 8");
  TORCH_CHECK(stride == 1 || stride == 2, "conv_dgrad supports stride 1 and 2");
  TORCH_CHECK((H + 2 * pad - KH) / stride + 1 == Ho && (W + 2 * pad - KW) / stride + 1 == Wo, "dgrad geometry");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31) && (int64_t)N * Ho * Wo < (1ll << 31), "conv_dgrad: too many pixels");
  auto dx = at::empty({N, H, W, C}, bf16_like(dy));
  const bf16* z = zero_page(dy.get_device());
  auto st = cur_stream();
  if (stride == 1 && pad == 1 && KH == 3 && KW == 3 && !add.has_value() && dcp::conv3x3_c64_supported(H, W, Co, C)) {
    // 64 -> 64 channel 3x3: the input gradient is the direct kernel's forward conv of dY with the
    // spatially flipped transposed weight, W'[c][kh][kw][co] = W[co][2-kh][2-kw][c] (conv3x3.hip:
    // one staged window per strip instead of nine tap gathers; ResNet-50 layer1 conv2 dgrad); the
    // kernel reads the taps of wt in reverse order (no flipped copy)
    const int blocks = dcp::conv3x3_c64_blocks(N, H, W, num_cus(dy.get_device()));
    dcp::launch_conv3x3_c64(bp(dy), bp(wt), bpm(dx), nullptr, z, N, H, W, blocks, st, nullptr, nullptr, 1);
    return dx;
  }
  if (stride == 1) {
    dcp::TapList t;
    t.n = KH * KW;
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw) {
        const int i = kh * KW + kw;
        t.dy[i] = pad - kh;
        t.dx[i] = pad - kw;
        t.widx[i] = i;
      }
    const bf16* addp = nullptr;
    if (add.has_value()) {
      CHECK_ACT(*add);
      TORCH_CHECK(add->sizes() == dx.sizes(), "conv_dgrad add shape");
      addp = bp(*add);
    }
    dcp::launch_tap_gemm(bp(dy), N, Ho, Wo, Co, bp(wt), C, KH * KW, bpm(dx), H, W, H, W, 1, 1, 0, 0, t, nullptr,
                         nullptr, 0, z, st, addp);
    return dx;
  }
  // stride 2: four parity classes of the input grid.  tg_parity_streams = 1: the classes run
  // concurrently on four pooled streams (fork / join through events; captured as parallel graph
  // branches), so one class's short-K tail overlaps the others (A/B)
  const bool par = dcp::g_tune[dcp::kDgradParityStreams] == 1;
  hipEvent_t fork_ev = nullptr;
  std::vector<hipStream_t> side;
  if (par) {
    fork_ev = parity_event(0);
    hipEventRecord(fork_ev, st);
  }
  int ncls = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      const int Hy = (H - ph + 1) / 2, Wy = (W - pw + 1) / 2;
      if (Hy <= 0 || Wy <= 0) continue;
      dcp::TapList t;
      t.n = 0;
      for (int kh = 0; kh < KH; ++kh) {
        if (((ph + pad - kh) % 2 + 2) % 2) continue;
        for (int kw = 0; kw < KW; ++kw) {
          if (((pw + pad - kw) % 2 + 2) % 2) continue;
          t.dy[t.n] = (ph + pad - kh) / 2;  // exact (even numerator)
          t.dx[t.n] = (pw + pad - kw) / 2;
          t.widx[t.n] = kh * KW + kw;
          ++t.n;
        }
      }
      hipStream_t cs = st;
      if (par) {
        cs = at::hip::getStreamFromPool(false, dy.get_device()).stream();
        hipStreamWaitEvent(cs, fork_ev, 0);
        side.push_back(cs);
      }
      dcp::launch_tap_gemm(bp(dy), N, Ho, Wo, Co, bp(wt), C, KH * KW, bpm(dx), H, W, Hy, Wy, 1, 2, ph, pw, t,
                           nullptr, nullptr, 0, z, cs);
      ++ncls;
    }
  for (size_t i = 0; i < side.size(); ++i) {  // join
    hipEvent_t e = parity_event(1 + (int)i);
    hipEventRecord(e, side[i]);
    hipStreamWaitEvent(st, e, 0);
  }
  if (add.has_value()) dx.add_(*add);
  return dx;
}

// Stride-1 dgrad fused with the backward reduction of the BN(+ReLU)(+residual) layer that
// produced this conv's input (y = that layer's BN input).  Returns the activation-masked
// input gradient g' [N,H,W,C] and the per-channel sums [2,C] = (sum g', sum g'*xhat).
std::tuple<Tensor, Tensor> conv_dgrad_bn(const Tensor& dy, const Tensor& wt, int64_t pad, const optional<Tensor>& add,
                                         const Tensor& y, const optional<Tensor>& res, const Tensor& scale,
                                         const Tensor& shift, const Tensor& mean, const Tensor& invstd, int64_t act,
                                         const optional<Tensor>& mask, double slope) {
  CHECK_ACT(dy);
  CHECK_ACT(wt);
  CHECK_ACT(y);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int C = wt.size(0), KH = wt.size(1), KW = wt.size(2);
  TORCH_CHECK(wt.size(3) == Co, "transposed weight Co mismatch");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "conv_dgrad_bn needs channel multiples of 8");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(3) == C, "conv_dgrad_bn: BN input shape");
  const int H = y.size(1), W = y.size(2);
  TORCH_CHECK(H + 2 * pad - KH + 1 == Ho && W + 2 * pad - KW + 1 == Wo, "conv_dgrad_bn: stride-1 geometry");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31), "conv_dgrad_bn: too many pixels");
  TORCH_CHECK(act == 0 || act == 1 || act == 2, "conv_dgrad_bn: act must be none, ReLU or leaky ReLU");
  TORCH_CHECK(act != 2 || (!mask.has_value() && !res.has_value()), "conv_dgrad_bn: leaky path has no mask / residual");
  for (const Tensor* t : {&scale, &shift, &mean, &invstd}) {
    CHECK_DEV(*t);
    CHECK_F32(*t);
    CHECK_CONTIG(*t);
    TORCH_CHECK(t->numel() == C, "conv_dgrad_bn: per-channel vector size");
  }
  auto dx = at::empty({N, H, W, C}, bf16_like(dy));
  const bf16* addp = nullptr;
  int add_s2 = 0, add_hc = 0, add_wc = 0;
  if (add.has_value()) {
    CHECK_ACT(*add);
    if (add->sizes() != dx.sizes()) {
      // a compact stride-2 gradient: the even (y, x) pixels of dx only (StridedGrad)
      add_hc = (H + 1) / 2;
      add_wc = (W + 1) / 2;
      TORCH_CHECK(add->dim() == 4 && add->size(0) == N && add->size(1) == add_hc && add->size(2) == add_wc &&
                      add->size(3) == C,
                  "conv_dgrad_bn add shape: [N,H,W,C] or the stride-2 subgrid [N,ceil(H/2),ceil(W/2),C]");
      add_s2 = 1;
    }
    addp = bp(*add);
  }
  const bf16* resp = nullptr;
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == dx.sizes(), "conv_dgrad_bn residual shape");
    resp = bp(*res);
  }
  const uint8_t* maskp = nullptr;
  if (mask.has_value()) {
    CHECK_DEV(*mask);
    CHECK_CONTIG(*mask);
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 == dx.numel(),
                "conv_dgrad_bn: mask must be uint8 [N,H,W,C/8]");
    maskp = mask->data_ptr<uint8_t>();
  }
  const int M = N * H * W;
  const int ntm = (M + 127) / 128;
  // per-tile partials + room for the chunk sums of the two-level deterministic reduce
  auto part = at::empty({(int64_t)(ntm + (ntm + 63) / 64) * 2 * C}, f32_like(dy));
  auto sums = at::empty({2, C}, f32_like(dy));
  dcp::TapList t;
  t.n = KH * KW;
  TORCH_CHECK(t.n <= dcp::kMaxTaps, "kernel too large");
  for (int kh = 0; kh < KH; ++kh)
    for (int kw = 0; kw < KW; ++kw) {
      const int i = kh * KW + kw;
      t.dy[i] = pad - kh;
      t.dx[i] = pad - kw;
      t.widx[i] = i;
    }
  dcp::BnBwdEpi e{bp(y), resp, scale.data_ptr<float>(), shift.data_ptr<float>(), mean.data_ptr<float>(),
                  invstd.data_ptr<float>(), part.data_ptr<float>(), (int)act, maskp, (float)slope, add_s2, add_hc,
                  add_wc};
  auto st = cur_stream();
  dcp::launch_tap_gemm(bp(dy), N, Ho, Wo, Co, bp(wt), C, KH * KW, bpm(dx), H, W, H, W, 1, 1, 0, 0, t, nullptr, nullptr,
                       0, zero_page(dy.get_device()), st, addp, &e);
  dcp::launch_split_reduce(part.data_ptr<float>(), ntm, 2 * C, sums.data_ptr<float>(), st);
  return {dx, sums};
}

// Weight-gradient configurations the autotuner (g_tune[kAutotune] = 1, DCP_AUTOTUNE) times per problem,
// as g_tune overrides: [5] workgroups per CU of the split-K plan, [7] = 2 no 256-tile kernel,
// [12] = 32 32-row k-tiles, [15] = 1 no direct 3x3 kernel, [27] = 64 at most 64 splits (one reduce
// launch instead of two: pays at small batches, where the launches dominate).  The split count changes the partial
// slabs, so the choice is made here, where they are allocated (see launch_tap_gemm for the
// forward / data-gradient side).  Every configuration reduces the split partials in a fixed
// order, but a different split count sums the rows in another order (fp32 rounding).
namespace {
struct WgCfg {
  int t5, t7, t12, t15, t27;
};
const WgCfg kWgCfgs[] = {{0, 0, 0, 0, 0}, {1, 0, 0, 0, 0}, {2, 0, 0, 0, 0},  {4, 0, 0, 0, 0},
                         {8, 0, 0, 0, 0}, {0, 2, 0, 0, 0}, {0, 0, 32, 0, 0}, {0, 0, 0, 1, 0},
                         {0, 0, 0, 0, 64}, {0, 2, 0, 0, 64}, {0, 0, 0, 1, 64}};
std::mutex g_wg_mu;
std::unordered_map<std::string, int> g_wg_choice;
struct WgOverride {
  int saved[5];
  explicit WgOverride(const WgCfg& c) {
    saved[0] = dcp::g_tune[dcp::kWgSplitsPerCu]; saved[1] = dcp::g_tune[dcp::kWgTileMode]; saved[2] = dcp::g_tune[dcp::kWgRows]; saved[3] = dcp::g_tune[dcp::kWg3x3];
    saved[4] = dcp::g_tune[dcp::kWgSplitCap];
    dcp::g_tune[dcp::kWgSplitsPerCu] = c.t5; dcp::g_tune[dcp::kWgTileMode] = c.t7; dcp::g_tune[dcp::kWgRows] = c.t12; dcp::g_tune[dcp::kWg3x3] = c.t15;
    dcp::g_tune[dcp::kWgSplitCap] = c.t27;
  }
  ~WgOverride() {
    dcp::g_tune[dcp::kWgSplitsPerCu] = saved[0]; dcp::g_tune[dcp::kWgTileMode] = saved[1]; dcp::g_tune[dcp::kWgRows] = saved[2]; dcp::g_tune[dcp::kWg3x3] = saved[3];
    dcp::g_tune[dcp::kWgSplitCap] = saved[4];
  }
};
}  // namespace

int64_t wgrad_autotune_entries() {
  std::lock_guard<std::mutex> lk(g_wg_mu);
  return (int64_t)g_wg_choice.size();
}

// dy [N,Ho,Wo,Co], x [N,H,W,C] -> dw fp32 [Co,KH,KW,C]
Tensor conv_wgrad(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(x.size(0) == N, "batch mismatch");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "conv_wgrad needs channel multiples of 8");
  TORCH_CHECK((H + 2 * pad - KH) / stride + 1 == Ho && (W + 2 * pad - KW) / stride + 1 == Wo, "wgrad geometry");
  TORCH_CHECK((int64_t)N * H * W < (1ll << 31) && (int64_t)N * Ho * Wo < (1ll << 31), "conv_wgrad: too many pixels");
  auto dw = at::empty({Co, KH, KW, C}, f32_like(dy));
  const auto taps = fwd_taps(KH, KW, pad);
  const int ncu = num_cus(dy.get_device());
  auto st = cur_stream();
  auto run = [&]() {
    const int splits = dcp::wgrad_plan_splits(N, Ho, Wo, Co, H, W, C, stride, taps, ncu);
    auto part = at::empty({splits > 1 ? (int64_t)(splits + (splits + 63) / 64) * dw.numel() : 4}, f32_like(dy));
    dcp::launch_wgrad(bp(dy), N, Ho, Wo, Co, bp(x), H, W, C, stride, taps, dw.data_ptr<float>(),
                      part.data_ptr<float>(), zero_page(dy.get_device()), ncu, st);
  };
  if (dcp::g_tune[dcp::kAutotune] != 1 || dcp::g_tune[dcp::kWgSplitsPerCu] || dcp::g_tune[dcp::kWgTileMode] || dcp::g_tune[dcp::kWgRows] || dcp::g_tune[dcp::kWg3x3] ||
      dcp::g_tune[dcp::kWgSplitCap] || (int64_t)N * Ho * Wo == 0) {
    run();
    return dw;
  }
  const std::string key = std::to_string(N) + " " + std::to_string(Ho) + " " + std::to_string(Wo) + " " +
                          std::to_string(Co) + " " + std::to_string(H) + " " + std::to_string(W) + " " +
                          std::to_string(C) + " " + std::to_string(KH) + " " + std::to_string(KW) + " " +
                          std::to_string(stride) + " " + std::to_string(pad);
  int choice = -1;
  {
    std::lock_guard<std::mutex> lk(g_wg_mu);
    auto it = g_wg_choice.find(key);
    if (it != g_wg_choice.end()) choice = it->second;
  }
  if (choice < 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      run();
      return dw;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f, t_heur = 1e30f;
    choice = 0;
    for (int c = 0; c < (int)(sizeof(kWgCfgs) / sizeof(kWgCfgs[0])); ++c) {
      WgOverride ov(kWgCfgs[c]);
      run();  // warm
      float t = 1e30f;
      for (int r = 0; r < 3; ++r) {
        hipEventRecord(e0, st);
        run();
        hipEventRecord(e1, st);
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
      std::lock_guard<std::mutex> lk(g_wg_mu);
      g_wg_choice[key] = choice;
    }
    if (getenv("DCP_AUTOTUNE_LOG"))
      fprintf(stderr, "[dcp-autotune] wgrad %s -> cfg %d (%.1f us)\n", key.c_str(), choice, best * 1e3f);
  }
  WgOverride ov(kWgCfgs[choice]);
  run();
  return dw;
}

// weight gradient for conv_fwd_geo's geometry (output grid taken from dy)
Tensor conv_wgrad_geo(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(x.size(0) == N && C % 8 == 0 && Co % 8 == 0 && KH * KW <= dcp::kMaxTaps, "conv_wgrad_geo shapes");
  TORCH_CHECK(pad >= 0 && pad < 64 && (Ho - 1) * stride - pad < H && (Wo - 1) * stride - pad < W,
              "conv_wgrad_geo grid");
  auto dw = at::empty({Co, KH, KW, C}, f32_like(dy));
  const auto taps = fwd_taps(KH, KW, pad);
  const int ncu = num_cus(dy.get_device());
  const int splits = dcp::wgrad_plan_splits(N, Ho, Wo, Co, H, W, C, stride, taps, ncu);
  auto part = at::empty({splits > 1 ? (int64_t)(splits + (splits + 63) / 64) * dw.numel() : 4}, f32_like(dy));
  dcp::launch_wgrad(bp(dy), N, Ho, Wo, Co, bp(x), H, W, C, stride, taps, dw.data_ptr<float>(),
                    part.data_ptr<float>(), zero_page(dy.get_device()), ncu, cur_stream());
  return dw;
}

// x [B,K] bf16, w [Npad,K] bf16 -> y [B,Npad] (= act(x w^T + b)); act 0 none, 1 ReLU, 2 sigmoid
Tensor linear_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int64_t act) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "linear shapes");
  const int B = x.size(0), K = x.size(1), Np = w.size(0);
  TORCH_CHECK(K % 8 == 0 && Np % 8 == 0, "linear needs K and N multiples of 8");
  if (bias.has_value()) {
    CHECK_F32(*bias);
    CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() >= 1 && bias->numel() <= Np, "bias longer than the output width");
  }
  auto y = at::empty({B, Np}, bf16_like(x));
  dcp::TapList t;
  t.n = 1;
  t.dy[0] = t.dx[0] = t.widx[0] = 0;
  TORCH_CHECK(act >= 0 && act <= 2, "linear act must be 0 (none), 1 (relu) or 2 (sigmoid)");
  // an unpadded bias (the output width rounded up for the GEMM): columns past it add 0
  dcp::launch_tap_gemm(bp(x), B, 1, 1, K, bp(w), Np, 1, bpm(y), 1, 1, 1, 1, 1, 1, 0, 0, t, nullptr, fp(bias),
                       (int)act, zero_page(x.get_device()), cur_stream(), nullptr, nullptr, nullptr, nullptr,
                       nullptr, bias.has_value() ? (int)bias->numel() : 0);
  return y;
}

// dy [B,N] bf16, x [B,K] bf16 -> dw fp32 [N,K]
Tensor linear_wgrad(const Tensor& dy, const Tensor& x) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int B = dy.size(0), Np = dy.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == B && K % 8 == 0 && Np % 8 == 0, "linear_wgrad shapes");
  auto dw = at::empty({Np, K}, f32_like(dy));
  dcp::TapList t;
  t.n = 1;
  t.dy[0] = t.dx[0] = t.widx[0] = 0;
  const int ncu = num_cus(dy.get_device());
  const int splits = dcp::wgrad_splits(B, Np, K, 1, ncu, nullptr);
  auto part = at::empty({splits > 1 ? (int64_t)(splits + (splits + 63) / 64) * dw.numel() : 4}, f32_like(dy));
  dcp::launch_wgrad(bp(dy), B, 1, 1, Np, bp(x), 1, 1, K, 1, t, dw.data_ptr<float>(), part.data_ptr<float>(),
                    zero_page(dy.get_device()), ncu, cur_stream());
  return dw;
}

// fp32 master [Co,KH,KW,Ci] -> bf16 [Co_pad,KH,KW,Ci] (+ transposed [Ci,KH,KW,Co_pad])
std::tuple<Tensor, Tensor> weight_prep(const Tensor& w, int64_t co_pad, bool transposed) {
  CHECK_DEV(w);
  CHECK_CONTIG(w);
  CHECK_F32(w);
  TORCH_CHECK(w.dim() == 4 || w.dim() == 2, "weight_prep expects 4-D or 2-D weights");
  const int Co = w.size(0);
  const int T = w.dim() == 4 ? w.size(1) * w.size(2) : 1;
  const int Ci = w.dim() == 4 ? w.size(3) : w.size(1);
  const int Cp = co_pad > Co ? co_pad : Co;
  std::vector<int64_t> shp = w.sizes().vec();
  shp[0] = Cp;
  auto wb = at::empty(shp, bf16_like(w));
  Tensor wt;
  if (transposed) {
    std::vector<int64_t> ts = w.sizes().vec();
    ts[0] = Ci;
    ts[ts.size() - 1] = Cp;
    wt = at::empty(ts, bf16_like(w));
  } else {
    wt = at::empty({0}, bf16_like(w));
  }
  dcp::launch_weight_prep(w.data_ptr<float>(), Co, T, Ci, Cp, bpm(wb), transposed ? bpm(wt) : nullptr, cur_stream());
  return {wb, wt};
}

Tensor grouped_conv_fwd(const Tensor& x, const Tensor& w, int64_t groups, int64_t stride, int64_t pad) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(C % groups == 0 && Co % groups == 0 && w.size(3) == C / groups, "grouped conv shapes");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "grouped conv channel multiples of 8");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  auto y = at::empty({N, Ho, Wo, Co}, bf16_like(x));
  auto frag = at::empty({std::max(dcp::gconv_frag_elems(C, groups, KH, KW), 8)}, bf16_like(x));
  dcp::launch_grouped_conv_fwd(bp(x), bp(w), bpm(y), bpm(frag), N, H, W, C, Ho, Wo, Co, groups, KH, KW, stride, pad,
                               cur_stream());
  return y;
}

// grouped conv forward + the output's BN partials [P][3][Co] (n, mean, M2) from the MFMA epilogue
// (an empty tensor when the shape runs the direct fallback kernel)
std::tuple<Tensor, Tensor> grouped_conv_fwd_stats(const Tensor& x, const Tensor& w, int64_t groups, int64_t stride,
                                                  int64_t pad) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(C % groups == 0 && Co % groups == 0 && w.size(3) == C / groups, "grouped conv shapes");
  TORCH_CHECK(C % 8 == 0 && Co % 8 == 0, "grouped conv channel multiples of 8");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  auto y = at::empty({N, Ho, Wo, Co}, bf16_like(x));
  auto frag = at::empty({std::max(dcp::gconv_frag_elems(C, groups, KH, KW), 8)}, bf16_like(x));
  auto part = at::empty({dcp::gconv_fwd_stat_blocks(N * Ho * Wo), 3, Co}, f32_like(x));
  const bool ok = dcp::launch_grouped_conv_fwd(bp(x), bp(w), bpm(y), bpm(frag), N, H, W, C, Ho, Wo, Co, groups, KH, KW,
                                               stride, pad, cur_stream(), part.data_ptr<float>());
  return {y, ok ? part : at::empty({0}, f32_like(x))};
}

Tensor grouped_conv_dgrad(const Tensor& dy, const Tensor& w, int64_t H, int64_t W, int64_t groups, int64_t stride,
                          int64_t pad) {
  CHECK_ACT(dy);
  CHECK_ACT(w);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int KH = w.size(1), KW = w.size(2), C = w.size(3) * groups;
  auto dx = at::empty({N, H, W, C}, bf16_like(dy));
  auto frag = at::empty({std::max(dcp::gconv_frag_elems(C, groups, KH, KW), 8)}, bf16_like(dy));
  dcp::launch_grouped_conv_dgrad(bp(dy), bp(w), bpm(dx), bpm(frag), N, H, W, C, Ho, Wo, Co, groups, KH, KW, stride, pad,
                                 cur_stream());
  return dx;
}

// grouped dgrad fused with the backward reduction of the ReLU BN that produced the conv input z:
// -> (g = dx * [z*scale + shift > 0], sums [2][C] = (sum g, sum g * (z - mean) * invstd)); an
// empty `sums` means the shape runs the unfused kernels (the caller reduces separately)
std::tuple<Tensor, Tensor> grouped_conv_dgrad_bn(const Tensor& dy, const Tensor& w, int64_t H, int64_t W,
                                                 int64_t groups, int64_t stride, int64_t pad, const Tensor& z,
                                                 const Tensor& scale, const Tensor& shift, const Tensor& mean,
                                                 const Tensor& invstd) {
  CHECK_ACT(dy);
  CHECK_ACT(w);
  CHECK_ACT(z);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int KH = w.size(1), KW = w.size(2), C = w.size(3) * groups;
  TORCH_CHECK(z.dim() == 4 && z.size(0) == N && z.size(1) == H && z.size(2) == W && z.size(3) == C,
              "grouped_conv_dgrad_bn: z must be the conv input [N,H,W,C]");
  for (const Tensor* t : {&scale, &shift, &mean, &invstd})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(),
                "grouped_conv_dgrad_bn: per-channel fp32 [C] coefficients");
  auto dx = at::empty({N, H, W, C}, bf16_like(dy));
  auto frag = at::empty({std::max(dcp::gconv_frag_elems(C, groups, KH, KW), 8)}, bf16_like(dy));
  const int npb = dcp::gconv_fwd_stat_blocks(N * H * W);
  auto part = at::empty({(int64_t)npb * 2 * C + ((npb + 63) / 64) * 2 * C}, f32_like(dy));
  dcp::GconvBnBwd bn{bp(z), scale.data_ptr<float>(), shift.data_ptr<float>(), mean.data_ptr<float>(),
                     invstd.data_ptr<float>(), part.data_ptr<float>()};
  if (!dcp::launch_gconv_mfma_dgrad(bp(dy), bp(w), bpm(dx), bpm(frag), N, H, W, C, Ho, Wo, Co, groups, KH, KW, stride,
                                    pad, cur_stream(), &bn)) {
    dcp::launch_grouped_conv_dgrad(bp(dy), bp(w), bpm(dx), bpm(frag), N, H, W, C, Ho, Wo, Co, groups, KH, KW, stride,
                                   pad, cur_stream());
    return {dx, at::empty({0}, f32_like(dy))};
  }
  auto sums = at::empty({2, C}, f32_like(dy));
  dcp::launch_split_reduce(part.data_ptr<float>(), npb, 2 * C, sums.data_ptr<float>(), cur_stream());
  return {dx, sums};
}

Tensor grouped_conv_wgrad(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t groups, int64_t stride,
                          int64_t pad) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  const int H = x.size(1), W = x.size(2), C = x.size(3);
  auto dw = at::empty({Co, KH, KW, C / groups}, f32_like(dy));
  const int splits = Co == C ? dcp::gconv_mfma_wgrad_splits(N, Ho, Wo, C, groups) : 0;
  const int fsplits = dcp::gconv_fallback_wgrad_splits(N * Ho * Wo, (int)dw.numel());
  auto part = at::empty({std::max({splits, fsplits, 1}) * (int64_t)dw.numel()}, f32_like(dy));
  dcp::launch_grouped_conv_wgrad(bp(dy), bp(x), dw.data_ptr<float>(), part.data_ptr<float>(), splits,
                                 zero_page(dy.get_device()), N, H, W, C, Ho,
                                 Wo, Co, groups, KH, KW, stride, pad, cur_stream());
  return dw;
}

// ---------------------------------------------------------------------------
// batch norm
// ---------------------------------------------------------------------------
// statistics given as first-level partials [P,3,C] (n, mean, M2) instead of conv slabs [R,2,C]
bool is_partials(const Tensor& t, int C) {
  return t.dim() == 3 && t.size(1) == 3 && t.size(2) == C && t.scalar_type() == at::kFloat;
}

// many (n, mean, M2) partials (e.g. one per stem workgroup): merged first in chunks of 128 rows
// (bn_partial_chunk_kernel), so the final merge is short; few: returned as they are
Tensor chunk_partials(const Tensor& part, int C) {
  const int P = part.size(0);
  const int chunks = dcp::bn_partial_chunks(P);
  if (chunks == 0) return part;
  auto tmp = at::empty({chunks, 3, C}, part.options());
  dcp::launch_bn_partial_chunk(part.data_ptr<float>(), P, C, tmp.data_ptr<float>(), cur_stream());
  return tmp;
}

// per-channel (n, mean, M2) [1,3,C] from conv slabs or partials (if given) or directly from x
Tensor bn_stats(const Tensor& x, const optional<Tensor>& slabs) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn channels must be a multiple of 8 and <= 2048");
  const bool from_slabs = slabs.has_value() && slabs->numel() > 0;
  auto out = at::empty({1, 3, C}, f32_like(x));
  if (from_slabs && is_partials(*slabs, C)) {
    const Tensor pr = chunk_partials(*slabs, C);
    dcp::launch_bn_merge(pr.data_ptr<float>(), pr.size(0), C, out.data_ptr<float>(), cur_stream());
    return out;
  }
  if (from_slabs)
    TORCH_CHECK(slabs->dim() == 3 && slabs->size(0) == (M + 127) / 128 && slabs->size(1) == 2 && slabs->size(2) == C,
                "slab shape");
  auto part = at::empty({dcp::bn_stats_partials(M, C, from_slabs), 3, C}, f32_like(x));
  dcp::launch_bn_stats(bp(x), from_slabs ? slabs->data_ptr<float>() : nullptr, M, C, part.data_ptr<float>(),
                       out.data_ptr<float>(), cur_stream());
  return out;
}

// local (single-rank) BN: statistics + finalize without the [1,3,C] round trip -> (mean, invstd,
// scale, shift); running stats updated in place.  Same numbers as bn_finalize(bn_stats(x)).
// iabn_eps >= 0: InplaceABN's effective weight |gamma| + iabn_eps, its reciprocal written to rgamma_out
std::tuple<Tensor, Tensor, Tensor, Tensor> bn_stats_finalize(const Tensor& x, const optional<Tensor>& slabs,
                                                             const optional<Tensor>& gamma,
                                                             const optional<Tensor>& beta,
                                                             const optional<Tensor>& run_mean,
                                                             const optional<Tensor>& run_var, double momentum,
                                                             double eps, double iabn_eps,
                                                             const optional<Tensor>& rgamma_out) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn channels must be a multiple of 8 and <= 2048");
  const bool from_slabs = slabs.has_value() && slabs->numel() > 0;
  auto coef = at::empty({4, C}, f32_like(x));
  float* cp = coef.data_ptr<float>();
  if (from_slabs && is_partials(*slabs, C)) {
    const Tensor pr = chunk_partials(*slabs, C);
    dcp::launch_bn_merge_finalize(pr.data_ptr<float>(), pr.size(0), C, (float)eps, fp(gamma), fp(beta), cp,
                                  cp + C, cp + 2 * C, cp + 3 * C, fpm(run_mean), fpm(run_var), (float)momentum,
                                  cur_stream(), (float)iabn_eps, fpm(rgamma_out));
    return {coef[0], coef[1], coef[2], coef[3]};
  }
  if (from_slabs)
    TORCH_CHECK(slabs->dim() == 3 && slabs->size(0) == (M + 127) / 128 && slabs->size(1) == 2 && slabs->size(2) == C,
                "slab shape");
  auto part = at::empty({dcp::bn_stats_partials(M, C, from_slabs), 3, C}, f32_like(x));
  dcp::launch_bn_stats_finalize(bp(x), from_slabs ? slabs->data_ptr<float>() : nullptr, M, C, part.data_ptr<float>(),
                                (float)eps, fp(gamma), fp(beta), cp, cp + C, cp + 2 * C, cp + 3 * C, fpm(run_mean),
                                fpm(run_var), (float)momentum, cur_stream(), (float)iabn_eps, fpm(rgamma_out));
  return {coef[0], coef[1], coef[2], coef[3]};
}

// per-device counters of bn_fin_act_kernel: zeroed once (outside any capture), re-armed by every
// launch; all BN launches of a device run on one stream at a time, so one triple serves them all
static uint32_t* fin_act_sync(int dev, hipStream_t st) {
  static std::mutex mu;
  static std::unordered_map<int, uint32_t*> bufs;
  std::lock_guard<std::mutex> lk(mu);
  auto it = bufs.find(dev);
  if (it != bufs.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  uint32_t* p = nullptr;
  if (hipMalloc(&p, 64) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
  bufs[dev] = p;
  return p;
}

// spin timeouts of bn_fin_act_kernel on this device so far (0 = every launch saw its finalize)
int64_t bn_fin_act_timeouts(const Tensor& like) {
  uint32_t* p = fin_act_sync(like.get_device(), cur_stream());
  if (p == nullptr) return 0;
  uint32_t v = 0;
  TORCH_CHECK(hipStreamSynchronize(cur_stream()) == hipSuccess && hipMemcpy(&v, p + 2, 4, hipMemcpyDeviceToHost) == hipSuccess,
              "bn_fin_act_timeouts: copy");
  return v;
}

// local training BN from conv slabs / partials: finalize + BN + act (+ residual) (+ act' mask bits) in
// ONE launch -> (y, mask or an empty tensor, mean, invstd, scale, shift); running stats updated in
// place.  Bit-identical to bn_stats_finalize followed by bn_act / bn_act_mask (the two-launch path it
// falls back to for deep slab stacks, during a first capture, or with g_tune bn_fin_act = 2).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> bn_fin_act(
    const Tensor& x, const Tensor& slabs, const optional<Tensor>& res, const optional<Tensor>& gamma,
    const optional<Tensor>& beta, const optional<Tensor>& run_mean, const optional<Tensor>& run_var, double momentum,
    double eps, int64_t act, double slope, bool want_mask, double iabn_eps, const optional<Tensor>& rgamma_out) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn channels must be a multiple of 8 and <= 2048");
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
  }
  const bool have = slabs.numel() > 0;  // empty: statistics from x itself (two-launch path)
  const bool part = have && is_partials(slabs, C);
  if (have && !part)
    TORCH_CHECK(slabs.dim() == 3 && slabs.size(0) == (M + 127) / 128 && slabs.size(1) == 2 && slabs.size(2) == C,
                "slab shape");
  auto y = at::empty_like(x);
  Tensor mask;
  if (want_mask) {
    std::vector<int64_t> ms = x.sizes().vec();
    ms.back() = C / 8;
    mask = at::empty(ms, x.options().dtype(at::kByte));
  } else {
    mask = at::empty({0}, x.options().dtype(at::kByte));
  }
  auto st = cur_stream();
  uint32_t* sync = dcp::g_tune[dcp::kBnFinAct] == 2 ? nullptr : fin_act_sync(x.get_device(), st);
  const bool fused = sync != nullptr && have && (part || (int)slabs.size(0) <= dcp::bn_direct_slabs());
  if (!fused) {
    auto [mean, invstd, scale, shift] = bn_stats_finalize(x, have ? optional<Tensor>(slabs) : optional<Tensor>(),
                                                          gamma, beta, run_mean, run_var, momentum, eps, iabn_eps,
                                                          rgamma_out);
    dcp::launch_bn_act_fwd(bp(x), res.has_value() ? bp(*res) : nullptr, scale.data_ptr<float>(),
                           shift.data_ptr<float>(), bpm(y), x.numel(), C, (int)act, (float)slope, st,
                           want_mask ? mask.data_ptr<uint8_t>() : nullptr);
    return {y, mask, mean, invstd, scale, shift};
  }
  auto coef = at::empty({4, C}, f32_like(x));
  float* cp = coef.data_ptr<float>();
  const Tensor src = part ? chunk_partials(slabs, C) : slabs;
  dcp::launch_bn_fin_act(bp(x), res.has_value() ? bp(*res) : nullptr, src.data_ptr<float>(), (int)src.size(0),
                         part ? 1 : 0, M, C, (float)eps, fp(gamma), fp(beta), cp, cp + C, cp + 2 * C, cp + 3 * C,
                         fpm(run_mean), fpm(run_var), (float)momentum, (float)iabn_eps, fpm(rgamma_out), bpm(y),
                         want_mask ? mask.data_ptr<uint8_t>() : nullptr, (int)act, (float)slope, sync, st);
  return {y, mask, coef[0], coef[1], coef[2], coef[3]};
}

// stem weight: 7x7 master [Co,7,7,C<=4] fp32 -> its s2d form written into w16 [Co,4,4,16] (in place)
void s2d_weight(const Tensor& w7, const Tensor& w16) {
  CHECK_DEV(w7);
  CHECK_F32(w7);
  CHECK_CONTIG(w7);
  CHECK_DEV(w16);
  CHECK_F32(w16);
  CHECK_CONTIG(w16);
  TORCH_CHECK(w7.dim() == 4 && w7.size(1) == 7 && w7.size(2) == 7 && w7.size(3) <= 4 && w16.dim() == 4 &&
                  w16.size(0) == w7.size(0) && w16.size(1) == 4 && w16.size(2) == 4 && w16.size(3) == 16,
              "s2d_weight shapes");
  dcp::launch_s2d_weight(w7.data_ptr<float>(), w7.size(0), w7.size(3), w16.data_ptr<float>(), cur_stream());
}

// gradient of the s2d form [Co,4,4,16] -> gradient of the 7x7 master [Co,7,7,C]
Tensor s2d_weight_bwd(const Tensor& g16, int64_t C) {
  CHECK_DEV(g16);
  CHECK_F32(g16);
  CHECK_CONTIG(g16);
  TORCH_CHECK(g16.dim() == 4 && g16.size(1) == 4 && g16.size(2) == 4 && g16.size(3) == 16 && C >= 1 && C <= 4,
              "s2d_weight_bwd shapes");
  auto g7 = at::empty({g16.size(0), 7, 7, C}, g16.options());
  dcp::launch_s2d_weight_bwd(g16.data_ptr<float>(), g16.size(0), (int)C, g7.data_ptr<float>(), cur_stream());
  return g7;
}

Tensor colsum(const Tensor& x) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0, "colsum channels");
  const int M = x.numel() / C;
  auto part = at::empty({dcp::colsum_partials(M), C}, f32_like(x));
  auto out = at::empty({C}, f32_like(x));
  dcp::launch_colsum(bp(x), M, C, part.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

// stats [W,3,C] (n, mean, M2 per rank) -> (mean, invstd, scale, shift); updates running stats in place
std::tuple<Tensor, Tensor, Tensor, Tensor> bn_finalize(const Tensor& st, const optional<Tensor>& gamma,
                                                       const optional<Tensor>& beta,
                                                       const optional<Tensor>& run_mean,
                                                       const optional<Tensor>& run_var, double momentum,
                                                       double eps, double iabn_eps,
                                                       const optional<Tensor>& rgamma_out) {
  CHECK_DEV(st);
  CHECK_F32(st);
  CHECK_CONTIG(st);
  TORCH_CHECK(st.dim() == 3 && st.size(1) == 3, "stats must be [W,3,C]");
  const int W = st.size(0), C = st.size(2);
  auto mean = at::empty({C}, st.options()), invstd = at::empty({C}, st.options());
  auto scale = at::empty({C}, st.options()), shift = at::empty({C}, st.options());
  dcp::launch_bn_finalize(st.data_ptr<float>(), W, C, (float)eps, fp(gamma), fp(beta), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(), fpm(run_mean),
                          fpm(run_var), (float)momentum, cur_stream(), (float)iabn_eps, fpm(rgamma_out));
  return {mean, invstd, scale, shift};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> bn_eval_coeff(const optional<Tensor>& gamma, const optional<Tensor>& beta,
                                                         const Tensor& run_mean, const Tensor& run_var, double eps) {
  CHECK_DEV(run_mean);
  const int C = run_mean.numel();
  auto mean = at::empty({C}, run_mean.options()), invstd = at::empty({C}, run_mean.options());
  auto scale = at::empty({C}, run_mean.options()), shift = at::empty({C}, run_mean.options());
  dcp::launch_bn_eval_coeff(C, (float)eps, fp(gamma), fp(beta), run_mean.data_ptr<float>(),
                            run_var.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                            scale.data_ptr<float>(), shift.data_ptr<float>(), cur_stream());
  return {mean, invstd, scale, shift};
}

Tensor bn_act(const Tensor& x, const optional<Tensor>& res, const Tensor& scale, const Tensor& shift, int64_t act,
              double slope) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && scale.numel() == C, "bn_act shapes (C % 8 == 0, C <= 2048)");
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
  }
  auto y = at::empty_like(x);
  dcp::launch_bn_act_fwd(bp(x), res.has_value() ? bp(*res) : nullptr, scale.data_ptr<float>(),
                         shift.data_ptr<float>(), bpm(y), x.numel(), C, act, (float)slope, cur_stream());
  return y;
}

// bn_act plus the activation mask act'(z) > 0 as bits: uint8 [..., C/8], bit e of byte c = channel 8c+e
std::tuple<Tensor, Tensor> bn_act_mask(const Tensor& x, const optional<Tensor>& res, const Tensor& scale,
                                       const Tensor& shift, int64_t act, double slope) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && scale.numel() == C, "bn_act_mask shapes (C % 8 == 0, C <= 2048)");
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
  }
  auto y = at::empty_like(x);
  std::vector<int64_t> ms = x.sizes().vec();
  ms.back() = C / 8;
  auto mask = at::empty(ms, x.options().dtype(at::kByte));
  dcp::launch_bn_act_fwd(bp(x), res.has_value() ? bp(*res) : nullptr, scale.data_ptr<float>(),
                         shift.data_ptr<float>(), bpm(y), x.numel(), C, act, (float)slope, cur_stream(),
                         mask.data_ptr<uint8_t>());
  return {y, mask};
}

// BN + act over x with a residual that is itself a raw BN input normalised on the fly
// (projection shortcut: y = act(x*scale + shift + res*rscale + rshift)) plus the act' mask bits.
std::tuple<Tensor, Tensor> bn2_act_mask(const Tensor& x, const Tensor& res, const Tensor& scale, const Tensor& shift,
                                        const Tensor& rscale, const Tensor& rshift, int64_t act, double slope) {
  CHECK_ACT(x);
  CHECK_ACT(res);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && scale.numel() == C && shift.numel() == C && rscale.numel() == C &&
                  rshift.numel() == C && res.sizes() == x.sizes(),
              "bn2_act_mask shapes (C % 8 == 0, C <= 2048, residual like x)");
  CHECK_F32(rscale);
  CHECK_F32(rshift);
  auto y = at::empty_like(x);
  std::vector<int64_t> ms = x.sizes().vec();
  ms.back() = C / 8;
  auto mask = at::empty(ms, x.options().dtype(at::kByte));
  dcp::launch_bn_act_fwd(bp(x), bp(res), scale.data_ptr<float>(), shift.data_ptr<float>(), bpm(y), x.numel(), C, act,
                         (float)slope, cur_stream(), mask.data_ptr<uint8_t>(), rscale.data_ptr<float>(),
                         rshift.data_ptr<float>());
  return {y, mask};
}

Tensor bn_bwd_reduce(const Tensor& dy, const Tensor& x, const optional<Tensor>& res, const Tensor& scale,
                     const Tensor& shift, const Tensor& mean, const Tensor& invstd, int64_t act, double slope,
                     bool inv) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int C = x.size(-1);
  TORCH_CHECK(!inv || ((act == 0 || act == 2) && !res.has_value()), "bn_bwd_reduce: inv needs an invertible act");
  TORCH_CHECK(dy.sizes() == x.sizes() && C % 8 == 0 && C <= 2048, "bn_bwd_reduce shapes");
  if (res.has_value()) TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "residual shape");
  const int M = x.numel() / C;
  auto part = at::empty({dcp::bn_bwd_reduce_blocks(M, C), 2, C}, f32_like(x));
  auto out = at::empty({2, C}, f32_like(x));
  dcp::launch_bn_bwd_reduce(bp(dy), bp(x), res.has_value() ? bp(*res) : nullptr, scale.data_ptr<float>(),
                            shift.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(), M, C, act,
                            (float)slope, part.data_ptr<float>(), out.data_ptr<float>(), cur_stream(), inv ? 1 : 0);
  return out;
}

std::tuple<Tensor, Tensor> bn_bwd_elemt(const Tensor& dy, const Tensor& x, const optional<Tensor>& res,
                                        const Tensor& scale, const Tensor& shift, const Tensor& mean,
                                        const Tensor& invstd, const optional<Tensor>& sums, double count, int64_t act,
                                        double slope, bool want_dres, bool inv, const optional<Tensor>& graw) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int C = x.size(-1);
  TORCH_CHECK(!inv || ((act == 0 || act == 2) && !res.has_value()), "bn_bwd_elemt: inv needs an invertible act");
  TORCH_CHECK(dy.sizes() == x.sizes() && C % 8 == 0 && C <= 2048, "bn_bwd_elemt shapes");
  auto dx = at::empty_like(x);
  // graw (InplaceABN, with sums): the second output is the raw weight's gradient sign(graw) * sums[1]
  TORCH_CHECK(!graw.has_value() || (sums.has_value() && !want_dres && graw->numel() == C), "bn_bwd_elemt graw");
  Tensor dres = want_dres ? at::empty_like(x) : (graw.has_value() ? at::empty({C}, f32_like(x)) : at::empty({0}, x.options()));
  dcp::launch_bn_bwd_elemt(bp(dy), bp(x), res.has_value() ? bp(*res) : nullptr, scale.data_ptr<float>(),
                           shift.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(), fp(sums),
                           (float)(1.0 / count), x.numel(), C, act, (float)slope, bpm(dx),
                           want_dres ? bpm(dres) : nullptr, cur_stream(), inv ? 1 : 0, fp(graw),
                           graw.has_value() ? dres.data_ptr<float>() : nullptr);
  return {dx, dres};
}

// Both BN input gradients of act(BN(x) + BN_r(r)) from the masked output gradient g (training
// statistics; sums/rsums are the [2][C] (sum g, sum g*xhat) of each BN).
std::tuple<Tensor, Tensor> bn2_bwd_elemt(const Tensor& g, const Tensor& x, const Tensor& r, const Tensor& scale,
                                         const Tensor& mean, const Tensor& invstd, const Tensor& sums,
                                         const Tensor& rscale, const Tensor& rmean, const Tensor& rinvstd,
                                         const Tensor& rsums, double count) {
  CHECK_ACT(g);
  CHECK_ACT(x);
  CHECK_ACT(r);
  const int C = x.size(-1);
  TORCH_CHECK(g.sizes() == x.sizes() && r.sizes() == x.sizes() && C % 8 == 0 && C <= 2048, "bn2_bwd_elemt shapes");
  for (const Tensor* t : {&scale, &mean, &invstd, &rscale, &rmean, &rinvstd})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "bn2_bwd_elemt [C] fp32");
  TORCH_CHECK(sums.numel() == 2 * C && rsums.numel() == 2 * C && sums.is_contiguous() && rsums.is_contiguous(),
              "bn2_bwd_elemt sums [2][C]");
  auto dx = at::empty_like(x);
  auto dr = at::empty_like(r);
  dcp::launch_bn2_bwd_elemt(bp(g), bp(x), bp(r), scale.data_ptr<float>(), mean.data_ptr<float>(),
                            invstd.data_ptr<float>(), sums.data_ptr<float>(), rscale.data_ptr<float>(),
                            rmean.data_ptr<float>(), rinvstd.data_ptr<float>(), rsums.data_ptr<float>(),
                            (float)(1.0 / count), x.numel(), C, bpm(dx), bpm(dr), cur_stream());
  return {dx, dr};
}

// ---------------------------------------------------------------------------
// pooling / layout
// ---------------------------------------------------------------------------
std::tuple<Tensor, Tensor> maxpool_fwd(const Tensor& x, int64_t k, int64_t s, int64_t p) {
  CHECK_ACT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k * k <= 255, "maxpool shapes");
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  auto idx = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  dcp::launch_maxpool_fwd(bp(x), bpm(y), idx.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, k, s, p, cur_stream());
  return {y, idx};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  CHECK_ACT(dy);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  dcp::launch_maxpool_bwd(bp(dy), idx.data_ptr<uint8_t>(), bpm(dx), N, H, W, C, Ho, Wo, k, s, p, cur_stream());
  return dx;
}

static void check_bn_vecs(std::initializer_list<const Tensor*> ts, int C) {
  for (const Tensor* t : ts) {
    CHECK_DEV(*t);
    CHECK_F32(*t);
    CHECK_CONTIG(*t);
    TORCH_CHECK(t->numel() == C, "per-channel vector size");
  }
}

static bool bn_pool_ok(int C) { return C % 8 == 0 && 256 % (C / 8) == 0; }

// max pool of act(x*scale + shift) (the stem BN-apply + ReLU + pool in one pass) -> (y, argmax)
std::tuple<Tensor, Tensor> bn_act_maxpool(const Tensor& x, const Tensor& scale, const Tensor& shift, int64_t act,
                                          int64_t k, int64_t s, int64_t p) {
  CHECK_ACT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(bn_pool_ok(C) && k * k <= 255 && (act == 0 || act == 1), "bn_act_maxpool shapes");
  check_bn_vecs({&scale, &shift}, C);
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  auto idx = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  dcp::launch_maxpool_fwd(bp(x), bpm(y), idx.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, k, s, p, cur_stream(),
                          scale.data_ptr<float>(), shift.data_ptr<float>(), (int)act);
  return {y, idx};
}

// backward reduction of BN(+act) -> max pool: [2, C] = (sum g', sum g' * xhat)
Tensor maxpool_bn_bwd_reduce(const Tensor& dy, const Tensor& idx, const Tensor& x, const Tensor& scale,
                             const Tensor& shift, const Tensor& mean, const Tensor& invstd, int64_t act, int64_t k,
                             int64_t s, int64_t p) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2);
  TORCH_CHECK(bn_pool_ok(C) && dy.size(0) == N && dy.size(3) == C && idx.sizes() == dy.sizes(), "maxpool_bn shapes");
  TORCH_CHECK(Ho == (H + 2 * p - k) / s + 1 && Wo == (W + 2 * p - k) / s + 1, "maxpool_bn geometry");
  check_bn_vecs({&scale, &shift, &mean, &invstd}, C);
  auto part = at::empty({dcp::maxpool_bn_bwd_blocks(), 2, C}, f32_like(x));
  auto sums = at::empty({2, C}, f32_like(x));
  dcp::launch_maxpool_bn_bwd(bp(dy), idx.data_ptr<uint8_t>(), bp(x), N, H, W, C, Ho, Wo, k, s, p,
                             scale.data_ptr<float>(), shift.data_ptr<float>(), mean.data_ptr<float>(),
                             invstd.data_ptr<float>(), (int)act, part.data_ptr<float>(), sums.data_ptr<float>(),
                             nullptr, 0.f, nullptr, cur_stream());
  return sums;
}

// elementwise pass: dx of the BN input from the pooled gradient and the global sums
Tensor maxpool_bn_bwd_elemt(const Tensor& dy, const Tensor& idx, const Tensor& x, const Tensor& scale,
                            const Tensor& shift, const Tensor& mean, const Tensor& invstd, int64_t act,
                            const Tensor& sums, double count, int64_t k, int64_t s, int64_t p) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2);
  TORCH_CHECK(bn_pool_ok(C) && dy.size(0) == N && dy.size(3) == C && idx.sizes() == dy.sizes(), "maxpool_bn shapes");
  TORCH_CHECK(Ho == (H + 2 * p - k) / s + 1 && Wo == (W + 2 * p - k) / s + 1, "maxpool_bn geometry");
  check_bn_vecs({&scale, &shift, &mean, &invstd}, C);
  TORCH_CHECK(sums.numel() == 2 * C && sums.is_contiguous(), "sums [2, C]");
  auto dx = at::empty_like(x);
  dcp::launch_maxpool_bn_bwd(bp(dy), idx.data_ptr<uint8_t>(), bp(x), N, H, W, C, Ho, Wo, k, s, p,
                             scale.data_ptr<float>(), shift.data_ptr<float>(), mean.data_ptr<float>(),
                             invstd.data_ptr<float>(), (int)act, nullptr, nullptr, sums.data_ptr<float>(),
                             (float)(1.0 / count), bpm(dx), cur_stream());
  return dx;
}

Tensor gap_fwd(const Tensor& x) {
  CHECK_ACT(x);
  const int N = x.size(0), C = x.size(-1);
  const int HW = x.numel() / (N * C);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && HW > 0, "gap channels");
  auto y = at::empty({N, C}, x.options());
  auto part = at::empty({dcp::hw_splits(N, HW, C), N, C}, f32_like(x));
  dcp::launch_gap_fwd(bp(x), bpm(y), part.data_ptr<float>(), N, HW, C, cur_stream());
  return y;
}

Tensor gap_bwd(const Tensor& dy, int64_t H, int64_t W, const optional<Tensor>& add) {
  CHECK_ACT(dy);
  const int N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(C % 8 == 0, "gap_bwd channels");
  if (add.has_value()) {
    CHECK_ACT(*add);
    TORCH_CHECK(add->dim() == 4 && add->size(0) == N && add->size(1) == H && add->size(2) == W && add->size(3) == C,
                "gap_bwd add shape");
  }
  auto dx = at::empty({N, H, W, C}, dy.options());
  dcp::launch_gap_bwd(bp(dy), bpm(dx), N, H * W, C, cur_stream(), add.has_value() ? bp(*add) : nullptr);
  return dx;
}

Tensor space_to_depth(const Tensor& x, int64_t b, bool inverse) {
  CHECK_ACT(x);
  const int N = x.size(0);
  if (!inverse) {
    const int H = x.size(1), W = x.size(2), C = x.size(3);
    TORCH_CHECK(H % b == 0 && W % b == 0, "space_to_depth needs H, W divisible by the block");
    auto y = at::empty({N, H / b, W / b, C * b * b}, x.options());
    dcp::launch_s2d(bp(x), bpm(y), N, H, W, C, b, 0, cur_stream());
    return y;
  }
  const int Hb = x.size(1), Wb = x.size(2), Cb = x.size(3);
  const int C = Cb / (b * b), H = Hb * b, W = Wb * b;
  auto y = at::empty({N, H, W, C}, x.options());
  dcp::launch_s2d(bp(x), bpm(y), N, H, W, C, b, 1, cur_stream());
  return y;
}

Tensor to_nhwc(const Tensor& src, bool nchw, int64_t cpad, double in_scale, const optional<Tensor>& mean,
               const optional<Tensor>& stdv) {
  CHECK_DEV(src);
  CHECK_CONTIG(src);
  TORCH_CHECK(src.scalar_type() == at::kByte || src.scalar_type() == at::kFloat, "to_nhwc input u8 or fp32");
  const int N = src.size(0);
  const int C = nchw ? src.size(1) : src.size(3);
  const int H = nchw ? src.size(2) : src.size(1);
  const int W = nchw ? src.size(3) : src.size(2);
  const int Cp = cpad > C ? cpad : C;
  auto y = at::empty({N, H, W, Cp}, src.options().dtype(at::kBFloat16));
  dcp::launch_to_nhwc(src.data_ptr(), src.scalar_type() == at::kByte, nchw, N, C, H, W, Cp, (float)in_scale,
                      fp(mean), fp(stdv), bpm(y), cur_stream());
  return y;
}

// image batch -> space-to-depth 2x2 NHWC input of the s2d stem [N, H/2, W/2, 16]
// Gathered raw records `src` (uint8, device) + per-image boxes `meta` (int64 [B][8], HOST tensor,
// validated here so no box can address outside its record) -> uint8 [B][Ho][Wo][3].
Tensor crop_resize(const Tensor& src, const Tensor& meta, int64_t Ho, int64_t Wo) {
  CHECK_DEV(src);
  CHECK_CONTIG(src);
  TORCH_CHECK(src.scalar_type() == at::kByte, "crop_resize src must be uint8");
  TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.dim() == 2 && meta.size(1) == 8 &&
                  meta.is_contiguous(),
              "crop_resize meta must be a contiguous host int64 [B, 8] tensor");
  TORCH_CHECK(Ho > 0 && Wo > 0 && Ho <= 8192 && Wo <= 8192, "crop_resize output size");
  const int64_t B = meta.size(0), nbytes = src.numel();
  const int64_t* m = meta.data_ptr<int64_t>();
  for (int64_t b = 0; b < B; ++b) {
    const int64_t* r = m + b * 8;
    const int64_t off = r[0], H = r[1], W = r[2], y0 = r[3], x0 = r[4], h = r[5], w = r[6];
    TORCH_CHECK(H > 0 && W > 0 && off >= 0 && off + H * W * 3 <= nbytes, "crop_resize: record ", b,
                " outside the gathered buffer");
    TORCH_CHECK(h > 0 && w > 0 && y0 >= 0 && x0 >= 0 && y0 + h <= H && x0 + w <= W, "crop_resize: box of image ", b,
                " outside its record");
  }
  auto out = at::empty({B, Ho, Wo, 3}, src.options());
  auto md = meta.to(src.device(), /*non_blocking=*/meta.is_pinned());
  dcp::launch_crop_resize(src.data_ptr<uint8_t>(), md.data_ptr<int64_t>(), (int)B, (int)Ho, (int)Wo,
                          out.data_ptr<uint8_t>(), cur_stream());
  return out;
}

Tensor to_nhwc_s2d(const Tensor& src, bool nchw, double in_scale, const optional<Tensor>& mean,
                   const optional<Tensor>& stdv, int64_t block) {
  CHECK_DEV(src);
  CHECK_CONTIG(src);
  TORCH_CHECK(src.scalar_type() == at::kByte || src.scalar_type() == at::kFloat, "to_nhwc_s2d input u8 or fp32");
  const int N = src.size(0);
  const int C = nchw ? src.size(1) : src.size(3);
  const int H = nchw ? src.size(2) : src.size(1);
  const int W = nchw ? src.size(3) : src.size(2);
  TORCH_CHECK(block == 2 || block == 4, "to_nhwc_s2d block is 2 or 4");
  const int b = (int)block, cq = b == 2 ? 4 : 3;
  TORCH_CHECK(C <= cq && H % b == 0 && W % b == 0, "to_nhwc_s2d needs <= ", cq, " channels and H, W divisible by ", b);
  auto y = at::empty({N, H / b, W / b, b * b * cq}, src.options().dtype(at::kBFloat16));
  dcp::launch_to_nhwc_s2d(src.data_ptr(), src.scalar_type() == at::kByte, nchw, N, C, H, W, (float)in_scale, fp(mean),
                          fp(stdv), bpm(y), cur_stream(), b);
  return y;
}

Tensor act_bwd(const Tensor& dy, const Tensor& y, int64_t act) {
  CHECK_ACT(dy);
  CHECK_ACT(y);
  TORCH_CHECK(dy.sizes() == y.sizes() && dy.numel() % 8 == 0, "act_bwd shapes");
  auto dx = at::empty_like(dy);
  dcp::launch_act_bwd(bp(dy), bp(y), bpm(dx), dy.numel(), (int)act, cur_stream());
  return dx;
}

Tensor prefix_mask(const Tensor& x, const Tensor& keep) {
  CHECK_ACT(x);
  TORCH_CHECK(keep.scalar_type() == at::kInt && keep.is_cuda(), "keep must be an int32 GPU scalar");
  auto y = at::empty_like(x);
  dcp::launch_prefix_mask(bp(x), bpm(y), x.size(0), x.size(1), keep.data_ptr<int>(), cur_stream());
  return y;
}

// peer access from the current device to `peer` (the IPC-mapped SyncBN mailboxes, parallel/peer.py)
void enable_peer_access(int64_t peer) {
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "enable_peer_access: hipGetDevice");
  if (peer == dev) return;
  int can = 0;
  TORCH_CHECK(hipDeviceCanAccessPeer(&can, dev, (int)peer) == hipSuccess && can, "no peer access from device ", dev,
              " to ", peer);
  const hipError_t e = hipDeviceEnablePeerAccess((int)peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return;
  }
  TORCH_CHECK(e == hipSuccess, "hipDeviceEnablePeerAccess: ", hipGetErrorString(e));
}

// SyncBN peer exchange (parallel/peer.py): src fp32 [n] -> dst fp32 [world * n] (mode 0) or [n] (mode 1)
void peer_exchange(const Tensor& src, const Tensor& dst, const Tensor& boxes, const Tensor& epoch, int64_t rank,
                   int64_t world, int64_t slot, int64_t mode, const Tensor& err, int64_t timeout_ms) {
  CHECK_DEV(src);
  CHECK_F32(src);
  CHECK_F32(dst);
  CHECK_CONTIG(src);
  CHECK_CONTIG(dst);
  TORCH_CHECK(boxes.scalar_type() == at::kLong && boxes.is_cuda() && boxes.numel() == world, "peer_exchange boxes");
  TORCH_CHECK(epoch.scalar_type() == at::kInt && err.scalar_type() == at::kInt && epoch.is_cuda() && err.is_cuda(),
              "peer_exchange epoch / err: int32 on the device");
  const int64_t n = src.numel();
  TORCH_CHECK(dst.numel() == (mode == 0 ? world * n : n), "peer_exchange dst size");
  TORCH_CHECK(dcp::launch_peer_exchange(src.data_ptr<float>(), (int)n, dst.data_ptr<float>(), boxes.data_ptr<int64_t>(),
                                        epoch.data_ptr<int>(), (int)rank, (int)world, (int)slot, (int)mode,
                                        err.data_ptr<int>(), (int)std::min<int64_t>(timeout_ms, INT32_MAX),
                                        cur_stream()),
              "peer_exchange: world / rank / size out of range");
}

// per-prefix-length (top-1, top-3) correct counts of TestNested; scalar = the one-workgroup-per-sample
// kernel (C <= 4096), else the rank-ballot fast path (any C)
Tensor nested_eval_impl(const Tensor& feat, const Tensor& W, const Tensor& labels, bool scalar) {
  CHECK_DEV(feat);
  CHECK_F32(feat);
  CHECK_F32(W);
  CHECK_CONTIG(feat);
  CHECK_CONTIG(W);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.device() == feat.device(),
              "nested_eval labels: int64 on the feature's device");
  const int B = feat.size(0), D = feat.size(1), C = W.size(1);
  TORCH_CHECK(W.size(0) == D && labels.numel() == B, "nested_eval shapes");
  auto counts = at::zeros({D, 2}, feat.options().dtype(at::kInt));
  if (B == 0 || D == 0) return counts;
  if (scalar) {
    TORCH_CHECK(C <= 4096, "nested_eval_scalar: C <= 4096");
    dcp::launch_nested_eval_scalar(feat.data_ptr<float>(), W.data_ptr<float>(), labels.data_ptr<int64_t>(), B, D, C,
                                   counts.data_ptr<int>(), cur_stream());
    return counts;
  }
  auto ws = at::empty({(int64_t)dcp::nested_eval_workspace(B, D, C)}, feat.options().dtype(at::kByte));
  dcp::launch_nested_eval(feat.data_ptr<float>(), W.data_ptr<float>(), labels.data_ptr<int64_t>(), B, D, C,
                          counts.data_ptr<int>(), ws.data_ptr(), cur_stream());
  return counts;
}

Tensor nested_eval(const Tensor& feat, const Tensor& W, const Tensor& labels) {
  return nested_eval_impl(feat, W, labels, false);
}

Tensor nested_eval_scalar(const Tensor& feat, const Tensor& W, const Tensor& labels) {
  return nested_eval_impl(feat, W, labels, true);
}

Tensor dwconv_fwd(const Tensor& x, const Tensor& filt, int64_t k, int64_t s, int64_t p, bool reflect) {
  CHECK_ACT(x);
  CHECK_F32(filt);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  dcp::launch_dwconv_fwd(bp(x), filt.data_ptr<float>(), bpm(y), N, H, W, C, Ho, Wo, k, s, p, reflect, cur_stream());
  return y;
}

Tensor dwconv_bwd(const Tensor& dy, const Tensor& filt, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p,
                  bool reflect) {
  CHECK_ACT(dy);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  dcp::launch_dwconv_bwd(bp(dy), filt.data_ptr<float>(), bpm(dx), N, H, W, C, Ho, Wo, k, s, p, reflect,
                         cur_stream());
  return dx;
}

Tensor chan_scale_fwd(const Tensor& x, const Tensor& g, const optional<Tensor>& res, bool relu) {
  CHECK_ACT(x);
  CHECK_ACT(g);
  const int N = x.size(0), C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && g.numel() == (int64_t)N * C, "chan_scale shapes");
  if (res.has_value()) {
    CHECK_ACT(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
  }
  auto y = at::empty_like(x);
  dcp::launch_chan_scale_fwd(bp(x), bp(g), res.has_value() ? bp(*res) : nullptr, bpm(y), N, x.numel() / (N * C), C,
                             relu ? 1 : 0, cur_stream());
  return y;
}

std::tuple<Tensor, Tensor, Tensor> chan_scale_bwd(const Tensor& dy, const Tensor& x, const Tensor& g,
                                                  const optional<Tensor>& res, bool relu, bool want_dres) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  CHECK_ACT(g);
  const int N = x.size(0), C = x.size(-1);
  const int HW = x.numel() / (N * C);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && HW > 0 && g.numel() == (int64_t)N * C, "chan_scale_bwd shapes");
  auto dx = at::empty_like(x);
  auto dg = at::empty({N, C}, bf16_like(x));  // the gate's dtype (autograd needs it; no cast launch)
  auto part = at::empty({dcp::hw_splits(N, HW, C), N, C}, f32_like(x));
  Tensor dres = want_dres ? at::empty_like(x) : at::empty({0}, x.options());
  dcp::launch_chan_scale_bwd(bp(dy), bp(x), bp(g), res.has_value() ? bp(*res) : nullptr, bpm(dx),
                             bpm(dg), part.data_ptr<float>(), want_dres ? bpm(dres) : nullptr, N, HW, C,
                             relu ? 1 : 0, cur_stream());
  return {dx, dg, dres};
}

// squeeze-excitation gate of a small batch (one workgroup): p [N,C] -> (h [N,R], g [N,C]);
// w1 [>=R, C], w2 [>=C, R] bf16 (the prepared weights, rows past R / C unused)
std::tuple<Tensor, Tensor> se_gate_fwd(const Tensor& p, const Tensor& w1, const optional<Tensor>& b1, const Tensor& w2,
                                       const optional<Tensor>& b2, int64_t R) {
  CHECK_ACT(p);
  CHECK_ACT(w1);
  CHECK_ACT(w2);
  TORCH_CHECK(p.dim() == 2, "se_gate_fwd: p [N,C]");
  const int N = p.size(0), C = p.size(1);
  TORCH_CHECK(dcp::se_gate_supported(N, C, (int)R) && w1.dim() == 2 && w1.size(0) >= R && w1.size(1) == C &&
                  w2.dim() == 2 && w2.size(0) >= C && w2.size(1) == R,
              "se_gate_fwd shapes");
  TORCH_CHECK((!b1.has_value() || b1->numel() >= R) && (!b2.has_value() || b2->numel() >= C), "se_gate_fwd bias");
  auto h = at::empty({N, R}, p.options());
  auto g = at::empty({N, C}, p.options());
  dcp::launch_se_gate_fwd(bp(p), bp(w1), fp(b1), bp(w2), fp(b2), bpm(h), bpm(g), N, C, (int)R, cur_stream());
  return {h, g};
}

// w1t = W1^T [C, >=R], w2t = W2^T [R, >=C] (the transposed prepared weights)
// -> (dp [N,C] bf16, dW1 [R,C], db1 [R], dW2 [C,R], db2 [C] fp32)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> se_gate_bwd(const Tensor& dg, const Tensor& g, const Tensor& h,
                                                               const Tensor& p, const Tensor& w1t, const Tensor& w2t) {
  CHECK_ACT(dg);
  CHECK_ACT(g);
  CHECK_ACT(h);
  CHECK_ACT(p);
  CHECK_ACT(w1t);
  CHECK_ACT(w2t);
  const int N = p.size(0), C = p.size(1), R = h.size(1);
  TORCH_CHECK(dcp::se_gate_supported(N, C, R) && dg.sizes() == p.sizes() && g.sizes() == p.sizes() && h.size(0) == N &&
                  w1t.dim() == 2 && w1t.size(0) == C && w1t.size(1) >= R && w2t.dim() == 2 && w2t.size(0) == R &&
                  w2t.size(1) >= C,
              "se_gate_bwd shapes");
  auto dp = at::empty_like(p);
  auto dw1 = at::empty({R, C}, f32_like(p));
  auto db1 = at::empty({R}, f32_like(p));
  auto dw2 = at::empty({C, R}, f32_like(p));
  auto db2 = at::empty({C}, f32_like(p));
  dcp::launch_se_gate_bwd(bp(dg), bp(g), bp(h), bp(p), bp(w1t), (int)w1t.size(1), bp(w2t), (int)w2t.size(1),
                          dw1.data_ptr<float>(), db1.data_ptr<float>(), dw2.data_ptr<float>(), db2.data_ptr<float>(),
                          bpm(dp), N, C, R, cur_stream());
  return {dp, dw1, db1, dw2, db2};
}

// ---------------------------------------------------------------------------
// losses
// ---------------------------------------------------------------------------
std::tuple<Tensor, Tensor> xent_fwd(const Tensor& logits, const Tensor& labels, int64_t C, double smoothing) {
  CHECK_DEV(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits rows must be contiguous");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda(), "labels int64 on GPU");
  const int B = logits.size(0), ld = logits.stride(0);
  TORCH_CHECK(C <= ld && labels.numel() == B, "xent shapes");
  auto loss = at::empty({B}, f32_like(logits));
  auto rank = at::empty({B}, logits.options().dtype(at::kInt));
  dcp::launch_xent_fwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B, ld, C,
                       labels.data_ptr<int64_t>(), loss.data_ptr<float>(), rank.data_ptr<int>(), (float)smoothing,
                       cur_stream());
  return {loss, rank};
}

// acc (fp64 [4]) += [loss_scale * sum(loss), #(rank < 1), #(rank < 3), nrows] over rank[:nrows]
void metric_accum(const Tensor& acc, const Tensor& loss, double loss_scale, const Tensor& rank, int64_t nrows) {
  CHECK_DEV(acc);
  TORCH_CHECK(acc.scalar_type() == at::kDouble && acc.is_contiguous() && acc.numel() >= 4, "acc: fp64 [4]");
  TORCH_CHECK(rank.scalar_type() == at::kInt && rank.is_contiguous() && rank.is_cuda(), "rank: int32 on GPU");
  TORCH_CHECK(nrows >= 0 && nrows <= rank.numel(), "metric_accum: nrows");
  const Tensor l = loss.to(at::kFloat).contiguous();
  dcp::launch_metric_accum(acc.data_ptr<double>(), l.data_ptr<float>(), (int)l.numel(), (float)loss_scale,
                           rank.data_ptr<int>(), (int)nrows, cur_stream());
}

// logits may be a column slice of a wider (padded) buffer: row stride = stride(0)
Tensor xent_bwd(const Tensor& logits, const Tensor& labels, int64_t C, const Tensor& grad_out, double scale,
                double smoothing, bool out_bf16) {
  CHECK_DEV(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits rows must be contiguous");
  const int B = logits.size(0), ld = logits.stride(0), ldo = logits.size(1);
  auto d = at::empty({B, ldo}, logits.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  auto g = grad_out.to(at::kFloat).contiguous();
  dcp::launch_xent_bwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, B, ld, C,
                       labels.data_ptr<int64_t>(), g.data_ptr<float>(), (float)scale, (float)smoothing, d.data_ptr(),
                       ldo, out_bf16, cur_stream());
  return d;
}

Tensor log_softmax_fwd(const Tensor& x, int64_t C) {
  CHECK_DEV(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "rows must be contiguous");
  const int B = x.size(0), ld = x.stride(0);
  auto y = at::empty({B, C}, f32_like(x));
  dcp::launch_log_softmax_fwd(x.data_ptr(), x.scalar_type() == at::kBFloat16, B, ld, C, y.data_ptr<float>(),
                              cur_stream());
  return y;
}

Tensor log_softmax_bwd(const Tensor& y, const Tensor& dy, int64_t ldo, bool out_bf16) {
  CHECK_DEV(y);
  const int B = y.size(0), C = y.size(1);
  auto dyc = dy.to(at::kFloat).contiguous();
  auto dx = at::empty({B, ldo}, y.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  dcp::launch_log_softmax_bwd(y.data_ptr<float>(), dyc.data_ptr<float>(), B, C, ldo, dx.data_ptr(), out_bf16,
                              cur_stream());
  return dx;
}

std::tuple<Tensor, Tensor> l2norm_rows(const Tensor& x, int64_t ldo, double eps, int64_t rows_out) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  const int R = x.size(0), D = x.size(1);
  const int Ro = rows_out < 0 ? R : (int)rows_out;
  TORCH_CHECK(Ro >= R && ldo >= D, "l2norm_rows: output smaller than input");
  auto y = at::empty({Ro, ldo}, x.options().dtype(at::kBFloat16));
  auto inv = at::empty({Ro}, f32_like(x));
  dcp::launch_l2norm_rows(x.data_ptr(), x.scalar_type() == at::kBFloat16, R, Ro, D, ldo, bpm(y),
                          inv.data_ptr<float>(), (float)eps, cur_stream());
  return {y, inv};
}

Tensor l2norm_bwd(const Tensor& dy, const Tensor& y, const Tensor& inv, int64_t D, bool out_bf16) {
  CHECK_DEV(dy);
  CHECK_CONTIG(dy);
  CHECK_ACT(y);
  const int R = dy.size(0);
  auto dx = at::empty({R, D}, dy.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  dcp::launch_l2norm_bwd(dy.data_ptr(), dy.scalar_type() == at::kBFloat16, dy.size(1), bp(y), y.size(1),
                         inv.data_ptr<float>(), R, D, dx.data_ptr(), out_bf16, cur_stream());
  return dx;
}

Tensor transpose2d(const Tensor& x) {
  CHECK_ACT(x);
  TORCH_CHECK(x.dim() == 2, "transpose2d expects a matrix");
  auto y = at::empty({x.size(1), x.size(0)}, x.options());
  dcp::launch_transpose2d(bp(x), bpm(y), x.size(0), x.size(1), cur_stream());
  return y;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> arcface_fwd(const Tensor& cosv, const Tensor& labels, int64_t C, double s,
                                                       double m, bool easy, bool want_logits) {
  CHECK_ACT(cosv);
  const int B = cosv.size(0), ld = cosv.size(1);
  const float cm = cosf((float)m), sm = sinf((float)m), th = cosf(3.14159265358979f - (float)m);
  const float mm = sinf(3.14159265358979f - (float)m) * (float)m;
  auto logits = want_logits ? at::empty({B, C}, f32_like(cosv)) : at::empty({0}, f32_like(cosv));
  auto loss = at::empty({B}, f32_like(cosv));
  auto rank = at::empty({B}, cosv.options().dtype(at::kInt));
  auto dphi = at::empty({B}, f32_like(cosv));
  dcp::launch_arcface_fwd(bp(cosv), B, ld, C, labels.data_ptr<int64_t>(), (float)s, cm, sm, th, mm, easy,
                          want_logits ? logits.data_ptr<float>() : nullptr, loss.data_ptr<float>(),
                          rank.data_ptr<int>(), dphi.data_ptr<float>(), cur_stream());
  return {loss, rank, dphi, logits};
}

Tensor arcface_bwd(const Tensor& cosv, const Tensor& labels, int64_t C, double s, double m, bool easy,
                   const Tensor& dphi, const Tensor& grad_out, double scale) {
  CHECK_ACT(cosv);
  const int B = cosv.size(0), ld = cosv.size(1);
  const float cm = cosf((float)m), sm = sinf((float)m), th = cosf(3.14159265358979f - (float)m);
  const float mm = sinf(3.14159265358979f - (float)m) * (float)m;
  auto g = grad_out.to(at::kFloat).contiguous();
  auto dcos = at::empty({B, ld}, cosv.options());
  dcp::launch_arcface_bwd(bp(cosv), B, ld, C, labels.data_ptr<int64_t>(), (float)s, cm, sm, th, mm, easy,
                          dphi.data_ptr<float>(), g.data_ptr<float>(), (float)scale, bpm(dcos), cur_stream());
  return dcos;
}

// x [R][D] -> (y [Rp][Dp] bf16 normalised rows, yT [Dp][Rp], inverse norms [Rp]) in one pass
std::tuple<Tensor, Tensor, Tensor> arcface_l2norm_t(const Tensor& x, int64_t Rp, int64_t Dp, double eps) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  const int R = x.size(0), D = x.size(1);
  auto y = at::empty({Rp, Dp}, x.options().dtype(at::kBFloat16));
  auto yT = at::empty({Dp, Rp}, x.options().dtype(at::kBFloat16));
  auto inv = at::empty({Rp}, f32_like(x));
  TORCH_CHECK(dcp::launch_arcface_l2norm_t(x.data_ptr(), x.scalar_type() == at::kBFloat16, R, D, (int)Rp, (int)Dp,
                                           bpm(y), bpm(yT), inv.data_ptr<float>(), (float)eps, cur_stream()),
              "arcface_l2norm_t: Rp % 64, D <= Dp in {128, 256}");
  return {y, yT, inv};
}

// Fused ArcFace head (arcface.hip): xn [Bp][Dp], wn [Cp][Dp] from l2norm_rows (zero padding rows).
// -> loss [B], rank [B], lse [Bp] and the per-row (target logit, d phi / d cos) [Bp][2] for backward
std::tuple<Tensor, Tensor, Tensor, Tensor> arcface_fused_fwd(const Tensor& xn, const Tensor& wn, const Tensor& labels,
                                                             int64_t B, int64_t C, double s, double m, bool easy) {
  CHECK_ACT(xn);
  CHECK_ACT(wn);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda() && labels.numel() == B, "arcface_fused labels");
  const int Bp = xn.size(0), Dp = xn.size(1), Cp = wn.size(0);
  TORCH_CHECK(wn.size(1) == Dp && Bp >= B && Cp >= C, "arcface_fused_fwd shapes");
  const int S = dcp::arcface_fused_fwd_splits(Bp, Cp);
  auto loss = at::empty({B}, f32_like(xn));
  auto rank = at::empty({B}, xn.options().dtype(at::kInt));
  auto lse = at::empty({Bp}, f32_like(xn));
  auto lab = at::empty({Bp, 2}, f32_like(xn));
  auto part = at::empty({(int64_t)S * Bp * 4}, f32_like(xn));
  TORCH_CHECK(dcp::launch_arcface_fused_fwd(bp(xn), bp(wn), labels.data_ptr<int64_t>(), B, Bp, C, Cp, Dp, (float)s,
                                            (float)m, easy, lab.data_ptr<float>(), part.data_ptr<float>(),
                                            loss.data_ptr<float>(), rank.data_ptr<int>(), lse.data_ptr<float>(),
                                            cur_stream()),
              "arcface_fused_fwd: unsupported shape (B, C padded to 64, D padded to 128 / 256)");
  return {loss, rank, lse, lab};
}

Tensor arcface_fused_dx(const Tensor& xn, const Tensor& wn, const Tensor& wnT, const Tensor& labels, const Tensor& lse,
                        const Tensor& lab, const Tensor& grad_out, double scale, const Tensor& inv_x, int64_t B,
                        int64_t C, int64_t D, double s, bool out_bf16) {
  CHECK_ACT(xn);
  CHECK_ACT(wn);
  CHECK_ACT(wnT);
  const int Bp = xn.size(0), Dp = xn.size(1), Cp = wn.size(0);
  TORCH_CHECK(wnT.size(0) == Dp && wnT.size(1) == Cp, "arcface_fused_dx: wnT [Dp][Cp]");
  auto g = grad_out.to(at::kFloat).contiguous();
  const int S = dcp::arcface_fused_dx_splits(Bp, Cp);
  auto part = at::empty({(int64_t)S * Bp * Dp}, f32_like(xn));
  auto dx = at::empty({B, D}, xn.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  TORCH_CHECK(dcp::launch_arcface_fused_dx(bp(xn), bp(wn), bp(wnT), labels.data_ptr<int64_t>(), B, Bp, C, Cp, Dp, D,
                                           (float)s, lab.data_ptr<float>(), lse.data_ptr<float>(), g.data_ptr<float>(),
                                           (float)scale, inv_x.data_ptr<float>(), part.data_ptr<float>(),
                                           dx.data_ptr(), out_bf16, cur_stream()),
              "arcface_fused_dx: unsupported shape");
  return dx;
}

Tensor arcface_fused_dw(const Tensor& xn, const Tensor& xnT, const Tensor& wn, const Tensor& labels, const Tensor& lse,
                        const Tensor& lab, const Tensor& grad_out, double scale, const Tensor& inv_w, int64_t B,
                        int64_t C, int64_t D, double s) {
  CHECK_ACT(xn);
  CHECK_ACT(xnT);
  CHECK_ACT(wn);
  const int Bp = xn.size(0), Dp = xn.size(1), Cp = wn.size(0);
  TORCH_CHECK(xnT.size(0) == Dp && xnT.size(1) == Bp, "arcface_fused_dw: xnT [Dp][Bp]");
  auto g = grad_out.to(at::kFloat).contiguous();
  auto dw = at::empty({C, D}, f32_like(xn));
  const int S = dcp::arcface_fused_dw_splits(Bp, Cp);
  auto part = at::empty({S > 1 ? (int64_t)S * Cp * Dp : 1}, f32_like(xn));
  TORCH_CHECK(dcp::launch_arcface_fused_dw(bp(xn), bp(xnT), bp(wn), labels.data_ptr<int64_t>(), B, Bp, C, Cp, Dp, D,
                                           (float)s, lab.data_ptr<float>(), lse.data_ptr<float>(), g.data_ptr<float>(),
                                           (float)scale, inv_w.data_ptr<float>(), part.data_ptr<float>(),
                                           dw.data_ptr<float>(), cur_stream()),
              "arcface_fused_dw: unsupported shape");
  return dw;
}

// ---------------------------------------------------------------------------
// optimizers (multi-tensor). table: int64 [n,6] = (p, g, s1, s2, shadow, numel); chunks int32 [k,2]
// ---------------------------------------------------------------------------
// table: MTEntry rows (dst, src, -, -, -, n); mode bit 0 = src bf16, bit 1 = dst bf16
void mt_copy(const Tensor& table, const Tensor& chunks, double scale, int64_t mode) {
  CHECK_DEV(table);
  CHECK_DEV(chunks);
  dcp::launch_mt_copy(reinterpret_cast<const dcp::MTEntry*>(table.data_ptr()),
                      reinterpret_cast<const int2*>(chunks.data_ptr()), chunks.size(0), (float)scale, (int)mode,
                      cur_stream());
}

void mt_sgd(const Tensor& table, const Tensor& chunks, double lr, double momentum, double dampening, double wd,
            bool nesterov, bool first, double grad_scale) {
  CHECK_DEV(table);
  CHECK_DEV(chunks);
  dcp::SgdHyper h{(float)lr, (float)momentum, (float)dampening, (float)wd, (float)grad_scale, nesterov ? 1 : 0,
                  first ? 1 : 0};
  dcp::launch_mt_sgd(reinterpret_cast<const dcp::MTEntry*>(table.data_ptr()),
                     reinterpret_cast<const int2*>(chunks.data_ptr()), chunks.size(0), h, cur_stream());
}

// step_dev (optional int32[1] on the device): the step count the bias corrections use, read by
// the kernel -- a HIP-graph replay then applies the current step's correction, not the captured one
void mt_adam(const Tensor& table, const Tensor& chunks, double lr, double beta1, double beta2, double eps, double wd,
             int64_t step, bool decoupled, double grad_scale, const c10::optional<Tensor>& step_dev) {
  CHECK_DEV(table);
  CHECK_DEV(chunks);
  dcp::AdamHyper h;
  h.step_dev = nullptr;
  if (step_dev.has_value() && step_dev->defined()) {
    CHECK_DEV((*step_dev));
    TORCH_CHECK(step_dev->scalar_type() == at::kInt && step_dev->numel() == 1, "mt_adam: step_dev int32[1]");
    h.step_dev = step_dev->data_ptr<int>();
  }
  h.lr = lr;
  h.beta1 = beta1;
  h.beta2 = beta2;
  h.eps = eps;
  h.wd = wd;
  h.grad_scale = grad_scale;
  h.bc1 = 1.0 - std::pow(beta1, (double)step);
  h.bc2 = 1.0 - std::pow(beta2, (double)step);
  h.decoupled = decoupled ? 1 : 0;
  dcp::launch_mt_adam(reinterpret_cast<const dcp::MTEntry*>(table.data_ptr()),
                      reinterpret_cast<const int2*>(chunks.data_ptr()), chunks.size(0), h, cur_stream());
}

// state int32 [4] = (prefix, mask, k, thr_bits) prepared by the caller; returns the threshold (fp32 GPU scalar)
Tensor cdr_threshold(const Tensor& table, const Tensor& chunks, const Tensor& state) {
  CHECK_DEV(state);
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() == 4, "cdr state int32[4]");
  auto hist = at::zeros({256}, state.options());
  dcp::launch_cdr_threshold(reinterpret_cast<const dcp::MTEntry*>(table.data_ptr()),
                            reinterpret_cast<const int2*>(chunks.data_ptr()), chunks.size(0),
                            reinterpret_cast<uint32_t*>(state.data_ptr()), reinterpret_cast<uint32_t*>(hist.data_ptr()),
                            cur_stream());
  return state.narrow(0, 3, 1).view(at::kFloat);
}

void cdr_mask(const Tensor& table, const Tensor& chunks, const Tensor& state, double clip) {
  dcp::launch_cdr_mask(reinterpret_cast<const dcp::MTEntry*>(table.data_ptr()),
                       reinterpret_cast<const int2*>(chunks.data_ptr()), chunks.size(0),
                       reinterpret_cast<const uint32_t*>(state.data_ptr()), (float)clip, cur_stream());
}

}  // namespace

// entries: int64 [E, 7] packed WPEntry table; blocks: int32 [B, 2] (entry, tile) -- both device tensors
void mt_weight_prep(const Tensor& entries, const Tensor& blocks) {
  CHECK_DEV(entries);
  CHECK_DEV(blocks);
  TORCH_CHECK(entries.scalar_type() == at::kLong && entries.dim() == 2 && entries.size(1) == 7, "entries [E,7] int64");
  TORCH_CHECK(blocks.scalar_type() == at::kInt && blocks.dim() == 2 && blocks.size(1) == 2, "blocks [B,2] int32");
  dcp::launch_mt_weight_prep(entries.data_ptr(), blocks.data_ptr(), (int)blocks.size(0), cur_stream());
}

// host int64 table -> int64 device tensor on `device_like`'s device (kernel-argument transport)
Tensor table_fill(const Tensor& host, const Tensor& device_like) {
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == at::kLong && host.is_contiguous(), "table_fill: host int64");
  CHECK_DEV(device_like);
  auto out = at::empty({host.numel()}, device_like.options().dtype(at::kLong));
  dcp::launch_table_fill(host.data_ptr<int64_t>(), host.numel(), out.data_ptr<int64_t>(), cur_stream());
  return out;
}

int64_t autotune_entries() { return dcp::tap_gemm_tuned_count() + wgrad_autotune_entries(); }

// the autotuner's decisions (tap GEMM "tg\t..." and weight-gradient "wg\t..." lines) for a tuning
// cache file (DCP_TUNE_CACHE, _ext.py): a later process replays them without timing anything
std::string autotune_export() {
  std::string out;
  const std::string tg = dcp::tap_gemm_tune_export();
  size_t pos = 0;
  while (pos < tg.size()) {
    const size_t nl = tg.find('\n', pos);
    out += "tg\t" + tg.substr(pos, (nl == std::string::npos ? tg.size() : nl) - pos) + "\n";
    pos = nl == std::string::npos ? tg.size() : nl + 1;
  }
  std::lock_guard<std::mutex> lk(g_wg_mu);
  for (const auto& kv : g_wg_choice) out += "wg\t" + kv.first + "\t" + std::to_string(kv.second) + "\n";
  return out;
}

int64_t autotune_import(const std::string& text) {
  std::string tg;
  int64_t n = 0;
  const int nwg = (int)(sizeof(kWgCfgs) / sizeof(kWgCfgs[0]));
  size_t pos = 0;
  while (pos < text.size()) {
    size_t nl = text.find('\n', pos);
    if (nl == std::string::npos) nl = text.size();
    const std::string line = text.substr(pos, nl - pos);
    pos = nl + 1;
    if (line.compare(0, 3, "tg\t") == 0) {
      tg += line.substr(3) + "\n";
    } else if (line.compare(0, 3, "wg\t") == 0) {
      const size_t tab = line.rfind('\t');
      if (tab <= 3) continue;
      const int c = atoi(line.c_str() + tab + 1);
      if (c < 0 || c >= nwg) continue;
      std::lock_guard<std::mutex> lk(g_wg_mu);
      g_wg_choice[line.substr(3, tab - 3)] = c;
      ++n;
    }
  }
  return n + dcp::tap_gemm_tune_import(tg);
}

void set_tuning(int64_t idx, int64_t value) {
  TORCH_CHECK(idx >= 0 && idx < dcp::kTuneSlots, "tuning index");
  dcp::g_tune[idx] = (int)value;
}

// "name=slot;..." of every named slot (tune.h): the Python mirror (tuning.py) is checked against it
std::string tuning_slots() {
  std::string out;
  for (const auto& t : dcp::kTuneSlotNames) out += std::string(t.name) + "=" + std::to_string(t.slot) + ";";
  return out;
}

TORCH_LIBRARY(dcp, m) {
  m.def("set_tuning(int idx, int value) -> ()", &set_tuning);
  m.def("tuning_slots() -> str", &tuning_slots);
  m.def("autotune_entries() -> int", &autotune_entries);
  m.def("autotune_export() -> str", &autotune_export);
  m.def("autotune_import(str text) -> int", &autotune_import);
  m.def("table_fill(Tensor host, Tensor device_like) -> Tensor", &table_fill);
  m.def("mt_weight_prep(Tensor entries, Tensor blocks) -> ()", &mt_weight_prep);
  m.def("conv_fwd(Tensor x, Tensor w, int stride, int pad, bool stats) -> (Tensor, Tensor)", &conv_fwd);
  m.def("conv_dgrad(Tensor dy, Tensor wt, int H, int W, int stride, int pad, Tensor? add=None) -> Tensor", &conv_dgrad);
  m.def(
      "conv_dgrad_bn(Tensor dy, Tensor wt, int pad, Tensor? add, Tensor y, Tensor? res, Tensor scale, Tensor shift, "
      "Tensor mean, Tensor invstd, int act, Tensor? mask=None, float slope=0.0) -> (Tensor, Tensor)",
      &conv_dgrad_bn);
  m.def("conv_wgrad(Tensor dy, Tensor x, int KH, int KW, int stride, int pad) -> Tensor", &conv_wgrad);
  m.def("linear_fwd(Tensor x, Tensor w, Tensor? bias, int act) -> Tensor", &linear_fwd);
  m.def("linear_wgrad(Tensor dy, Tensor x) -> Tensor", &linear_wgrad);
  m.def("weight_prep(Tensor w, int co_pad, bool transposed) -> (Tensor, Tensor)", &weight_prep);
  m.def("grouped_conv_fwd(Tensor x, Tensor w, int groups, int stride, int pad) -> Tensor", &grouped_conv_fwd);
  m.def("grouped_conv_fwd_stats(Tensor x, Tensor w, int groups, int stride, int pad) -> (Tensor, Tensor)",
        &grouped_conv_fwd_stats);
  m.def("grouped_conv_dgrad_bn(Tensor dy, Tensor w, int H, int W, int groups, int stride, int pad, Tensor z, "
        "Tensor scale, Tensor shift, Tensor mean, Tensor invstd) -> (Tensor, Tensor)",
        &grouped_conv_dgrad_bn);
  m.def("grouped_conv_dgrad(Tensor dy, Tensor w, int H, int W, int groups, int stride, int pad) -> Tensor",
        &grouped_conv_dgrad);
  m.def("grouped_conv_wgrad(Tensor dy, Tensor x, int KH, int KW, int groups, int stride, int pad) -> Tensor",
        &grouped_conv_wgrad);
  m.def("bn_stats(Tensor x, Tensor? slabs) -> Tensor", &bn_stats);
  m.def("colsum(Tensor x) -> Tensor", &colsum);
  m.def(
      "bn_stats_finalize(Tensor x, Tensor? slabs, Tensor? gamma, Tensor? beta, Tensor? run_mean, Tensor? run_var, "
      "float momentum, float eps, float iabn_eps=-1., Tensor(a!)? rgamma_out=None) -> (Tensor, Tensor, Tensor, Tensor)",
      &bn_stats_finalize);
  m.def(
      "bn_finalize(Tensor stats, Tensor? gamma, Tensor? beta, Tensor? run_mean, Tensor? run_var, float momentum, "
      "float eps, float iabn_eps=-1., Tensor(a!)? rgamma_out=None) -> (Tensor, Tensor, Tensor, Tensor)",
      &bn_finalize);
  m.def(
      "bn_eval_coeff(Tensor? gamma, Tensor? beta, Tensor run_mean, Tensor run_var, float eps) -> (Tensor, Tensor, "
      "Tensor, Tensor)",
      &bn_eval_coeff);
  m.def("bn2_act_mask(Tensor x, Tensor res, Tensor scale, Tensor shift, Tensor rscale, Tensor rshift, int act, "
        "float slope) -> (Tensor, Tensor)",
        &bn2_act_mask);
  m.def("bn2_bwd_elemt(Tensor g, Tensor x, Tensor r, Tensor scale, Tensor mean, Tensor invstd, Tensor sums, "
        "Tensor rscale, Tensor rmean, Tensor rinvstd, Tensor rsums, float count) -> (Tensor, Tensor)",
        &bn2_bwd_elemt);
  m.def("bn_act(Tensor x, Tensor? res, Tensor scale, Tensor shift, int act, float slope) -> Tensor", &bn_act);
  m.def("bn_fin_act(Tensor x, Tensor slabs, Tensor? res, Tensor? gamma, Tensor? beta, Tensor? run_mean, "
        "Tensor? run_var, float momentum, float eps, int act, float slope, bool want_mask, float iabn_eps=-1., "
        "Tensor(a!)? rgamma_out=None) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)",
        &bn_fin_act);
  m.def("bn_fin_act_timeouts(Tensor like) -> int", &bn_fin_act_timeouts);
  m.def("bn_act_mask(Tensor x, Tensor? res, Tensor scale, Tensor shift, int act, float slope) -> (Tensor, Tensor)",
        &bn_act_mask);
  m.def(
      "bn_bwd_reduce(Tensor dy, Tensor x, Tensor? res, Tensor scale, Tensor shift, Tensor mean, Tensor invstd, int "
      "act, float slope, bool inv=False) -> Tensor",
      &bn_bwd_reduce);
  m.def(
      "bn_bwd_elemt(Tensor dy, Tensor x, Tensor? res, Tensor scale, Tensor shift, Tensor mean, Tensor invstd, "
      "Tensor? sums, float count, int act, float slope, bool want_dres, bool inv=False, Tensor? graw=None) "
      "-> (Tensor, Tensor)",
      &bn_bwd_elemt);
  m.def("maxpool_fwd(Tensor x, int k, int s, int p) -> (Tensor, Tensor)", &maxpool_fwd);
  m.def("conv_fwd_pro(Tensor x, Tensor w, Tensor scale, Tensor shift, bool stats) -> (Tensor, Tensor)", &conv_fwd_pro);
  m.def("conv_wgrad_pro(Tensor dy, Tensor x, Tensor scale, Tensor shift) -> Tensor", &conv_wgrad_pro);
  m.def("maxpool_bwd(Tensor dy, Tensor idx, int H, int W, int k, int s, int p) -> Tensor", &maxpool_bwd);
  m.def("bn_act_maxpool(Tensor x, Tensor scale, Tensor shift, int act, int k, int s, int p) -> (Tensor, Tensor)",
        &bn_act_maxpool);
  m.def(
      "maxpool_bn_bwd_reduce(Tensor dy, Tensor idx, Tensor x, Tensor scale, Tensor shift, Tensor mean, "
      "Tensor invstd, int act, int k, int s, int p) -> Tensor",
      &maxpool_bn_bwd_reduce);
  m.def(
      "maxpool_bn_bwd_elemt(Tensor dy, Tensor idx, Tensor x, Tensor scale, Tensor shift, Tensor mean, "
      "Tensor invstd, int act, Tensor sums, float count, int k, int s, int p) -> Tensor",
      &maxpool_bn_bwd_elemt);
  m.def("gap_fwd(Tensor x) -> Tensor", &gap_fwd);
  m.def("gap_bwd(Tensor dy, int H, int W, Tensor? add=None) -> Tensor", &gap_bwd);
  m.def("space_to_depth(Tensor x, int b, bool inverse) -> Tensor", &space_to_depth);
  m.def("to_nhwc(Tensor src, bool nchw, int cpad, float in_scale, Tensor? mean, Tensor? std) -> Tensor", &to_nhwc);
  m.def("crop_resize(Tensor src, Tensor meta, int Ho, int Wo) -> Tensor", &crop_resize);
  m.def("to_nhwc_s2d(Tensor src, bool nchw, float in_scale, Tensor? mean, Tensor? std, int block=2) -> Tensor", &to_nhwc_s2d);
  m.def("conv_fwd_geo(Tensor x, Tensor w, int stride, int pad, int Ho, int Wo, bool stats) -> (Tensor, Tensor)",
        &conv_fwd_geo);
  m.def("stem_fwd(Tensor x, Tensor w, bool stats) -> (Tensor, Tensor)", &stem_fwd);
  m.def("stem_bwd_fusable(Tensor z) -> bool", &stem_bwd_fusable);
  m.def("stem_bn_pool_bwd(Tensor dy, Tensor idx, Tensor z, Tensor x16, Tensor scale, Tensor shift, Tensor mean, "
        "Tensor invstd, int act) -> (Tensor, Tensor)",
        &stem_bn_pool_bwd);
  m.def("stem_bwd_dw(Tensor tot, Tensor sums, Tensor scale, Tensor invstd, float count) -> Tensor", &stem_bwd_dw);
  m.def("conv_wgrad_geo(Tensor dy, Tensor x, int KH, int KW, int stride, int pad) -> Tensor", &conv_wgrad_geo);
  m.def("act_bwd(Tensor dy, Tensor y, int act) -> Tensor", &act_bwd);
  m.def("prefix_mask(Tensor x, Tensor keep) -> Tensor", &prefix_mask);
  m.def("nested_eval(Tensor feat, Tensor W, Tensor labels) -> Tensor", &nested_eval);
  m.def("enable_peer_access(int peer) -> ()", &enable_peer_access);
  m.def("conv3x3_fwd_pro(Tensor x, Tensor w, Tensor scale, Tensor shift, bool stats) -> (Tensor, Tensor)",
        &conv3x3_fwd_pro);
  m.def("conv3x3_wgrad_pro(Tensor dy, Tensor x, Tensor scale, Tensor shift) -> Tensor", &conv3x3_wgrad_pro);
  m.def("conv3x3_pro_fits(int N, int H, int W, int C, int Co) -> bool", &conv3x3_pro_fits);
  m.def("peer_exchange(Tensor src, Tensor(a!) dst, Tensor boxes, Tensor(b!) epoch, int rank, int world, int slot, "
        "int mode, Tensor(c!) err, int timeout_ms) -> ()", &peer_exchange);
  m.def("nested_eval_scalar(Tensor feat, Tensor W, Tensor labels) -> Tensor", &nested_eval_scalar);
  m.def("dwconv_fwd(Tensor x, Tensor filt, int k, int s, int p, bool reflect) -> Tensor", &dwconv_fwd);
  m.def("dwconv_bwd(Tensor dy, Tensor filt, int H, int W, int k, int s, int p, bool reflect) -> Tensor", &dwconv_bwd);
  m.def("chan_scale_fwd(Tensor x, Tensor g, Tensor? res, bool relu) -> Tensor", &chan_scale_fwd);
  m.def("se_gate_fwd(Tensor p, Tensor w1, Tensor? b1, Tensor w2, Tensor? b2, int R) -> (Tensor, Tensor)", &se_gate_fwd);
  m.def("se_gate_bwd(Tensor dg, Tensor g, Tensor h, Tensor p, Tensor w1t, Tensor w2t) -> (Tensor, Tensor, Tensor, Tensor, "
        "Tensor)",
        &se_gate_bwd);
  m.def("chan_scale_bwd(Tensor dy, Tensor x, Tensor g, Tensor? res, bool relu, bool want_dres) -> (Tensor, Tensor, "
        "Tensor)",
        &chan_scale_bwd);
  m.def("xent_fwd(Tensor logits, Tensor labels, int C, float smoothing) -> (Tensor, Tensor)", &xent_fwd);
  m.def("metric_accum(Tensor(a!) acc, Tensor loss, float loss_scale, Tensor rank, int nrows) -> ()", &metric_accum);
  m.def(
      "xent_bwd(Tensor logits, Tensor labels, int C, Tensor grad_out, float scale, float smoothing, bool out_bf16) "
      "-> Tensor",
      &xent_bwd);
  m.def("log_softmax_fwd(Tensor x, int C) -> Tensor", &log_softmax_fwd);
  m.def("log_softmax_bwd(Tensor y, Tensor dy, int ldo, bool out_bf16) -> Tensor", &log_softmax_bwd);
  m.def("s2d_weight(Tensor w7, Tensor(a!) w16) -> ()", &s2d_weight);
  m.def("s2d_weight_bwd(Tensor g16, int C) -> Tensor", &s2d_weight_bwd);
  m.def("l2norm_rows(Tensor x, int ldo, float eps, int rows_out=-1) -> (Tensor, Tensor)", &l2norm_rows);
  m.def("l2norm_bwd(Tensor dy, Tensor y, Tensor inv, int D, bool out_bf16) -> Tensor", &l2norm_bwd);
  m.def("transpose2d(Tensor x) -> Tensor", &transpose2d);
  m.def("arcface_l2norm_t(Tensor x, int Rp, int Dp, float eps) -> (Tensor, Tensor, Tensor)", &arcface_l2norm_t);
  m.def("arcface_fused_fwd(Tensor xn, Tensor wn, Tensor labels, int B, int C, float s, float m, bool easy) -> "
        "(Tensor, Tensor, Tensor, Tensor)", &arcface_fused_fwd);
  m.def("arcface_fused_dx(Tensor xn, Tensor wn, Tensor wnT, Tensor labels, Tensor lse, Tensor lab, Tensor grad_out, "
        "float scale, Tensor inv_x, int B, int C, int D, float s, bool out_bf16) -> Tensor", &arcface_fused_dx);
  m.def("arcface_fused_dw(Tensor xn, Tensor xnT, Tensor wn, Tensor labels, Tensor lse, Tensor lab, Tensor grad_out, "
        "float scale, Tensor inv_w, int B, int C, int D, float s) -> Tensor", &arcface_fused_dw);
  m.def(
      "arcface_fwd(Tensor cosv, Tensor labels, int C, float s, float m, bool easy, bool want_logits) -> (Tensor, "
      "Tensor, Tensor, Tensor)",
      &arcface_fwd);
  m.def(
      "arcface_bwd(Tensor cosv, Tensor labels, int C, float s, float m, bool easy, Tensor dphi, Tensor grad_out, "
      "float scale) -> Tensor",
      &arcface_bwd);
  m.def(
      "mt_sgd(Tensor table, Tensor chunks, float lr, float momentum, float dampening, float wd, bool nesterov, bool "
      "first, float grad_scale) -> ()",
      &mt_sgd);
  m.def(
      "mt_adam(Tensor table, Tensor chunks, float lr, float beta1, float beta2, float eps, float wd, int step, bool "
      "decoupled, float grad_scale, Tensor? step_dev=None) -> ()",
      &mt_adam);
  m.def("cdr_threshold(Tensor table, Tensor chunks, Tensor state) -> Tensor", &cdr_threshold);
  m.def("mt_copy(Tensor table, Tensor chunks, float scale, int mode) -> ()", &mt_copy);
  m.def(
      "conv_fwd_affine(Tensor x, Tensor w, int stride, int pad, Tensor scale, Tensor shift, int act, float slope, "
      "Tensor? res) -> Tensor",
      &conv_fwd_affine);
  m.def("act_scale_bwd(Tensor dy, Tensor y, Tensor scale, int act, float slope, bool want_g) -> (Tensor, Tensor)",
        &act_scale_bwd);
  m.def("dropout_fwd(Tensor x, float p, int seed, Tensor(a!) offset) -> (Tensor, Tensor)", &dropout_fwd);
  m.def("iabn_gamma(Tensor g, float eps) -> (Tensor, Tensor)", &iabn_gamma);
  m.def("sign_mul(Tensor d, Tensor g) -> Tensor", &sign_mul);
  m.def("dropout_bwd(Tensor dy, float p, int seed, Tensor used) -> Tensor", &dropout_bwd);
  m.def("adaptive_avg_pool(Tensor x, int OH, int OW) -> Tensor", &adaptive_avg_pool);
  m.def("adaptive_avg_pool_bwd(Tensor dy, int H, int W) -> Tensor", &adaptive_avg_pool_bwd);
  m.def("cdr_mask(Tensor table, Tensor chunks, Tensor state, float clip) -> ()", &cdr_mask);
}
