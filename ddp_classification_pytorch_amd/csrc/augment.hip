// On-device augmentation for the native shard loader (csrc/host/loader.cpp, data/shards.py).
//
// crop_resize: for every image b of a gathered batch of raw uint8 HWC records (variable size,
// record b at meta[b][0] bytes into `src`), resample the crop box (y0, x0, h, w) to Ho x Wo with
// bilinear interpolation (half-pixel centres, edge clamp: F.interpolate(mode="bilinear",
// align_corners=False) on the crop) and optionally mirror it horizontally.  This is the tensor
// half of torchvision's RandomResizedCrop + RandomHorizontalFlip / Resize + CenterCrop
// (BASELINE/main.py:58-76, CDR/main.py:112-130, NESTED/train.py:40-65); the host thread pool only
// samples the boxes and gathers bytes.  The uint8 output feeds the to_nhwc / to_nhwc_s2d
// normalisation kernels (misc.hip).
//
// One thread per output pixel; the 4 source taps x 3 channels are byte loads from L2-resident
// records (a 256x256 record is 192 KB), the output is written as 3 bytes per lane (contiguous per
// wave).  The pass moves ~150 KB per 224x224 image: a few microseconds per 1k-image batch.
#include <cstdint>
#include <cstdio>

#include "common.cuh"
#include "launchers.h"

namespace dcp {

__global__ void __launch_bounds__(256) crop_resize_kernel(const uint8_t* __restrict__ src,
                                                          const int64_t* __restrict__ meta, int B, int Ho, int Wo,
                                                          uint8_t* __restrict__ out) {
  const uint32_t per = (uint32_t)Ho * Wo;
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= per * (uint32_t)B) return;
  const uint32_t b = p / per, r = p - b * per;
  const int oy = r / Wo, ox0 = r - oy * Wo;
  const int64_t* m = meta + (size_t)b * 8;
  const uint8_t* img = src + m[0];
  const int W = (int)m[2];
  const int cy = (int)m[3], cx = (int)m[4], ch = (int)m[5], cw = (int)m[6];
  const int ox = m[7] ? Wo - 1 - ox0 : ox0;
  // F.interpolate(bilinear, align_corners=False): src = (dst + 0.5) * in/out - 0.5, clamped at 0
  float sy = fmaxf(((float)oy + 0.5f) * ((float)ch / (float)Ho) - 0.5f, 0.f);
  float sx = fmaxf(((float)ox + 0.5f) * ((float)cw / (float)Wo) - 0.5f, 0.f);
  int y0 = min((int)sy, ch - 1), x0 = min((int)sx, cw - 1);
  const float ly = sy - (float)y0, lx = sx - (float)x0;
  const int y1 = min(y0 + 1, ch - 1), x1 = min(x0 + 1, cw - 1);
  const uint8_t* r0 = img + ((size_t)(cy + y0) * W + cx) * 3;
  const uint8_t* r1 = img + ((size_t)(cy + y1) * W + cx) * 3;
  uint8_t* o = out + (size_t)p * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float a = (float)r0[x0 * 3 + c], bb = (float)r0[x1 * 3 + c];
    const float cc = (float)r1[x0 * 3 + c], d = (float)r1[x1 * 3 + c];
    const float top = a + (bb - a) * lx, bot = cc + (d - cc) * lx;
    const float v = top + (bot - top) * ly;
    o[c] = (uint8_t)fminf(fmaxf(floorf(v + 0.5f), 0.f), 255.f);
  }
}

void launch_crop_resize(const uint8_t* src, const int64_t* meta, int B, int Ho, int Wo, uint8_t* out,
                        hipStream_t s) {
  const size_t total = (size_t)B * Ho * Wo;
  if (total == 0) return;
  if (total >= (1ull << 32)) {
    fprintf(stderr, "crop_resize: %zu output pixels exceed the 32-bit index range\n", total);
    abort();
  }
  hipLaunchKernelGGL(crop_resize_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, meta, B, Ho, Wo,
                     out);
}

}  // namespace dcp
