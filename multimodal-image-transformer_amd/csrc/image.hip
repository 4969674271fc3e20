// Image normalisation for the data path: the rescale + normalise +
// HWC -> CHW stage of the HF image processors the reference feeds its encoder with
// (dataset.py:135 and model.py:192 via AutoImageProcessor; ViT: rescale 1/255, mean = std = 0.5,
// tf/models/vit/image_processing_vit.py; CLIP: OPENAI_CLIP mean/std, tf/utils/constants.py:5-6).
// The resampling (PIL bilinear / bicubic resize, centre crop) stays on the host where the
// reference does it, so the uint8 pixels entering this kernel are the reference's own.
//
//   dst[b, c, y, x] = ((float)src[b, y, x, c] / 255 - mean[c]) / std[c]
//
// in the same fp32 operation order as the processors' numpy code (correctly rounded divisions:
// bit-identical to the processor's pixel_values). Pure byte streaming, HBM-bound: each thread
// moves 4 pixels (12 B in, 3 x 16 B out, one 16-B store per channel plane).
#include <algorithm>

#include "common.h"

namespace {

__global__ __launch_bounds__(256) void normalize_u8_kernel(long npix4, long hw, const uint8_t* __restrict__ src,
                                                          float* __restrict__ dst, float m0, float m1, float m2,
                                                          float s0, float s1, float s2) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < npix4; i += (long)gridDim.x * blockDim.x) {
  const long p = i * 4;                // 4-pixel group i: first pixel (global index over B*H*W)
  const long b = p / hw, q = p - b * hw;  // hw % 4 == 0: a group never straddles two images
  const uint32_t* s4 = (const uint32_t*)(src + p * 3);
  const uint32_t w0 = s4[0], w1 = s4[1], w2 = s4[2];
  const uint8_t px[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                          (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                          (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
  float* o = dst + b * 3 * hw + q;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    f32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ((float)px[3 * k + c] / 255.0f - mean[c]) / stdv[c];
    *(f32x4*)(o + c * hw) = v;
  }
  }
}

}  // namespace

extern "C" int mit_image_normalize(long B, long H, long W, const uint8_t* src, float* dst, const float* mean3,
                                   const float* std3, void* stream) {
  MIT_CHECK_ARG(mean3 && std3, "mit_image_normalize: null mean/std");
  MIT_RECORD([=, m0 = mean3[0], m1 = mean3[1], m2 = mean3[2], s0 = std3[0], s1 = std3[1], s2 = std3[2]]() {
    const float m[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
    return mit_image_normalize(B, H, W, src, dst, m, sd, stream);
  });
  MIT_CHECK_ARG(src && dst && mean3 && std3, "mit_image_normalize: null pointer");
  MIT_CHECK_ARG(B >= 0 && H > 0 && W > 0, "mit_image_normalize: bad extent");
  MIT_CHECK_ARG((H * W) % 4 == 0, "mit_image_normalize: H*W must be a multiple of 4");
  MIT_CHECK_ARG(((uintptr_t)src % 4) == 0 && ((uintptr_t)dst % 16) == 0,
                "mit_image_normalize: src 4-B / dst 16-B alignment");
  const long npix4 = B * H * W / 4;
  if (npix4 == 0) return MIT_OK;
  const unsigned grid = (unsigned)std::min<long>((npix4 + 255) / 256, 16384);
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, npix4, H * W, src,
                     dst, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  MIT_LAUNCH_CHECK("mit_image_normalize");
  return MIT_OK;
}
