// Image preprocessing on the GPU: ImagePreprocessor.process
// (reference inference/preprocessing.py:181-276: BGR->RGB, bilinear resize to the model size,
// /255, ImageNet mean/std) for a batch of uint8 HWC frames in ONE launch, writing straight into
// the layout and dtype the model consumes (NHWC bf16 for the token path, or NCHW fp32/fp16 like
// the reference's tensor), so the streaming path (config E) needs no host-side conversion.
// Resize = torch F.interpolate(mode='bilinear', align_corners=False) semantics.
#include "hv_common.h"
#include <hip/hip_fp16.h>

namespace {

__device__ __forceinline__ void store_one(void* out, int dt, long i, float v) {
  if (dt == HV_BF16) ((unsigned short*)out)[i] = f2bf(v);
  else if (dt == HV_F16) ((__half*)out)[i] = __float2half(v);
  else ((float*)out)[i] = v;
}

__global__ void __launch_bounds__(256) k_preprocess(const uint8_t* __restrict__ img, int n, int h, int w, int swap_rb,
                                                    int oh, int ow, float m0, float m1, float m2, float s0, float s1,
                                                    float s2, int dt, int nhwc, void* out) {
  const long total = (long)n * oh * ow;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ox = (int)(i % ow);
  const int oy = (int)((i / ow) % oh);
  const int b = (int)(i / ((long)ow * oh));
  const float sy = (float)h / oh, sx = (float)w / ow;
  float fy = fmaxf((oy + 0.5f) * sy - 0.5f, 0.f), fx = fmaxf((ox + 0.5f) * sx - 0.5f, 0.f);
  const int y0 = min((int)fy, h - 1), x0 = min((int)fx, w - 1);
  const int y1 = min(y0 + 1, h - 1), x1 = min(x0 + 1, w - 1);
  const float ly = fy - y0, lx = fx - x0;
  const uint8_t* base = img + (long)b * h * w * 3;
  const uint8_t* p00 = base + ((long)y0 * w + x0) * 3;
  const uint8_t* p01 = base + ((long)y0 * w + x1) * 3;
  const uint8_t* p10 = base + ((long)y1 * w + x0) * 3;
  const uint8_t* p11 = base + ((long)y1 * w + x1) * 3;
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int sc = swap_rb ? 2 - c : c;                   // output channel c (RGB) reads BGR slot 2-c
    const float top = (1.f - lx) * (p00[sc] * (1.f / 255.f)) + lx * (p01[sc] * (1.f / 255.f));
    const float bot = (1.f - lx) * (p10[sc] * (1.f / 255.f)) + lx * (p11[sc] * (1.f / 255.f));
    const float v = ((1.f - ly) * top + ly * bot - mean[c]) / stdv[c];
    const long o = nhwc ? i * 3 + c : (((long)b * 3 + c) * oh + oy) * ow + ox;
    store_one(out, dt, o, v);
  }
}

}  // namespace

extern "C" int hv_preprocess(const uint8_t* img, int n, int h, int w, int swap_rb, int out_h, int out_w,
                             const float* mean_std /* host [6]: mean rgb, std rgb */, int out_dtype, int nhwc,
                             void* out, hv_stream_t stream) {
  if (!img || !out || !mean_std || n <= 0 || h <= 0 || w <= 0 || out_h <= 0 || out_w <= 0) return HV_EINVAL;
  if (out_dtype != HV_F32 && out_dtype != HV_BF16 && out_dtype != HV_F16) return HV_EINVAL;
  const long total = (long)n * out_h * out_w;
  k_preprocess<<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
      img, n, h, w, swap_rb, out_h, out_w, mean_std[0], mean_std[1], mean_std[2], mean_std[3], mean_std[4], mean_std[5],
      out_dtype, nhwc, out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
