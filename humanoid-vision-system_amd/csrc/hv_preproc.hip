// Image preprocessing on the GPU: ImagePreprocessor.process
// (reference inference/preprocessing.py:181-276: BGR->RGB, bilinear resize to the model size,
// /255, ImageNet mean/std) for a batch of uint8 HWC frames in ONE launch, writing straight into
// the layout and dtype the model consumes (NHWC bf16 for the token path, or NCHW fp32/fp16 like
// the reference's tensor), so the streaming path (config E) needs no host-side conversion.
// Two resize semantics:
//   * hv_preprocess:     torch F.interpolate(mode='bilinear', align_corners=False) -- what the
//                        reference's kornia GPU path (K.Resize bilinear, preprocessing.py:148-152)
//                        computes;
//   * hv_preprocess_pil: the reference's default path when kornia is absent (it is not in
//                        requirements.txt): torchvision Resize on a PIL image = Pillow's
//                        Image.resize(BILINEAR) (Pillow==10.0.0, requirements.txt:6; libImaging
//                        Resample.c, unchanged through 12.x): a separable triangle filter whose
//                        support widens with the downscale factor (antialiasing), 22-bit fixed-point
//                        coefficients, a uint8-rounded horizontal pass then a uint8-rounded vertical
//                        pass -- reproduced bit-exactly (integer arithmetic), then ToTensor (/255)
//                        and Normalize in fp32 exactly as torchvision does ((u / 255 - mean) / std).
#include <math.h>

#include <vector>

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

// ---- Pillow-exact bilinear resample (see the file header).  Table (int32), built on the host by
// hv_pil_resample_tables: [ksh, ksv, hb[2*ow], hk[ow*ksh], vb[2*oh], vk[oh*ksv]].
constexpr int kPilPrec = 22;   // PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int pil_clip8(int v) {
  return v >= (1 << kPilPrec << 8) ? 255 : (v <= 0 ? 0 : (v >> kPilPrec));
}

__global__ void __launch_bounds__(256) k_preprocess_pil(const uint8_t* __restrict__ img, int n, int h, int w,
                                                        int swap_rb, int oh, int ow, const int* __restrict__ tab,
                                                        float m0, float m1, float m2, float s0, float s1, float s2,
                                                        int dt, int nhwc, void* out) {
  const long total = (long)n * oh * ow;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ox = (int)(i % ow);
  const int oy = (int)((i / ow) % oh);
  const int b = (int)(i / ((long)ow * oh));
  const int ksh = tab[0], ksv = tab[1];
  const int* hb = tab + 2;
  const int* hk = hb + 2 * ow;
  const int* vb = hk + (long)ow * ksh;
  const int* vk = vb + 2 * oh;
  const int xmin = hb[2 * ox], xn = hb[2 * ox + 1];
  const int ymin = vb[2 * oy], yn = vb[2 * oy + 1];
  const int* kx = hk + (long)ox * ksh;
  const int* ky = vk + (long)oy * ksv;
  HV_DCHECK(xmin >= 0 && xn <= ksh && xmin + xn <= w && ymin >= 0 && yn <= ksv && ymin + yn <= h);
  const uint8_t* base = img + (long)b * h * w * 3;
  int acc[3] = {1 << (kPilPrec - 1), 1 << (kPilPrec - 1), 1 << (kPilPrec - 1)};
  for (int y = 0; y < yn; ++y) {
    const uint8_t* row = base + ((long)(ymin + y) * w + xmin) * 3;
    int hs[3] = {1 << (kPilPrec - 1), 1 << (kPilPrec - 1), 1 << (kPilPrec - 1)};
    for (int x = 0; x < xn; ++x) {
      const int k = kx[x];
      hs[0] += row[3 * x + 0] * k;
      hs[1] += row[3 * x + 1] * k;
      hs[2] += row[3 * x + 2] * k;
    }
    const int kyv = ky[y];
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += pil_clip8(hs[c]) * kyv;
  }
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int sc = swap_rb ? 2 - c : c;                   // RGB channel c reads BGR slot 2 - c
    const float u = (float)pil_clip8(acc[sc]);
    const float v = __fdiv_rn(__fdiv_rn(u, 255.0f) - mean[c], stdv[c]);   // ToTensor, Normalize (IEEE div)
    const long o = nhwc ? i * 3 + c : (((long)b * 3 + c) * oh + oy) * ow + ox;
    store_one(out, dt, o, v);
  }
}

// Resample.c precompute_coeffs (bilinear filter, support 1) + normalize_coeffs_8bpc, in the same
// double arithmetic; returns the kernel size.
int pil_coeffs(int in_size, int out_size, std::vector<int>& bounds, std::vector<int>& kk) {
  const double in0 = 0.0, in1 = (double)(float)in_size;
  double scale = (in1 - in0) / out_size, filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  bounds.assign(2 * out_size, 0);
  kk.assign((size_t)out_size * ksize, 0);
  std::vector<double> pre(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double wgt = t < 1.0 ? 1.0 - t : 0.0;
      pre[x] = wgt;
      ww += wgt;
    }
    for (int x = 0; x < xmax; ++x) {
      const double k = ww != 0.0 ? pre[x] / ww : pre[x];
      kk[(size_t)xx * ksize + x] = k < 0 ? (int)(-0.5 + k * (1 << kPilPrec)) : (int)(0.5 + k * (1 << kPilPrec));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

}  // namespace

extern "C" size_t hv_pil_table_ints(int in_h, int in_w, int out_h, int out_w) {
  if (in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0) return 0;
  auto ks = [](int in, int out) {
    double f = (double)in / out;
    if (f < 1.0) f = 1.0;
    return (size_t)((int)ceil(f) * 2 + 1);
  };
  return 2 + 2 * (size_t)out_w + (size_t)out_w * ks(in_w, out_w) + 2 * (size_t)out_h + (size_t)out_h * ks(in_h, out_h);
}

extern "C" int hv_pil_resample_tables(int in_h, int in_w, int out_h, int out_w, int* table) {
  if (!table || in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0) return HV_EINVAL;
  std::vector<int> hb, hk, vb, vk;
  const int ksh = pil_coeffs(in_w, out_w, hb, hk);
  const int ksv = pil_coeffs(in_h, out_h, vb, vk);
  int* p = table;
  *p++ = ksh;
  *p++ = ksv;
  for (int v : hb) *p++ = v;
  for (int v : hk) *p++ = v;
  for (int v : vb) *p++ = v;
  for (int v : vk) *p++ = v;
  return HV_OK;
}

extern "C" int hv_preprocess_pil(const uint8_t* img, int n, int h, int w, int swap_rb, int out_h, int out_w,
                                 const int* table_dev, const float* mean_std, int out_dtype, int nhwc, void* out,
                                 hv_stream_t stream) {
  if (!img || !out || !mean_std || !table_dev || n <= 0 || h <= 0 || w <= 0 || out_h <= 0 || out_w <= 0)
    return HV_EINVAL;
  if (out_dtype != HV_F32 && out_dtype != HV_BF16 && out_dtype != HV_F16) return HV_EINVAL;
  const long total = (long)n * out_h * out_w;
  k_preprocess_pil<<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
      img, n, h, w, swap_rb, out_h, out_w, table_dev, mean_std[0], mean_std[1], mean_std[2], mean_std[3], mean_std[4],
      mean_std[5], out_dtype, nhwc, out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

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
