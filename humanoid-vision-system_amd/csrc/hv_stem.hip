// Direct 3x3 stem convolution (gfx950): the backbone's first ConvMHCLayer conv
// (vision_backbone.py:230, Conv2d(3, 32, 3, stride 2, pad 1) + eval BN + SiLU) straight from the
// NCHW fp32 image.
//
// With 3 input channels the contraction is K = 27: an implicit GEMM spends its time on a
// K-tile that is 58% padding and on the separate NCHW -> NHWC conversion pass (the pair ran at
// 16 TFLOP/s, 0.23 ms at B=16 640^2).  The layer is HBM-bound (78.6 MB image in, 105 MB NHWC
// bf16 out at B=16), so one thread per output pixel computes all COUT channels in fp32
// registers: the 27 input taps are loaded once (rounded to the storage type exactly like the
// conversion pass did), the weights sit k-major in LDS (broadcast reads, one 16-B read per 4
// output channels), and the pixel's COUT outputs leave as whole 16-B stores -- consecutive
// threads write consecutive 64-B pixel rows.  Arithmetic matches the GEMM path term for term
// (bf16 x bf16 products, fp32 sums, acc * scale + bias, activation); only the summation order
// differs.
#include "hv_common.h"

namespace {

template <typename T> __device__ __forceinline__ float stor_round(float v);
template <> __device__ __forceinline__ float stor_round<float>(float v) { return v; }
template <> __device__ __forceinline__ float stor_round<unsigned short>(float v) { return bf2f(f2bf(v)); }

template <typename T> __device__ __forceinline__ void store8(T* p, const float* v);
template <> __device__ __forceinline__ void store8<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <> __device__ __forceinline__ void store8<unsigned short>(unsigned short* p, const float* v) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                            pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}

constexpr int kStemCin = 3, kStemTaps = 9 * kStemCin;

template <typename T, int COUT>
__global__ void __launch_bounds__(256) k_conv_stem(const float* __restrict__ x, int n, int h, int w, int oh,
                                                   int ow, int stride, int pad, const T* __restrict__ wt,
                                                   int ldw, const float* scale, const float* bias, int act,
                                                   T* __restrict__ y) {
  __shared__ float4 ws[kStemTaps][COUT / 4];        // k-major: the COUT weights of tap k
  __shared__ float sc[COUT], bi[COUT];
  for (int i = threadIdx.x; i < kStemTaps * COUT; i += 256) {
    const int co = i / kStemTaps, k = i % kStemTaps;
    reinterpret_cast<float*>(&ws[k][0])[co] = Elem<T>::load(wt, (long)co * ldw + k);
  }
  for (int i = threadIdx.x; i < COUT; i += 256) {
    sc[i] = scale ? scale[i] : 1.f;
    bi[i] = bias ? bias[i] : 0.f;
  }
  __syncthreads();
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)n * oh * ow) return;
  const int ox = p % ow;
  const long q = p / ow;
  const int oy = q % oh;
  const int b = q / oh;
  float in[kStemTaps];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * stride - pad + ky;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * stride - pad + kx;
      const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
#pragma unroll
      for (int ci = 0; ci < kStemCin; ++ci)
        in[(ky * 3 + kx) * kStemCin + ci] =
            ok ? stor_round<T>(x[(((long)b * kStemCin + ci) * h + iy) * w + ix]) : 0.f;
    }
  }
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = 0.f;
#pragma unroll
  for (int k = 0; k < kStemTaps; ++k) {
#pragma unroll
    for (int c4 = 0; c4 < COUT / 4; ++c4) {
      const float4 wv = ws[k][c4];
      acc[4 * c4 + 0] = fmaf(in[k], wv.x, acc[4 * c4 + 0]);
      acc[4 * c4 + 1] = fmaf(in[k], wv.y, acc[4 * c4 + 1]);
      acc[4 * c4 + 2] = fmaf(in[k], wv.z, acc[4 * c4 + 2]);
      acc[4 * c4 + 3] = fmaf(in[k], wv.w, acc[4 * c4 + 3]);
    }
  }
  T* out = y + p * COUT;
#pragma unroll
  for (int c8 = 0; c8 < COUT / 8; ++c8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c8 * 8 + j;
      v[j] = hv_act(acc[c] * sc[c] + bi[c], act);
    }
    store8<T>(out + c8 * 8, v);
  }
}

// ---------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolution with 32 input channels (stem[1] 32->32 and stem[2] 32->64 at
// 320x320, vision_backbone.py:231-232): K = 288 is not a multiple of the LDS-DMA kernels' 64-deep
// k-tile, and the register-staged implicit GEMM re-gathers every input pixel 9 times from L2 with
// a 64-wide N tile of which N = 32 fills half (0.165 ms per launch at B=16, ~1.2 TB/s).
// Here a workgroup owns a 4 x 64 output-pixel tile: its (4+2) x (64+2) x 32-channel input halo is
// loaded ONCE into LDS, the weights live in registers for the whole workgroup (one 16x16x32 A
// fragment per (tap, 16-channel tile): 9 x N/16), and wave w computes output row w as
// D^T[channel][pixel] = W . X^T -- the tap's 32 input channels are exactly one MFMA k-step, the
// B fragment (16 pixels x 8 channels per lane group) is one conflict-free 16-B LDS read shared by
// the N/16 channel tiles, and each lane ends with 4 consecutive output channels of one pixel
// (8-B stores, 64 contiguous bytes per pixel across the 4 lane groups).  Same per-tap k order as
// the GEMM path (kh, kw, c); epilogue = hv_gemm_epi.h's (alpha*scale, bias, act).
using bf = unsigned short;
__device__ __forceinline__ f32x4 mfma_bf16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

constexpr int C3_CIN = 32, C3_TW = 64, C3_TH = 4, C3_HW = C3_TW + 2, C3_HH = C3_TH + 2;

template <int NT>
__global__ void __launch_bounds__(256) k_conv3x3_c32(const hv_gemm_desc d, int tiles_x, int tiles_y) {
  __shared__ __attribute__((aligned(16))) bf halo[C3_HH * C3_HW * C3_CIN];   // 25,344 B
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  // XCD-aware order: the 8 XCDs take contiguous runs of tiles (neighbours share halo rows in L2)
  const int G = gridDim.x;
  int bid = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int H = d.conv_h, W = d.conv_w;
  const int x0 = tx * C3_TW, y0 = ty * C3_TH;
  const bf* X = (const bf*)d.A;
  const bf* Wt = (const bf*)d.B;
  uint4 wf[9][NT];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      wf[t][nt] = *reinterpret_cast<const uint4*>(Wt + (long)(nt * 16 + fr) * d.ldb + t * C3_CIN + g * 8);
  constexpr int CHUNKS = C3_HH * C3_HW * 4;         // 16-B chunks (4 per pixel)
  for (int c = tid; c < CHUNKS; c += 256) {
    const int q = c & 3, pix = c >> 2;
    const int hx = pix % C3_HW, hy = pix / C3_HW;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(X + (((long)b * H + iy) * W + ix) * C3_CIN + q * 8);
    *reinterpret_cast<uint4*>(halo + pix * C3_CIN + q * 8) = v;
  }
  __syncthreads();
  f32x4 acc[4][NT];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[pt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const uint4 bfr = *reinterpret_cast<const uint4*>(halo + ((w + ky) * C3_HW + pt * 16 + fr + kx) * C3_CIN + g * 8);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[pt][nt] = mfma_bf16(wf[ky * 3 + kx][nt], bfr, acc[pt][nt]);
      }
  const int oy = y0 + w;
  if (oy >= H) return;
  const bool gelu_fast = d.act == HV_ACT_GELU;
  float sc[NT][4], bi[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nt * 16 + 4 * g + j;
      sc[nt][j] = d.scale ? d.scale[n] * d.alpha : d.alpha;
      bi[nt][j] = d.bias ? d.bias[n] : 0.f;
    }
  bf* C = (bf*)d.C;
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const int ox = x0 + pt * 16 + fr;
    if (ox >= W) continue;
    const long m = ((long)b * H + oy) * W + ox;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = acc[pt][nt][j] * sc[nt][j] + bi[nt][j];
        v[j] = gelu_fast ? hv_gelu_fast(x) : hv_act(x, d.act);
      }
      *reinterpret_cast<uint2*>(C + m * d.ldc + nt * 16 + 4 * g) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
}

}  // namespace

// hv_gemm's dispatch (hv_gemm.hip) routes eligible convolutions here; HV_EUNSUPPORTED otherwise.
int hv_conv3x3_c32(const hv_gemm_desc& d, hipStream_t s) {
  if (d.dtype != HV_BF16 || d.c_dtype != HV_BF16 || d.conv_k != 3 || d.conv_stride != 1 || d.conv_pad != 1 ||
      d.conv_c != C3_CIN || d.conv_transposed || d.epi_mode || d.residual || d.A2 || d.a_mean)
    return HV_EUNSUPPORTED;
  if ((d.N != 32 && d.N != 64) || d.ldc != d.N || d.ldb % 8 || d.ldb < 9 * C3_CIN ||
      d.conv_oh != d.conv_h || d.conv_ow != d.conv_w || (((uintptr_t)d.A | (uintptr_t)d.B | (uintptr_t)d.C) & 15))
    return HV_EUNSUPPORTED;
  const int tiles_x = hv_cdiv(d.conv_w, C3_TW), tiles_y = hv_cdiv(d.conv_h, C3_TH);
  const long grid = (long)d.conv_n * tiles_x * tiles_y;
  if (grid <= 0 || grid > 0x7fffffffL) return HV_EUNSUPPORTED;
  if (d.N == 32) k_conv3x3_c32<2><<<(unsigned)grid, 256, 0, s>>>(d, tiles_x, tiles_y);
  else k_conv3x3_c32<4><<<(unsigned)grid, 256, 0, s>>>(d, tiles_x, tiles_y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_conv_stem(int dtype, const float* x, int n, int cin, int h, int w, int k, int stride, int pad,
                            const void* wt, int ldw, int cout, const float* scale, const float* bias, int act,
                            void* y, hv_stream_t stream) {
  if (cin != kStemCin || k != 3 || stride < 1 || pad < 0 || n <= 0 || h <= 0 || w <= 0 || ldw < kStemTaps)
    return HV_EUNSUPPORTED;
  if ((cout != 32 && cout != 64) || (((uintptr_t)y) & 15)) return HV_EUNSUPPORTED;
  if (dtype != HV_BF16 && dtype != HV_F32) return HV_EINVAL;
  const int oh = (h + 2 * pad - 3) / stride + 1, ow = (w + 2 * pad - 3) / stride + 1;
  if (oh <= 0 || ow <= 0) return HV_EINVAL;
  const long total = (long)n * oh * ow;
  const unsigned grid = (unsigned)hv_cdiv(total, 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == HV_BF16) {
    if (cout == 32)
      k_conv_stem<unsigned short, 32><<<grid, 256, 0, s>>>(x, n, h, w, oh, ow, stride, pad, (const unsigned short*)wt,
                                                           ldw, scale, bias, act, (unsigned short*)y);
    else
      k_conv_stem<unsigned short, 64><<<grid, 256, 0, s>>>(x, n, h, w, oh, ow, stride, pad, (const unsigned short*)wt,
                                                           ldw, scale, bias, act, (unsigned short*)y);
  } else {
    if (cout == 32)
      k_conv_stem<float, 32><<<grid, 256, 0, s>>>(x, n, h, w, oh, ow, stride, pad, (const float*)wt, ldw, scale,
                                                  bias, act, (float*)y);
    else
      k_conv_stem<float, 64><<<grid, 256, 0, s>>>(x, n, h, w, oh, ow, stride, pad, (const float*)wt, ldw, scale,
                                                  bias, act, (float*)y);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}
