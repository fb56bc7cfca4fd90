// Direct 3x3 stem convolution (gfx950): the backbone's first ConvMHCLayer conv
// (vision_backbone.py:230, Conv2d(3, 32, 3, stride 2, pad 1) + eval BN + SiLU) straight from the
// NCHW fp32 image.
//
// With 3 input channels the contraction is K = 27: an implicit GEMM spends its time on a
// K-tile that is 58% padding and on the separate NCHW -> NHWC conversion pass (the pair ran at
// 16 TFLOP/s, 0.23 ms at B=16 640^2).  The layer is HBM-bound (78.6 MB image in, 105 MB NHWC
// bf16 out at B=16): the 27 input taps of a pixel are loaded once per lane (rounded to the
// storage type exactly like the conversion pass did), weights live in registers, and the
// pixel's COUT outputs leave as one contiguous run.  Arithmetic matches the GEMM path term for term
// (bf16 x bf16 products, fp32 sums, acc * scale + bias, activation); only the summation order
// differs.
#include <type_traits>

#include "hv_common.h"

namespace {

template <typename T> __device__ __forceinline__ float stor_round(float v);
template <> __device__ __forceinline__ float stor_round<float>(float v) { return v; }
template <> __device__ __forceinline__ float stor_round<unsigned short>(float v) { return bf2f(f2bf(v)); }

constexpr int kStemCin = 3, kStemTaps = 9 * kStemCin;

// x: NCHW fp32 (TI = float, NHWC = false; rounded to T on load) or NHWC T (the engine's
// preprocessed input) -- both layouts give the same values, hence the same outputs.
// Work split: COUT/4 adjacent lanes share an output pixel, each owning 4 output channels whose
// 27 x 4 weights stay in registers for the whole (grid-stride) walk over pixels; the lanes of a
// pixel load the same 27 taps (one coalesced address per pixel) and together store the pixel's
// COUT outputs as one contiguous run.  (One thread per pixel with all COUT channels made the
// compiler hoist every weight read of the unrolled tap loop: 512 VGPRs + scratch, 1.9 ms at
// B=16.)
template <typename T> __device__ __forceinline__ void store4(T* p, const float* v);
template <> __device__ __forceinline__ void store4<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void store4<unsigned short>(unsigned short* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

template <typename T, int COUT, typename TI, bool NHWC>
__global__ void __launch_bounds__(256) k_conv_stem(const TI* __restrict__ x, int n, int h, int w, int oh,
                                                   int ow, int stride, int pad, const T* __restrict__ wt,
                                                   int ldw, const float* scale, const float* bias, int act,
                                                   T* __restrict__ y) {
  constexpr int Q = COUT / 4, PPB = 256 / Q;           // lanes per pixel, pixels per block step
  const int q = threadIdx.x % Q;
  float4 wr[kStemTaps];
#pragma unroll
  for (int k = 0; k < kStemTaps; ++k)
    wr[k] = make_float4(Elem<T>::load(wt, (long)(4 * q + 0) * ldw + k), Elem<T>::load(wt, (long)(4 * q + 1) * ldw + k),
                        Elem<T>::load(wt, (long)(4 * q + 2) * ldw + k), Elem<T>::load(wt, (long)(4 * q + 3) * ldw + k));
  float sc[4], bi[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sc[j] = scale ? scale[4 * q + j] : 1.f;
    bi[j] = bias ? bias[4 * q + j] : 0.f;
  }
  const long npix = (long)n * oh * ow;
  for (long p = (long)blockIdx.x * PPB + threadIdx.x / Q; p < npix; p += (long)gridDim.x * PPB) {
    const int ox = p % ow;
    const long qq = p / ow;
    const int oy = qq % oh;
    const int b = qq / oh;
    float in[kStemTaps];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * stride - pad + ky;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * stride - pad + kx;
        const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
#pragma unroll
        for (int ci = 0; ci < kStemCin; ++ci) {
          float v = 0.f;
          if (ok) {
            if constexpr (NHWC) v = Elem<TI>::load(x, (((long)b * h + iy) * w + ix) * kStemCin + ci);
            else v = stor_round<T>(x[(((long)b * kStemCin + ci) * h + iy) * w + ix]);
          }
          in[(ky * 3 + kx) * kStemCin + ci] = v;
        }
      }
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kStemTaps; ++k) {
      acc[0] = fmaf(in[k], wr[k].x, acc[0]);
      acc[1] = fmaf(in[k], wr[k].y, acc[1]);
      acc[2] = fmaf(in[k], wr[k].z, acc[2]);
      acc[3] = fmaf(in[k], wr[k].w, acc[3]);
    }
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = hv_act(acc[j] * sc[j] + bi[j], act);
    store4<T>(y + p * COUT + 4 * q, v);
  }
}

// ---------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolution with 32 input channels (stem[1] 32->32 and stem[2] 32->64 at
// 320x320, vision_backbone.py:231-232): K = 288 is not a multiple of the LDS-DMA kernels' 64-deep
// k-tile, and the register-staged implicit GEMM re-gathers every input pixel 9 times from L2 with
// a 64-wide N tile of which N = 32 fills half (0.165 ms per launch at B=16, ~1.2 TB/s).
// Here a workgroup owns a 4 x 64 output-pixel tile: its (4+2) x (64+2) x 32-channel input halo is
// loaded ONCE into LDS, the weights live in registers for the whole workgroup (one 16x16x32 A
// fragment per (tap, 16-channel tile): 9 x 2 per wave), and wave w of a group computes row w as
// D^T[channel][pixel] = W . X^T -- the tap's 32 input channels are exactly one MFMA k-step, the
// B fragment (16 pixels x 8 channels per lane group) is one conflict-free 16-B LDS read shared by
// the N/16 channel tiles (conflict-free through the chunk swizzle below), and each lane ends with 4 consecutive output channels of one pixel
// (8-B stores, 64 contiguous bytes per pixel across the 4 lane groups).  Same per-tap k order as
// the GEMM path (kh, kw, c); epilogue = hv_gemm_epi.h's (alpha*scale, bias, act).
using bf = unsigned short;
__device__ __forceinline__ f32x4 mfma_bf16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

constexpr int C3_CIN = 32, C3_TW = 64, C3_TH = 4, C3_HW = C3_TW + 2, C3_HH = C3_TH + 2;

// 16-B chunk q of halo pixel p lives at chunk q ^ (2 * ((p >> 2) & 1)): a B-fragment read
// (ds_read_b128, 16-lane groups of pixels p..p+15 with chunk g for lanes 0-3 / 12-15 and g+1 for
// 4-11, or the reverse) then hits 16 distinct 4-bank sets.  Unswizzled, pixels p and p+4 share
// banks (64 B per pixel): 2-way on every read (SQ_LDS_BANK_CONFLICT 0.46 of the LDS cycles).
__device__ __forceinline__ int c3_chunk(int pix, int q) { return q ^ (((pix >> 2) & 1) << 1); }

// NT = N/16 channel tiles; the workgroup has NT/2 groups of 4 waves, group h computing channel
// tiles 2h, 2h+1 (so a wave holds 18 weight fragments + 8 accumulators at any N: 128 VGPRs)
template <int NT>
__global__ void __launch_bounds__(128 * NT) k_conv3x3_c32(const hv_gemm_desc d, int tiles_x, int tiles_y) {
  __shared__ __attribute__((aligned(16))) bf halo[C3_HH * C3_HW * C3_CIN];   // 25,344 B
  const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 3, hgrp = tid >> 8;
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
  uint4 wf[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      wf[t][nt] = *reinterpret_cast<const uint4*>(Wt + (long)((2 * hgrp + nt) * 16 + fr) * d.ldb + t * C3_CIN + g * 8);
  constexpr int CHUNKS = C3_HH * C3_HW * 4;         // 16-B chunks (4 per pixel)
  for (int c = tid; c < CHUNKS; c += 128 * NT) {
    const int q = c & 3, pix = c >> 2;
    const int hx = pix % C3_HW, hy = pix / C3_HW;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint4*>(X + (((long)b * H + iy) * W + ix) * C3_CIN + q * 8);
    *reinterpret_cast<uint4*>(halo + pix * C3_CIN + c3_chunk(pix, q) * 8) = v;
  }
  __syncthreads();
  f32x4 acc[4][2];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[pt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int pix = (w + ky) * C3_HW + pt * 16 + fr + kx;
        const uint4 bfr = *reinterpret_cast<const uint4*>(halo + pix * C3_CIN + c3_chunk(pix, g) * 8);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[pt][nt] = mfma_bf16(wf[ky * 3 + kx][nt], bfr, acc[pt][nt]);
      }
  const int oy = y0 + w;
  if (oy >= H) return;
  const bool gelu_fast = d.act == HV_ACT_GELU;
  float sc[2][4], bi[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = (2 * hgrp + nt) * 16 + 4 * g + j;
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
    for (int nt = 0; nt < 2; ++nt) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = acc[pt][nt][j] * sc[nt][j] + bi[nt][j];
        v[j] = gelu_fast ? hv_gelu_fast(x) : hv_act(x, d.act);
      }
      *reinterpret_cast<uint2*>(C + m * d.ldc + (2 * hgrp + nt) * 16 + 4 * g) =
          make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
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
  else k_conv3x3_c32<4><<<(unsigned)grid, 512, 0, s>>>(d, tiles_x, tiles_y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

namespace {

// bf16 stem on the matrix cores: the workgroup stages the input rows of a TOH x 64 output-pixel
// tile ((TOH-1)*s+3 rows x (64-1)*s+3 columns x 3 channels, rounded to bf16) in LDS with
// coalesced row loads, then each wave runs the whole 27(->32)-deep contraction of 16 pixels x
// 16 channels as ONE 16x16x32 MFMA: the B fragment is the pixel's 8 taps k = 8g..8g+7 (k order
// kh, kw, cin as the weights; k >= 27 zero) gathered from LDS through a per-lane offset table,
// the A fragments (weights) stay in registers.  Same instruction, operands and k order as the
// implicit-GEMM path's single K-step, so the outputs match it; the NHWC and NCHW inputs give
// the same values.  Lane (pixel fr, group g) ends with 4 consecutive channels -> 8-B stores.
// TOH output rows per workgroup: 8 for big batches (the stride-2 window re-reads 1/8 of its
// rows instead of 1/2 at 2 rows), 2 when 8 would leave CUs idle (B=1: 200 workgroups)
constexpr int STM_TOW = 64, STM_IW = (STM_TOW - 1) * 2 + 3;   // stride <= 2

template <int COUT, typename TI, bool NHWC, int STM_TOH>
__global__ void __launch_bounds__(256) k_conv_stem_mfma(const TI* __restrict__ x, int n, int h, int w, int oh,
                                                        int ow, int stride, int pad, const unsigned short* __restrict__ wt,
                                                        int ldw, const float* scale, const float* bias, int act,
                                                        unsigned short* __restrict__ y, int tiles_x, int tiles_y) {
  constexpr int NT = COUT / 16, STM_IH = (STM_TOH - 1) * 2 + 3;
  __shared__ float xs[kStemCin][STM_IH][STM_IW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * STM_TOH, ox0 = tx * STM_TOW;
  const int iy0 = oy0 * stride - pad, ix0 = ox0 * stride - pad;
  const int rows = (STM_TOH - 1) * stride + 3, cols = (STM_TOW - 1) * stride + 3;
  // stage the input tile (rounded to bf16 exactly as the NHWC conversion pass stores it)
  if constexpr (NHWC) {
    for (int i = tid; i < rows * cols * kStemCin; i += 256) {
      const int ci = i % kStemCin, rc = i / kStemCin, c = rc % cols, r = rc / cols;
      const int iy = iy0 + r, ix = ix0 + c;
      float v = 0.f;
      if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = Elem<TI>::load(x, (((long)b * h + iy) * w + ix) * kStemCin + ci);
      xs[ci][r][c] = v;
    }
  } else {
    for (int i = tid; i < kStemCin * rows * cols; i += 256) {
      const int c = i % cols, rr = i / cols, r = rr % rows, ci = rr / rows;
      const int iy = iy0 + r, ix = ix0 + c;
      float v = 0.f;
      if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = bf2f(f2bf(x[(((long)b * kStemCin + ci) * h + iy) * w + ix]));
      xs[ci][r][c] = v;
    }
  }
  // weights (A operand): channel tile nt, row fr, k = 8g .. 8g+7
  uint4 wf[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    unsigned short e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * g + j;
      e[j] = k < kStemTaps ? wt[(long)(nt * 16 + fr) * ldw + k] : (unsigned short)0;
    }
    wf[nt] = make_uint4(e[0] | (unsigned)e[1] << 16, e[2] | (unsigned)e[3] << 16, e[4] | (unsigned)e[5] << 16,
                        e[6] | (unsigned)e[7] << 16);
  }
  // this lane's 8 taps as LDS offsets relative to the pixel's window origin (-1: zero pad of k)
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j;
    const int tap = k / kStemCin, ci = k % kStemCin;
    off[j] = k < kStemTaps ? (ci * STM_IH + tap / 3) * STM_IW + tap % 3 : -1;
  }
  float sc[NT][4], bi[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = nt * 16 + 4 * g + j;
      sc[nt][j] = scale ? scale[c] : 1.f;
      bi[nt][j] = bias ? bias[c] : 0.f;
    }
  __syncthreads();
  const float* xf = &xs[0][0][0];
  // STM_TOH * 64 pixels = groups of 16; wave wv takes groups wv, wv + 4, ...
#pragma unroll 2
  for (int q = 0; q < STM_TOH * STM_TOW / 64; ++q) {
    const int p = (wv + 4 * q) * 16 + fr;             // pixel within the tile (B column = fr)
    const int py = p / STM_TOW, px = p % STM_TOW;
    const int base = py * stride * STM_IW + px * stride;
    float v8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v8[j] = off[j] >= 0 ? xf[base + off[j]] : 0.f;
    const uint4 xb = make_uint4(pack_bf16x2(v8[0], v8[1]), pack_bf16x2(v8[2], v8[3]), pack_bf16x2(v8[4], v8[5]),
                                pack_bf16x2(v8[6], v8[7]));
    const int oy = oy0 + py, ox = ox0 + px;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[nt]),
                                                                __builtin_bit_cast(bf16x8, xb),
                                                                f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if (oy < oh && ox < ow) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = hv_act(acc[j] * sc[nt][j] + bi[nt][j], act);
        *reinterpret_cast<uint2*>(y + (((long)b * oh + oy) * ow + ox) * COUT + nt * 16 + 4 * g) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  }
}

}  // namespace

template <typename T, int COUT>
void launch_stem(const void* x, int x_nhwc, int n, int h, int w, int oh, int ow, int stride, int pad, const void* wt,
                 int ldw, const float* scale, const float* bias, int act, void* y, unsigned grid, hipStream_t s) {
  if constexpr (std::is_same<T, unsigned short>::value) {
    if (stride <= 2) {                                  // the MFMA kernel (bf16)
      const int tiles_x = hv_cdiv(ow, STM_TOW);
      const bool tall = (long)n * tiles_x * hv_cdiv(oh, 8) >= 1024;
      const int tiles_y = hv_cdiv(oh, tall ? 8 : 2);
      const unsigned g2 = (unsigned)((long)n * tiles_x * tiles_y);
      auto us = (const unsigned short*)wt;
      auto yo = (unsigned short*)y;
      if (x_nhwc) {
        auto xi = (const unsigned short*)x;
        if (tall) k_conv_stem_mfma<COUT, unsigned short, true, 8><<<g2, 256, 0, s>>>(xi, n, h, w, oh, ow, stride, pad, us, ldw, scale, bias, act, yo, tiles_x, tiles_y);
        else k_conv_stem_mfma<COUT, unsigned short, true, 2><<<g2, 256, 0, s>>>(xi, n, h, w, oh, ow, stride, pad, us, ldw, scale, bias, act, yo, tiles_x, tiles_y);
      } else {
        auto xi = (const float*)x;
        if (tall) k_conv_stem_mfma<COUT, float, false, 8><<<g2, 256, 0, s>>>(xi, n, h, w, oh, ow, stride, pad, us, ldw, scale, bias, act, yo, tiles_x, tiles_y);
        else k_conv_stem_mfma<COUT, float, false, 2><<<g2, 256, 0, s>>>(xi, n, h, w, oh, ow, stride, pad, us, ldw, scale, bias, act, yo, tiles_x, tiles_y);
      }
      return;
    }
  }
  if (x_nhwc)
    k_conv_stem<T, COUT, T, true><<<grid, 256, 0, s>>>((const T*)x, n, h, w, oh, ow, stride, pad, (const T*)wt, ldw,
                                                      scale, bias, act, (T*)y);
  else
    k_conv_stem<T, COUT, float, false><<<grid, 256, 0, s>>>((const float*)x, n, h, w, oh, ow, stride, pad,
                                                           (const T*)wt, ldw, scale, bias, act, (T*)y);
}

extern "C" int hv_conv_stem(int dtype, const void* x, int x_nhwc, int n, int cin, int h, int w, int k, int stride,
                            int pad, const void* wt, int ldw, int cout, const float* scale, const float* bias,
                            int act, void* y, hv_stream_t stream) {
  if (cin != kStemCin || k != 3 || stride < 1 || pad < 0 || n <= 0 || h <= 0 || w <= 0 || ldw < kStemTaps)
    return HV_EUNSUPPORTED;
  if ((cout != 32 && cout != 64) || (((uintptr_t)y) & 15)) return HV_EUNSUPPORTED;
  if (dtype != HV_BF16 && dtype != HV_F32) return HV_EINVAL;
  const int oh = (h + 2 * pad - 3) / stride + 1, ow = (w + 2 * pad - 3) / stride + 1;
  if (oh <= 0 || ow <= 0) return HV_EINVAL;
  const long total = (long)n * oh * ow;
  const long per = 256 / (cout / 4);                    // pixels per block step
  const long want = (total + per - 1) / per;
  const unsigned grid = (unsigned)(want < 2048 ? want : 2048);   // grid-stride: ~8 blocks per CU
  hipStream_t s = (hipStream_t)stream;
  if (dtype == HV_BF16) {
    if (cout == 32) launch_stem<unsigned short, 32>(x, x_nhwc, n, h, w, oh, ow, stride, pad, wt, ldw, scale, bias, act, y, grid, s);
    else launch_stem<unsigned short, 64>(x, x_nhwc, n, h, w, oh, ow, stride, pad, wt, ldw, scale, bias, act, y, grid, s);
  } else {
    if (cout == 32) launch_stem<float, 32>(x, x_nhwc, n, h, w, oh, ow, stride, pad, wt, ldw, scale, bias, act, y, grid, s);
    else launch_stem<float, 64>(x, x_nhwc, n, h, w, oh, ow, stride, pad, wt, ldw, scale, bias, act, y, grid, s);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}
