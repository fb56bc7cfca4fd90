// Normalisation, layout, pointwise, attention and decode kernels of the HybridVision path
// (gfx950).  All activations are token-major (NHWC / [tokens, channels]); T is the storage
// type (float or bf16 bits), arithmetic is fp32.
#include "hv_common.h"

#include <cstring>

namespace {

using bf = unsigned short;

// ---------------------------------------------------------------- row statistics / norms
// One wave per row; two-pass mean / variance from the row held in L1.
template <typename T>
__global__ void __launch_bounds__(256) k_row_stats(const T* __restrict__ x, long ldx, int rows,
                                                   int cols, float eps, float* mean, float* rstd) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const T* p = x + (long)r * ldx;
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) s += Elem<T>::load(p, j);
  const float mu = wave_sum(s) / cols;
  float v = 0.f;
  for (int j = lane; j < cols; j += 64) { const float d = Elem<T>::load(p, j) - mu; v += d * d; }
  v = wave_sum(v) / cols;
  if (lane == 0) { mean[r] = mu; rstd[r] = rsqrtf(v + eps); }
}

template <typename TX, typename TY>
__global__ void __launch_bounds__(256) k_layernorm(const TX* __restrict__ x, int rows, int cols,
                                                   float eps, const float* gamma, const float* beta,
                                                   TY* y, const void* res, int res_dt) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const TX* p = x + (long)r * cols;
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) s += Elem<TX>::load(p, j);
  const float mu = wave_sum(s) / cols;
  float v = 0.f;
  for (int j = lane; j < cols; j += 64) { const float d = Elem<TX>::load(p, j) - mu; v += d * d; }
  const float rs = rsqrtf(wave_sum(v) / cols + eps);
  TY* q = y + (long)r * cols;
  for (int j = lane; j < cols; j += 64) {
    float o = (Elem<TX>::load(p, j) - mu) * rs;
    if (gamma) o = o * gamma[j] + beta[j];
    if (res) o += res_dt == HV_BF16 ? bf2f(((const bf*)res)[(long)r * cols + j])
                                    : ((const float*)res)[(long)r * cols + j];
    Elem<TY>::store(q, j, o);
  }
}

// ---- vectorised row kernels: G lanes per row (power of two <= 64), each lane NP vectors of 8
// elements (one 16-B bf16 load or two 16-B fp32 loads), the row held in registers between the
// mean and variance passes.  Used when cols % 8 == 0 and the rows are 16-B aligned.
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <> struct Vec8<unsigned short> {
  static __device__ __forceinline__ void load(const unsigned short* p, float (&v)[8]) {
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __uint_as_float(w[q] << 16);
      v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(unsigned short* p, const float (&v)[8]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                              pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  }
};

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// mean / rstd of the row held by this lane group (NP x 8 values per lane, `ok` masks the tail)
template <int G, int NP>
__device__ __forceinline__ void group_stats(const float (&x)[NP][8], const bool (&ok)[NP], int cols, float eps,
                                            float& mu, float& rs) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q)
    if (ok[q])
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[q][j];
  mu = group_sum<G>(s) / cols;
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q)
    if (ok[q])
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = x[q][j] - mu; v += d * d; }
  rs = rsqrtf(group_sum<G>(v) / cols + eps);
}

template <typename T, int G, int NP>
__global__ void __launch_bounds__(256) k_row_stats_v(const T* __restrict__ x, long ldx, int rows, int cols,
                                                     float eps, float* mean, float* rstd) {
  const int r = blockIdx.x * (256 / G) + threadIdx.x / G, l = threadIdx.x % G;
  if (r >= rows) return;
  const T* p = x + (long)r * ldx;
  float v[NP][8];
  bool ok[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int c0 = (q * G + l) * 8;
    ok[q] = c0 < cols;
    if (ok[q]) Vec8<T>::load(p + c0, v[q]);
  }
  float mu, rs;
  group_stats<G, NP>(v, ok, cols, eps, mu, rs);
  if (l == 0) { mean[r] = mu; rstd[r] = rs; }
}

template <typename TX, typename TY, int G, int NP>
__global__ void __launch_bounds__(256) k_layernorm_v(const TX* __restrict__ x, int rows, int cols, float eps,
                                                     const float* gamma, const float* beta, TY* y, const void* res,
                                                     int res_dt) {
  const int r = blockIdx.x * (256 / G) + threadIdx.x / G, l = threadIdx.x % G;
  if (r >= rows) return;
  const TX* p = x + (long)r * cols;
  float v[NP][8];
  bool ok[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int c0 = (q * G + l) * 8;
    ok[q] = c0 < cols;
    if (ok[q]) Vec8<TX>::load(p + c0, v[q]);
  }
  // gamma / beta / residual of a short row (NP <= 2) loaded with x, so their latency hides under
  // the statistics instead of following them; longer rows load them per part (registers)
  constexpr bool PRE = NP <= 2;
  float gp[PRE ? NP : 1][8], bp[PRE ? NP : 1][8], rp[PRE ? NP : 1][8];
  if constexpr (PRE) {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (!ok[q]) continue;
      const int c0 = (q * G + l) * 8;
      if (gamma) { Vec8<float>::load(gamma + c0, gp[q]); Vec8<float>::load(beta + c0, bp[q]); }
      if (res) {
        if (res_dt == HV_BF16) Vec8<unsigned short>::load((const unsigned short*)res + (long)r * cols + c0, rp[q]);
        else Vec8<float>::load((const float*)res + (long)r * cols + c0, rp[q]);
      }
    }
  }
  float mu, rs;
  group_stats<G, NP>(v, ok, cols, eps, mu, rs);
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    if (!ok[q]) continue;
    const int c0 = (q * G + l) * 8;
    float o[8], g[8], b[8], rv[8];
    if constexpr (PRE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { g[j] = gp[q][j]; b[j] = bp[q][j]; rv[j] = rp[q][j]; }
    } else {
      if (gamma) { Vec8<float>::load(gamma + c0, g); Vec8<float>::load(beta + c0, b); }
      if (res) {
        if (res_dt == HV_BF16) Vec8<unsigned short>::load((const unsigned short*)res + (long)r * cols + c0, rv);
        else Vec8<float>::load((const float*)res + (long)r * cols + c0, rv);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (v[q][j] - mu) * rs;
      if (gamma) o[j] = o[j] * g[j] + b[j];
      if (res) o[j] += rv[j];
    }
    Vec8<TY>::store(y + (long)r * cols + c0, o);
  }
}

// (G, NP) for a row of `cols` (cols % 8 == 0, cols <= 4096)
static inline void row_shape(int cols, int& G, int& NP) {
  const int nv = cols / 8;
  G = 8;
  while (G < nv && G < 64) G <<= 1;
  NP = 1;
  while (NP * G < nv) NP <<= 1;
}

#define HV_ROW_SHAPES(G, NP, CALL)                                                     \
  switch (G * 16 + NP) {                                                               \
    case 8 * 16 + 1: { constexpr int G_ = 8, NP_ = 1; CALL; } break;                   \
    case 16 * 16 + 1: { constexpr int G_ = 16, NP_ = 1; CALL; } break;                 \
    case 32 * 16 + 1: { constexpr int G_ = 32, NP_ = 1; CALL; } break;                 \
    case 64 * 16 + 1: { constexpr int G_ = 64, NP_ = 1; CALL; } break;                 \
    case 64 * 16 + 2: { constexpr int G_ = 64, NP_ = 2; CALL; } break;                 \
    case 64 * 16 + 4: { constexpr int G_ = 64, NP_ = 4; CALL; } break;                 \
    case 64 * 16 + 8: { constexpr int G_ = 64, NP_ = 8; CALL; } break;                 \
    default: return HV_EUNSUPPORTED;                                                   \
  }

// out = x * gate[b, c] (+ identity), 8 channels per thread (c % 8 == 0, 16-B aligned)
template <typename T>
__global__ void k_scale_residual_v(const T* __restrict__ x, const float* gate, const T* identity, int hw, int c,
                                   long total8, T* y) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i8 >= total8) return;
  const long i = i8 * 8;
  const int ch = i % c;
  const long b = i / ((long)hw * c);
  float v[8], g[8];
  Vec8<T>::load(x + i, v);
  Vec8<float>::load(gate + b * c + ch, g);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= g[j];
  if (identity) {
    float r[8];
    Vec8<T>::load(identity + i, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += r[j];
  }
  Vec8<T>::store(y + i, v);
}

// RMSNorm (manifold_layers.py:449-456): x / sqrt(mean(x^2) + eps) * scale
template <typename T>
__global__ void __launch_bounds__(256) k_rmsnorm(const T* __restrict__ x, int rows, int cols,
                                                 float eps, const float* scale, T* y) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const T* p = x + (long)r * cols;
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) { const float a = Elem<T>::load(p, j); s += a * a; }
  const float rms = sqrtf(wave_sum(s) / cols + eps);
  for (int j = lane; j < cols; j += 64)
    Elem<T>::store(y + (long)r * cols, j, Elem<T>::load(p, j) / rms * scale[j]);
}

// ---------------------------------------------------------------- mHC coefficient prep
// gc[i,k] = g_i s(raw[i,k]) - mean_i(g_i s(raw[i,k])) ; u[k] = sum_i b_i s(raw[i,k])
// Two passes over 64x64 tiles (grid = Hd/64 x D/64): column partial sums, then centre + write.
constexpr int PT = 64;
__global__ void __launch_bounds__(256) k_prep_pre_sum(int D, int Hd, const float* __restrict__ raw,
                                                      const float* gamma, const float* beta,
                                                      float* part /* [2][nrb][Hd] */) {
  __shared__ float red[2][4][PT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * PT + lane, rb = blockIdx.y, nrb = gridDim.y;
  float sg = 0.f, sb = 0.f;
  if (k < Hd) {
    for (int r = w; r < PT; r += 4) {
      const int i = rb * PT + r;
      if (i >= D) break;
      const float s = 1.0f / (1.0f + expf(-raw[(long)i * Hd + k]));
      sg += gamma[i] * s;
      sb += beta[i] * s;
    }
  }
  red[0][w][lane] = sg;
  red[1][w][lane] = sb;
  __syncthreads();
  if (w == 0 && k < Hd) {
    part[(long)rb * Hd + k] = (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]);
    part[(long)(nrb + rb) * Hd + k] = (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]);
  }
}

__global__ void __launch_bounds__(256) k_prep_pre_write(int D, int Hd, const float* __restrict__ raw,
                                                        const float* gamma, const float* part, float* gc,
                                                        int gct, float* u) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * PT + lane, rb = blockIdx.y, nrb = gridDim.y;
  if (k >= Hd) return;
  float sg = 0.f, sb = 0.f;
  for (int r = 0; r < nrb; ++r) { sg += part[(long)r * Hd + k]; sb += part[(long)(nrb + r) * Hd + k]; }
  const float mean = sg / D;
  if (rb == 0 && w == 0) u[k] = sb;
  for (int r = w; r < PT; r += 4) {
    const int i = rb * PT + r;
    if (i >= D) break;
    const float s = 1.0f / (1.0f + expf(-raw[(long)i * Hd + k]));
    gc[gct ? (long)k * D + i : (long)i * Hd + k] = gamma[i] * s - mean;
  }
}

// y[n] = sum_k W[n, k] x[k] + b[n]  (fp32 GEMV, one wave per output)
__global__ void __launch_bounds__(256) k_gemv(const float* __restrict__ W, const float* __restrict__ x,
                                              const float* b, int N, int K, float* y) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const float* row = W + (long)n * K;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += row[k] * x[k];
  s = wave_sum(s);
  if (lane == 0) y[n] = s + (b ? b[n] : 0.f);
}

// row means of H_res (rows 0..D-1) and H_post = 2 s(raw) (rows D..D+Hd-1); one wave per row
__global__ void __launch_bounds__(256) k_prep_rowmean(int D, int Hd, const float* hres,
                                                      const float* hpost_raw, float* rm) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= D + Hd) return;
  float s = 0.f;
  if (r < D) {
    for (int j = lane; j < D; j += 64) s += hres[(long)r * D + j];
  } else {
    const float* p = hpost_raw + (long)(r - D) * D;
    for (int j = lane; j < D; j += 64) s += 2.0f / (1.0f + expf(-p[j]));
  }
  s = wave_sum(s);
  if (lane == 0) rm[r] = s / D;
}

// wct[j][i] = src[i][j] - rm[i], src = [H_res ; 2 s(H_post_raw)] ([D+Hd, D]); 32x32 LDS tiles
__global__ void __launch_bounds__(256) k_prep_wct(int D, int Hd, const float* hres,
                                                  const float* hpost_raw, const float* rm,
                                                  float* wct) {
  __shared__ float tile[32][33];
  const int Kc = D + Hd;
  const int i0 = blockIdx.x * 32, j0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int i = i0 + r, j = j0 + tx;
    float v = 0.f;
    if (i < Kc && j < D) {
      v = i < D ? hres[(long)i * D + j]
                : 2.0f / (1.0f + expf(-hpost_raw[(long)(i - D) * D + j]));
      v -= rm[i];
    }
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int j = j0 + r, i = i0 + tx;
    if (j < D && i < Kc) wct[(long)j * Kc + i] = tile[tx][r];
  }
}

// ---------------------------------------------------------------- casts / layout
template <typename T>
__global__ void k_cast(const float* __restrict__ x, long n, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) Elem<T>::store(y, i, x[i]);
}

template <typename T>
__global__ void k_nchw_to_nhwc(const float* __restrict__ x, int n, int c, int h, int w, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)n * c * h * w;
  if (i >= total) return;
  const int ci = i % c;
  const long p = i / c;                 // n*h*w index
  const int b = p / ((long)h * w);
  const long hw = p % ((long)h * w);
  Elem<T>::store(y, i, x[((long)b * c + ci) * h * w + hw]);
}

template <typename T>
__global__ void k_maxpool2x2(const T* __restrict__ x, int n, int h, int w, int c, T* y) {
  const int oh = h / 2, ow = w / 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)n * oh * ow * c;
  if (i >= total) return;
  const int ci = i % c;
  long p = i / c;
  const int ox = p % ow; p /= ow;
  const int oy = p % oh;
  const int b = p / oh;
  const T* base = x + (((long)b * h + 2 * oy) * w + 2 * ox) * c + ci;
  const float v = fmaxf(fmaxf(Elem<T>::load(base, 0), Elem<T>::load(base, c)),
                        fmaxf(Elem<T>::load(base, (long)w * c), Elem<T>::load(base, (long)w * c + c)));
  Elem<T>::store(y, i, v);
}

// 2x2 max pool (stride 2) with the SE gate applied first, 8 channels per thread, 16-B loads:
// max_q(x_q * g) = g * max_q(x_q) for the positive sigmoid gate, and storage rounding is
// monotone, so this equals scale_residual (no identity) followed by k_maxpool2x2 bit for bit
// while reading the un-pooled map once (gate == nullptr: plain max pool).
template <typename T>
__global__ void __launch_bounds__(256) k_scale_maxpool_v(const T* __restrict__ x, const float* gate, int n,
                                                         int h, int w, int c, long total8, T* y) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i8 >= total8) return;
  const int oh = h / 2, ow = w / 2, cv = c / 8;
  const int cg = i8 % cv;
  long p = i8 / cv;
  const int ox = p % ow; p /= ow;
  const int oy = p % oh;
  const int b = p / oh;
  const T* base = x + (((long)b * h + 2 * oy) * w + 2 * ox) * c + cg * 8;
  float v0[8], v1[8], v2[8], v3[8];
  Vec8<T>::load(base, v0);
  Vec8<T>::load(base + c, v1);
  Vec8<T>::load(base + (long)w * c, v2);
  Vec8<T>::load(base + (long)w * c + c, v3);
  float g[8];
  if (gate) Vec8<float>::load(gate + (long)b * c + cg * 8, g);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v0[j] = fmaxf(fmaxf(v0[j], v1[j]), fmaxf(v2[j], v3[j]));
    if (gate) v0[j] *= g[j];
  }
  Vec8<T>::store(y + i8 * 8, v0);
}

// channel sums over pixel chunks: part[n, chunk, c].  A block covers CM_UNROLL row steps of
// RPI = 256 / (c / VEC) rows; each thread issues its CM_UNROLL 16-byte row-vector loads before
// summing them (independent loads in flight instead of one dependent load per step), so the
// pass runs at the memory rate rather than one load latency per row.
constexpr int CM_UNROLL = 8;
__host__ __device__ constexpr int cm_rows_per_chunk(int c, int vec) { return (256 / (c / vec)) * CM_UNROLL; }

template <typename T>
__global__ void __launch_bounds__(256) k_chan_partial(const T* __restrict__ x, int hw, int c,
                                                      int nchunk, float* part) {
  // Requires c % VEC == 0 and c / VEC <= 256 (checked by the launcher).
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[256 * VEC];
  const int chunk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int cv = c / VEC, rpi = 256 / cv;
  const int g = t % cv, r = t / cv;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  if (r < rpi) {
    const int p0 = chunk * rpi * CM_UNROLL + r;
    const T* base = x + (long)b * hw * c + g * VEC;
    uint4 v[CM_UNROLL];
#pragma unroll
    for (int u = 0; u < CM_UNROLL; ++u) {
      const int p = p0 + u * rpi;
      v[u] = p < hw ? *reinterpret_cast<const uint4*>(base + (long)p * c) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < CM_UNROLL; ++u) {
      const T* e = reinterpret_cast<const T*>(&v[u]);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += Elem<T>::load(e, j);
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[t * VEC + j] = acc[j];
  __syncthreads();
  // red[(r*cv + g)*VEC + j] holds channel g*VEC+j of row-slot r; sum the rpi slots in order
  for (int ch = t; ch < c; ch += 256) {
    float s = 0.f;
    for (int q = 0; q < rpi; ++q) s += red[q * c + ch];
    part[((long)b * nchunk + chunk) * c + ch] = s;
  }
}

// out[b, ch] = inv * sum_k part[b, k, ch]: block = 64 channels x 4 lanes over the chunks (lane q
// takes chunks q, q+4, ...), lanes combined in a fixed order (deterministic)
__global__ void __launch_bounds__(256) k_chan_final(const float* part, int n, int nchunk, int c, float inv,
                                                    float* out) {
  __shared__ float red[256];
  const int b = blockIdx.y, ch = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  float s = 0.f;
  if (ch < c) {
#pragma unroll 8
    for (int k = q; k < nchunk; k += 4) s += part[((long)b * nchunk + k) * c + ch];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (q == 0 && ch < c)
    out[(long)b * c + ch] = ((red[threadIdx.x] + red[threadIdx.x + 64]) + (red[threadIdx.x + 128] + red[threadIdx.x + 192])) * inv;
}

// SE gate MLP (vision_backbone.py:77-83): one block per image.  The block reads its pooled row
// into LDS before writing its gate row, so `pooled` may alias `gate` (hv_se_gate).
__global__ void __launch_bounds__(256) k_se_mlp(const float* pooled, int c, int cr, const float* w1,
                                                const float* b1, const float* w2, const float* b2,
                                                float* gate) {
  extern __shared__ float sh[];
  float* p = sh;           // [c]
  float* h = sh + c;       // [cr]
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < c; i += blockDim.x) p[i] = pooled[(long)b * c + i];
  __syncthreads();
  for (int o = threadIdx.x; o < cr; o += blockDim.x) {
    float s = b1[o];
    for (int i = 0; i < c; ++i) s += w1[(long)o * c + i] * p[i];
    h[o] = hv_silu(s);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < c; o += blockDim.x) {
    float s = b2[o];
    for (int i = 0; i < cr; ++i) s += w2[(long)o * cr + i] * h[i];
    gate[(long)b * c + o] = 1.0f / (1.0f + expf(-s));
  }
}

// Batched SE MLP over many workgroups (the one-block-per-image kernel above leaves B=1 on ONE
// workgroup whose threads walk whole weight rows with strided loads: ~10 us per site).  Stage 1:
// one wave per hidden unit o, lanes across the input channels (coalesced weight-row reads), the
// dots of up to NB images accumulated together and reduced by xor shuffles; stage 2 the same per
// output channel over the hidden vector.  Fixed summation order: deterministic.
template <int NB, int ACT>
__global__ void __launch_bounds__(256) k_se_fc(const float* __restrict__ in, int n, int k, int nout,
                                               const float* __restrict__ w, const float* __restrict__ bias,
                                               float* __restrict__ out) {
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int b0 = blockIdx.y * NB;
  if (o >= nout) return;
  float acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = 0.f;
  const float* wr = w + (long)o * k;
  for (int i = lane; i < k; i += 64) {
    const float wv = wr[i];
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (b0 + j < n) acc[j] += wv * in[(long)(b0 + j) * k + i];
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = wave_sum(acc[j]);
  if (lane < NB && b0 + lane < n) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < NB; ++j) if (j == lane) v = acc[j];
    v += bias[o];
    out[(long)(b0 + lane) * nout + o] = ACT == 0 ? hv_silu(v) : 1.0f / (1.0f + expf(-v));
  }
}

template <typename T>
__global__ void k_scale_residual(const T* __restrict__ x, const float* gate, const T* identity,
                                 int hw, int c, long total, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int ch = i % c;
  const long b = i / ((long)hw * c);
  float v = Elem<T>::load(x, i) * gate[b * c + ch];
  if (identity) v += Elem<T>::load(identity, i);
  Elem<T>::store(y, i, v);
}

template <typename T>
__global__ void k_upsample_add(const T* __restrict__ a, const T* __restrict__ bsrc, int n, int h,
                               int w, int c, int hb, int wb, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)n * h * w * c;
  if (i >= total) return;
  const int ch = i % c;
  long p = i / c;
  const int x = p % w; p /= w;
  const int yy = p % h;
  const int b = p / h;
  // nearest: src = floor(dst * in / out) (F.interpolate mode='nearest')
  const int sy = min((int)((float)yy * ((float)hb / (float)h)), hb - 1);
  const int sx = min((int)((float)x * ((float)wb / (float)w)), wb - 1);
  const float v = Elem<T>::load(a, i) + Elem<T>::load(bsrc, (((long)b * hb + sy) * wb + sx) * c + ch);
  Elem<T>::store(y, i, v);
}

// FPN top-down step, 8 channels per thread (c % 8 == 0, 16-B aligned rows): the element-per-
// thread form ran at ~1 TB/s on the 80x80x256 level (64-bit index division per element)
template <typename T>
__global__ void k_upsample_add_v(const T* __restrict__ a, const T* __restrict__ bsrc, int n, int h, int w, int c,
                                 int hb, int wb, T* __restrict__ y) {
  const int cv = c >> 3;
  const long total = (long)n * h * w * cv;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int ch = (int)(i % cv) * 8;
  const long p = i / cv;                         // output pixel (b, yy, x)
  const int x = (int)(p % w);
  const long q = p / w;
  const int yy = (int)(q % h);
  const int b = (int)(q / h);
  const int sy = min((int)((float)yy * ((float)hb / (float)h)), hb - 1);
  const int sx = min((int)((float)x * ((float)wb / (float)w)), wb - 1);
  float va[8], vb[8];
  Vec8<T>::load(a + p * c + ch, va);
  Vec8<T>::load(bsrc + (((long)b * hb + sy) * wb + sx) * c + ch, vb);
#pragma unroll
  for (int e = 0; e < 8; ++e) va[e] += vb[e];
  Vec8<T>::store(y + p * c + ch, va);
}

template <typename T>
__global__ void k_add_scaled(const T* a, const T* b, long n, float alpha, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) Elem<T>::store(y, i, (Elem<T>::load(a, i) + Elem<T>::load(b, i)) * alpha);
}

// 8 elements per thread (n % 8 == 0, 16-B aligned)
template <typename T>
__global__ void k_add_scaled_v(const T* __restrict__ a, const T* __restrict__ b, long n8, float alpha, T* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float va[8], vb[8];
  Vec8<T>::load(a + i * 8, va);
  Vec8<T>::load(b + i * 8, vb);
#pragma unroll
  for (int e = 0; e < 8; ++e) va[e] = (va[e] + vb[e]) * alpha;
  Vec8<T>::store(y + i * 8, va);
}

template <typename T>
__global__ void k_add_rowvec(const T* x, const float* v, int p, int c, long total, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int ch = i % c;
  const long b = i / ((long)p * c);
  Elem<T>::store(y, i, Elem<T>::load(x, i) + v[b * c + ch]);
}

// F.interpolate(mode='linear', align_corners=False) of [L, D] -> [Lout, D]
__global__ void k_interp_linear(const float* src, int L, int D, int Lout, float* dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Lout * D) return;
  const int o = i / D, d = i % D;
  const float scale = (float)L / (float)Lout;
  float s = scale * ((float)o + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  const int x0 = (int)s;
  const int x1 = x0 + (x0 < L - 1 ? 1 : 0);
  const float l1 = s - (float)x0, l0 = 1.0f - l1;
  dst[i] = l0 * src[(long)x0 * D + d] + l1 * src[(long)x1 * D + d];
}

// ---------------------------------------------------------------- transformer pieces
template <typename T>
__global__ void __launch_bounds__(256) k_vit_tokens(const T* x, const float* cls, const float* pos,
                                                    const float* scale, int n, int tokens, int d, T* y) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int L = tokens + 1;
  if (r >= n * L) return;
  const int b = r / L, t = r % L;
  float s = 0.f;
  for (int j = lane; j < d; j += 64) {
    const float v = (t == 0 ? cls[j] : Elem<T>::load(x, ((long)b * tokens + t - 1) * d + j)) +
                    pos[(long)t * d + j];
    s += v * v;
  }
  const float rms = sqrtf(wave_sum(s) / d + 1e-8f);
  for (int j = lane; j < d; j += 64) {
    const float v = (t == 0 ? cls[j] : Elem<T>::load(x, ((long)b * tokens + t - 1) * d + j)) +
                    pos[(long)t * d + j];
    Elem<T>::store(y, (long)r * d + j, v / rms * scale[j]);
  }
}

// softmax(q k^T * scale) v: one thread per query, key/value tiles staged in LDS with an
// online softmax; q/k/v/out are [n, L, heads*HD].
template <typename T, int HD>
__global__ void __launch_bounds__(128) k_attention(const T* q, const T* k, const T* v, T* out,
                                                   int L, int heads, float sm_scale) {
  constexpr int KT = 128;
  __shared__ float ks[KT][HD], vs[KT][HD];
  const int b = blockIdx.z, h = blockIdx.y;
  const int qi = blockIdx.x * 128 + threadIdx.x;
  const int D = heads * HD;
  const long base = (long)b * L * D + h * HD;
  float qv[HD], o[HD];
  const bool active = qi < L;
#pragma unroll
  for (int j = 0; j < HD; ++j) {
    qv[j] = active ? Elem<T>::load(q, base + (long)qi * D + j) * sm_scale : 0.f;
    o[j] = 0.f;
  }
  float mx = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += KT) {
    __syncthreads();
    for (int e = threadIdx.x; e < KT * HD; e += 128) {
      const int kk = e / HD, j = e % HD;
      const bool in = k0 + kk < L;
      ks[kk][j] = in ? Elem<T>::load(k, base + (long)(k0 + kk) * D + j) : 0.f;
      vs[kk][j] = in ? Elem<T>::load(v, base + (long)(k0 + kk) * D + j) : 0.f;
    }
    __syncthreads();
    const int kn = min(KT, L - k0);
    for (int kk = 0; kk < kn; ++kk) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < HD; ++j) s += qv[j] * ks[kk][j];
      if (s > mx) {
        const float f = expf(mx - s);
        l *= f;
#pragma unroll
        for (int j = 0; j < HD; ++j) o[j] *= f;
        mx = s;
      }
      const float p = expf(s - mx);
      l += p;
#pragma unroll
      for (int j = 0; j < HD; ++j) o[j] += p * vs[kk][j];
    }
  }
  if (active) {
    const float inv = 1.0f / l;
#pragma unroll
    for (int j = 0; j < HD; ++j) Elem<T>::store(out, base + (long)qi * D + j, o[j] * inv);
  }
}

// ---- bf16 MFMA attention, head dim 32 (manifold_layers.py:404-427 core).
// One wave = 16 queries, no LDS, no barriers.  Every product is computed transposed so a lane
// owns one query:  S^T = K Q^T (lane: 4+4 keys of query fr), online softmax in the log2
// domain with max/sum across the 4 lane groups (xor 16/32), then O^T += V^T P^T where the
// 32-key contraction uses the permuted key order {4g..4g+3, 16+4g..16+4g+3} on BOTH
// operands (P straight from the S^T registers; V^T rows from the pre-transposed vt).
__global__ void k_vt_pad(const unsigned short* __restrict__ v, int L, int Lp, int heads,
                         unsigned short* __restrict__ vt) {
  // vt[b][h][d][key] = v[b][key][h*32 + d], zero for L <= key < Lp
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int bh = blockIdx.y, b = bh / heads, h = bh % heads;
  if (i >= 32L * Lp) return;
  const int d = i / Lp, key = i % Lp;
  vt[(long)bh * 32 * Lp + i] = key < L ? v[((long)b * L + key) * heads * 32 + h * 32 + d] : (unsigned short)0;
}

__global__ void __launch_bounds__(256) k_attention_mfma(const unsigned short* __restrict__ q,
                                                        const unsigned short* __restrict__ k,
                                                        const unsigned short* __restrict__ vt,
                                                        unsigned short* __restrict__ out, int L, int Lp,
                                                        int heads, float sl2) {
  const int b = blockIdx.z, h = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int D = heads * 32;
  const int q0 = blockIdx.x * 64 + w * 16;
  if (q0 >= L) return;
  const unsigned short* qb = q + (long)b * L * D + h * 32;
  const unsigned short* kb = k + (long)b * L * D + h * 32;
  const unsigned short* vb = vt + ((long)b * heads + h) * 32 * Lp;
  const uint4 qf = *reinterpret_cast<const uint4*>(qb + (long)min(q0 + fr, L - 1) * D + fg * 8);
  f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += 32) {
    const uint4 kf0 = *reinterpret_cast<const uint4*>(kb + (long)min(k0 + fr, L - 1) * D + fg * 8);
    const uint4 kf1 = *reinterpret_cast<const uint4*>(kb + (long)min(k0 + 16 + fr, L - 1) * D + fg * 8);
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf0), __builtin_bit_cast(bf16x8, qf), z, 0, 0, 0);
    const f32x4 s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf1), __builtin_bit_cast(bf16x8, qf), z, 0, 0, 0);
    float t[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[j] = (k0 + fg * 4 + j < L) ? s0[j] * sl2 : -INFINITY;
      t[4 + j] = (k0 + 16 + fg * 4 + j < L) ? s1[j] * sl2 : -INFINITY;
    }
    float mx = fmaxf(fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3])), fmaxf(fmaxf(t[4], t[5]), fmaxf(t[6], t[7])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float corr = __builtin_amdgcn_exp2f(m - mn);
    float p[8], ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { p[j] = __builtin_amdgcn_exp2f(t[j] - mn); ps += p[j]; }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o0[j] *= corr; o1[j] *= corr; }
    const uint4 pf = make_uint4(pack_bf16x2(p[0], p[1]), pack_bf16x2(p[2], p[3]), pack_bf16x2(p[4], p[5]),
                                pack_bf16x2(p[6], p[7]));
    const unsigned short* v0 = vb + (long)fr * Lp + k0 + fg * 4;
    const unsigned short* v1 = vb + (long)(16 + fr) * Lp + k0 + fg * 4;
    const uint2 a0 = *reinterpret_cast<const uint2*>(v0), a1 = *reinterpret_cast<const uint2*>(v0 + 16);
    const uint2 c0 = *reinterpret_cast<const uint2*>(v1), c1 = *reinterpret_cast<const uint2*>(v1 + 16);
    o0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, make_uint4(a0.x, a0.y, a1.x, a1.y)),
                                                 __builtin_bit_cast(bf16x8, pf), o0, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, make_uint4(c0.x, c0.y, c1.x, c1.y)),
                                                 __builtin_bit_cast(bf16x8, pf), o1, 0, 0, 0);
  }
  if (q0 + fr < L) {
    const float inv = 1.0f / l;
    unsigned short* ob = out + ((long)b * L + q0 + fr) * D + h * 32 + fg * 4;
    *reinterpret_cast<uint2*>(ob) = make_uint2(pack_bf16x2(o0[0] * inv, o0[1] * inv), pack_bf16x2(o0[2] * inv, o0[3] * inv));
    *reinterpret_cast<uint2*>(ob + 16) = make_uint2(pack_bf16x2(o1[0] * inv, o1[1] * inv), pack_bf16x2(o1[2] * inv, o1[3] * inv));
  }
}

template <typename T>
__global__ void k_gather_rows(const T* x, long stride_rows, int n, int c, T* y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * c) return;
  const int b = i / c, j = i % c;
  y[i] = x[(long)b * stride_rows * c + j];
}

// ---------------------------------------------------------------- YOLO decode
// One wave per group of YG = 8 consecutive cells (b, a, y, x): the group's predictions
// ([YG][P], contiguous) and scores ([YG][nc], contiguous) are swept by all 64 lanes with
// flat indices, so every store instruction covers 256 contiguous bytes (one wave per cell
// left a 21-lane second pass per 85-float row and serial box stores).  The scores are kept
// in LDS; the argmax per cell is then done by an 8-lane group (first index wins ties, like a
// sequential scan), and lanes 0..YG-1 decode one box each.
constexpr int YG = 8;
constexpr int YMAXP = 256;                 // 5 + nc <= 256

template <typename T>
__global__ void __launch_bounds__(256) k_yolo_decode(const T* __restrict__ logits, int n, int h, int w,
                                                     int A, int nc, const float* anchor_wh,
                                                     float* pred, float* boxes, float* scores,
                                                     float* cscore, int64_t* cidx, float* obj, float* det) {
  __shared__ float sc_s[4][YG * (YMAXP - 5)];
  __shared__ float ob_s[4][YG];
  __shared__ long so_s[4][YG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long total = (long)n * A * h * w;
  const long c0 = ((long)blockIdx.x * 4 + wv) * YG;          // first cell of this wave
  if (c0 >= total) return;                                     // wave-uniform; no block barrier below
  const int ncell = (int)min((long)YG, total - c0);
  const int P = 5 + nc;
  // lane c < ncell computes the logits offset of cell c0 + c (64-bit div/mod once per cell,
  // not per element) into LDS; the sweeps below read it from there
  long soff = 0;
  if (lane < ncell) {
    const long cell = c0 + lane;
    const int x = cell % w;
    long t = cell / w;
    const int y = t % h; t /= h;
    const int a = t % A;
    const int b = t / A;
    soff = (((long)b * h + y) * w + x) * (long)(A * P) + (long)a * P;
    ob_s[wv][lane] = 1.0f / (1.0f + expf(-Elem<T>::load(logits + soff, 4)));
    so_s[wv][lane] = soff;
  }
  auto src_of = [&](int c) -> const T* { return logits + so_s[wv][c]; };
  __builtin_amdgcn_wave_barrier();
  // predictions: raw logits, flat over [ncell][P] (P > 64: the cell index advances by <= 1)
  {
    int c = lane / P, k = lane - c * P;
    for (int i = lane; i < ncell * P; i += 64) {
      pred[c0 * P + i] = Elem<T>::load(src_of(c), k);
      k += 64;
      while (k >= P) { k -= P; ++c; }
    }
  }
  // scores = sigmoid(obj) * sigmoid(cls), flat over [ncell][nc]
  {
    int c = lane / nc, k = lane - c * nc;
    for (int i = lane; i < ncell * nc; i += 64) {
      const float cp = 1.0f / (1.0f + expf(-Elem<T>::load(src_of(c), 5 + k)));
      const float sv = ob_s[wv][c] * cp;
      scores[c0 * nc + i] = sv;
      if (det) det[(c0 + c) * P + 5 + k] = cp;
      sc_s[wv][i] = sv;
      k += 64;
      while (k >= nc) { k -= nc; ++c; }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // argmax per cell: lane group g (8 lanes) owns cell g
  {
    const int g = lane >> 3, j = lane & 7;
    float best = -1.f;
    int bi = 0x7fffffff;
    if (g < ncell)
      for (int k = j; k < nc; k += 8) {
        const float v = sc_s[wv][g * nc + k];
        if (v > best) { best = v; bi = k; }
      }
#pragma unroll
    for (int off = 4; off > 0; off >>= 1) {
      const float ob = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (j == 0 && g < ncell) {
      cscore[c0 + g] = best;
      cidx[c0 + g] = bi;
    }
  }
  if (lane < ncell) {
    const long cell = c0 + lane;
    const int x = cell % w;
    long t = cell / w;
    const int y = t % h; t /= h;
    const int a = t % A;
    const T* src = logits + soff;
    const float v0 = Elem<T>::load(src, 0), v1 = Elem<T>::load(src, 1);
    const float v2 = Elem<T>::load(src, 2), v3 = Elem<T>::load(src, 3);
    const float sx = 1.0f / (1.0f + expf(-v0)), sy = 1.0f / (1.0f + expf(-v1));
    const float bx = ((float)x + sx) / (float)w, by = ((float)y + sy) / (float)h;
    const float bw = anchor_wh[2 * a] * expf(v2), bh = anchor_wh[2 * a + 1] * expf(v3);
    *reinterpret_cast<float4*>(boxes + cell * 4) = make_float4(bx - bw / 2, by - bh / 2, bx + bw / 2, by + bh / 2);
    obj[cell] = ob_s[wv][lane];
    if (det) {
      float* dr = det + cell * P;
      dr[0] = bx - bw / 2; dr[1] = by - bh / 2; dr[2] = bx + bw / 2; dr[3] = by + bh / 2;
      dr[4] = ob_s[wv][lane];
    }
  }
}

}  // namespace

// ============================================================== C ABI
extern "C" int hv_row_stats(int dtype, const void* x, long ldx, int rows, int cols, float eps,
                            float* mean, float* rstd, hv_stream_t stream) {
  if (rows <= 0 || cols <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (cols % 8 == 0 && cols <= 4096 && ldx % 8 == 0 && ((uintptr_t)x & 15) == 0) {
    int G, NP;
    row_shape(cols, G, NP);
    HV_ROW_SHAPES(G, NP, HV_DISPATCH(dtype, (k_row_stats_v<T, G_, NP_><<<hv_cdiv(rows, 256 / G_), 256, 0, s>>>(
                                                (const T*)x, ldx, rows, cols, eps, mean, rstd))));
  } else {
    HV_DISPATCH(dtype, (k_row_stats<T><<<hv_cdiv(rows, 4), 256, 0, s>>>((const T*)x, ldx, rows, cols, eps, mean,
                                                                          rstd)));
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_layernorm(int x_dtype, const void* x, int rows, int cols, float eps,
                            const float* gamma, const float* beta, int y_dtype, void* y,
                            const void* res_out, int res_dtype, hv_stream_t stream) {
  if (rows <= 0 || cols <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (cols % 8 == 0 && cols <= 4096 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
      ((uintptr_t)res_out & 15) == 0 && ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0 &&
      (x_dtype == HV_F32 || x_dtype == HV_BF16) && (y_dtype == HV_F32 || y_dtype == HV_BF16)) {
    int G, NP;
    row_shape(cols, G, NP);
    const unsigned grid = hv_cdiv(rows, 256 / G);
#define HV_LN_V(TX, TY)                                                                                  \
  HV_ROW_SHAPES(G, NP, (k_layernorm_v<TX, TY, G_, NP_><<<grid, 256, 0, s>>>((const TX*)x, rows, cols, eps, \
                                                                            gamma, beta, (TY*)y, res_out, res_dtype)))
    if (x_dtype == HV_F32 && y_dtype == HV_F32) { HV_LN_V(float, float); }
    else if (x_dtype == HV_F32) { HV_LN_V(float, bf); }
    else if (y_dtype == HV_BF16) { HV_LN_V(bf, bf); }
    else { HV_LN_V(bf, float); }
#undef HV_LN_V
    HV_CHECK_LAUNCH();
    return HV_OK;
  }
  const dim3 g(hv_cdiv(rows, 4));
  if (x_dtype == HV_F32 && y_dtype == HV_F32)
    k_layernorm<float, float><<<g, 256, 0, s>>>((const float*)x, rows, cols, eps, gamma, beta, (float*)y, res_out, res_dtype);
  else if (x_dtype == HV_F32 && y_dtype == HV_BF16)
    k_layernorm<float, bf><<<g, 256, 0, s>>>((const float*)x, rows, cols, eps, gamma, beta, (bf*)y, res_out, res_dtype);
  else if (x_dtype == HV_BF16 && y_dtype == HV_BF16)
    k_layernorm<bf, bf><<<g, 256, 0, s>>>((const bf*)x, rows, cols, eps, gamma, beta, (bf*)y, res_out, res_dtype);
  else if (x_dtype == HV_BF16 && y_dtype == HV_F32)
    k_layernorm<bf, float><<<g, 256, 0, s>>>((const bf*)x, rows, cols, eps, gamma, beta, (float*)y, res_out, res_dtype);
  else
    return HV_EINVAL;
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_rmsnorm(int dtype, const void* x, int rows, int cols, float eps,
                          const float* scale, void* y, hv_stream_t stream) {
  if (rows <= 0 || cols <= 0 || !scale) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_rmsnorm<T><<<hv_cdiv(rows, 4), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, rows, cols, eps, scale, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_mhc_prep(int D, int Hd, const float* h_pre_raw, const float* h_post_raw,
                           const float* h_res, const float* gamma_pre, const float* beta_pre,
                           float* gc, int gct, float* u, float* wct, float* rm, hv_stream_t stream) {
  if (D <= 0 || Hd <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(hv_cdiv(Hd, PT), hv_cdiv(D, PT));
  // column partials live in the tail of `wct` (written last, after its own pass)
  float* part = wct + (long)D * (D + Hd) - 2L * g.y * Hd;
  if (2L * g.y * Hd > (long)D * (D + Hd)) return HV_EUNSUPPORTED;
  k_prep_pre_sum<<<g, 256, 0, s>>>(D, Hd, h_pre_raw, gamma_pre, beta_pre, part);
  k_prep_pre_write<<<g, 256, 0, s>>>(D, Hd, h_pre_raw, gamma_pre, part, gc, gct, u);
  k_prep_rowmean<<<hv_cdiv(D + Hd, 4), 256, 0, s>>>(D, Hd, h_res, h_post_raw, rm);
  k_prep_wct<<<dim3(hv_cdiv(D + Hd, 32), hv_cdiv(D, 32)), 256, 0, s>>>(D, Hd, h_res, h_post_raw, rm, wct);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_cast(const float* x, long n, int y_dtype, void* y, hv_stream_t stream) {
  if (n <= 0) return n == 0 ? HV_OK : HV_EINVAL;
  HV_DISPATCH(y_dtype, (k_cast<T><<<hv_cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(x, n, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_nchw_to_nhwc(const float* x, int n, int c, int h, int w, int y_dtype, void* y,
                               hv_stream_t stream) {
  const long total = (long)n * c * h * w;
  if (total <= 0) return HV_EINVAL;
  HV_DISPATCH(y_dtype, (k_nchw_to_nhwc<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                            x, n, c, h, w, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_maxpool2x2(int dtype, const void* x, int n, int h, int w, int c, void* y,
                             hv_stream_t stream) {
  const long total = (long)n * (h / 2) * (w / 2) * c;
  if (total <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_maxpool2x2<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, n, h, w, c, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_scale_maxpool2x2(int dtype, const void* x, const float* gate, int n, int h, int w, int c,
                                   void* y, hv_stream_t stream) {
  const long total = (long)n * (h / 2) * (w / 2) * c;
  if (total <= 0 || c % 8 || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gate) & 15)) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_scale_maxpool_v<T><<<hv_cdiv(total / 8, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, gate, n, h, w, c, total / 8, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// sized for the smaller fp32 chunk (vec 4) when that is a valid layout, else for bf16 (vec 8)
extern "C" size_t hv_channel_mean_work_floats(int n, int hw, int c) {
  if (c <= 0 || hw <= 0 || n <= 0) return 0;
  const int vec = (c % 4 == 0 && c / 4 <= 256) ? 4 : 8;
  const int rows = cm_rows_per_chunk(c < vec ? vec : c, vec);
  return (size_t)n * ((hw + rows - 1) / rows) * c;
}

extern "C" int hv_channel_mean(int dtype, const void* x, int n, int hw, int c, float* out,
                               float* work, hv_stream_t stream) {
  if (n <= 0 || hw <= 0 || c <= 0 || !work) return HV_EINVAL;
  const int vec = dtype == HV_BF16 ? 8 : 4;
  if (c % vec || c / vec > 256 || ((uintptr_t)x & 15)) return HV_EINVAL;
  const int rows = cm_rows_per_chunk(c, vec);
  const int nchunk = (hw + rows - 1) / rows;
  hipStream_t s = (hipStream_t)stream;
  HV_DISPATCH(dtype, (k_chan_partial<T><<<dim3(nchunk, n), 256, 0, s>>>(
                          (const T*)x, hw, c, nchunk, work)));
  k_chan_final<<<dim3(hv_cdiv(c, 64), n), 256, 0, s>>>(work, n, nchunk, c, 1.0f / hw, out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_se_mlp2(const float* pooled, int n, int c, int cr, const float* w1, const float* b1,
                          const float* w2, const float* b2, float* hidden, float* gate, hv_stream_t stream);
extern "C" int hv_se_mlp(const float* pooled, int n, int c, int cr, const float* w1, const float* b1,
                         const float* w2, const float* b2, float* gate, hv_stream_t stream) {
  return hv_se_mlp2(pooled, n, c, cr, w1, b1, w2, b2, nullptr, gate, stream);
}
extern "C" int hv_se_mlp2(const float* pooled, int n, int c, int cr, const float* w1, const float* b1,
                          const float* w2, const float* b2, float* hidden, float* gate, hv_stream_t stream) {
  if (n <= 0 || c <= 0 || cr <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 4 && hidden) {      // measured: at n = 16 the per-image kernel wins (9.8 vs 15.8 + 8.2 us)
    // batched two-stage form (many workgroups); the hidden vector goes through caller scratch
    if (n == 1) {
      k_se_fc<1, 0><<<hv_cdiv(cr, 4), 256, 0, s>>>(pooled, n, c, cr, w1, b1, hidden);
      k_se_fc<1, 1><<<hv_cdiv(c, 4), 256, 0, s>>>(hidden, n, cr, c, w2, b2, gate);
    } else {
      k_se_fc<4, 0><<<hv_cdiv(cr, 4), 256, 0, s>>>(pooled, n, c, cr, w1, b1, hidden);
      k_se_fc<4, 1><<<hv_cdiv(c, 4), 256, 0, s>>>(hidden, n, cr, c, w2, b2, gate);
    }
  } else {
    k_se_mlp<<<n, 256, (c + cr) * sizeof(float), s>>>(pooled, c, cr, w1, b1, w2, b2, gate);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// Whole SE gate of an NHWC map in one call (vision_backbone.py:77-83, the channel_attention call
// of ConvMHCLayer.forward): chunk sums, the fixed-order final reduce into `gate` (used as the
// pooled buffer), then the MLP in place -- the launches of hv_channel_mean + hv_se_mlp2, bitwise
// equal to that pair.  (Finishing the mean inside the per-image MLP saved the reduce launch but
// walked nchunk partials per channel serially: 24.5 vs 9.8 + 6.6 us per site, slower in-model,
// profiles/r04/se_gate_fused_mean_rejected.txt.)
extern "C" int hv_se_gate(int dtype, const void* x, int n, int hw, int c, int cr, const float* w1,
                          const float* b1, const float* w2, const float* b2, float* work, float* hidden,
                          float* gate, hv_stream_t stream) {
  if (n <= 0 || hw <= 0 || c <= 0 || cr <= 0 || !work || !gate) return HV_EINVAL;
  const int rc = hv_channel_mean(dtype, x, n, hw, c, gate, work, stream);
  if (rc != HV_OK) return rc;
  return hv_se_mlp2(gate, n, c, cr, w1, b1, w2, b2, hidden, gate, stream);
}

extern "C" int hv_scale_residual(int dtype, const void* x, const float* gate, const void* identity,
                                 int n, int hw, int c, void* y, hv_stream_t stream) {
  const long total = (long)n * hw * c;
  if (total <= 0) return HV_EINVAL;
  if (c % 8 == 0 && (((uintptr_t)x | (uintptr_t)identity | (uintptr_t)y | (uintptr_t)gate) & 15) == 0) {
    HV_DISPATCH(dtype, (k_scale_residual_v<T><<<hv_cdiv(total / 8, 256), 256, 0, (hipStream_t)stream>>>(
                            (const T*)x, gate, (const T*)identity, hw, c, total / 8, (T*)y)));
  } else {
    HV_DISPATCH(dtype, (k_scale_residual<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                            (const T*)x, gate, (const T*)identity, hw, c, total, (T*)y)));
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_upsample_add(int dtype, const void* a, const void* b, int n, int h, int w, int c,
                               int hb, int wb, void* y, hv_stream_t stream) {
  const long total = (long)n * h * w * c;
  if (total <= 0) return HV_EINVAL;
  if (c % 8 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) & 15) == 0) {
    HV_DISPATCH(dtype, (k_upsample_add_v<T><<<hv_cdiv(total / 8, 256), 256, 0, (hipStream_t)stream>>>(
                            (const T*)a, (const T*)b, n, h, w, c, hb, wb, (T*)y)));
    HV_CHECK_LAUNCH();
    return HV_OK;
  }
  HV_DISPATCH(dtype, (k_upsample_add<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)a, (const T*)b, n, h, w, c, hb, wb, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_add_scaled(int dtype, const void* a, const void* b, long count, float alpha,
                             void* y, hv_stream_t stream) {
  if (count <= 0) return HV_EINVAL;
  if (count % 8 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) & 15) == 0) {
    HV_DISPATCH(dtype, (k_add_scaled_v<T><<<hv_cdiv(count / 8, 256), 256, 0, (hipStream_t)stream>>>(
                            (const T*)a, (const T*)b, count / 8, alpha, (T*)y)));
    HV_CHECK_LAUNCH();
    return HV_OK;
  }
  HV_DISPATCH(dtype, (k_add_scaled<T><<<hv_cdiv(count, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)a, (const T*)b, count, alpha, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_add_rowvec(int dtype, const void* x, const float* v, int n, int p, int c, void* y,
                             hv_stream_t stream) {
  const long total = (long)n * p * c;
  if (total <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_add_rowvec<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, v, p, c, total, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_interp_linear(const float* src, int L, int D, int Lout, float* dst,
                                hv_stream_t stream) {
  if (L <= 0 || D <= 0 || Lout <= 0) return HV_EINVAL;
  k_interp_linear<<<hv_cdiv((long)Lout * D, 256), 256, 0, (hipStream_t)stream>>>(src, L, D, Lout, dst);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_vit_tokens(int dtype, const void* x, const float* cls, const float* pos,
                             const float* scale, int n, int tokens, int d, void* y,
                             hv_stream_t stream) {
  if (n <= 0 || tokens <= 0 || d <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_vit_tokens<T><<<hv_cdiv((long)n * (tokens + 1), 4), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, cls, pos, scale, n, tokens, d, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}



// ---- general attention (MultiHeadManifoldAttention.forward with cross-attention, a key padding
// mask or need_weights; manifold_layers.py:386-434): one lane per query row, 32-key K/V tiles
// staged in LDS as fp32, online softmax; optional second pass writes the probabilities.
// A row whose keys are all masked gives NaN, as softmax over all -inf does in the reference.
template <typename T, int HD>
__global__ void __launch_bounds__(64) k_attention_general(const T* __restrict__ q, const T* __restrict__ k,
                                                          const T* __restrict__ v,
                                                          const unsigned char* __restrict__ mask, T* __restrict__ o,
                                                          float* __restrict__ wts, int Lq, int Lk, int heads,
                                                          float scale) {
  constexpr int KT = 32;
  __shared__ float ks[KT][HD + 1];
  __shared__ float vs[KT][HD + 1];
  __shared__ unsigned char ms[KT];
  const int D = heads * HD;
  const int h = blockIdx.y, b = blockIdx.z;
  const int i = blockIdx.x * 64 + threadIdx.x;
  const bool live = i < Lq;
  float qr[HD], acc[HD];
  const T* qp = q + ((long)b * Lq + (live ? i : 0)) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    qr[d] = Elem<T>::load(qp, d) * scale;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < Lk; j0 += KT) {
    __syncthreads();
    for (int e = threadIdx.x; e < KT * HD; e += 64) {
      const int jj = e / HD, d = e - jj * HD;
      const int j = j0 + jj;
      float kv = 0.f, vv = 0.f;
      if (j < Lk) {
        const long off = ((long)b * Lk + j) * D + h * HD + d;
        kv = Elem<T>::load(k, off);
        vv = Elem<T>::load(v, off);
      }
      ks[jj][d] = kv;
      vs[jj][d] = vv;
    }
    if (threadIdx.x < KT) {
      const int j = j0 + threadIdx.x;
      ms[threadIdx.x] = j < Lk ? (mask ? mask[(long)b * Lk + j] : 0) : 1;
    }
    __syncthreads();
    for (int jj = 0; jj < KT; ++jj) {
      if (ms[jj]) continue;
      float sc = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) sc = fmaf(qr[d], ks[jj][d], sc);
      const float mn = fmaxf(m, sc);
      const float corr = __expf(m - mn), p = __expf(sc - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc[d] = fmaf(acc[d], corr, p * vs[jj][d]);
      m = mn;
    }
  }
  if (live) {
    const float inv = l > 0.f ? 1.f / l : NAN;
    T* op = o + ((long)b * Lq + i) * D + h * HD;
#pragma unroll
    for (int d = 0; d < HD; ++d) Elem<T>::store(op, d, acc[d] * inv);
  }
  if (!wts) return;
  float* wp = wts + (((long)b * heads + h) * Lq + (live ? i : 0)) * Lk;
  for (int j0 = 0; j0 < Lk; j0 += KT) {
    __syncthreads();
    for (int e = threadIdx.x; e < KT * HD; e += 64) {
      const int jj = e / HD, d = e - jj * HD;
      const int j = j0 + jj;
      ks[jj][d] = j < Lk ? Elem<T>::load(k, ((long)b * Lk + j) * D + h * HD + d) : 0.f;
    }
    if (threadIdx.x < KT) {
      const int j = j0 + threadIdx.x;
      ms[threadIdx.x] = j < Lk ? (mask ? mask[(long)b * Lk + j] : 0) : 1;
    }
    __syncthreads();
    if (!live) continue;
    for (int jj = 0; jj < KT && j0 + jj < Lk; ++jj) {
      float p;
      if (l == 0.f) {
        p = NAN;
      } else if (ms[jj]) {
        p = 0.f;
      } else {
        float sc = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) sc = fmaf(qr[d], ks[jj][d], sc);
        p = __expf(sc - m) / l;
      }
      wp[j0 + jj] = p;
    }
  }
}


// ---- one query row per workgroup (the CLS query of the encoder's last block, Lq = 1): the keys
// are split over the 256 threads, each keeps an online-softmax partial (max, sum, acc[HD]); the
// partials merge through wave shuffles and LDS.
template <typename T, int HD>
__global__ void __launch_bounds__(256) k_attention_row(const T* __restrict__ q, const T* __restrict__ k,
                                                       const T* __restrict__ v, const unsigned char* __restrict__ mask,
                                                       T* __restrict__ o, int Lq, int Lk, int heads, float scale) {
  __shared__ float red[4][HD + 2];
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int D = heads * HD;
  float qr[HD], acc[HD];
  const T* qp = q + ((long)b * Lq + i) * D + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    qr[d] = Elem<T>::load(qp, d) * scale;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = threadIdx.x; j < Lk; j += 256) {
    if (mask && mask[(long)b * Lk + j]) continue;
    const long off = ((long)b * Lk + j) * D + h * HD;
    float sc = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) sc = fmaf(qr[d], Elem<T>::load(k, off + d), sc);
    const float mn = fmaxf(m, sc);
    const float corr = __expf(m - mn), p = __expf(sc - mn);
    l = l * corr + p;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc[d] = fmaf(acc[d], corr, p * Elem<T>::load(v, off + d));
    m = mn;
  }
  // merge (m, l, acc) across the wave, then across the 4 waves
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1) {
    const float m2 = __shfl_xor(m, sh, 64), l2 = __shfl_xor(l, sh, 64);
    const float mn = fmaxf(m, m2);
    const float c1 = mn == -INFINITY ? 0.f : __expf(m - mn), c2 = mn == -INFINITY ? 0.f : __expf(m2 - mn);
    l = l * c1 + l2 * c2;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc[d] = acc[d] * c1 + __shfl_xor(acc[d], sh, 64) * c2;
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = m;
    red[w][1] = l;
#pragma unroll
    for (int d = 0; d < HD; ++d) red[w][2 + d] = acc[d];
  }
  __syncthreads();
  if (threadIdx.x < HD) {
    float mm = -INFINITY;
    for (int ww = 0; ww < 4; ++ww) mm = fmaxf(mm, red[ww][0]);
    float ll = 0.f, aa = 0.f;
    for (int ww = 0; ww < 4; ++ww) {
      const float c = mm == -INFINITY ? 0.f : __expf(red[ww][0] - mm);
      ll += red[ww][1] * c;
      aa += red[ww][2 + threadIdx.x] * c;
    }
    Elem<T>::store(o + ((long)b * Lq + i) * D + h * HD, threadIdx.x, ll > 0.f ? aa / ll : NAN);
  }
}

// ---- batched byte-range copies (hv_copy_segments): 16 KiB per block, segment found by binary
// search over the block prefix table passed by value.  24 ranges per launch keep the by-value
// table under 1 KiB: with 64 (2.1 KiB of kernel arguments) a rocprofv3 --pmc run of a training
// step crashed inside the launch (SIGSEGV at a mapping boundary in the profiler-intercepted
// dispatch path; unprofiled runs were unaffected)
constexpr int kCopyMax = 24;
constexpr long long kCopyChunk = 16384;
struct CopyBatch {
  int count;
  const unsigned char* src[kCopyMax];
  unsigned char* dst[kCopyMax];
  long long bytes[kCopyMax];
  long long block_start[kCopyMax + 1];
};

__global__ void __launch_bounds__(256) k_copy_segments(const CopyBatch cb) {
  const long long b = blockIdx.x;
  int lo = 0, hi = cb.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cb.block_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const unsigned char* src = cb.src[lo];
  unsigned char* dst = cb.dst[lo];
  const long long beg = (b - cb.block_start[lo]) * kCopyChunk;
  const long long end = beg + kCopyChunk < cb.bytes[lo] ? beg + kCopyChunk : cb.bytes[lo];
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const long long vend = beg + ((end - beg) & ~15LL);
    for (long long i = beg + threadIdx.x * 16LL; i < vend; i += 256 * 16)
      *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    for (long long i = vend + threadIdx.x; i < end; i += 256) dst[i] = src[i];
  } else {
    for (long long i = beg + threadIdx.x; i < end; i += 256) dst[i] = src[i];
  }
}

extern "C" int hv_attention(int dtype, const void* q, const void* k, const void* v, void* out,
                            int n, int L, int heads, int hd, float sm_scale, hv_stream_t stream) {
  if (n <= 0 || L <= 0 || heads <= 0) return HV_EINVAL;
  if (hd != 32) return HV_EUNSUPPORTED;
  const dim3 g(hv_cdiv(L, 128), heads, n);
  hv_diag_count(HV_KF_ATTN_SCALAR);
  HV_DISPATCH(dtype, (k_attention<T, 32><<<g, 128, 0, (hipStream_t)stream>>>(
                          (const T*)q, (const T*)k, (const T*)v, (T*)out, L, heads, sm_scale)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_attention_work_elems(int n, int L, int heads, int hd) {
  return (size_t)n * heads * hd * ((L + 31) / 32 * 32);
}

extern "C" int hv_attention_mfma(const void* q, const void* k, const void* v, void* vt_work, void* out,
                                 int n, int L, int heads, int hd, float sm_scale, hv_stream_t stream) {
  if (n <= 0 || L <= 0 || heads <= 0 || !vt_work) return HV_EINVAL;
  if (hd != 32 || (((uintptr_t)q | (uintptr_t)k | (uintptr_t)vt_work | (uintptr_t)out) & 15)) return HV_EUNSUPPORTED;
  const int Lp = (L + 31) / 32 * 32;
  hipStream_t s = (hipStream_t)stream;
  hv_diag_count(HV_KF_ATTN_MFMA);
  k_vt_pad<<<dim3(hv_cdiv(32L * Lp, 256), n * heads), 256, 0, s>>>((const unsigned short*)v, L, Lp, heads,
                                                                   (unsigned short*)vt_work);
  k_attention_mfma<<<dim3(hv_cdiv(L, 64), heads, n), 256, 0, s>>>(
      (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)vt_work, (unsigned short*)out, L, Lp,
      heads, sm_scale * 1.4426950408889634f);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_gather_rows(int dtype, const void* x, long stride_rows, int n, int c, void* y,
                              hv_stream_t stream) {
  if (n <= 0 || c <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_gather_rows<T><<<hv_cdiv((long)n * c, 256), 256, 0, (hipStream_t)stream>>>(
                          (const T*)x, stride_rows, n, c, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_yolo_decode(int dtype, const void* logits, int n, int h, int w, int A, int nc,
                              const float* anchor_wh, float* predictions, float* boxes,
                              float* scores, float* class_scores, int64_t* class_indices,
                              float* objectness, float* detections, hv_stream_t stream) {
  const long total = (long)n * A * h * w;
  if (total <= 0 || nc <= 0) return HV_EINVAL;
  if (nc + 5 > YMAXP || ((uintptr_t)boxes & 15)) return HV_EUNSUPPORTED;
  HV_DISPATCH(dtype, (k_yolo_decode<T><<<hv_cdiv(total, 4L * YG), 256, 0, (hipStream_t)stream>>>(
                          (const T*)logits, n, h, w, A, nc, anchor_wh, predictions, boxes, scores,
                          class_scores, class_indices, objectness, detections)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// ---------------------------------------------------------------- parameter preparation
namespace {
// w [cout, cin, k, k] fp32 -> y [cout, k, k, cin] (implicit-GEMM B operand), optional row scale
template <typename T>
__global__ void k_conv_weight_prep(const float* __restrict__ w, int cout, int cin, int k,
                                   const float* scale, T* y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)cout * cin * k * k;
  if (i >= total) return;
  const int ci = i % cin;
  long t = i / cin;
  const int kw = t % k; t /= k;
  const int kh = t % k;
  const int co = t / k;
  float v = w[(((long)co * cin + ci) * k + kh) * k + kw];
  if (scale) v *= scale[co];
  Elem<T>::store(y, i, v);
}

// eval BatchNorm (+ conv bias) folded to a per-channel affine:  s = g / sqrt(v + eps),
// b' = beta + (bias - mean) * s   (vision_backbone.py:113, feature_fusion.py:44, yolo_head.py:122)
__global__ void k_bn_fold(int c, const float* g, const float* beta, const float* mean,
                          const float* var, const float* cbias, float eps, float* s_out,
                          float* b_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= c) return;
  const float s = g ? g[i] / sqrtf(var[i] + eps) : 1.0f;
  const float cb = cbias ? cbias[i] : 0.f;
  s_out[i] = s;
  b_out[i] = g ? beta[i] + (cb - mean[i]) * s : cb;
}
}  // namespace

extern "C" int hv_conv_weight_prep(const float* w, int cout, int cin, int k, const float* scale,
                                   int y_dtype, void* y, hv_stream_t stream) {
  const long total = (long)cout * cin * k * k;
  if (total <= 0) return HV_EINVAL;
  HV_DISPATCH(y_dtype, (k_conv_weight_prep<T><<<hv_cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(
                            w, cout, cin, k, scale, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_bn_fold(int c, const float* gamma, const float* beta, const float* mean,
                          const float* var, const float* conv_bias, float eps, float* scale_out,
                          float* bias_out, hv_stream_t stream) {
  if (c <= 0) return HV_EINVAL;
  k_bn_fold<<<hv_cdiv(c, 256), 256, 0, (hipStream_t)stream>>>(c, gamma, beta, mean, var, conv_bias,
                                                               eps, scale_out, bias_out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_gemv(const float* W, const float* x, const float* b, int N, int K, float* y,
                       hv_stream_t stream) {
  if (N <= 0 || K <= 0) return HV_EINVAL;
  k_gemv<<<hv_cdiv(N, 4), 256, 0, (hipStream_t)stream>>>(W, x, b, N, K, y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_copy_segments(const hv_copy_segment* segs, int count, hv_stream_t stream) {
  if (count < 0 || (count > 0 && !segs)) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < count; base += kCopyMax) {
    CopyBatch cb;
    cb.count = 0;
    long long blocks = 0;
    for (int i = base; i < count && i < base + kCopyMax; ++i) {
      if (segs[i].bytes < 0 || (segs[i].bytes > 0 && (!segs[i].src || !segs[i].dst))) return HV_EINVAL;
      if (segs[i].bytes == 0) continue;
      cb.src[cb.count] = (const unsigned char*)segs[i].src;
      cb.dst[cb.count] = (unsigned char*)segs[i].dst;
      cb.bytes[cb.count] = segs[i].bytes;
      cb.block_start[cb.count] = blocks;
      blocks += (segs[i].bytes + kCopyChunk - 1) / kCopyChunk;
      ++cb.count;
    }
    if (cb.count == 0) continue;
    cb.block_start[cb.count] = blocks;
    k_copy_segments<<<(unsigned)blocks, 256, 0, s>>>(cb);
    HV_CHECK_LAUNCH();
  }
  return HV_OK;
}

// Host bytes -> device through kernel arguments (1 KiB per launch): a captured graph records the
// bytes by value in its kernel nodes, so a table upload inside a capture needs no pinned staging
// buffer (pinning new host memory is refused while a stream captures) and nothing to keep alive.
constexpr int kArgBytes = 1024;                  // kernel-argument bytes per launch (see kCopyMax)
struct ArgBytes {
  unsigned int w[kArgBytes / 4];
};
__global__ void __launch_bounds__(256) k_write_bytes(const ArgBytes a, int n, unsigned char* dst) {
  for (int i = threadIdx.x; i < n; i += 256) dst[i] = (unsigned char)(a.w[i >> 2] >> (8 * (i & 3)));
}

extern "C" int hv_write_bytes(void* dst, const void* src, long long n, hv_stream_t stream) {
  if (n < 0 || (n > 0 && (!dst || !src))) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  for (long long off = 0; off < n; off += kArgBytes) {
    const int m = (int)(n - off < kArgBytes ? n - off : kArgBytes);
    ArgBytes a;
    memset(&a, 0, sizeof(a));
    memcpy(&a, (const unsigned char*)src + off, (size_t)m);
    k_write_bytes<<<1, 256, 0, s>>>(a, m, (unsigned char*)dst + off);
    HV_CHECK_LAUNCH();
  }
  return HV_OK;
}

extern "C" int hv_attention_general(int dtype, const void* q, const void* k, const void* v,
                                    const unsigned char* key_padding_mask, void* out, float* weights, int n,
                                    int Lq, int Lk, int heads, int hd, float sm_scale, hv_stream_t stream) {
  if (n <= 0 || Lq <= 0 || Lk <= 0 || heads <= 0 || !q || !k || !v || !out) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hv_diag_count(HV_KF_ATTN_GENERAL);
  if (!weights && Lq <= 4 && hd == 32) {      // CLS-query rows: keys split over a workgroup
    HV_DISPATCH(dtype, (k_attention_row<T, 32><<<dim3(Lq, heads, n), 256, 0, s>>>(
                            (const T*)q, (const T*)k, (const T*)v, key_padding_mask, (T*)out, Lq, Lk, heads, sm_scale)));
    HV_CHECK_LAUNCH();
    return HV_OK;
  }
  const dim3 g(hv_cdiv(Lq, 64), heads, n);
#define HV_ATTN_GEN(HDV)                                                                            \
  HV_DISPATCH(dtype, (k_attention_general<T, HDV><<<g, 64, 0, s>>>((const T*)q, (const T*)k, (const T*)v, \
                                                                 key_padding_mask, (T*)out, weights, Lq, Lk,  \
                                                                 heads, sm_scale)))
  if (hd == 16) HV_ATTN_GEN(16);
  else if (hd == 32) HV_ATTN_GEN(32);
  else if (hd == 64) HV_ATTN_GEN(64);
  else return HV_EUNSUPPORTED;
#undef HV_ATTN_GEN
  HV_CHECK_LAUNCH();
  return HV_OK;
}
