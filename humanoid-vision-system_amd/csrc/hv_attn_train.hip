// Attention of MultiHeadManifoldAttention in training mode (manifold_layers.py:404-427):
// softmax(q k^T * scale) with dropout on the probabilities (:418), times v; and its backward.
// q/k/v/o token-major [n, L, heads*hd] (the layout the mHC projections produce), hd <= 64.
// One wave per query row (forward, dq) or key row (dk, dv); lanes sweep the other index.
// The forward stores lse = log-sum-exp of the scaled scores so the backward rebuilds P
// exactly; the dropout mask is regenerated from (seed, ((b*H + h)*L + i)*L + j).
#include "hv_common.h"

namespace {


template <typename T> __device__ __forceinline__ float ldv(const T* p, long i);
template <> __device__ __forceinline__ float ldv<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ldv<unsigned short>(const unsigned short* p, long i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void stv(T* p, long i, float v);
template <> __device__ __forceinline__ void stv<float>(float* p, long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stv<unsigned short>(unsigned short* p, long i, float v) { p[i] = f2bf(v); }

template <typename T, int HD>
__device__ __forceinline__ float dot_row(const float* a, const T* row) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < HD; ++d) s += a[d] * ldv<T>(row, d);
  return s;
}

// forward: wave per (b, h, i)
template <typename T, int HD>
__global__ void __launch_bounds__(256) k_attn_fwd(const T* q, const T* k, const T* v, T* o, float* lse, int n, int L,
                                                  int H, int hd, float scale, float p, uint32_t seed) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)n * H * L) return;
  const int i = (int)(row % L);
  const int h = (int)((row / L) % H);
  const int b = (int)(row / ((long)L * H));
  const int D = H * hd;
  float qi[HD];
  const T* qrow = q + ((long)b * L + i) * D + h * hd;
  _Pragma("unroll") for (int d = 0; d < HD; ++d) qi[d] = ldv<T>(qrow, d) * scale;
  float mx = -INFINITY;
  for (int j = lane; j < L; j += 64) mx = fmaxf(mx, dot_row<T, HD>(qi, k + ((long)b * L + j) * D + h * hd));
  mx = wave_max(mx);
  float se = 0.f;
  for (int j = lane; j < L; j += 64) se += __expf(dot_row<T, HD>(qi, k + ((long)b * L + j) * D + h * hd) - mx);
  se = wave_sum(se);
  const float l = mx + __logf(se);
  float acc[HD];
  _Pragma("unroll") for (int d = 0; d < HD; ++d) acc[d] = 0.f;
  const unsigned long long base = (unsigned long long)row * L;
  for (int j = lane; j < L; j += 64) {
    const float s = dot_row<T, HD>(qi, k + ((long)b * L + j) * D + h * hd);
    const float pj = __expf(s - l) * hv_drop_scale(seed, base + j, p);
    const T* vr = v + ((long)b * L + j) * D + h * hd;
    _Pragma("unroll") for (int d = 0; d < HD; ++d) acc[d] += pj * ldv<T>(vr, d);
  }
  T* orow = o + ((long)b * L + i) * D + h * hd;
  _Pragma("unroll") for (int d = 0; d < HD; ++d) {
    const float t = wave_sum(acc[d]);
    if (lane == 0) stv<T>(orow, d, t);
  }
  if (lane == 0) lse[row] = l;
}

// dq and Drow = dout . o: wave per query row
template <typename T, int HD>
__global__ void __launch_bounds__(256) k_attn_bwd_q(const T* q, const T* k, const T* v, const T* o, const T* dout,
                                                    const float* lse, int n, int L, int H, int hd, float scale, float p,
                                                    uint32_t seed, T* dq, float* Drow) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long)n * H * L) return;
  const int i = (int)(row % L);
  const int h = (int)((row / L) % H);
  const int b = (int)(row / ((long)L * H));
  const int D = H * hd;
  const long off = ((long)b * L + i) * D + h * hd;
  float qi[HD], gi[HD], acc[HD];
  float Di = 0.f;
  _Pragma("unroll") for (int d = 0; d < HD; ++d) {
    qi[d] = ldv<T>(q + off, d) * scale;
    gi[d] = ldv<T>(dout + off, d);
    Di += gi[d] * ldv<T>(o + off, d);
    acc[d] = 0.f;
  }
  const float l = lse[row];
  const unsigned long long base = (unsigned long long)row * L;
  for (int j = lane; j < L; j += 64) {
    const T* kr = k + ((long)b * L + j) * D + h * hd;
    const T* vr = v + ((long)b * L + j) * D + h * hd;
    const float P = __expf(dot_row<T, HD>(qi, kr) - l);
    const float dP = dot_row<T, HD>(gi, vr) * hv_drop_scale(seed, base + j, p);
    const float dS = P * (dP - Di);
    _Pragma("unroll") for (int d = 0; d < HD; ++d) acc[d] += dS * ldv<T>(kr, d);
  }
  _Pragma("unroll") for (int d = 0; d < HD; ++d) {
    const float t = wave_sum(acc[d]);
    if (lane == 0) stv<T>(dq + off, d, t * scale);
  }
  if (lane == 0) Drow[row] = Di;
}

// dk, dv: wave per key row
template <typename T, int HD>
__global__ void __launch_bounds__(256) k_attn_bwd_kv(const T* q, const T* k, const T* v, const T* dout,
                                                     const float* lse, const float* Drow, int n, int L, int H, int hd,
                                                     float scale, float p, uint32_t seed, T* dk, T* dv) {
  const long krow = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (krow >= (long)n * H * L) return;
  const int j = (int)(krow % L);
  const int h = (int)((krow / L) % H);
  const int b = (int)(krow / ((long)L * H));
  const int D = H * hd;
  const long off = ((long)b * L + j) * D + h * hd;
  float kj[HD], vj[HD], ak[HD], av[HD];
  _Pragma("unroll") for (int d = 0; d < HD; ++d) {
    kj[d] = ldv<T>(k + off, d);
    vj[d] = ldv<T>(v + off, d);
    ak[d] = 0.f;
    av[d] = 0.f;
  }
  const long rbase = ((long)b * H + h) * L;      // query rows of this (b, h)
  for (int i = lane; i < L; i += 64) {
    const T* qr = q + ((long)b * L + i) * D + h * hd;
    const T* gr = dout + ((long)b * L + i) * D + h * hd;
    const float s = dot_row<T, HD>(kj, qr) * scale;
    const float P = __expf(s - lse[rbase + i]);
    const float m = hv_drop_scale(seed, (unsigned long long)(rbase + i) * L + j, p);
    const float dP = dot_row<T, HD>(vj, gr) * m;
    const float dS = P * (dP - Drow[rbase + i]);
    const float pm = P * m;
    _Pragma("unroll") for (int d = 0; d < HD; ++d) {
      ak[d] += dS * ldv<T>(qr, d);
      av[d] += pm * ldv<T>(gr, d);
    }
  }
  _Pragma("unroll") for (int d = 0; d < HD; ++d) {
    const float t1 = wave_sum(ak[d]);
    const float t2 = wave_sum(av[d]);
    if (lane == 0) {
      stv<T>(dk + off, d, t1 * scale);
      stv<T>(dv + off, d, t2);
    }
  }
}

}  // namespace

extern "C" int hv_attention_train(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int n,
                                  int L, int heads, int hd, float sm_scale, float drop_p, unsigned int seed,
                                  hv_stream_t stream) {
  if (!q || !k || !v || !o || !lse || hd != 32) return HV_EINVAL;
  const unsigned grid = hv_cdiv((long)n * heads * L, 4);
  HV_DISPATCH(dtype, (k_attn_fwd<T, 32><<<grid, 256, 0, (hipStream_t)stream>>>((const T*)q, (const T*)k, (const T*)v,
                                                                           (T*)o, lse, n, L, heads, hd, sm_scale,
                                                                           drop_p, seed)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_attention_backward(int dtype, const void* q, const void* k, const void* v, const void* o,
                                     const void* dout, const float* lse, int n, int L, int heads, int hd,
                                     float sm_scale, float drop_p, unsigned int seed, void* dq, void* dk, void* dv,
                                     float* work, hv_stream_t stream) {
  if (!q || !k || !v || !o || !dout || !lse || !dq || !dk || !dv || !work || hd != 32) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = hv_cdiv((long)n * heads * L, 4);
  HV_DISPATCH(dtype, (k_attn_bwd_q<T, 32><<<grid, 256, 0, s>>>((const T*)q, (const T*)k, (const T*)v, (const T*)o,
                                                           (const T*)dout, lse, n, L, heads, hd, sm_scale, drop_p,
                                                           seed, (T*)dq, work)));
  HV_DISPATCH(dtype, (k_attn_bwd_kv<T, 32><<<grid, 256, 0, s>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout,
                                                            lse, work, n, L, heads, hd, sm_scale, drop_p, seed,
                                                            (T*)dk, (T*)dv)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}
