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
                                                  int H, int hd, float scale, float p, uint32_t seed, const unsigned int* soff) {
  seed = hv_seed(seed, soff);
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
                                                    uint32_t seed, const unsigned int* soff, T* dq, float* Drow) {
  seed = hv_seed(seed, soff);
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
                                                     float scale, float p, uint32_t seed, const unsigned int* soff, T* dk, T* dv) {
  seed = hv_seed(seed, soff);
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


// =====================================================================================
// MFMA path (bf16, hd = 32) -- the same math as above on the matrix cores.  Layout trick of the
// inference kernel (hv_ops.hip k_attention_mfma): S^T = K Q^T with mfma_f32_16x16x32_bf16 puts
// one query per lane column (lane & 15) and four keys per lane row group in registers; the
// contraction over keys (P V, dS K) then takes those registers directly as the B operand, with
// the key order permuted identically in the A operand read from a transposed, padded
// [b*H][32][Lp] copy (k_tpad).  The key-parallel backward uses S = Q K^T instead (one key per
// lane column, queries in registers) so dV = Pd^T dO and dK = dS^T Q contract over queries the
// same way; dQ comes from a query-parallel pass.  Dropout keep(i, j) and the lse convention are
// those of the scalar kernels above, so either path's forward pairs with either backward.
// transposed, zero-padded copy of one [n, L, H*32] operand: out[(b*H + h)][d][j] (j < Lp)
__global__ void k_tpad(const unsigned short* __restrict__ x, int L, int Lp, int heads, unsigned short* __restrict__ out) {
  const int bh = blockIdx.y;
  const int b = bh / heads, h = bh % heads;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= 32L * Lp) return;
  const int d = (int)(e / Lp), j = (int)(e % Lp);
  out[(long)bh * 32 * Lp + e] = j < L ? x[((long)b * L + j) * heads * 32 + h * 32 + d] : (unsigned short)0;
}

__device__ __forceinline__ f32x4 mfma32(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// A-operand fragment of a transposed [32][Lp] operand: row d, keys {k0 + 4g .. +3, k0 + 16 + 4g .. +3}
__device__ __forceinline__ uint4 tfrag(const unsigned short* t, int Lp, int d, int k0, int g) {
  const unsigned short* r = t + (long)d * Lp + k0 + g * 4;
  const uint2 a = *reinterpret_cast<const uint2*>(r), c = *reinterpret_cast<const uint2*>(r + 16);
  return make_uint4(a.x, a.y, c.x, c.y);
}

__device__ __forceinline__ uint4 rowfrag(const unsigned short* base, long row, int D, int g) {
  return *reinterpret_cast<const uint4*>(base + row * D + g * 8);
}

// forward: wave = 16 queries, online softmax over 32-key tiles; o and lse (natural log of the
// scaled scores) as k_attn_fwd
__global__ void __launch_bounds__(256) k_attn_fwd_mfma(const unsigned short* __restrict__ q,
                                                       const unsigned short* __restrict__ k,
                                                       const unsigned short* __restrict__ vt,
                                                       unsigned short* __restrict__ out, float* __restrict__ lse,
                                                       int L, int Lp, int heads, float sl2, float p, uint32_t seed, const unsigned int* soff) {
  seed = hv_seed(seed, soff);
  const int b = blockIdx.z, h = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int D = heads * 32;
  const int q0 = blockIdx.x * 64 + w * 16;
  if (q0 >= L) return;
  const unsigned short* qb = q + (long)b * L * D + h * 32;
  const unsigned short* kb = k + (long)b * L * D + h * 32;
  const unsigned short* vb = vt + ((long)b * heads + h) * 32 * Lp;
  const int qi = min(q0 + fr, L - 1);
  const uint4 qf = rowfrag(qb, qi, D, fg);
  const unsigned long long rbase = ((unsigned long long)((long)b * heads + h) * L + (q0 + fr)) * L;
  f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += 32) {
    const uint4 kf0 = rowfrag(kb, min(k0 + fr, L - 1), D, fg);
    const uint4 kf1 = rowfrag(kb, min(k0 + 16 + fr, L - 1), D, fg);
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s0 = mfma32(kf0, qf, z), s1 = mfma32(kf1, qf, z);
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
    float pp[8], ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { pp[j] = __builtin_amdgcn_exp2f(t[j] - mn); ps += pp[j]; }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
    if (p > 0.f) {                                        // dropout on the probabilities (1/(1-p) or 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[j] *= hv_drop_scale(seed, rbase + k0 + fg * 4 + j, p);
        pp[4 + j] *= hv_drop_scale(seed, rbase + k0 + 16 + fg * 4 + j, p);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { o0[j] *= corr; o1[j] *= corr; }
    const uint4 pf = make_uint4(pack_bf16x2(pp[0], pp[1]), pack_bf16x2(pp[2], pp[3]), pack_bf16x2(pp[4], pp[5]),
                                pack_bf16x2(pp[6], pp[7]));
    o0 = mfma32(tfrag(vb, Lp, fr, k0, fg), pf, o0);
    o1 = mfma32(tfrag(vb, Lp, 16 + fr, k0, fg), pf, o1);
  }
  if (q0 + fr < L) {
    const float inv = 1.0f / l;
    unsigned short* ob = out + ((long)b * L + q0 + fr) * D + h * 32 + fg * 4;
    *reinterpret_cast<uint2*>(ob) = make_uint2(pack_bf16x2(o0[0] * inv, o0[1] * inv), pack_bf16x2(o0[2] * inv, o0[3] * inv));
    *reinterpret_cast<uint2*>(ob + 16) = make_uint2(pack_bf16x2(o1[0] * inv, o1[1] * inv), pack_bf16x2(o1[2] * inv, o1[3] * inv));
    if (fg == 0) lse[((long)b * heads + h) * L + q0 + fr] = (m + __builtin_amdgcn_logf(l)) * 0.69314718055994531f;
  }
}

// Delta[b, h, i] = sum_j P_ij keep_ij dP_ij with exactly the P (fp32, rebuilt from lse) and dP
// (dO V^T on the MFMA) the dS passes use, so every row of dS = P (keep dP - Delta) sums to zero up
// to fp32 rounding -- as in the reference's autograd, where softmax's backward forms
// sum_j P_ij dP_ij from its own P and dP (manifold_layers.py:417, fp32 under autocast).  The
// FlashAttention shortcut Delta = dO . O (this file's kernel until round 6) takes O as STORED, in bf16, and
// formed with bf16-rounded P: near-uniform attention (dP_ij ~ Delta_i for every key, the state at
// init) turns that 2^-9 mismatch into a large relative error of dS, which the backward carries
// through every earlier block (round 6: the ViT gradient groups at 2.8-3.6x the reference's own
// bf16 error, tools/vit_grad_probe.py).  Wave = 16 queries, loop over 32-key tiles (the dQ
// kernel's layout).
__global__ void __launch_bounds__(256) k_attn_delta_pdp(const unsigned short* __restrict__ q,
                                                        const unsigned short* __restrict__ k,
                                                        const unsigned short* __restrict__ v,
                                                        const unsigned short* __restrict__ dout,
                                                        const float* __restrict__ lse, int L, int heads, float scale,
                                                        float p, uint32_t seed, const unsigned int* soff,
                                                        float* __restrict__ delta) {
  seed = hv_seed(seed, soff);
  const int b = blockIdx.z, h = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int D = heads * 32;
  const int q0 = blockIdx.x * 64 + w * 16;
  if (q0 >= L) return;
  const long bh = (long)b * heads + h;
  const unsigned short* kb = k + (long)b * L * D + h * 32;
  const unsigned short* vb = v + (long)b * L * D + h * 32;
  const int qi = q0 + fr;
  const bool qval = qi < L;
  const uint4 qf = rowfrag(q + (long)b * L * D + h * 32, min(qi, L - 1), D, fg);
  const uint4 gf = rowfrag(dout + (long)b * L * D + h * 32, min(qi, L - 1), D, fg);
  const float l2e = 1.4426950408889634f, sl2 = scale * l2e;
  const float lq = qval ? lse[bh * L + qi] * l2e : 0.f;
  const unsigned long long rbase = ((unsigned long long)(bh * L + qi)) * L;
  float acc = 0.f;
  for (int k0 = 0; k0 < L; k0 += 32) {
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s0 = mfma32(rowfrag(kb, min(k0 + fr, L - 1), D, fg), qf, z);
    const f32x4 s1 = mfma32(rowfrag(kb, min(k0 + 16 + fr, L - 1), D, fg), qf, z);
    const f32x4 g0 = mfma32(rowfrag(vb, min(k0 + fr, L - 1), D, fg), gf, z);
    const f32x4 g1 = mfma32(rowfrag(vb, min(k0 + 16 + fr, L - 1), D, fg), gf, z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int key = k0 + (j < 4 ? 0 : 16) + fg * 4 + (j & 3);
      if (qval && key < L) {
        const float sv = j < 4 ? s0[j] : s1[j - 4];
        const float gv = j < 4 ? g0[j] : g1[j - 4];
        acc = fmaf(__builtin_amdgcn_exp2f(sv * sl2 - lq) * hv_drop_scale(seed, rbase + key, p), gv, acc);
      }
    }
  }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  if (qval && fg == 0) delta[bh * L + qi] = acc;
}

// dK, dV: wave = 16 keys (S = Q K^T layout: key in the lane column, 4 queries per lane row group),
// loop over 32-query tiles
__global__ void __launch_bounds__(256) k_attn_bwd_kv_mfma(const unsigned short* __restrict__ q,
                                                          const unsigned short* __restrict__ k,
                                                          const unsigned short* __restrict__ v,
                                                          const unsigned short* __restrict__ qt,
                                                          const unsigned short* __restrict__ dot,
                                                          const unsigned short* __restrict__ dout,
                                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                                          int L, int Lp, int heads, float scale, float p, uint32_t seed, const unsigned int* soff,
                                                          unsigned short* __restrict__ dk, unsigned short* __restrict__ dv) {
  seed = hv_seed(seed, soff);
  const int b = blockIdx.z, h = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int D = heads * 32;
  const int kb0 = blockIdx.x * 64 + w * 16;
  if (kb0 >= L) return;
  const long bh = (long)b * heads + h;
  const unsigned short* qb = q + (long)b * L * D + h * 32;
  const unsigned short* kbp = k + (long)b * L * D + h * 32;
  const unsigned short* vbp = v + (long)b * L * D + h * 32;
  const unsigned short* dob = dout + (long)b * L * D + h * 32;
  const unsigned short* qtb = qt + bh * 32 * Lp;
  const unsigned short* dotb = dot + bh * 32 * Lp;
  const float* lseb = lse + bh * L;
  const float* delb = delta + bh * L;
  const int key = kb0 + fr;
  const bool kval = key < L;
  const uint4 kf = rowfrag(kbp, min(key, L - 1), D, fg);     // B operand: K^T[d][key]
  const uint4 vf = rowfrag(vbp, min(key, L - 1), D, fg);     // B operand: V^T[d][key]
  const float l2e = 1.4426950408889634f, sl2 = scale * l2e;
  f32x4 dk0 = f32x4{0.f, 0.f, 0.f, 0.f}, dk1 = dk0, dv0 = dk0, dv1 = dk0;
  for (int q0 = 0; q0 < L; q0 += 32) {
    float pd[8], ds[8];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int qa = q0 + half * 16;
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 sv = mfma32(rowfrag(qb, min(qa + fr, L - 1), D, fg), kf, z);    // S[qa + 4fg + j][key]
      const f32x4 dpv = mfma32(rowfrag(dob, min(qa + fr, L - 1), D, fg), vf, z);  // dPd[qa + 4fg + j][key]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qi = qa + fg * 4 + j;
        float P = 0.f, keep = 0.f;
        if (qi < L && kval) {
          P = __builtin_amdgcn_exp2f(sv[j] * sl2 - lseb[qi] * l2e);
          keep = hv_drop_scale(seed, ((unsigned long long)(bh * L + qi)) * L + key, p);   // 1/(1-p) or 0
        }
        pd[half * 4 + j] = P * keep;
        ds[half * 4 + j] = (qi < L && kval) ? P * (dpv[j] * keep - delb[qi]) : 0.f;
      }
    }
    const uint4 pf = make_uint4(pack_bf16x2(pd[0], pd[1]), pack_bf16x2(pd[2], pd[3]), pack_bf16x2(pd[4], pd[5]),
                                pack_bf16x2(pd[6], pd[7]));
    const uint4 sf = make_uint4(pack_bf16x2(ds[0], ds[1]), pack_bf16x2(ds[2], ds[3]), pack_bf16x2(ds[4], ds[5]),
                                pack_bf16x2(ds[6], ds[7]));
    dv0 = mfma32(tfrag(dotb, Lp, fr, q0, fg), pf, dv0);        // dV^T[d][key] += dO^T[d][q] Pd[q][key]
    dv1 = mfma32(tfrag(dotb, Lp, 16 + fr, q0, fg), pf, dv1);
    dk0 = mfma32(tfrag(qtb, Lp, fr, q0, fg), sf, dk0);         // dK^T[d][key] += Q^T[d][q] dS[q][key]
    dk1 = mfma32(tfrag(qtb, Lp, 16 + fr, q0, fg), sf, dk1);
  }
  if (kval) {
    unsigned short* kr = dk + ((long)b * L + key) * D + h * 32 + fg * 4;
    unsigned short* vr = dv + ((long)b * L + key) * D + h * 32 + fg * 4;
    *reinterpret_cast<uint2*>(kr) = make_uint2(pack_bf16x2(dk0[0] * scale, dk0[1] * scale), pack_bf16x2(dk0[2] * scale, dk0[3] * scale));
    *reinterpret_cast<uint2*>(kr + 16) = make_uint2(pack_bf16x2(dk1[0] * scale, dk1[1] * scale), pack_bf16x2(dk1[2] * scale, dk1[3] * scale));
    *reinterpret_cast<uint2*>(vr) = make_uint2(pack_bf16x2(dv0[0], dv0[1]), pack_bf16x2(dv0[2], dv0[3]));
    *reinterpret_cast<uint2*>(vr + 16) = make_uint2(pack_bf16x2(dv1[0], dv1[1]), pack_bf16x2(dv1[2], dv1[3]));
  }
}

// dQ: wave = 16 queries (S^T layout as the forward), loop over 32-key tiles
__global__ void __launch_bounds__(256) k_attn_bwd_q_mfma(const unsigned short* __restrict__ q,
                                                         const unsigned short* __restrict__ k,
                                                         const unsigned short* __restrict__ v,
                                                         const unsigned short* __restrict__ kt,
                                                         const unsigned short* __restrict__ dout,
                                                         const float* __restrict__ lse, const float* __restrict__ delta,
                                                         int L, int Lp, int heads, float scale, float p, uint32_t seed, const unsigned int* soff,
                                                         unsigned short* __restrict__ dq) {
  seed = hv_seed(seed, soff);
  const int b = blockIdx.z, h = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fg = lane >> 4;
  const int D = heads * 32;
  const int q0 = blockIdx.x * 64 + w * 16;
  if (q0 >= L) return;
  const long bh = (long)b * heads + h;
  const unsigned short* kb = k + (long)b * L * D + h * 32;
  const unsigned short* vb = v + (long)b * L * D + h * 32;
  const unsigned short* ktb = kt + bh * 32 * Lp;
  const int qi = q0 + fr;
  const bool qval = qi < L;
  const uint4 qf = rowfrag(q + (long)b * L * D + h * 32, min(qi, L - 1), D, fg);
  const uint4 gf = rowfrag(dout + (long)b * L * D + h * 32, min(qi, L - 1), D, fg);
  const float l2e = 1.4426950408889634f, sl2 = scale * l2e;
  const float lq = qval ? lse[bh * L + qi] * l2e : 0.f;
  const float dq_delta = qval ? delta[bh * L + qi] : 0.f;
  const unsigned long long rbase = ((unsigned long long)(bh * L + qi)) * L;
  f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  for (int k0 = 0; k0 < L; k0 += 32) {
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s0 = mfma32(rowfrag(kb, min(k0 + fr, L - 1), D, fg), qf, z);
    const f32x4 s1 = mfma32(rowfrag(kb, min(k0 + 16 + fr, L - 1), D, fg), qf, z);
    const f32x4 g0 = mfma32(rowfrag(vb, min(k0 + fr, L - 1), D, fg), gf, z);
    const f32x4 g1 = mfma32(rowfrag(vb, min(k0 + 16 + fr, L - 1), D, fg), gf, z);
    float ds[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int key = k0 + (j < 4 ? 0 : 16) + fg * 4 + (j & 3);
      const float sv = j < 4 ? s0[j] : s1[j - 4];
      const float gv = j < 4 ? g0[j] : g1[j - 4];
      float d = 0.f;
      if (qval && key < L) {
        const float P = __builtin_amdgcn_exp2f(sv * sl2 - lq);
        const float keep = hv_drop_scale(seed, rbase + key, p);
        d = P * (gv * keep - dq_delta);
      }
      ds[j] = d;
    }
    const uint4 sf = make_uint4(pack_bf16x2(ds[0], ds[1]), pack_bf16x2(ds[2], ds[3]), pack_bf16x2(ds[4], ds[5]),
                                pack_bf16x2(ds[6], ds[7]));
    a0 = mfma32(tfrag(ktb, Lp, fr, k0, fg), sf, a0);          // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
    a1 = mfma32(tfrag(ktb, Lp, 16 + fr, k0, fg), sf, a1);
  }
  if (qval) {
    unsigned short* r = dq + ((long)b * L + qi) * D + h * 32 + fg * 4;
    *reinterpret_cast<uint2*>(r) = make_uint2(pack_bf16x2(a0[0] * scale, a0[1] * scale), pack_bf16x2(a0[2] * scale, a0[3] * scale));
    *reinterpret_cast<uint2*>(r + 16) = make_uint2(pack_bf16x2(a1[0] * scale, a1[1] * scale), pack_bf16x2(a1[2] * scale, a1[3] * scale));
  }
}

}  // namespace

extern "C" size_t hv_attention_train_mfma_work_elems(int n, int L, int heads) {
  const long Lp = (L + 31) / 32 * 32;
  return (size_t)n * heads * 32 * Lp;     // one transposed padded operand (bf16 elements)
}

extern "C" int hv_attention_train_mfma(const void* q, const void* k, const void* v, void* o, float* lse, int n, int L,
                                       int heads, float sm_scale, float drop_p, unsigned int seed,
                                       const unsigned int* seed_offset, void* vt_work,
                                       hv_stream_t stream) {
  if (!q || !k || !v || !o || !lse || !vt_work || n <= 0 || L <= 0 || heads <= 0) return HV_EINVAL;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o | (uintptr_t)vt_work) & 15) return HV_EUNSUPPORTED;
  const int Lp = (L + 31) / 32 * 32;
  hipStream_t s = (hipStream_t)stream;
  hv_diag_count(HV_KF_ATTN_MFMA);
  k_tpad<<<dim3(hv_cdiv(32L * Lp, 256), n * heads), 256, 0, s>>>((const unsigned short*)v, L, Lp, heads,
                                                                (unsigned short*)vt_work);
  k_attn_fwd_mfma<<<dim3(hv_cdiv(L, 64), heads, n), 256, 0, s>>>(
      (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)vt_work, (unsigned short*)o, lse, L, Lp,
      heads, sm_scale * 1.4426950408889634f, drop_p, seed, seed_offset);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

/* work: 3 transposed padded operands (bf16, 3 * hv_attention_train_mfma_work_elems) then n*heads*L
   floats (Delta) */
extern "C" int hv_attention_backward_mfma(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                          const float* lse, int n, int L, int heads, float sm_scale, float drop_p,
                                          unsigned int seed, const unsigned int* seed_offset, void* dq, void* dk,
                                          void* dv, void* work, hv_stream_t stream) {
  if (!q || !k || !v || !o || !dout || !lse || !dq || !dk || !dv || !work || n <= 0 || L <= 0) return HV_EINVAL;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o | (uintptr_t)dout | (uintptr_t)work | (uintptr_t)dq |
       (uintptr_t)dk | (uintptr_t)dv) & 15)
    return HV_EUNSUPPORTED;
  const int Lp = (L + 31) / 32 * 32;
  const size_t te = hv_attention_train_mfma_work_elems(n, L, heads);
  unsigned short* qt = (unsigned short*)work;
  unsigned short* kt = qt + te;
  unsigned short* dot = kt + te;
  float* delta = (float*)(dot + te);
  hipStream_t s = (hipStream_t)stream;
  hv_diag_count(HV_KF_ATTN_MFMA);
  const dim3 tg(hv_cdiv(32L * Lp, 256), n * heads);
  k_tpad<<<tg, 256, 0, s>>>((const unsigned short*)q, L, Lp, heads, qt);
  k_tpad<<<tg, 256, 0, s>>>((const unsigned short*)k, L, Lp, heads, kt);
  k_tpad<<<tg, 256, 0, s>>>((const unsigned short*)dout, L, Lp, heads, dot);
  const dim3 g(hv_cdiv(L, 64), heads, n);
  k_attn_delta_pdp<<<g, 256, 0, s>>>((const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v,
                                     (const unsigned short*)dout, lse, L, heads, sm_scale, drop_p, seed, seed_offset,
                                     delta);
  k_attn_bwd_kv_mfma<<<g, 256, 0, s>>>((const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, qt,
                                       dot, (const unsigned short*)dout, lse, delta, L, Lp, heads, sm_scale, drop_p,
                                       seed, seed_offset, (unsigned short*)dk, (unsigned short*)dv);
  k_attn_bwd_q_mfma<<<g, 256, 0, s>>>((const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, kt,
                                      (const unsigned short*)dout, lse, delta, L, Lp, heads, sm_scale, drop_p, seed,
                                      seed_offset, (unsigned short*)dq);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_attention_train(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int n,
                                  int L, int heads, int hd, float sm_scale, float drop_p, unsigned int seed,
                                  const unsigned int* seed_offset, hv_stream_t stream) {
  if (!q || !k || !v || !o || !lse || hd != 32) return HV_EINVAL;
  const unsigned grid = hv_cdiv((long)n * heads * L, 4);
  HV_DISPATCH(dtype, (k_attn_fwd<T, 32><<<grid, 256, 0, (hipStream_t)stream>>>((const T*)q, (const T*)k, (const T*)v,
                                                                           (T*)o, lse, n, L, heads, hd, sm_scale,
                                                                           drop_p, seed, seed_offset)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_attention_backward(int dtype, const void* q, const void* k, const void* v, const void* o,
                                     const void* dout, const float* lse, int n, int L, int heads, int hd,
                                     float sm_scale, float drop_p, unsigned int seed, const unsigned int* seed_offset,
                                     void* dq, void* dk, void* dv, float* work, hv_stream_t stream) {
  if (!q || !k || !v || !o || !dout || !lse || !dq || !dk || !dv || !work || hd != 32) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = hv_cdiv((long)n * heads * L, 4);
  HV_DISPATCH(dtype, (k_attn_bwd_q<T, 32><<<grid, 256, 0, s>>>((const T*)q, (const T*)k, (const T*)v, (const T*)o,
                                                           (const T*)dout, lse, n, L, heads, hd, sm_scale, drop_p,
                                                           seed, seed_offset, (T*)dq, work)));
  HV_DISPATCH(dtype, (k_attn_bwd_kv<T, 32><<<grid, 256, 0, s>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout,
                                                            lse, work, n, L, heads, hd, sm_scale, drop_p, seed,
                                                            seed_offset, (T*)dk, (T*)dv)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}
