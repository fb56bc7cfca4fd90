// Epilogue shared by the two MFMA GEMM kernels (hv_gemm.hip, hv_gemm_glds.hip).
//
//   acc' = acc                                        (plain / LN-prologue kernels)
//        = rstd[m] * (acc - mean[m] * colsum[n])      (LN_EPI: LayerNorm of A applied AFTER the
//                                                      product -- exact because
//                                                      ((a - mean) rstd) . b = rstd (a.b - mean sum(b)))
//   v = act(alpha * scale[n] * acc' + bias[n])  (+ residual[m or m % r_mod, n])  -> c_dtype
//   (GELU into a bf16 result without residual uses hv_gelu_fast, |err| <= 2.6e-5)
//
// Both kernels accumulate every 16x16 sub-tile TRANSPOSED (B fragment as the MFMA A operand),
// so a lane holds 4 consecutive columns of one row: one 8-byte (bf16) or 16-byte (fp32)
// store per sub-tile instead of four scattered 2-byte stores, and one LN row statistic.
#pragma once
#include "hv_common.h"

// Training epilogue modes (hv_gemm_desc.epi_mode 1/2, see hv_kernels.h).  A lane holds 4
// consecutive columns: the pre-activation is stored / loaded as one 8-byte (bf16) or 16-byte
// (fp32) vector when the row allows it.
__device__ __forceinline__ f32x4 epi_train(const hv_gemm_desc& d, const f32x4 acc, int row, int col, const f32x4 sc,
                                           const f32x4 bi, const f32x4 cs, float mean, float rstd, bool ln_epi) {
  f32x4 v;
  const bool aux_bf = d.aux_dtype == HV_BF16;
  const bool vec = col + 4 <= d.N && (d.ld_aux & 3) == 0 && ((((uintptr_t)d.aux) & 15) == 0);
  const long ai = (long)row * d.ld_aux + col;
  const unsigned long long idx0 = (unsigned long long)row * d.N + col;
  float z[4];
  if (d.epi_mode == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = acc[j];
      if (ln_epi) x = rstd * (x - mean * cs[j]);
      z[j] = x * sc[j] + bi[j];
    }
    if (vec) {
      if (aux_bf) {
        const uint2 pk = make_uint2(pack_bf16x2(z[0], z[1]), pack_bf16x2(z[2], z[3]));
        *reinterpret_cast<uint2*>((unsigned short*)d.aux + ai) = pk;
        // the activation sees the value the backward will see (rounded when stored in bf16)
        z[0] = __uint_as_float(pk.x << 16); z[1] = __uint_as_float(pk.x & 0xffff0000u);
        z[2] = __uint_as_float(pk.y << 16); z[3] = __uint_as_float(pk.y & 0xffff0000u);
      } else {
        *reinterpret_cast<float4*>((float*)d.aux + ai) = make_float4(z[0], z[1], z[2], z[3]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (col + j >= d.N) break;
        if (aux_bf) {
          ((unsigned short*)d.aux)[ai + j] = f2bf(z[j]);
          z[j] = bf2f(f2bf(z[j]));
        } else {
          ((float*)d.aux)[ai + j] = z[j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = hv_act(z[j], d.act) * hv_drop_scale(d.drop_seed, idx0 + j, d.drop_p);
  } else {
    if (vec) {
      if (aux_bf) {
        const uint2 t = *reinterpret_cast<const uint2*>((const unsigned short*)d.aux + ai);
        z[0] = __uint_as_float(t.x << 16); z[1] = __uint_as_float(t.x & 0xffff0000u);
        z[2] = __uint_as_float(t.y << 16); z[3] = __uint_as_float(t.y & 0xffff0000u);
      } else {
        const float4 t = *reinterpret_cast<const float4*>((const float*)d.aux + ai);
        z[0] = t.x; z[1] = t.y; z[2] = t.z; z[3] = t.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        z[j] = col + j < d.N ? (aux_bf ? bf2f(((const unsigned short*)d.aux)[ai + j]) : ((const float*)d.aux)[ai + j])
                             : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = acc[j] * d.alpha * hv_drop_scale(d.drop_seed, idx0 + j, d.drop_p) * hv_act_grad(z[j], d.act);
  }
  return v;
}

// Per-lane column constants of the epilogue (scale * alpha, bias, LN column sums).
template <int RN>
struct EpiCols {
  float sc[RN][4], bi[RN][4], cs[RN][4];
};

// One 16-row sub-tile row A of the wave's accumulators.  The row-tile index is a template
// parameter (instantiated A = 0 .. RM-1 by epi_rows), so every acc[A][b] is a constant index:
// a runtime-indexed row loop that the unroller declines (large RM x RN x body) would leave the
// accumulator array in scratch memory.
template <int A, bool LN_EPI, bool TRAIN, int WN, int RM, int RN>
__device__ __forceinline__ void epi_rowtile(const hv_gemm_desc& d, const f32x4 (&acc)[RM][RN], const EpiCols<RN>& k,
                                            int m0, int n0) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid / WN, wc = wid % WN;
  const int fr = lane & 15, fg = lane >> 4;
  const bool c_bf = d.c_dtype == HV_BF16, r_bf = d.r_dtype == HV_BF16;
  const bool gelu_fast = c_bf && !d.residual;
  const bool vec = (((uintptr_t)d.C) & 15) == 0 && d.ldc % 4 == 0 &&
                   (!d.residual || ((((uintptr_t)d.residual) & 15) == 0 && d.ldr % 4 == 0));
  const int row = m0 + wr * (RM * 16) + A * 16 + fr;
  if (row >= d.M) return;
  float mean = 0.f, rstd = 1.f;
  if constexpr (LN_EPI) {
    mean = d.a_mean[row];
    rstd = d.a_rstd[row];
  }
  const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
#pragma unroll
  for (int b = 0; b < RN; ++b) {
    const int col = n0 + wc * (RN * 16) + b * 16 + fg * 4;
    if (col >= d.N) continue;
    float v[4];
    if constexpr (!TRAIN) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = acc[A][b][j];
        if constexpr (LN_EPI) x = rstd * (x - mean * k.cs[b][j]);
        x = x * k.sc[b][j] + k.bi[b][j];
        v[j] = (gelu_fast && d.act == HV_ACT_GELU) ? hv_gelu_fast(x) : hv_act(x, d.act);
      }
    } else {
      const f32x4 t = epi_train(d, acc[A][b], row, col, f32x4{k.sc[b][0], k.sc[b][1], k.sc[b][2], k.sc[b][3]},
                                f32x4{k.bi[b][0], k.bi[b][1], k.bi[b][2], k.bi[b][3]},
                                f32x4{k.cs[b][0], k.cs[b][1], k.cs[b][2], k.cs[b][3]}, mean, rstd, LN_EPI);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    }
    if (vec && col + 4 <= d.N) {
      if (d.residual) {
        if (r_bf) {
          const uint2 r = *reinterpret_cast<const uint2*>((const unsigned short*)d.residual + rrow * d.ldr + col);
          v[0] += __uint_as_float(r.x << 16);
          v[1] += __uint_as_float(r.x & 0xffff0000u);
          v[2] += __uint_as_float(r.y << 16);
          v[3] += __uint_as_float(r.y & 0xffff0000u);
        } else {
          const float4 r = *reinterpret_cast<const float4*>((const float*)d.residual + rrow * d.ldr + col);
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
      }
      if (c_bf)
        *reinterpret_cast<uint2*>((unsigned short*)d.C + (long)row * d.ldc + col) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      else
        *reinterpret_cast<float4*>((float*)d.C + (long)row * d.ldc + col) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (col + j >= d.N) break;
        float x = v[j];
        if (d.residual)
          x += r_bf ? bf2f(((const unsigned short*)d.residual)[rrow * d.ldr + col + j])
                    : ((const float*)d.residual)[rrow * d.ldr + col + j];
        const long o = (long)row * d.ldc + col + j;
        if (c_bf) ((unsigned short*)d.C)[o] = f2bf(x);
        else ((float*)d.C)[o] = x;
      }
    }
  }
}

template <int A, bool LN_EPI, bool TRAIN, int WN, int RM, int RN>
__device__ __forceinline__ void epi_rows(const hv_gemm_desc& d, const f32x4 (&acc)[RM][RN], const EpiCols<RN>& k,
                                         int m0, int n0) {
  if constexpr (A < RM) {
    epi_rowtile<A, LN_EPI, TRAIN, WN, RM, RN>(d, acc, k, m0, n0);
    epi_rows<A + 1, LN_EPI, TRAIN, WN, RM, RN>(d, acc, k, m0, n0);
  }
}

// WN waves along N (WM = waves / WN along M); every wave owns an (RM*16) x (RN*16) sub-tile.
template <int BM, int BN, bool LN_EPI, bool TRAIN = false, int WN = 2, int RM = BM / 32, int RN = BN / 32>
__device__ __forceinline__ void gemm_epilogue(const hv_gemm_desc& d, const f32x4 (&acc)[RM][RN],
                                              int m0, int n0) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wc = wid % WN;
  const int fg = lane >> 4;
  EpiCols<RN> k;
#pragma unroll
  for (int b = 0; b < RN; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * (RN * 16) + b * 16 + fg * 4 + j;
      const bool ok = col < d.N;
      k.sc[b][j] = (d.scale && ok) ? d.scale[col] * d.alpha : d.alpha;
      k.bi[b][j] = (d.bias && ok) ? d.bias[col] : 0.f;
      k.cs[b][j] = 0.f;
      if constexpr (LN_EPI) k.cs[b][j] = ok ? d.b_colsum[col] : 0.f;
    }
  epi_rows<0, LN_EPI, TRAIN, WN, RM, RN>(d, acc, k, m0, n0);
}
