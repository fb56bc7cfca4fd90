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
// dropout seed of a training epilogue (hv_gemm_desc.drop_seed + *seed_offset), loaded once
__device__ __forceinline__ uint32_t epi_seed(const hv_gemm_desc& d) {
  return d.drop_p > 0.f ? hv_seed(d.drop_seed, d.seed_offset) : 0u;
}

// Training activations: bf16 outputs take the fast GELU (|err| <= 2.6e-5, far below bf16
// resolution) and its exact derivative in the backward, as the inference epilogue does -- the
// erf form and its derivative were ~60 VALU instructions per element of the write-bound
// training GEMMs; fp32 (parity) outputs keep the exact erf GELU.
__device__ __forceinline__ float epi_train_act(const hv_gemm_desc& d, float z) {
  return (d.act == HV_ACT_GELU && d.c_dtype == HV_BF16) ? hv_gelu_fast(z) : hv_act(z, d.act);
}
// the backward differentiates the GELU its forward ran: that forward wrote its output in the dtype
// of the stored pre-activation (aux, every mode-1 caller), which is not necessarily the dtype of
// this launch's dX (c_dtype) -- the form is keyed on aux_dtype, as k_act_bwd keys on the pre-act
__device__ __forceinline__ float epi_train_act_grad(const hv_gemm_desc& d, float z) {
  return (d.act == HV_ACT_GELU && d.aux_dtype == HV_BF16) ? hv_gelu_grad_fast(z) : hv_act_grad(z, d.act);
}

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
    const uint32_t sd_ = epi_seed(d);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = epi_train_act(d, z[j]) * hv_drop_scale(sd_, idx0 + j, d.drop_p);
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
    const uint32_t sd_ = epi_seed(d);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = acc[j] * d.alpha * hv_drop_scale(sd_, idx0 + j, d.drop_p) * epi_train_act_grad(d, z[j]);
  }
  return v;
}

// Per-lane column constants of the epilogue (scale * alpha, bias, LN column sums).
template <int RN>
struct EpiCols {
  float sc[RN][4], bi[RN][4], cs[RN][4];
};

// Column (cbase + b*16 + j) constants as ONE batch of independent loads: clamped column indices,
// a uniform branch per (possibly null) array, bounds applied afterwards.  Written per element as
// `p && col < N ? p[col] : x`, hipcc branches around every load and waits vmcnt(0) inside each
// branch -- 16-48 serialized round trips per epilogue (round-2 ISA of every GEMM kernel).
template <int RN, bool LN_EPI>
__device__ __forceinline__ void epi_load_cols(const hv_gemm_desc& d, EpiCols<RN>& k, int cbase) {
  int cc[RN][4];
#pragma unroll
  for (int b = 0; b < RN; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) cc[b][j] = min(cbase + b * 16 + j, d.N - 1);
  if (d.scale) {
#pragma unroll
    for (int b = 0; b < RN; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) k.sc[b][j] = d.scale[cc[b][j]];
  } else {
#pragma unroll
    for (int b = 0; b < RN; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) k.sc[b][j] = 1.f;
  }
  if (d.bias) {
#pragma unroll
    for (int b = 0; b < RN; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) k.bi[b][j] = d.bias[cc[b][j]];
  } else {
#pragma unroll
    for (int b = 0; b < RN; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) k.bi[b][j] = 0.f;
  }
#pragma unroll
  for (int b = 0; b < RN; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) k.cs[b][j] = LN_EPI ? d.b_colsum[cc[b][j]] : 0.f;
#pragma unroll
  for (int b = 0; b < RN; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = cbase + b * 16 + j < d.N;
      k.sc[b][j] = d.scale && ok ? k.sc[b][j] * d.alpha : d.alpha;
      k.bi[b][j] = ok ? k.bi[b][j] : 0.f;
      k.cs[b][j] = ok ? k.cs[b][j] : 0.f;
    }
}

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
  epi_load_cols<RN, LN_EPI>(d, k, n0 + wc * (RN * 16) + fg * 4);
  epi_rows<0, LN_EPI, TRAIN, WN, RM, RN>(d, acc, k, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// LDS-staged epilogue (inference modes, epi_mode 0).  The fragment layout above writes 16 rows x
// 32 bytes per store instruction, which holds the GEMM's output stream to ~1 TB/s; here each wave
// first writes v = act(scale * acc' + bias) as fp32 into an LDS image of SLAB rows x BN columns
// (16-B chunk c of row r at c ^ (r & 7): conflict-free float4 writes), then every thread of the
// workgroup streams whole rows out: 8 consecutive columns per thread, residual read with one
// 16-B load, one 16-B bf16 (or two fp32) store.  Same arithmetic, same rounding as gemm_epilogue
// (bit-identical outputs).  The slab is the tile (SLAB = BM) or, for the 256x256 kernel, one wave
// group's 128 rows at a time; `smem` must hold SLAB * BN * 4 bytes and be free (no DMA in flight,
// no pending reads) -- the caller's last barrier guarantees that.
// 16-B chunk c of LDS-image row r (CPR chunks per row) lives at c ^ (r & 7)
template <int CPR>
__device__ __forceinline__ float4* epi_lds_chunk(unsigned char* smem, int r, int c) {
  return reinterpret_cast<float4*>(smem + ((long)r * CPR + (c ^ (r & 7))) * 16);
}

// Row tile A of the wave's accumulators -> LDS image rows lrow0 + A*16 + fr (fp32, activation
// applied).  Template recursion over A keeps every acc index a constant.
template <int A, bool LN_EPI, int RM, int RN, int CPR, bool TRAIN = false>
__device__ __forceinline__ void epi_stage_rows(const hv_gemm_desc& d, const f32x4 (&acc)[RM][RN], const EpiCols<RN>& k,
                                               int grow0, int lrow0, int lcol0, unsigned char* smem) {
  if constexpr (A < RM) {
    const int lane = threadIdx.x & 63, fr = lane & 15, fg = lane >> 4;
    const bool gelu_fast = d.c_dtype == HV_BF16 && !d.residual;
    const int row = grow0 + A * 16 + fr;
    float mean = 0.f, rstd = 1.f;
    if constexpr (LN_EPI) {
      const int rr = row < d.M ? row : d.M - 1;
      mean = d.a_mean[rr];
      rstd = d.a_rstd[rr];
    }
#pragma unroll
    for (int b = 0; b < RN; ++b) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = acc[A][b][j];
        if constexpr (TRAIN) {
          // training modes stage the pre-activation (mode 1) / the scaled product (mode 2); the
          // write-out applies act + dropout (or their backward) on whole rows
          if (d.epi_mode == 1) {
            if constexpr (LN_EPI) x = rstd * (x - mean * k.cs[b][j]);
            v[j] = x * k.sc[b][j] + k.bi[b][j];
          } else {
            v[j] = x * d.alpha;
          }
        } else {
          if constexpr (LN_EPI) x = rstd * (x - mean * k.cs[b][j]);
          x = x * k.sc[b][j] + k.bi[b][j];
          v[j] = (gelu_fast && d.act == HV_ACT_GELU) ? hv_gelu_fast(x) : hv_act(x, d.act);
        }
      }
      *epi_lds_chunk<CPR>(smem, lrow0 + A * 16 + fr, (lcol0 + b * 16) / 4 + fg) = make_float4(v[0], v[1], v[2], v[3]);
    }
    epi_stage_rows<A + 1, LN_EPI, RM, RN, CPR, TRAIN>(d, acc, k, grow0, lrow0, lcol0, smem);
  }
}

// Coalesced write-out of an LDS image of SLAB rows (tile rows r0 ..) x BN columns.
// training write-out of 8 staged values (row, col .. col+7): mode 1 stores the pre-activation z
// to aux (rounded like the fragment epilogue) and returns act(z) * keep; mode 2 reads aux and
// returns z * keep * act'(aux).  keep(m, n) = hv_drop_scale(seed, m * N + n), as epi_train.
__device__ __forceinline__ void epi_train8(const hv_gemm_desc& d, float (&v)[8], int row, int col, bool vec8) {
  const bool aux_bf = d.aux_dtype == HV_BF16;
  const long ai = (long)row * d.ld_aux + col;
  const unsigned long long idx0 = (unsigned long long)row * d.N + col;
  const bool av = vec8 && (d.ld_aux & 7) == 0 && ((((uintptr_t)d.aux) & 15) == 0);
  float z[8];
  if (d.epi_mode == 1) {
    if (av && aux_bf) {
      const uint4 pk = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                                  pack_bf16x2(v[6], v[7]));
      *reinterpret_cast<uint4*>((unsigned short*)d.aux + ai) = pk;
      const unsigned pw[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        z[2 * q] = __uint_as_float(pw[q] << 16);
        z[2 * q + 1] = __uint_as_float(pw[q] & 0xffff0000u);
      }
    } else if (av) {
      float* o = (float*)d.aux + ai;
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = v[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        z[j] = v[j];
        if (col + j >= d.N) continue;
        if (aux_bf) {
          ((unsigned short*)d.aux)[ai + j] = f2bf(v[j]);
          z[j] = bf2f(f2bf(v[j]));
        } else {
          ((float*)d.aux)[ai + j] = v[j];
        }
      }
    }
    const uint32_t sd_ = epi_seed(d);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = epi_train_act(d, z[j]) * hv_drop_scale(sd_, idx0 + j, d.drop_p);
  } else {
    if (av && aux_bf) {
      const uint4 t = *reinterpret_cast<const uint4*>((const unsigned short*)d.aux + ai);
      const unsigned tw[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        z[2 * q] = __uint_as_float(tw[q] << 16);
        z[2 * q + 1] = __uint_as_float(tw[q] & 0xffff0000u);
      }
    } else if (av) {
      const float4 t0 = *reinterpret_cast<const float4*>((const float*)d.aux + ai);
      const float4 t1 = *reinterpret_cast<const float4*>((const float*)d.aux + ai + 4);
      z[0] = t0.x; z[1] = t0.y; z[2] = t0.z; z[3] = t0.w; z[4] = t1.x; z[5] = t1.y; z[6] = t1.z; z[7] = t1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        z[j] = col + j < d.N ? (aux_bf ? bf2f(((const unsigned short*)d.aux)[ai + j]) : ((const float*)d.aux)[ai + j])
                             : 0.f;
    }
    const uint32_t sd_ = epi_seed(d);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * hv_drop_scale(sd_, idx0 + j, d.drop_p) * epi_train_act_grad(d, z[j]);
  }
}

// Scalar write-out (C or residual not 16-B aligned / strided): element stores.
template <int BN, int NT, int SLAB, bool TRAIN>
__device__ __forceinline__ void epi_writeout_s(const hv_gemm_desc& d, int r0, int n0, unsigned char* smem) {
  const bool c_bf = d.c_dtype == HV_BF16, r_bf = d.r_dtype == HV_BF16;
  constexpr int TPR = BN / 8, RPP = NT / TPR;
#pragma unroll
  for (int p = 0; p < SLAB / RPP; ++p) {
    const int lr = p * RPP + threadIdx.x / TPR;
    const int c8 = (threadIdx.x % TPR) * 8;
    const int row = r0 + lr, col = n0 + c8;
    if (row >= d.M || col >= d.N) continue;
    const float4 lo = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4), hi = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4 + 1);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    if constexpr (TRAIN) epi_train8(d, v, row, col, false);
    const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
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

// RES: 0 no residual, 1 bf16 residual, 2 fp32 residual (vector path).  The residual rows of every
// pass are loaded BEFORE the first store: a load issued after a store is waited for with vmcnt,
// which counts in issue order, so interleaved it would also wait for every earlier store's write
// (one store round trip per pass, round-2 ISA).
template <int BN, int NT, int SLAB, bool TRAIN, int RES>
__device__ __forceinline__ void epi_writeout_v(const hv_gemm_desc& d, int r0, int n0, unsigned char* smem) {
  const bool c_bf = d.c_dtype == HV_BF16, r_bf = d.r_dtype == HV_BF16;
  constexpr int TPR = BN / 8;                 // threads per row
  constexpr int RPP = NT / TPR;               // rows per pass
  constexpr int NP = SLAB / RPP;
  const int c8 = (threadIdx.x % TPR) * 8;
  const int col = n0 + c8;
  const bool vcol = col + 8 <= d.N;           // whole 8-column vector (the vector path's condition)
  uint4 rb[RES == 1 ? NP : 1];
  float4 rf[RES == 2 ? NP : 1][2];
  if constexpr (RES != 0) {
    if (vcol) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int row = min(r0 + p * RPP + (int)threadIdx.x / TPR, d.M - 1);
        const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
        if constexpr (RES == 1) {
          rb[p] = *reinterpret_cast<const uint4*>((const unsigned short*)d.residual + rrow * d.ldr + col);
        } else {
          rf[p][0] = *reinterpret_cast<const float4*>((const float*)d.residual + rrow * d.ldr + col);
          rf[p][1] = *reinterpret_cast<const float4*>((const float*)d.residual + rrow * d.ldr + col + 4);
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int lr = p * RPP + threadIdx.x / TPR;
    const int row = r0 + lr;
    if (row >= d.M || col >= d.N) continue;
    const float4 lo = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4), hi = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4 + 1);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    // training mode 2 loads its aux row here, after the previous pass's stores: preloaded for
    // every pass like the residual (za[NP][8]) it measured 13 % slower on the 64x128 kernel
    // (scratch spills at the 3-per-CU register budget)
    if constexpr (TRAIN) epi_train8(d, v, row, col, vcol);
    if (vcol) {
      if constexpr (RES == 1) {
        const unsigned rw[4] = {rb[p].x, rb[p].y, rb[p].z, rb[p].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] += __uint_as_float(rw[q] << 16);
          v[2 * q + 1] += __uint_as_float(rw[q] & 0xffff0000u);
        }
      } else if constexpr (RES == 2) {
        v[0] += rf[p][0].x; v[1] += rf[p][0].y; v[2] += rf[p][0].z; v[3] += rf[p][0].w;
        v[4] += rf[p][1].x; v[5] += rf[p][1].y; v[6] += rf[p][1].z; v[7] += rf[p][1].w;
      }
      if (c_bf) {
        *reinterpret_cast<uint4*>((unsigned short*)d.C + (long)row * d.ldc + col) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7]));
      } else {
        float* o = (float*)d.C + (long)row * d.ldc + col;
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else {
      const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (col + j >= d.N) break;
        float x = v[j];
        if (RES != 0)
          x += r_bf ? bf2f(((const unsigned short*)d.residual)[rrow * d.ldr + col + j])
                    : ((const float*)d.residual)[rrow * d.ldr + col + j];
        const long o = (long)row * d.ldc + col + j;
        if (c_bf) ((unsigned short*)d.C)[o] = f2bf(x);
        else ((float*)d.C)[o] = x;
      }
    }
  }
}

// Mode-2 (gradient) write-out with the aux rows loaded ONE PASS AHEAD (default; HV_GV_TRAIN_NOPF
// selects the per-pass form below -- base-640 B=16 training step 146.1 / 146.7 vs 148.6 / 149.2 ms
// alternating, profiles/r04/train_pf_ab.txt):
// the aux load of pass p+1 is issued before the stores of pass p, so it is not queued behind
// them (vmcnt retires in issue order) -- one extra 8-value row in registers instead of the
// per-pass store round trip, and not the all-pass preload that spilled.  Same arithmetic and
// order as epi_train8 + epi_writeout_v: bitwise equal.
template <int BN, int NT, int SLAB, int RES>
__device__ __forceinline__ void epi_writeout_m2pf(const hv_gemm_desc& d, int r0, int n0, unsigned char* smem) {
  const bool c_bf = d.c_dtype == HV_BF16, a_bf = d.aux_dtype == HV_BF16;
  constexpr int TPR = BN / 8, RPP = NT / TPR, NP = SLAB / RPP;
  const int c8 = (threadIdx.x % TPR) * 8;
  const int col = n0 + c8;
  const bool vcol = col + 8 <= d.N;
  const bool av = vcol && (d.ld_aux & 7) == 0 && ((((uintptr_t)d.aux) & 15) == 0);
  const uint32_t sd_ = epi_seed(d);
  auto aux_row = [&](int p, float (&z)[8]) {
    const int row = min(r0 + p * RPP + (int)threadIdx.x / TPR, d.M - 1);
    const long ai = (long)row * d.ld_aux + col;
    if (av && a_bf) {
      const uint4 t = *reinterpret_cast<const uint4*>((const unsigned short*)d.aux + ai);
      const unsigned tw[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        z[2 * q] = __uint_as_float(tw[q] << 16);
        z[2 * q + 1] = __uint_as_float(tw[q] & 0xffff0000u);
      }
    } else if (av) {
      const float4 t0 = *reinterpret_cast<const float4*>((const float*)d.aux + ai);
      const float4 t1 = *reinterpret_cast<const float4*>((const float*)d.aux + ai + 4);
      z[0] = t0.x; z[1] = t0.y; z[2] = t0.z; z[3] = t0.w; z[4] = t1.x; z[5] = t1.y; z[6] = t1.z; z[7] = t1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        z[j] = col + j < d.N ? (a_bf ? bf2f(((const unsigned short*)d.aux)[ai + j]) : ((const float*)d.aux)[ai + j])
                             : 0.f;
    }
  };
  uint4 rb[RES == 1 ? NP : 1];
  float4 rf[RES == 2 ? NP : 1][2];
  if constexpr (RES != 0) {
    if (vcol) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int row = min(r0 + p * RPP + (int)threadIdx.x / TPR, d.M - 1);
        const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
        if constexpr (RES == 1) {
          rb[p] = *reinterpret_cast<const uint4*>((const unsigned short*)d.residual + rrow * d.ldr + col);
        } else {
          rf[p][0] = *reinterpret_cast<const float4*>((const float*)d.residual + rrow * d.ldr + col);
          rf[p][1] = *reinterpret_cast<const float4*>((const float*)d.residual + rrow * d.ldr + col + 4);
        }
      }
    }
  }
  // colsum_part: column sums of C as stored over this tile's rows (per-thread, then over the RPP
  // threads of a column group through LDS); the branch is uniform (a kernel argument)
  const bool want_cs = d.colsum_part != nullptr;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float za[8], zb[8];
  aux_row(0, za);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    float (&z)[8] = (p & 1) ? zb : za;
    float (&zn)[8] = (p & 1) ? za : zb;
    if (p + 1 < NP) aux_row(p + 1, zn);
    const int lr = p * RPP + threadIdx.x / TPR;
    const int row = r0 + lr;
    if (row >= d.M || col >= d.N) continue;
    const float4 lo = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4), hi = *epi_lds_chunk<BN / 4>(smem, lr, c8 / 4 + 1);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const unsigned long long idx0 = (unsigned long long)row * d.N + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * hv_drop_scale(sd_, idx0 + j, d.drop_p) * epi_train_act_grad(d, z[j]);
    if (vcol) {
      if constexpr (RES == 1) {
        const unsigned rw[4] = {rb[p].x, rb[p].y, rb[p].z, rb[p].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] += __uint_as_float(rw[q] << 16);
          v[2 * q + 1] += __uint_as_float(rw[q] & 0xffff0000u);
        }
      } else if constexpr (RES == 2) {
        v[0] += rf[p][0].x; v[1] += rf[p][0].y; v[2] += rf[p][0].z; v[3] += rf[p][0].w;
        v[4] += rf[p][1].x; v[5] += rf[p][1].y; v[6] += rf[p][1].z; v[7] += rf[p][1].w;
      }
      if (c_bf) {
        const uint4 pk = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                                    pack_bf16x2(v[6], v[7]));
        *reinterpret_cast<uint4*>((unsigned short*)d.C + (long)row * d.ldc + col) = pk;
        if (want_cs) {
          const unsigned pw[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            csum[2 * q] += __uint_as_float(pw[q] << 16);
            csum[2 * q + 1] += __uint_as_float(pw[q] & 0xffff0000u);
          }
        }
      } else {
        float* o = (float*)d.C + (long)row * d.ldc + col;
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        if (want_cs)
#pragma unroll
          for (int j = 0; j < 8; ++j) csum[j] += v[j];
      }
    } else {
      const long rrow = d.r_mod > 0 ? row % d.r_mod : row;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (col + j >= d.N) break;
        float x = v[j];
        if (RES != 0)
          x += d.r_dtype == HV_BF16 ? bf2f(((const unsigned short*)d.residual)[rrow * d.ldr + col + j])
                                    : ((const float*)d.residual)[rrow * d.ldr + col + j];
        const long o = (long)row * d.ldc + col + j;
        if (c_bf) {
          const unsigned short h = f2bf(x);
          ((unsigned short*)d.C)[o] = h;
          csum[j] += bf2f(h);
        } else {
          ((float*)d.C)[o] = x;
          csum[j] += x;
        }
      }
    }
  }
  if (want_cs) {
    // every thread's reads of the staged tile are done before its LDS is reused
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);                 // [RPP][BN]
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(threadIdx.x / TPR) * BN + c8 + j] = csum[j];
    __syncthreads();
    if ((int)threadIdx.x < BN && n0 + (int)threadIdx.x < d.N) {
      float t = 0.f;
      for (int q = 0; q < RPP; ++q) t += red[q * BN + threadIdx.x];       // fixed order
      const long b0 = r0 / 64, cidx = n0 + threadIdx.x;
      d.colsum_part[b0 * d.N + cidx] = t;
#pragma unroll
      for (int e = 1; e < SLAB / 64; ++e) d.colsum_part[(b0 + e) * d.N + cidx] = 0.f;
    }
  }
}

template <int BN, int NT, int SLAB, bool TRAIN = false>
__device__ __forceinline__ void epi_writeout(const hv_gemm_desc& d, int r0, int n0, unsigned char* smem) {
  const bool vec = (((uintptr_t)d.C) & 15) == 0 && d.ldc % 8 == 0 &&
                   (!d.residual || ((((uintptr_t)d.residual) & 15) == 0 && d.ldr % 8 == 0));
  // coalesced write-out: thread -> (row, 8 columns); the vector path needs aligned C / residual
  if constexpr (TRAIN) {
    if (vec && d.epi_mode == 2 && !(d.variant & HV_GV_TRAIN_NOPF)) {
      if (!d.residual) epi_writeout_m2pf<BN, NT, SLAB, 0>(d, r0, n0, smem);
      else if (d.r_dtype == HV_BF16) epi_writeout_m2pf<BN, NT, SLAB, 1>(d, r0, n0, smem);
      else epi_writeout_m2pf<BN, NT, SLAB, 2>(d, r0, n0, smem);
      return;
    }
  }
  if (!vec) epi_writeout_s<BN, NT, SLAB, TRAIN>(d, r0, n0, smem);
  else if (!d.residual) epi_writeout_v<BN, NT, SLAB, TRAIN, 0>(d, r0, n0, smem);
  else if (d.r_dtype == HV_BF16) epi_writeout_v<BN, NT, SLAB, TRAIN, 1>(d, r0, n0, smem);
  else epi_writeout_v<BN, NT, SLAB, TRAIN, 2>(d, r0, n0, smem);
}

template <int BM, int BN, bool LN_EPI, int WN, int RM, int RN, int NT, int SLAB, bool TRAIN = false>
__device__ __forceinline__ void gemm_epilogue_staged(const hv_gemm_desc& d, const f32x4 (&acc)[RM][RN], int m0, int n0,
                                                     unsigned char* smem) {
  static_assert(BN % 8 == 0 && SLAB % 16 == 0 && (BM == SLAB || BM == 2 * SLAB), "shape");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid / WN, wc = wid % WN;
  const int fg = lane >> 4;
  EpiCols<RN> k;
  epi_load_cols<RN, LN_EPI>(d, k, n0 + wc * (RN * 16) + fg * 4);
  const int wrow0 = wr * (RM * 16);
  if constexpr (BM == SLAB) {
    epi_stage_rows<0, LN_EPI, RM, RN, BN / 4, TRAIN>(d, acc, k, m0 + wrow0, wrow0, wc * (RN * 16), smem);
    __syncthreads();
    epi_writeout<BN, NT, SLAB, TRAIN>(d, m0, n0, smem);
  } else {
    static_assert(!TRAIN, "two-slab staging is inference-only");                                      // two slabs: the waves of rows [0, SLAB) first
    if (wrow0 < SLAB) epi_stage_rows<0, LN_EPI, RM, RN, BN / 4>(d, acc, k, m0 + wrow0, wrow0, wc * (RN * 16), smem);
    __syncthreads();
    epi_writeout<BN, NT, SLAB>(d, m0, n0, smem);
    __syncthreads();
    if (wrow0 >= SLAB)
      epi_stage_rows<0, LN_EPI, RM, RN, BN / 4>(d, acc, k, m0 + wrow0, wrow0 - SLAB, wc * (RN * 16), smem);
    __syncthreads();
    epi_writeout<BN, NT, SLAB>(d, m0 + SLAB, n0, smem);
  }
}
