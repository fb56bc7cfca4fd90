// MFMA GEMM for gfx950 with fused prologues (LayerNorm-on-load, implicit im2col,
// K-concatenation) and epilogues (scale, bias, activation, residual).
//
// One kernel template serves every dense contraction of the HybridVision path:
//   * convolutions (vision_backbone.py:42-49, feature_fusion.py:33-49/65, yolo_head.py:120-127/139,
//     vit_encoder_decoder.py:94-97/146-152) as implicit GEMM over NHWC activations, with the
//     eval BatchNorm folded into a per-column scale/bias and the activation in the epilogue;
//   * the mHC GEMM chain (manifold_layers.py:250-264) with the pre-LayerNorm applied while the
//     A tile is loaded and [x | h2] concatenated along K for the residual+contract product;
//   * nn.Linear layers (transformer MLP, output projection).
//
// Layout: A rows K-contiguous ([M][lda]); B is [N][ldb] (nn.Linear / reordered conv weight
// layout); C is [M][ldc].  Each k-step stages 64 bytes of every A and B row through LDS
// (rows padded to 80 B: conflict-light ds_read_b128), double-buffered with register
// prefetch.  The same 16-byte LDS fragment feeds one v_mfma_f32_16x16x32_bf16 (bf16) or
// four v_mfma_f32_16x16x4_f32 (fp32: lane group g takes k = 4g..4g+3, the k-order inside a
// 16-deep step is permuted identically for A and B, so the products are exact).
// 256 threads = 4 waves in a 2x2 grid; block -> tile mapping is XCD-aware (bijective).
#include <atomic>

#include "hv_common.h"
#include "hv_gemm_epi.h"

namespace {

constexpr int ROWB = 80;                // bytes per LDS row (64 data + 16 pad)

template <typename T> struct Tr;
template <> struct Tr<float> { static constexpr int EPC = 4; };           // elems per 16 B chunk
template <> struct Tr<unsigned short> { static constexpr int EPC = 8; };

enum { AM_DENSE = 0, AM_LN = 1, AM_CONV = 2, AM_CONV_SCALAR = 3, AM_CONVT = 4 };

__device__ __forceinline__ float ldT(const float* p, long i) { return p[i]; }
__device__ __forceinline__ float ldT(const unsigned short* p, long i) { return bf2f(p[i]); }

__device__ __forceinline__ float ld_any(const void* p, int dt, long i) {
  return dt == HV_BF16 ? bf2f(((const unsigned short*)p)[i]) : ((const float*)p)[i];
}

// pack/unpack a 16-byte chunk
template <typename T> struct Chunk;
template <> struct Chunk<float> {
  static __device__ __forceinline__ void unpack(uint4 v, float* f) {
    f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                      __float_as_uint(f[3]));
  }
};
template <> struct Chunk<unsigned short> {
  static __device__ __forceinline__ void unpack(uint4 v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// Load one 16-byte chunk [k, k+EPC) of a K-contiguous row with tail handling.
template <typename T>
__device__ __forceinline__ uint4 load_row_chunk(const T* row, int k, int K) {
  constexpr int EPC = Tr<T>::EPC;
  if (k + EPC <= K) return *reinterpret_cast<const uint4*>(row + k);
  if (k >= K) return make_uint4(0, 0, 0, 0);
  float f[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) f[e] = (k + e < K) ? ldT(row, k + e) : 0.f;
  return Chunk<T>::pack(f);
}

struct RowCtx {        // per-thread context of one A row it stages
  const void* base;    // dense: row pointer; conv: image pointer
  int valid;
  int ih0, iw0;        // conv
  float mean, rstd;    // LN prologue
};

template <typename T, int BM, int BN, int AMODE, bool TRAIN>
__global__ void __launch_bounds__(256) gemm_kernel(const hv_gemm_desc d) {
  constexpr int EPC = Tr<T>::EPC;
  constexpr int KSTEP = 4 * EPC;          // elements per 64-byte k-step
  constexpr int AR = BM / 64;             // A chunks staged per thread per k-step
  constexpr int BR = BN / 64;
  constexpr int RM = BM / 32, RN = BN / 32;
  constexpr bool IS_BF16 = sizeof(T) == 2;

  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * (BM + BN) * ROWB];
  unsigned char* As = smem;                       // [2][BM][ROWB]
  unsigned char* Bs = smem + 2 * BM * ROWB;       // [2][BN][ROWB]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  // XCD-aware bijective remap of the linear block id (blocks b and b+8 share an XCD).
  const int tilesN = (d.N + BN - 1) / BN;
  const int tilesM = (d.M + BM - 1) / BM;
  const int nwg = tilesM * tilesN;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tm = bid / tilesN, tn = bid % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread staging contexts (rows fixed across the K loop) ----
  RowCtx rc[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int c = tid + 256 * i;
    const int row = m0 + (c >> 2);
    rc[i].valid = row < d.M;
    rc[i].mean = 0.f; rc[i].rstd = 1.f;
    const int rr = rc[i].valid ? row : 0;
    if constexpr (AMODE == AM_CONV || AMODE == AM_CONV_SCALAR || AMODE == AM_CONVT) {
      const int hw = d.conv_oh * d.conv_ow;
      const int b = rr / hw, p = rr % hw;
      const int oh = p / d.conv_ow, ow = p % d.conv_ow;
      if constexpr (AMODE == AM_CONVT) {         // row = forward input pixel (ih, iw)
        rc[i].ih0 = oh + d.conv_pad;
        rc[i].iw0 = ow + d.conv_pad;
      } else {
        rc[i].ih0 = oh * d.conv_stride - d.conv_pad;
        rc[i].iw0 = ow * d.conv_stride - d.conv_pad;
      }
      rc[i].base = (const T*)d.A + (long)b * d.conv_h * d.conv_w * d.conv_c;
    } else {
      rc[i].ih0 = rc[i].iw0 = 0;
      rc[i].base = (const T*)d.A + (long)rr * d.lda;
      if constexpr (AMODE == AM_LN) {
        rc[i].mean = d.a_mean[rr];
        rc[i].rstd = d.a_rstd[rr];
      }
    }
  }
  const T* brow[BR];
  bool bvalid[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int c = tid + 256 * i;
    const int n = n0 + (c >> 2);
    bvalid[i] = n < d.N;
    brow[i] = (const T*)d.B + (long)(bvalid[i] ? n : 0) * d.ldb;
  }

  auto load_a = [&](int i, int k) -> uint4 {
    const RowCtx& r = rc[i];
    if (!r.valid) return make_uint4(0, 0, 0, 0);
    if constexpr (AMODE == AM_DENSE || AMODE == AM_LN) {
      uint4 v;
      if (d.A2 != nullptr && k >= d.k1) {
        const int row = m0 + ((tid + 256 * i) >> 2);
        v = load_row_chunk<T>((const T*)d.A2 + (long)row * d.lda2, k - d.k1, d.K - d.k1);
        return v;
      }
      v = load_row_chunk<T>((const T*)r.base, k, d.A2 ? d.k1 : d.K);
      if constexpr (AMODE == AM_LN) {
        float f[EPC];
        Chunk<T>::unpack(v, f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) f[e] = (k + e < d.K) ? (f[e] - r.mean) * r.rstd : 0.f;
        v = Chunk<T>::pack(f);
      }
      return v;
    } else if constexpr (AMODE == AM_CONV) {
      // whole chunk inside one filter tap because conv_c % EPC == 0
      if (k >= d.K) return make_uint4(0, 0, 0, 0);
      const int tap = k / d.conv_c, ci = k - tap * d.conv_c;
      const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
      const int ih = r.ih0 + kh, iw = r.iw0 + kw;
      if ((unsigned)ih >= (unsigned)d.conv_h || (unsigned)iw >= (unsigned)d.conv_w)
        return make_uint4(0, 0, 0, 0);
      return *reinterpret_cast<const uint4*>((const T*)r.base +
                                            ((long)ih * d.conv_w + iw) * d.conv_c + ci);
    } else if constexpr (AMODE == AM_CONVT) {
      // transposed conv (dgrad): tap (kh, kw) of input pixel reads output pixel (th/s, tw/s)
      if (k >= d.K) return make_uint4(0, 0, 0, 0);
      const int tap = k / d.conv_c, ci = k - tap * d.conv_c;
      const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
      const int th = r.ih0 - kh, tw = r.iw0 - kw;
      if (th < 0 || tw < 0 || th % d.conv_stride || tw % d.conv_stride) return make_uint4(0, 0, 0, 0);
      const int oh = th / d.conv_stride, ow = tw / d.conv_stride;
      if (oh >= d.conv_h || ow >= d.conv_w) return make_uint4(0, 0, 0, 0);
      return *reinterpret_cast<const uint4*>((const T*)r.base + ((long)oh * d.conv_w + ow) * d.conv_c + ci);
    } else {
      float f[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        const int kk = k + e;
        float v = 0.f;
        if (kk < d.K) {
          const int tap = kk / d.conv_c, ci = kk - tap * d.conv_c;
          const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
          const int ih = r.ih0 + kh, iw = r.iw0 + kw;
          if ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
            v = ldT((const T*)r.base, ((long)ih * d.conv_w + iw) * d.conv_c + ci);
        }
        f[e] = v;
      }
      return Chunk<T>::pack(f);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[AR], rb[BR];
  const int nk = (d.K + KSTEP - 1) / KSTEP;

  auto gload = [&](int kt) {
    const int kbase = kt * KSTEP;
#pragma unroll
    for (int i = 0; i < AR; ++i) ra[i] = load_a(i, kbase + ((tid + 256 * i) & 3) * EPC);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int k = kbase + ((tid + 256 * i) & 3) * EPC;
      rb[i] = bvalid[i] ? load_row_chunk<T>(brow[i], k, d.K) : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<uint4*>(As + (buf * BM + (c >> 2)) * ROWB + (c & 3) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<uint4*>(Bs + (buf * BN + (c >> 2)) * ROWB + (c & 3) * 16) = rb[i];
    }
  };

  gload(0);
  sstore(0);
  __syncthreads();

  const int frow = lane & 15, fchunk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    uint4 fa[RM], fb[RN];
#pragma unroll
    for (int a = 0; a < RM; ++a)
      fa[a] = *reinterpret_cast<const uint4*>(
          As + (buf * BM + wr * (BM / 2) + a * 16 + frow) * ROWB + fchunk * 16);
#pragma unroll
    for (int b = 0; b < RN; ++b)
      fb[b] = *reinterpret_cast<const uint4*>(
          Bs + (buf * BN + wc * (BN / 2) + b * 16 + frow) * ROWB + fchunk * 16);
    if constexpr (IS_BF16) {
#pragma unroll
      for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fb[b]), __builtin_bit_cast(bf16x8, fa[a]), acc[a][b], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int a = 0; a < RM; ++a) {
          const uint32_t av = s == 0 ? fa[a].x : s == 1 ? fa[a].y : s == 2 ? fa[a].z : fa[a].w;
#pragma unroll
          for (int b = 0; b < RN; ++b) {
            const uint32_t bv = s == 0 ? fb[b].x : s == 1 ? fb[b].y : s == 2 ? fb[b].z : fb[b].w;
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(bv), __uint_as_float(av),
                                                             acc[a][b], 0, 0, 0);
          }
        }
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue (hv_gemm_epi.h: sub-tiles accumulated transposed; LN prologue already applied)
  gemm_epilogue<BM, BN, false, TRAIN>(d, acc, m0, n0);
}

template <typename T, int BM, int BN, bool TRAIN>
int launch_mode_t(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, BM) * hv_cdiv(d.N, BN);
  constexpr int EPC = Tr<T>::EPC;
  hv_diag_count(HV_KF_GEMM_REGSTAGE);
  if (d.conv_k > 0 && d.conv_transposed) {
    gemm_kernel<T, BM, BN, AM_CONVT, TRAIN><<<grid, 256, 0, s>>>(d);
  } else if (d.conv_k > 0) {
    if (d.conv_c % EPC == 0)
      gemm_kernel<T, BM, BN, AM_CONV, TRAIN><<<grid, 256, 0, s>>>(d);
    else
      gemm_kernel<T, BM, BN, AM_CONV_SCALAR, TRAIN><<<grid, 256, 0, s>>>(d);
  } else if (d.a_mean) {
    gemm_kernel<T, BM, BN, AM_LN, TRAIN><<<grid, 256, 0, s>>>(d);
  } else {
    gemm_kernel<T, BM, BN, AM_DENSE, TRAIN><<<grid, 256, 0, s>>>(d);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

template <typename T, int BM, int BN>
int launch_mode(const hv_gemm_desc& d, hipStream_t s) {
  // training epilogues are separate instantiations: the inference kernels keep their registers
  if constexpr (BM * BN > 128 * 64) {
    if (d.epi_mode) return HV_EUNSUPPORTED;     // never selected (launch_typed picks 64x128)
    return launch_mode_t<T, BM, BN, false>(d, s);
  } else {
    return d.epi_mode ? launch_mode_t<T, BM, BN, true>(d, s) : launch_mode_t<T, BM, BN, false>(d, s);
  }
}

template <typename T>
int launch_typed(const hv_gemm_desc& d, hipStream_t s) {
  // tile choice: 128x128 when both sides are large, thinner tiles for narrow N or few rows
  const long tiles128 = (long)hv_cdiv(d.M, 128) * hv_cdiv(d.N, 128);
  if (d.N <= 64) return launch_mode<T, 128, 64>(d, s);
  if (tiles128 < 512 && d.M > 64) return launch_mode<T, 64, 128>(d, s);
  if (d.M <= 64 || d.epi_mode) return launch_mode<T, 64, 128>(d, s);
  return launch_mode<T, 128, 128>(d, s);
}

}  // namespace

int hv_gemm_glds(const hv_gemm_desc& d, hipStream_t s);   // hv_gemm_glds.hip

int hv_conv3x3_c32(const hv_gemm_desc& d, hipStream_t s);   // hv_stem.hip

extern "C" int hv_gemm(const hv_gemm_desc* dp, hv_stream_t stream) {
  if (!dp) return HV_EINVAL;
  const hv_gemm_desc& d = *dp;
  if (d.M <= 0 || d.N <= 0 || d.K <= 0 || !d.A || !d.B || !d.C) return HV_EINVAL;
  const int epc = d.dtype == HV_BF16 ? 8 : 4;
  if (d.conv_k > 0) {
    if (d.K != d.conv_k * d.conv_k * d.conv_c || d.M != d.conv_n * d.conv_oh * d.conv_ow)
      return HV_EINVAL;
    if (d.a_mean || d.A2) return HV_EUNSUPPORTED;
    if (d.conv_transposed && (d.conv_c % epc || d.conv_stride < 1)) return HV_EUNSUPPORTED;
  } else {
    if (d.lda % epc) return HV_EUNSUPPORTED;
    if (d.A2 && (d.k1 % (4 * epc) || d.lda2 % epc)) return HV_EUNSUPPORTED;
  }
  if (d.ldb % epc) return HV_EUNSUPPORTED;
  if (((uintptr_t)d.A | (uintptr_t)d.B) & 15) return HV_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (d.colsum_part) {
    // only the LDS-DMA kernel's staged gradient epilogue (epi_writeout_m2pf) sums the columns:
    // every other path refuses the call instead of silently leaving the partials unwritten
    const bool ok = d.epi_mode == 2 && d.dtype == HV_BF16 && !d.conv_transposed && d.splitk <= 1 &&
                    !(d.variant & (HV_GV_REGSTAGE | HV_GV_FLAT_TRAIN | HV_GV_TRAIN_NOPF | HV_GV_TRAIN_BIG)) &&
                    (d.variant & HV_GV_TILE_MASK) <= 4 && !(d.conv_k == 3 && d.conv_c == 32) &&
                    (((uintptr_t)d.C) & 15) == 0 && d.ldc % 8 == 0 &&
                    (!d.residual || ((((uintptr_t)d.residual) & 15) == 0 && d.ldr % 8 == 0));
    return ok ? hv_gemm_glds(d, s) : HV_EUNSUPPORTED;
  }
  if (!(d.variant & HV_GV_REGSTAGE)) {
    if (d.conv_k == 3 && d.conv_c == 32) {               // halo-tiled 3x3 conv, Cin = 32 (hv_stem.hip)
      const int rc = hv_conv3x3_c32(d, s);
      if (rc != HV_EUNSUPPORTED) return rc;
    }
    const int rc = hv_gemm_glds(d, s);
    if (rc != HV_EUNSUPPORTED) return rc;
  }
  if (d.dtype == HV_BF16) return launch_typed<unsigned short>(d, s);
  if (d.dtype == HV_F32) return launch_typed<float>(d, s);
  return HV_EINVAL;
}
