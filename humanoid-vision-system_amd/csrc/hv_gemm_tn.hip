// Weight-gradient GEMM for gfx950:  C[N1, N2] (+)= sum_p A[p, n1] * B'[p, n2]
//
// The training-step contraction over tokens/pixels: dW = dY^T X for every Linear and the mHC
// coefficient matrices (manifold_layers.py:253-264 autograd), and dW = dY^T im2col(X) for every
// convolution (vision_backbone.py:42-49, feature_fusion.py:33-49, yolo_head.py:120-139 autograd).
// Both operands are stored token-major (the contraction index p is the ROW index), so the MFMA
// wants them "k-strided".  Each k-step stages a [KSTEP p-rows][tile columns] image of A and B in
// LDS with coalesced 16-byte row reads and the MFMA fragments come out of it with the CDNA4
// transposing LDS read ds_read_b64_tr_b16 (bf16) or plain scalar reads (fp32, 16x16x4 MFMA).
//
// k order inside a 32-deep bf16 step is permuted identically for both operands (lane group g
// takes p = 4g..4g+3 and 16+4g..16+4g+3): the two transposed reads of a 32-lane half then cover
// 8 consecutive image rows, conflict-free with a 32-byte row pad.
// Split-K over p: blockIdx.y owns a p range, partials go to `work` and hv_wgrad_reduce sums them
// in a fixed order (deterministic).  B may be an implicit im2col of an NHWC image.
// KM > 1 (hv_wgrad_desc.variant HV_WV_K64): each LDS stage holds KM k-steps (one barrier per
// KM x 32 rows); the MFMAs run in the same k order, and the p partition is the KM = 1 plan's, so
// the result is bitwise the KM = 1 result (a stage past a split's end multiplies zero rows).
#include "hv_common.h"

typedef short v4i16 __attribute__((ext_vector_type(4)));

namespace {

template <typename T> struct TnTr;
template <> struct TnTr<unsigned short> { static constexpr int KSTEP = 32; static constexpr int EPC = 8; };
template <> struct TnTr<float> { static constexpr int KSTEP = 16; static constexpr int EPC = 4; };

__device__ __forceinline__ v4i16 tr_read(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(const_cast<unsigned char*>(p)));
}

// BGATHER: 0 dense B, 1 conv im2col with 16-B channel chunks, 2 conv im2col scalar
template <typename T, int BM, int BN, int BGATHER, int KM = 1>
__global__ void __launch_bounds__(256) gemm_tn_kernel(const hv_wgrad_desc d, int p_chunk) {
  constexpr int KSTEP = TnTr<T>::KSTEP * KM, EPC = TnTr<T>::EPC;
  constexpr int KS1 = TnTr<T>::KSTEP;               // MFMA k-step (rows per permuted block)
  constexpr int APITCH = BM * (int)sizeof(T) + 32;
  constexpr int BPITCH = BN * (int)sizeof(T) + 32;
  constexpr int ACH = KSTEP * BM / EPC / 256;       // 16-B chunks per thread per k-step
  constexpr int BCH = KSTEP * BN / EPC / 256;
  constexpr int ACPR = BM / EPC, BCPR = BN / EPC;   // chunks per image row
  constexpr int RM = BM / 32, RN = BN / 32;
  constexpr bool IS_BF16 = sizeof(T) == 2;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small for 256 threads");

  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * KSTEP * (APITCH + BPITCH)];
  unsigned char* As = smem;
  unsigned char* Bs = smem + 2 * KSTEP * APITCH;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tilesN = (d.N2 + BN - 1) / BN;
  const int tm = blockIdx.x / tilesN, tn = blockIdx.x % tilesN;
  const int n10 = tm * BM, n20 = tn * BN;
  const long pbeg = (long)blockIdx.y * p_chunk;
  const long pend = min((long)d.P, pbeg + p_chunk);
  const int nk = (int)((pend - pbeg + KSTEP - 1) / KSTEP);

  uint4 ra[ACH], rb[BCH];

  auto load_b_chunk = [&](long p, int col) -> uint4 {
    if (p >= pend || col >= d.N2) return make_uint4(0, 0, 0, 0);
    if constexpr (BGATHER == 0) {
      return *reinterpret_cast<const uint4*>((const T*)d.B + p * d.ldb + col);
    } else {
      const int hw = d.conv_oh * d.conv_ow;
      const int img = (int)(p / hw), q = (int)(p - (long)img * hw);
      const int oh = q / d.conv_ow, ow = q - oh * d.conv_ow;
      const T* base = (const T*)d.B + (long)img * d.conv_h * d.conv_w * d.conv_c;
      if constexpr (BGATHER == 1) {
        const int tap = col / d.conv_c, ci = col - tap * d.conv_c;
        const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
        const int ih = oh * d.conv_stride - d.conv_pad + kh, iw = ow * d.conv_stride - d.conv_pad + kw;
        if ((unsigned)ih >= (unsigned)d.conv_h || (unsigned)iw >= (unsigned)d.conv_w) return make_uint4(0, 0, 0, 0);
        return *reinterpret_cast<const uint4*>(base + ((long)ih * d.conv_w + iw) * d.conv_c + ci);
      } else {
        T v[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          v[e] = T(0);
          const int cc = col + e;
          if (cc < d.N2) {
            const int tap = cc / d.conv_c, ci = cc - tap * d.conv_c;
            const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
            const int ih = oh * d.conv_stride - d.conv_pad + kh, iw = ow * d.conv_stride - d.conv_pad + kw;
            if ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
              v[e] = base[((long)ih * d.conv_w + iw) * d.conv_c + ci];
          }
        }
        return *reinterpret_cast<const uint4*>(v);
      }
    }
  };

  auto gload = [&](int kt) {
    const long p0 = pbeg + (long)kt * KSTEP;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + 256 * i;
      const int r = c / ACPR, col = n10 + (c % ACPR) * EPC;
      const long p = p0 + r;
      ra[i] = (p < pend && col < d.N1) ? *reinterpret_cast<const uint4*>((const T*)d.A + p * d.lda + col)
                                       : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + 256 * i;
      const int r = c / BCPR, col = n20 + (c % BCPR) * EPC;
      rb[i] = load_b_chunk(p0 + r, col);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<uint4*>(As + (buf * KSTEP + c / ACPR) * APITCH + (c % ACPR) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<uint4*>(Bs + (buf * KSTEP + c / BCPR) * BPITCH + (c % BCPR) * 16) = rb[i];
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pq = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int h = 0; h < KM; ++h) {
    const unsigned char* sa = As + (buf * KSTEP + h * KS1) * APITCH;
    const unsigned char* sb = Bs + (buf * KSTEP + h * KS1) * BPITCH;
    if constexpr (IS_BF16) {
      bf16x8 fa[RM], fb[RN];
#pragma unroll
      for (int a = 0; a < RM; ++a) {
        const int col = wr * (BM / 2) + a * 16 + 4 * pq;
        const v4i16 lo = tr_read(sa + (4 * g + q) * APITCH + col * 2);
        const v4i16 hi = tr_read(sa + (16 + 4 * g + q) * APITCH + col * 2);
        fa[a] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const int col = wc * (BN / 2) + b * 16 + 4 * pq;
        const v4i16 lo = tr_read(sb + (4 * g + q) * BPITCH + col * 2);
        const v4i16 hi = tr_read(sb + (16 + 4 * g + q) * BPITCH + col * 2);
        fb[b] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = 4 * s + g;
        float fa[RM], fb[RN];
#pragma unroll
        for (int a = 0; a < RM; ++a)
          fa[a] = *reinterpret_cast<const float*>(sa + row * APITCH + (wr * (BM / 2) + a * 16 + li) * 4);
#pragma unroll
        for (int b = 0; b < RN; ++b)
          fb[b] = *reinterpret_cast<const float*>(sb + row * BPITCH + (wc * (BN / 2) + b * 16 + li) * 4);
#pragma unroll
        for (int a = 0; a < RM; ++a)
#pragma unroll
          for (int b = 0; b < RN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[b], fa[a], acc[a][b], 0, 0, 0);
      }
    }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // acc[a][b] is the transposed 16x16 sub-tile: lane holds C[n1 = .. + li][n2 = .. + 4g .. 4g+3]
  const bool direct = gridDim.y == 1;
  float* out = direct ? d.C : d.work + (long)blockIdx.y * d.N1 * d.N2;
  const long ldo = direct ? d.ldc : d.N2;
  const bool add = direct && d.accumulate;
#pragma unroll
  for (int a = 0; a < RM; ++a) {
    const int n1 = n10 + wr * (BM / 2) + a * 16 + li;
    if (n1 >= d.N1) continue;
#pragma unroll
    for (int b = 0; b < RN; ++b) {
      const int n2 = n20 + wc * (BN / 2) + b * 16 + 4 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (n2 + j >= d.N2) break;
        float* o = out + (long)n1 * ldo + n2 + j;
        *o = add ? *o + acc[a][b][j] : acc[a][b][j];
      }
    }
  }
}

__global__ void k_wgrad_reduce(const float* __restrict__ work, int splits, int N1, int N2, float* C, long ldc,
                               int accumulate) {
  const long total = (long)N1 * N2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // four independent accumulators (loads in flight), fixed combination order: deterministic
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int k = 0;
    for (; k + 3 < splits; k += 4) {
      s0 += work[k * total + i];
      s1 += work[(k + 1) * total + i];
      s2 += work[(k + 2) * total + i];
      s3 += work[(k + 3) * total + i];
    }
    for (; k < splits; ++k) s0 += work[k * total + i];
    const float s = (s0 + s1) + (s2 + s3);
    const long n1 = i / N2, n2 = i - n1 * N2;
    float* o = C + n1 * ldc + n2;
    *o = accumulate ? *o + s : s;
  }
}

// Many-split form (splits > 64, small outputs over many pixels): a block owns 64 output columns
// and its 4 thread groups take the splits g, g + 4, ... with 8 loads in flight each, combined in
// a fixed order through LDS (deterministic).  The one-thread-per-output form above would wait
// splits / 4 memory latencies per thread.
__global__ void __launch_bounds__(256) k_wgrad_reduce_many(const float* __restrict__ work, int splits, int N1,
                                                           int N2, float* C, long ldc, int accumulate) {
  __shared__ float part[4][64];
  const long total = (long)N1 * N2;
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long i = blockIdx.x * 64L + c;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    int k = g;
    for (; k + 28 < splits; k += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += work[(long)(k + 4 * u) * total + i];
    }
    for (int u = 0; k < splits; k += 4, ++u) a[u] += work[(long)k * total + i];
  }
  part[g][c] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (g == 0 && i < total) {
    const float s = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
    const long n1 = i / N2, n2 = i - n1 * N2;
    float* o = C + n1 * ldc + n2;
    *o = accumulate ? *o + s : s;
  }
}

struct TnPlan {
  int bm, bn, splits, p_chunk;
};

// split cap: 256 (small outputs over many pixels -- e.g. 128 x 64 over 409,600 pixels is ONE
// tile, which at the round-4 cap of 64 ran on 64 workgroups); HV_WV_CAP64 keeps the old cap
// (a 1024-workgroup target with up to 1024 splits measured slower: 128.55 -> 132.48 ms/step,
// profiles/r05/wgrad_plan_ab.txt)
constexpr int kTnMaxSplits = 256;

TnPlan plan_tn(int P, int N1, int N2, int kstep, int max_splits = kTnMaxSplits) {
  TnPlan t;
  t.bm = N1 >= 128 ? 128 : 64;
  t.bn = N2 >= 128 ? 128 : 64;
  const long tiles = (long)hv_cdiv(N1, t.bm) * hv_cdiv(N2, t.bn);
  const long ksteps = (P + kstep - 1) / kstep;
  // aim for >= 512 workgroups: 1024 split the pixels twice as finely and doubled the fp32
  // partial traffic + reduce; base-640 B=16 training step 146.5 / 146.4 vs 150.3 / 149.5 ms
  // (profiles/r04/wgrad_split_ab.txt)
  long s = (512 + tiles - 1) / tiles;
  s = s < 1 ? 1 : s;
  const long max_s = ksteps / 4 > 0 ? ksteps / 4 : 1; // each split keeps >= 4 k-steps
  s = s > max_s ? max_s : s;
  s = s > max_splits ? max_splits : s;
  const long per = (ksteps + s - 1) / s;
  t.p_chunk = (int)(per * kstep);
  t.splits = (int)((P + t.p_chunk - 1) / t.p_chunk);
  if (t.splits < 1) t.splits = 1;
  return t;
}

template <typename T, int BM, int BN, int KM>
void launch_tn_k(const hv_wgrad_desc& d, const TnPlan& pl, hipStream_t s) {
  dim3 grid(hv_cdiv(d.N1, BM) * hv_cdiv(d.N2, BN), pl.splits);
  constexpr int EPC = TnTr<T>::EPC;
  if (d.conv_k > 0) {
    if (d.conv_c % EPC == 0) gemm_tn_kernel<T, BM, BN, 1, KM><<<grid, 256, 0, s>>>(d, pl.p_chunk);
    else gemm_tn_kernel<T, BM, BN, 2, KM><<<grid, 256, 0, s>>>(d, pl.p_chunk);
  } else {
    gemm_tn_kernel<T, BM, BN, 0, KM><<<grid, 256, 0, s>>>(d, pl.p_chunk);
  }
}

template <typename T, int BM, int BN>
int launch_tn(const hv_wgrad_desc& d, const TnPlan& pl, hipStream_t s) {
  if (sizeof(T) == 2 && (d.variant & HV_WV_K64)) launch_tn_k<T, BM, BN, 2>(d, pl, s);
  else launch_tn_k<T, BM, BN, 1>(d, pl, s);
  HV_CHECK_LAUNCH();
  if (pl.splits > 64) {
    const long total = (long)d.N1 * d.N2;
    k_wgrad_reduce_many<<<(unsigned)((total + 63) / 64), 256, 0, s>>>(d.work, pl.splits, d.N1, d.N2, d.C, d.ldc,
                                                                      d.accumulate);
    HV_CHECK_LAUNCH();
  } else if (pl.splits > 1) {
    const long total = (long)d.N1 * d.N2;
    const long nb = (total + 255) / 256;
    const unsigned blocks = (unsigned)(nb < 4096 ? nb : 4096);
    k_wgrad_reduce<<<blocks, 256, 0, s>>>(d.work, pl.splits, d.N1, d.N2, d.C, d.ldc, d.accumulate);
    HV_CHECK_LAUNCH();
  }
  return HV_OK;
}

template <typename T>
int dispatch_tn(const hv_wgrad_desc& d, const TnPlan& pl, hipStream_t s) {
  if (pl.bm == 128 && pl.bn == 128) return launch_tn<T, 128, 128>(d, pl, s);
  if (pl.bm == 128) return launch_tn<T, 128, 64>(d, pl, s);
  if (pl.bn == 128) return launch_tn<T, 64, 128>(d, pl, s);
  return launch_tn<T, 64, 64>(d, pl, s);
}

}  // namespace

extern "C" size_t hv_wgrad_work_floats(int dtype, int P, int N1, int N2) {
  const TnPlan pl = plan_tn(P, N1, N2, dtype == HV_BF16 ? 32 : 16);
  return pl.splits > 1 ? (size_t)pl.splits * N1 * N2 : 0;
}

extern "C" int hv_wgrad(const hv_wgrad_desc* dp, hv_stream_t stream) {
  if (!dp) return HV_EINVAL;
  const hv_wgrad_desc& d = *dp;
  if (d.P <= 0 || d.N1 <= 0 || d.N2 <= 0 || !d.A || !d.B || !d.C) return HV_EINVAL;
  const int epc = d.dtype == HV_BF16 ? 8 : 4;
  if (d.lda % epc || d.N1 % epc || (((uintptr_t)d.A) & 15) || (((uintptr_t)d.B) & 15)) return HV_EUNSUPPORTED;
  if (d.conv_k > 0) {
    if (d.N2 != d.conv_k * d.conv_k * d.conv_c || d.P != d.conv_n * d.conv_oh * d.conv_ow) return HV_EINVAL;
  } else if (d.ldb % epc || d.N2 % epc) {
    return HV_EUNSUPPORTED;
  }
  const TnPlan pl = plan_tn(d.P, d.N1, d.N2, d.dtype == HV_BF16 ? 32 : 16,
                            (d.variant & HV_WV_CAP64) ? 64 : kTnMaxSplits);
  if (pl.splits > 1 && !d.work) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (d.dtype == HV_BF16) return dispatch_tn<unsigned short>(d, pl, s);
  if (d.dtype == HV_F32) return dispatch_tn<float>(d, pl, s);
  return HV_EINVAL;
}
