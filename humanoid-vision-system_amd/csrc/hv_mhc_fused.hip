// Fused mHC token chain (gfx950, bf16 MFMA), replacing the six launches of the unfused path
// (row stats, 3 GEMMs, LayerNorm) for the mHC sites with D <= 128:
//
//   z   = (x - mean) * rstd                    (LN_pre core; gamma/beta folded into A1/c1)
//   h1  = GELU(z A1 + c1)          [T x 2HD]   produced KC = 32 columns at a time
//   h2  = GELU(h1 W2^T + b2)       [T x HD]    accumulated in registers over the 2HD chunks
//   y   = [x | h2] Wc              [T x D]     Wc = centred [H_res ; H_post]
//   out = LN_post(y) * g2 + b2' (+ residual)   computed from the GEMM3 accumulators
//
// Reference: ManifoldHyperConnection.forward (manifold_layers.py:223-280); the algebra
// (fold + centring) is in hv_amd/manifold.py and DESIGN.md.  Only x is read and out written:
// the [T, 2HD] and [T, HD] intermediates never leave the registers.
//
// Layout of the work: every wave owns TPW = 16*TB tokens end to end.  All three products are
// computed TRANSPOSED (weights as the MFMA A operand, activations as B), so a lane always
// holds 4 consecutive hidden units of ONE token; two such 16-wide tiles are exactly the B
// fragment of the next product when its 32-deep contraction runs in the permuted order
// {4g..4g+3, 16+4g..16+4g+3} (lane group g) -- which the weight (A) fragment then also uses.
// So h1 -> GEMM2 and h2 -> GEMM3 go register to register, no LDS, no cross-wave exchange.
// The weights are the only shared data: per 32-wide chunk of 2HD, the A1^T rows and the W2
// columns of that chunk are DMA'd (global_load_lds, 16 B/lane, XOR-swizzled rows) into a
// double-buffered LDS stage shared by the 8 waves -- one barrier per chunk -- and Wc^T is
// streamed the same way for GEMM3.  GELU is hv_gelu_fast (|err| <= 2.6e-5, below bf16).
#include <atomic>

#include "hv_common.h"

namespace {

__device__ __forceinline__ f32x4 mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                 c, 0, 0, 0);
}

__device__ __forceinline__ void dma16(const void* src, unsigned char* lds_wave_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
#else
  (void)src; (void)lds_wave_base;
#endif
}

template <int D, int HD, int TB_, int NW_ = 8>
struct Cfg {
  static constexpr int NW = NW_, NT = 64 * NW_;
  static constexpr int TB = TB_;                   // 16-token blocks per wave (acc2: HT*TB tiles)
  static constexpr int TPW = 16 * TB, BM = NW * TPW;
  static constexpr int KC = 32, NCH = 2 * HD / KC;
  static constexpr int HT = HD / 16, DT = D / 16, KS1 = D / 32;
  static constexpr int CPA = D / 8;                // 16-B chunks per A1^T row (2D bytes)
  static constexpr int A1B = KC * D * 2;           // bytes of one A1^T chunk  [KC rows x D]
  static constexpr int W2B = HD * 64;              // bytes of one W2 chunk    [HD rows x 32 k]
  static constexpr int STAGE = A1B + W2B;
  static constexpr int WCB = D * 64;               // bytes of one Wc^T k-chunk [D rows x 32 k]
  static constexpr int KS3 = (D + HD) / 32;
  static constexpr int LDS = 2 * (STAGE > WCB ? STAGE : WCB);
  static_assert(HD % 32 == 0 && D % 32 == 0 && TB >= 1, "shape");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// 64-byte rows (W2 / Wc^T chunks): 16-B chunk c of row r lives at c ^ ((r >> 2) & 3), which
// makes the permuted 8-byte fragment reads (ds_read_b64, 32-lane groups) conflict-free.
__device__ __forceinline__ int swz64(int r, int c) { return c ^ ((r >> 2) & 3); }

// An 8-byte fragment read kept a ds_read_b64.  Left to itself the compiler pairs the reads of
// rows r and r + 16 (1 KiB apart) into ds_read2st64_b64, whose bank map is (a/4) mod 32 in
// 16-lane groups: there this pattern is 2-way conflicted (rocprofv3 SQ_LDS_BANK_CONFLICT: 45% of
// the LDS cycles of the D = 32 / 64 kernels).  A volatile access is never merged.
template <bool NOMERGE>
__device__ __forceinline__ uint2 lds_b64(const unsigned char* p) {
  if constexpr (NOMERGE) {
    typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
    const unsigned long long v = *(lds_u64*)(p);
    return make_uint2((unsigned)v, (unsigned)(v >> 32));
  } else {
    return *reinterpret_cast<const uint2*>(p);
  }
}
// A1^T rows (2D bytes, CPA chunks): chunk c of row r at c ^ (r & (CPA - 1)).
template <int CPA>
__device__ __forceinline__ int swzA(int r, int c) { return c ^ (r & (CPA - 1)); }

template <int D, int HD, int TB_, int MINB, int NW_ = 8, bool NOMERGE = false>
__global__ void __launch_bounds__(64 * NW_, MINB) mhc_fused_kernel(
    const unsigned short* __restrict__ x, int T,
    const unsigned short* __restrict__ a1t,   // [2HD, D]
    const float* __restrict__ c1,             // [2HD]
    const unsigned short* __restrict__ w2,    // [HD, 2HD]
    const float* __restrict__ b2,             // [HD]
    const unsigned short* __restrict__ wct,   // [D, D+HD]
    const float* __restrict__ g_post, const float* __restrict__ b_post,
    const unsigned short* __restrict__ res,   // optional [T, D], added after LN_post
    unsigned short* __restrict__ out) {
  using C = Cfg<D, HD, TB_, NW_>;
  constexpr int TB = C::TB, KC = C::KC;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long tw = (long)blockIdx.x * C::BM + w * C::TPW;     // first token of this wave

  // ---- weight chunk DMA: A1^T rows [ch*KC, +KC) and W2 columns [ch*KC, +KC) -> stage st
  auto issue_chunk = [&](int ch, int st) {
    unsigned char* sa = smem + st * C::STAGE;
    unsigned char* sw = sa + C::A1B;
#pragma unroll
    for (int p0 = 0; p0 < KC * C::CPA; p0 += C::NT) {
      const int p = p0 + tid;
      if (p0 + (tid & ~63) < KC * C::CPA) {                   // wave-uniform
        const int r = p / C::CPA, pc = p % C::CPA;
        dma16(a1t + (long)(ch * KC + r) * D + swzA<C::CPA>(r, pc) * 8, sa + (p - lane) * 16);
      }
    }
#pragma unroll
    for (int p0 = 0; p0 < HD * 4; p0 += C::NT) {
      const int p = p0 + tid;
      if (p0 + (tid & ~63) < HD * 4) {
        const int r = p >> 2, pc = p & 3;
        dma16(w2 + (long)r * (2 * HD) + ch * KC + swz64(r, pc) * 8, sw + (p - lane) * 16);
      }
    }
  };
  auto issue_wc = [&](int ks, int st) {
    unsigned char* sb = smem + st * C::WCB;
#pragma unroll
    for (int p0 = 0; p0 < D * 4; p0 += C::NT) {
      const int p = p0 + tid;
      if (p0 + (tid & ~63) < D * 4) {
        const int r = p >> 2, pc = p & 3;
        dma16(wct + (long)r * (D + HD) + ks * 32 + swz64(r, pc) * 8, sb + (p - lane) * 16);
      }
    }
  };

  issue_chunk(0, 0);

  // ---- x fragments (B operand, standard k order) and LN_pre -> z fragments
  // (x is re-read from L2 for GEMM3 rather than held across the chunk loop)
  uint4 zf[TB][C::KS1];
#pragma unroll
  for (int tb = 0; tb < TB; ++tb) {
    const long tok = min(tw + tb * 16 + fr, (long)T - 1);
    uint4 xf[C::KS1];
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      xf[ks] = *reinterpret_cast<const uint4*>(x + tok * D + ks * 32 + fg * 8);
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) s += __uint_as_float(wv[e] << 16) + __uint_as_float(wv[e] & 0xffff0000u);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(wv[e] << 16) - mu, b = __uint_as_float(wv[e] & 0xffff0000u) - mu;
        q += a * a + b * b;
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
      uint32_t zv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        zv[e] = pack_bf16x2((__uint_as_float(wv[e] << 16) - mu) * rs, (__uint_as_float(wv[e] & 0xffff0000u) - mu) * rs);
      zf[tb][ks] = make_uint4(zv[0], zv[1], zv[2], zv[3]);
    }
  }

  // ---- GEMM1 + GEMM2 over the 2HD chunks
  f32x4 acc2[C::HT][TB];
#pragma unroll
  for (int h = 0; h < C::HT; ++h)
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) acc2[h][tb] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < C::NCH; ++ch) {
    const int st = ch & 1;
    const float4 cb0 = *reinterpret_cast<const float4*>(c1 + ch * KC + fg * 4);
    const float4 cb1 = *reinterpret_cast<const float4*>(c1 + ch * KC + 16 + fg * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                   // chunk ch landed; stage st^1 is free
    if (ch + 1 < C::NCH) issue_chunk(ch + 1, st ^ 1);
    const unsigned char* sa = smem + st * C::STAGE;
    const unsigned char* sw = sa + C::A1B;

    // GEMM1 (transposed): h1^T[hidden ct*16 + 4g + j][token] ; A = A1^T rows from LDS
    uint4 hb[TB];
    {
      f32x4 g1[2][TB];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int r = ct * 16 + fr;
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) g1[ct][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < C::KS1; ++ks) {
          const uint4 af = *reinterpret_cast<const uint4*>(sa + r * (2 * D) + swzA<C::CPA>(r, ks * 4 + fg) * 16);
#pragma unroll
          for (int tb = 0; tb < TB; ++tb) g1[ct][tb] = mfma(af, zf[tb][ks], g1[ct][tb]);
        }
      }
#pragma unroll
      for (int tb = 0; tb < TB; ++tb)
        hb[tb] = make_uint4(pack_bf16x2(hv_gelu_fast(g1[0][tb][0] + cb0.x), hv_gelu_fast(g1[0][tb][1] + cb0.y)),
                            pack_bf16x2(hv_gelu_fast(g1[0][tb][2] + cb0.z), hv_gelu_fast(g1[0][tb][3] + cb0.w)),
                            pack_bf16x2(hv_gelu_fast(g1[1][tb][0] + cb1.x), hv_gelu_fast(g1[1][tb][1] + cb1.y)),
                            pack_bf16x2(hv_gelu_fast(g1[1][tb][2] + cb1.z), hv_gelu_fast(g1[1][tb][3] + cb1.w)));
    }
    // GEMM2 (transposed): acc2[ht] += W2[ht*16 + fr][perm k] . h1^T ; permuted k order
#pragma unroll
    for (int h = 0; h < C::HT; ++h) {
      const int r = h * 16 + fr;
      const uint2 lo = lds_b64<NOMERGE>(sw + r * 64 + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
      const uint2 hi = lds_b64<NOMERGE>(sw + r * 64 + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
      const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) acc2[h][tb] = mfma(af, hb[tb], acc2[h][tb]);
      if ((h & 7) == 7) __builtin_amdgcn_sched_barrier(0);   // bound the fragments in flight
    }
  }

  // ---- GEMM3 (transposed): y^T[d][token] = Wc^T[d][k] . [x | h2]^T, Wc^T streamed via LDS
  f32x4 acc3[C::DT][TB];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();                                     // every wave is done with the chunk stages
  issue_wc(0, 0);
#pragma unroll
  for (int ks = 0; ks < C::KS3; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ks + 1 < C::KS3) issue_wc(ks + 1, (ks + 1) & 1);
    const unsigned char* sb = smem + (ks & 1) * C::WCB;
    uint4 xg[TB], h2f[TB];
    if (ks < C::KS1) {
#pragma unroll
      for (int tb = 0; tb < TB; ++tb)
        xg[tb] = *reinterpret_cast<const uint4*>(x + min(tw + tb * 16 + fr, (long)T - 1) * D + ks * 32 + fg * 8);
    } else {
      // h2 = GELU(acc2 + b2) for hidden [32s, 32s+32): two transposed tiles -> one B fragment
      // in the permuted k order, built just before use (acc2 tiles die here)
      const int s2 = ks - C::KS1;
      const float4 ba = *reinterpret_cast<const float4*>(b2 + s2 * 32 + fg * 4);
      const float4 bb = *reinterpret_cast<const float4*>(b2 + s2 * 32 + 16 + fg * 4);
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) {
        const f32x4 p = acc2[ks >= C::KS1 ? 2 * s2 : 0][tb], q = acc2[ks >= C::KS1 ? 2 * s2 + 1 : 0][tb];
        h2f[tb] = make_uint4(pack_bf16x2(hv_gelu_fast(p[0] + ba.x), hv_gelu_fast(p[1] + ba.y)),
                             pack_bf16x2(hv_gelu_fast(p[2] + ba.z), hv_gelu_fast(p[3] + ba.w)),
                             pack_bf16x2(hv_gelu_fast(q[0] + bb.x), hv_gelu_fast(q[1] + bb.y)),
                             pack_bf16x2(hv_gelu_fast(q[2] + bb.z), hv_gelu_fast(q[3] + bb.w)));
      }
    }
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int r = dt * 16 + fr;
      if (ks < C::KS1) {                               // x part: standard k order
        const uint4 af = *reinterpret_cast<const uint4*>(sb + r * 64 + swz64(r, fg) * 16);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = mfma(af, xg[tb], acc3[dt][tb]);
      } else {                                         // h2 part: permuted k order
        const uint2 lo = lds_b64<NOMERGE>(sb + r * 64 + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
        const uint2 hi = lds_b64<NOMERGE>(sb + r * 64 + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
        const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = mfma(af, h2f[tb], acc3[dt][tb]);
      }
    }
  }

  // ---- LN_post per token (lane: token tb*16 + fr, columns dt*16 + 4g + j) + residual
#pragma unroll
  for (int tb = 0; tb < TB; ++tb) {
    float s = 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) s += (acc3[dt][tb][0] + acc3[dt][tb][1]) + (acc3[dt][tb][2] + acc3[dt][tb][3]);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float dd = acc3[dt][tb][j] - mu; q += dd * dd; }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float inv = rsqrtf(q * (1.0f / D) + 1e-5f);
    const long tok = tw + tb * 16 + fr;
    if (tok >= T) continue;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int col = dt * 16 + fg * 4;
      const float4 gp = *reinterpret_cast<const float4*>(g_post + col);
      const float4 bp = *reinterpret_cast<const float4*>(b_post + col);
      float v0 = (acc3[dt][tb][0] - mu) * inv * gp.x + bp.x;
      float v1 = (acc3[dt][tb][1] - mu) * inv * gp.y + bp.y;
      float v2 = (acc3[dt][tb][2] - mu) * inv * gp.z + bp.z;
      float v3 = (acc3[dt][tb][3] - mu) * inv * gp.w + bp.w;
      if (res) {
        const uint2 r2 = *reinterpret_cast<const uint2*>(res + tok * D + col);
        v0 += __uint_as_float(r2.x << 16);
        v1 += __uint_as_float(r2.x & 0xffff0000u);
        v2 += __uint_as_float(r2.y << 16);
        v3 += __uint_as_float(r2.y & 0xffff0000u);
      }
      *reinterpret_cast<uint2*>(out + tok * D + col) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

template <int D, int HD, int TB, int MINB, int NW = 8, bool NOMERGE = false>
int launch(const hv_mhc_fused_args* a, hipStream_t s) {
  using C = Cfg<D, HD, TB, NW>;
  auto k = mhc_fused_kernel<D, HD, TB, MINB, NW, NOMERGE>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  hv_diag_count(HV_KF_MHC_FUSED);
  k<<<hv_cdiv(a->T, C::BM), C::NT, C::LDS, s>>>(
      (const unsigned short*)a->x, a->T, (const unsigned short*)a->a1t, a->c1, (const unsigned short*)a->w2,
      a->b2, (const unsigned short*)a->wct, a->g_post, a->b_post, (const unsigned short*)a->residual,
      (unsigned short*)a->out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// ---------------------------------------------------------------------------------------------
// Software-pipelined per-wave kernel (D = 32, 64).  Same work split and arithmetic as
// mhc_fused_kernel (bitwise-equal outputs), restructured around what the ISA of that kernel showed:
//  * its chunk loop waited vmcnt(0) right after issuing the next chunk's DMA (the c1 global loads
//    in the loop make hipcc drain the whole counter before their first use), so every chunk's
//    weight DMA was fully exposed;
//  * GEMM1 -> GELU -> GEMM2 of one chunk is a dependency chain: the ~170 GELU VALU of a chunk
//    had no MFMAs of the same wave beside them.
// Here c1 lives in LDS, the DMAs are inline asm (untracked by the compiler, waited with an
// explicit vmcnt one chunk later), the weight chunks stream through a 3-stage ring, and
// iteration ch computes GEMM1 + GELU of chunk ch+1 beside GEMM2 of chunk ch (independent
// instruction streams the scheduler interleaves: matrix pipe || VALU).  Wc^T goes to LDS whole
// in the last two iterations (the two stages no chunk needs any more), so GEMM3 runs barrier-free.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void mhc_glds16(const void* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}
#pragma clang diagnostic pop

template <int D, int HD, int TB_, int MINB, int NW_, bool NOMERGE>
__global__ void __launch_bounds__(64 * NW_, MINB) mhc_fused_pipe_kernel(
    const unsigned short* __restrict__ x, int T, const unsigned short* __restrict__ a1t, const float* __restrict__ c1,
    const unsigned short* __restrict__ w2, const float* __restrict__ b2, const unsigned short* __restrict__ wct,
    const float* __restrict__ g_post, const float* __restrict__ b_post, const unsigned short* __restrict__ res,
    unsigned short* __restrict__ out) {
  using C = Cfg<D, HD, TB_, NW_>;
  constexpr int TB = C::TB, KC = C::KC, NCH = C::NCH;
  constexpr int WPS = C::STAGE / C::WCB;                 // Wc^T k-chunks per stage
  static_assert(NCH >= 3 && C::KS3 <= 2 * WPS, "Wc^T fits the two stages freed by the last chunks");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* const c1s = reinterpret_cast<float*>(smem + 3 * C::STAGE);   // 2HD (+KC pad) floats
  // b2 [HD], g_post [D], b_post [D] in LDS too: read from global inside the GEMM3 / LN_post
  // loops, each load was waited for on its own (and, once stores had been issued, behind them)
  float* const b2s = c1s + 2 * HD + KC;
  float* const gps = b2s + HD;
  float* const bps = gps + D;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int fr = lane & 15, fg = lane >> 4;
  const long tw = (long)blockIdx.x * C::BM + w * C::TPW;

  auto issue_chunk = [&](int ch, int st) {
    const unsigned sa = lds0 + st * C::STAGE, sw = sa + C::A1B;
#pragma unroll
    for (int p0 = 0; p0 < KC * C::CPA; p0 += C::NT) {
      if (p0 + wu * 64 < KC * C::CPA) {
        const int p = p0 + tid, r = p / C::CPA, pc = p % C::CPA;
        mhc_glds16(a1t + (long)(ch * KC + r) * D + swzA<C::CPA>(r, pc) * 8, sa + (p0 + wu * 64) * 16);
      }
    }
#pragma unroll
    for (int p0 = 0; p0 < HD * 4; p0 += C::NT) {
      if (p0 + wu * 64 < HD * 4) {
        const int p = p0 + tid, r = p >> 2, pc = p & 3;
        mhc_glds16(w2 + (long)r * (2 * HD) + ch * KC + swz64(r, pc) * 8, sw + (p0 + wu * 64) * 16);
      }
    }
  };
  constexpr int WST_A = NCH % 3, WST_B = (NCH + 1) % 3;  // stages chunks NCH, NCH+1 would use
  auto wc_chunk = [&](int ks) -> int { return (ks < WPS ? WST_A : WST_B) * C::STAGE + (ks % WPS) * C::WCB; };
  auto issue_wc = [&](int k0, int k1) {                  // Wc^T k-chunks [k0, k1)
#pragma unroll
    for (int ks = k0; ks < k1; ++ks) {
#pragma unroll
      for (int p0 = 0; p0 < D * 4; p0 += C::NT) {
        if (p0 + wu * 64 < D * 4) {
          const int p = p0 + tid, r = p >> 2, pc = p & 3;
          mhc_glds16(wct + (long)r * (D + HD) + ks * 32 + swz64(r, pc) * 8, lds0 + wc_chunk(ks) + (p0 + wu * 64) * 16);
        }
      }
    }
  };

  // ---- prologue: x and c1 loaded (c1 -> LDS) before the first DMA, so the compiler's waits for
  // them never cover a DMA; chunks 0 and 1 in flight under LN_pre -> z fragments
  uint4 xin[TB][C::KS1];
#pragma unroll
  for (int tb = 0; tb < TB; ++tb)
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks)
      xin[tb][ks] = *reinterpret_cast<const uint4*>(x + min(tw + tb * 16 + fr, (long)T - 1) * D + ks * 32 + fg * 8);
  for (int i = tid; i < 2 * HD; i += C::NT) c1s[i] = c1[i];
  for (int i = tid; i < HD; i += C::NT) b2s[i] = b2[i];
  for (int i = tid; i < D; i += C::NT) {
    gps[i] = g_post[i];
    bps[i] = b_post[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  issue_chunk(0, 0);
  issue_chunk(1, 1);
  uint4 zf[TB][C::KS1];
#pragma unroll
  for (int tb = 0; tb < TB; ++tb) {
    uint4 xf[C::KS1];
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      xf[ks] = xin[tb][ks];
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) s += __uint_as_float(wv[e] << 16) + __uint_as_float(wv[e] & 0xffff0000u);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(wv[e] << 16) - mu, b = __uint_as_float(wv[e] & 0xffff0000u) - mu;
        q += a * a + b * b;
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
      uint32_t zv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        zv[e] = pack_bf16x2((__uint_as_float(wv[e] << 16) - mu) * rs, (__uint_as_float(wv[e] & 0xffff0000u) - mu) * rs);
      zf[tb][ks] = make_uint4(zv[0], zv[1], zv[2], zv[3]);
    }
  }

  // GEMM1 (transposed) + GELU of chunk ch from stage ch % 3 -> B fragments of GEMM2 (permuted k)
  auto gemm1 = [&](int ch, uint4 (&hb)[TB]) {
    const unsigned char* sa = smem + (ch % 3) * C::STAGE;
    const float4 cb0 = *reinterpret_cast<const float4*>(c1s + ch * KC + fg * 4);
    const float4 cb1 = *reinterpret_cast<const float4*>(c1s + ch * KC + 16 + fg * 4);
    f32x4 g1[2][TB];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int r = ct * 16 + fr;
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) g1[ct][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < C::KS1; ++ks) {
        const uint4 af = *reinterpret_cast<const uint4*>(sa + r * (2 * D) + swzA<C::CPA>(r, ks * 4 + fg) * 16);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) g1[ct][tb] = mfma(af, zf[tb][ks], g1[ct][tb]);
      }
    }
#pragma unroll
    for (int tb = 0; tb < TB; ++tb)
      hb[tb] = make_uint4(pack_bf16x2(hv_gelu_fast(g1[0][tb][0] + cb0.x), hv_gelu_fast(g1[0][tb][1] + cb0.y)),
                          pack_bf16x2(hv_gelu_fast(g1[0][tb][2] + cb0.z), hv_gelu_fast(g1[0][tb][3] + cb0.w)),
                          pack_bf16x2(hv_gelu_fast(g1[1][tb][0] + cb1.x), hv_gelu_fast(g1[1][tb][1] + cb1.y)),
                          pack_bf16x2(hv_gelu_fast(g1[1][tb][2] + cb1.z), hv_gelu_fast(g1[1][tb][3] + cb1.w)));
  };

  f32x4 acc2[C::HT][TB];
#pragma unroll
  for (int h = 0; h < C::HT; ++h)
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) acc2[h][tb] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                       // chunks 0, 1 and c1 in LDS
  uint4 hb[TB];
  gemm1(0, hb);

  for (int ch = 0; ch < NCH; ++ch) {
    if (ch > 0) {
      // this wave's DMAs of chunk ch+1 landed; every wave's reads of iteration ch-1 retired
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    if (ch + 2 < NCH) issue_chunk(ch + 2, (ch + 2) % 3);
    else if (ch + 2 == NCH) issue_wc(0, WPS < C::KS3 ? WPS : C::KS3);   // stage NCH % 3
    else if (WPS < C::KS3) issue_wc(WPS, C::KS3);                     // stage (NCH + 1) % 3
    // GEMM1 + GELU of chunk ch+1 (the last iteration computes an unused chunk from the Wc stage:
    // straight-line code, no branch between the two instruction streams)
    uint4 hn[TB];
    gemm1(ch + 1 < NCH ? ch + 1 : NCH, hn);
    // GEMM2 (transposed) of chunk ch: acc2[h] += W2[h*16 + fr][perm k] . h1^T
    const unsigned char* sw = smem + (ch % 3) * C::STAGE + C::A1B;
#pragma unroll
    for (int h = 0; h < C::HT; ++h) {
      const int r = h * 16 + fr;
      const uint2 lo = lds_b64<NOMERGE>(sw + r * 64 + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
      const uint2 hi = lds_b64<NOMERGE>(sw + r * 64 + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
      const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) acc2[h][tb] = mfma(af, hb[tb], acc2[h][tb]);
    }
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) hb[tb] = hn[tb];
  }

  // ---- GEMM3 (transposed): y^T = Wc^T . [x | h2]^T, every Wc^T k-chunk resident
  uint4 xg[TB][C::KS1];
#pragma unroll
  for (int tb = 0; tb < TB; ++tb)
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks)
      xg[tb][ks] = *reinterpret_cast<const uint4*>(x + min(tw + tb * 16 + fr, (long)T - 1) * D + ks * 32 + fg * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  f32x4 acc3[C::DT][TB];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < C::KS3; ++ks) {
    const unsigned char* sb = smem + wc_chunk(ks);
    if (ks < C::KS1) {
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        const int r = dt * 16 + fr;
        const uint4 af = *reinterpret_cast<const uint4*>(sb + r * 64 + swz64(r, fg) * 16);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = mfma(af, xg[tb][ks], acc3[dt][tb]);
      }
    } else {
      const int s2 = ks - C::KS1;
      const float4 ba = *reinterpret_cast<const float4*>(b2s + s2 * 32 + fg * 4);
      const float4 bb = *reinterpret_cast<const float4*>(b2s + s2 * 32 + 16 + fg * 4);
      uint4 h2f[TB];
#pragma unroll
      for (int tb = 0; tb < TB; ++tb) {
        const f32x4 p = acc2[2 * s2][tb], q = acc2[2 * s2 + 1][tb];
        h2f[tb] = make_uint4(pack_bf16x2(hv_gelu_fast(p[0] + ba.x), hv_gelu_fast(p[1] + ba.y)),
                             pack_bf16x2(hv_gelu_fast(p[2] + ba.z), hv_gelu_fast(p[3] + ba.w)),
                             pack_bf16x2(hv_gelu_fast(q[0] + bb.x), hv_gelu_fast(q[1] + bb.y)),
                             pack_bf16x2(hv_gelu_fast(q[2] + bb.z), hv_gelu_fast(q[3] + bb.w)));
      }
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        const int r = dt * 16 + fr;
        const uint2 lo = lds_b64<NOMERGE>(sb + r * 64 + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
        const uint2 hi = lds_b64<NOMERGE>(sb + r * 64 + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
        const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) acc3[dt][tb] = mfma(af, h2f[tb], acc3[dt][tb]);
      }
    }
  }

  // ---- LN_post per token (lane: token tb*16 + fr, columns dt*16 + 4g + j) + residual; the
  // residual of every (tb, dt) is loaded before the first store (a load behind a store waits for it)
  constexpr bool PRE = D >= 64;     // D = 32 (TB = 4): the preloaded residual would spill
  uint2 rres[TB][C::DT];
  if (PRE && res) {
#pragma unroll
    for (int tb = 0; tb < TB; ++tb)
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
        rres[tb][dt] = *reinterpret_cast<const uint2*>(res + min(tw + tb * 16 + fr, (long)T - 1) * D + dt * 16 + fg * 4);
  }
#pragma unroll
  for (int tb = 0; tb < TB; ++tb) {
    float s = 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) s += (acc3[dt][tb][0] + acc3[dt][tb][1]) + (acc3[dt][tb][2] + acc3[dt][tb][3]);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float dd = acc3[dt][tb][j] - mu; q += dd * dd; }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float inv = rsqrtf(q * (1.0f / D) + 1e-5f);
    const long tok = tw + tb * 16 + fr;
    if (tok >= T) continue;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int col = dt * 16 + fg * 4;
      const float4 gp = *reinterpret_cast<const float4*>(gps + col);
      const float4 bp = *reinterpret_cast<const float4*>(bps + col);
      float v0 = (acc3[dt][tb][0] - mu) * inv * gp.x + bp.x;
      float v1 = (acc3[dt][tb][1] - mu) * inv * gp.y + bp.y;
      float v2 = (acc3[dt][tb][2] - mu) * inv * gp.z + bp.z;
      float v3 = (acc3[dt][tb][3] - mu) * inv * gp.w + bp.w;
      if (res) {
        const uint2 r2 = PRE ? rres[tb][dt] : *reinterpret_cast<const uint2*>(res + tok * D + col);
        v0 += __uint_as_float(r2.x << 16);
        v1 += __uint_as_float(r2.x & 0xffff0000u);
        v2 += __uint_as_float(r2.y << 16);
        v3 += __uint_as_float(r2.y & 0xffff0000u);
      }
      *reinterpret_cast<uint2*>(out + tok * D + col) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

template <int D, int HD, int TB, int MINB, int NW, bool NOMERGE>
int launch_pipe(const hv_mhc_fused_args* a, hipStream_t s) {
  using C = Cfg<D, HD, TB, NW>;
  constexpr int LDS = 3 * C::STAGE + (2 * HD + C::KC + HD + 2 * D) * 4;
  static_assert(LDS <= 80 * 1024, "two workgroups per CU");
  auto k = mhc_fused_pipe_kernel<D, HD, TB, MINB, NW, NOMERGE>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hv_diag_count(HV_KF_MHC_FUSED);
  k<<<hv_cdiv(a->T, C::BM), C::NT, LDS, s>>>(
      (const unsigned short*)a->x, a->T, (const unsigned short*)a->a1t, a->c1, (const unsigned short*)a->w2,
      a->b2, (const unsigned short*)a->wct, a->g_post, a->b_post, (const unsigned short*)a->residual,
      (unsigned short*)a->out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// ---------------------------------------------------------------------------------------------
// Split-hidden variant (D = 128, HD = 512).  The kernel above gives every wave 16 tokens end to
// end, so each W2 fragment read from LDS (1 KB) feeds ONE MFMA: at D = 128 the loop is LDS- and
// latency-bound (~400 TF/s).  Here a 4-wave workgroup owns TOK = 64 tokens and splits the HIDDEN
// dimension: wave w accumulates h2 for hidden units [w*HD/4, (w+1)*HD/4) of all 64 tokens, so
// every W2 fragment feeds TT = 4 MFMAs and every h1 fragment HQT = 8 (register blocking 8 x 4).
//   GEMM1  wave w computes the h1 chunk (32 hidden, GELU) for ITS 16 tokens and writes it, already
//          in the GEMM2 B-fragment layout, to an LDS slot (double-buffered by chunk parity)
//   GEMM2  wave w: acc2[8 hidden tiles][4 token tiles] += W2 chunk rows (its quarter) . h1 chunk
//   GEMM3  split-K over the waves: wave w contracts its h2 quarter (+ one 32-wide x chunk) into a
//          partial y for all 64 tokens; the 4 partials meet in LDS (fixed order -> deterministic)
//          in two column halves; LN_post + residual per token from registers.
// Weight chunks (A1^T rows + W2 columns) stream through a 3-stage DMA ring, one barrier per chunk:
// chunk c+2 is DMA'd while GEMM1(c+1) and GEMM2(c) run.
template <int D, int HD, int NG>
struct Cfg2 {
  static constexpr int NW = 4 * NG, NT = 64 * NW;
  static constexpr int TOKG = 32768 / HD, TOK = NG * TOKG, TT = TOKG / 16;   // tokens per group / WG
  static constexpr int TW1 = TOK / NW, TBW = TW1 / 16;                         // GEMM1 tokens per wave
  static constexpr int HQ = HD / 4, HQT = HQ / 16, KC = 32, NCH = 2 * HD / KC, KS1 = D / 32, CPA = D / 8;
  static constexpr int XPW = KS1 / 4;                                 // 32-wide x chunks per quarter wave
  static constexpr int A1B = KC * D * 2, W2B = HD * 64, STAGE = A1B + W2B, H1B = (TOK / 16) * 1024;
  static constexpr int MAIN = 3 * STAGE + 2 * H1B + 2 * HD * 4;       // + c1 (fp32) kept in LDS
  static constexpr int A1P = KC * CPA / NT, W2P = HD * 4 / NT;        // chunk DMA pieces per thread
  // GEMM3 column parts of 32 output columns: one part's Wc^T slice (all D + HD k) fits a stage
  static constexpr int NP = D / 32, DP = D / NP, DT3 = DP / 16, KT3 = (D + HD) / 32;
  static constexpr int WCP = KT3 * DP * 64, PROW = DP + 4, PARTG = 4 * TOKG * PROW * 4;   // per group
  static constexpr int RTW = TOKG / 4, LPT = 64 / RTW, CPL = DP / LPT;            // reduce: tokens / lanes
  static constexpr int WPT = KT3 * DP * 4 / NT;                                   // Wc DMA pieces / thread
  // GEMM3 phase: Wc parts ping-pong in the stages of chunks NCH, NCH+1 (mod 3); group 0's partials
  // in the third stage, group 1's from 3*STAGE on (over the h1 slots and c1)
  static constexpr int LDS3 = 3 * STAGE + (NG > 1 ? PARTG : 0);
  static constexpr int LDS = MAIN > LDS3 ? MAIN : LDS3;
  static_assert(TBW >= 1 && HQT % 2 == 0 && KS1 % 4 == 0 && KS1 <= 8 && DT3 >= 1 && CPL % 4 == 0, "shape");
  static_assert(KC * CPA % NT == 0 && HD * 4 % NT == 0, "uniform chunk DMA per thread");
  static_assert(WCP <= STAGE && PARTG <= STAGE && NG <= 2 && KT3 * DP * 4 % NT == 0, "GEMM3 layout");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// SPLITW: the end-of-iteration wait leaves the W2 half of chunk ch+2 in flight (it is first read
// one iteration later than the A1^T half), so the larger W2 DMA gets two iterations of cover
template <int D, int HD, int NG, bool SPLITW = false>
__global__ void __launch_bounds__(256 * NG, 1) mhc_fused2_kernel(
    const unsigned short* __restrict__ x, int T, const unsigned short* __restrict__ a1t,
    const float* __restrict__ c1, const unsigned short* __restrict__ w2, const float* __restrict__ b2,
    const unsigned short* __restrict__ wct, const float* __restrict__ g_post, const float* __restrict__ b_post,
    const unsigned short* __restrict__ res, unsigned short* __restrict__ out) {
  using C = Cfg2<D, HD, NG>;
  constexpr int KC = C::KC, TT = C::TT, TBW = C::TBW, HQT = C::HQT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* const h1s = smem + 3 * C::STAGE;
  float* const c1s = reinterpret_cast<float*>(h1s + 2 * C::H1B);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int gq = w >> 2, qq = w & 3;                   // token group, hidden quarter of this wave
  const int fr = lane & 15, fg = lane >> 4;
  const long t0 = (long)blockIdx.x * C::TOK;
  const long tg0 = t0 + gq * C::TOKG;                  // first token of this wave's group
  const long tw = t0 + w * C::TW1;                     // first GEMM1 token of this wave

  // weight DMAs as inline asm (mhc_glds16): hipcc does not track them, so it no longer waits
  // vmcnt(0) before every fragment read of the other stages (it cannot tell them apart from the
  // stage being filled); every wait below is explicit
  auto issue_chunk = [&](int ch, int st) {
    const unsigned sa = lds0 + st * C::STAGE, sw = sa + C::A1B;
#pragma unroll
    for (int p0 = 0; p0 < KC * C::CPA; p0 += C::NT) {
      if (p0 + wu * 64 < KC * C::CPA) {
        const int p = p0 + tid, r = p / C::CPA, pc = p % C::CPA;
        mhc_glds16(a1t + (long)(ch * KC + r) * D + swzA<C::CPA>(r, pc) * 8, sa + (p0 + wu * 64) * 16);
      }
    }
#pragma unroll
    for (int p0 = 0; p0 < HD * 4; p0 += C::NT) {
      if (p0 + wu * 64 < HD * 4) {
        const int p = p0 + tid, r = p >> 2, pc = p & 3;
        mhc_glds16(w2 + (long)r * (2 * HD) + ch * KC + swz64(r, pc) * 8, sw + (p0 + wu * 64) * 16);
      }
    }
  };
  // c1 goes to LDS once: a global load inside the chunk loop would be younger than the chunk
  // DMA just issued, and vmcnt retires in order -- GEMM1 would wait for the whole DMA each chunk
  for (int i = tid; i < 2 * HD; i += C::NT) c1s[i] = c1[i];
  auto issue_wc = [&](int dp) {                        // Wc^T rows [dp*DP, +DP), all k -> stage (NCH+dp&1)%3
    const unsigned dst = lds0 + ((C::NCH + (dp & 1)) % 3) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::WPT; ++i) {
      const int p = i * C::NT + tid;
      const int kc = p / (C::DP * 4), r = (p >> 2) % C::DP, pc = p & 3;
      mhc_glds16(wct + (long)(dp * C::DP + r) * (D + HD) + kc * 32 + swz64(r, pc) * 8, dst + (i * C::NT + wu * 64) * 16);
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // c1 loads retired before the first DMA
  issue_chunk(0, 0);
  issue_chunk(1, 1);

  // ---- LN_pre of this wave's GEMM1 tokens -> z fragments (B operand of GEMM1, standard k order)
  uint4 zf[TBW][C::KS1];
#pragma unroll
  for (int tb = 0; tb < TBW; ++tb) {
    const long tok = min(tw + tb * 16 + fr, (long)T - 1);
    uint4 xf[C::KS1];
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      xf[ks] = *reinterpret_cast<const uint4*>(x + tok * D + ks * 32 + fg * 8);
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) s += __uint_as_float(wv[e] << 16) + __uint_as_float(wv[e] & 0xffff0000u);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(wv[e] << 16) - mu, b = __uint_as_float(wv[e] & 0xffff0000u) - mu;
        q += a * a + b * b;
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int ks = 0; ks < C::KS1; ++ks) {
      const uint32_t wv[4] = {xf[ks].x, xf[ks].y, xf[ks].z, xf[ks].w};
      uint32_t zv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        zv[e] = pack_bf16x2((__uint_as_float(wv[e] << 16) - mu) * rs, (__uint_as_float(wv[e] & 0xffff0000u) - mu) * rs);
      zf[tb][ks] = make_uint4(zv[0], zv[1], zv[2], zv[3]);
    }
  }

  // GEMM1 of chunk ch for this wave's tokens -> h1 slot `par`, in the GEMM2 B-fragment layout
  auto gemm1 = [&](int ch, int par) {
    const unsigned char* sa = smem + (ch % 3) * C::STAGE;
    const float4 cb0 = *reinterpret_cast<const float4*>(c1s + ch * KC + fg * 4);
    const float4 cb1 = *reinterpret_cast<const float4*>(c1s + ch * KC + 16 + fg * 4);
    unsigned char* slot = h1s + par * C::H1B;
#pragma unroll
    for (int tb = 0; tb < TBW; ++tb) {
      f32x4 g0 = f32x4{0.f, 0.f, 0.f, 0.f}, g1v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < C::KS1; ++ks) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(sa + fr * (2 * D) + swzA<C::CPA>(fr, ks * 4 + fg) * 16);
        const uint4 a1 = *reinterpret_cast<const uint4*>(sa + (16 + fr) * (2 * D) +
                                                         swzA<C::CPA>(16 + fr, ks * 4 + fg) * 16);
        g0 = mfma(a0, zf[tb][ks], g0);
        g1v = mfma(a1, zf[tb][ks], g1v);
      }
      const uint4 hb = make_uint4(pack_bf16x2(hv_gelu_fast(g0[0] + cb0.x), hv_gelu_fast(g0[1] + cb0.y)),
                                  pack_bf16x2(hv_gelu_fast(g0[2] + cb0.z), hv_gelu_fast(g0[3] + cb0.w)),
                                  pack_bf16x2(hv_gelu_fast(g1v[0] + cb1.x), hv_gelu_fast(g1v[1] + cb1.y)),
                                  pack_bf16x2(hv_gelu_fast(g1v[2] + cb1.z), hv_gelu_fast(g1v[3] + cb1.w)));
      *reinterpret_cast<uint4*>(slot + ((w * TBW + tb) * 64 + lane) * 16) = hb;
    }
  };

  f32x4 acc2[HQT][TT];
#pragma unroll
  for (int h = 0; h < HQT; ++h)
#pragma unroll
    for (int t = 0; t < TT; ++t) acc2[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                     // chunks 0, 1 landed
  gemm1(0, 0);
  __syncthreads();                                     // h1(0) visible

  for (int ch = 0; ch < C::NCH; ++ch) {
    if (ch + 2 < C::NCH) issue_chunk(ch + 2, (ch + 2) % 3);
    else issue_wc(ch + 2 - C::NCH);                    // GEMM3's first two Wc parts ride the tail
    const unsigned char* sw = smem + (ch % 3) * C::STAGE + C::A1B;
    const unsigned char* slot = h1s + (ch & 1) * C::H1B + gq * TT * 1024;
    uint4 bf[TT];                                      // h1 chunk fragments of the group's tokens
#pragma unroll
    for (int t = 0; t < TT; ++t) bf[t] = *reinterpret_cast<const uint4*>(slot + (t * 64 + lane) * 16);
#pragma unroll
    for (int hl = 0; hl < HQT; ++hl) {
      const int r = (qq * HQT + hl) * 16 + fr;
      const uint2 lo = lds_b64<true>(sw + r * 64 + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
      const uint2 hi = lds_b64<true>(sw + r * 64 + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
      const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
      for (int t = 0; t < TT; ++t) acc2[hl][t] = mfma(af, bf[t], acc2[hl][t]);
    }
    // GEMM1 of chunk ch+1 AFTER GEMM2 in program order: its h1 ds_write ends the iteration, so
    // nothing keeps the scheduler from moving its fragment reads, MFMAs and GELU VALU up between
    // GEMM2's MFMAs (in the other order GEMM2's reads could not pass the write).  The last
    // iteration recomputes chunk NCH-1 into the idle h1 slot: straight-line code, no branch.
    gemm1(ch + 1 < C::NCH ? ch + 1 : C::NCH - 1, (ch + 1) & 1);
    // this wave's DMAs of chunk ch+2 (or the Wc part) landed; every wave's reads of this
    // iteration retired and its h1(ch+1) writes visible.  SPLITW: only the A1^T half of chunk
    // ch+2 (read by GEMM1 next iteration) and everything older -- W2(ch+1) included -- landed;
    // in the Wc tail only the part before the newest
    if constexpr (SPLITW) {
      if (ch + 2 < C::NCH) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::W2P) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::WPT) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // ---- h2 = GELU(acc2 + b2) as GEMM3 B fragments (pairs of hidden tiles, permuted k order)
  uint4 h2f[HQT / 2][TT];
#pragma unroll
  for (int j = 0; j < HQT / 2; ++j) {
    const int hb0 = (qq * HQT + 2 * j) * 16;
    const float4 ba = *reinterpret_cast<const float4*>(b2 + hb0 + fg * 4);
    const float4 bb = *reinterpret_cast<const float4*>(b2 + hb0 + 16 + fg * 4);
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      const f32x4 p = acc2[2 * j][t], q = acc2[2 * j + 1][t];
      h2f[j][t] = make_uint4(pack_bf16x2(hv_gelu_fast(p[0] + ba.x), hv_gelu_fast(p[1] + ba.y)),
                             pack_bf16x2(hv_gelu_fast(p[2] + ba.z), hv_gelu_fast(p[3] + ba.w)),
                             pack_bf16x2(hv_gelu_fast(q[0] + bb.x), hv_gelu_fast(q[1] + bb.y)),
                             pack_bf16x2(hv_gelu_fast(q[2] + bb.z), hv_gelu_fast(q[3] + bb.w)));
    }
  }
  // x chunks qq, qq + 4, ... (32 input columns each) on quarter qq
  uint4 xg[C::XPW][TT];
#pragma unroll
  for (int xc = 0; xc < C::XPW; ++xc)
#pragma unroll
    for (int t = 0; t < TT; ++t)
      xg[xc][t] = *reinterpret_cast<const uint4*>(x + min(tg0 + t * 16 + fr, (long)T - 1) * D + (qq + 4 * xc) * 32 +
                                                  fg * 8);

  // ---- GEMM3 (split-K over the 4 quarter waves of a group) + cross-wave reduce, NP column parts;
  // part dp+2's Wc DMA overlaps the reduce of part dp and the MFMAs of part dp+1
  float* const part = reinterpret_cast<float*>(gq == 0 ? smem + ((C::NCH + 2) % 3) * C::STAGE
                                                       : smem + 3 * C::STAGE);
  const int ltok = lane % C::RTW;                      // reduce / LN mapping: token, CPL columns
  const int cb = (lane / C::RTW) * C::CPL;
  float y[C::NP][C::CPL];
#pragma unroll
  for (int dp = 0; dp < C::NP; ++dp) {
    if (dp + 1 < C::NP) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::WPT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                      // Wc part dp visible; part dp-1 reduced
    const unsigned char* wcp = smem + ((C::NCH + (dp & 1)) % 3) * C::STAGE;
    f32x4 acc3[C::DT3][TT];
#pragma unroll
    for (int dt = 0; dt < C::DT3; ++dt)
#pragma unroll
      for (int t = 0; t < TT; ++t) acc3[dt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < HQT / 2; ++j) {
      const int kc = (D + qq * C::HQ) / 32 + j;
#pragma unroll
      for (int dt = 0; dt < C::DT3; ++dt) {
        const int r = dt * 16 + fr;
        const unsigned char* row = wcp + (kc * C::DP + r) * 64;
        const uint2 lo = lds_b64<true>(row + swz64(r, fg >> 1) * 16 + (fg & 1) * 8);
        const uint2 hi = lds_b64<true>(row + swz64(r, 2 + (fg >> 1)) * 16 + (fg & 1) * 8);
        const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int t = 0; t < TT; ++t) acc3[dt][t] = mfma(af, h2f[j][t], acc3[dt][t]);
      }
    }
#pragma unroll
    for (int xc = 0; xc < C::XPW; ++xc) {
#pragma unroll
      for (int dt = 0; dt < C::DT3; ++dt) {
        const int r = dt * 16 + fr;
        const uint4 af = *reinterpret_cast<const uint4*>(wcp + ((qq + 4 * xc) * C::DP + r) * 64 + swz64(r, fg) * 16);
#pragma unroll
        for (int t = 0; t < TT; ++t) acc3[dt][t] = mfma(af, xg[xc][t], acc3[dt][t]);
      }
    }
    // partial y^T tiles -> part[quarter][token][col]  (lane: token t*16 + fr, cols dt*16 + 4fg ..)
    float* pw = part + (long)qq * C::TOKG * C::PROW;
#pragma unroll
    for (int dt = 0; dt < C::DT3; ++dt)
#pragma unroll
      for (int t = 0; t < TT; ++t)
        *reinterpret_cast<f32x4*>(pw + (t * 16 + fr) * C::PROW + dt * 16 + fg * 4) = acc3[dt][t];
    __syncthreads();                                   // partials written; Wc part dp no longer read
    if (dp + 2 < C::NP) issue_wc(dp + 2);
    const float* pg = part + (qq * C::RTW + ltok) * C::PROW + cb;
#pragma unroll
    for (int c = 0; c < C::CPL; c += 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(pg + c);
#pragma unroll
      for (int s2 = 1; s2 < 4; ++s2) v += *reinterpret_cast<const f32x4*>(pg + s2 * C::TOKG * C::PROW + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[dp][c + j] = v[j];
    }
  }

  // ---- LN_post (+ residual) per token: lanes ltok, ltok + RTW, ... share a token
  float s = 0.f;
#pragma unroll
  for (int dp = 0; dp < C::NP; ++dp)
#pragma unroll
    for (int c = 0; c < C::CPL; ++c) s += y[dp][c];
#pragma unroll
  for (int o = C::RTW; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mu = s * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int dp = 0; dp < C::NP; ++dp)
#pragma unroll
    for (int c = 0; c < C::CPL; ++c) { const float d0 = y[dp][c] - mu; q += d0 * d0; }
#pragma unroll
  for (int o = C::RTW; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
  const float inv = rsqrtf(q * (1.0f / D) + 1e-5f);
  const long tok = tg0 + qq * C::RTW + ltok;
  if (tok < T) {
    // every load (LN_post affine, residual) issued before the first store: a load behind a
    // store is waited for together with it (vmcnt retires in order)
    float4 gpa[C::NP][C::CPL / 4], bpa[C::NP][C::CPL / 4];
    uint4 rr4[C::NP][C::CPL / 8];
#pragma unroll
    for (int dp = 0; dp < C::NP; ++dp)
#pragma unroll
      for (int c = 0; c < C::CPL; c += 4) {
        gpa[dp][c / 4] = *reinterpret_cast<const float4*>(g_post + dp * C::DP + cb + c);
        bpa[dp][c / 4] = *reinterpret_cast<const float4*>(b_post + dp * C::DP + cb + c);
      }
    if (res) {
#pragma unroll
      for (int dp = 0; dp < C::NP; ++dp)
#pragma unroll
        for (int c = 0; c < C::CPL; c += 8)
          rr4[dp][c / 8] = *reinterpret_cast<const uint4*>(res + tok * D + dp * C::DP + cb + c);
    }
#pragma unroll
    for (int dp = 0; dp < C::NP; ++dp) {
      const int col0 = dp * C::DP + cb;
#pragma unroll
      for (int c = 0; c < C::CPL; c += 8) {
        const int col = col0 + c;
        const float4 ga = gpa[dp][c / 4], gb = gpa[dp][c / 4 + 1];
        const float4 ba = bpa[dp][c / 4], bb = bpa[dp][c / 4 + 1];
        const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
        const float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (y[dp][c + e] - mu) * inv * gg[e] + bv[e];
        if (res) {
          const uint4 r4 = rr4[dp][c / 8];
          const uint32_t rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += __uint_as_float(rr[e] << 16);
            v[2 * e + 1] += __uint_as_float(rr[e] & 0xffff0000u);
          }
        }
        *reinterpret_cast<uint4*>(out + tok * D + col) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      }
    }
  }
}

template <int D, int HD, int NG, bool SPLITW = false>
int launch2(const hv_mhc_fused_args* a, hipStream_t s) {
  using C = Cfg2<D, HD, NG>;
  auto k = mhc_fused2_kernel<D, HD, NG, SPLITW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  hv_diag_count(HV_KF_MHC_FUSED);
  k<<<hv_cdiv(a->T, C::TOK), C::NT, C::LDS, s>>>(
      (const unsigned short*)a->x, a->T, (const unsigned short*)a->a1t, a->c1, (const unsigned short*)a->w2,
      a->b2, (const unsigned short*)a->wct, a->g_post, a->b_post, (const unsigned short*)a->residual,
      (unsigned short*)a->out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

}  // namespace

extern "C" int hv_mhc_tok_supported(int D, int Hd);
int hv_mhc_tok_launch(const hv_mhc_fused_args* a, int n, hipStream_t s);

extern "C" int hv_mhc_fused_supported(int D, int Hd, int dtype, int variant) {
  if (dtype != HV_BF16) return 0;
  if (variant & HV_MV_TOK)
    return (variant & (HV_MV_TOKSPLIT2 | HV_MV_TOKSPLIT4)) ? (D == 256 && (Hd == 512 || Hd == 1024))
                                                           : hv_mhc_tok_supported(D, Hd);
  return (D == 32 && Hd == 128) || (D == 64 && Hd == 256) || (D == 128 && Hd == 512) ||
         (D == 256 && Hd == 512 && (variant & (HV_MV_WIDE | HV_MV_SPLIT256)));
}

static int mhc_args_ok(const hv_mhc_fused_args* a) {
  if (!a || a->T <= 0 || !a->x || !a->a1t || !a->c1 || !a->w2 || !a->b2 || !a->wct || !a->g_post || !a->b_post ||
      !a->out)
    return HV_EINVAL;
  if (!hv_mhc_fused_supported(a->D, a->Hd, a->dtype, a->variant)) return HV_EUNSUPPORTED;
  const uintptr_t al = (uintptr_t)a->x | (uintptr_t)a->a1t | (uintptr_t)a->w2 | (uintptr_t)a->wct |
                       (uintptr_t)a->out | (uintptr_t)a->c1 | (uintptr_t)a->b2 | (uintptr_t)a->g_post |
                       (uintptr_t)a->b_post | (uintptr_t)a->residual;
  if (al & 15) return HV_EUNSUPPORTED;
  return HV_OK;
}

extern "C" int hv_mhc_fused_group(const hv_mhc_fused_args* a, int n, hv_stream_t stream) {
  if (!a || n < 1 || n > 3) return HV_EINVAL;
  for (int i = 0; i < n; ++i) {
    const int e = mhc_args_ok(a + i);
    if (e != HV_OK) return e;
    if (a[i].D != a[0].D || a[i].Hd != a[0].Hd || a[i].T != a[0].T || a[i].dtype != a[0].dtype ||
        a[i].variant != a[0].variant)
      return HV_EINVAL;
  }
  if (!(a[0].variant & HV_MV_TOK)) return HV_EUNSUPPORTED;
  return hv_mhc_tok_launch(a, n, (hipStream_t)stream);
}

extern "C" int hv_mhc_fused(const hv_mhc_fused_args* a, hv_stream_t stream) {
  const int e = mhc_args_ok(a);
  if (e != HV_OK) return e;
  const int shape = a->variant & HV_MV_SHAPE_MASK;
  hipStream_t s = (hipStream_t)stream;
  if (a->variant & HV_MV_TOK) return hv_mhc_tok_launch(a, 1, s);
  // default for D = 32 / 64: the software-pipelined per-wave kernel with unmerged fragment reads
  // (tools/mhc_ab.py, gpurun_out r3 mhcpipe3: D=64 T=1.6M 0.849 vs 0.979 ms, T=409,600 0.220 vs
  // 0.265; D=32 T=1.6M 0.321 vs 0.346; in-model graph 19.94 vs 20.26 ms/step, bitwise equal).
  // measured (tools/mhc_variants.py): more tokens per wave wins while acc2 fits in registers;
  // (tools/mhc_ab.py) 4-wave workgroups, two per CU, beat one 8-wave workgroup by 16-20% at
  // every D (the two groups' chunk barriers no longer coincide, so one group's MFMAs cover the
  // other's DMA wait + barrier).  Variant 2 = the 8-wave groups; variant 1 = three 4-wave
  // groups per CU (register cap 170): 2x slower.  Also measured slower: 1.5x tokens per wave
  // (TB 6 / 3, 35-60%) and 2-wave groups (4x) -- all register spills.
  if (a->D == 32) {
    if (shape == 8) return launch_pipe<32, 128, 4, 2, 4, false>(a, s);
    if (shape == 9) return launch_pipe<32, 128, 4, 2, 4, true>(a, s);
    if (shape == 7) return launch<32, 128, 4, 2, 4, true>(a, s);
    if (shape == 10) return launch<32, 128, 4, 2, 4>(a, s);
    if (shape == 1) return launch<32, 128, 4, 3, 4>(a, s);
    if (shape == 2) return launch<32, 128, 4, 1>(a, s);
    return launch_pipe<32, 128, 4, 2, 4, true>(a, s);
  }
  if (a->D == 64) {
    if (shape == 8) return launch_pipe<64, 256, 2, 2, 4, false>(a, s);
    if (shape == 9) return launch_pipe<64, 256, 2, 2, 4, true>(a, s);
    if (shape == 7) return launch<64, 256, 2, 2, 4, true>(a, s);
    if (shape == 10) return launch<64, 256, 2, 2, 4>(a, s);
    if (shape == 1) return launch<64, 256, 2, 3, 4>(a, s);
    if (shape == 2) return launch<64, 256, 2, 1>(a, s);
    return launch_pipe<64, 256, 2, 2, 4, true>(a, s);
  }
  if (a->D == 128) {
    // default: the split-hidden kernel (hidden dimension across 4 waves, 2 token groups per
    // workgroup) -- tools/mhc_ab.py: 0.306 vs 0.329 ms at T = 102400, 0.073 vs 0.088 at 25600;
    // variant 5 = the per-wave 4-wave kernel, 2 = per-wave 8-wave
    if (shape == 2) return launch<128, 512, 1, 1>(a, s);
    if (shape == 5) return launch<128, 512, 1, 2, 4>(a, s);
    if (shape == 12) return launch2<128, 512, 2, true>(a, s);
    return launch2<128, 512, 2>(a, s);
  }
  // D = 256 (ViT / FPN / head sites, Hd = 512): the split-hidden kernel, one 4-wave group of 64
  // tokens per workgroup (three 48 KiB weight stages fill the LDS)
  if (a->variant & HV_MV_SPLIT256) {
    if (shape == 12) return launch2<256, 512, 1, true>(a, s);
    return launch2<256, 512, 1>(a, s);
  }
  // D=256 (ViT, off by default): at T=6416 / 25600 the unfused chain wins (65 / 150 us vs
  // 94 / 139 us fused, tools/mhc_ab.py); 8-wave groups here, variant 1 = 4-wave
  if (shape == 1) return launch<256, 512, 1, 1, 4>(a, s);
  return launch<256, 512, 1, 1>(a, s);
}
