// Token-tile fused mHC chain (gfx950, bf16 MFMA) for sites whose token count is too small for
// the chunk-streaming kernels of hv_mhc_fused.hip to fill the chip: the ViT's 37 (D=256, Hd=512)
// sites at 6,416 tokens (B=16) / 401 (B=1), and the D=128 / D=256 backbone sites at B=1.
//
//   z   = (x - mean) * rstd                    (LN_pre core; gamma/beta folded into A1/c1)
//   h1  = GELU(z A1 + c1)          [TW x 2HD]
//   h2  = GELU(h1 W2^T + b2)       [TW x HD]
//   y   = [x | h2] Wc              [TW x D]    Wc = centred [H_res ; H_post]
//   out = LN_post(y) * g + b (+ residual)
//
// Reference: ManifoldHyperConnection.forward (manifold_layers.py:223-280); the fold / centring
// algebra is in hv_amd/manifold.py and DESIGN.md §2.
//
// Work split.  A 512-thread workgroup owns TW = 16 or 32 tokens and runs the whole chain for
// them; the 8 waves split the OUTPUT units of every product (GEMM1: 2HD/8 hidden units per wave,
// GEMM2: HD/8, GEMM3: D/8), so no wave ever shares a weight with another and the weights need no
// LDS at all: every weight fragment is loaded by its one consumer straight from L2 into the
// MFMA A registers (32 contiguous bytes per lane = two 32-deep k-steps; four lanes read one
// 128-B line), through a register ring PF k-pairs deep that runs ACROSS the phase boundaries
// (the next product's first fragments are in flight during this product's epilogue and barrier).
// Activations travel between the waves through LDS as MFMA B-fragment images (1 KiB per 16-token
// tile and 32-deep k-step, lane l at byte 16 l: conflict-free ds_read_b128 / ds_write_b128).
//
// Products are computed transposed (weights = A, activations = B), so a lane ends a product
// holding one token's 4 consecutive output rows per 16-row tile.  The k order inside every
// 64-deep k-pair is permuted so that 4 tiles of one product are exactly 2 B fragments of the next:
// lane group g (lanes 16g..16g+15) holds k = 16g+0..7 in the even k-step and 16g+8..15 in the odd
// one; the producing product's A rows are taken in the matching order (tile q, row i -> unit
// 16(i/4) + 4q + i%4 of its 64-unit group: a free choice of which rows a lane loads).
//
// Bound: each workgroup streams every weight of the site once (2 MB at D=256, Hd=512), so a
// workgroup is L2-bandwidth-bound (~20 us at ~100 GB/s per CU) rather than MFMA-bound (6.4 us of
// MFMA for 32 tokens); the kernel exists for grids of tens to a few hundred workgroups, where the
// 64-128-token workgroups of hv_mhc_fused.hip leave most CUs idle.  A group launch runs up to
// three sites that read the same x (the attention's q / k / v projections) as one grid.
#include <type_traits>

#include "hv_common.h"

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));   // native vector: no struct memcpy
                                                                 // (HIP's uint4 kept the ring in scratch)
__device__ __forceinline__ f32x4 mfma_t(v4u a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                 c, 0, 0, 0);
}

struct TokSite {
  const unsigned short* x;
  const unsigned short* a1t;   // [2HD, D]
  const unsigned short* w2;    // [HD, 2HD]
  const unsigned short* wct;   // [D, D+HD]
  const unsigned short* res;   // optional [T, D]
  const float* c1;             // [2HD]
  const float* b2;             // [HD]
  const float* g_post;         // [D]
  const float* b_post;         // [D]
  unsigned short* out;         // [T, D]
};
constexpr int kTokMaxSites = 3;
struct TokArgs {
  TokSite s[kTokMaxSites];
  int T;
};

template <int D, int HD, int TW>
struct CfgT {
  static constexpr int NW = 8, NT = 512, TT = TW / 16;
  static constexpr int KS1 = D / 32, KP1 = D / 64;                 // GEMM1 contraction (D)
  static constexpr int KS2 = 2 * HD / 32, KP2 = 2 * HD / 64;       // GEMM2 contraction (2HD)
  static constexpr int KSH = HD / 32;                              // h2 k-steps of GEMM3
  static constexpr int XP = D / 64, KP3 = (D + HD) / 64;           // GEMM3 contraction (D + HD)
  static constexpr int N1W = 2 * HD / NW, G1 = N1W / 64;           // GEMM1 units per wave, 64-unit groups
  static constexpr int N2W = HD / NW, G2 = N2W / 64;
  static constexpr int N3W = D / NW, J3 = N3W / 16;                // GEMM3 output columns per wave, tiles
  static constexpr int S1 = G1 * KP1, S2 = G2 * KP2, S3 = KP3, S = S1 + S2 + S3;   // flat k-pair schedule
  // LDS: B-fragment images (1 KiB per token tile and k-step; z is dead after GEMM1, so h2 is
  // written over it), fp32 constants, then one 4 KiB weight transposer per wave
  static constexpr int ZB = TT * KS1 * 1024, H2B = TT * KSH * 1024;
  static constexpr int ZF = 0, H2F = 0, XF = ZB > H2B ? ZB : H2B, H1F = XF + TT * KS1 * 1024;
  static constexpr int CST = H1F + TT * KS2 * 1024;
  static constexpr int C1S = CST, B2S = C1S + 2 * HD * 4, GPS = B2S + HD * 4, BPS = GPS + D * 4;
  static constexpr int TRS = BPS + D * 4, LDS = TRS + NW * 4096;
  static constexpr int YROW = D + 4;                               // fp32 y rows (aliases H1F)
  static constexpr int CPL = D / 64;                               // LN_post columns per lane
  static_assert(TW == 16 || TW == 32, "token tile");
  static_assert(D % 128 == 0 && HD % 512 == 0 && G1 >= 1 && G2 >= 1 && J3 >= 1 && J3 <= 4, "shape");
  static_assert(TW * YROW * 4 <= TT * KS2 * 1024, "y fits the h1 images");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E) -- the ring of weight
// registers is indexed by the step, which must be a constant for the ring to stay in registers
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Weight stream.  A weight fragment in the MFMA A layout (lane l: row l % 16, 16 B at k-chunk
// l / 16) makes every lane of a load instruction read a different row -- 64 separate 16-B requests
// per instruction, which held the stream at ~36 GB/s per CU.  Instead each load instruction reads
// 8 whole 128-B row segments (lane l: row l / 8, 16-B chunk l % 8: ~106 GB/s per CU measured), the
// wave writes them to its private 4 KiB LDS transposer (2 tiles x 16 rows x 128 B; no barrier: one
// wave's DS operations execute in order) and reads them back as A fragments.  Chunk c of row r is
// stored at slot c ^ tsw(r): conflict-free for the ds_write_b128 (8-lane groups, one row each) and
// for the fragment ds_read_b128 (16-lane groups over 16 rows x 2 chunks; found by search).
__device__ __forceinline__ int tsw(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }

template <int D, int HD, int TW, int PF>
__global__ void __launch_bounds__(512, 1) mhc_tok_kernel(TokArgs args) {
  using C = CfgT<D, HD, TW>;
  constexpr int TT = C::TT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // site by uniform selects: indexing the by-value kernarg array with blockIdx.y would copy it to
  // scratch
  const int sy = blockIdx.y;
  const TokSite st = sy == 0 ? args.s[0] : (sy == 1 ? args.s[1] : args.s[2]);
  const int T = args.T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long t0 = (long)blockIdx.x * TW;
  const unsigned short* __restrict__ x = st.x;
  const unsigned short* __restrict__ a1t = st.a1t;
  const unsigned short* __restrict__ w2 = st.w2;
  const unsigned short* __restrict__ wct = st.wct;

  // ---- fp32 constants -> LDS (read in the epilogues: an epilogue global load would sit behind
  // the in-flight weight loads, vmcnt retires in order)
  float* const c1s = reinterpret_cast<float*>(smem + C::C1S);
  float* const b2s = reinterpret_cast<float*>(smem + C::B2S);
  float* const gps = reinterpret_cast<float*>(smem + C::GPS);
  float* const bps = reinterpret_cast<float*>(smem + C::BPS);
  for (int i = tid; i < 2 * HD / 4; i += C::NT)
    reinterpret_cast<float4*>(c1s)[i] = reinterpret_cast<const float4*>(st.c1)[i];
  for (int i = tid; i < HD / 4; i += C::NT)
    reinterpret_cast<float4*>(b2s)[i] = reinterpret_cast<const float4*>(st.b2)[i];
  for (int i = tid; i < D / 4; i += C::NT) {
    reinterpret_cast<float4*>(gps)[i] = reinterpret_cast<const float4*>(st.g_post)[i];
    reinterpret_cast<float4*>(bps)[i] = reinterpret_cast<const float4*>(st.b_post)[i];
  }

  // ---- x of this wave's token tile (waves 0..TT-1), issued before the weight ring
  uint4 xv[C::KP1][2];
  if (w < TT) {
    const long tok = min(t0 + w * 16 + fr, (long)T - 1);
#pragma unroll
    for (int p = 0; p < C::KP1; ++p) {
      xv[p][0] = *reinterpret_cast<const uint4*>(x + tok * D + 64 * p + 16 * fg);
      xv[p][1] = *reinterpret_cast<const uint4*>(x + tok * D + 64 * p + 16 * fg + 8);
    }
  }

  // ---- flat k-pair schedule over the three products.  Step s covers one 64-deep k-pair of 4
  // (GEMM1/2) or J3 (GEMM3) 16-row tiles: instruction i reads rows 8 (i & 1) + lane / 8 of tile
  // i / 2, whole 128-B k-pair segments (see tsw)
  const int lr = lane >> 3, lc = lane & 7;
  auto load_step = [&](auto sc, v4u (&r)[8]) {
    constexpr int s = decltype(sc)::value;
    if constexpr (s < C::S1) {
      constexpr int g = s / C::KP1, p = s % C::KP1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;     // row rr of tile q -> unit (permuted order)
        const int u = w * C::N1W + 64 * g + 16 * (rr >> 2) + 4 * q + (rr & 3);
        r[i] = *reinterpret_cast<const v4u*>(a1t + (long)u * D + 64 * p + 8 * (lc ^ tsw(rr)));
      }
    } else if constexpr (s < C::S1 + C::S2) {
      constexpr int s2 = s - C::S1, g = s2 / C::KP2, p = s2 % C::KP2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;
        const int u = w * C::N2W + 64 * g + 16 * (rr >> 2) + 4 * q + (rr & 3);
        r[i] = *reinterpret_cast<const v4u*>(w2 + (long)u * (2 * HD) + 64 * p + 8 * (lc ^ tsw(rr)));
      }
    } else {
      constexpr int p = s - C::S1 - C::S2;
#pragma unroll
      for (int i = 0; i < 2 * C::J3; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;     // GEMM3 output columns in natural order
        r[i] = *reinterpret_cast<const v4u*>(wct + (long)(w * C::N3W + 16 * q + rr) * (D + HD) + 64 * p +
                                               8 * (lc ^ tsw(rr)));
      }
    }
  };
  // the wave's transposer: write instructions [4h, 4h + 4) (tiles 2h, 2h + 1), read their fragments
  unsigned char* const trs = smem + C::TRS + w * 4096;
  auto transpose_half = [&](auto hc, auto nc, const v4u (&r)[8], v4u (&a)[4][2]) {
    constexpr int h = decltype(hc)::value, ntiles = decltype(nc)::value;
    static_for<4 * h, (4 * h + 4 < 2 * ntiles ? 4 * h + 4 : 2 * ntiles)>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      *reinterpret_cast<v4u*>(trs + ((i >> 1) & 1) * 2048 + (8 * (i & 1) + lr) * 128 + 16 * lc) = r[i];
    });
    static_for<2 * h, (2 * h + 2 < ntiles ? 2 * h + 2 : ntiles)>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
#pragma unroll
      for (int e = 0; e < 2; ++e)
        a[q][e] = *reinterpret_cast<const v4u*>(trs + (q & 1) * 2048 + fr * 128 + 16 * ((2 * fg + e) ^ tsw(fr)));
    });
  };
  v4u ring[PF][8];
  static_for<0, PF>([&](auto ic) __attribute__((always_inline)) { load_step(ic, ring[decltype(ic)::value]); });

  // ---- LN_pre (waves 0..TT-1): x and z = (x - mean) * rstd as B-fragment images
  if (w < TT) {
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) s += __uint_as_float(v[e] << 16) + __uint_as_float(v[e] & 0xffff0000u);
      }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = __uint_as_float(v[e] << 16) - mu, b = __uint_as_float(v[e] & 0xffff0000u) - mu;
          q += a * a + b * b;
        }
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
        uint32_t z[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          z[e] = pack_bf16x2((__uint_as_float(v[e] << 16) - mu) * rs, (__uint_as_float(v[e] & 0xffff0000u) - mu) * rs);
        const int blk = (w * C::KS1 + 2 * p + h) * 1024 + lane * 16;
        *reinterpret_cast<uint4*>(smem + C::XF + blk) = xv[p][h];
        *reinterpret_cast<uint4*>(smem + C::ZF + blk) = make_uint4(z[0], z[1], z[2], z[3]);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();       // z / x images and the constants visible (vmcnt NOT drained)

  f32x4 acc[4][TT];
  // epilogue of GEMM1 / GEMM2 (64-unit group at `unit0`): bias + GELU -> the even / odd k-step
  // images of k-pair unit0 / 64 of the next product
  auto act_store = [&](const float* bias, int unit0, int img, int ks_img) __attribute__((always_inline)) {
    const float4* bp = reinterpret_cast<const float4*>(bias + unit0 + 16 * fg);
    const float4 bq[4] = {bp[0], bp[1], bp[2], bp[3]};
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      uint32_t hv[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 a = acc[q][t];
        hv[2 * q] = pack_bf16x2(hv_gelu_fast(a[0] + bq[q].x), hv_gelu_fast(a[1] + bq[q].y));
        hv[2 * q + 1] = pack_bf16x2(hv_gelu_fast(a[2] + bq[q].z), hv_gelu_fast(a[3] + bq[q].w));
      }
      const int kp = unit0 / 64;
      unsigned char* b0 = smem + img + ((t * ks_img + 2 * kp) * 1024) + lane * 16;
      *reinterpret_cast<uint4*>(b0) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
      *reinterpret_cast<uint4*>(b0 + 1024) = make_uint4(hv[4], hv[5], hv[6], hv[7]);
    }
  };

  static_for<0, C::S>([&](auto sc) __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value;
    constexpr int NTL = s < C::S1 + C::S2 ? 4 : C::J3;   // tiles of this step
    v4u raw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = ring[s % PF][i];
    if constexpr (s + PF < C::S) load_step(std::integral_constant<int, s + PF>{}, ring[s % PF]);
    // keep the refill here: left alone the scheduler sinks it next to its use (vmcnt(0) waits)
    __builtin_amdgcn_sched_barrier(0);
    v4u cur[4][2];
    transpose_half(std::integral_constant<int, 0>{}, std::integral_constant<int, NTL>{}, raw, cur);
    if constexpr (NTL > 2) transpose_half(std::integral_constant<int, 1>{}, std::integral_constant<int, NTL>{}, raw, cur);
    if constexpr (s < C::S1) {
      // ------------------------------------------------ GEMM1: z [TW x D] -> h1 units of group g
      constexpr int g = s / C::KP1, p = s % C::KP1;
      if constexpr (p == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < TT; ++t) acc[q][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const unsigned char* bz = smem + C::ZF + (t * C::KS1 + 2 * p) * 1024 + lane * 16;
        const uint4 be = *reinterpret_cast<const uint4*>(bz), bo = *reinterpret_cast<const uint4*>(bz + 1024);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q][t] = mfma_t(cur[q][0], be, acc[q][t]);
          acc[q][t] = mfma_t(cur[q][1], bo, acc[q][t]);
        }
      }
      if constexpr (p == C::KP1 - 1) act_store(c1s, w * C::N1W + 64 * g, C::H1F, C::KS2);
      if constexpr (s == C::S1 - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // h1 images complete
      }
    } else if constexpr (s < C::S1 + C::S2) {
      // ------------------------------------------------ GEMM2: h1 [TW x 2HD] -> h2 units of group g
      constexpr int s2 = s - C::S1, g = s2 / C::KP2, p = s2 % C::KP2;
      if constexpr (p == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < TT; ++t) acc[q][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const unsigned char* bh = smem + C::H1F + (t * C::KS2 + 2 * p) * 1024 + lane * 16;
        const uint4 be = *reinterpret_cast<const uint4*>(bh), bo = *reinterpret_cast<const uint4*>(bh + 1024);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q][t] = mfma_t(cur[q][0], be, acc[q][t]);
          acc[q][t] = mfma_t(cur[q][1], bo, acc[q][t]);
        }
      }
      if constexpr (p == C::KP2 - 1) act_store(b2s, w * C::N2W + 64 * g, C::H2F, C::KSH);
      if constexpr (s == C::S1 + C::S2 - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // h2 images complete; h1 no longer read (y may overwrite it)
      }
    } else {
      // ------------------------------------------------ GEMM3: [x | h2] [TW x (D+HD)] -> y columns
      constexpr int p = s - C::S1 - C::S2;
      if constexpr (p == 0)
#pragma unroll
        for (int j = 0; j < C::J3; ++j)
#pragma unroll
          for (int t = 0; t < TT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const unsigned char* bb = p < C::XP ? smem + C::XF + (t * C::KS1 + 2 * p) * 1024
                                            : smem + C::H2F + (t * C::KSH + 2 * (p - C::XP)) * 1024;
        const uint4 be = *reinterpret_cast<const uint4*>(bb + lane * 16);
        const uint4 bo = *reinterpret_cast<const uint4*>(bb + 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < C::J3; ++j) {
          acc[j][t] = mfma_t(cur[j][0], be, acc[j][t]);
          acc[j][t] = mfma_t(cur[j][1], bo, acc[j][t]);
        }
      }
    }
  });

  // ---- y^T tiles -> fp32 rows in LDS (over the h1 images), then LN_post (+ residual) per token
  float* const ys = reinterpret_cast<float*>(smem + C::H1F);
#pragma unroll
  for (int j = 0; j < C::J3; ++j)
#pragma unroll
    for (int t = 0; t < TT; ++t)
      *reinterpret_cast<f32x4*>(ys + (t * 16 + fr) * C::YROW + w * C::N3W + 16 * j + 4 * fg) = acc[j][t];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  constexpr int CPL = C::CPL;
  float gv[CPL], bv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) { gv[c] = gps[lane * CPL + c]; bv[c] = bps[lane * CPL + c]; }
#pragma unroll
  for (int i = 0; i < TW / 8; ++i) {
    const int lt = w + 8 * i;
    const long tok = t0 + lt;
    float v[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) v[c] = ys[lt * C::YROW + lane * CPL + c];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) s += v[c];
    const float mu = wave_sum(s) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) { const float d0 = v[c] - mu; q += d0 * d0; }
    const float inv = rsqrtf(wave_sum(q) * (1.0f / D) + 1e-5f);
    if (tok < T) {
      float o[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) o[c] = (v[c] - mu) * inv * gv[c] + bv[c];
      unsigned short* op = st.out + tok * D + lane * CPL;
      if (st.res) {
        const unsigned short* rp = st.res + tok * D + lane * CPL;
#pragma unroll
        for (int c = 0; c < CPL; ++c) o[c] += bf2f(rp[c]);
      }
      uint32_t pk[CPL / 2];
#pragma unroll
      for (int c = 0; c < CPL / 2; ++c) pk[c] = pack_bf16x2(o[2 * c], o[2 * c + 1]);
      if constexpr (CPL == 2) {
        *reinterpret_cast<uint32_t*>(op) = pk[0];
      } else if constexpr (CPL == 4) {
        *reinterpret_cast<uint2*>(op) = make_uint2(pk[0], pk[1]);
      } else {
#pragma unroll
        for (int c = 0; c < CPL / 8; ++c)
          *reinterpret_cast<uint4*>(op + 8 * c) = make_uint4(pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Hidden-split form (HV_MV_TOKSPLIT2 / 4; D = 256, Hd = 512 or 1024, 16-token tiles).  With few tiles
// (T = 401 at B=1: 26 workgroups) every workgroup streaming all 2 MB of the site's weights leaves
// most CUs idle; here NSPL workgroups share a tile, part s owning the h2 units
// [s HD/NSPL, (s+1) HD/NSPL): each part runs GEMM1 in full (the h1 all of GEMM2 reads), GEMM2 for
// its h2 units only (the 8 waves split the contraction four / two ways per 64-unit group and
// sum in LDS in fixed order), and the share of GEMM3 those units (+ x columns [s D/NSPL, ..))
// contribute.  The parts' fp32 partial y go to a workspace; the LAST part to finish (agent-scope
// release + ticket counter, acquire) sums them in part order (deterministic) and runs LN_post.
// Weight bytes per workgroup: A1 + (W2 + Wc) / NSPL (0.86 MB at NSPL = 4 instead of 2 MB).
template <int D, int HD, int NSPL>
struct CfgS {
  static constexpr int NW = 8, NT = 512, TW = 16;
  static constexpr int KS1 = D / 32, KP1 = D / 64;                 // GEMM1 contraction (D)
  static constexpr int KS2 = 2 * HD / 32, KP2 = 2 * HD / 64;       // GEMM2 contraction (2HD)
  static constexpr int HDS = HD / NSPL;                            // h2 units of one part
  static constexpr int NG2 = HDS / 64, WPG = NW / NG2, KPW2 = KP2 / WPG;   // unit groups, waves per group, k-pairs per wave
  static constexpr int XPP = D / NSPL / 64;                        // x k-pairs of this part's GEMM3 share
  static constexpr int KP3 = XPP + NG2;                            // + its h2 k-pairs
  static constexpr int N1W = 2 * HD / NW, G1 = N1W / 64;
  static constexpr int N3W = D / NW, J3 = N3W / 16;
  static constexpr int S1 = G1 * KP1, S2 = KPW2, S3 = KP3, S = S1 + S2 + S3;
  // LDS: z (then this part's h2 images) | x images | h1 images | GEMM2 partials | constants | transposers | flag
  static constexpr int ZB = KS1 * 1024, H2B = (HDS / 32) * 1024;
  static constexpr int ZF = 0, H2F = 0, XF = ZB > H2B ? ZB : H2B, H1F = XF + KS1 * 1024;
  static constexpr int R2F = H1F + KS2 * 1024;                     // [NW][4 tiles][64 lanes] f32x4 (WPG > 1)
  static constexpr int R2B = WPG > 1 ? NW * 4 * 64 * 16 : 0;
  static constexpr int C1S = R2F + R2B, B2S = C1S + 2 * HD * 4, GPS = B2S + HD * 4, BPS = GPS + D * 4;
  static constexpr int TRS = BPS + D * 4, FLAG = TRS + NW * 4096, LDS = FLAG + 16;
  static constexpr int CPL = D / 64;                               // LN_post columns per lane
  static_assert(NG2 >= 1 && NW % NG2 == 0 && KP2 % WPG == 0 && XPP >= 1 && (D / NSPL) % 64 == 0, "split shape");
  static_assert(D % 128 == 0 && G1 >= 1 && J3 >= 1 && J3 <= 4 && CPL == 4, "shape");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct TokSplitArgs {
  TokSite s[kTokMaxSites];
  int T, tiles;
  float* work;       // [sites][tiles][NSPL][16][D] fp32 partial y
  int* count;        // [sites][tiles] arrival counters, zero before the launch (left zero)
};

template <int D, int HD, int NSPL, int PF>
__global__ void __launch_bounds__(512, 1) mhc_toks_kernel(TokSplitArgs args) {
  using C = CfgS<D, HD, NSPL>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int sy = blockIdx.y;
  const TokSite st = sy == 0 ? args.s[0] : (sy == 1 ? args.s[1] : args.s[2]);
  const int T = args.T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int tile = blockIdx.x / NSPL, part = blockIdx.x % NSPL;
  const long t0 = (long)tile * 16;
  const unsigned short* __restrict__ x = st.x;
  const unsigned short* __restrict__ a1t = st.a1t;
  const unsigned short* __restrict__ w2 = st.w2;
  const unsigned short* __restrict__ wct = st.wct;

  float* const c1s = reinterpret_cast<float*>(smem + C::C1S);
  float* const b2s = reinterpret_cast<float*>(smem + C::B2S);
  float* const gps = reinterpret_cast<float*>(smem + C::GPS);
  float* const bps = reinterpret_cast<float*>(smem + C::BPS);
  for (int i = tid; i < 2 * HD / 4; i += C::NT)
    reinterpret_cast<float4*>(c1s)[i] = reinterpret_cast<const float4*>(st.c1)[i];
  for (int i = tid; i < HD / 4; i += C::NT)
    reinterpret_cast<float4*>(b2s)[i] = reinterpret_cast<const float4*>(st.b2)[i];
  for (int i = tid; i < D / 4; i += C::NT) {
    reinterpret_cast<float4*>(gps)[i] = reinterpret_cast<const float4*>(st.g_post)[i];
    reinterpret_cast<float4*>(bps)[i] = reinterpret_cast<const float4*>(st.b_post)[i];
  }
  uint4 xv[C::KP1][2];
  if (w == 0) {
    const long tok = min(t0 + fr, (long)T - 1);
#pragma unroll
    for (int p = 0; p < C::KP1; ++p) {
      xv[p][0] = *reinterpret_cast<const uint4*>(x + tok * D + 64 * p + 16 * fg);
      xv[p][1] = *reinterpret_cast<const uint4*>(x + tok * D + 64 * p + 16 * fg + 8);
    }
  }

  // flat k-pair schedule: GEMM1 (all 2HD units), GEMM2 (this wave's contraction share of its unit
  // group), GEMM3 (this part's x / h2 k-pairs)
  const int lr = lane >> 3, lc = lane & 7;
  const int g2 = w / C::WPG, kq = w % C::WPG;
  auto load_step = [&](auto sc, v4u (&r)[8]) {
    constexpr int s = decltype(sc)::value;
    if constexpr (s < C::S1) {
      constexpr int g = s / C::KP1, p = s % C::KP1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;
        const int u = w * C::N1W + 64 * g + 16 * (rr >> 2) + 4 * q + (rr & 3);
        r[i] = *reinterpret_cast<const v4u*>(a1t + (long)u * D + 64 * p + 8 * (lc ^ tsw(rr)));
      }
    } else if constexpr (s < C::S1 + C::S2) {
      constexpr int s2 = s - C::S1;
      const int kp = kq * C::KPW2 + s2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;
        const int u = part * C::HDS + 64 * g2 + 16 * (rr >> 2) + 4 * q + (rr & 3);
        r[i] = *reinterpret_cast<const v4u*>(w2 + (long)u * (2 * HD) + 64 * kp + 8 * (lc ^ tsw(rr)));
      }
    } else {
      constexpr int p = s - C::S1 - C::S2;
      const int col0 = p < C::XPP ? 64 * (part * C::XPP + p) : D + part * C::HDS + 64 * (p - C::XPP);
#pragma unroll
      for (int i = 0; i < 2 * C::J3; ++i) {
        const int rr = 8 * (i & 1) + lr, q = i >> 1;
        r[i] = *reinterpret_cast<const v4u*>(wct + (long)(w * C::N3W + 16 * q + rr) * (D + HD) + col0 +
                                               8 * (lc ^ tsw(rr)));
      }
    }
  };
  unsigned char* const trs = smem + C::TRS + w * 4096;
  auto transpose_half = [&](auto hc, auto nc, const v4u (&r)[8], v4u (&a)[4][2]) {
    constexpr int h = decltype(hc)::value, ntiles = decltype(nc)::value;
    static_for<4 * h, (4 * h + 4 < 2 * ntiles ? 4 * h + 4 : 2 * ntiles)>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      *reinterpret_cast<v4u*>(trs + ((i >> 1) & 1) * 2048 + (8 * (i & 1) + lr) * 128 + 16 * lc) = r[i];
    });
    static_for<2 * h, (2 * h + 2 < ntiles ? 2 * h + 2 : ntiles)>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
#pragma unroll
      for (int e = 0; e < 2; ++e)
        a[q][e] = *reinterpret_cast<const v4u*>(trs + (q & 1) * 2048 + fr * 128 + 16 * ((2 * fg + e) ^ tsw(fr)));
    });
  };
  v4u ring[PF][8];
  static_for<0, PF>([&](auto ic) __attribute__((always_inline)) { load_step(ic, ring[decltype(ic)::value]); });

  // LN_pre (wave 0): x and z = (x - mean) * rstd as B-fragment images
  if (w == 0) {
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) s += __uint_as_float(v[e] << 16) + __uint_as_float(v[e] & 0xffff0000u);
      }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = __uint_as_float(v[e] << 16) - mu, b = __uint_as_float(v[e] & 0xffff0000u) - mu;
          q += a * a + b * b;
        }
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int p = 0; p < C::KP1; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t v[4] = {xv[p][h].x, xv[p][h].y, xv[p][h].z, xv[p][h].w};
        uint32_t z[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          z[e] = pack_bf16x2((__uint_as_float(v[e] << 16) - mu) * rs, (__uint_as_float(v[e] & 0xffff0000u) - mu) * rs);
        const int blk = (2 * p + h) * 1024 + lane * 16;
        *reinterpret_cast<uint4*>(smem + C::XF + blk) = xv[p][h];
        *reinterpret_cast<uint4*>(smem + C::ZF + blk) = make_uint4(z[0], z[1], z[2], z[3]);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc[4];
  auto act_store = [&](const float* bias, int unit0, int img, int ks_img) __attribute__((always_inline)) {
    const float4* bp = reinterpret_cast<const float4*>(bias + unit0 + 16 * fg);
    const float4 bq[4] = {bp[0], bp[1], bp[2], bp[3]};
    uint32_t hv[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 a = acc[q];
      hv[2 * q] = pack_bf16x2(hv_gelu_fast(a[0] + bq[q].x), hv_gelu_fast(a[1] + bq[q].y));
      hv[2 * q + 1] = pack_bf16x2(hv_gelu_fast(a[2] + bq[q].z), hv_gelu_fast(a[3] + bq[q].w));
    }
    (void)ks_img;
    unsigned char* b0 = smem + img + (2 * (unit0 / 64)) * 1024 + lane * 16;
    *reinterpret_cast<uint4*>(b0) = make_uint4(hv[0], hv[1], hv[2], hv[3]);
    *reinterpret_cast<uint4*>(b0 + 1024) = make_uint4(hv[4], hv[5], hv[6], hv[7]);
  };

  static_for<0, C::S>([&](auto sc) __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value;
    constexpr int NTL = s < C::S1 + C::S2 ? 4 : C::J3;
    v4u raw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = ring[s % PF][i];
    if constexpr (s + PF < C::S) load_step(std::integral_constant<int, s + PF>{}, ring[s % PF]);
    __builtin_amdgcn_sched_barrier(0);
    v4u cur[4][2];
    transpose_half(std::integral_constant<int, 0>{}, std::integral_constant<int, NTL>{}, raw, cur);
    if constexpr (NTL > 2) transpose_half(std::integral_constant<int, 1>{}, std::integral_constant<int, NTL>{}, raw, cur);
    if constexpr (s < C::S1) {
      // GEMM1: z [16 x D] -> h1 units of group g (all 2HD units: every part needs all of h1)
      constexpr int g = s / C::KP1, p = s % C::KP1;
      if constexpr (p == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned char* bz = smem + C::ZF + (2 * p) * 1024 + lane * 16;
      const uint4 be = *reinterpret_cast<const uint4*>(bz), bo = *reinterpret_cast<const uint4*>(bz + 1024);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q] = mfma_t(cur[q][0], be, acc[q]);
        acc[q] = mfma_t(cur[q][1], bo, acc[q]);
      }
      if constexpr (p == C::KP1 - 1) act_store(c1s, w * C::N1W + 64 * g, C::H1F, C::KS2);
      if constexpr (s == C::S1 - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // h1 images complete (z no longer read)
      }
    } else if constexpr (s < C::S1 + C::S2) {
      // GEMM2: this wave's k-pairs [kq KPW2, (kq+1) KPW2) of unit group g2 of this part
      constexpr int s2 = s - C::S1;
      if constexpr (s2 == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kp = kq * C::KPW2 + s2;
      const unsigned char* bh = smem + C::H1F + (2 * kp) * 1024 + lane * 16;
      const uint4 be = *reinterpret_cast<const uint4*>(bh), bo = *reinterpret_cast<const uint4*>(bh + 1024);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q] = mfma_t(cur[q][0], be, acc[q]);
        acc[q] = mfma_t(cur[q][1], bo, acc[q]);
      }
      if constexpr (s2 == C::KPW2 - 1) {
        // contraction shares of a unit group -> LDS; its first wave sums them in share order,
        // adds b2, GELU -> the h2 images of this part (over z)
        if (kq != 0)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4*>(smem + C::R2F + ((w * 4 + q) * 64 + lane) * 16) = acc[q];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kq == 0) {
#pragma unroll
          for (int k = 1; k < C::WPG; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[q] += *reinterpret_cast<const f32x4*>(smem + C::R2F + (((w + k) * 4 + q) * 64 + lane) * 16);
          act_store(b2s + part * C::HDS, 64 * g2, C::H2F, C::HDS / 32);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // this part's h2 images complete
      }
    } else {
      // GEMM3 share: [x k-pairs of this part | this part's h2] -> partial y columns
      constexpr int p = s - C::S1 - C::S2;
      if constexpr (p == 0)
#pragma unroll
        for (int j = 0; j < C::J3; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned char* bb = p < C::XPP ? smem + C::XF + (2 * (part * C::XPP + p)) * 1024
                                           : smem + C::H2F + (2 * (p - C::XPP)) * 1024;
      const uint4 be = *reinterpret_cast<const uint4*>(bb + lane * 16);
      const uint4 bo = *reinterpret_cast<const uint4*>(bb + 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < C::J3; ++j) {
        acc[j] = mfma_t(cur[j][0], be, acc[j]);
        acc[j] = mfma_t(cur[j][1], bo, acc[j]);
      }
    }
  });

  // ---- partial y -> workspace; the last part of the tile to arrive reduces (fixed part order).
  // Hand-off (cdna_hip_programming.md Guideline 16): every wave drains its stores, lane 0
  // releases at agent scope and adds to the tile's counter, the last adder acquires, then plain
  // loads.  (Round 5's fence-free write-through variant measured equal and was removed: it relied
  // on measured, not architectural, visibility.)
  const long tbase = ((long)sy * args.tiles + tile) * NSPL;
  float* const wsp = args.work + (tbase + part) * 16 * D;
#pragma unroll
  for (int j = 0; j < C::J3; ++j)
    *reinterpret_cast<f32x4*>(wsp + fr * D + w * C::N3W + 16 * j + 4 * fg) = acc[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* const flag = reinterpret_cast<int*>(smem + C::FLAG);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* const cnt = args.count + (long)sy * args.tiles + tile;
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == NSPL - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // zero for the next launch
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;

  constexpr int CPL = C::CPL;
  float gv[CPL], bv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) { gv[c] = gps[lane * CPL + c]; bv[c] = bps[lane * CPL + c]; }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lt = w + 8 * i;
    const long tok = t0 + lt;
    const float* src = args.work + tbase * 16 * D + lt * D + lane * CPL;
    f32x4 yq[NSPL];
#pragma unroll
    for (int q = 0; q < NSPL; ++q) yq[q] = *reinterpret_cast<const f32x4*>(src + (long)q * 16 * D);
    f32x4 yv = yq[0];
#pragma unroll
    for (int q = 1; q < NSPL; ++q) yv += yq[q];
    float v[CPL] = {yv[0], yv[1], yv[2], yv[3]};
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) s += v[c];
    const float mu = wave_sum(s) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) { const float d0 = v[c] - mu; q += d0 * d0; }
    const float inv = rsqrtf(wave_sum(q) * (1.0f / D) + 1e-5f);
    if (tok < T) {
      float o[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) o[c] = (v[c] - mu) * inv * gv[c] + bv[c];
      if (st.res) {
        const unsigned short* rp = st.res + tok * D + lane * CPL;
#pragma unroll
        for (int c = 0; c < CPL; ++c) o[c] += bf2f(rp[c]);
      }
      *reinterpret_cast<uint2*>(st.out + tok * D + lane * CPL) =
          make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
    }
  }
}

template <int D, int HD, int NSPL, int PF>
int launch_toks(const TokSplitArgs& ta, int nsites, hipStream_t s) {
  using C = CfgS<D, HD, NSPL>;
  auto k = mhc_toks_kernel<D, HD, NSPL, PF>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  hv_diag_count(HV_KF_MHC_FUSED);
  k<<<dim3(ta.tiles * NSPL, nsites), C::NT, C::LDS, s>>>(ta);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

template <int D, int HD, int TW, int PF>
int launch_tok(const TokArgs& ta, int nsites, hipStream_t s) {
  using C = CfgT<D, HD, TW>;
  auto k = mhc_tok_kernel<D, HD, TW, PF>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  hv_diag_count(HV_KF_MHC_FUSED);
  k<<<dim3(hv_cdiv(ta.T, TW), nsites), C::NT, C::LDS, s>>>(ta);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

}  // namespace

// (D, Hd) pairs of the token-tile kernel
extern "C" int hv_mhc_tok_supported(int D, int Hd) {
  return (D == 128 && Hd == 512) || (D == 256 && Hd == 512) || (D == 256 && Hd == 1024);
}

// Launch n <= 3 sites of equal (D, Hd, T) as one grid (called by hv_mhc_fused / hv_mhc_fused_group
// after argument validation).  Token tile: HV_MV_TOK16 forces 16 tokens, otherwise 32 where the
// shape allows it.
int hv_mhc_tok_launch(const hv_mhc_fused_args* a, int n, hipStream_t s) {
  if (n < 1 || n > kTokMaxSites) return HV_EINVAL;
  TokArgs ta{};
  ta.T = a[0].T;
  for (int i = 0; i < n; ++i) {
    ta.s[i] = TokSite{(const unsigned short*)a[i].x, (const unsigned short*)a[i].a1t, (const unsigned short*)a[i].w2,
                      (const unsigned short*)a[i].wct, (const unsigned short*)a[i].residual, a[i].c1, a[i].b2,
                      a[i].g_post, a[i].b_post, (unsigned short*)a[i].out};
  }
  const bool t16 = (a[0].variant & HV_MV_TOK16) != 0;
  const int D = a[0].D, Hd = a[0].Hd;
  const int spl = a[0].variant & HV_MV_TOKSPLIT4 ? 4 : (a[0].variant & HV_MV_TOKSPLIT2 ? 2 : 1);
  if (spl > 1) {
    // hidden-split form: workspace + zeroed arrival counters from the caller (hv_kernels.h)
    if (D != 256 || (Hd != 512 && Hd != 1024) || !a[0].split_work || !a[0].split_count) return HV_EINVAL;
    TokSplitArgs sa{};
    for (int i = 0; i < n; ++i) sa.s[i] = ta.s[i];
    sa.T = ta.T;
    sa.tiles = hv_cdiv(ta.T, 16);
    sa.work = a[0].split_work;
    sa.count = a[0].split_count;
    if (Hd == 1024) return spl == 4 ? launch_toks<256, 1024, 4, 2>(sa, n, s) : launch_toks<256, 1024, 2, 2>(sa, n, s);
    return spl == 4 ? launch_toks<256, 512, 4, 2>(sa, n, s) : launch_toks<256, 512, 2, 2>(sa, n, s);
  }
  if (D == 128 && Hd == 512) return t16 ? launch_tok<128, 512, 16, 2>(ta, n, s) : launch_tok<128, 512, 32, 2>(ta, n, s);
  if (D == 256 && Hd == 512) return t16 ? launch_tok<256, 512, 16, 2>(ta, n, s) : launch_tok<256, 512, 32, 2>(ta, n, s);
  if (D == 256 && Hd == 1024) return launch_tok<256, 1024, 16, 2>(ta, n, s);
  return HV_EUNSUPPORTED;
}
