// Fused mHC token chain (gfx950, bf16 MFMA), replacing the six launches of the unfused path
// (row stats, 3 GEMMs, LayerNorm) for every site with D <= 256 and hidden width <= 512:
//
//   z   = (x - mean) * rstd                    (LN_pre core; gamma/beta folded into A1/c1)
//   h1  = GELU(z A1 + c1)          [BM x 2HD]  produced KC columns at a time, never stored
//   h2  = GELU(h1 W2^T + b2)       [BM x HD]   accumulated in registers over the 2HD chunks
//   y   = [x | h2] Wc              [BM x D]    Wc = centred [H_res ; H_post]
//   out = LN_post(y) * g2 + b2' (+ residual)   computed from the GEMM3 accumulators
//
// Reference: ManifoldHyperConnection.forward (manifold_layers.py:223-280); the algebra
// (fold + centring) is documented in hv_amd/manifold.py and DESIGN.md.  Per token tile only x
// (D*2 bytes/token) is read and out written: the [T, 2HD] and [T, HD] intermediates of the
// unfused chain never reach HBM.
//
// Weights are not staged through LDS: every weight element a workgroup needs is consumed by
// exactly one lane as an MFMA B fragment, so each lane loads its 16-byte fragments straight
// from L2 into a 2-slot register ring (chunk c+1 is in flight while chunk c computes).  LDS
// holds the x/z tile, a double-buffered h1 chunk (one barrier per chunk), h2 and a small
// LayerNorm exchange.  GEMM1 and GEMM2 are computed transposed (weights as the MFMA A operand)
// so each lane ends with 4 consecutive hidden units of one token: GELU + bf16 pack + one
// 8-byte LDS store per tile.  GELU is hv_gelu_fast (|err| <= 2.6e-5, below bf16 resolution).
#include "hv_common.h"

namespace {

template <int D, int HD, int NW>
struct Cfg {
  static constexpr int NT = 64 * NW;
  static constexpr int BM = 4096 * NW / HD;       // acc2: BM x HD/NW per wave = 16 tiles (64 regs)
  static constexpr int KC = 32;                   // 2HD chunk per step (one MFMA k-step)
  static constexpr int NCH = 2 * HD / KC;
  static constexpr int NV = (D + 63) / 64;        // row values per lane in row-wise passes
  static constexpr int XS = D * 2 + 16;           // x / z row stride (bytes), == 16 mod 64
  static constexpr int H1S = KC * 2 + 16;
  static constexpr int H2S = HD * 2 + 16;
  // GEMM1: (BM/16) x (KC/16) tiles over NW waves
  static constexpr int T1W = (BM / 16) * (KC / 16) / NW;
  // GEMM2: wave owns HD/NW columns x all BM rows
  static constexpr int R2 = BM / 16, C2 = HD / NW / 16;
  // GEMM3: (BM/16) row tiles x (D/16) col tiles; CG column groups per row tile
  static constexpr int CG = NW > BM / 16 ? NW / (BM / 16) : 1;
  static constexpr int RT3 = (BM / 16) * CG / NW;
  static constexpr int CT3 = (D / 16) / CG;
  static constexpr int KS3 = (D + HD) / 32;
  // LDS carve
  static constexpr int OFF_X = 0;
  static constexpr int OFF_Z = BM * XS;
  static constexpr int OFF_H1 = 2 * BM * XS;      // 2 buffers
  static constexpr int OFF_H2 = OFF_H1 + 2 * BM * H1S;
  static constexpr int OFF_RED = OFF_H2 + BM * H2S;   // [BM][CG] floats
  static constexpr int LDS = OFF_RED + BM * CG * 4;
  static_assert(R2 * C2 == 16, "acc2 tiling");
  static_assert(T1W >= 1 && (BM / 16) * (KC / 16) % NW == 0, "gemm1 tiling");
  static_assert(RT3 >= 1 && CT3 >= 1 && (D / 16) % CG == 0, "gemm3 tiling");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ uint4 lds16(const unsigned char* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4 gl16(const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ f32x4 mfma(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                 c, 0, 0, 0);
}

template <int D, int HD, int NW>
__global__ void __launch_bounds__(64 * NW) mhc_fused_kernel(
    const unsigned short* __restrict__ x, int T,
    const unsigned short* __restrict__ a1t,   // [2HD, D]
    const float* __restrict__ c1,             // [2HD]
    const unsigned short* __restrict__ w2,    // [HD, 2HD]
    const float* __restrict__ b2,             // [HD]
    const unsigned short* __restrict__ wct,   // [D, D+HD]
    const float* __restrict__ g_post, const float* __restrict__ b_post,
    const unsigned short* __restrict__ res,   // optional [T, D], added after LN_post
    unsigned short* __restrict__ out) {
  using C = Cfg<D, HD, NW>;
  constexpr int BM = C::BM, KC = C::KC;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long t0 = (long)blockIdx.x * BM;

  // ---------------- weight-fragment ring (registers), 2 slots
  uint4 fb1[2][C::T1W][D / 32];      // GEMM1 A fragments (rows of A1^T)
  uint4 fb2[2][C::C2];               // GEMM2 A fragments (rows of W2)
  float4 cb1[2][C::T1W];             // c1 for the 4 hidden rows a lane holds per GEMM1 tile
  auto load_chunk = [&](int slot, int ch) {
#pragma unroll
    for (int i = 0; i < C::T1W; ++i) {
      const int t = w * C::T1W + i, ct = t % (KC / 16);
      const int n = ch * KC + ct * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) fb1[slot][i][ks] = gl16(a1t + (long)n * D + ks * 32 + fg * 8);
      cb1[slot][i] = *reinterpret_cast<const float4*>(c1 + ch * KC + ct * 16 + fg * 4);
    }
#pragma unroll
    for (int b = 0; b < C::C2; ++b)
      fb2[slot][b] = gl16(w2 + (long)(w * (HD / NW) + b * 16 + fr) * (2 * HD) + ch * KC + fg * 8);
  };
  load_chunk(0, 0);
  load_chunk(1, 1);

  // ---------------- phase 0: x tile -> LDS; LN_pre -> z (bf16)
  {
    constexpr int CH = D / 8;
    for (int c = tid; c < BM * CH; c += C::NT) {
      const int r = c / CH, k = c % CH;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t0 + r < T) v = gl16(x + (t0 + r) * D + k * 8);
      *reinterpret_cast<uint4*>(smem + C::OFF_X + r * C::XS + k * 16) = v;
    }
  }
  __syncthreads();
  for (int r = w; r < BM; r += NW) {
    const unsigned short* xr = (const unsigned short*)(smem + C::OFF_X + r * C::XS);
    float v[C::NV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      const int j = lane + 64 * i;
      v[i] = j < D ? bf2f(xr[j]) : 0.f;
      s += v[i];
    }
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      const int j = lane + 64 * i;
      v[i] = j < D ? v[i] - mu : 0.f;
      q += v[i] * v[i];
    }
    const float rs = rsqrtf(wave_sum(q) / D + 1e-5f);
    unsigned short* zr = (unsigned short*)(smem + C::OFF_Z + r * C::XS);
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      const int j = lane + 64 * i;
      if (j < D) zr[j] = f2bf(v[i] * rs);
    }
  }
  __syncthreads();

  // ---------------- phase 1: 2HD chunks
  f32x4 acc2[C::R2][C::C2];
#pragma unroll
  for (int a = 0; a < C::R2; ++a)
#pragma unroll
    for (int b = 0; b < C::C2; ++b) acc2[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ch = 0; ch < C::NCH; ++ch) {
    const int slot = ch & 1;
    unsigned char* h1 = smem + C::OFF_H1 + slot * BM * C::H1S;
    // GEMM1 transposed (h1^T = A1^T z^T): a lane ends with 4 consecutive hidden units of one
    // token, i.e. one 8-byte row segment of h1 -> one ds_write_b64 of two packed bf16 pairs
#pragma unroll
    for (int i = 0; i < C::T1W; ++i) {
      const int t = w * C::T1W + i, rt = t / (KC / 16), ct = t % (KC / 16);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks)
        acc = mfma(fb1[slot][i][ks], lds16(smem + C::OFF_Z + (rt * 16 + fr) * C::XS + ks * 64 + fg * 16), acc);
      const float4 bias = cb1[slot][i];
      const uint32_t lo = pack_bf16x2(hv_gelu_fast(acc[0] + bias.x), hv_gelu_fast(acc[1] + bias.y));
      const uint32_t hi = pack_bf16x2(hv_gelu_fast(acc[2] + bias.z), hv_gelu_fast(acc[3] + bias.w));
      *reinterpret_cast<uint2*>(h1 + (rt * 16 + fr) * C::H1S + (ct * 16 + fg * 4) * 2) = make_uint2(lo, hi);
    }
    __syncthreads();
    uint4 fa[C::R2];
#pragma unroll
    for (int a = 0; a < C::R2; ++a) fa[a] = lds16(h1 + (a * 16 + fr) * C::H1S + fg * 16);
    // GEMM2 transposed too (acc2[a][b] holds h2^T: 4 hidden units x 1 token per lane)
#pragma unroll
    for (int b = 0; b < C::C2; ++b)
#pragma unroll
      for (int a = 0; a < C::R2; ++a) acc2[a][b] = mfma(fb2[slot][b], fa[a], acc2[a][b]);
    if (ch + 2 < C::NCH) load_chunk(slot, ch + 2);
  }

  // ---------------- phase 2: h2 = GELU(acc2 + b2) -> LDS (row-major [token][hidden])
#pragma unroll
  for (int b = 0; b < C::C2; ++b) {
    const int col = w * (HD / NW) + b * 16 + fg * 4;
    const float4 bias = *reinterpret_cast<const float4*>(b2 + col);
#pragma unroll
    for (int a = 0; a < C::R2; ++a) {
      const uint32_t lo = pack_bf16x2(hv_gelu_fast(acc2[a][b][0] + bias.x), hv_gelu_fast(acc2[a][b][1] + bias.y));
      const uint32_t hi = pack_bf16x2(hv_gelu_fast(acc2[a][b][2] + bias.z), hv_gelu_fast(acc2[a][b][3] + bias.w));
      *reinterpret_cast<uint2*>(smem + C::OFF_H2 + (a * 16 + fr) * C::H2S + col * 2) = make_uint2(lo, hi);
    }
  }
  __syncthreads();

  // ---------------- phase 3: y = [x | h2] Wc ; wave = (row-tile group, column group)
  const int rg = w / C::CG, cg = w % C::CG;
  f32x4 acc3[C::RT3][C::CT3];
#pragma unroll
  for (int r = 0; r < C::RT3; ++r)
#pragma unroll
    for (int c = 0; c < C::CT3; ++c) acc3[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 fw[2][C::CT3];
  auto load_wc = [&](int slot, int ks) {
#pragma unroll
    for (int c = 0; c < C::CT3; ++c)
      fw[slot][c] = gl16(wct + (long)((cg * C::CT3 + c) * 16 + fr) * (D + HD) + ks * 32 + fg * 8);
  };
  load_wc(0, 0);
  load_wc(1, 1);
#pragma unroll
  for (int ks = 0; ks < C::KS3; ++ks) {
    const int slot = ks & 1;
#pragma unroll
    for (int r = 0; r < C::RT3; ++r) {
      const int row = (rg * C::RT3 + r) * 16 + fr;
      const uint4 fa = ks < D / 32 ? lds16(smem + C::OFF_X + row * C::XS + ks * 64 + fg * 16)
                                   : lds16(smem + C::OFF_H2 + row * C::H2S + (ks - D / 32) * 64 + fg * 16);
#pragma unroll
      for (int c = 0; c < C::CT3; ++c) acc3[r][c] = mfma(fw[slot][c], fa, acc3[r][c]);   // transposed tile
    }
    if (ks + 2 < C::KS3) load_wc(slot, ks + 2);
  }

  // ---------------- phase 4: LN_post from the accumulators
  // acc3[r][c] is a transposed tile: lane -> token (rg*RT3 + r)*16 + fr, columns
  // (cg*CT3 + c)*16 + fg*4 .. +3.  A token's row = 4 lane groups x CT3 tiles (x CG waves).
  float* red = (float*)(smem + C::OFF_RED);
  float mu[C::RT3], rs[C::RT3];
#pragma unroll
  for (int r = 0; r < C::RT3; ++r) {
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < C::CT3; ++c) sum += (acc3[r][c][0] + acc3[r][c][1]) + (acc3[r][c][2] + acc3[r][c][3]);
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    mu[r] = sum;
  }
  if constexpr (C::CG > 1) {
#pragma unroll
    for (int r = 0; r < C::RT3; ++r)
      if (fg == 0) red[((rg * C::RT3 + r) * 16 + fr) * C::CG + cg] = mu[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < C::RT3; ++r) {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < C::CG; ++g) sum += red[((rg * C::RT3 + r) * 16 + fr) * C::CG + g];
      mu[r] = sum;
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < C::RT3; ++r) {
    mu[r] *= 1.0f / D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < C::CT3; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float dd = acc3[r][c][j] - mu[r]; q += dd * dd; }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    rs[r] = q;
  }
  if constexpr (C::CG > 1) {
#pragma unroll
    for (int r = 0; r < C::RT3; ++r)
      if (fg == 0) red[((rg * C::RT3 + r) * 16 + fr) * C::CG + cg] = rs[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < C::RT3; ++r) {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < C::CG; ++g) sum += red[((rg * C::RT3 + r) * 16 + fr) * C::CG + g];
      rs[r] = sum;
    }
  }
  float4 gp[C::CT3], bp[C::CT3];
#pragma unroll
  for (int c = 0; c < C::CT3; ++c) {
    gp[c] = *reinterpret_cast<const float4*>(g_post + (cg * C::CT3 + c) * 16 + fg * 4);
    bp[c] = *reinterpret_cast<const float4*>(b_post + (cg * C::CT3 + c) * 16 + fg * 4);
  }
#pragma unroll
  for (int r = 0; r < C::RT3; ++r) {
    const float inv = rsqrtf(rs[r] * (1.0f / D) + 1e-5f);
    const long row = t0 + (rg * C::RT3 + r) * 16 + fr;
    if (row >= T) continue;
#pragma unroll
    for (int c = 0; c < C::CT3; ++c) {
      const int col = (cg * C::CT3 + c) * 16 + fg * 4;
      float v0 = (acc3[r][c][0] - mu[r]) * inv * gp[c].x + bp[c].x;
      float v1 = (acc3[r][c][1] - mu[r]) * inv * gp[c].y + bp[c].y;
      float v2 = (acc3[r][c][2] - mu[r]) * inv * gp[c].z + bp[c].z;
      float v3 = (acc3[r][c][3] - mu[r]) * inv * gp[c].w + bp[c].w;
      if (res) {
        const uint2 q = *reinterpret_cast<const uint2*>(res + row * D + col);
        v0 += __uint_as_float(q.x << 16);
        v1 += __uint_as_float(q.x & 0xffff0000u);
        v2 += __uint_as_float(q.y << 16);
        v3 += __uint_as_float(q.y & 0xffff0000u);
      }
      *reinterpret_cast<uint2*>(out + row * D + col) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

template <int D, int HD, int NW>
int launch(const hv_mhc_fused_args* a, hipStream_t s) {
  using C = Cfg<D, HD, NW>;
  auto k = mhc_fused_kernel<D, HD, NW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  k<<<hv_cdiv(a->T, C::BM), C::NT, C::LDS, s>>>(
      (const unsigned short*)a->x, a->T, (const unsigned short*)a->a1t, a->c1, (const unsigned short*)a->w2,
      a->b2, (const unsigned short*)a->wct, a->g_post, a->b_post, (const unsigned short*)a->residual,
      (unsigned short*)a->out);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

int g_fused_wide = 0;

}  // namespace

extern "C" int hv_mhc_fused_supported(int D, int Hd, int dtype) {
  if (dtype != HV_BF16) return 0;
  // (256, 512) is instantiated but not dispatched by default: at D = 256 the per-tile weight
  // re-stream (1.9 MB per 64 tokens) makes it slower than the unfused GEMM chain.
  return (D == 32 && Hd == 128) || (D == 64 && Hd == 256) || (D == 128 && Hd == 512) ||
         (D == 256 && Hd == 512 && g_fused_wide);
}
extern "C" void hv_mhc_fused_enable_wide(int on) { g_fused_wide = on; }

extern "C" int hv_mhc_fused(const hv_mhc_fused_args* a, hv_stream_t stream) {
  if (!a || a->T <= 0) return HV_EINVAL;
  if (!hv_mhc_fused_supported(a->D, a->Hd, a->dtype)) return HV_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (a->D == 32) return launch<32, 128, 4>(a, s);
  if (a->D == 64) return launch<64, 256, 8>(a, s);
  if (a->D == 128) return launch<128, 512, 8>(a, s);
  return launch<256, 512, 8>(a, s);
}
