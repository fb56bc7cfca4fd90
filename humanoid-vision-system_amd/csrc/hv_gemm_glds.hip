// bf16 MFMA GEMM with direct-to-LDS staging (global_load_lds_dwordx4) for gfx950.
//
// Serves the plain, K-concatenated and implicit-im2col operands of hv_gemm when K is a
// multiple of 64 (every large contraction of the HybridVision path): each k-step stages
// 64 bf16 (128 B) of every A and B row straight into LDS with one 16-byte LDS-DMA per
// lane; the LDS image is XOR-swizzled (16-B chunk c of row r lives at chunk c ^ (r & 7)),
// the swizzle applied on the per-lane SOURCE address because the LDS destination of a
// global_load_lds is lane-linear.  Two LDS stages: the DMA of tile t+1 is in flight while
// the MFMAs of tile t run.  Out-of-image conv taps read a zero line; rows past M are
// clamped (computed, never stored).
#include "hv_common.h"
#include "hv_gemm_epi.h"

__device__ __attribute__((aligned(64))) uint4 hv_glds_zero_line[4];   // read by out-of-image taps

namespace {

constexpr int ROW = 128;                    // bytes per LDS row (64 bf16)

// 16-byte LDS-DMA: lane l's 16 bytes land at lds_base + 16*l (lds_base wave-uniform)
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#else
  (void)src; (void)lds_base;
#endif
}

template <int BM, int BN, bool CONV, bool TRAIN>
__global__ void __launch_bounds__(256) gemm_glds_kernel(const hv_gemm_desc d) {
  constexpr int STAGE_BYTES = (BM + BN) * ROW;
  constexpr int AI = BM / 32;               // A wave-instructions (8 rows each) per wave
  constexpr int BI = BN / 32;
  constexpr int RM = BM / 32, RN = BN / 32;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

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

  // ---- per-lane source rows: wave instruction i covers tile rows 8*(wid*AI+i) .. +7
  const int lrow = lane >> 3;               // row within the 8-row group
  const int pchunk = lane & 7;              // physical 16-B chunk this lane fills
  const unsigned short* arow[AI];
  int aih[AI], aiw[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wid * AI + i) * 8 + lrow;
    int row = m0 + r;
    row = row < d.M ? row : d.M - 1;
    if constexpr (CONV) {
      const int hw = d.conv_oh * d.conv_ow;
      const int b = row / hw, p = row % hw;
      const int oh = p / d.conv_ow, ow = p % d.conv_ow;
      aih[i] = oh * d.conv_stride - d.conv_pad;
      aiw[i] = ow * d.conv_stride - d.conv_pad;
      arow[i] = (const unsigned short*)d.A + (long)b * d.conv_h * d.conv_w * d.conv_c;
    } else {
      aih[i] = aiw[i] = 0;
      arow[i] = (const unsigned short*)d.A + (long)row * d.lda;
    }
  }
  const unsigned short* brow[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (wid * BI + i) * 8 + lrow;
    int n = n0 + r;
    n = n < d.N ? n : d.N - 1;
    brow[i] = (const unsigned short*)d.B + (long)n * d.ldb;
  }
  const int lchunk = pchunk ^ (lrow & 7);   // logical chunk fetched by this lane (rows 8-aligned)

  auto stage = [&](int buf, int kt) {
    unsigned char* sa = smem + buf * STAGE_BYTES;
    unsigned char* sb = sa + BM * ROW;
    const int k = kt * 64 + lchunk * 8;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const void* src;
      if constexpr (CONV) {
        const int tap = k / d.conv_c, ci = k - tap * d.conv_c;
        const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
        const int ih = aih[i] + kh, iw = aiw[i] + kw;
        src = ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
                  ? (const void*)(arow[i] + ((long)ih * d.conv_w + iw) * d.conv_c + ci)
                  : (const void*)hv_glds_zero_line;
      } else {
        if (d.A2 != nullptr && k >= d.k1) {
          const int row = min(m0 + (wid * AI + i) * 8 + lrow, d.M - 1);
          src = (const unsigned short*)d.A2 + (long)row * d.lda2 + (k - d.k1);
        } else {
          src = arow[i] + k;
        }
      }
      glds16(src, sa + (wid * AI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16(brow[i] + k, sb + (wid * BI + i) * 1024);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = d.K / 64;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    const unsigned char* sa = smem + buf * STAGE_BYTES;
    const unsigned char* sb = sa + BM * ROW;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lc = s * 4 + fg;
      uint4 fa[RM], fb[RN];
#pragma unroll
      for (int a = 0; a < RM; ++a) {
        const int r = wr * (BM / 2) + a * 16 + fr;
        fa[a] = *reinterpret_cast<const uint4*>(sa + r * ROW + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const int r = wc * (BN / 2) + b * 16 + fr;
        fb[b] = *reinterpret_cast<const uint4*>(sb + r * ROW + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[b]),
                                                              __builtin_bit_cast(bf16x8, fa[a]), acc[a][b], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue (shared with the register-staged kernel; acc holds transposed sub-tiles;
  //      LN_EPI: LayerNorm after the product)
  if (d.a_mean) gemm_epilogue<BM, BN, true, TRAIN>(d, acc, m0, n0);
  else gemm_epilogue<BM, BN, false, TRAIN>(d, acc, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 along M x 4 along N, 128x64 per wave, 32 accumulators), BK = 64,
// one 128-KiB LDS array with two K-tile buffers.  The LDS-DMA of tile k+1 is issued right after
// the barrier that opens tile k and stays in flight across the whole compute of tile k: raw
// s_barrier (no implicit vmcnt(0) drain) + an explicit vmcnt(0) only where tile k+1 is needed.
// MFMA clusters at raised wave priority.  (MI355X guide §5: the 128x128 two-barrier structure
// tops out near 900 TF; this is the ~1 block/CU pipelined structure.)
constexpr int B256_STAGE = 512 * ROW;       // (256 A + 256 B rows) x 128 B per K-tile buffer

template <bool CONV>
__global__ void __launch_bounds__(512) gemm_glds256_kernel(const hv_gemm_desc d) {
  constexpr int BM = 256, BN = 256, AI = 4, BI = 4;   // glds instructions per wave per tile (8 rows each)
  constexpr int RM = 8, RN = 4;                       // 16x16 sub-tiles per wave
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * B256_STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
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

  const int lrow = lane >> 3, pchunk = lane & 7;
  const unsigned short* arow[AI];
  int aih[AI], aiw[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    int row = m0 + (wid * AI + i) * 8 + lrow;
    row = row < d.M ? row : d.M - 1;
    if constexpr (CONV) {
      const int hw = d.conv_oh * d.conv_ow;
      const int b = row / hw, p = row % hw;
      const int oh = p / d.conv_ow, ow = p % d.conv_ow;
      aih[i] = oh * d.conv_stride - d.conv_pad;
      aiw[i] = ow * d.conv_stride - d.conv_pad;
      arow[i] = (const unsigned short*)d.A + (long)b * d.conv_h * d.conv_w * d.conv_c;
    } else {
      aih[i] = aiw[i] = 0;
      arow[i] = (const unsigned short*)d.A + (long)row * d.lda;
    }
  }
  const unsigned short* brow[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    int n = n0 + (wid * BI + i) * 8 + lrow;
    n = n < d.N ? n : d.N - 1;
    brow[i] = (const unsigned short*)d.B + (long)n * d.ldb;
  }
  const int lchunk = pchunk ^ (lrow & 7);

  auto stage = [&](int buf, int kt) {
    unsigned char* sa = smem + buf * B256_STAGE;
    unsigned char* sb = sa + BM * ROW;
    const int k = kt * 64 + lchunk * 8;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const void* src;
      if constexpr (CONV) {
        const int tap = k / d.conv_c, ci = k - tap * d.conv_c;
        const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
        const int ih = aih[i] + kh, iw = aiw[i] + kw;
        src = ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
                  ? (const void*)(arow[i] + ((long)ih * d.conv_w + iw) * d.conv_c + ci)
                  : (const void*)hv_glds_zero_line;
      } else {
        if (d.A2 != nullptr && k >= d.k1) {
          const int row = min(m0 + (wid * AI + i) * 8 + lrow, d.M - 1);
          src = (const unsigned short*)d.A2 + (long)row * d.lda2 + (k - d.k1);
        } else {
          src = arow[i] + k;
        }
      }
      glds16(src, sa + (wid * AI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16(brow[i] + k, sb + (wid * BI + i) * 1024);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = d.K / 64;
  const int fr = lane & 15, fg = lane >> 4;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's part of tile kt landed
    __builtin_amdgcn_s_barrier();                            // ... everyone's; buffer buf^1 is free
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);                 // in flight across this tile's compute
    const unsigned char* sa = smem + buf * B256_STAGE;
    const unsigned char* sb = sa + BM * ROW;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lc = s * 4 + fg;
      uint4 fb[RN];
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const int r = wc * 64 + b * 16 + fr;
        fb[b] = *reinterpret_cast<const uint4*>(sb + r * ROW + ((lc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {                          // two row halves of the wave's 128 rows
        uint4 fa[RM / 2];
#pragma unroll
        for (int a = 0; a < RM / 2; ++a) {
          const int r = wr * 128 + (h * 4 + a) * 16 + fr;
          fa[a] = *reinterpret_cast<const uint4*>(sa + r * ROW + ((lc ^ (r & 7)) << 4));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < RM / 2; ++a)
#pragma unroll
          for (int b = 0; b < RN; ++b)
            acc[h * 4 + a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, fb[b]), __builtin_bit_cast(bf16x8, fa[a]), acc[h * 4 + a][b], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  if (d.a_mean) gemm_epilogue<BM, BN, true, false, 4, RM, RN>(d, acc, m0, n0);
  else gemm_epilogue<BM, BN, false, false, 4, RM, RN>(d, acc, m0, n0);
}

int launch256(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, 256) * hv_cdiv(d.N, 256);
  if (d.conv_k > 0) gemm_glds256_kernel<true><<<grid, 512, 0, s>>>(d);
  else gemm_glds256_kernel<false><<<grid, 512, 0, s>>>(d);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

template <int BM, int BN>
int launch(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, BM) * hv_cdiv(d.N, BN);
  if (d.epi_mode) {
    if constexpr (BM * BN > 128 * 64) {
      return HV_EUNSUPPORTED;                   // never selected: the training epilogue uses 64x128
    } else {
      if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, true><<<grid, 256, 0, s>>>(d);
      else gemm_glds_kernel<BM, BN, false, true><<<grid, 256, 0, s>>>(d);
    }
  } else {
    if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, false><<<grid, 256, 0, s>>>(d);
    else gemm_glds_kernel<BM, BN, false, false><<<grid, 256, 0, s>>>(d);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

}  // namespace

int hv_gemm_big_tile_mode();   // hv_gemm.hip
int hv_gemm_small_tile_mode();  // hv_gemm.hip

// Returns HV_EUNSUPPORTED when the shape/mode is not covered (caller falls back).
int hv_gemm_glds(const hv_gemm_desc& d, hipStream_t s) {
  if (d.dtype != HV_BF16 || d.K % 64 || d.conv_transposed) return HV_EUNSUPPORTED;
  if (d.a_mean && (!d.b_colsum || d.A2 || d.conv_k > 0)) return HV_EUNSUPPORTED;
  if (d.conv_k > 0 ? (d.conv_c % 8) : (d.lda % 8)) return HV_EUNSUPPORTED;
  if (d.A2 && (d.k1 % 64 || d.lda2 % 8)) return HV_EUNSUPPORTED;
  if (d.ldb % 8) return HV_EUNSUPPORTED;
  const long t128 = (long)hv_cdiv(d.M, 128) * hv_cdiv(d.N, 128);
  const long t256 = (long)hv_cdiv(d.M, 256) * hv_cdiv(d.N, 256);
  if (!d.epi_mode && (hv_gemm_big_tile_mode() == 2 ||
                      (hv_gemm_big_tile_mode() == 1 && d.N >= 256 && t256 >= 192)))
    return launch256(d, s);
  if (d.N <= 64) return launch<128, 64>(d, s);
  // small grids (the ViT / head mHC GEMMs: M = 16 x 401 tokens): 64x64 tiles fill the 256 CUs
  const long t64x128 = (long)hv_cdiv(d.M, 64) * hv_cdiv(d.N, 128);
  if (hv_gemm_small_tile_mode() && t64x128 < 320) return launch<64, 64>(d, s);
  if (d.M <= 64 || t128 < 256 || d.epi_mode) return launch<64, 128>(d, s);   // 128x128 + training epilogue: acc demoted to scratch, 2x slower
  return launch<128, 128>(d, s);
}
