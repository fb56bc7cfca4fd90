// Persistent small-K bf16 GEMM for gfx950 (K <= 512): the LN-epilogue GEMM1s of the mHC sites
// (25600x2048x256, 102400x1024x256, 6416x3072x256, 6400x4096x512 ...) and the 1x1 convolutions.
//
// At K <= 512 a 128x128 tile is 1-8 MFMA k-steps, so the non-persistent ring kernel spends most of
// a tile's life in its prologue (first DMA round trip) and its epilogue (LDS staging + barriers),
// and its output stream -- the dominant byte count here (25600x2048 bf16 = 105 MB against 14 MB
// of operands) -- runs at 1.2-1.5 TB/s (tools/k256_probe2.py).  This kernel:
//
//  * is PERSISTENT: grid = 2 workgroups per CU, each walks tiles r*G + remap(bid) (XCD-aware per
//    round, so the 16 N-tiles of one A row block share an L2);
//  * keeps ONE continuous LDS-DMA k-stream across its tiles: the last k-step of tile t issues the
//    DMA of tile t+1's first k-tile, so that round trip overlaps tile t's MFMAs and epilogue;
//  * has a REGISTER epilogue with 16-byte stores and no LDS: the B tile's rows are loaded
//    N-PERMUTED (LDS row b*16 + 4g + j of a wave's half <- physical column 16g + 4b + j), so after
//    the transposed MFMAs lane (fr, g) holds 16 CONSECUTIVE output columns of one row across its
//    four 16x16 sub-tiles -> two 16-byte bf16 stores (64 contiguous bytes per 4 lanes), LDS free
//    for the next tile's DMA, no barrier in the epilogue.
//
// Same arithmetic as hv_gemm_epi.h (LN after the product, scale*alpha, bias, act, residual), same
// MFMA k-order as the ring kernel -> identical results.
#include <atomic>

#include "hv_common.h"

namespace {

constexpr int SK_ROW = 128;                         // bytes per LDS row (64 bf16 of K)
constexpr int SK_BM = 128, SK_BN = 128;
constexpr int SK_STAGE = (SK_BM + SK_BN) * SK_ROW;  // 32 KiB per k-tile buffer

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void sk_glds16(const void* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}
#pragma clang diagnostic pop

// physical column (within a wave's 64) of LDS B row q = b*16 + 4g + j
__device__ __forceinline__ int sk_perm(int q) { return ((q & 15) >> 2) * 16 + (q >> 4) * 4 + (q & 3); }

// tile of round `round` for this workgroup: XCD-aware inside full rounds (consecutive tiles on
// one XCD, as the ring kernel's remap), identity in the last partial round; -1 = done
__device__ __forceinline__ int sk_tile(int round, int ntiles) {
  const int G = gridDim.x, bid = blockIdx.x;
  const long base = (long)round * G;
  if (base + G <= ntiles) {
    const int xcd = bid & 7, q = G >> 3, r = G & 7;
    return (int)base + (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  return base + bid < ntiles ? (int)(base + bid) : -1;
}

// DIAG (variant HV_GV_SK_DIAG1 / 2, tools/k256_probe2.py only): 1 = skip the stores, 2 = skip the
// k-loop (DMA + MFMA) -- the two halves of a tile's time, measured apart.  0 in the product.
template <bool LN, int DIAG = 0>
__global__ void __launch_bounds__(256, 2) gemm_sk_kernel(const hv_gemm_desc d, int ntiles) {
  constexpr int AI = SK_BM / 32, BI = SK_BN / 32, RM = 4, RN = 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * SK_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7, lchunk = pchunk ^ (lrow & 7);
  const int tilesN = (d.N + SK_BN - 1) / SK_BN;
  const int nk = d.K / 64;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(wid);

  // per-lane DMA source rows of a tile: A rows m0 + r, B rows n0 + permuted(r)
  struct Src {
    const unsigned short* a[AI];
    const unsigned short* b[BI];
  };
  auto src_of = [&](int tile, Src& s) {
    const int m0 = (tile / tilesN) * SK_BM, n0 = (tile % tilesN) * SK_BN;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = min(m0 + (wid * AI + i) * 8 + lrow, d.M - 1);
      s.a[i] = (const unsigned short*)d.A + (long)row * d.lda;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int r = (wid * BI + i) * 8 + lrow;             // LDS B row 0..127
      const int n = min(n0 + (r >> 6) * 64 + sk_perm(r & 63), d.N - 1);
      s.b[i] = (const unsigned short*)d.B + (long)n * d.ldb;
    }
  };
  auto stage = [&](const Src& s, int buf, int kt) {
    const unsigned la = lds0 + buf * SK_STAGE + wu * AI * 1024;
    const unsigned lb = lds0 + buf * SK_STAGE + SK_BM * SK_ROW + wu * BI * 1024;
    const int k = kt * 64 + lchunk * 8;
#pragma unroll
    for (int i = 0; i < AI; ++i) sk_glds16(s.a[i] + k, la + i * 1024);
#pragma unroll
    for (int i = 0; i < BI; ++i) sk_glds16(s.b[i] + k, lb + i * 1024);
  };

  int tile = sk_tile(0, ntiles);
  if (tile < 0) return;                                    // workgroup-uniform
  Src cur, nxt;
  src_of(tile, cur);
  stage(cur, 0, 0);
  int buf = 0;
  const bool c_bf = d.c_dtype == HV_BF16, r_bf = d.r_dtype == HV_BF16;
  const bool gelu_fast = c_bf && !d.residual;
  const bool vec = (((uintptr_t)d.C) & 15) == 0 && d.ldc % 8 == 0 &&
                   (!d.residual || ((((uintptr_t)d.residual) & 15) == 0 && d.ldr % 8 == 0));

  bool prev_full = false;       // the previous tile's epilogue issued exactly its full-tile stores
  bool early1 = false;          // ... and, before them, this tile's k-tile 1 DMA
  for (int round = 0;; ++round) {
    const int next = sk_tile(round + 1, ntiles);
    if (next >= 0) src_of(next, nxt);
    const int m0 = (tile / tilesN) * SK_BM, n0 = (tile % tilesN) * SK_BN;
    // this wave stores whole 16-byte vectors for every row of its 64x64 sub-tile: exactly
    // 2 (bf16) or 4 (fp32) stores per 16-row block, no scalar tail
    const bool full = vec && m0 + wr * 64 + 64 <= d.M && n0 + wc * 64 + 64 <= d.N;
    f32x4 acc[RM][RN];
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
      for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMAs of k-tile kt (and the previous tile's epilogue stores) done; every
      // wave's reads of the other buffer retired -> it may be refilled
      // (at kt = 0 the previous epilogue's >= 8 stores are younger than this k-tile's DMAs: a
      // counted wait leaves them in flight instead of stalling on their write acknowledgements)
      // Waits: the previous tile's epilogue issued this tile's k-tile 1 (when early1) and then its
      // stores, both younger than k-tile 0's DMA; k-tile 1's DMA is older than those stores only.
      // So the stores' write acknowledgements are waited for at k-step 2 at the earliest.
      if (kt == 0 && early1) {
        if (prev_full) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else if (kt == 0 && prev_full) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else if (kt == 1 && early1 && prev_full) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt == 0 && early1) {
        // k-tile 1 already in flight (issued in the previous epilogue)
      } else if (kt + 1 < nk) {
        stage(cur, buf ^ 1, kt + 1);
      } else if (next >= 0) {
        stage(nxt, buf ^ 1, 0);                            // next tile's first k-tile
      }
      const unsigned char* sa = smem + buf * SK_STAGE;
      const unsigned char* sb = sa + SK_BM * SK_ROW;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int lc = s * 4 + fg;
        uint4 fa[RM], fb[RN];
#pragma unroll
        for (int a = 0; a < RM; ++a) {
          const int r = wr * (SK_BM / 2) + a * 16 + fr;
          fa[a] = *reinterpret_cast<const uint4*>(sa + r * SK_ROW + ((lc ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int b = 0; b < RN; ++b) {
          const int r = wc * (SK_BN / 2) + b * 16 + fr;
          fb[b] = *reinterpret_cast<const uint4*>(sb + r * SK_ROW + ((lc ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int a = 0; a < RM; ++a)
#pragma unroll
          for (int b = 0; b < RN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[b]),
                                                                __builtin_bit_cast(bf16x8, fa[a]), acc[a][b], 0, 0, 0);
      }
      buf ^= 1;
    }

    // epilogue constants, loaded after the k-loop (held across it they spill at 2 workgroups per
    // CU); vmcnt retires in order, so their wait also covers the next tile's first DMA -- which the
    // next k-step waits for anyway
    const int col0 = n0 + wc * 64 + fg * 16;
    float sc[16], bi[16], cs[16], mean[RM], rstd[RM];
    // one batch of independent loads (clamped columns, uniform null branches; see epi_load_cols)
    {
      int cc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) cc[j] = min(col0 + j, d.N - 1);
      if (d.scale) {
#pragma unroll
        for (int j = 0; j < 16; ++j) sc[j] = d.scale[cc[j]];
      }
      if (d.bias) {
#pragma unroll
        for (int j = 0; j < 16; ++j) bi[j] = d.bias[cc[j]];
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) cs[j] = LN ? d.b_colsum[cc[j]] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const bool ok = col0 + j < d.N;
        sc[j] = (d.scale && ok) ? sc[j] * d.alpha : d.alpha;
        bi[j] = (d.bias && ok) ? bi[j] : 0.f;
        cs[j] = ok ? cs[j] : 0.f;
      }
    }
#pragma unroll
    for (int a = 0; a < RM; ++a) {
      const int row = min(m0 + wr * 64 + a * 16 + fr, d.M - 1);
      mean[a] = 0.f;
      rstd[a] = 1.f;
      if constexpr (LN) {
        mean[a] = d.a_mean[row];
        rstd[a] = d.a_rstd[row];
      }
    }
    // the next tile's k-tile 1 goes out BEFORE this epilogue's stores (into the buffer of this
    // tile's last k-step, free once every wave is past it): vmcnt retires in issue order, so with
    // the stores issued first the next tile's k-step 1 wait covered their write acknowledgements
    // (one exposed store round trip per tile; the output stream ran at ~2 TB/s, tools/sk_probe.py)
    const bool fast = full && c_bf && !d.residual && DIAG == 0;
    // the early DMA path holds a workgroup barrier, so its condition must be WORKGROUP-uniform:
    // `full` is per wave (an edge column tile with N % 128 in 64..127 has full wc=0 waves and
    // partial wc=1 waves), the whole 128x128 tile being in range is not -- and implies `full`
    // (hence `fast`) for all four waves
    const bool tile_full = vec && m0 + SK_BM <= d.M && n0 + SK_BN <= d.N;
    const bool early_next = fast && tile_full && next >= 0 && nk >= 2;
    // ---- register epilogue: lane (fr, fg) owns columns col0 .. col0+15 of rows m0 + wr*64 + a*16 + fr
    if (fast) {
      // full bf16 tile, no residual: every value first (acc dies as it goes), then the next tile's
      // k-tile 1 DMA, then the 8 whole-row stores
      uint4 sv[2 * RM];
      const bool lo = fr < 8;
#pragma unroll
      for (int a = 0; a < RM; ++a) {
        float v[16];
#pragma unroll
        for (int b = 0; b < RN; ++b)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = b * 4 + j;
            float x = acc[a][b][j];
            if constexpr (LN) x = rstd[a] * (x - mean[a] * cs[c]);
            x = x * sc[c] + bi[c];
            v[c] = gelu_fast && d.act == HV_ACT_GELU ? hv_gelu_fast(x) : hv_act(x, d.act);
          }
        uint32_t p[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) p[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
        uint32_t rv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          rv[e] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(lo ? p[4 + e] : p[e]), 0x128, 0xF, 0xF, false);
        sv[2 * a] = lo ? make_uint4(p[0], p[1], p[2], p[3]) : make_uint4(rv[0], rv[1], rv[2], rv[3]);
        sv[2 * a + 1] = lo ? make_uint4(rv[0], rv[1], rv[2], rv[3]) : make_uint4(p[4], p[5], p[6], p[7]);
      }
      if (early_next) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                      // every wave past the last k-step's reads
        stage(nxt, buf ^ 1, 1);
      }
      unsigned short* cb = (unsigned short*)d.C;
#pragma unroll
      for (int a = 0; a < RM; ++a) {
        const int row = m0 + wr * 64 + a * 16 + fr;
        const int r1 = lo ? row : row - 8, r2 = lo ? row + 8 : row;
        const int cc = col0 + (lo ? 0 : 8);
        *reinterpret_cast<uint4*>(cb + (long)r1 * d.ldc + cc) = sv[2 * a];
        *reinterpret_cast<uint4*>(cb + (long)r2 * d.ldc + cc) = sv[2 * a + 1];
      }
    }
#pragma unroll
    for (int a = 0; a < RM; ++a) {
      if (DIAG == 1 || fast) continue;
      const int row = m0 + wr * 64 + a * 16 + fr;           // this lane's row (may be >= M: no store)
      const int rowc = min(row, d.M - 1);
      float v[16];
#pragma unroll
      for (int b = 0; b < RN; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = b * 4 + j;
          float x = acc[a][b][j];
          if constexpr (LN) x = rstd[a] * (x - mean[a] * cs[c]);
          x = x * sc[c] + bi[c];
          v[c] = (gelu_fast && d.act == HV_ACT_GELU) ? hv_gelu_fast(x) : hv_act(x, d.act);
        }
      const long rrow = d.r_mod > 0 ? rowc % d.r_mod : rowc;
      if (vec && col0 + 16 <= d.N) {                        // same for the lane pair (fr, fr ^ 8)
        if (d.residual) {
          if (r_bf) {
            const unsigned short* rp = (const unsigned short*)d.residual + rrow * d.ldr + col0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint4 r4 = *reinterpret_cast<const uint4*>(rp + h * 8);
              const uint32_t w4[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v[h * 8 + 2 * e] += __uint_as_float(w4[e] << 16);
                v[h * 8 + 2 * e + 1] += __uint_as_float(w4[e] & 0xffff0000u);
              }
            }
          } else {
            const float* rp = (const float*)d.residual + rrow * d.ldr + col0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float4 r4 = *reinterpret_cast<const float4*>(rp + q * 4);
              v[q * 4] += r4.x; v[q * 4 + 1] += r4.y; v[q * 4 + 2] += r4.z; v[q * 4 + 3] += r4.w;
            }
          }
        }
        if (c_bf) {
          // whole 128-byte rows per store instruction: lanes fr and fr ^ 8 (DPP row_ror:8) swap one
          // 16-byte half, so instruction 1 writes rows 0..7 of the block, instruction 2 rows 8..15,
          // each row's 64 columns by 8 lanes (a lane's 16 columns alone make 64-byte pieces, which
          // measured 1.6 TB/s against 6.2 for whole lines)
          uint32_t p[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) p[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
          const bool lo = fr < 8;
          uint32_t rv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rv[e] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(lo ? p[4 + e] : p[e]), 0x128, 0xF, 0xF, false);
          const uint4 s1 = lo ? make_uint4(p[0], p[1], p[2], p[3]) : make_uint4(rv[0], rv[1], rv[2], rv[3]);
          const uint4 s2 = lo ? make_uint4(rv[0], rv[1], rv[2], rv[3]) : make_uint4(p[4], p[5], p[6], p[7]);
          const int r1 = lo ? row : row - 8, r2 = lo ? row + 8 : row;
          const int cc = col0 + (lo ? 0 : 8);
          unsigned short* cb = (unsigned short*)d.C;
          if (r1 < d.M) *reinterpret_cast<uint4*>(cb + (long)r1 * d.ldc + cc) = s1;
          if (r2 < d.M) *reinterpret_cast<uint4*>(cb + (long)r2 * d.ldc + cc) = s2;
        } else if (row < d.M) {
          float* cp = (float*)d.C + (long)row * d.ldc + col0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(cp + q * 4) = make_float4(v[q * 4], v[q * 4 + 1], v[q * 4 + 2], v[q * 4 + 3]);
        }
      } else if (row < d.M) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int col = col0 + c;
          if (col >= d.N) break;
          float x = v[c];
          if (d.residual)
            x += r_bf ? bf2f(((const unsigned short*)d.residual)[rrow * d.ldr + col])
                      : ((const float*)d.residual)[rrow * d.ldr + col];
          const long o = (long)row * d.ldc + col;
          if (c_bf) ((unsigned short*)d.C)[o] = f2bf(x);
          else ((float*)d.C)[o] = x;
        }
      }
    }
    if (next < 0) break;
    prev_full = full;
    early1 = early_next;
    tile = next;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------------------------
// B-RESIDENT, column-stationary variant for K = 64 * NK (NK = 3, 4: the K = 256 GEMM1s of the
// mHC sites), one 4-wave workgroup per CU.  The kernel above waits vmcnt(0) at every k-step (one
// k-tile in flight: at K = 256 each tile pays ~4 DMA round trips) and its per-tile epilogue
// constants are compiler-tracked global loads, whose waits would drain any deeper prefetch.  Here:
//  * every workgroup owns ONE 128-column block for its whole life (XCD-aware: the column blocks
//    of a row block are consecutive workgroups, so an A row panel is fetched into one L2): the
//    B panel (128 x K, N-permuted as above) is DMA'd to LDS once, and the column constants
//    (scale, bias, LN column sums) are loaded once, before any DMA is in flight;
//  * only A streams, through an NS-stage ring with NS-1 k-tiles in flight across tile
//    boundaries; every wait is an explicit counted vmcnt (the in-flight groups, plus the previous
//    tile's 8 stores while they are younger than the awaited group);
//  * the LN row statistics of a tile ride its first A k-tile's DMA group into an LDS slot
//    (double-buffered by tile parity), so the epilogue reads them with ds_reads.
// Same per-element k order and epilogue arithmetic as gemm_sk_kernel: bitwise-equal outputs.
template <bool LN, int NK, int NS>
__global__ void __launch_bounds__(256, 1) gemm_skr_kernel(const hv_gemm_desc d, int tilesM, int tilesN, int slots) {
  static_assert(NK >= NS - 1 && NK <= 4, "prefetch stays within one tile boundary; B panel <= 64 KiB");
  constexpr int AI = SK_BM / 32, BI = SK_BN / 32, RM = 4, RN = 4;
  constexpr int KT = SK_BM * SK_ROW;                     // 16 KiB: one 128-row x 64-k image
  constexpr int BPANEL = NK * KT, RING = BPANEL, RCS = RING + NS * KT;
  constexpr int GA = AI + (LN ? 1 : 0);                  // DMA instructions per wave per A group (+ row stats)
  __shared__ __attribute__((aligned(16))) unsigned char smem[RCS + (LN ? 2 * 4096 : 16)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = lane >> 3, pchunk = lane & 7, lchunk = pchunk ^ (lrow & 7);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  int L;
  {
    const int G = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q = G >> 3, r = G & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int cb = L % tilesN, s0 = L / tilesN;
  if (s0 >= slots || s0 >= tilesM) return;               // workgroup-uniform
  const int n0 = cb * SK_BN;
  const int ntl = (tilesM - s0 + slots - 1) / slots;     // tiles of this workgroup: s0, s0 + slots, ...

  // ---- column constants, waited for before the first DMA
  const int col0 = n0 + wc * 64 + fg * 16;
  float sc[16], bi[16], cs[16];
  {
    // unconditional loads from clamped columns (a null pointer reads a dummy operand), selected
    // afterwards: one batch of independent loads, not a branch + wait per element
    const float* psc = d.scale ? d.scale : (const float*)d.B;
    const float* pbi = d.bias ? d.bias : (const float*)d.B;
    const float* pcs = LN ? d.b_colsum : (const float*)d.B;
    float keep = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int colc = min(col0 + j, d.N - 1);
      sc[j] = psc[colc];
      bi[j] = pbi[colc];
      cs[j] = pcs[colc];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const bool ok = col0 + j < d.N;
      sc[j] = (d.scale && ok) ? sc[j] * d.alpha : d.alpha;
      bi[j] = (d.bias && ok) ? bi[j] : 0.f;
      cs[j] = (LN && ok) ? cs[j] : 0.f;
      keep += sc[j] + bi[j] + cs[j];
    }
    asm volatile("" ::"v"(keep));                         // the loads complete here, nothing else pending
  }
  // ---- B panel -> LDS (k-tile kt at kt * KT; rows N-permuted like gemm_sk_kernel)
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (wid * BI + i) * 8 + lrow;
    const int n = min(n0 + (r >> 6) * 64 + sk_perm(r & 63), d.N - 1);
    const unsigned short* bp = (const unsigned short*)d.B + (long)n * d.ldb + lchunk * 8;
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) sk_glds16(bp + kt * 64, lds0 + kt * KT + wu * BI * 1024 + i * 1024);
  }
  // ---- A stream: the DMA cursor (dt-th tile of this workgroup, k-tile dk) runs NS-1 groups ahead
  int dt = 0, dk = 0, g_issued = 0;
  auto issue = [&]() {
    const int tm = s0 + dt * slots;
    const unsigned la = lds0 + RING + (g_issued % NS) * KT + wu * AI * 1024;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = min(tm * SK_BM + (wid * AI + i) * 8 + lrow, d.M - 1);
      sk_glds16((const unsigned short*)d.A + (long)row * d.lda + dk * 64 + lchunk * 8, la + i * 1024);
    }
    if constexpr (LN) {
      // row statistics of tile dt (first group only; later groups reload them -- same bytes, so
      // the group size stays fixed): wave w -> {mean, rstd}[w >> 1] rows (w & 1) * 64 .. +63
      const float* src = (wu >> 1) ? d.a_rstd : d.a_mean;
      const int r0 = min(tm * SK_BM + (wu & 1) * 64 + (lane & 15) * 4, d.M - 4 < 0 ? 0 : d.M - 4);
      sk_glds16(src + r0, lds0 + RCS + (dt & 1) * 4096 + wu * 1024);
    }
    ++g_issued;
    if (++dk == NK) { dk = 0; ++dt; }
  };
  const int total = ntl * NK;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < total) issue();

  const bool c_bf = d.c_dtype == HV_BF16;
  const bool gelu_fast = c_bf;
  const bool vec = (((uintptr_t)d.C) & 15) == 0 && d.ldc % 8 == 0;
  bool prev_full = false;
  for (int t = 0; t < ntl; ++t) {
    const int tm = s0 + t * slots;
    const int m0 = tm * SK_BM;
    const bool last = t == ntl - 1;
    f32x4 acc[RM][RN];
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
      for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      // wait for this wave's A group of step (t, kt): the younger groups (NS-2 of them, the ones
      // carrying a tile's row statistics one instruction longer) and, while the previous tile's
      // 8 stores are younger still (kt <= NS-2), those stay in flight; the last tile waits for all
      constexpr int base = [] {
        int n = 0;
        for (int dd = 1; dd <= NS - 2; ++dd) n += AI + (LN ? 1 : 0);
        return n;
      }();
      (void)base;
      if (last) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        // every group has GA instructions (LN groups always carry the row-statistics DMA)
        constexpr int young = (NS - 2) * GA;
        if (prev_full && kt <= NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(young + 8) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(young) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (g_issued < total) issue();
      const int g = t * NK + kt;
      const unsigned char* sa = smem + RING + (g % NS) * KT;
      const unsigned char* sb = smem + kt * KT;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int lc = s * 4 + fg;
        uint4 fa[RM], fb[RN];
#pragma unroll
        for (int a = 0; a < RM; ++a) {
          const int r = wr * (SK_BM / 2) + a * 16 + fr;
          fa[a] = *reinterpret_cast<const uint4*>(sa + r * SK_ROW + ((lc ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int b = 0; b < RN; ++b) {
          const int r = wc * (SK_BN / 2) + b * 16 + fr;
          fb[b] = *reinterpret_cast<const uint4*>(sb + r * SK_ROW + ((lc ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int a = 0; a < RM; ++a)
#pragma unroll
          for (int b = 0; b < RN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[b]),
                                                                __builtin_bit_cast(bf16x8, fa[a]), acc[a][b], 0, 0, 0);
      }
    }
    // ---- register epilogue (gemm_sk_kernel's, without residual): 16 consecutive columns per lane
    const bool full = vec && m0 + wr * 64 + 64 <= d.M && n0 + wc * 64 + 64 <= d.N;
    const float* rc = reinterpret_cast<const float*>(smem + RCS + (t & 1) * 4096);
#pragma unroll
    for (int a = 0; a < RM; ++a) {
      const int row = m0 + wr * 64 + a * 16 + fr;
      float mean = 0.f, rstd = 1.f;
      if constexpr (LN) {
        const int lr = wr * 64 + a * 16 + fr;              // slot of wave (lr >> 6) (+2 for rstd)
        mean = rc[(lr >> 6) * 256 + (lr & 63)];
        rstd = rc[(2 + (lr >> 6)) * 256 + (lr & 63)];
      }
      float v[16];
#pragma unroll
      for (int b = 0; b < RN; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = b * 4 + j;
          float x = acc[a][b][j];
          if constexpr (LN) x = rstd * (x - mean * cs[c]);
          x = x * sc[c] + bi[c];
          v[c] = (gelu_fast && d.act == HV_ACT_GELU) ? hv_gelu_fast(x) : hv_act(x, d.act);
        }
      if (vec && col0 + 16 <= d.N) {
        if (c_bf) {
          uint32_t pk[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
          const bool lo = fr < 8;
          uint32_t rv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rv[e] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(lo ? pk[4 + e] : pk[e]), 0x128, 0xF, 0xF, false);
          const uint4 s1 = lo ? make_uint4(pk[0], pk[1], pk[2], pk[3]) : make_uint4(rv[0], rv[1], rv[2], rv[3]);
          const uint4 s2 = lo ? make_uint4(rv[0], rv[1], rv[2], rv[3]) : make_uint4(pk[4], pk[5], pk[6], pk[7]);
          const int r1 = lo ? row : row - 8, r2 = lo ? row + 8 : row;
          const int cc = col0 + (lo ? 0 : 8);
          unsigned short* cbp = (unsigned short*)d.C;
          if (r1 < d.M) *reinterpret_cast<uint4*>(cbp + (long)r1 * d.ldc + cc) = s1;
          if (r2 < d.M) *reinterpret_cast<uint4*>(cbp + (long)r2 * d.ldc + cc) = s2;
        } else if (row < d.M) {
          float* cp = (float*)d.C + (long)row * d.ldc + col0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(cp + q * 4) = make_float4(v[q * 4], v[q * 4 + 1], v[q * 4 + 2], v[q * 4 + 3]);
        }
      } else if (row < d.M) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int col = col0 + c;
          if (col >= d.N) break;
          const long o = (long)row * d.ldc + col;
          if (c_bf) ((unsigned short*)d.C)[o] = f2bf(v[c]);
          else ((float*)d.C)[o] = v[c];
        }
      }
    }
    // exactly 8 full-tile stores per wave only for bf16 full tiles (fp32 stores 16)
    prev_full = full && c_bf;
  }
}

std::atomic<int> g_cus{0};

}  // namespace

// Returns HV_EUNSUPPORTED when the shape/mode is not this kernel's (the caller falls back).
// force (variant tile code 6, tests): any supported shape, even below one round of tiles.
int hv_gemm_smallk(const hv_gemm_desc& d0, hipStream_t s, bool force) {
  if (!force && (d0.variant & HV_GV_NO_SMALLK)) return HV_EUNSUPPORTED;
  hv_gemm_desc d = d0;
  // a 1x1 stride-1 unpadded convolution is the plain GEMM over the NHWC pixel rows
  if (d.conv_k == 1 && d.conv_stride == 1 && d.conv_pad == 0 && !d.conv_transposed) {
    d.conv_k = 0;
    d.lda = d.conv_c;
  }
  if (d.dtype != HV_BF16 || d.conv_k > 0 || d.conv_transposed || d.A2 || d.epi_mode) return HV_EUNSUPPORTED;
  if (d.K % 64 || d.K > 512 || d.lda % 8 || d.ldb % 8) return HV_EUNSUPPORTED;
  if (d.a_mean && !d.b_colsum) return HV_EUNSUPPORTED;
  if (!force && d.N < 256) return HV_EUNSUPPORTED;        // narrow outputs: the ring kernel's tiles fill better
  const long ntiles = (long)hv_cdiv(d.M, SK_BM) * hv_cdiv(d.N, SK_BN);
  int cus = g_cus.load(std::memory_order_relaxed);
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || cus <= 0)
      cus = 256;
    g_cus = cus;
  }
  if (!force && ntiles < 2L * cus) return HV_EUNSUPPORTED;   // under one persistent round: nothing to overlap
  hv_diag_count(HV_KF_GEMM_SMALLK);
  if ((d.variant & (HV_GV_SK_RES3 | HV_GV_SK_RES4)) && !d.residual && (d.K == 192 || d.K == 256) &&
      !(d.variant & (HV_GV_SK_DIAG1 | HV_GV_SK_DIAG2)) && (!d.a_mean || (d.M >= 4 && d.M % 4 == 0))) {
    // (the LN row statistics ride the A DMA as 16-byte groups of 4 rows: with M % 4 != 0 the
    // clamped last group would shift rows, so those shapes take the streaming kernel)
    // B-resident column-stationary kernel: one workgroup per CU, each on one column block
    const int tilesM = hv_cdiv(d.M, SK_BM), tilesN = hv_cdiv(d.N, SK_BN);
    const int slots = tilesN > cus ? 1 : cus / tilesN;
    const int grid = slots * tilesN;
    const bool r4 = d.variant & HV_GV_SK_RES4;
#define HV_SKR(LN_, NK_)                                                                               \
  (r4 ? gemm_skr_kernel<LN_, NK_, 4><<<grid, 256, 0, s>>>(d, tilesM, tilesN, slots)                     \
      : gemm_skr_kernel<LN_, NK_, 3><<<grid, 256, 0, s>>>(d, tilesM, tilesN, slots))
    if (d.K == 256) { if (d.a_mean) HV_SKR(true, 4); else HV_SKR(false, 4); }
    else { if (d.a_mean) HV_SKR(true, 3); else HV_SKR(false, 3); }
#undef HV_SKR
    HV_CHECK_LAUNCH();
    return HV_OK;
  }
  const int grid = (int)(ntiles < 2L * cus ? ntiles : 2L * cus);
  if (d.variant & HV_GV_SK_DIAG1) gemm_sk_kernel<false, 1><<<grid, 256, 0, s>>>(d, (int)ntiles);
  else if (d.variant & HV_GV_SK_DIAG2) gemm_sk_kernel<false, 2><<<grid, 256, 0, s>>>(d, (int)ntiles);
  else if (d.a_mean) gemm_sk_kernel<true><<<grid, 256, 0, s>>>(d, (int)ntiles);
  else gemm_sk_kernel<false><<<grid, 256, 0, s>>>(d, (int)ntiles);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
