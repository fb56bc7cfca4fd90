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
//
// This header holds the kernel templates; the instantiations are spread over several
// translation units (hv_gemm_glds_*.hip, one per tile shape and epilogue family) so the build
// compiles them in parallel -- one TU with all 62 instantiations took 12.6 min.
#pragma once
#include <atomic>

#include "hv_common.h"
#include "hv_gemm_epi.h"
#include <type_traits>

// read by out-of-image taps; one copy per translation unit (each TU is its own code object)
static __device__ __attribute__((aligned(64))) uint4 hv_glds_zero_line[4];

// A/B knob (hv_gemm_desc.variant): dense GEMMs with K % 64 != 0 back on the register-staged
// kernel (the round-4 routing)
#define HV_GV_NO_DENSE_KTAIL 0x200000

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

// The same 16-byte LDS-DMA as inline asm (M0 = wave-uniform LDS byte address).  The compiler
// does not track it, so it does not drain vmcnt before every ds_read that follows the issue
// (it cannot tell the other buffer's DMA from this buffer's reads); the kernel that uses it
// waits for its DMAs itself with explicit vmcnt.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16_asm(const void* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}
#pragma clang diagnostic pop

// Implicit-im2col K position of a 64-wide K-tile when conv_c % 64 == 0 (every conv this path
// serves but the K-tail ones): the tile lies inside ONE tap, so its source offset
// ((kh * W + kw) * C + ci) is wave-uniform.  Advanced by one K-tile per call instead of
// recomputed with per-lane integer divisions (the old address path cost ~130 VALU per K-tile
// per wave against 32 MFMAs, rocprofv3 + ISA, profiles/r03).
struct ConvK {
  int kh, kw, ci;
  __device__ void init(const hv_gemm_desc& d, int kt) {
    const int k = kt * 64, tap = k / d.conv_c;
    ci = k - tap * d.conv_c;
    kh = tap / d.conv_k;
    kw = tap - kh * d.conv_k;
  }
  __device__ void advance(const hv_gemm_desc& d) {
    ci += 64;
    if (ci == d.conv_c) {
      ci = 0;
      if (++kw == d.conv_k) { kw = 0; ++kh; }
    }
  }
  __device__ int offset(const hv_gemm_desc& d) const { return (kh * d.conv_w + kw) * d.conv_c + ci; }
};

// Workgroups per CU the LDS ring admits (at most 4), declared as every instantiation's minimum
// occupancy: the epilogues would otherwise grow past the register budget of that occupancy
// (64x128 at 3 per CU needs <= 168 VGPRs; unbounded the compiler took 172)
template <int TM, int TN, int TS, bool TT>
struct GldsOcc {
  static constexpr int lds_w = (160 * 1024) / (TS * (TM + TN) * 128);
  static constexpr int value = lds_w < 1 ? 1 : (lds_w > 4 ? 4 : lds_w);
};

// Wait until at most `ahead` younger K-tiles (DPT DMA instructions each) are still in flight
// (vmcnt takes an immediate: one branch per possible count)
template <int DPT, int MAXA>
__device__ __forceinline__ void ring_wait(int ahead) {
  if constexpr (MAXA > 0) {
    if (ahead >= MAXA) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXA * DPT) : "memory");
      return;
    }
    ring_wait<DPT, MAXA - 1>(ahead);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int BM, int BN, bool CONV, bool TRAIN, bool STAGED = false, int NS = 2, bool SPLIT = false>
__global__ void __launch_bounds__(256, (GldsOcc<BM, BN, NS, TRAIN>::value)) gemm_glds_kernel(const hv_gemm_desc d) {
  static_assert(NS >= 2 && NS <= 8, "stages");
  constexpr int STAGE_BYTES = (BM + BN) * ROW;
  constexpr int AI = BM / 32;               // A wave-instructions (8 rows each) per wave
  constexpr int BI = BN / 32;
  constexpr int RM = BM / 32, RN = BN / 32;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE_BYTES];

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
  HV_DCHECK(tm < tilesM && (CONV || d.K % 64 == 0 || (d.A2 == nullptr && d.K % 8 == 0)) && (d.A2 == nullptr || d.k1 % 64 == 0));

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
  // conv fast path (conv_c % 64 == 0): per-lane element offset of the output pixel's (kh, kw) =
  // (0, 0) input position; a K-tile adds the wave-uniform ConvK offset
  const bool cfast = CONV && d.conv_c % 64 == 0;
  int apix[AI];                              // (< 2^31 elements per image on every path)
  ConvK ck;
  if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < AI; ++i)
      apix[i] = (aih[i] * d.conv_w + aiw[i]) * d.conv_c + lchunk * 8;
  }

  // DMA of K-tile kt into ring buffer buf (inline asm: the compiler does not track it, so it does
  // not drain vmcnt before the ds_reads of the other buffers; the loop waits with counted vmcnt).
  // Called for consecutive kt (the conv fast path advances ck once per call).
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  auto stage = [&](int buf, int kt) {
    const unsigned la = lds0 + buf * STAGE_BYTES + wu * AI * 1024;
    const unsigned lb = lds0 + buf * STAGE_BYTES + BM * ROW + wu * BI * 1024;
    const int k = kt * 64 + lchunk * 8;
    if (CONV && cfast) {
      const int koff = ck.offset(d);
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int ih = aih[i] + ck.kh, iw = aiw[i] + ck.kw;
        const void* src = ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
                              ? (const void*)(arow[i] + apix[i] + koff) : (const void*)hv_glds_zero_line;
        glds16_asm(src, la + i * 1024);
      }
#pragma unroll
      for (int i = 0; i < BI; ++i) glds16_asm(brow[i] + k, lb + i * 1024);
      ck.advance(d);
      return;
    }
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const void* src;
      if constexpr (CONV) {
        const int tap = k / d.conv_c, ci = k - tap * d.conv_c;
        const int kh = tap / d.conv_k, kw = tap - kh * d.conv_k;
        const int ih = aih[i] + kh, iw = aiw[i] + kw;
        src = (k < d.K && (unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
                  ? (const void*)(arow[i] + ((long)ih * d.conv_w + iw) * d.conv_c + ci)
                  : (const void*)hv_glds_zero_line;
      } else {
        if (d.A2 != nullptr && k >= d.k1) {
          const int row = min(m0 + (wid * AI + i) * 8 + lrow, d.M - 1);
          src = (const unsigned short*)d.A2 + (long)row * d.lda2 + (k - d.k1);
        } else {
          // dense K % 64 != 0 (K % 8 == 0, no A2): the last K-tile's tail reads the zero line
          src = k < d.K ? (const void*)(arow[i] + k) : (const void*)hv_glds_zero_line;
        }
      }
      glds16_asm(src, la + i * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const void* src = brow[i] + k;
      src = k < d.K ? src : (const void*)hv_glds_zero_line;   // K tail (padded conv, or dense K % 64 != 0)
      glds16_asm(src, lb + i * 1024);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (d.K + 63) / 64;         // conv: K % 64 != 0 allowed, the tail reads zeros
  // split-K: this workgroup's slice [kb, kb + nk) of the K-tiles (blockIdx.y = slice)
  const int kb = SPLIT ? (int)(((long)nkt * blockIdx.y) / d.splitk) : 0;
  const int nk = SPLIT ? (int)(((long)nkt * (blockIdx.y + 1)) / d.splitk) - kb : nkt;
  constexpr int DPT = AI + BI;              // DMA instructions per wave per K-tile
  // ring of NS buffers, NS-1 K-tiles in flight.  Iteration kt: wait for this wave's DMAs of tile
  // kt (the younger tiles stay in flight), barrier (every wave's tile kt landed, every wave's
  // reads of tile kt-1 retired), refill the buffer of tile kt-1 with tile kt+NS-1, compute kt.
  if constexpr (CONV) {
    if (cfast) ck.init(d, kb);
  }
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) stage(t, kb + t);

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    ring_wait<DPT, NS - 2>(min(NS - 2, nk - 1 - kt));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) stage((kt + NS - 1) % NS, kb + kt + NS - 1);
    const unsigned char* sa = smem + (kt % NS) * STAGE_BYTES;
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
  }
  // every wave's last reads retired before the (staged) epilogue reuses the LDS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  if constexpr (SPLIT) {
    // raw fp32 partials of this K slice -> splitk_work[slice][row][col] (a lane holds 4
    // consecutive columns of one row per sub-tile, as in gemm_epilogue); the last workgroup of
    // the tile to arrive sums the slices in slice order and runs the normal epilogue
    const long mn = (long)d.M * d.N;
    const bool v4 = (d.N & 3) == 0;
    float* wk = d.splitk_work + (long)blockIdx.y * mn;
#pragma unroll
    for (int a = 0; a < RM; ++a) {
      const int row = m0 + wr * (RM * 16) + a * 16 + fr;
      if (row >= d.M) continue;
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const int col = n0 + wc * (RN * 16) + b * 16 + fg * 4;
        if (v4 && col + 4 <= d.N) {
          *reinterpret_cast<f32x4*>(wk + (long)row * d.N + col) = acc[a][b];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (col + j < d.N) wk[(long)row * d.N + col + j] = acc[a][b][j];
        }
      }
    }
    // publish: every wave drains its partial stores, ONE agent-scope release (L2 write-back) by
    // lane 0, then the ticket; the last arriver alone acquires (one L1 invalidate).  The flag
    // lives in the staging array (a second __shared__ object can make hipcc drain vmcnt before
    // every k-step's LDS reads).  __threadfence() in every thread -- the form this replaced --
    // made each wave write back and invalidate (measured 31 us per fused split-K launch)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* const last = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int prev = __hip_atomic_fetch_add(d.splitk_count + bid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int l = prev == d.splitk - 1;
      if (l) {
        __hip_atomic_store(d.splitk_count + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // zero for the next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = l;
    }
    __syncthreads();
    if (!*last) return;
    __syncthreads();                                  // every wave read the flag before the LDS is reused
#pragma unroll
    for (int a = 0; a < RM; ++a) {
      const int row = min(m0 + wr * (RM * 16) + a * 16 + fr, d.M - 1);
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const int col = n0 + wc * (RN * 16) + b * 16 + fg * 4;
        f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int sl = 0; sl < d.splitk; ++sl) {
          const float* p = d.splitk_work + sl * mn + (long)row * d.N + col;
          if (v4 && col + 4 <= d.N) {
            t += *reinterpret_cast<const f32x4*>(p);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (col + j < d.N) t[j] += p[j];
          }
        }
        acc[a][b] = t;
      }
    }
  }
  // ---- epilogue (shared with the register-staged kernel; acc holds transposed sub-tiles;
  //      LN_EPI: LayerNorm after the product)
  if constexpr (STAGED) {
    if (d.a_mean) gemm_epilogue_staged<BM, BN, true, 2, RM, RN, 256, BM, TRAIN>(d, acc, m0, n0, smem);
    else gemm_epilogue_staged<BM, BN, false, 2, RM, RN, 256, BM, TRAIN>(d, acc, m0, n0, smem);
  } else {
    if (d.a_mean) gemm_epilogue<BM, BN, true, TRAIN>(d, acc, m0, n0);
    else gemm_epilogue<BM, BN, false, TRAIN>(d, acc, m0, n0);
  }
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves in two groups (wr = wave / 4: 128 rows each; wc = wave % 4: 64 columns
// each), BK = 64, one 128-KiB LDS array holding two K-tile buffers ([256 A rows | 256 B rows] x
// 128 B, the same XOR-swizzled image as above).
//
// PING-PONG: every K-tile is four phases, one 64x32 quadrant of the wave's 128x64 output per
// phase (16 MFMAs over K = 64); a phase is a LOAD section (ds_read of the quadrant's fragments,
// LDS-DMA issue, counted vmcnt) and an MFMA section, each closed by a raw s_barrier.  Group 1
// runs one barrier behind group 0, so on every SIMD (waves w and w+4 share one) one wave reads
// LDS while the other keeps the matrix core busy.
//
//   phase 1 reads A top (rows g*128 + 0..63) + B left (cols wc*64 + 0..31)  -> quadrant (T, L)
//   phase 2 reads B right                                                    -> (T, R)
//   phase 3 reads A bottom                                                   -> (B, R)
//   phase 4 reads nothing (fragments still in registers)                     -> (B, L)
//
// A K-tile's buffer is staged in three PARTS, each freed by a phase's reads: TL (A top + B left,
// 4 DMAs per wave), R (B right, 2), B (A bottom, 2).  K-tile t+2 goes into K-tile t's buffer part
// by part as soon as the part is free: TL in phase 2, R in phase 3, B in phase 4 (WAR: every
// load section ends with lgkmcnt(0) before its barrier, so group 1's phase-p reads are complete
// before group 0's phase-(p+1) load section).  Prefetch distance ~1.5-2 K-tiles.  RAW: before
// the barrier that ends the load section preceding a part's first read, every wave waits with a
// counted vmcnt for its own DMAs of that part (the younger DMAs stay in flight); readers of
// group 0 are one barrier, of group 1 two barriers past every wave's wait.  DMAs are issued with
// inline asm (glds16_asm) so the compiler does not drain vmcnt before the ds_reads.
constexpr int B256_STAGE = 512 * ROW;       // (256 A + 256 B rows) x 128 B per K-tile buffer

template <int AH, int BH>
__device__ __forceinline__ void pp_quadrant(f32x4 (&acc)[8][4], const uint4 (&fa)[4][2], const uint4 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[AH * 4 + a][BH * 2 + b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, fb[b][s]), __builtin_bit_cast(bf16x8, fa[a][s]), acc[AH * 4 + a][BH * 2 + b],
            0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

#define PP_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define PP_SYNC_LDS() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

template <bool CONV, bool STAGED, bool TRAIN = false>
__global__ void __launch_bounds__(512) gemm_pp256_kernel(const hv_gemm_desc d) {
  constexpr int BM = 256, BN = 256;
  constexpr int RM = 8, RN = 4;                       // 16x16 sub-tiles per wave (128 x 64)
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

  // staging map: DMA i of this wave covers 8 consecutive tile rows; i = 0,1 the A-top / B-left
  // part, i = 2,3 the A-bottom / B-right part (16 row groups per part, two per wave)
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int lrow = lane >> 3, pchunk = lane & 7;
  int arow0[4], brow0[4];                              // first tile row / column of DMA i (uniform)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wu * 2 + (i & 1);
    arow0[i] = (q >> 3) * 128 + (i >> 1) * 64 + (q & 7) * 8;
    brow0[i] = (q >> 2) * 64 + (i >> 1) * 32 + (q & 3) * 8;
  }
  const unsigned short* arow[4];
  int aih[4], aiw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int row = m0 + arow0[i] + lrow;
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
  const unsigned short* brow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int n = n0 + brow0[i] + lrow;
    n = n < d.N ? n : d.N - 1;
    brow[i] = (const unsigned short*)d.B + (long)n * d.ldb;
  }
  const int lchunk = pchunk ^ (lrow & 7);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  // conv fast path (conv_c % 64 == 0): wave-uniform K-tile offsets (ConvK), per-lane pixel base;
  // ckn = the position of the next K-tile whose A parts are staged (K-tiles are staged in order)
  int apix[4];
  ConvK ckn;
  if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < 4; ++i) apix[i] = (aih[i] * d.conv_w + aiw[i]) * d.conv_c + lchunk * 8;
    ckn.init(d, 0);
  }
  auto dma_a_fast = [&](int buf, const ConvK& c, int koff, int i) {
    const int ih = aih[i] + c.kh, iw = aiw[i] + c.kw;
    const void* src = ((unsigned)ih < (unsigned)d.conv_h && (unsigned)iw < (unsigned)d.conv_w)
                          ? (const void*)(arow[i] + apix[i] + koff) : (const void*)hv_glds_zero_line;
    glds16_asm(src, lds0 + buf * B256_STAGE + arow0[i] * ROW);
  };

  auto dma_a = [&](int buf, int kt, int i) {
    const int k = kt * 64 + lchunk * 8;
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
        const int row = min(m0 + arow0[i] + lrow, d.M - 1);
        src = (const unsigned short*)d.A2 + (long)row * d.lda2 + (k - d.k1);
      } else {
        src = arow[i] + k;
      }
    }
    glds16_asm(src, lds0 + buf * B256_STAGE + arow0[i] * ROW);
  };
  auto dma_b = [&](int buf, int kt, int i) {
    glds16_asm(brow[i] + kt * 64 + lchunk * 8, lds0 + buf * B256_STAGE + BM * ROW + brow0[i] * ROW);
  };
  // the A parts of K-tile kt: TL (rows 0, 1) then B (rows 2, 3); ckn is advanced after part B
  // (this kernel only runs convs with K % 64 == 0, i.e. conv_c % 64 == 0: always the fast path)
  auto part_tl = [&](int buf, int kt) {
    if constexpr (CONV) {
      const int koff = ckn.offset(d);
      dma_a_fast(buf, ckn, koff, 0);
      dma_a_fast(buf, ckn, koff, 1);
    } else {
      dma_a(buf, kt, 0);
      dma_a(buf, kt, 1);
    }
    dma_b(buf, kt, 0);
    dma_b(buf, kt, 1);
  };
  auto part_r = [&](int buf, int kt) { dma_b(buf, kt, 2); dma_b(buf, kt, 3); };
  auto part_b = [&](int buf, int kt) {
    if constexpr (CONV) {
      const int koff = ckn.offset(d);
      dma_a_fast(buf, ckn, koff, 2);
      dma_a_fast(buf, ckn, koff, 3);
      ckn.advance(d);
    } else {
      dma_a(buf, kt, 2);
      dma_a(buf, kt, 3);
    }
  };

  const int fr = lane & 15, fg = lane >> 4;
  // fragment reads: A rows wr*128 + half*64 + a*16 + fr, B cols wc*64 + half*32 + b*16 + fr;
  // k-slice s of the 64-deep tile = 16-B chunks {4s + fg}
  auto read_a = [&](const unsigned char* sa, int half, uint4 (&fa)[4][2]) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = wr * 128 + half * 64 + a * 16 + fr, lc = s * 4 + fg;
        fa[a][s] = *reinterpret_cast<const uint4*>(sa + r * ROW + ((lc ^ (r & 7)) << 4));
      }
  };
  auto read_b = [&](const unsigned char* sb, int half, uint4 (&fb)[2][2]) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = wc * 64 + half * 32 + b * 16 + fr, lc = s * 4 + fg;
        fb[b][s] = *reinterpret_cast<const uint4*>(sb + r * ROW + ((lc ^ (r & 7)) << 4));
      }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = d.K / 64;
  // prologue: K-tiles 0 and 1 in part order; K-tile 0's TL part retired before the first read
  part_tl(0, 0); part_r(0, 0); part_b(0, 0);
  if (nk > 1) {
    part_tl(1, 1); part_r(1, 1); part_b(1, 1);
    PP_VMCNT(12);
  } else {
    PP_VMCNT(4);
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();            // group 1 runs one barrier behind

  uint4 fa[4][2], fbl[2][2], fbr[2][2];
  // K-tile kt from buffer BUF (compile-time, unrolled by two)
  auto ktile = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    const unsigned char* sa = smem + BUF * B256_STAGE;
    const unsigned char* sb = sa + BM * ROW;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 1: A top + B left; then K-tile kt's R part must have landed
    read_a(sa, 0, fa);
    read_b(sb, 0, fbl);
    if (n1) PP_VMCNT(10); else PP_VMCNT(2);
    PP_SYNC_LDS();
    __builtin_amdgcn_s_barrier();
    pp_quadrant<0, 0>(acc, fa, fbl);
    __builtin_amdgcn_s_barrier();
    // phase 2: B right; K-tile kt+2's TL part into the freed TL region; then kt's B part landed
    read_b(sb, 1, fbr);
    if (n2) {
      part_tl(BUF, kt + 2);
      PP_VMCNT(12);
    } else if (n1) {
      PP_VMCNT(8);
    } else {
      PP_VMCNT(0);
    }
    PP_SYNC_LDS();
    __builtin_amdgcn_s_barrier();
    pp_quadrant<0, 1>(acc, fa, fbr);
    __builtin_amdgcn_s_barrier();
    // phase 3: A bottom; K-tile kt+2's R part
    read_a(sa, 1, fa);
    if (n2) part_r(BUF, kt + 2);
    PP_SYNC_LDS();
    __builtin_amdgcn_s_barrier();
    pp_quadrant<1, 1>(acc, fa, fbr);
    __builtin_amdgcn_s_barrier();
    // phase 4: K-tile kt+2's B part; then K-tile kt+1's TL part landed
    if (n2) {
      part_b(BUF, kt + 2);
      PP_VMCNT(12);
    } else if (n1) {
      PP_VMCNT(4);
    }
    __builtin_amdgcn_s_barrier();
    pp_quadrant<1, 0>(acc, fa, fbl);
    __builtin_amdgcn_s_barrier();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    ktile(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nk) ktile(std::integral_constant<int, 1>{}, kt + 1);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();            // equal barrier counts
  if constexpr (STAGED) {
    if (d.a_mean) gemm_epilogue_staged<BM, BN, true, 4, RM, RN, 512, 128>(d, acc, m0, n0, smem);
    else gemm_epilogue_staged<BM, BN, false, 4, RM, RN, 512, 128>(d, acc, m0, n0, smem);
  } else {
    if (d.a_mean) gemm_epilogue<BM, BN, true, TRAIN, 4, RM, RN>(d, acc, m0, n0);
    else gemm_epilogue<BM, BN, false, TRAIN, 4, RM, RN>(d, acc, m0, n0);
  }
}

// ring depth per tile: the small tiles have short K-steps that cannot cover the DMA latency
// with one tile in flight (64x64: 4 buffers = 64 KiB, 64x128 / 128x64: 3 = 72 KiB)
template <int BM, int BN>
constexpr int deep_stages() { return BM * BN <= 64 * 64 ? 4 : (BM * BN <= 128 * 64 ? 3 : 2); }

template <int BM, int BN>
void glds_count() {
  hv_diag_count(BM == 128 && BN == 128 ? HV_KF_GEMM_GLDS_128x128 : BM == 64 && BN == 128 ? HV_KF_GEMM_GLDS_64x128
                : BM == 128 ? HV_KF_GEMM_GLDS_128x64 : HV_KF_GEMM_GLDS_64x64);
}

// training epilogues (epi_mode 1/2): 2-stage ring (the deeper ring measured slower with the
// training epilogues' register footprint: train step 183.7 vs 176.0 ms)
template <int BM, int BN>
int launch_train(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, BM) * hv_cdiv(d.N, BN);
  glds_count<BM, BN>();
  if (!(d.variant & HV_GV_FLAT_TRAIN)) {
    if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, true, true, 2><<<grid, 256, 0, s>>>(d);
    else gemm_glds_kernel<BM, BN, false, true, true, 2><<<grid, 256, 0, s>>>(d);
  } else {
    if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, true, false, 2><<<grid, 256, 0, s>>>(d);
    else gemm_glds_kernel<BM, BN, false, true, false, 2><<<grid, 256, 0, s>>>(d);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// inference epilogues: LDS-staged (+25-35 % at K <= 512) unless the call asks for the
// fragment-layout one (HV_GV_FLAT_EPI)
template <int BM, int BN, int NS>
int launch_infer_ns(const hv_gemm_desc& d, hipStream_t s) {
  const unsigned grid = hv_cdiv(d.M, BM) * hv_cdiv(d.N, BN);
  glds_count<BM, BN>();
  if (!(d.variant & HV_GV_FLAT_EPI)) {
    if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, false, true, NS><<<grid, 256, 0, s>>>(d);
    else gemm_glds_kernel<BM, BN, false, false, true, NS><<<grid, 256, 0, s>>>(d);
  } else {
    if (d.conv_k > 0) gemm_glds_kernel<BM, BN, true, false, false, NS><<<grid, 256, 0, s>>>(d);
    else gemm_glds_kernel<BM, BN, false, false, false, NS><<<grid, 256, 0, s>>>(d);
  }
  HV_CHECK_LAUNCH();
  return HV_OK;
}

template <int BM, int BN>
int launch_infer(const hv_gemm_desc& d, hipStream_t s) {
  constexpr int NS = deep_stages<BM, BN>();
  if constexpr (BM == 64 && BN == 64) {
    // 8-stage ring (128 KB LDS, one workgroup per CU), opt-in (HV_GV_DEEP8): built for the B=1
    // frame's small grids on the theory that their k-loop waits on DMA latency / K-tiles in
    // flight -- measured no faster than the 4-stage ring (the 2-stage ring is fastest there) and
    // B=1 p50 5.23 vs 4.97-5.04 ms (profiles/r04/deep8_rejected.txt): the per-K-tile cost is the
    // barrier / LDS-read / MFMA dependency chain of a lone workgroup, not the DMA
    if (d.variant & HV_GV_DEEP8) return launch_infer_ns<64, 64, 8>(d, s);
  }
  if constexpr (NS > 2) {
    if (!(d.variant & HV_GV_SHALLOW)) return launch_infer_ns<BM, BN, NS>(d, s);
  }
  return launch_infer_ns<BM, BN, 2>(d, s);
}

}  // namespace

// per-TU launchers (hv_gemm_glds_*.hip)
int hv_glds_infer_64x64(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_infer_32x64(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_infer_64x128(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_infer_128x64(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_infer_128x128(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_train_64x64(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_train_64x128(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_train_128x64(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_train_128x128(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_launch256(const hv_gemm_desc& d, hipStream_t s);
int hv_glds_launch_splitk(const hv_gemm_desc& d, hipStream_t s);
