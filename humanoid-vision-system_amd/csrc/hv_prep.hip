// Grouped per-forward parameter preparation for gfx950.
//
// The reference rebuilds every mHC site's constrained matrices on every forward
// (ManifoldHyperConnection.constrained_matrices, manifold_layers.py:205-221) and, under GPU
// autocast, re-casts every weight it touches.  Done site by site that is ~10 tiny launches
// per mHC site and 2 per Conv-BN pair (about a thousand per forward, each a few
// microseconds of mostly idle GPU).  Here every site of the model is one entry of a device
// table and each phase is one launch over the concatenated block ranges of all entries:
//   hv_mhc_prep_group: 4 launches for all 76 mHC sites (column sums / row means, centred
//                      Gc + u + Wc^T, fold GEMM A1^T = W1 Gc^T on MFMA + c1 = W1 u + b1,
//                      row sums of the stored A1^T for the GEMM's LayerNorm epilogue);
//   hv_wprep_group:    1 launch for every cast and every Conv(+BN) weight reorder/fold.
// A block finds its entry by binary search over the entries' exclusive block prefixes.
#include "hv_common.h"

#include <type_traits>

namespace {

constexpr int PT = 64;           // H_pre tiles: 64 (k) x 64 (i)

struct PrepSizes {
  int ntk, nrb;                  // column tiles over Hd, row blocks over D
  int colsum, rowmean, write, wct, fold, gemv, rowsum;
};

__host__ __device__ inline PrepSizes prep_sizes(int D, int Hd, int fold) {
  PrepSizes s;
  s.ntk = (Hd + PT - 1) / PT;
  s.nrb = (D + PT - 1) / PT;
  s.colsum = s.ntk * s.nrb;
  s.rowmean = (D + Hd + 3) / 4;
  s.write = s.ntk * s.nrb;
  s.wct = ((D + Hd + 31) / 32) * ((D + 31) / 32);
  s.fold = fold ? (2 * Hd / 64) * ((D + 63) / 64) : 0;
  s.gemv = fold ? (2 * Hd + 15) / 16 : 0;
  s.rowsum = ((fold ? 2 * Hd : Hd) + 3) / 4;
  return s;
}

// scratch carve: gc [D*Hd] | u [Hd] | rm [D+Hd] | part [2*nrb*Hd]
struct Scratch {
  float *gc, *u, *rm, *part;
};
__device__ inline Scratch carve(const hv_mhc_prep_entry& e) {
  const PrepSizes s = prep_sizes(e.D, e.Hd, e.fold);
  Scratch c;
  c.gc = e.scratch;
  c.u = c.gc + (long)e.D * e.Hd;
  c.rm = c.u + e.Hd;
  c.part = c.rm + e.D + e.Hd;
  (void)s;
  return c;
}

template <typename E, int PH>
__device__ inline int find_entry(const E* t, int count, int b) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {                       // last entry with blk <= b
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].blk[PH] <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// ------------------------------------------------------------------ phase 1
__global__ void __launch_bounds__(256) k_pg1(const hv_mhc_prep_entry* __restrict__ tab, int count) {
  __shared__ float red[2][4][PT];
  const int ei = find_entry<hv_mhc_prep_entry, 0>(tab, count, blockIdx.x);
  const hv_mhc_prep_entry& e = tab[ei];
  const int D = e.D, Hd = e.Hd;
  const PrepSizes s = prep_sizes(D, Hd, e.fold);
  const Scratch sc = carve(e);
  int b = blockIdx.x - e.blk[0];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (b < s.colsum) {
    // column partials over 64 rows: sum_i g_i s(raw[i,k]) and sum_i b_i s(raw[i,k])
    const int kt = b % s.ntk, rb = b / s.ntk;
    const int k = kt * PT + lane;
    float sg = 0.f, sb = 0.f;
    if (k < Hd) {
      for (int r = w; r < PT; r += 4) {
        const int i = rb * PT + r;
        if (i >= D) break;
        const float v = sigm(e.h_pre_raw[(long)i * Hd + k]);
        sg += e.gamma_pre[i] * v;
        sb += e.beta_pre[i] * v;
      }
    }
    red[0][w][lane] = sg;
    red[1][w][lane] = sb;
    __syncthreads();
    if (w == 0 && k < Hd) {
      sc.part[(long)rb * Hd + k] = (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]);
      sc.part[(long)(s.nrb + rb) * Hd + k] = (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]);
    }
    return;
  }
  b -= s.colsum;
  // row means of H_res (rows < D) and of H_post = 2 s(H_post_raw) (rows D..D+Hd-1)
  const int r = b * 4 + w;
  if (r >= D + Hd) return;
  float acc = 0.f;
  if (r < D) {
    for (int j = lane; j < D; j += 64) acc += e.h_res[(long)r * D + j];
  } else {
    const float* p = e.h_post_raw + (long)(r - D) * D;
    for (int j = lane; j < D; j += 64) acc += 2.0f * sigm(p[j]);
  }
  acc = wave_sum(acc);
  if (lane == 0) sc.rm[r] = acc / D;
}

// ------------------------------------------------------------------ phase 2
template <typename T>
__global__ void __launch_bounds__(256) k_pg2(const hv_mhc_prep_entry* __restrict__ tab, int count) {
  __shared__ float tile[PT][PT + 1];
  const int ei = find_entry<hv_mhc_prep_entry, 1>(tab, count, blockIdx.x);
  const hv_mhc_prep_entry& e = tab[ei];
  const int D = e.D, Hd = e.Hd;
  const PrepSizes s = prep_sizes(D, Hd, e.fold);
  const Scratch sc = carve(e);
  int b = blockIdx.x - e.blk[1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (b < s.write) {
    const int kt = b % s.ntk, rb = b / s.ntk;
    const int k = kt * PT + lane;
    float sg = 0.f, sb = 0.f;
    if (k < Hd)
      for (int q = 0; q < s.nrb; ++q) { sg += sc.part[(long)q * Hd + k]; sb += sc.part[(long)(s.nrb + q) * Hd + k]; }
    const float mean = sg / D;
    if (rb == 0 && w == 0 && k < Hd) {
      if (e.fold) sc.u[k] = sb; else e.c1[k] = sb;
    }
    if (e.fold) {
      if (k < Hd)
        for (int r = w; r < PT; r += 4) {
          const int i = rb * PT + r;
          if (i >= D) break;
          sc.gc[(long)i * Hd + k] = e.gamma_pre[i] * sigm(e.h_pre_raw[(long)i * Hd + k]) - mean;
        }
    } else {
      // Gc^T [Hd, D] in the compute dtype, transposed through LDS for coalesced stores
      for (int r = w; r < PT; r += 4) {
        const int i = rb * PT + r;
        tile[r][lane] = (k < Hd && i < D) ? e.gamma_pre[i] * sigm(e.h_pre_raw[(long)i * Hd + k]) - mean : 0.f;
      }
      __syncthreads();
      for (int r = w; r < PT; r += 4) {
        const int kk = kt * PT + r, i = rb * PT + lane;
        if (kk < Hd && i < D) Elem<T>::store((T*)e.a1, (long)kk * D + i, tile[lane][r]);
      }
    }
    return;
  }
  b -= s.write;
  // Wc^T[j][i] = src[i][j] - rm[i], src = [H_res ; 2 s(H_post_raw)] ([D+Hd, D]); 32x32 tiles
  const int Kc = D + Hd;
  const int nti = (Kc + 31) / 32;
  const int i0 = (b % nti) * 32, j0 = (b / nti) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int i = i0 + r, j = j0 + tx;
    float v = 0.f;
    if (i < Kc && j < D) {
      v = i < D ? e.h_res[(long)i * D + j] : 2.0f * sigm(e.h_post_raw[(long)(i - D) * D + j]);
      v -= sc.rm[i];
    }
    tile[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int j = j0 + r, i = i0 + tx;
    if (j < D && i < Kc) Elem<T>::store((T*)e.wct, (long)j * Kc + i, tile[tx][r]);
  }
}

// ------------------------------------------------------------------ phase 3: fold GEMM
// A1^T[m, n] = sum_k W1[m, k] Gc[n, k]  (M = 2Hd, N = D, K = Hd), 64x64 tiles, 4 waves 2x2,
// k-steps of 32 staged through LDS after an fp32 -> compute-type convert.  bf16: one
// v_mfma_f32_16x16x32_bf16 per 16x16 sub-tile; fp32: v_mfma_f32_16x16x4_f32 x 8 (exact
// products; lane group g takes k = 4g..4g+3 of each 16-deep half).
template <typename T>
__device__ __forceinline__ void fold_tile(const hv_mhc_prep_entry& e, const Scratch& sc, int tile, char* lds) {
  constexpr bool BF = std::is_same<T, unsigned short>::value;
  // LDS row bytes: 32 k + pad.  bf16: 96-B rows put the 16 rows of each ds_read_b128 lane group
  // (rows 0-3 / 12-15 at chunk fg, 4-11 at fg+1, or the reverse) on 16 distinct 4-bank sets
  // ((6 r + c) mod 16 is a bijection there); the 80-B rows had rows r and r+3 colliding
  // (SQ_LDS_BANK_CONFLICT 0.36 of the LDS cycles)
  constexpr int RB = BF ? 96 : 144;
  const int D = e.D, K = e.Hd;
  const int ntn = (D + 63) / 64;
  const int m0 = (tile / ntn) * 64, n0 = (tile % ntn) * 64;
  char* As = lds;
  char* Bs = lds + 64 * RB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int lr = t >> 2, lq = (t & 3) * 8;
  const float* Ar = e.w1 + (long)(m0 + lr) * K + lq;
  const bool bvalid = n0 + lr < D;
  const float* Br = sc.gc + (long)(bvalid ? n0 + lr : 0) * K + lq;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // register double buffering: the next k-step's global loads are issued before this step's
  // MFMAs, so their latency overlaps the compute instead of stalling every k-step
  float4 na0 = *reinterpret_cast<const float4*>(Ar);
  float4 na1 = *reinterpret_cast<const float4*>(Ar + 4);
  float4 nb0 = make_float4(0.f, 0.f, 0.f, 0.f), nb1 = nb0;
  if (bvalid) {
    nb0 = *reinterpret_cast<const float4*>(Br);
    nb1 = *reinterpret_cast<const float4*>(Br + 4);
  }
  for (int k0 = 0; k0 < K; k0 += 32) {
    const float4 a0 = na0, a1 = na1, b0 = nb0, b1 = nb1;
    __syncthreads();
    if constexpr (BF) {
      const u16x8 pa = {f2bf(a0.x), f2bf(a0.y), f2bf(a0.z), f2bf(a0.w), f2bf(a1.x), f2bf(a1.y), f2bf(a1.z), f2bf(a1.w)};
      const u16x8 pb = {f2bf(b0.x), f2bf(b0.y), f2bf(b0.z), f2bf(b0.w), f2bf(b1.x), f2bf(b1.y), f2bf(b1.z), f2bf(b1.w)};
      *reinterpret_cast<u16x8*>(As + lr * RB + lq * 2) = pa;
      *reinterpret_cast<u16x8*>(Bs + lr * RB + lq * 2) = pb;
    } else {
      *reinterpret_cast<float4*>(As + lr * RB + lq * 4) = a0;
      *reinterpret_cast<float4*>(As + lr * RB + lq * 4 + 16) = a1;
      *reinterpret_cast<float4*>(Bs + lr * RB + lq * 4) = b0;
      *reinterpret_cast<float4*>(Bs + lr * RB + lq * 4 + 16) = b1;
    }
    __syncthreads();
    if (k0 + 32 < K) {
      na0 = *reinterpret_cast<const float4*>(Ar + k0 + 32);
      na1 = *reinterpret_cast<const float4*>(Ar + k0 + 36);
      if (bvalid) {
        nb0 = *reinterpret_cast<const float4*>(Br + k0 + 32);
        nb1 = *reinterpret_cast<const float4*>(Br + k0 + 36);
      }
    }
    const int fr = lane & 15, fg = lane >> 4;
    if constexpr (BF) {
      uint4 fa[2], fb[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[a] = *reinterpret_cast<const uint4*>(As + (wr * 32 + a * 16 + fr) * RB + fg * 16);
#pragma unroll
      for (int c = 0; c < 2; ++c) fb[c] = *reinterpret_cast<const uint4*>(Bs + (wc * 32 + c * 16 + fr) * RB + fg * 16);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[a]),
                                                              __builtin_bit_cast(bf16x8, fb[c]), acc[a][c], 0, 0, 0);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float4 fa[2], fb[2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
          fa[a] = *reinterpret_cast<const float4*>(As + (wr * 32 + a * 16 + fr) * RB + (h * 16 + fg * 4) * 4);
#pragma unroll
        for (int c = 0; c < 2; ++c)
          fb[c] = *reinterpret_cast<const float4*>(Bs + (wc * 32 + c * 16 + fr) * RB + (h * 16 + fg * 4) * 4);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a].x, fb[c].x, acc[a][c], 0, 0, 0);
            acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a].y, fb[c].y, acc[a][c], 0, 0, 0);
            acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a].z, fb[c].z, acc[a][c], 0, 0, 0);
            acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a].w, fb[c].w, acc[a][c], 0, 0, 0);
          }
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = n0 + wc * 32 + c * 16 + (lane & 15);
      if (col >= D) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + wr * 32 + a * 16 + (lane >> 4) * 4 + j;
        Elem<T>::store((T*)e.a1, (long)row * D + col, acc[a][c][j]);
      }
    }
}

template <typename T>
__global__ void __launch_bounds__(256) k_pg3(const hv_mhc_prep_entry* __restrict__ tab, int count) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 64 * 144];
  // hardware order: an XCD-local remap (each XCD a contiguous range of tiles, so the tiles of
  // one W1 row block share an L2) measured SLOWER, 577 vs 408 us per forward -- the round-robin
  // deal spreads each row block's tiles over all eight XCDs' HBM request queues at once
  const int bx = blockIdx.x;
  const int ei = find_entry<hv_mhc_prep_entry, 2>(tab, count, bx);
  const hv_mhc_prep_entry& e = tab[ei];
  const PrepSizes s = prep_sizes(e.D, e.Hd, e.fold);
  const Scratch sc = carve(e);
  const int b = bx - e.blk[2];
  if (b < s.fold) {
    fold_tile<T>(e, sc, b, lds);
    return;
  }
  // c1 = W1 u + b1: 16 rows per block, 4 per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, K = e.Hd;
  for (int q = 0; q < 4; ++q) {
    const int m = (b - s.fold) * 16 + w * 4 + q;
    if (m >= 2 * e.Hd) break;
    const float* row = e.w1 + (long)m * K;
    float acc = 0.f;
    for (int k = lane; k < K; k += 64) acc += row[k] * sc.u[k];
    acc = wave_sum(acc);
    if (lane == 0) e.c1[m] = acc + (e.b1 ? e.b1[m] : 0.f);
  }
}

// ------------------------------------------------------------------ phase 4
// cs[n] = sum_k a1[n, k] over the values as stored (bf16-rounded in bf16 mode), so the
// LN-after-GEMM epilogue rstd (x.a1 - mean cs) equals LN-before-GEMM on the same operand.
template <typename T>
__global__ void __launch_bounds__(256) k_pg4(const hv_mhc_prep_entry* __restrict__ tab, int count) {
  const int ei = find_entry<hv_mhc_prep_entry, 3>(tab, count, blockIdx.x);
  const hv_mhc_prep_entry& e = tab[ei];
  const int rows = e.fold ? 2 * e.Hd : e.Hd, K = e.D;
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x - e.blk[3]) * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* p = (const T*)e.a1 + (long)r * K;
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) acc += Elem<T>::load(p, k);
  acc = wave_sum(acc);
  if (lane == 0) e.cs[r] = acc;
}

// ------------------------------------------------------------------ weight prep group
constexpr int WP_CAST_CHUNK = 4096;   // elements per block (cast)
constexpr int WP_CONV_ROWS = 4;       // output channels per block (conv), one wave each
constexpr int WP_MAX_TAPS = 9;        // staged reorder: kernels up to 3x3

template <typename T>
__device__ __forceinline__ void wp_cast(const hv_wprep_entry& e, int b) {
  const long base = (long)b * WP_CAST_CHUNK;
  const long end = min((long)e.n, base + WP_CAST_CHUNK);
  T* y = (T*)e.dst;
  const bool vec = ((((uintptr_t)e.src) | ((uintptr_t)e.dst)) & 15) == 0;
  if (vec && end - base == WP_CAST_CHUNK) {
    // 8 elements per thread and pass: two 16-byte loads, one 16-byte bf16 store (the scalar
    // 2-byte stores this replaced held the cast pass near half the HBM rate); all loads first
#pragma unroll
    for (int q = 0; q < WP_CAST_CHUNK / 2048; ++q) {
      const long i = base + (q * 256 + threadIdx.x) * 8;
      const float4 v0 = *reinterpret_cast<const float4*>(e.src + i);
      const float4 v1 = *reinterpret_cast<const float4*>(e.src + i + 4);
      if constexpr (std::is_same<T, unsigned short>::value) {
        *reinterpret_cast<uint4*>(y + i) = make_uint4(pack_bf16x2(v0.x, v0.y), pack_bf16x2(v0.z, v0.w),
                                                      pack_bf16x2(v1.x, v1.y), pack_bf16x2(v1.z, v1.w));
      } else {
        *reinterpret_cast<float4*>(y + i) = v0;
        *reinterpret_cast<float4*>(y + i + 4) = v1;
      }
    }
  } else {
    for (long i = base + threadIdx.x; i < end; i += 256) Elem<T>::store(y, i, e.src[i]);
  }
}

template <typename T>
__device__ __forceinline__ void wp_conv(const hv_wprep_entry& e, int b, float* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int co = b * WP_CONV_ROWS + w;
  if (co >= e.n) return;
  const float sc = e.gamma ? e.gamma[co] / sqrtf(e.var[co] + e.eps) : 1.0f;
  if (lane == 0) {
    const float cb = e.cbias ? e.cbias[co] : 0.f;
    if (e.scale_out) e.scale_out[co] = sc;
    if (e.bias_out) e.bias_out[co] = e.gamma ? e.beta[co] + (cb - e.mean[co]) * sc : cb;
  }
  const int cin = e.cin, k = e.k, kt = k * k, kk = kt * cin;
  const float* wr = e.src + (long)co * kk;
  T* yr = (T*)e.dst + (long)co * e.ldk;
  if (cin % 64 == 0 && kt <= WP_MAX_TAPS && (((uintptr_t)wr) & 15) == 0) {
    // 64 input channels per trip: their kt taps are one contiguous source run (64 * kt floats),
    // loaded with 16-byte coalesced loads into this wave's LDS slice, then written out tap by
    // tap as 64 consecutive outputs.  The element loop below issues one 4-byte load per lane
    // and waits for it before the store (the store may alias the source for the compiler):
    // latency-bound at a few bytes in flight per wave
    float* sl = lds + (threadIdx.x >> 6) * (64 * WP_MAX_TAPS);
    const int n4 = 16 * kt;
    for (int c0 = 0; c0 < cin; c0 += 64) {
      const float4* s4 = reinterpret_cast<const float4*>(wr + (long)c0 * kt);
      float4 v[(64 * WP_MAX_TAPS / 4 + 63) / 64];
#pragma unroll
      for (int q = 0; q < (64 * WP_MAX_TAPS / 4 + 63) / 64; ++q)
        if (lane + 64 * q < n4) v[q] = s4[lane + 64 * q];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < (64 * WP_MAX_TAPS / 4 + 63) / 64; ++q)
        if (lane + 64 * q < n4) *reinterpret_cast<float4*>(sl + 4 * (lane + 64 * q)) = v[q];
      // one wave's LDS operations complete in order: its own slice needs no barrier
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int t = 0; t < kt; ++t) Elem<T>::store(yr, (long)t * cin + c0 + lane, sl[lane * kt + t]);
      __builtin_amdgcn_wave_barrier();
    }
    for (int i = kk + lane; i < e.ldk; i += 64) Elem<T>::store(yr, i, 0.f);
    return;
  }
  for (int i = lane; i < e.ldk; i += 64) {
    float v = 0.f;
    if (i < kk) {
      const int ci = i % cin, t = i / cin;          // i = (kh*k + kw)*cin + ci
      v = wr[(long)ci * k * k + t];               // BN scale stays in the GEMM epilogue
    }
    Elem<T>::store(yr, i, v);
  }
}

__device__ inline int find_wp(const hv_wprep_entry* t, int count, int b) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].blk <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) k_wprep(const hv_wprep_entry* __restrict__ tab, int count) {
  __shared__ __attribute__((aligned(16))) float lds[WP_CONV_ROWS * 64 * WP_MAX_TAPS];
  const hv_wprep_entry& e = tab[find_wp(tab, count, blockIdx.x)];
  const int b = blockIdx.x - e.blk;
  if (e.kind == 0) {
    if (e.dtype == HV_BF16) wp_cast<unsigned short>(e, b); else wp_cast<float>(e, b);
  } else {
    if (e.dtype == HV_BF16) wp_conv<unsigned short>(e, b, lds); else wp_conv<float>(e, b, lds);
  }
}

}  // namespace

extern "C" size_t hv_mhc_prep_scratch_floats(int D, int Hd) {
  const PrepSizes s = prep_sizes(D, Hd, 1);
  return (size_t)D * Hd + Hd + (D + Hd) + 2L * s.nrb * Hd;
}

extern "C" void hv_mhc_prep_blocks(int D, int Hd, int fold, int* out4) {
  const PrepSizes s = prep_sizes(D, Hd, fold);
  out4[0] = s.colsum + s.rowmean;
  out4[1] = s.write + s.wct;
  out4[2] = s.fold + s.gemv;
  out4[3] = s.rowsum;
}

extern "C" int hv_mhc_prep_group(const hv_mhc_prep_entry* tab, int count, int dtype, const int* totals,
                                 hv_stream_t stream) {
  if (count <= 0 || !tab || !totals) return HV_EINVAL;
  if (dtype != HV_F32 && dtype != HV_BF16) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (totals[0] > 0) k_pg1<<<totals[0], 256, 0, s>>>(tab, count);
  if (totals[1] > 0) HV_DISPATCH(dtype, (k_pg2<T><<<totals[1], 256, 0, s>>>(tab, count)));
  if (totals[2] > 0) HV_DISPATCH(dtype, (k_pg3<T><<<totals[2], 256, 0, s>>>(tab, count)));
  if (totals[3] > 0) HV_DISPATCH(dtype, (k_pg4<T><<<totals[3], 256, 0, s>>>(tab, count)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_wprep_blocks(int kind, long n, int cin, int k) {
  (void)cin;
  (void)k;
  if (kind == 0) return (int)((n + WP_CAST_CHUNK - 1) / WP_CAST_CHUNK);
  return (int)((n + WP_CONV_ROWS - 1) / WP_CONV_ROWS);
}

extern "C" int hv_wprep_group(const hv_wprep_entry* tab, int count, int total_blocks, hv_stream_t stream) {
  if (count <= 0 || total_blocks <= 0 || !tab) return HV_EINVAL;
  k_wprep<<<total_blocks, 256, 0, (hipStream_t)stream>>>(tab, count);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
