// Grouped Sinkhorn-Knopp projection for gfx950.
//
// Replaces SinkhornKnoppProjection.forward (reference src/models/manifold_layers.py:32-93).
// The reference rescales the whole matrix in place 2*iters times and reads three host
// scalars per iteration (.item(), :68,73,76).  Every step of that loop is a row or a
// column scaling, so M_t = diag(a_t) K diag(b_t) with K = softmax(raw/tau)*m fixed:
//     r_t  = a_t (.) (K b_t)            (row sums, :66)
//     a_t+1 = a_t / (r_t + eps)         (:67)
//     c_t  = b_t (.) (K^T a_t+1)        (column sums, :71)
//     b_t+1 = b_t / (c_t + eps)         (:72)
// K is read, never rewritten: each iteration is one fused "row dots + column partial
// sums" pass over K (L2/MALL resident) and one tiny column-reduce pass.  Every matrix of
// every mHC site of the model shares the same 2*iters+2 launches (a device table of
// entries), nothing syncs with the host, and the a/b/r vectors of every iteration stay in
// the workspace for the analytic backward.  Summation order is fixed -> bitwise
// reproducible.
#include <mutex>

#include "hv_common.h"

namespace {

constexpr int RB = 16;          // rows per block in the row pass (4 per wave)
constexpr int MAXQ = 32;        // up to 64*32 = 2048 columns held per lane

struct Work {                   // carve of hv_sinkhorn_entry::work
  float* a;                     // [(iters+1), batch*n]
  float* b;                     // [(iters+1), batch*m]
  float* r;                     // [iters, batch*n]
  float* part;                  // [batch, ceil(n/RB), m] column partials
};

__device__ __forceinline__ Work carve(const hv_sinkhorn_entry& e) {
  Work w;
  const long bn = (long)e.batch * e.n, bm = (long)e.batch * e.m;
  w.a = e.work;
  w.b = w.a + (long)(e.iters + 1) * bn;
  w.r = w.b + (long)(e.iters + 1) * bm;
  w.part = w.r + (long)e.iters * bn;
  return w;
}

// Entries of at most 256 x 256 (65 of the model's 76 matrices: D = 32 .. 256) run the whole
// projection in ONE workgroup (sk_small: K in registers, all iterations inside); the grouped
// multi-launch passes below skip them and handle only the large ones (D = 512, 1024, 1792).
// small_max = 0 sends every entry through the grouped passes (A/B knob hv_sinkhorn_set_small).
__device__ __forceinline__ bool sk_is_small(const hv_sinkhorn_entry& e, int small_max) {
  return e.batch == 1 && e.n <= small_max && e.m <= small_max;
}

// Find the entry whose [start, start+len) range contains idx (entries sorted by start).
template <int FIELD>
__device__ __forceinline__ int entry_start(const hv_sinkhorn_entry& e) {
  return FIELD == 0 ? e.row_start : (FIELD == 1 ? e.row_block_start : e.col_start);
}
template <int FIELD>
__device__ __forceinline__ int find_entry(const hv_sinkhorn_entry* t, int count, int idx) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (entry_start<FIELD>(t[mid]) <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}
template <int FIELD>
__device__ __forceinline__ int find_entry_wave(const hv_sinkhorn_entry* t, int count, int idx);
// Per-lane idx inside [first, last] (wave-uniform bounds): when both ends fall in one entry (the
// common case -- the large entries' column ranges are multiples of 64) two ballots decide it.
template <int FIELD>
__device__ __forceinline__ int find_entry_span(const hv_sinkhorn_entry* t, int count, int idx, int first,
                                               int last) {
  const int e0 = find_entry_wave<FIELD>(t, count, first);
  const int e1 = find_entry_wave<FIELD>(t, count, last);
  return e0 == e1 ? e0 : find_entry<FIELD>(t, count, idx);
}
// The same for a wave-uniform idx: each lane reads one entry's start, a ballot counts the starts
// <= idx.  One memory round trip per 64 entries instead of log2(count) dependent ones (the
// grouped passes are latency-bound launches, ~20 per forward).  Whole wave must be active.
template <int FIELD>
__device__ __forceinline__ int find_entry_wave(const hv_sinkhorn_entry* t, int count, int idx) {
  const int lane = threadIdx.x & 63;
  int n_le = 0;
  for (int base = 0; base < count; base += 64) {
    const int k = base + lane;
    const int st = k < count ? entry_start<FIELD>(t[k]) : 0x7fffffff;
    n_le += __popcll(__ballot(st <= idx));
  }
  return n_le - 1;
}

// Fixed-order sum of nrb row-block partials of one column (stride m): eight independent
// accumulators keep eight loads in flight, so the largest matrix (n = 1792: 112 partials)
// no longer serialises ~100 dependent L2/MALL round trips on the few waves that own it.
__device__ __forceinline__ float sum_partials(const float* __restrict__ part, int nrb, long m) {
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = 0;
  for (; r + 8 <= nrb; r += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += part[(long)(r + k) * m];
  }
  for (int k = 0; r < nrb; ++r, ++k) s[k] += part[(long)r * m];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// K = softmax(raw / tau, -1) * m (manifold_layers.py:56-57); a_0 = b_0 = 1.
__global__ void __launch_bounds__(256) sk_init(const hv_sinkhorn_entry* __restrict__ tab,
                                               int count, int total_rows, int small_max) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const hv_sinkhorn_entry e = tab[find_entry_wave<0>(tab, count, g)];
  if (sk_is_small(e, small_max)) return;
  const int row = g - e.row_start;               // row within batch*n
  const float* src = e.raw + (long)row * e.m;
  float* dst = e.out + (long)row * e.m;
  const float inv_tau = 1.0f / e.tau;
  float mx = -INFINITY;
  for (int j = lane; j < e.m; j += 64) mx = fmaxf(mx, src[j] * inv_tau);
  mx = wave_max(mx);
  float s = 0.f;
  for (int j = lane; j < e.m; j += 64) s += __expf(src[j] * inv_tau - mx);
  s = wave_sum(s);
  const float k = (float)e.m / s;
  for (int j = lane; j < e.m; j += 64) dst[j] = __expf(src[j] * inv_tau - mx) * k;
  Work w = carve(e);
  if (lane == 0) w.a[row] = 1.0f;
}

__global__ void __launch_bounds__(256) sk_init_cols(const hv_sinkhorn_entry* __restrict__ tab,
                                                    int count, int total_cols, int small_max) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  const int w0 = g & ~63;
  if (w0 >= total_cols) return;                  // wave-uniform
  const int gl = g < total_cols ? g : total_cols - 1;
  const hv_sinkhorn_entry e = tab[find_entry_span<2>(tab, count, gl, w0, min(w0 + 63, total_cols - 1))];
  if (g >= total_cols || sk_is_small(e, small_max)) return;
  carve(e).b[g - e.col_start] = 1.0f;
}

// Iteration t, pass 1: row dots -> r_t, a_t+1 ; column partial sums of a_t+1 (.) K.
__global__ void __launch_bounds__(256) sk_rows(const hv_sinkhorn_entry* __restrict__ tab,
                                               int count, int t, int small_max) {
  __shared__ float colpart[4][64 * MAXQ];
  const hv_sinkhorn_entry e = tab[find_entry_wave<1>(tab, count, blockIdx.x)];
  if (t >= e.iters || sk_is_small(e, small_max)) return;
  const Work w = carve(e);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nrb = (e.n + RB - 1) / RB;
  const int lb = blockIdx.x - e.row_block_start;  // local row block
  const int bidx = lb / nrb, rb = lb % nrb;
  HV_DCHECK(lb >= 0 && bidx < e.batch && e.m <= 64 * MAXQ);
  const int m = e.m, n = e.n;
  const int nq = (m + 63) >> 6;
  const float* K = e.out + (long)bidx * n * m;
  const float* bt = w.b + (long)t * e.batch * m + (long)bidx * m;
  const float* at = w.a + (long)t * e.batch * n + (long)bidx * n;
  float* an = w.a + (long)(t + 1) * e.batch * n + (long)bidx * n;
  float* rt = w.r + (long)t * e.batch * n + (long)bidx * n;

  // all RB/4 rows of this wave are loaded before any reduction: one memory round trip per
  // pass instead of one per row (the row pass is latency-bound: 21 launches per forward)
  constexpr int RW = RB / 4;
  const int i0 = rb * RB + wv * RW;
  float bq[MAXQ], acc[MAXQ], kv[RW][MAXQ];
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int j = lane + 64 * q;
    bq[q] = (q < nq && j < m) ? bt[j] : 0.f;
    acc[q] = 0.f;
  }
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    const float* Ki = K + (long)(i0 + rr) * m;
    const bool ok = i0 + rr < n;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int j = lane + 64 * q;
      kv[rr][q] = (ok && q < nq && j < m) ? Ki[j] : 0.f;
    }
  }
  float dot[RW], ar[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) ar[rr] = i0 + rr < n ? at[i0 + rr] : 0.f;
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    dot[rr] = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) dot[rr] += kv[rr][q] * bq[q];
  }
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) dot[rr] = wave_sum(dot[rr]);
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    const int i = i0 + rr;
    if (i >= n) break;
    const float ai = ar[rr];
    const float r = ai * dot[rr];
    const float a1 = ai / (r + e.eps);
    if (lane == 0) { rt[i] = r; an[i] = a1; }
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) acc[q] += a1 * kv[rr][q];
  }
#pragma unroll
  for (int q = 0; q < MAXQ; ++q)
    if (q < nq) colpart[wv][lane + 64 * q] = acc[q];
  __syncthreads();
  float* part = w.part + ((long)bidx * nrb + rb) * m;
  for (int j = threadIdx.x; j < m; j += 256)
    part[j] = (colpart[0][j] + colpart[1][j]) + (colpart[2][j] + colpart[3][j]);
}

// Iteration t, pass 2: c_t = b_t (.) sum(partials); b_t+1 = b_t / (c_t + eps).  A block owns 64
// consecutive columns; its 4 waves sum interleaved quarters of the nrb partial rows (8 loads in
// flight each), combined in a fixed order through LDS.
__global__ void __launch_bounds__(256) sk_cols(const hv_sinkhorn_entry* __restrict__ tab,
                                               int count, int total_cols, int t, int small_max) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g0 = blockIdx.x * 64;                // < total_cols by the grid
  const int g = g0 + lane;
  const int gl = g < total_cols ? g : total_cols - 1;
  const hv_sinkhorn_entry e = tab[find_entry_span<2>(tab, count, gl, g0, min(g0 + 63, total_cols - 1))];
  const bool live = g < total_cols && t < e.iters && !sk_is_small(e, small_max);
  float s = 0.f, bprev = 0.f;
  int c = 0;
  const long bm = (long)e.batch * e.m;
  if (live) {
    c = g - e.col_start;                     // within batch*m
    HV_DCHECK(c >= 0 && c < e.batch * e.m);
    if (wv == 0) bprev = carve(e).b[(long)t * bm + c];   // issued before the partial sums
    const int bidx = c / e.m, j = c % e.m;
    const int nrb = (e.n + RB - 1) / RB;
    const float* part = carve(e).part + (long)bidx * nrb * e.m + j;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int r = wv, k = 0;
    for (; r + 28 < nrb; r += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += part[(long)(r + 4 * u) * e.m];
    }
    for (; r < nrb; r += 4, k = (k + 1) & 7) acc[k] += part[(long)r * e.m];
    s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv != 0 || !live) return;
  s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  const float cs = bprev * s;
  carve(e).b[(long)(t + 1) * bm + c] = bprev / (cs + e.eps);
}

// M = diag(a_T) K diag(b_T) in place; history[t] = |mean_i r_t,i - 1| (:76-77).
__global__ void __launch_bounds__(256) sk_final(const hv_sinkhorn_entry* __restrict__ tab,
                                                int count, int total_rows, int small_max) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const hv_sinkhorn_entry e = tab[find_entry_wave<0>(tab, count, g)];
  if (sk_is_small(e, small_max)) return;
  const Work w = carve(e);
  const int row = g - e.row_start;
  const int bidx = row / e.n;
  const long bn = (long)e.batch * e.n, bm = (long)e.batch * e.m;
  const float ai = w.a[(long)e.iters * bn + row];
  const float* bT = w.b + (long)e.iters * bm + (long)bidx * e.m;
  float* M = e.out + (long)row * e.m;
  for (int j = lane; j < e.m; j += 64) M[j] = ai * M[j] * bT[j];
  if (e.history) {                         // history[t] reduced by the wave of row t (row 0 used
    for (int t = row; t < e.iters; t += (int)bn) {   // to do all of them: a ~160 us serial tail)
      const float* rt = w.r + (long)t * bn;
      float s = 0.f;
      for (long i = lane; i < bn; i += 64) s += rt[i];
      s = wave_sum(s);
      if (lane == 0) e.history[t] = fabsf(s / (float)bn - 1.0f);
    }
  }
}


// ---- one workgroup per small entry (n, m <= 256): thread (tr, tc) of a 32 x 32 grid (1,024
// threads) holds K rows tr + 32 i, columns tc + 32 j in registers (R x R, R <= 8) for all
// iterations.  Row dots reduce over the 32 lanes of a row group (xor shuffles), column sums over
// the 32 row groups through LDS in a fixed order -- deterministic.  Writes the same a/b/r
// history as the grouped passes (the backward reads it) and M / convergence_history.
constexpr int SKG = 32;                    // thread grid side
template <int R, bool FULL>
__device__ __forceinline__ void sk_small_body(const hv_sinkhorn_entry& e, float* sm) {
  const int t = threadIdx.x, tr = t / SKG, tc = t % SKG;
  const int n = e.n, m = e.m, iters = e.iters;
  const Work w = carve(e);
  float* bl = sm;                        // [256] current b
  float* al = sm + 256;                  // [256] current a
  float* part = sm + 512;                // [SKG][256] column partials
  float* rh = sm + 512 + SKG * 256;      // [iters][256] row sums (history)
  float kv[R][R];
  const float inv_tau = 1.0f / e.tau;
  // K = softmax(raw / tau, -1) * m
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = tr + SKG * i;
    const bool rv = FULL || row < n;
    float x[R];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int col = tc + SKG * j;
      x[j] = (rv && (FULL || col < m)) ? e.raw[(long)row * m + col] * inv_tau : -INFINITY;
      mx = fmaxf(mx, x[j]);
    }
#pragma unroll
    for (int o = SKG / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      x[j] = (rv && (FULL || tc + SKG * j < m)) ? __expf(x[j] - mx) : 0.f;
      sum += x[j];
    }
#pragma unroll
    for (int o = SKG / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    const float k = rv ? (float)m / sum : 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) kv[i][j] = rv ? x[j] * k : 0.f;
  }
  if (t < m) { bl[t] = 1.0f; w.b[t] = 1.0f; }
  if (t < n) { al[t] = 1.0f; w.a[t] = 1.0f; }
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    // rows: r_i = a_i (K b)_i ; a_i <- a_i / (r_i + eps)
    float bj[R];
#pragma unroll
    for (int j = 0; j < R; ++j) bj[j] = (FULL || tc + SKG * j < m) ? bl[tc + SKG * j] : 0.f;
    float anew[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) d += kv[i][j] * bj[j];
#pragma unroll
      for (int o = SKG / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      const int row = tr + SKG * i;
      const float ai = (FULL || row < n) ? al[row] : 0.f;
      const float r = ai * d;
      anew[i] = (FULL || row < n) ? ai / (r + e.eps) : 0.f;
      if (tc == 0 && (FULL || row < n)) {
        rh[it * 256 + row] = r;
        w.r[(long)it * n + row] = r;
        w.a[(long)(it + 1) * n + row] = anew[i];
      }
    }
    __syncthreads();                       // every read of al / bl of this iteration done
    // columns: partial over this thread's rows of a_new (.) K
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float c = 0.f;
#pragma unroll
      for (int i = 0; i < R; ++i) c += anew[i] * kv[i][j];
      if (FULL || tc + SKG * j < m) part[tr * 256 + tc + SKG * j] = c;
    }
    if (tc == 0) {
#pragma unroll
      for (int i = 0; i < R; ++i)
        if (FULL || tr + SKG * i < n) al[tr + SKG * i] = anew[i];
    }
    __syncthreads();
    if (t < m) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < SKG; ++g) s += part[g * 256 + t];
      const float b = bl[t];
      const float c = b * s;
      const float bn = b / (c + e.eps);
      bl[t] = bn;
      w.b[(long)(it + 1) * m + t] = bn;
    }
    __syncthreads();
  }
  // M = diag(a_T) K diag(b_T)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = tr + SKG * i;
    if (!FULL && row >= n) continue;
    const float ai = al[row];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int col = tc + SKG * j;
      if (FULL || col < m) e.out[(long)row * m + col] = ai * kv[i][j] * bl[col];
    }
  }
  // history[t] = |mean_i r_t,i - 1| (fixed-order sum)
  if (e.history && t < iters) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += rh[t * 256 + i];
    e.history[t] = fabsf(s / (float)n - 1.0f);
  }
}

__global__ void __launch_bounds__(1024) sk_small(const hv_sinkhorn_entry* __restrict__ tab, int count, int small_max) {
  extern __shared__ float sk_sm[];
  const hv_sinkhorn_entry e = tab[blockIdx.x];
  if (!sk_is_small(e, small_max)) return;
  const int mx = e.n > e.m ? e.n : e.m;
  // FULL: n == m == 32 R (the model's D = 32, 64, 128, 256) -- no bounds masks, which keeps the
  // R = 8 body (64 K values per thread) inside the 128 VGPRs of a 1,024-thread workgroup
  const bool full = e.n == e.m && (e.n == 32 || e.n == 64 || e.n == 128 || e.n == 256);
  if (mx <= 32) { if (full) sk_small_body<1, true>(e, sk_sm); else sk_small_body<1, false>(e, sk_sm); }
  else if (mx <= 64) { if (full) sk_small_body<2, true>(e, sk_sm); else sk_small_body<2, false>(e, sk_sm); }
  else if (mx <= 128) { if (full) sk_small_body<4, true>(e, sk_sm); else sk_small_body<4, false>(e, sk_sm); }
  else { if (full) sk_small_body<8, true>(e, sk_sm); else sk_small_body<8, false>(e, sk_sm); }
}

}  // namespace

extern "C" size_t hv_sinkhorn_work_floats(int batch, int n, int m, int iters) {
  const size_t bn = (size_t)batch * n, bm = (size_t)batch * m;
  const size_t nrb = (size_t)(n + RB - 1) / RB;
  return (size_t)(iters + 1) * bn + (size_t)(iters + 1) * bm + (size_t)iters * bn +
         (size_t)batch * nrb * m;
}

namespace {
size_t sk_small_lds(int max_iters) {
  // the small entries: one workgroup each, every iteration inside (LDS: a, b, partials, history)
  return (size_t)(512 + SKG * 256 + (max_iters > 0 ? max_iters : 1) * 256) * sizeof(float);
}

int sk_launch_small(const hv_sinkhorn_entry* tab, int count, int max_iters, hipStream_t s) {
  const size_t lds = sk_small_lds(max_iters);
  if (lds > 160 * 1024) return HV_EUNSUPPORTED;
  static std::once_flag attr;
  std::call_once(attr, [] {
    (void)hipFuncSetAttribute((const void*)sk_small, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  sk_small<<<count, 1024, lds, s>>>(tab, count, 256);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// sm: entries up to sm x sm (batch 1) are the single-workgroup kernel's and skipped here; 0 = none
int sk_launch_large(const hv_sinkhorn_entry* tab, int count, int total_rows, int total_row_blocks, int total_cols,
                    int max_iters, hipStream_t s, int sm = 256) {
  sk_init<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows, sm);
  sk_init_cols<<<hv_cdiv(total_cols, 256), 256, 0, s>>>(tab, count, total_cols, sm);
  HV_CHECK_LAUNCH();
  for (int t = 0; t < max_iters; ++t) {
    sk_rows<<<total_row_blocks, 256, 0, s>>>(tab, count, t, sm);
    sk_cols<<<hv_cdiv(total_cols, 64), 256, 0, s>>>(tab, count, total_cols, t, sm);
  }
  HV_CHECK_LAUNCH();
  sk_final<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows, sm);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
}  // namespace

extern "C" int hv_sinkhorn_group_forward(const hv_sinkhorn_entry* tab, int count, int total_rows,
                                         int total_row_blocks, int total_cols, int max_iters,
                                         hv_stream_t stream) {
  return hv_sinkhorn_group_forward_part(tab, count, total_rows, total_row_blocks, total_cols, max_iters, 0, stream);
}

extern "C" int hv_sinkhorn_group_forward_part(const hv_sinkhorn_entry* tab, int count, int total_rows,
                                              int total_row_blocks, int total_cols, int max_iters, int part,
                                              hv_stream_t stream) {
  if (!tab || count <= 0 || total_rows <= 0 || max_iters < 0 || part < 0 || part > 2) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hv_diag_count(HV_KF_SINKHORN_GROUP);
  // more iterations than the single-workgroup kernel's LDS history holds: part 0 runs every
  // entry through the grouped passes instead; part 1 (small entries alone) cannot
  const bool small_fits = sk_small_lds(max_iters) <= 160 * 1024;
  if (part == 0 && !small_fits)
    return sk_launch_large(tab, count, total_rows, total_row_blocks, total_cols, max_iters, s, 0);
  if (part != 2) {
    const int rc = sk_launch_small(tab, count, max_iters, s);
    if (rc != HV_OK) return rc;
  }
  if (part != 1) return sk_launch_large(tab, count, total_rows, total_row_blocks, total_cols, max_iters, s);
  return HV_OK;
}

extern "C" int hv_sinkhorn_small_max_iters(void) {
  int it = 1;
  while (sk_small_lds(it + 1) <= 160 * 1024) ++it;
  return it;
}


// ============================================================================ backward
// Reverse-mode through every step (autograd of manifold_layers.py:56-73), G = dL/dM kept
// dense in `draw`.  With M after the column step of iteration t = diag(a_t+1) K diag(b_t+1)
// and 1/(c_t + eps) = b_t+1 / b_t, 1/(r_t + eps) = a_t+1 / a_t (forward identities):
//   column step:  s_j = b_t+1,j sum_i G_ij a_t+1,i K_ij ;  G_ij <- (G_ij - s_j) b_t+1,j / b_t,j
//   row step:     s_i = a_t+1,i sum_j G_ij K_ij b_t,j   ;  G_ij <- (G_ij - s_i) a_t+1,i / a_t,i
//   softmax:      draw_ij = K_ij (G_ij - sum_j' G_ij' K_ij' / m) / tau
// One fused row pass per iteration (column-step update, row step, next column partials) +
// one column reduce, like the forward.
namespace {

struct BWork {
  float* K;      // [batch*n, m]
  float* part;   // [batch, nrb, m]
  float* s;      // [batch*m]
};
__device__ __forceinline__ BWork bcarve(const hv_sinkhorn_bwd_entry& e) {
  BWork w;
  const long bn = (long)e.fwd.batch * e.fwd.n, bm = (long)e.fwd.batch * e.fwd.m;
  const long nrb = (e.fwd.n + RB - 1) / RB;
  w.K = e.bwork;
  w.part = w.K + bn * e.fwd.m;
  w.s = w.part + (long)e.fwd.batch * nrb * e.fwd.m;
  (void)bm;
  return w;
}

template <int FIELD>
__device__ __forceinline__ int find_bentry(const hv_sinkhorn_bwd_entry* t, int count, int idx) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    int s = FIELD == 0 ? t[mid].fwd.row_start : (FIELD == 1 ? t[mid].fwd.row_block_start : t[mid].fwd.col_start);
    if (s <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// K = softmax(raw/tau)*m into bwork; G = dout into draw.
__global__ void __launch_bounds__(256) skb_init(const hv_sinkhorn_bwd_entry* __restrict__ tab, int count,
                                                int total_rows) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const hv_sinkhorn_bwd_entry e = tab[find_bentry<0>(tab, count, g)];
  const int row = g - e.fwd.row_start, m = e.fwd.m;
  const float* src = e.fwd.raw + (long)row * m;
  const BWork w = bcarve(e);
  float* K = w.K + (long)row * m;
  const float inv_tau = 1.0f / e.fwd.tau;
  float mx = -INFINITY;
  for (int j = lane; j < m; j += 64) mx = fmaxf(mx, src[j] * inv_tau);
  mx = wave_max(mx);
  float s = 0.f;
  for (int j = lane; j < m; j += 64) s += __expf(src[j] * inv_tau - mx);
  s = wave_sum(s);
  const float k = (float)m / s;
  for (int j = lane; j < m; j += 64) {
    K[j] = __expf(src[j] * inv_tau - mx) * k;
    e.draw[(long)row * m + j] = e.dout[(long)row * m + j];
  }
}

// column partials of G (.) a_{t+1} (.) K for the column step of iteration t = iters-1
__global__ void __launch_bounds__(256) skb_colpart0(const hv_sinkhorn_bwd_entry* __restrict__ tab, int count) {
  const hv_sinkhorn_bwd_entry e = tab[find_bentry<1>(tab, count, blockIdx.x)];
  if (e.fwd.iters <= 0) return;
  const int n = e.fwd.n, m = e.fwd.m, t = e.fwd.iters - 1;
  const int nrb = (n + RB - 1) / RB;
  const int lb = blockIdx.x - e.fwd.row_block_start;
  const int bidx = lb / nrb, rb = lb % nrb;
  const Work fw = carve(e.fwd);
  const BWork w = bcarve(e);
  const float* a1 = fw.a + (long)(t + 1) * e.fwd.batch * n + (long)bidx * n;
  float* part = w.part + ((long)bidx * nrb + rb) * m;
  for (int j = threadIdx.x; j < m; j += 256) {
    float acc = 0.f;
    for (int r = 0; r < RB; ++r) {
      const int i = rb * RB + r;
      if (i >= n) break;
      const long o = ((long)bidx * n + i) * m + j;
      acc += e.draw[o] * a1[i] * w.K[o];
    }
    part[j] = acc;
  }
}

// s_j = b_{t+1,j} * sum over row blocks
__global__ void __launch_bounds__(256) skb_cols(const hv_sinkhorn_bwd_entry* __restrict__ tab, int count,
                                                int total_cols, int t) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= total_cols) return;
  const hv_sinkhorn_bwd_entry e = tab[find_bentry<2>(tab, count, g)];
  if (t >= e.fwd.iters) return;
  const Work fw = carve(e.fwd);
  const BWork w = bcarve(e);
  const int c = g - e.fwd.col_start;
  const int bidx = c / e.fwd.m, j = c % e.fwd.m;
  const int nrb = (e.fwd.n + RB - 1) / RB;
  const float* part = w.part + (long)bidx * nrb * e.fwd.m + j;
  float s = 0.f;
  s += sum_partials(part, nrb, e.fwd.m);
  const long bm = (long)e.fwd.batch * e.fwd.m;
  w.s[c] = fw.b[(long)(t + 1) * bm + c] * s;
}

// fused: column-step update (iteration t), row step (iteration t), next column partials (t-1)
__global__ void __launch_bounds__(256) skb_rows(const hv_sinkhorn_bwd_entry* __restrict__ tab, int count, int t) {
  __shared__ float bt_s[64 * MAXQ];
  __shared__ float cf_s[64 * MAXQ];
  __shared__ float sj_s[64 * MAXQ];
  __shared__ float colpart[4][64 * MAXQ];
  const hv_sinkhorn_bwd_entry e = tab[find_bentry<1>(tab, count, blockIdx.x)];
  if (t >= e.fwd.iters) return;
  const int n = e.fwd.n, m = e.fwd.m;
  const int nrb = (n + RB - 1) / RB;
  const int lb = blockIdx.x - e.fwd.row_block_start;
  const int bidx = lb / nrb, rb = lb % nrb;
  const Work fw = carve(e.fwd);
  const BWork w = bcarve(e);
  const long bn = (long)e.fwd.batch * n, bm = (long)e.fwd.batch * m;
  const float* bt = fw.b + (long)t * bm + (long)bidx * m;
  const float* bt1 = fw.b + (long)(t + 1) * bm + (long)bidx * m;
  const float* at = fw.a + (long)t * bn + (long)bidx * n;
  const float* at1 = fw.a + (long)(t + 1) * bn + (long)bidx * n;
  const float* sj = w.s + (long)bidx * m;
  for (int j = threadIdx.x; j < m; j += 256) {
    bt_s[j] = bt[j];
    cf_s[j] = bt1[j] / bt[j];
    sj_s[j] = sj[j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nq = (m + 63) >> 6;
  float acc[MAXQ];
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) acc[q] = 0.f;
  for (int rr = 0; rr < RB / 4; ++rr) {
    const int i = rb * RB + wv * (RB / 4) + rr;
    if (i >= n) break;
    const long ro = ((long)bidx * n + i) * m;
    float gq[MAXQ], kq[MAXQ];
    float dot = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int j = lane + 64 * q;
      gq[q] = 0.f; kq[q] = 0.f;
      if (q < nq && j < m) {
        kq[q] = w.K[ro + j];
        gq[q] = (e.draw[ro + j] - sj_s[j]) * cf_s[j];          // column-step backward
        dot += gq[q] * kq[q] * bt_s[j];
      }
    }
    dot = wave_sum(dot);
    const float a1 = at1[i];
    const float si = a1 * dot;
    const float rf = a1 / at[i];
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int j = lane + 64 * q;
      if (q < nq && j < m) {
        const float gn = (gq[q] - si) * rf;                  // row-step backward
        e.draw[ro + j] = gn;
        acc[q] += gn * at[i] * kq[q];                        // partial for column step t-1
      }
    }
  }
  if (t == 0) return;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q)
    if (q < nq) colpart[wv][lane + 64 * q] = acc[q];
  __syncthreads();
  float* part = w.part + ((long)bidx * nrb + rb) * m;
  for (int j = threadIdx.x; j < m; j += 256)
    part[j] = (colpart[0][j] + colpart[1][j]) + (colpart[2][j] + colpart[3][j]);
}

// softmax backward: draw = K (G - rowdot(G, K)/m) / tau
__global__ void __launch_bounds__(256) skb_final(const hv_sinkhorn_bwd_entry* __restrict__ tab, int count,
                                                 int total_rows) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const hv_sinkhorn_bwd_entry e = tab[find_bentry<0>(tab, count, g)];
  const int row = g - e.fwd.row_start, m = e.fwd.m;
  const BWork w = bcarve(e);
  const float* K = w.K + (long)row * m;
  float* G = e.draw + (long)row * m;
  float d = 0.f;
  for (int j = lane; j < m; j += 64) d += G[j] * K[j];
  d = wave_sum(d) / (float)m;
  const float it = 1.0f / e.fwd.tau;
  for (int j = lane; j < m; j += 64) G[j] = K[j] * (G[j] - d) * it;
}

}  // namespace

extern "C" size_t hv_sinkhorn_bwd_work_floats(int batch, int n, int m) {
  const size_t nrb = (size_t)(n + RB - 1) / RB;
  return (size_t)batch * n * m + (size_t)batch * nrb * m + (size_t)batch * m;
}

extern "C" int hv_sinkhorn_group_backward(const hv_sinkhorn_bwd_entry* tab, int count, int total_rows,
                                          int total_row_blocks, int total_cols, int max_iters, hv_stream_t stream) {
  if (!tab || count <= 0 || total_rows <= 0 || max_iters < 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  skb_init<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows);
  if (max_iters > 0) skb_colpart0<<<total_row_blocks, 256, 0, s>>>(tab, count);
  HV_CHECK_LAUNCH();
  // entries with fewer iterations join the reverse sweep when t < their iters; their first
  // column partials come from skb_colpart0, later ones from the fused row pass
  for (int t = max_iters - 1; t >= 0; --t) {
    skb_cols<<<hv_cdiv(total_cols, 256), 256, 0, s>>>(tab, count, total_cols, t);
    skb_rows<<<total_row_blocks, 256, 0, s>>>(tab, count, t);
  }
  HV_CHECK_LAUNCH();
  skb_final<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_abi_version(void) { return HV_ABI_VERSION; }
extern "C" void hv_struct_sizes(int* out5) {
  out5[0] = (int)sizeof(hv_sinkhorn_entry);
  out5[1] = (int)sizeof(hv_gemm_desc);
  out5[2] = (int)sizeof(hv_mhc_fused_args);
  out5[3] = (int)sizeof(hv_mhc_prep_entry);
  out5[4] = (int)sizeof(hv_wprep_entry);
}
