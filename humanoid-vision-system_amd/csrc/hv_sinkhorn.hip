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

// Find the entry whose [start, start+len) range contains idx (entries sorted by start).
template <int FIELD>
__device__ __forceinline__ int find_entry(const hv_sinkhorn_entry* t, int count, int idx) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    int s = FIELD == 0 ? t[mid].row_start : (FIELD == 1 ? t[mid].row_block_start : t[mid].col_start);
    if (s <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
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
                                               int count, int total_rows) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const int ei = find_entry<0>(tab, count, g);
  const hv_sinkhorn_entry e = tab[ei];
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
                                                    int count, int total_cols) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= total_cols) return;
  const hv_sinkhorn_entry e = tab[find_entry<2>(tab, count, g)];
  carve(e).b[g - e.col_start] = 1.0f;
}

// Iteration t, pass 1: row dots -> r_t, a_t+1 ; column partial sums of a_t+1 (.) K.
__global__ void __launch_bounds__(256) sk_rows(const hv_sinkhorn_entry* __restrict__ tab,
                                               int count, int t) {
  __shared__ float colpart[4][64 * MAXQ];
  const int ei = find_entry<1>(tab, count, blockIdx.x);
  const hv_sinkhorn_entry e = tab[ei];
  if (t >= e.iters) return;
  const Work w = carve(e);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nrb = (e.n + RB - 1) / RB;
  const int lb = blockIdx.x - e.row_block_start;  // local row block
  const int bidx = lb / nrb, rb = lb % nrb;
  const int m = e.m, n = e.n;
  const int nq = (m + 63) >> 6;
  const float* K = e.out + (long)bidx * n * m;
  const float* bt = w.b + (long)t * e.batch * m + (long)bidx * m;
  const float* at = w.a + (long)t * e.batch * n + (long)bidx * n;
  float* an = w.a + (long)(t + 1) * e.batch * n + (long)bidx * n;
  float* rt = w.r + (long)t * e.batch * n + (long)bidx * n;

  float bq[MAXQ], acc[MAXQ];
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int j = lane + 64 * q;
    bq[q] = (q < nq && j < m) ? bt[j] : 0.f;
    acc[q] = 0.f;
  }
  for (int rr = 0; rr < RB / 4; ++rr) {
    const int i = rb * RB + wv * (RB / 4) + rr;
    if (i >= n) break;
    const float* Ki = K + (long)i * m;
    float kv[MAXQ];
    float dot = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int j = lane + 64 * q;
      kv[q] = (q < nq && j < m) ? Ki[j] : 0.f;
      dot += kv[q] * bq[q];
    }
    dot = wave_sum(dot);
    const float ai = at[i];
    const float r = ai * dot;
    const float a1 = ai / (r + e.eps);
    if (lane == 0) { rt[i] = r; an[i] = a1; }
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) acc[q] += a1 * kv[q];
  }
#pragma unroll
  for (int q = 0; q < MAXQ; ++q)
    if (q < nq) colpart[wv][lane + 64 * q] = acc[q];
  __syncthreads();
  float* part = w.part + ((long)bidx * nrb + rb) * m;
  for (int j = threadIdx.x; j < m; j += 256)
    part[j] = (colpart[0][j] + colpart[1][j]) + (colpart[2][j] + colpart[3][j]);
}

// Iteration t, pass 2: c_t = b_t (.) sum(partials); b_t+1 = b_t / (c_t + eps).
__global__ void __launch_bounds__(256) sk_cols(const hv_sinkhorn_entry* __restrict__ tab,
                                               int count, int total_cols, int t) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= total_cols) return;
  const int ei = find_entry<2>(tab, count, g);
  const hv_sinkhorn_entry e = tab[ei];
  if (t >= e.iters) return;
  const Work w = carve(e);
  const int c = g - e.col_start;           // within batch*m
  const int bidx = c / e.m, j = c % e.m;
  const int nrb = (e.n + RB - 1) / RB;
  const float* part = w.part + (long)bidx * nrb * e.m + j;
  const float s = sum_partials(part, nrb, e.m);
  const long bm = (long)e.batch * e.m;
  const float b = w.b[(long)t * bm + c];
  const float cs = b * s;
  w.b[(long)(t + 1) * bm + c] = b / (cs + e.eps);
}

// M = diag(a_T) K diag(b_T) in place; history[t] = |mean_i r_t,i - 1| (:76-77).
__global__ void __launch_bounds__(256) sk_final(const hv_sinkhorn_entry* __restrict__ tab,
                                                int count, int total_rows) {
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= total_rows) return;
  const int ei = find_entry<0>(tab, count, g);
  const hv_sinkhorn_entry e = tab[ei];
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

}  // namespace

extern "C" size_t hv_sinkhorn_work_floats(int batch, int n, int m, int iters) {
  const size_t bn = (size_t)batch * n, bm = (size_t)batch * m;
  const size_t nrb = (size_t)(n + RB - 1) / RB;
  return (size_t)(iters + 1) * bn + (size_t)(iters + 1) * bm + (size_t)iters * bn +
         (size_t)batch * nrb * m;
}

extern "C" int hv_sinkhorn_group_forward(const hv_sinkhorn_entry* tab, int count, int total_rows,
                                         int total_row_blocks, int total_cols, int max_iters,
                                         hv_stream_t stream) {
  hv_diag_count(HV_KF_SINKHORN_GROUP);
  if (!tab || count <= 0 || total_rows <= 0 || max_iters < 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  sk_init<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows);
  sk_init_cols<<<hv_cdiv(total_cols, 256), 256, 0, s>>>(tab, count, total_cols);
  HV_CHECK_LAUNCH();
  for (int t = 0; t < max_iters; ++t) {
    sk_rows<<<total_row_blocks, 256, 0, s>>>(tab, count, t);
    sk_cols<<<hv_cdiv(total_cols, 256), 256, 0, s>>>(tab, count, total_cols, t);
  }
  HV_CHECK_LAUNCH();
  sk_final<<<hv_cdiv(total_rows, 4), 256, 0, s>>>(tab, count, total_rows);
  HV_CHECK_LAUNCH();
  return HV_OK;
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

extern "C" int hv_abi_version(void) { return 1; }
extern "C" void hv_struct_sizes(int* out5) {
  out5[0] = (int)sizeof(hv_sinkhorn_entry);
  out5[1] = (int)sizeof(hv_gemm_desc);
  out5[2] = (int)sizeof(hv_mhc_fused_args);
  out5[3] = (int)sizeof(hv_mhc_prep_entry);
  out5[4] = (int)sizeof(hv_wprep_entry);
}
