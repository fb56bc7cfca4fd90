// Stability monitor of the mHC sites (reference src/models/manifold_layers.py:282-316,
// ManifoldHyperConnection._monitor_stability): eigenvalues of the symmetric part of every
// H_res, the signal-growth ratio and the row/column-sum errors -- on the device, grouped over
// all sites, no host sync.
//
// Eigenvalues (torch.linalg.eigvalsh((H + H^T) / 2), :288-290) as a two-phase symmetric
// eigensolver in fp64 (the matrices are fp32; fp64 keeps the result at fp32 resolution for
// n = 1792, where an fp32 reduction would lose ~n*eps):
//   1. Householder tridiagonalisation (the dsytd2 recurrence).  Step k reflects column k below
//      the diagonal: v_k (v_k[k+1] = 1), tau_k, e_k = beta; p = tau B v, w = p - (tau/2)(p.v) v,
//      B -= v w^T + w v^T on the trailing block B = A[k+1:, k+1:].  The rank-2 update of step k
//      is applied LAZILY inside step k+1's pass: one read + one write of the trailing block per
//      step (the eager form reads it twice).  Two launches per step for the whole table:
//        sye_hh   one workgroup per active matrix: w_{k-1} from p_{k-1}; row k (= column k,
//                 symmetric) with the pending update applied; the reflector of step k
//        sye_symv one wave per trailing row of every active matrix: apply update k-1 to the
//                 row (stored), accumulate the row's dot with v_k -> p_k
//   2. Bisection on the tridiagonal T (d, e) with Sturm counts (the dstebz recurrence, pivmin
//      guard), one lane per eigenvalue, (d, e^2) in LDS.  The j-th lane's result is the j-th
//      smallest eigenvalue, so the output is ascending like eigvalsh.
// Matrices sort by n descending on the host: the active matrices of step k are then a prefix
// of the table and their trailing-row prefix sums are S_i - i*(k+1) (S = prefix of n).
#include <float.h>

#include "hv_common.h"

namespace {

constexpr int SYE_MAXN = 2048;
constexpr int SYE_PER = SYE_MAXN / 256;   // column elements per thread in sye_hh

struct EigWork {
  double *A, *v, *w, *p, *d, *e, *e2, *scal;   // scal: tau[2] (step parity), gl, gu, pivmin
};
__device__ __forceinline__ EigWork eig_carve(const hv_symeig_entry& t) {
  EigWork w;
  const long n = t.n;
  w.A = t.work;
  w.v = w.A + n * n;          // 2 * n (parity of the step)
  w.w = w.v + 2 * n;
  w.p = w.w + n;
  w.d = w.p + n;
  w.e = w.d + n;
  w.e2 = w.e + n;
  w.scal = w.e2 + n;
  return w;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// 256-thread block sum; scratch: 4 doubles of LDS.  All threads get the total.
__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) scratch[wv] = v;
  __syncthreads();
  return (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
}

// A = (h + h^T) / 2 in fp64.  grid (x, count), block 256.
__global__ void __launch_bounds__(256) sye_init(const hv_symeig_entry* __restrict__ tab) {
  const hv_symeig_entry t = tab[blockIdx.y];
  const int n = t.n;
  double* A = t.work;
  const long nn = (long)n * n;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < nn; idx += (long)gridDim.x * 256) {
    const int i = (int)(idx / n), j = (int)(idx - (long)i * n);
    A[idx] = 0.5 * ((double)t.h[idx] + (double)t.h[(long)j * n + i]);
  }
}

// Step k, one workgroup per active matrix (blockIdx.x < number of matrices with n >= k + 3).
__global__ void __launch_bounds__(256) sye_hh(const hv_symeig_entry* __restrict__ tab, int k) {
  __shared__ double red[4];
  __shared__ double x0s;
  const hv_symeig_entry t = tab[blockIdx.x];
  const int n = t.n;
  HV_DCHECK(n >= k + 3 && n <= SYE_MAXN);
  const EigWork W = eig_carve(t);
  const double* vp = W.v + (long)((k + 1) & 1) * n;   // v_{k-1}
  double* vc = W.v + (long)(k & 1) * n;               // v_k
  const int tid = threadIdx.x;
  double wk = 0.0, vk = 0.0, kc = 0.0;
  if (k >= 1) {                                       // w_{k-1} = p - (tau/2)(p.v) v over rows >= k
    double s = 0.0;
    for (int i = k + tid; i < n; i += 256) s += W.p[i] * vp[i];
    kc = 0.5 * W.scal[(k + 1) & 1] * block_sum_d(s, red);
    for (int i = k + tid; i < n; i += 256) W.w[i] = W.p[i] - kc * vp[i];
    wk = W.p[k] - kc * vp[k];
    vk = vp[k];
  }
  // row k from column k on (the pending update of step k-1 applied, never stored: row k is
  // not read again)
  double c[SYE_PER];
  double sig = 0.0;
#pragma unroll
  for (int q = 0; q < SYE_PER; ++q) {
    const int i = k + tid + q * 256;
    double a = 0.0;
    if (i < n) {
      a = W.A[(long)k * n + i];
      if (k >= 1) a -= vp[i] * wk + (W.p[i] - kc * vp[i]) * vk;
      if (i == k) W.d[k] = a;
      if (i == k + 1) x0s = a;
      if (i >= k + 2) sig += a * a;
    }
    c[q] = a;
  }
  sig = block_sum_d(sig, red);                        // its barriers also publish x0s
  const double x0 = x0s;
  double tau = 0.0, beta = x0, scale = 0.0;
  if (sig > 0.0) {
    const double nrm = sqrt(x0 * x0 + sig);
    beta = x0 >= 0.0 ? -nrm : nrm;
    tau = (beta - x0) / beta;
    scale = 1.0 / (x0 - beta);
  }
#pragma unroll
  for (int q = 0; q < SYE_PER; ++q) {
    const int i = k + tid + q * 256;
    if (i >= k + 1 && i < n) vc[i] = i == k + 1 ? (sig > 0.0 ? 1.0 : 0.0) : c[q] * scale;
  }
  if (tid == 0) {
    W.e[k] = beta;
    W.scal[k & 1] = tau;
  }
}

// Step k: one wave per trailing row i in [k+1, n) of every active matrix.
__global__ void __launch_bounds__(256) sye_symv(const hv_symeig_entry* __restrict__ tab, int active, int k,
                                                int total_rows) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= total_rows) return;
  // largest e < active with S_e - e*(k+1) <= g   (row_start = S_e)
  int lo = 0, hi = active - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].row_start - mid * (k + 1) <= g) lo = mid; else hi = mid - 1;
  }
  const hv_symeig_entry t = tab[lo];
  const int n = t.n;
  const int i = k + 1 + (g - (t.row_start - lo * (k + 1)));
  HV_DCHECK(i < n);
  const EigWork W = eig_carve(t);
  const double* vp = W.v + (long)((k + 1) & 1) * n;
  const double* vc = W.v + (long)(k & 1) * n;
  double* row = W.A + (long)i * n;
  double acc = 0.0;
  if (k >= 1) {
    const double vi = vp[i], wi = W.w[i];
    for (int j = k + 1 + lane; j < n; j += 64) {
      const double a = row[j] - (vi * W.w[j] + wi * vp[j]);
      row[j] = a;
      acc += a * vc[j];
    }
  } else {
    for (int j = 1 + lane; j < n; j += 64) acc += row[j] * vc[j];
  }
  acc = wave_sum_d(acc);
  if (lane == 0) W.p[i] = W.scal[k & 1] * acc;
}

// The last pending update (step n-3) on the trailing 2x2 block -> (d, e) complete; e^2,
// Gershgorin bounds and pivmin.  One workgroup per matrix.
__global__ void __launch_bounds__(256) sye_tail(const hv_symeig_entry* __restrict__ tab) {
  __shared__ double red[4];
  __shared__ double mn[4], mx[4];
  const hv_symeig_entry t = tab[blockIdx.x];
  const int n = t.n;
  const EigWork W = eig_carve(t);
  if (threadIdx.x == 0) {
    const double* A = W.A;
    if (n >= 3) {
      const int k = n - 3;
      const double* v = W.v + (long)(k & 1) * n;
      const double tau = W.scal[k & 1];
      const int a = n - 2, b = n - 1;
      const double kc = 0.5 * tau * (W.p[a] * v[a] + W.p[b] * v[b]);
      const double wa = W.p[a] - kc * v[a], wb = W.p[b] - kc * v[b];
      W.d[a] = A[(long)a * n + a] - 2.0 * v[a] * wa;
      W.e[a] = A[(long)b * n + a] - (v[b] * wa + wb * v[a]);
      W.d[b] = A[(long)b * n + b] - 2.0 * v[b] * wb;
    } else if (n == 2) {
      W.d[0] = A[0];
      W.e[0] = A[2];
      W.d[1] = A[3];
    } else {
      W.d[0] = A[0];
    }
  }
  __syncthreads();
  double lo = DBL_MAX, hi = -DBL_MAX, emax = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const double em = i > 0 ? fabs(W.e[i - 1]) : 0.0, ep = i < n - 1 ? fabs(W.e[i]) : 0.0;
    lo = fmin(lo, W.d[i] - em - ep);
    hi = fmax(hi, W.d[i] + em + ep);
    if (i < n - 1) {
      W.e2[i] = W.e[i] * W.e[i];
      emax = fmax(emax, W.e2[i]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { mn[wv] = lo; mx[wv] = hi; red[wv] = emax; }
  __syncthreads();
  if (threadIdx.x == 0) {
    lo = fmin(fmin(mn[0], mn[1]), fmin(mn[2], mn[3]));
    hi = fmax(fmax(mx[0], mx[1]), fmax(mx[2], mx[3]));
    emax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    const double pivmin = DBL_MIN * fmax(1.0, emax);
    const double pad = 2.0 * DBL_EPSILON * fmax(fabs(lo), fabs(hi)) + 4.0 * pivmin + 1e-300;
    W.scal[2] = lo - pad;
    W.scal[3] = hi + pad;
    W.scal[4] = pivmin;
  }
}

// Bisection: grid (ceil(maxn/256), count); lane j of an entry finds its j-th smallest eigenvalue.
__global__ void __launch_bounds__(256) sye_bisect(const hv_symeig_entry* __restrict__ tab) {
  __shared__ double sd[SYE_MAXN], se2[SYE_MAXN];
  const hv_symeig_entry t = tab[blockIdx.y];
  const int n = t.n;
  if ((int)blockIdx.x * 256 >= n) return;
  const EigWork W = eig_carve(t);
  for (int i = threadIdx.x; i < n; i += 256) {
    sd[i] = W.d[i];
    se2[i] = i < n - 1 ? W.e2[i] : 0.0;
  }
  __syncthreads();
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const double pivmin = W.scal[4];
  double lo = W.scal[2], hi = W.scal[3];
  // invariant: count(lo) <= j < count(hi), count(x) = #eigenvalues < x
  for (int it = 0; it < 128; ++it) {
    const double tol = fmax(1e-11, 1e-10 * fmax(fabs(lo), fabs(hi)));
    if (hi - lo <= tol) break;
    const double x = 0.5 * (lo + hi);
    int cnt = 0;
    double q = sd[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      q = sd[i] - x - se2[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    if (cnt > j) hi = x; else lo = x;
  }
  t.eig[j] = (float)(0.5 * (lo + hi));
}

// ---------------------------------------------------------------- signal ratio / sum errors
// partials per block: [sum_rows |x_in|, sum_rows |x_out|, sum(H) chunk]
template <typename T>
__global__ void __launch_bounds__(256) stab_partial(const T* __restrict__ xin, const T* __restrict__ xout,
                                                    int rows, int D, const float* __restrict__ h, long hn,
                                                    float* __restrict__ part) {
  __shared__ float red[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float sin_ = 0.f, sout = 0.f;
  for (int r = blockIdx.x * 4 + wv; r < rows; r += gridDim.x * 4) {
    float a = 0.f, b = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float u = Elem<T>::load(xin, (size_t)r * D + c), v = Elem<T>::load(xout, (size_t)r * D + c);
      a += u * u;
      b += v * v;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    sin_ += sqrtf(a);
    sout += sqrtf(b);
  }
  float hs = 0.f;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < hn; idx += (long)gridDim.x * 256) hs += h[idx];
  // sin_/sout are wave-uniform: one lane per wave contributes
  const float s0 = block_sum(lane == 0 ? sin_ : 0.f, red);
  const float s1 = block_sum(lane == 0 ? sout : 0.f, red);
  const float s2 = block_sum(hs, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x * 3 + 0] = s0;
    part[blockIdx.x * 3 + 1] = s1;
    part[blockIdx.x * 3 + 2] = s2;
  }
}

__global__ void __launch_bounds__(64) stab_final(const float* __restrict__ part, int nb, int rows, int n,
                                                 float* __restrict__ history, int slot, float* __restrict__ out3) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  for (int b = threadIdx.x; b < nb; b += 64) {
    s0 += part[b * 3 + 0];
    s1 += part[b * 3 + 1];
    s2 += part[b * 3 + 2];
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (threadIdx.x == 0) {
    const float ratio = (s1 / (float)rows) / (s0 / (float)rows + 1e-8f);
    const float err = fabsf(s2 / (float)n - 1.0f);
    out3[0] = ratio;
    out3[1] = err;
    out3[2] = err;
    if (history) history[slot] = ratio;
  }
}

constexpr int STAB_MAXB = 512;

}  // namespace

extern "C" size_t hv_symeig_work_doubles(int n) { return (size_t)n * n + 8 * (size_t)n + 8; }

extern "C" int hv_symeig_group(const hv_symeig_entry* dev_table, const int* host_n, int count, hv_stream_t stream) {
  if (count <= 0) return HV_OK;
  if (!dev_table || !host_n) return HV_EINVAL;
  for (int i = 0; i < count; ++i)
    if (host_n[i] < 1 || host_n[i] > SYE_MAXN || (i && host_n[i] > host_n[i - 1])) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int maxn = host_n[0];
  sye_init<<<dim3(64, count), 256, 0, s>>>(dev_table);
  HV_CHECK_LAUNCH();
  for (int k = 0; k + 3 <= maxn; ++k) {
    int active = 0;
    long rows = 0;                                  // trailing rows [k+1, n) of the active matrices
    while (active < count && host_n[active] >= k + 3) rows += host_n[active++] - k - 1;
    sye_hh<<<active, 256, 0, s>>>(dev_table, k);
    HV_CHECK_LAUNCH();
    sye_symv<<<(int)((rows + 3) / 4), 256, 0, s>>>(dev_table, active, k, (int)rows);
    HV_CHECK_LAUNCH();
  }
  sye_tail<<<count, 256, 0, s>>>(dev_table);
  HV_CHECK_LAUNCH();
  sye_bisect<<<dim3((maxn + 255) / 256, count), 256, 0, s>>>(dev_table);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_stability_work_floats(int rows) {
  (void)rows;
  return 3 * STAB_MAXB;
}

extern "C" int hv_stability_stats(int dtype, const void* x_in, const void* x_out, int rows, int D,
                                  const float* h, int n, float* work, float* history, int slot, float* out3,
                                  hv_stream_t stream) {
  if (rows <= 0 || D <= 0 || n <= 0 || !x_in || !x_out || !h || !work || !out3) return HV_EINVAL;
  if (history && (slot < 0 || slot >= 1000)) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const long hn = (long)n * n;
  int nb = (int)std::min<long>(STAB_MAXB, std::max<long>((rows + 3) / 4, (hn + 255) / 256));
  nb = std::max(nb, 1);
  if (dtype == HV_F32)
    stab_partial<float><<<nb, 256, 0, s>>>((const float*)x_in, (const float*)x_out, rows, D, h, hn, work);
  else if (dtype == HV_BF16)
    stab_partial<unsigned short><<<nb, 256, 0, s>>>((const unsigned short*)x_in, (const unsigned short*)x_out,
                                                    rows, D, h, hn, work);
  else
    return HV_EUNSUPPORTED;
  HV_CHECK_LAUNCH();
  stab_final<<<1, 64, 0, s>>>(work, nb, rows, n, history, slot, out3);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
