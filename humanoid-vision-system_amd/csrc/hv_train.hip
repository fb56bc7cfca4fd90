// Training-step kernels for gfx950: BatchNorm batch statistics and its
// backward, row-norm (LayerNorm / RMSNorm) training forward + backward with fused dropout,
// activation backward, column reductions for bias gradients, weight-operand layouts for the
// dgrad GEMMs, squeeze-excite / pooling / upsample / token-assembly backward, the fused
// YOLOLoss forward+backward, and grad-norm clipping + AdamW over a parameter table.
//
// All reductions are two-pass with a fixed order (bitwise reproducible run to run).
#include "hv_common.h"

#define HV_CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace {

template <typename T> __device__ __forceinline__ float ld(const T* p, long i);
template <> __device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ld<unsigned short>(const unsigned short* p, long i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, long i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<unsigned short>(unsigned short* p, long i, float v) { p[i] = f2bf(v); }

__device__ __forceinline__ float ld_dt(const void* p, int dt, long i) {
  return dt == HV_BF16 ? bf2f(((const unsigned short*)p)[i]) : ((const float*)p)[i];
}
__device__ __forceinline__ void st_dt(void* p, int dt, long i, float v) {
  if (dt == HV_BF16) ((unsigned short*)p)[i] = f2bf(v);
  else ((float*)p)[i] = v;
}

// ------------------------------------------------------------------ weight layouts
__global__ void k_dgrad_wprep(const float* __restrict__ w, int cout, int cin, int k, int flip, int dt, void* y) {
  const long total = (long)cout * cin * k * k;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // i over y [ci][kh][kw][co]
    const int co = (int)(i % cout);
    long r = i / cout;
    const int kw = (int)(r % k); r /= k;
    const int kh = (int)(r % k);
    const int ci = (int)(r / k);
    const int sh = flip ? k - 1 - kh : kh, sw = flip ? k - 1 - kw : kw;
    st_dt(y, dt, i, w[(((long)co * cin + ci) * k + sh) * k + sw]);
  }
}

__global__ void k_transpose_cast(const float* __restrict__ x, int rows, int cols, int dt, void* y) {
  __shared__ float tile[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int row = by + r, col = bx + tx;
    tile[r][tx] = (row < rows && col < cols) ? x[(long)row * cols + col] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int orow = bx + r, ocol = by + tx;                 // y[cols][rows]
    if (orow < cols && ocol < rows) st_dt(y, dt, (long)orow * rows + ocol, tile[tx][r]);
  }
}

// grouped transpose / cast (hv_transpose_group): 32x32 tiles of every entry of a device table;
// a block finds its entry by binary search over the entries' first blocks
__global__ void __launch_bounds__(256) k_transpose_group(const hv_transpose_entry* __restrict__ tab, int count) {
  __shared__ float tile[32][33];
  const int b = blockIdx.x;
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].blk <= b) lo = mid; else hi = mid - 1;
  }
  const hv_transpose_entry& e = tab[lo];
  const int tcols = (e.cols + 31) / 32, t = b - e.blk;
  const int bx = (t % tcols) * 32, by = (t / tcols) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  if (!e.transpose) {
    for (int r = ty; r < 32; r += 8) {
      const int row = by + r, col = bx + tx;
      if (row < e.rows && col < e.cols) st_dt(e.y, e.y_dtype, (long)row * e.cols + col, ld_dt(e.x, e.x_dtype, (long)row * e.cols + col));
    }
    return;
  }
  for (int r = ty; r < 32; r += 8) {
    const int row = by + r, col = bx + tx;
    tile[r][tx] = (row < e.rows && col < e.cols) ? ld_dt(e.x, e.x_dtype, (long)row * e.cols + col) : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int orow = bx + r, ocol = by + tx;                 // y[cols][rows]
    if (orow < e.cols && ocol < e.rows) st_dt(e.y, e.y_dtype, (long)orow * e.rows + ocol, tile[tx][r]);
  }
}

__global__ void k_conv_grad_reorder(const float* __restrict__ g, int cout, int cin, int k, float* y) {
  const long total = (long)cout * cin * k * k;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // i over y [co][ci][kh][kw]
    const int kw = (int)(i % k);
    long r = i / k;
    const int kh = (int)(r % k); r /= k;
    const int ci = (int)(r % cin);
    const int co = (int)(r / cin);
    y[i] = g[(long)co * k * k * cin + (kh * k + kw) * cin + ci];
  }
}

// ------------------------------------------------------------------ column reductions
// chunking of `rows` for the simple two-pass column reduction (wide rows only)
__host__ __device__ inline int red_chunks(long rows) {
  long c = (rows + 63) / 64;
  return (int)(c > 1024 ? 1024 : (c < 1 ? 1 : c));
}

template <typename T>
__global__ void __launch_bounds__(256) k_colsum_part(const T* __restrict__ x, long ldx, long rows, int cols,
                                                     int nchunk, float* part) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y;
  if (col >= cols) return;
  const long per = (rows + nchunk - 1) / nchunk;
  const long r0 = ch * per, r1 = min(rows, r0 + per);
  float s = 0.f;
  for (long r = r0; r < r1; ++r) s += ld<T>(x, r * ldx + col);
  part[(long)ch * cols + col] = s;
}

__global__ void k_colsum_final(const float* part, int nchunk, int cols, float* out, int accumulate) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= cols) return;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += part[(long)c * cols + col];
  out[col] = accumulate ? out[col] + s : s;
}

// Generic coalesced column reduction over token-major [rows, cols] tensors: each thread owns
// 4 consecutive columns (8-byte bf16 / 16-byte fp32 loads), RPI = 256 / (cols/4) rows advance
// together, block partials are combined in LDS, and k_colred_final sums the block partials
// (8 row-groups x 32 columns per block) in a fixed order.
//   CR_SUM     sum a                                  (bias gradients)
//   CR_SUMSQ   sum a, sum a^2                         (BatchNorm batch statistics)
//   CR_BNBWD   sum g, sum g*xhat,  g = dy act'(xhat gamma + beta), xhat = (x - mean) rstd
//   CR_DOT     sum a*b (b NULL: sum a) per image       (SE gate / broadcast-add backward)
//   CR_ROWN    sum g*xhat, sum g,  g = dy keep, xhat = (x - mean_row) rstd_row  (LN/RMS params)
enum { CR_SUM = 0, CR_SUMSQ = 1, CR_BNBWD = 2, CR_DOT = 3, CR_ROWN = 4 };

struct ColRed {
  const void* a;       // x (or dy for CR_SUM / CR_DOT)
  const void* b;       // dy (CR_BNBWD / CR_ROWN) or the second factor (CR_DOT)
  long rows;           // rows per image (CR_DOT) or total
  int cols;
  const float* mean;   // per column (BN) or per row (ROWN, may be NULL for RMS)
  const float* rstd;
  const float* gamma;
  const float* beta;
  int act;
  float p;
  uint32_t seed;
  const unsigned int* soff;   // device seed offset (hv_kernels.h), may be NULL
};

template <typename T> __device__ __forceinline__ void ld4(const T* p, long i, float (&v)[4]);
template <> __device__ __forceinline__ void ld4<float>(const float* p, long i, float (&v)[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p + i);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
template <> __device__ __forceinline__ void ld4<unsigned short>(const unsigned short* p, long i, float (&v)[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p + i);
  v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
  v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
}

template <int MODE> struct CrNV { static constexpr int V = (MODE == CR_SUM || MODE == CR_DOT) ? 1 : 2; };

template <typename TA, typename TB, int MODE, int NCH>
__global__ void __launch_bounds__(256) k_colred(const ColRed r, int nblk, float* part) {
  constexpr int NV = CrNV<MODE>::V;
  __shared__ float sm[NV * 1024];
  const int cpr = r.cols >> 2;
  const int rpi = cpr <= 256 ? 256 / cpr : 1;
  const int tid = threadIdx.x;
  const int rsub = cpr <= 256 ? tid / cpr : 0;
  const int img = blockIdx.y;
  const long base = (long)img * r.rows * r.cols;
  float acc[NV][NCH][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[v][c][j] = 0.f;
  if (rsub < rpi) {
    // U rows per trip: all their loads are issued before any is consumed (the one-load-per-trip
    // loop ran at load latency); the values are then accumulated in the original row order, so
    // the sums are bitwise those of the one-row loop
    constexpr int U = NCH == 1 ? 4 : (NCH == 2 ? 2 : 1);
    constexpr bool HASB = MODE != CR_SUM && MODE != CR_SUMSQ;
    const long step = (long)nblk * rpi;
    for (long r0 = (long)blockIdx.x * rpi; r0 < r.rows; r0 += U * step) {
      float a[U][NCH][4], b[U][NCH][4];
      float rmu[U], rrs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long row = r0 + u * step + rsub;
        rmu[u] = 0.f;
        rrs[u] = 1.f;
        if (row >= r.rows) continue;
        if constexpr (MODE == CR_ROWN) {
          rmu[u] = r.mean ? r.mean[row] : 0.f;
          rrs[u] = r.rstd[row];
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int ch = cpr <= 256 ? tid % cpr : tid + 256 * c;
          if (ch >= cpr) continue;
          const long o = base + row * r.cols + ch * 4;
          ld4<TA>((const TA*)r.a, o, a[u][c]);
          if constexpr (HASB) {
            if (MODE != CR_DOT || r.b) ld4<TB>((const TB*)r.b, o, b[u][c]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long row = r0 + u * step + rsub;
        if (row >= r.rows) break;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int ch = cpr <= 256 ? tid % cpr : tid + 256 * c;
          if (ch >= cpr) continue;
          const int col = ch * 4;
          const long o = base + row * r.cols + col;
          if constexpr (MODE == CR_SUM) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[0][c][j] += a[u][c][j];
          } else if constexpr (MODE == CR_SUMSQ) {
#pragma unroll
            for (int j = 0; j < 4; ++j) { acc[0][c][j] += a[u][c][j]; acc[1][c][j] += a[u][c][j] * a[u][c][j]; }
          } else if constexpr (MODE == CR_DOT) {
            if (r.b) {
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[0][c][j] += a[u][c][j] * b[u][c][j];
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[0][c][j] += a[u][c][j];
            }
          } else if constexpr (MODE == CR_BNBWD) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int cc = col + j;
              const float xh = (a[u][c][j] - r.mean[cc]) * r.rstd[cc];
              const float g = b[u][c][j] * hv_act_grad(xh * (r.gamma ? r.gamma[cc] : 1.f) + (r.beta ? r.beta[cc] : 0.f), r.act);
              acc[0][c][j] += g;
              acc[1][c][j] += g * xh;
            }
          } else {  // CR_ROWN
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float xh = (a[u][c][j] - rmu[u]) * rrs[u];
              const float g = b[u][c][j] * hv_drop_scale(hv_seed(r.seed, r.soff), (unsigned long long)(o + j), r.p);
              acc[0][c][j] += g * xh;
              acc[1][c][j] += g;
            }
          }
        }
      }
    }
  }
  float* out = part + ((long)img * nblk + blockIdx.x) * NV * r.cols;
  if (cpr <= 256) {
    // combine the rpi row groups of the block in LDS (rpi * cols <= 1024)
    if (rsub < rpi) {
      const int col = (tid % cpr) * 4;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[v * 1024 + rsub * r.cols + col + j] = acc[v][0][j];
    }
    __syncthreads();
    for (int i = tid; i < NV * r.cols; i += 256) {
      const int v = i / r.cols, col = i - v * r.cols;
      float t = 0.f;
      for (int q = 0; q < rpi; ++q) t += sm[v * 1024 + q * r.cols + col];
      out[i] = t;
    }
  } else {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = tid + 256 * c;
      if (ch >= cpr) continue;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[v * r.cols + ch * 4 + j] = acc[v][c][j];
    }
  }
}

// sums[img][i] (+)= sum over the nblk partials of column i (i < width); 8 row groups x 32 columns
// 8 columns x 32 partial-row groups per block (the former 32 x 8 left a 64-column reduce on 4
// workgroups, each thread walking 64 partials in series: ~14 us per launch, 459 launches per
// training step); four independent accumulators per thread, combined in a fixed order
// (deterministic).
// sums_hi: columns >= split go to sums_hi[col - split] instead (one image; the LN gamma / beta
// gradients straight into their parameters' buffers)
__global__ void __launch_bounds__(256) k_colred_final(const float* part, int nblk, int width, float* sums,
                                                      int accumulate, float* sums_hi, int split) {
  __shared__ float sm[32][9];
  const int img = blockIdx.y;
  const int c = threadIdx.x & 7, g = threadIdx.x >> 3;
  const int col = blockIdx.x * 8 + c;
  float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
  if (col < width) {
    const float* p = part + (long)img * nblk * width + col;
    int b = g;
    for (; b + 96 < nblk; b += 128) {
      t0 += p[(long)b * width];
      t1 += p[(long)(b + 32) * width];
      t2 += p[(long)(b + 64) * width];
      t3 += p[(long)(b + 96) * width];
    }
    for (; b < nblk; b += 32) t0 += p[(long)b * width];
  }
  sm[g][c] = (t0 + t1) + (t2 + t3);
  __syncthreads();
  if (g == 0 && col < width) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 32; ++q) s += sm[q][c];
    float* o = sums_hi && col >= split ? sums_hi + (col - split) : sums + (long)img * width + col;
    *o = accumulate ? *o + s : s;
  }
}

// block cap of the partial pass: 1,024 (4 per CU: enough rows in flight for the BN / LN backward
// reductions over 409,600 pixels; 512 -> 1024 measured 127.8-128.2 -> 126.7 ms per training step,
// 2,048 no further gain, profiles/r05/colred_cap_ab.txt).  HV_COLRED_CAP (64..4096, read once per
// process) overrides it for A/Bs.
inline long colred_cap() {
  static const long c = [] {
    const char* e = getenv("HV_COLRED_CAP");
    const long v = e ? atol(e) : 1024;
    return v < 64 ? 64L : (v > 4096 ? 4096L : v);
  }();
  return c;
}

inline int colred_blocks(long rows, int cols, int imgs) {
  const int cpr = cols / 4;
  const int rpi = cpr <= 256 ? 256 / cpr : 1;
  long b = (rows + (long)rpi * 8 - 1) / ((long)rpi * 8);
  const long cm = colred_cap();
  const long cap = imgs > 1 ? (cm / imgs > 8 ? cm / imgs : 8) : cm;
  b = b > cap ? cap : (b < 1 ? 1 : b);
  return (int)b;
}

inline bool colred_ok(int cols) { return cols % 4 == 0 && cols / 4 <= 1024; }

inline size_t colred_work(long rows, int cols, int imgs, int nv) {
  return (size_t)imgs * colred_blocks(rows, cols, imgs) * nv * cols;
}

// launch part + final; sums receives [imgs][NV*cols] (NV-major per image)
template <typename TA, typename TB, int MODE>
int colred_run(const ColRed& r, int imgs, float* work, float* sums, int accumulate, hipStream_t s,
               float* sums_hi = nullptr, int split = 0) {
  constexpr int NV = CrNV<MODE>::V;
  const int nblk = colred_blocks(r.rows, r.cols, imgs);
  const int cpr = r.cols / 4;
  dim3 grid(nblk, imgs);
  if (cpr <= 256) k_colred<TA, TB, MODE, 1><<<grid, 256, 0, s>>>(r, nblk, work);
  else if (cpr <= 512) k_colred<TA, TB, MODE, 2><<<grid, 256, 0, s>>>(r, nblk, work);
  else k_colred<TA, TB, MODE, 4><<<grid, 256, 0, s>>>(r, nblk, work);
  k_colred_final<<<dim3(hv_cdiv(NV * r.cols, 8), imgs), 256, 0, s>>>(work, nblk, NV * r.cols, sums, accumulate,
                                                                    sums_hi, split);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// ------------------------------------------------------------------ BatchNorm (train)
__global__ void k_bn_stats_post(const float* sums, int c, long rows, float eps, float momentum, float* mean,
                                float* rstd, float* rmean, float* rvar) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= c) return;
  const double m = (double)sums[col] / (double)rows;
  double var = (double)sums[c + col] / (double)rows - m * m;
  var = var < 0.0 ? 0.0 : var;
  mean[col] = (float)m;
  rstd[col] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[col] = (1.f - momentum) * rmean[col] + momentum * (float)m;
  if (rvar) {
    const double unb = rows > 1 ? var * (double)rows / (double)(rows - 1) : var;
    rvar[col] = (1.f - momentum) * rvar[col] + momentum * (float)unb;
  }
}

__global__ void k_bn_bwd_post(const float* sums, int c, float* dgamma, float* dbeta) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= c) return;
  if (dbeta) dbeta[col] = sums[col];
  if (dgamma) dgamma[col] = sums[c + col];
}

template <typename T>
__global__ void k_bn_apply(const T* __restrict__ x, long total, int c, const float* mean, const float* rstd,
                           const float* g, const float* b, int act, T* y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    const float z = (ld<T>(x, i) - mean[col]) * rstd[col] * (g ? g[col] : 1.f) + (b ? b[col] : 0.f);
    st<T>(y, i, hv_act(z, act));
  }
}

template <typename T>
__global__ void k_bn_bwd_apply(const T* __restrict__ x, const T* __restrict__ dy, long rows, int c,
                               const float* mean, const float* rstd, const float* g, const float* b, int act,
                               const float* sums, T* dx) {
  const long total = rows * c;
  const float inv = 1.0f / (float)rows;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    const float rs = rstd[col], gg = g ? g[col] : 1.f, bb = b ? b[col] : 0.f;
    const float xh = (ld<T>(x, i) - mean[col]) * rs;
    const float gr = ld<T>(dy, i) * hv_act_grad(xh * gg + bb, act);
    st<T>(dx, i, gg * rs * (gr - sums[col] * inv - xh * sums[c + col] * inv));
  }
}

// ------------------------------------------------------------------ row norms (train)
constexpr int RQ = 32;     // columns per row supported: up to 64 * RQ = 2048

// Row kernels use a G-lane group per row (G = pow2 >= cols/4, <= 64): each lane owns 4
// consecutive columns per pass (8-byte bf16 / 16-byte fp32 vector access), NP passes cover the
// row, 64/G rows share a wave, group reductions are xor-shuffles inside the group.
template <typename T> __device__ __forceinline__ void st4(T* p, long i, const float (&v)[4]);
template <> __device__ __forceinline__ void st4<float>(float* p, long i, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void st4<unsigned short>(unsigned short* p, long i, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p + i) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// mode 0 LayerNorm, 1 RMSNorm
template <typename TX, typename TY, int G, int NP>
__global__ void __launch_bounds__(256) k_rownorm_train(int mode, const TX* __restrict__ x, int rows, int cols,
                                                       float eps, const float* g, const float* b, float p,
                                                       uint32_t seed, const unsigned int* soff, TY* y,
                                                       const TY* res, float* mean, float* rstd) {
  seed = hv_seed(seed, soff);
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63, gl = lane % G;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G;
  const bool ok = row < rows;
  const long base = (ok ? row : 0) * cols;
  float v[NP][4];
  float sm = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = (q * G + gl) * 4;
    if (ok && col < cols) ld4<TX>(x, base + col, v[q]);
    else v[q][0] = v[q][1] = v[q][2] = v[q][3] = 0.f;
    sm += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
  }
  const float mu = mode == 0 ? group_sum<G>(sm) / cols : 0.f;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = (q * G + gl) * 4;
    if (col < cols) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[q][j] - mu; var += d * d; }
    }
  }
  var = group_sum<G>(var);
  const float rs = 1.0f / sqrtf(var / cols + eps);
  if (!ok) return;
  if (gl == 0) {
    if (mean) mean[row] = mu;
    rstd[row] = rs;
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = (q * G + gl) * 4;
    if (col >= cols) continue;
    float o[4];
    float r4[4] = {0.f, 0.f, 0.f, 0.f};
    if (res) ld4<TY>(res, base + col, r4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float val = (v[q][j] - mu) * rs * (g ? g[col + j] : 1.f) + (b ? b[col + j] : 0.f);
      o[j] = val * hv_drop_scale(seed, (unsigned long long)(base + col + j), p) + r4[j];
    }
    st4<TY>(y, base + col, o);
  }
}

template <typename TX, typename TD, typename TO, int G, int NP>
__global__ void __launch_bounds__(256) k_rownorm_bwd(int mode, const TX* __restrict__ x, const TD* __restrict__ dy,
                                                     int rows, int cols, const float* mean, const float* rstd,
                                                     const float* g, float p, uint32_t seed,
                                                     const unsigned int* soff, TO* dx, const TO* dx_add) {
  seed = hv_seed(seed, soff);
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63, gl = lane % G;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G;
  const bool ok = row < rows;
  const long base = (ok ? row : 0) * cols;
  const float mu = (ok && mode == 0) ? mean[row] : 0.f, rs = ok ? rstd[row] : 1.f;
  float xh[NP][4], gg[NP][4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = (q * G + gl) * 4;
    float a[4] = {0.f, 0.f, 0.f, 0.f}, d[4] = {0.f, 0.f, 0.f, 0.f};
    if (ok && col < cols) {
      ld4<TX>(x, base + col, a);
      ld4<TD>(dy, base + col, d);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xh[q][j] = (a[j] - mu) * rs;
      const bool in = ok && col < cols;
      const float gr = in ? d[j] * hv_drop_scale(seed, (unsigned long long)(base + col + j), p) : 0.f;
      gg[q][j] = gr * ((g && in) ? g[col + j] : 1.f);
      s1 += gg[q][j];
      s2 += gg[q][j] * xh[q][j];
    }
  }
  s1 = group_sum<G>(s1) / cols;
  s2 = group_sum<G>(s2) / cols;
  if (!ok) return;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = (q * G + gl) * 4;
    if (col >= cols) continue;
    float o[4];
    float ad[4] = {0.f, 0.f, 0.f, 0.f};
    if (dx_add) ld4<TO>(dx_add, base + col, ad);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = (mode == 0 ? rs * (gg[q][j] - s1 - xh[q][j] * s2) : rs * (gg[q][j] - xh[q][j] * s2)) + ad[j];
    st4<TO>(dx, base + col, o);
  }
}

// (G, NP) for a row of `cols` columns
inline void rown_shape(int cols, int* G, int* NP) {
  const int q = (cols + 3) / 4;
  int g = 1;
  while (g < q && g < 64) g <<= 1;
  *G = g;
  *NP = (q + g - 1) / g;
}

template <typename TX, typename TY>
int rown_train_launch(int mode, const void* x, int rows, int cols, float eps, const float* gamma, const float* beta,
                      float p, uint32_t seed, const unsigned int* soff, void* y, const void* res, float* mean,
                      float* rstd, hipStream_t s) {
  int G, NP;
  rown_shape(cols, &G, &NP);
  const unsigned grid = hv_cdiv(rows, 4 * (64 / G));
#define RT(GG, PP) k_rownorm_train<TX, TY, GG, PP><<<grid, 256, 0, s>>>(mode, (const TX*)x, rows, cols, eps, gamma, \
      beta, p, seed, soff, (TY*)y, (const TY*)res, mean, rstd)
  if (G == 8) RT(8, 1);
  else if (G == 16) RT(16, 1);
  else if (G == 32) RT(32, 1);
  else if (G == 64 && NP == 1) RT(64, 1);
  else if (G == 64 && NP == 2) RT(64, 2);
  else if (G == 64 && NP <= 4) RT(64, 4);
  else if (G == 64 && NP <= 8) RT(64, 8);
  else return HV_EUNSUPPORTED;
#undef RT
  HV_CHECK_LAUNCH();
  return HV_OK;
}

template <typename TX, typename TD, typename TO>
int rown_bwd_launch(int mode, const void* x, const void* dy, int rows, int cols, const float* mean, const float* rstd,
                    const float* gamma, float p, uint32_t seed, const unsigned int* soff, void* dx,
                    const void* dx_add, hipStream_t s) {
  int G, NP;
  rown_shape(cols, &G, &NP);
  const unsigned grid = hv_cdiv(rows, 4 * (64 / G));
#define RBK(GG, PP) k_rownorm_bwd<TX, TD, TO, GG, PP><<<grid, 256, 0, s>>>(mode, (const TX*)x, (const TD*)dy, rows, \
      cols, mean, rstd, gamma, p, seed, soff, (TO*)dx, (const TO*)dx_add)
  if (G == 8) RBK(8, 1);
  else if (G == 16) RBK(16, 1);
  else if (G == 32) RBK(32, 1);
  else if (G == 64 && NP == 1) RBK(64, 1);
  else if (G == 64 && NP == 2) RBK(64, 2);
  else if (G == 64 && NP <= 4) RBK(64, 4);
  else if (G == 64 && NP <= 8) RBK(64, 8);
  else return HV_EUNSUPPORTED;
#undef RBK
  HV_CHECK_LAUNCH();
  return HV_OK;
}

// ------------------------------------------------------------------ elementwise
template <typename T>
__global__ void k_act_bwd(const T* __restrict__ dy, const T* __restrict__ pre, long n, int act, float p,
                          uint32_t seed, const unsigned int* soff, T* dpre) {
  seed = hv_seed(seed, soff);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st<T>(dpre, i, ld<T>(dy, i) * hv_drop_scale(seed, (unsigned long long)i, p) *
                       ((sizeof(T) == 2 && act == HV_ACT_GELU) ? hv_gelu_grad_fast(ld<T>(pre, i))
                                                                : hv_act_grad(ld<T>(pre, i), act)));
}

template <typename T>
__global__ void k_dropout(const T* __restrict__ x, long n, float p, uint32_t seed, const unsigned int* soff, T* y) {
  seed = hv_seed(seed, soff);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st<T>(y, i, ld<T>(x, i) * hv_drop_scale(seed, (unsigned long long)i, p));
}

// ------------------------------------------------------------------ SE / pooling / upsample
// per image: recompute the SE MLP and backpropagate dgate -> dpooled; keep ds / act / dh for
// the parameter reductions.  work per image: [c ds][cr act][cr dh]
__global__ void __launch_bounds__(256) k_se_bwd_img(const float* pooled, const float* dgate, int c, int cr,
                                                    const float* w1, const float* b1, const float* w2,
                                                    const float* b2, float* dpooled, float* work) {
  extern __shared__ float sm[];
  float* h = sm;            // [cr]
  float* ds = sm + cr;      // [c]
  const int img = blockIdx.x;
  const float* p = pooled + (long)img * c;
  float* wk = work + (long)img * (c + 2 * cr);
  for (int r = threadIdx.x; r < cr; r += blockDim.x) {
    float s = b1[r];
    for (int k = 0; k < c; ++k) s += w1[(long)r * c + k] * p[k];
    h[r] = s;
    wk[c + r] = hv_silu(s);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < c; j += blockDim.x) {
    float s = b2[j];
    for (int r = 0; r < cr; ++r) s += w2[(long)j * cr + r] * hv_silu(h[r]);
    const float gt = hv_sigmoid(s);
    const float d = dgate[(long)img * c + j] * gt * (1.f - gt);
    ds[j] = d;
    wk[j] = d;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < cr; r += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < c; ++j) s += w2[(long)j * cr + r] * ds[j];
    const float dh = s * hv_act_grad(h[r], HV_ACT_SILU);
    wk[c + cr + r] = dh;
    h[r] = dh;      // reuse: dh
  }
  __syncthreads();
  for (int k = threadIdx.x; k < c; k += blockDim.x) {
    float s = 0.f;
    for (int r = 0; r < cr; ++r) s += w1[(long)r * c + k] * h[r];
    dpooled[(long)img * c + k] = s;
  }
}

// parameter gradients of the SE MLP, summed over images in order
__global__ void k_se_bwd_params(const float* pooled, const float* work, int n, int c, int cr, float* dw1,
                                float* db1, float* dw2, float* db2) {
  const long total = 2L * c * cr + c + cr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    if (i < (long)c * cr) {                 // dw2[j][r] = sum ds[j] act[r]
      const int j = (int)(i / cr), r = (int)(i % cr);
      for (int b = 0; b < n; ++b) s += work[(long)b * (c + 2 * cr) + j] * work[(long)b * (c + 2 * cr) + c + r];
      dw2[i] = s;
    } else if (i < 2L * c * cr) {           // dw1[r][k] = sum dh[r] pooled[k]
      const long t = i - (long)c * cr;
      const int r = (int)(t / c), k = (int)(t % c);
      for (int b = 0; b < n; ++b) s += work[(long)b * (c + 2 * cr) + c + cr + r] * pooled[(long)b * c + k];
      dw1[t] = s;
    } else if (i < 2L * c * cr + c) {
      const int j = (int)(i - 2L * c * cr);
      for (int b = 0; b < n; ++b) s += work[(long)b * (c + 2 * cr) + j];
      db2[j] = s;
    } else {
      const int r = (int)(i - 2L * c * cr - c);
      for (int b = 0; b < n; ++b) s += work[(long)b * (c + 2 * cr) + c + cr + r];
      db1[r] = s;
    }
  }
}

template <typename T>
__global__ void k_se_bwd_apply(const T* __restrict__ dout, const float* gate, const float* dpooled, int hw, int c,
                               long total, float inv_hw, T* dy) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    const long img = i / ((long)hw * c);
    st<T>(dy, i, ld<T>(dout, i) * gate[img * c + col] + dpooled[img * c + col] * inv_hw);
  }
}

template <typename T>
__global__ void k_maxpool_bwd(const T* __restrict__ x, const T* __restrict__ dy, int n, int h, int w, int c, T* dx) {
  const int oh = h / 2, ow = w / 2;
  const long total = (long)n * oh * ow * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    long r = i / c;
    const int ox = (int)(r % ow); r /= ow;
    const int oy = (int)(r % oh);
    const int b = (int)(r / oh);
    long idx[4];
    int best = 0;
    float bv = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int yy = 2 * oy + (t >> 1), xx = 2 * ox + (t & 1);
      idx[t] = (((long)b * h + yy) * w + xx) * c + col;
      const float v = ld<T>(x, idx[t]);
      if (t == 0 || v > bv) { bv = v; best = t; }
    }
    const float g = ld<T>(dy, i);
#pragma unroll
    for (int t = 0; t < 4; ++t) st<T>(dx, idx[t], t == best ? g : 0.f);
  }
}

template <typename T>
__global__ void k_upsample_bwd(const T* __restrict__ dy, int n, int h, int w, int c, int hb, int wb, T* db) {
  const int fy = h / hb, fx = w / wb;
  const long total = (long)n * hb * wb * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    long r = i / c;
    const int bx = (int)(r % wb); r /= wb;
    const int by = (int)(r % hb);
    const int b = (int)(r / hb);
    float s = 0.f;
    for (int yy = 0; yy < fy; ++yy)
      for (int xx = 0; xx < fx; ++xx) s += ld<T>(dy, (((long)b * h + by * fy + yy) * w + bx * fx + xx) * c + col);
    st<T>(db, i, s);
  }
}

template <typename T>
__global__ void k_vit_assemble(const T* x, const float* cls, const float* pos, int n, int t, int d, T* z) {
  const long total = (long)n * (t + 1) * d;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % d);
    const long r = i / d;
    const int tok = (int)(r % (t + 1));
    const long b = r / (t + 1);
    const float v = tok == 0 ? cls[col] : ld<T>(x, (b * t + tok - 1) * d + col);
    st<T>(z, i, v + pos[(long)tok * d + col]);
  }
}

template <typename T>
__global__ void k_vit_assemble_bwd(const T* dz, int n, int t, int d, T* dx, float* dcls, float* dpos) {
  const long total = (long)(t + 1) * d;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % d);
    const int tok = (int)(i / d);
    float s = 0.f;
    for (int b = 0; b < n; ++b) {
      const float g = ld<T>(dz, ((long)b * (t + 1) + tok) * d + col);
      s += g;
      if (tok > 0) st<T>(dx, ((long)b * t + tok - 1) * d + col, g);
    }
    dpos[i] = s;
    if (tok == 0) dcls[col] = s;
  }
}

template <typename T>
__global__ void k_scatter_rows(const T* dy, long stride, int n, int c, T* dx) {
  const long total = (long)n * stride * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % c);
    const long r = i / c;
    const long b = r / stride;
    st<T>(dx, i, (r % stride) == 0 ? ld<T>(dy, b * c + col) : 0.f);
  }
}

// ------------------------------------------------------------------ YOLO loss
// object count: block partial counts added atomically (integer-valued floats < 2^24: exact in
// any order, so deterministic)
// Small fills as kernels, not hipMemsetAsync: inside a captured training step these become
// kernel nodes ordered like every other launch (the memset-node form of the object-count reset
// left the first replay's YOLO loss normalised by a wrong count on some runs --
// tools/train_bisect.py: identical predictions, total 2002.99 vs 1700.07).
__global__ void k_fill_f32(float* p, int n, float v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void __launch_bounds__(256) k_yolo_count(const float* targets, long cells, int P, float* nobj) {
  __shared__ float scratch[16];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < cells; i += (long)gridDim.x * 256)
    s += targets[i * P + 4] > 0.5f ? 1.f : 0.f;
  s = block_sum(s, scratch);
  if (threadIdx.x == 0 && s > 0.f) atomicAdd(nobj, s);
}

__device__ __forceinline__ float bce_logits(float x, float t) {
  return fmaxf(x, 0.f) - x * t + log1pf(__expf(-fabsf(x)));
}

// one thread per (image, anchor, y, x) cell; block partials of the 4 raw sums
template <typename T, typename TD>
__global__ void __launch_bounds__(256) k_yolo_loss(const T* __restrict__ lg, const float* __restrict__ tg, int n,
                                                   int h, int w, int A, int P, float lc, float lo, float ln,
                                                   float lcl, const float* nobj, TD* dlg, float* part) {
  __shared__ float scratch[16];
  const long cells = (long)n * A * h * w;
  const long cell = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const float N = nobj[0];
  const float inv = N > 0.f ? 1.0f / N : 0.f;
  float s_coord = 0.f, s_obj = 0.f, s_noobj = 0.f, s_cls = 0.f;
  if (cell < cells) {
    long r = cell;
    const int x = (int)(r % w); r /= w;
    const int y = (int)(r % h); r /= h;
    const int a = (int)(r % A);
    const int b = (int)(r / A);
    const long lbase = (((long)b * h + y) * w + x) * (long)(A * P) + (long)a * P;   // NHWC logits
    const float* t = tg + cell * P;                                               // [n, A, h, w, P]
    const float t4 = t[4];
    const bool obj = t4 > 0.5f, noobj = t4 < 0.5f;
    for (int k = 0; k < P; ++k) {
      const float p = ld<T>(lg, lbase + k);
      float gr = 0.f;
      if (k < 4) {
        if (obj) {
          const float d = p - t[k];
          s_coord += d * d;
          gr = lc * inv * 2.f * d;
        }
      } else if (k == 4) {
        if (obj) { s_obj += bce_logits(p, t4); gr = lo * inv * (hv_sigmoid(p) - t4); }
        else if (noobj) { s_noobj += bce_logits(p, t4); gr = ln * inv * (hv_sigmoid(p) - t4); }
      } else if (obj) {
        s_cls += bce_logits(p, t[k]);
        gr = lcl * inv * (hv_sigmoid(p) - t[k]);
      }
      st<TD>(dlg, lbase + k, N > 0.f ? gr : 0.f);
    }
  }
  s_coord = block_sum(s_coord, scratch);
  s_obj = block_sum(s_obj, scratch);
  s_noobj = block_sum(s_noobj, scratch);
  s_cls = block_sum(s_cls, scratch);
  if (threadIdx.x == 0) {
    float* o = part + (long)blockIdx.x * 4;
    o[0] = s_coord; o[1] = s_obj; o[2] = s_noobj; o[3] = s_cls;
  }
}

__global__ void k_yolo_final(const float* part, int nblk, const float* nobj, float lc, float lo, float ln, float lcl,
                             float* sums) {
  // lanes 0..3 of the one wave: component sums; the weighted total is formed from the lanes'
  // registers (shuffles), not by reading back the other lanes' global stores
  const int t = threadIdx.x;
  float s = 0.f;
  if (t < 4)
    for (int b = 0; b < nblk; ++b) s += part[(long)b * 4 + t];
  const float N = nobj[0];
  const float v = N > 0.f ? s : 0.f;
  const float s0 = __shfl(v, 0), s1 = __shfl(v, 1), s2 = __shfl(v, 2), s3 = __shfl(v, 3);
  if (t < 4) sums[t] = v;
  if (t == 0) {
    sums[4] = N > 0.f ? (lc * s0 + lo * s1 + ln * s2 + lcl * s3) / N : 0.f;
    sums[5] = N;
  }
}

// ------------------------------------------------------------------ clipping + AdamW
constexpr int PB_ELEMS = 2048;     // parameter elements per block

__device__ __forceinline__ int find_param(const hv_param_entry* t, int count, int blk) {
  int lo = 0, hi = count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].blk <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) k_grad_sq(const hv_param_entry* tab, int count, const int* active, float* part) {
  __shared__ float scratch[16];
  const int ei = find_param(tab, count, blockIdx.x);
  const hv_param_entry e = tab[ei];
  const long b0 = (long)(blockIdx.x - e.blk) * PB_ELEMS;
  float s = 0.f;
  if (e.grad && (!active || active[ei])) {
    for (long i = b0 + threadIdx.x; i < min(e.n, b0 + PB_ELEMS); i += 256) {
      const float g = e.grad[i];
      s += g * g;
    }
  }
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    reinterpret_cast<int*>(part)[gridDim.x + blockIdx.x] = e.group;   // group of this block
  }
}

__global__ void __launch_bounds__(256) k_grad_norm_final(int nblk, const float* part, int groups, float m0,
                                                         float m1, float m2, float m3, float* norms, float* coefs) {
  __shared__ float scratch[16];
  const float mx[4] = {m0, m1, m2, m3};
  const int* grp = reinterpret_cast<const int*>(part) + nblk;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblk; b += 256) {
    const int g = grp[b];
    const double v = part[b];
    acc[0] += g == 0 ? v : 0.0;
    acc[1] += g == 1 ? v : 0.0;
    acc[2] += g == 2 ? v : 0.0;
    acc[3] += g == 3 ? v : 0.0;
  }
  for (int g = 0; g < groups; ++g) {
    const float tot = block_sum((float)acc[g], scratch);
    if (threadIdx.x == 0) {
      const float nrm = sqrtf(tot);
      norms[g] = nrm;
      const float c = mx[g] / (nrm + 1e-6f);
      coefs[g] = c < 1.f ? c : 1.f;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_adamw(const hv_param_entry* tab, int count, const float* coefs, float lr,
                                               float b1, float b2, float eps, float wd, float bc1, float bc2s,
                                               const int* __restrict__ steps, const int* __restrict__ active,
                                               const float* __restrict__ hyper) {
  const int ei = find_param(tab, count, blockIdx.x);
  const hv_param_entry e = tab[ei];
  if (!e.grad || (active && !active[ei])) return;     // no gradient this step: no decay, no update
  if (hyper) {                                  // device hyper-parameters (a scheduler's lr per step)
    lr = hyper[0]; b1 = hyper[1]; b2 = hyper[2]; eps = hyper[3]; wd = hyper[4];
  }
  if (steps) {                                  // per-parameter bias correction (torch state['step'])
    const float t = (float)max(steps[ei], 1);
    bc1 = 1.f - powf(b1, t);
    bc2s = sqrtf(1.f - powf(b2, t));
  }
  const long b0 = (long)(blockIdx.x - e.blk) * PB_ELEMS;
  const float cf = coefs ? coefs[e.group] : 1.f;
  const float step = lr / bc1;
  for (long i = b0 + threadIdx.x; i < min(e.n, b0 + PB_ELEMS); i += 256) {
    const float g = e.grad[i] * cf;
    const float m = b1 * e.exp_avg[i] + (1.f - b1) * g;
    const float v = b2 * e.exp_avg_sq[i] + (1.f - b2) * g * g;
    e.exp_avg[i] = m;
    e.exp_avg_sq[i] = v;
    const float denom = sqrtf(v) / bc2s + eps;
    float p = e.param[i] * (1.f - lr * wd);
    e.param[i] = p - step * m / denom;
  }
}

// ------------------------------------------------------------------ mHC coefficient backward
// d/d(H_pre_raw, gamma_pre, beta_pre) from dGc (gradient of the centred folded gate) and du:
// dG = dGc - colmean_i(dGc) (adjoint of the centring), dS = gamma_i dG + beta_i du_j,
// dH_pre_raw = dS s(1-s), dgamma_i = sum_j dG_ij s_ij, dbeta_i = sum_j du_j s_ij.  Wave per row i.
__global__ void __launch_bounds__(256) k_mhc_pre_bwd(const float* __restrict__ dgc, const float* __restrict__ colsum,
                                                     const float* __restrict__ du, const float* __restrict__ hraw,
                                                     const float* gamma, const float* beta, int D, int Hd,
                                                     float* dhraw, float* dgamma, float* dbeta) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= D) return;
  const float gi = gamma ? gamma[i] : 1.f, bi = beta ? beta[i] : 0.f, invD = 1.0f / D;
  float sg = 0.f, sb = 0.f;
  for (int j = lane; j < Hd; j += 64) {
    const long o = (long)i * Hd + j;
    const float sj = hv_sigmoid(hraw[o]);
    const float dg = dgc[o] - colsum[j] * invD;
    sg += dg * sj;
    sb += du[j] * sj;
    dhraw[o] = (gi * dg + bi * du[j]) * sj * (1.f - sj);
  }
  sg = wave_sum(sg);
  sb = wave_sum(sb);
  if (lane == 0) {
    dgamma[i] = sg;
    dbeta[i] = sb;
  }
}

// rows r < D: dH_res = dWc_x - rowmean;  rows r >= D: dH_post_raw = (dWc_h - rowmean) 2 s(1-s)
__global__ void __launch_bounds__(256) k_mhc_post_bwd(const float* __restrict__ dwx, const float* __restrict__ dwh,
                                                      const float* __restrict__ hpost_raw, int D, int Hd, float* dhres,
                                                      float* dhpost) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= D + Hd) return;
  const bool res = r < D;
  const float* src = res ? dwx + (long)r * D : dwh + (long)(r - D) * D;
  float m = 0.f;
  for (int j = lane; j < D; j += 64) m += src[j];
  m = wave_sum(m) / D;
  for (int j = lane; j < D; j += 64) {
    const float v = src[j] - m;
    if (res) {
      dhres[(long)r * D + j] = v;
    } else {
      const long o = (long)(r - D) * D + j;
      const float sp = hv_sigmoid(hpost_raw[o]);
      dhpost[o] = v * 2.f * sp * (1.f - sp);
    }
  }
}

inline unsigned grid_for(long n) {
  long b = (n + 255) / 256;
  return (unsigned)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

}  // namespace

// ====================================================================== C ABI
extern "C" int hv_dgrad_weight_prep(const float* w, int cout, int cin, int k, int flip, int y_dtype, void* y,
                                    hv_stream_t stream) {
  if (!w || !y || cout <= 0 || cin <= 0 || k <= 0) return HV_EINVAL;
  k_dgrad_wprep<<<grid_for((long)cout * cin * k * k), 256, 0, (hipStream_t)stream>>>(w, cout, cin, k, flip, y_dtype, y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_transpose_cast(const float* x, int rows, int cols, int y_dtype, void* y, hv_stream_t stream) {
  if (!x || !y || rows <= 0 || cols <= 0) return HV_EINVAL;
  dim3 grid(hv_cdiv(cols, 32), hv_cdiv(rows, 32));
  k_transpose_cast<<<grid, 256, 0, (hipStream_t)stream>>>(x, rows, cols, y_dtype, y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_transpose_blocks(int rows, int cols) {
  return (rows <= 0 || cols <= 0) ? 0 : (int)(hv_cdiv(rows, 32) * hv_cdiv(cols, 32));
}

extern "C" int hv_transpose_group(const hv_transpose_entry* tab, int count, int total_blocks, hv_stream_t stream) {
  if (!tab || count <= 0 || total_blocks <= 0) return HV_EINVAL;
  k_transpose_group<<<total_blocks, 256, 0, (hipStream_t)stream>>>(tab, count);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_conv_grad_reorder(const float* g, int cout, int cin, int k, float* y, hv_stream_t stream) {
  if (!g || !y) return HV_EINVAL;
  k_conv_grad_reorder<<<grid_for((long)cout * cin * k * k), 256, 0, (hipStream_t)stream>>>(g, cout, cin, k, y);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_colsum_final(const float* part, int nblk, int cols, float* out, int accumulate,
                               hv_stream_t stream) {
  if (!part || !out || nblk <= 0 || cols <= 0) return HV_EINVAL;
  k_colred_final<<<dim3(hv_cdiv(cols, 8), 1), 256, 0, (hipStream_t)stream>>>(part, nblk, cols, out, accumulate, nullptr, 0);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_colsum_work_floats(int rows, int cols) {
  return colred_ok(cols) ? colred_work(rows, cols, 1, 1) : (size_t)red_chunks(rows) * cols;
}

extern "C" int hv_colsum(int dtype, const void* x, long ldx, int rows, int cols, float* out, int accumulate,
                         float* work, hv_stream_t stream) {
  if (!x || !out || !work || rows <= 0 || cols <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (colred_ok(cols) && ldx == cols) {
    ColRed r{};
    r.a = x; r.rows = rows; r.cols = cols;
    HV_DISPATCH(dtype, (colred_run<T, T, CR_SUM>(r, 1, work, out, accumulate, s)));
    return HV_OK;
  }
  const int nch = red_chunks(rows);
  dim3 grid(hv_cdiv(cols, 256), nch);
  HV_DISPATCH(dtype, (k_colsum_part<T><<<grid, 256, 0, s>>>((const T*)x, ldx, rows, cols, nch, work)));
  k_colsum_final<<<hv_cdiv(cols, 256), 256, 0, s>>>(work, nch, cols, out, accumulate);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_bn_work_floats(int rows, int c) { return colred_work(rows, c, 1, 2) + 2 * (size_t)c; }

extern "C" int hv_bn_stats(int dtype, const void* x, int rows, int c, float eps, float momentum, float* mean,
                           float* rstd, float* running_mean, float* running_var, float* work, hv_stream_t stream) {
  if (!x || !mean || !rstd || !work || rows <= 0 || c <= 0 || !colred_ok(c)) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float* sums = work + colred_work(rows, c, 1, 2);
  ColRed r{};
  r.a = x; r.rows = rows; r.cols = c;
  HV_DISPATCH(dtype, (colred_run<T, T, CR_SUMSQ>(r, 1, work, sums, 0, s)));
  k_bn_stats_post<<<hv_cdiv(c, 256), 256, 0, s>>>(sums, c, rows, eps, momentum, mean, rstd, running_mean, running_var);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_bn_apply(int dtype, const void* x, int rows, int c, const float* mean, const float* rstd,
                           const float* gamma, const float* beta, int act, void* y, hv_stream_t stream) {
  if (!x || !y || !mean || !rstd) return HV_EINVAL;
  const long total = (long)rows * c;
  HV_DISPATCH(dtype, (k_bn_apply<T><<<grid_for(total), 256, 0, (hipStream_t)stream>>>(
                         (const T*)x, total, c, mean, rstd, gamma, beta, act, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_bn_backward(int dtype, const void* x, const void* dy, int rows, int c, const float* mean,
                              const float* rstd, const float* gamma, const float* beta, int act, void* dx,
                              float* dgamma, float* dbeta, float* work, hv_stream_t stream) {
  if (!x || !dy || !dx || !work || rows <= 0 || c <= 0 || !colred_ok(c)) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float* sums = work + colred_work(rows, c, 1, 2);     // [sum g | sum g xhat]
  ColRed r{};
  r.a = x; r.b = dy; r.rows = rows; r.cols = c;
  r.mean = mean; r.rstd = rstd; r.gamma = gamma; r.beta = beta; r.act = act;
  HV_DISPATCH(dtype, (colred_run<T, T, CR_BNBWD>(r, 1, work, sums, 0, s)));
  k_bn_bwd_post<<<hv_cdiv(c, 256), 256, 0, s>>>(sums, c, dgamma, dbeta);
  const long total = (long)rows * c;
  HV_DISPATCH(dtype, (k_bn_bwd_apply<T><<<grid_for(total), 256, 0, s>>>((const T*)x, (const T*)dy, rows, c, mean,
                                                                        rstd, gamma, beta, act, sums, (T*)dx)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_rownorm_train(int mode, int x_dtype, const void* x, int rows, int cols, float eps,
                                const float* gamma, const float* beta, float drop_p, unsigned int seed,
                                const unsigned int* seed_offset, int y_dtype, void* y, const void* residual,
                                float* mean, float* rstd, hv_stream_t stream) {
  if (!x || !y || !rstd || rows <= 0 || cols <= 0 || cols % 4 || cols > 64 * RQ || (mode == 0 && !mean))
    return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == HV_F32 && y_dtype == HV_F32)
    return rown_train_launch<float, float>(mode, x, rows, cols, eps, gamma, beta, drop_p, seed, seed_offset, y, residual, mean, rstd, s);
  if (x_dtype == HV_F32 && y_dtype == HV_BF16)
    return rown_train_launch<float, unsigned short>(mode, x, rows, cols, eps, gamma, beta, drop_p, seed, seed_offset, y, residual,
                                                    mean, rstd, s);
  if (x_dtype == HV_BF16 && y_dtype == HV_BF16)
    return rown_train_launch<unsigned short, unsigned short>(mode, x, rows, cols, eps, gamma, beta, drop_p, seed, seed_offset, y,
                                                             residual, mean, rstd, s);
  if (x_dtype == HV_BF16 && y_dtype == HV_F32)
    return rown_train_launch<unsigned short, float>(mode, x, rows, cols, eps, gamma, beta, drop_p, seed, seed_offset, y, residual,
                                                    mean, rstd, s);
  return HV_EINVAL;
}

extern "C" size_t hv_rownorm_work_floats(int rows, int cols) {
  return colred_ok(cols) ? colred_work(rows, cols, 1, 2) + 2 * (size_t)cols : 0;
}

extern "C" int hv_rownorm_backward(int mode, int x_dtype, const void* x, int dy_dtype, const void* dy, int rows,
                                   int cols, const float* mean, const float* rstd, const float* gamma, float drop_p,
                                   unsigned int seed, const unsigned int* seed_offset, int dx_dtype, void* dx,
                                   const void* dx_add, float* dgamma, float* dbeta, float* work, hv_stream_t stream) {
  if (!x || !dy || !dx || !rstd || rows <= 0 || cols <= 0 || cols > 64 * RQ || (mode == 0 && !mean))
    return HV_EINVAL;
  const bool params = dgamma || dbeta;
  if (params && (!work || !colred_ok(cols))) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (cols % 4) return HV_EINVAL;
  const int key = x_dtype * 4 + dy_dtype * 2 + dx_dtype;
  int rc;
#define RB_LAUNCH(TX, TD, TO) rc = rown_bwd_launch<TX, TD, TO>(mode, x, dy, rows, cols, mean, rstd, gamma, drop_p, seed, \
      seed_offset, dx, dx_add, s)
  switch (key) {
    case 0: RB_LAUNCH(float, float, float); break;
    case 1: RB_LAUNCH(float, float, unsigned short); break;
    case 2: RB_LAUNCH(float, unsigned short, float); break;
    case 3: RB_LAUNCH(float, unsigned short, unsigned short); break;
    case 4: RB_LAUNCH(unsigned short, float, float); break;
    case 5: RB_LAUNCH(unsigned short, float, unsigned short); break;
    case 6: RB_LAUNCH(unsigned short, unsigned short, float); break;
    case 7: RB_LAUNCH(unsigned short, unsigned short, unsigned short); break;
    default: return HV_EINVAL;
  }
#undef RB_LAUNCH
  if (rc) return rc;
  if (params) {
    // [sum g xhat | sum g] written straight into dgamma / dbeta (the scratch row for a missing one)
    float* sums = work + colred_work(rows, cols, 1, 2);
    float* lo = dgamma ? dgamma : sums;
    float* hi = dbeta ? dbeta : sums + cols;
    ColRed r{};
    r.a = x; r.b = dy; r.rows = rows; r.cols = cols;
    r.mean = mode == 0 ? mean : nullptr; r.rstd = rstd; r.p = drop_p; r.seed = seed; r.soff = seed_offset;
    int rc;
    if (x_dtype == HV_F32 && dy_dtype == HV_F32) rc = colred_run<float, float, CR_ROWN>(r, 1, work, lo, 0, s, hi, cols);
    else if (x_dtype == HV_F32) rc = colred_run<float, unsigned short, CR_ROWN>(r, 1, work, lo, 0, s, hi, cols);
    else if (dy_dtype == HV_F32) rc = colred_run<unsigned short, float, CR_ROWN>(r, 1, work, lo, 0, s, hi, cols);
    else rc = colred_run<unsigned short, unsigned short, CR_ROWN>(r, 1, work, lo, 0, s, hi, cols);
    if (rc) return rc;
  }
  return HV_OK;
}

extern "C" int hv_act_backward(int dtype, const void* dy, const void* pre, long n, int act, float drop_p,
                               unsigned int seed, const unsigned int* seed_offset, void* dpre, hv_stream_t stream) {
  if (!dy || !pre || !dpre || n <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_act_bwd<T><<<grid_for(n), 256, 0, (hipStream_t)stream>>>((const T*)dy, (const T*)pre, n, act,
                                                                                 drop_p, seed, seed_offset,
                                                                                 (T*)dpre)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_dropout(int dtype, const void* x, long n, float drop_p, unsigned int seed,
                          const unsigned int* seed_offset, void* y, hv_stream_t stream) {
  if (!x || !y || n <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_dropout<T><<<grid_for(n), 256, 0, (hipStream_t)stream>>>((const T*)x, n, drop_p, seed, seed_offset, (T*)y)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_chan_dot_work_floats(int n, int hw, int c) { return colred_work(hw, c, n, 1); }

extern "C" int hv_chan_dot(int dtype, const void* a, const void* b, int n, int hw, int c, float* out, float* work,
                           hv_stream_t stream) {
  if (!a || !out || !work || n <= 0 || hw <= 0 || c <= 0 || !colred_ok(c)) return HV_EINVAL;
  ColRed r{};
  r.a = a; r.b = b; r.rows = hw; r.cols = c;
  HV_DISPATCH(dtype, (colred_run<T, T, CR_DOT>(r, n, work, out, 0, (hipStream_t)stream)));
  return HV_OK;
}

extern "C" int hv_se_mlp_backward(const float* pooled, const float* dgate, int n, int c, int cr, const float* w1,
                                  const float* b1, const float* w2, const float* b2, float* dpooled, float* dw1,
                                  float* db1, float* dw2, float* db2, float* work, hv_stream_t stream) {
  if (!pooled || !dgate || !dpooled || !work || n <= 0 || c <= 0 || cr <= 0) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  k_se_bwd_img<<<n, 256, (size_t)(cr + c) * sizeof(float), s>>>(pooled, dgate, c, cr, w1, b1, w2, b2, dpooled, work);
  k_se_bwd_params<<<grid_for(2L * c * cr + c + cr), 256, 0, s>>>(pooled, work, n, c, cr, dw1, db1, dw2, db2);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_se_backward_apply(int dtype, const void* dout, const float* gate, const float* dpooled, int n,
                                    int hw, int c, void* dy, hv_stream_t stream) {
  if (!dout || !gate || !dpooled || !dy) return HV_EINVAL;
  const long total = (long)n * hw * c;
  HV_DISPATCH(dtype, (k_se_bwd_apply<T><<<grid_for(total), 256, 0, (hipStream_t)stream>>>(
                         (const T*)dout, gate, dpooled, hw, c, total, 1.0f / hw, (T*)dy)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_maxpool2x2_backward(int dtype, const void* x, const void* dy, int n, int h, int w, int c, void* dx,
                                      hv_stream_t stream) {
  if (!x || !dy || !dx || (h & 1) || (w & 1)) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_maxpool_bwd<T><<<grid_for((long)n * (h / 2) * (w / 2) * c), 256, 0, (hipStream_t)stream>>>(
                         (const T*)x, (const T*)dy, n, h, w, c, (T*)dx)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_upsample_backward(int dtype, const void* dy, int n, int h, int w, int c, int hb, int wb, void* db,
                                    hv_stream_t stream) {
  if (!dy || !db || hb <= 0 || wb <= 0 || h % hb || w % wb) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_upsample_bwd<T><<<grid_for((long)n * hb * wb * c), 256, 0, (hipStream_t)stream>>>(
                         (const T*)dy, n, h, w, c, hb, wb, (T*)db)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_vit_assemble(int dtype, const void* x, const float* cls, const float* pos, int n, int tokens, int d,
                               void* z, hv_stream_t stream) {
  if (!x || !cls || !pos || !z) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_vit_assemble<T><<<grid_for((long)n * (tokens + 1) * d), 256, 0, (hipStream_t)stream>>>(
                         (const T*)x, cls, pos, n, tokens, d, (T*)z)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_vit_assemble_backward(int dtype, const void* dz, int n, int tokens, int d, void* dx, float* dcls,
                                        float* dpos, hv_stream_t stream) {
  if (!dz || !dx || !dcls || !dpos) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_vit_assemble_bwd<T><<<grid_for((long)(tokens + 1) * d), 256, 0, (hipStream_t)stream>>>(
                         (const T*)dz, n, tokens, d, (T*)dx, dcls, dpos)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_scatter_rows(int dtype, const void* dy, long stride_rows, int n, int c, void* dx,
                               hv_stream_t stream) {
  if (!dy || !dx || stride_rows <= 0) return HV_EINVAL;
  HV_DISPATCH(dtype, (k_scatter_rows<T><<<grid_for((long)n * stride_rows * c), 256, 0, (hipStream_t)stream>>>(
                         (const T*)dy, stride_rows, n, c, (T*)dx)));
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_yolo_loss_work_floats(int n, int h, int w, int A) {
  return 8 + (size_t)hv_cdiv((long)n * A * h * w, 256) * 4;
}

extern "C" int hv_yolo_loss(int dtype, const void* logits, const float* targets, int n, int h, int w, int A, int P,
                            float l_coord, float l_obj, float l_noobj, float l_cls, float* sums, int d_dtype,
                            void* dlogits, float* work, hv_stream_t stream) {
  if (!logits || !targets || !sums || !dlogits || !work || P < 6) return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const long cells = (long)n * A * h * w;
  float* nobj = work;
  float* part = work + 8;
  const unsigned nblk = hv_cdiv(cells, 256);
  k_fill_f32<<<1, 256, 0, s>>>(nobj, 1, 0.f);
  k_yolo_count<<<(unsigned)((cells + 255) / 256 < 1024 ? (cells + 255) / 256 : 1024), 256, 0, s>>>(targets, cells, P, nobj);
#define YL_LAUNCH(T, TD) k_yolo_loss<T, TD><<<nblk, 256, 0, s>>>((const T*)logits, targets, n, h, w, A, P, l_coord, \
      l_obj, l_noobj, l_cls, nobj, (TD*)dlogits, part)
  if (dtype == HV_F32 && d_dtype == HV_F32) YL_LAUNCH(float, float);
  else if (dtype == HV_BF16 && d_dtype == HV_BF16) YL_LAUNCH(unsigned short, unsigned short);
  else if (dtype == HV_BF16 && d_dtype == HV_F32) YL_LAUNCH(unsigned short, float);
  else if (dtype == HV_F32 && d_dtype == HV_BF16) YL_LAUNCH(float, unsigned short);
  else return HV_EINVAL;
#undef YL_LAUNCH
  k_yolo_final<<<1, 64, 0, s>>>(part, nblk, nobj, l_coord, l_obj, l_noobj, l_cls, sums);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_param_blocks(long n) { return (int)((n + PB_ELEMS - 1) / PB_ELEMS); }

extern "C" int hv_grad_norms(const hv_param_entry* tab, int count, int total_blocks, int groups,
                             const float* max_norm, float* norms, float* coefs, float* work, const int* active,
                             hv_stream_t stream) {
  if (!tab || count <= 0 || total_blocks <= 0 || groups < 1 || groups > 4 || !max_norm || !norms || !coefs || !work)
    return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  k_grad_sq<<<total_blocks, 256, 0, s>>>(tab, count, active, work);
  float m[4] = {1.f, 1.f, 1.f, 1.f};
  for (int g = 0; g < groups; ++g) m[g] = max_norm[g];
  k_grad_norm_final<<<1, 256, 0, s>>>(total_blocks, work, groups, m[0], m[1], m[2], m[3], norms, coefs);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_adamw(const hv_param_entry* tab, int count, int total_blocks, const float* coefs, float lr,
                        float beta1, float beta2, float eps, float weight_decay, int step, const int* steps,
                        const int* active, hv_stream_t stream) {
  if (!tab || count <= 0 || total_blocks <= 0 || (step < 1 && !steps)) return HV_EINVAL;
  const float bc1 = 1.f - powf(beta1, (float)max(step, 1));
  const float bc2s = sqrtf(1.f - powf(beta2, (float)max(step, 1)));
  k_adamw<<<total_blocks, 256, 0, (hipStream_t)stream>>>(tab, count, coefs, lr, beta1, beta2, eps, weight_decay, bc1,
                                                         bc2s, steps, active, nullptr);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" int hv_adamw_dev(const hv_param_entry* tab, int count, int total_blocks, const float* coefs,
                            const float* hyper, const int* steps, const int* active, hv_stream_t stream) {
  if (!tab || count <= 0 || total_blocks <= 0 || !hyper || !steps) return HV_EINVAL;
  k_adamw<<<total_blocks, 256, 0, (hipStream_t)stream>>>(tab, count, coefs, 0.f, 0.f, 0.f, 0.f, 0.f, 1.f, 1.f, steps,
                                                         active, hyper);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_mhc_param_backward_work_floats(int D, int Hd) {
  return colred_ok(Hd) ? colred_work(D, Hd, 1, 1) + Hd : (size_t)red_chunks(D) * Hd + Hd;
}

extern "C" int hv_mhc_param_backward(int D, int Hd, const float* dgc, const float* du, const float* h_pre_raw,
                                     const float* gamma_pre, const float* beta_pre, const float* dwc_x,
                                     const float* dwc_h, const float* h_post_raw, float* dh_pre_raw, float* dgamma,
                                     float* dbeta, float* dh_res, float* dh_post_raw, float* work,
                                     hv_stream_t stream) {
  if (!dgc || !du || !h_pre_raw || !dwc_x || !dwc_h || !h_post_raw || !dh_pre_raw || !dgamma || !dbeta || !dh_res ||
      !dh_post_raw || !work || D <= 0 || Hd <= 0)
    return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const size_t wpart = colred_ok(Hd) ? colred_work(D, Hd, 1, 1) : (size_t)red_chunks(D) * Hd;
  float* colsum = work + wpart;
  const int rc = hv_colsum(HV_F32, dgc, Hd, D, Hd, colsum, 0, work, stream);
  if (rc) return rc;
  k_mhc_pre_bwd<<<hv_cdiv(D, 4), 256, 0, s>>>(dgc, colsum, du, h_pre_raw, gamma_pre, beta_pre, D, Hd, dh_pre_raw,
                                               dgamma, dbeta);
  k_mhc_post_bwd<<<hv_cdiv(D + Hd, 4), 256, 0, s>>>(dwc_x, dwc_h, h_post_raw, D, Hd, dh_res, dh_post_raw);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
