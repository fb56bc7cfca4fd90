// Detection post-processing on the GPU: YOLODetectionHead.post_process +
// non_max_suppression (reference yolo_head.py:571-731), the whole batch in two launches with no
// host round trip per box (the reference does one .item() per kept box).
//
// Stage 1, one workgroup per (image, scale): candidates with class_score > conf_thr, sorted by
// score exactly as the reference's torch.sort leaves them (below), then greedy NMS: the best
// remaining box is kept and every remaining box with IoU >= iou_thr (the reference keeps
// IoU < thr) is suppressed, until max_det are kept or none remain.  Stage 2, one workgroup per
// image: the same over the concatenation of the per-scale survivors (scale 0 first, each in kept
// order), the reference's final cross-scale pass.  IoU exactly as compute_iou
// (yolo_head.py:733-750): inter / (area1 + area2 - inter + 1e-6).
//
// The order.  Up to NMS_BITONIC candidates are compacted into LDS (any order) and bitonic-sorted
// by (score, index); with no two scores equal that is the only sorted order, so it is the
// reference's.  With ties, or more candidates, the reference's UNSTABLE order is rebuilt: the
// candidates in cell order go through a restatement of libstdc++'s introsort (exact_sort below)
// -- only over the prefix the greedy reads (NMS_PREFIX0, widened 4x whenever the greedy runs off
// it before max_det), and in LDS once the segments meeting that prefix fit there.  The greedy
// decides 64 candidates per step from an IoU bit matrix (greedy below), reading boxes from an
// LDS cache; suppressed candidates are marked in place (the index's sign bit) and the kept ones
// are written out at the end in parallel.  Neither the candidate count nor max_det has a cap.
#include "hv_common.h"
#include <climits>

namespace {

constexpr int NMS_CAP = 6144;       // candidates held in LDS per segment (48 KiB): the exact sort's
                                    // window and the greedy's prefix when it fits
constexpr int NMS_THREADS = 1024;
constexpr int NMS_DEAD = INT_MIN;   // sign bit of Cand::idx: suppressed
constexpr int NMS_PREFIX0 = 1024;   // first prefix of the exact sort the greedy reads (widened 4x)
constexpr int NMS_XL = 6144;        // exact-sort window (and greedy box cache) held in LDS
constexpr int NMS_BITONIC = 2048;
constexpr int NMS_WAVE = 64;        // segments this small are finished by one wave in registers   // above: straight to the exact sort (as fast, and bf16 scores tie)

struct Cand {
  float score;
  int idx;                          // stage 1: flattened cell; stage 2: seg * max_det + k
};

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
  return a.score > b.score || (a.score == b.score && a.idx < b.idx);
}

__device__ __forceinline__ float iou(const float4 a, const float4 b) {
  const float ix1 = fmaxf(a.x, b.x), iy1 = fmaxf(a.y, b.y);
  const float ix2 = fminf(a.z, b.z), iy2 = fminf(a.w, b.w);
  const float inter = fmaxf(ix2 - ix1, 0.f) * fmaxf(iy2 - iy1, 0.f);
  const float a1 = (a.z - a.x) * (a.w - a.y);
  const float a2 = (b.z - b.x) * (b.w - b.y);
  return inter / (a1 + a2 - inter + 1e-6f);
}

__device__ __forceinline__ int pow2ceil(int n) {
  int m = 1;
  while (m < n) m <<= 1;
  return m;
}

__device__ __forceinline__ void cmpx(Cand* c, int i, int l, bool desc) {
  const Cand a = c[i], b = c[l];
  if (desc ? better(b, a) : better(a, b)) { c[i] = b; c[l] = a; }
}

// bitonic sort of c[0..n) in LDS (n <= NMS_BITONIC), best first; pads to a power of two
__device__ void lds_sort(Cand* c, int n) {
  const int m = pow2ceil(n);
  for (int i = n + threadIdx.x; i < m; i += blockDim.x) c[i] = Cand{-INFINITY, INT_MAX};
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) cmpx(c, i, l, (i & k) == 0);
      }
      __syncthreads();
    }
  }
}

// ---- exact restatement of the reference's sort -------------------------------------------------
// non_max_suppression sorts with torch.sort(scores, descending=True) (yolo_head.py:700), which on
// the CPU is libstdc++ std::sort (introsort) over (value, index) pairs with comp(a, b) =
// a.value > b.value -- NOT stable: for tied scores the kept order is whatever introsort leaves
// (oracle/std_sort.py restates it and pins it against torch.sort).  Scores without ties have one
// sorted order, so the bitonic sort above is exact for them; a segment with a tie (n > 16: up
// to 16 elements std::sort is an insertion sort, i.e. stable) is re-sorted here from its original
// order, reproducing introsort's permutation exactly but level-synchronously across the
// workgroup:
//  * every segment of one recursion level (all share the same depth_limit) is partitioned at
//    once.  After __move_median_to_first, Hoare's __unguarded_partition swaps the k-th "left
//    stopper" (position > first with !(v > pivot)) with the k-th "right stopper" (counted from
//    the end, !(pivot > v)) for k = 1..K while l_k < r_k, and returns cut = min(l_{K+1}, r_K)
//    (r_0 = inf): ranks come from two block-wide scans (prefix of left, suffix of right flags);
//  * depth_limit 0 -> that segment is heap-sorted (make_heap + sort_heap, serial per segment,
//    as __partial_sort does);
//  * __final_insertion_sort over the whole array only reorders within the <= 16-element leaves
//    (nothing on the right of a cut is strictly better than anything on its left), so it is a
//    stable insertion sort per leaf, one thread per leaf.
// The arrays live in the workspace (global memory, coherent within the workgroup across its
// barriers) while the segments that meet the prefix span more than NMS_XL positions; from then on
// that window moves to LDS (A into the candidate array, the index arrays as 16-bit) and the
// remaining levels -- most of them -- run there.
template <typename I>
struct XW {
  I *lo, *hi, *PL, *SR, *Lp, *Rp, *cut, *fl;   // each >= window + 1 entries
};
using u16 = unsigned short;
using XWork = XW<int>;
constexpr int XWORK_ARRAYS = 8;

template <typename I>
__device__ __forceinline__ XW<I> xw_at(I* base, long stride) {
  XW<I> w;
  w.lo = base; w.hi = base + stride; w.PL = base + 2 * stride; w.SR = base + 3 * stride;
  w.Lp = base + 4 * stride; w.Rp = base + 5 * stride; w.cut = base + 6 * stride; w.fl = base + 7 * stride;
  return w;
}

__device__ __forceinline__ bool xcomp(const Cand& a, const Cand& b) { return a.score > b.score; }

__device__ __forceinline__ void xswap(Cand* A, int i, int j) {
  const Cand t = A[i]; A[i] = A[j]; A[j] = t;
}

// std::__move_median_to_first(result, a, b, c)
__device__ void median_to_first(Cand* A, int r, int a, int b, int c) {
  if (xcomp(A[a], A[b])) {
    if (xcomp(A[b], A[c])) xswap(A, r, b);
    else if (xcomp(A[a], A[c])) xswap(A, r, c);
    else xswap(A, r, a);
  } else if (xcomp(A[a], A[c])) xswap(A, r, a);
  else if (xcomp(A[b], A[c])) xswap(A, r, c);
  else xswap(A, r, b);
}

// std::__adjust_heap + std::__push_heap on F[0..len)
__device__ void adjust_heap(Cand* F, int hole, int len, Cand value) {
  const int top = hole;
  int child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (xcomp(F[child], F[child - 1])) --child;
    F[hole] = F[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    F[hole] = F[child - 1];
    hole = child - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && xcomp(F[parent], value)) {
    F[hole] = F[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  F[hole] = value;
}

// std::__partial_sort(first, last, last) = make_heap + sort_heap
__device__ void heap_sort(Cand* F, int len) {
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      adjust_heap(F, parent, len, F[parent]);
      if (parent == 0) break;
    }
  }
  for (int last = len; last > 1;) {
    --last;
    const Cand v = F[last];
    F[last] = F[0];
    adjust_heap(F, 0, last, v);
  }
}

// stable insertion sort (std::__insertion_sort)
__device__ void insertion_sort(Cand* F, int len) {
  for (int i = 1; i < len; ++i) {
    const Cand v = F[i];
    int j = i;
    while (j > 0 && xcomp(v, F[j - 1])) { F[j] = F[j - 1]; --j; }
    F[j] = v;
  }
}

// exclusive scan of one value per thread in thread order; *total = the sum.  Two counts travel
// packed in one 64-bit value (low and high 32 bits), one scan for both.  One barrier: the wave
// totals alternate between two buffers by the caller's call counter `ph` (uniform over the
// workgroup), so a call never overwrites what a slow wave may still read from the previous one.
__device__ long long block_excl_scan(long long v, long long* total, int& ph) {
  __shared__ long long s_w[2][NMS_THREADS / 64];
  long long* sw = s_w[ph & 1];
  ++ph;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  long long x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sw[wv] = x;
  __syncthreads();
  long long before = 0, all = 0;
  for (int i = 0; i < nw; ++i) {
    const long long t = sw[i];
    before += i < wv ? t : 0;
    all += t;
  }
  *total = all;
  return before + x - v;
}

// ---- one segment of <= 64 positions sorted by one wave, in registers ----------------------------
// Lane j holds A[l + j]; every lane also holds its segment's bounds [slo, shi) (lane indices) and
// depth budget sd (-1 = heap-sorted), so all segments of the wave are partitioned at once with
// ballots instead of block barriers: the k-th left / right stopper of a segment is found by rank
// through a 64-entry per-wave LDS table, pairs swap through ds_bpermute.  Same permutation as the
// block levels (and std::sort); leaves end with a stable rank sort.
__device__ __forceinline__ float lane_f(float v, int src) { return __shfl(v, src); }
__device__ __forceinline__ int lane_i(int v, int src) { return __shfl(v, src); }
__device__ __forceinline__ float rl_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ void wl_f(float& v, int lane, float x) {   // lane `lane` := x (uniform)
  if ((int)(threadIdx.x & 63) == lane) v = x;
}
__device__ __forceinline__ void wl_i(int& v, int lane, int x) {
  if ((int)(threadIdx.x & 63) == lane) v = x;
}

// A heap-sort operand held by one wave: element e (uniform) lives in register e / 64 of lane
// e % 64 (x_wave_sort: one register).  (Four registers for the block levels' heap-sort fallback
// of segments up to 256 measured ~4x slower than the one-thread LDS form: every access is R
// readlanes plus selects on one dependent chain.)
template <int R>
struct WReg {
  float s[R];
  int x[R];
};

template <int R>
__device__ __forceinline__ float wr_s(const WReg<R>& w, int e) {
  float v = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if ((e >> 6) == r) v = rl_f(w.s[r], e & 63);
  return v;
}
template <int R>
__device__ __forceinline__ int wr_x(const WReg<R>& w, int e) {
  int v = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if ((e >> 6) == r) v = __builtin_amdgcn_readlane(w.x[r], e & 63);
  return v;
}
template <int R>
__device__ __forceinline__ void wr_set(WReg<R>& w, int e, float vs, int vi) {
#pragma unroll
  for (int r = 0; r < R; ++r)
    if ((e >> 6) == r) {
      wl_f(w.s[r], e & 63, vs);
      wl_i(w.x[r], e & 63, vi);
    }
}

// std::__adjust_heap on elements [a, a + len) of w, serially with uniform indices
template <int R>
__device__ void wave_adjust_heap(WReg<R>& w, int a, int hole, int len, float vs, int vi) {
  const int top = hole;
  int child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (wr_s(w, a + child) > wr_s(w, a + child - 1)) --child;
    wr_set(w, a + hole, wr_s(w, a + child), wr_x(w, a + child));
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    wr_set(w, a + hole, wr_s(w, a + child - 1), wr_x(w, a + child - 1));
    hole = child - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && wr_s(w, a + parent) > vs) {
    wr_set(w, a + hole, wr_s(w, a + parent), wr_x(w, a + parent));
    hole = parent;
    parent = (hole - 1) / 2;
  }
  wr_set(w, a + hole, vs, vi);
}

// std::__partial_sort(first, last, last) = make_heap + sort_heap on elements [a, a + len)
template <int R>
__device__ void wave_heap_sort(WReg<R>& w, int a, int len) {
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      wave_adjust_heap(w, a, parent, len, wr_s(w, a + parent), wr_x(w, a + parent));
      if (parent == 0) break;
    }
  }
  for (int last = len; last > 1;) {
    --last;
    const float vs = wr_s(w, a + last);
    const int vi = wr_x(w, a + last);
    wr_set(w, a + last, wr_s(w, a), wr_x(w, a));
    wave_adjust_heap(w, a, 0, last, vs, vi);
  }
}

// std::sort's treatment of the segment A[l, h) (h - l <= 64) with depth budget d, in one wave;
// LL / RR: this wave's 64-entry rank tables
__device__ void x_wave_sort(Cand* A, int l, int h, int d, unsigned char* LL, unsigned char* RR) {
  const int j = threadIdx.x & 63, m = h - l;
  float sc = -INFINITY;
  int ix = 0;
  if (j < m) { const Cand e = A[l + j]; sc = e.score; ix = e.idx; }
  int slo = j < m ? 0 : j, shi = j < m ? m : j + 1, sd = d;
  const unsigned long long below = (1ull << j) - 1, above = ~((2ull << j) - 1);
  for (;;) {
    const int sz = shi - slo;
    const bool act = sz > 16 && sd >= 0;
    if (!__ballot(act)) break;
    unsigned long long hz = __ballot(act && j == slo && sd == 0);
    while (hz) {                         // spent budgets: std::__partial_sort
      const int s0 = __builtin_ctzll(hz);
      hz &= hz - 1;
      const int e0 = __builtin_amdgcn_readlane(shi, s0);
      WReg<1> w1{{sc}, {ix}};
      wave_heap_sort(w1, s0, e0 - s0);
      sc = w1.s[0];
      ix = w1.x[0];
      if (j >= s0 && j < e0) sd = -1;
    }
    const bool part = act && sd > 0;
    // __move_median_to_first(slo, slo + 1, slo + sz / 2, shi - 1), per segment
    const int a = slo + 1, b = slo + sz / 2, c = shi - 1;
    const float va = lane_f(sc, a), vb = lane_f(sc, b), vc = lane_f(sc, c);
    int X;
    if (va > vb) X = vb > vc ? b : (va > vc ? c : a);
    else X = va > vc ? a : (vb > vc ? c : b);
    int src = j;
    if (part) src = j == slo ? X : (j == X ? slo : j);
    sc = lane_f(sc, src);
    ix = lane_i(ix, src);
    const float p = lane_f(sc, slo);
    const bool fL = part && j > slo && !(sc > p), fR = part && j > slo && !(p > sc);
    const unsigned long long bL = __ballot(fL), bR = __ballot(fR);
    const unsigned long long seg = (shi >= 64 ? ~0ull : ((1ull << shi) - 1)) & ~((1ull << slo) - 1);
    const int cntL = __popcll(bL & seg), cntR = __popcll(bR & seg);
    const int kL = __popcll(bL & seg & below) + 1, kR = __popcll(bR & seg & above) + 1;
    if (fL) LL[slo + kL] = (unsigned char)j;
    if (fR) RR[slo + kR] = (unsigned char)j;
    __builtin_amdgcn_wave_barrier();
    const int rP = fL && kL <= cntR ? (int)RR[slo + kL] : -1;
    const int lP = fR && kR <= cntL ? (int)LL[slo + kR] : 64;
    const bool swL = fL && rP > j, swR = fR && lP < j;
    const int K = __popcll(__ballot(swL) & seg);
    int cut = 0;
    if (part) cut = K == 0 ? (int)LL[slo + 1]
                           : (K + 1 <= cntL ? min((int)LL[slo + K + 1], (int)RR[slo + K]) : (int)RR[slo + K]);
    __builtin_amdgcn_wave_barrier();     // the tables are rewritten by the next level
    src = swL ? rP : (swR ? lP : j);
    sc = lane_f(sc, src);
    ix = lane_i(ix, src);
    if (part) {
      if (j < cut) shi = cut;
      else slo = cut;
      --sd;
    }
  }
  // __final_insertion_sort within the leaves: stable rank by score (heap-sorted runs stay put)
  int rank = j - slo;
  const bool leaf = sd >= 0 && shi - slo <= 16;
  if (__ballot(leaf & (j < m))) {
    int r = 0;
    for (int dd = 0; dd < 16; ++dd) {
      const int i = slo + dd;
      const float si = lane_f(sc, min(i, 63));
      if (i < shi) r += (si > sc) || (si == sc && i < j);
    }
    if (leaf) rank = r;
  }
  if (j < m) A[l + slo + rank] = Cand{sc, ix};
}

// Each segment carries its own std::sort depth budget, kept at Lp[head] (Lp[l + k] is written
// for k >= 1 only); X_DONE marks a segment the heap-sort fallback has finished.
template <typename I>
__device__ __forceinline__ I x_done() { return (I)~(I)0; }

template <typename I>
__device__ __forceinline__ bool x_active(int l, int h, int limit, I d) {
  return h - l > 16 && l < limit && d != x_done<I>();
}

constexpr int XHEAP_MAX = 8;
struct XHeap {                           // segments whose depth budget is spent, this level
  int n, l[XHEAP_MAX], h[XHEAP_MAX];
};

// one recursion level: every active segment of A[0, E) partitioned at once (see above); a segment
// whose budget is spent is heap-sorted instead (std::__partial_sort).  The split leaves s_any =
// "an active segment of more than NMS_WAVE remains" and s_end = the last active one's end (the
// caller alternates two pairs of them between levels, so the level never waits for their readers).
template <typename I>
__device__ void x_level(Cand* __restrict__ A, const XW<I> w, int E, int limit, int& s_any, int& s_end, int& ph,
                        XHeap& hp) {
  const int T = blockDim.x, t = threadIdx.x;
  // distinct arrays: lets the compiler batch the loads of consecutive elements
  I* __restrict__ lo = w.lo; I* __restrict__ hi = w.hi; I* __restrict__ PL = w.PL; I* __restrict__ SR = w.SR;
  I* __restrict__ Lp = w.Lp; I* __restrict__ Rp = w.Rp; I* __restrict__ cut = w.cut; I* __restrict__ fl = w.fl;
  for (int i = t; i < E; i += T) {       // pivots: __unguarded_partition_pivot (or the heap sort)
    const int l = lo[i], h = hi[i];
    if (l != i) continue;
    const I d = Lp[l];
    if (!x_active(l, h, limit, d)) continue;
    if (d == 0) {
      const int slot = h - l <= (int)blockDim.x ? atomicAdd(&hp.n, 1) : XHEAP_MAX;
      if (slot < XHEAP_MAX) {
        hp.l[slot] = l;                  // the whole workgroup takes it below
        hp.h[slot] = h;
      } else {
        heap_sort(A + l, h - l);
        Lp[l] = x_done<I>();
      }
    } else {
      median_to_first(A, l, l + 1, l + (h - l) / 2, h - 1);
    }
  }
  __syncthreads();
  // spent budgets of up to blockDim.x positions: with no two scores equal the heap sort's result
  // is THE sorted order, so a parallel rank sort gives it exactly; any tie -> the serial heap sort
  // (its tie order is what std::sort leaves)
  for (int q = 0, nq = min(hp.n, XHEAP_MAX); q < nq; ++q) {
    const int l = hp.l[q], m = hp.h[q] - l;
    Cand e{0.f, 0};
    int rank = 0, tie = 0;
    if (t < m) {
      e = A[l + t];
      for (int j = 0; j < m; ++j) {
        const float v = A[l + j].score;
        rank += v > e.score;
        tie |= v == e.score && j != t;
      }
    }
    if (!__syncthreads_or(tie)) {        // (also: every read of the segment is done)
      if (t < m) A[l + rank] = e;
    } else if (t == 0) {
      heap_sort(A + l, m);
    }
    if (t == 0) Lp[l] = x_done<I>();
    __syncthreads();
  }
  if (t == 0) hp.n = 0;                  // next read after this level's barriers
  if (t == 0) SR[E] = 0;
  __syncthreads();
  const int C = (E + T - 1) / T;
  const int c0 = min(E, t * C), c1 = min(E, c0 + C);
  int cL = 0, cR = 0;                    // stopper flags over this thread's chunk
#pragma unroll 4
  for (int i = c0; i < c1; ++i) {
    const int l = lo[i], h = hi[i];
    int f = 0;
    if (i > l && x_active(l, h, limit, Lp[l])) {
      const float p = A[l].score, v = A[i].score;
      f = (!(v > p) ? 1 : 0) | (!(p > v) ? 2 : 0);
    }
    fl[i] = f;
    cL += f & 1;
    cR += f >> 1;
  }
  long long tot2;
  const long long ex2 = block_excl_scan((long long)cL | ((long long)cR << 32), &tot2, ph);
  const int exL = (int)(ex2 & 0xffffffffLL), exR = (int)(ex2 >> 32), totR = (int)(tot2 >> 32);
  int run = exL;                         // PL[i] = left stoppers in [0, i]
#pragma unroll 4
  for (int i = c0; i < c1; ++i) { run += fl[i] & 1; PL[i] = run; }
  run = totR - exR - cR;                 // SR[i] = right stoppers in [i, E)
#pragma unroll 4
  for (int i = c1 - 1; i >= c0; --i) { run += fl[i] >> 1; SR[i] = run; }
  __syncthreads();
  for (int i = t; i < E; i += T) {       // l_k, r_k by rank within the segment
    const int f = fl[i];
    if (!f) continue;
    const int l = lo[i], h = hi[i];
    if (f & 1) Lp[l + PL[i] - PL[l]] = i;
    if (f & 2) Rp[l + SR[i] - SR[h]] = i;
  }
  __syncthreads();
  for (int i = t; i < E; i += T) {       // the swaps (disjoint pairs) and each segment's cut
    if (!(fl[i] & 1)) continue;
    const int l = lo[i], h = hi[i];
    const int k = PL[i] - PL[l];
    const int cntL = PL[h - 1] - PL[l], cntR = SR[l + 1] - SR[h];
    const int r = k <= cntR ? (int)Rp[l + k] : -1;
    int ct = -1;
    if (r > i) {
      xswap(A, i, r);
      const bool next = k + 1 <= cntL && k + 1 <= cntR && Lp[l + k + 1] < Rp[l + k + 1];
      if (!next) ct = k + 1 <= cntL ? min((int)Lp[l + k + 1], r) : r;
    } else if (k == 1) {
      ct = i;                            // no swap at all: cut = l_1
    }
    if (ct >= 0) {
      cut[l] = ct;
      Rp[l] = Lp[l] - 1;                 // the children's budget (Rp[l + k]: k >= 1 only)
    }
  }
  if (t == 0) { s_any = 0; s_end = 0; }
  __syncthreads();
  for (int i = t; i < E; i += T) {       // [first, cut) and [cut, last), one level deeper
    const int l = lo[i], h = hi[i];
    if (!x_active(l, h, limit, Lp[l])) continue;   // Lp[l] may already be the child's: same test
    const int c = cut[l];
    const int nl = i < c ? l : c, nh = i < c ? c : h;
    lo[i] = nl;
    hi[i] = nh;
    if (i == nl) {                       // one thread per new segment
      const I d = Rp[l];
      Lp[nl] = d;
      if (x_active(nl, nh, limit, d)) {
        atomicMax(&s_end, nh);
        if (nh - nl > NMS_WAVE) s_any = 1;   // smaller ones finish in x_wave_phase
      }
    }
  }
  __syncthreads();
}

// every active segment of [0, E) (all <= NMS_WAVE here): one wave each, waves over head chunks
template <typename I>
__device__ void x_wave_phase(Cand* A, const XW<I> w, int E, int limit) {
  __shared__ unsigned char s_rank[NMS_THREADS / 64][2][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int base = wv * 64; base < E; base += nw * 64) {
    const int i = base + lane;
    int h = 0, d = 0;
    bool hd = false;
    if (i < E) {
      const int l = w.lo[i];
      h = w.hi[i];
      if (l == i) {
        const I dd = w.Lp[l];
        hd = x_active(l, h, limit, dd);
        d = (int)dd;
      }
    }
    unsigned long long hm = __ballot(hd);
    while (hm) {
      const int s0 = __builtin_ctzll(hm);
      hm &= hm - 1;
      x_wave_sort(A, base + s0, __builtin_amdgcn_readlane(h, s0), __builtin_amdgcn_readlane(d, s0),
                  s_rank[wv][0], s_rank[wv][1]);
    }
  }
  __syncthreads();
}

// __final_insertion_sort = a stable sort of every leaf meeting the prefix [0, P)
template <typename I>
__device__ void x_leaves(Cand* A, const XW<I> w, int P) {
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const int l = w.lo[i], h = w.hi[i];
    if (l == i && h - l <= 16) insertion_sort(A + l, h - l);
  }
  __syncthreads();
}

// Hoare partition of the ONE segment A[l, h) (global) with all threads: the straddler phase of
// exact_sort.  Waves own contiguous runs of 64-position rounds (coalesced), stopper ranks come
// from ballots plus one scan of the wave totals, and the k-th pair is read by rank (coalesced).
// Returns the cut (std::__unguarded_partition_pivot).
__device__ int x_partition1(Cand* __restrict__ A, int l, int h, const XWork w, int& ph) {
  __shared__ int s_cut;
  const int T = blockDim.x, t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = T >> 6;
  int* __restrict__ Lp = w.Lp;
  int* __restrict__ Rp = w.Rp;
  if (t == 0) median_to_first(A, l, l + 1, l + (h - l) / 2, h - 1);
  __syncthreads();
  const float p = A[l].score;
  const int rounds = (h - l - 1 + 63) >> 6, rpw = (rounds + nw - 1) / nw;
  const int r0 = min(rounds, wv * rpw), r1 = min(rounds, r0 + rpw);
  const unsigned long long below = (1ull << lane) - 1;
  int cL = 0, cR = 0;
  for (int r = r0; r < r1; ++r) {
    const int i = l + 1 + (r << 6) + lane;
    bool fL = false, fR = false;
    if (i < h) { const float v = A[i].score; fL = !(v > p); fR = !(p > v); }
    cL += __popcll(__ballot(fL));
    cR += __popcll(__ballot(fR));
  }
  long long tot;                         // lane 63 carries its wave's counts: every lane gets the
  const long long ex = block_excl_scan(lane == 63 ? (long long)cL | ((long long)cR << 32) : 0, &tot, ph);
  int bL = (int)(ex & 0xffffffffLL), bR = (int)(ex >> 32);   // ... counts of the waves before it
  const int totL = (int)(tot & 0xffffffffLL), totR = (int)(tot >> 32);
  for (int r = r0; r < r1; ++r) {
    const int i = l + 1 + (r << 6) + lane;
    bool fL = false, fR = false;
    if (i < h) { const float v = A[i].score; fL = !(v > p); fR = !(p > v); }
    const unsigned long long mL = __ballot(fL), mR = __ballot(fR);
    if (fL) Lp[1 + bL + __popcll(mL & below)] = i;          // k-th left stopper from the left
    if (fR) Rp[totR - bR - __popcll(mR & below)] = i;       // k-th right stopper from the right
    bL += __popcll(mL);
    bR += __popcll(mR);
  }
  __syncthreads();
  for (int k = 1 + t; k <= totL; k += T) {
    const int i = Lp[k];
    const int r = k <= totR ? Rp[k] : -1;
    if (r > i) {
      xswap(A, i, r);
      const bool next = k + 1 <= totL && k + 1 <= totR && Lp[k + 1] < Rp[k + 1];
      if (!next) s_cut = k + 1 <= totL ? min(Lp[k + 1], r) : r;
    } else if (k == 1) {
      s_cut = i;
    }
  }
  __syncthreads();
  return s_cut;
}

// A[0..n) (global) in its ORIGINAL order -> std::sort's permutation of positions [0, limit): a
// segment lying wholly at or past `limit` is never partitioned further (what std::sort does there
// cannot move anything into the prefix: every element left of a cut is >= every element right of
// it), so the greedy NMS -- which reads the sorted order front to back and usually stops at
// max_det long before the end -- only pays for the top levels over all n plus the prefix.
// Segments are independent, each with its own depth budget, so the order they are partitioned
// in does not matter:
//  * straddler phase (n > NMS_XL >= limit): only the segment holding position limit-1 is
//    partitioned while it reaches past NMS_XL; the pieces left of it wait in a list;
//  * then every segment meeting the prefix is partitioned level-synchronously, in LDS (c and wl)
//    once they all lie in [0, NMS_XL), in the workspace before that.
// Returns true when the sorted prefix is in c, false when it is in A.  depth < 0: std::sort's
// own limit 2 * floor(log2 n); otherwise forced (tests reach the heap-sort fallback with it).
__device__ bool exact_sort(Cand* A, int n, const XWork wg, Cand* c, const XW<u16> wl, int depth, int limit,
                           int& ph) {
  constexpr int XSEG_MAX = 64;           // > 2 log2(2^30): one piece per straddler level
  __shared__ int s_any[2], s_end[2], s_win[2];
  __shared__ XHeap s_heap;
  __shared__ int s_seg[XSEG_MAX][3];     // (l, h, depth) of the waiting pieces
  const int T = blockDim.x, t = threadIdx.x;
  const int P = min(n, limit);
  if (depth < 0) depth = n > 0 ? 2 * (31 - __clz(n)) : 0;
  int sl = 0, sh = n, sd = depth, nseg = 0;      // the straddler (uniform)
  if (n > NMS_XL && P <= NMS_XL) {
    while (sh > NMS_XL && sh - sl > 16 && sd > 0 && nseg < XSEG_MAX - 1) {
      const int ct = x_partition1(A, sl, sh, wg, ph);
      --sd;
      if (ct <= P - 1) {                 // [sl, ct) lies in the prefix: it waits
        if (t == 0) { s_seg[nseg][0] = sl; s_seg[nseg][1] = ct; s_seg[nseg][2] = sd; }
        ++nseg;
        sl = ct;
      } else {
        sh = ct;                         // [ct, sh) lies past the prefix: never read
      }
    }
    if (t == 0) { s_seg[nseg][0] = sl; s_seg[nseg][1] = sh; s_seg[nseg][2] = sd; }
    ++nseg;
  } else {
    if (t == 0) { s_seg[0][0] = 0; s_seg[0][1] = n; s_seg[0][2] = depth; }
    nseg = 1;
  }
  __syncthreads();
  const int W0 = sh;                     // every piece lies in [0, W0)
  bool inl = W0 <= NMS_XL;
  if (inl)
    for (int i = t; i < W0; i += T) c[i] = A[i];
  int any = 0;
  for (int s = 0; s < nseg; ++s) {
    const int l = s_seg[s][0], h = s_seg[s][1], d = s_seg[s][2];
    for (int i = l + t; i < h; i += T) {
      if (inl) { wl.lo[i] = (u16)l; wl.hi[i] = (u16)h; }
      else { wg.lo[i] = l; wg.hi[i] = h; }
    }
    if (t == 0) {
      if (inl) wl.Lp[l] = (u16)d;
      else wg.Lp[l] = d;
    }
    any |= h - l > NMS_WAVE && l < limit;
  }
  if (t == 0) { s_any[0] = any; s_end[0] = W0; s_heap.n = 0; }
  __syncthreads();
  int Ew = W0;                            // the active segments' extent for the wave phase
  for (int lv = 0;; ++lv) {
    const int q = lv & 1;
    if (!s_any[q]) {
      Ew = s_end[q];
      break;
    }
    const int E = s_end[q];              // positions past E belong to no active segment
    if (inl) {
      x_level(c, wl, E, limit, s_any[q ^ 1], s_end[q ^ 1], ph, s_heap);
      continue;
    }
    x_level(A, wg, E, limit, s_any[q ^ 1], s_end[q ^ 1], ph, s_heap);
    // the window: every segment meeting [0, P) ends by the active ones' end or P-1's segment's
    if (t == 0) s_win[q] = max(s_end[q ^ 1], P > 0 ? wg.hi[P - 1] : 0);   // s_end = 0: none active
    __syncthreads();
    const int W = s_win[q];
    if (W <= NMS_XL) {
      for (int i = t; i < W; i += T) {
        c[i] = A[i];
        wl.lo[i] = (u16)wg.lo[i];
        wl.hi[i] = (u16)wg.hi[i];
        wl.Lp[i] = (u16)wg.Lp[i];        // the budgets at the heads (the rest is not read)
      }
      __syncthreads();
      inl = true;
    }
  }
  if (inl) {
    x_wave_phase(c, wl, Ew, limit);
    x_leaves(c, wl, P);
  } else {
    x_wave_phase(A, wg, Ew, limit);
    x_leaves(A, wg, P);
  }
  return inl;
}

// any equal neighbours among sorted c[0..n)?  (n <= 16: std::sort is then stable anyway)
__device__ bool has_ties(const Cand* c, int n) {
  int tie = 0;
  if (n > 16)
    for (int i = 1 + threadIdx.x; i < n; i += blockDim.x) tie |= c[i].score == c[i - 1].score;
  return __syncthreads_or(tie);
}

// greedy NMS over sorted c[0..n) (LDS or global), 64 candidates (one wave's ballot) at a time:
//  * all waves: the tile's 64x64 "row suppresses later column" bit matrix (IoU >= thr), beside
//    the sweep that suppresses every candidate from this tile on by the previous tile's kept boxes
//    (so each candidate has met every kept box of the earlier tiles before its tile is decided);
//  * wave 0: the sequential greedy over the tile with scalar bit operations -- the lowest live
//    candidate is kept and its row clears the ones it suppresses -- stopping at max_det.
// That is the one-box-at-a-time greedy exactly, with two barriers per 64 candidates instead of
// one per kept box.  box(idx) -> the candidate's xyxy box, cached in LDS (bc) for the first
// NMS_XL positions.  Suppressed candidates are marked in place, so the kept boxes are the
// unsuppressed positions of c[0..*last] (emit_kept writes them).  Returns the kept count.
template <typename BoxFn>
__device__ int greedy(Cand* c, int n, float iou_thr, int max_det, float4* bc, BoxFn box, int* last) {
  __shared__ unsigned long long s_row[64];
  __shared__ float4 s_kb[2][64];         // the kept boxes of a tile, by tile parity
  __shared__ int s_kn[2], s_kept, s_last;
  const int T = blockDim.x, t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = T >> 6;
  *last = -1;
  if (n <= 0) return 0;
  const int nb = min(n, NMS_XL);
  for (int i = t; i < nb; i += T) bc[i] = box(c[i].idx);
  if (t == 0) { s_kn[0] = s_kn[1] = 0; s_kept = 0; s_last = -1; }
  __syncthreads();
  auto boxat = [&](int i) { return i < nb ? bc[i] : box(c[i].idx & INT_MAX); };
  for (int t0 = 0, tp = 0; t0 < n; t0 += 64, tp ^= 1) {
    const int kn = s_kn[tp ^ 1];
    for (int i = t0 + t; kn > 0 && i < n; i += T) {
      const int id = c[i].idx;
      if (id < 0) continue;
      const float4 bx = boxat(i);
      for (int k = 0; k < kn; ++k)
        if (!(iou(s_kb[tp ^ 1][k], bx) < iou_thr)) { c[i].idx = id | NMS_DEAD; break; }
    }
    for (int r = wv; r < 64; r += nw) {
      const int pr = t0 + r, pc = t0 + lane;
      bool sup = false;
      if (pc < n && lane > r && c[pr].idx >= 0) sup = !(iou(boxat(pr), boxat(pc)) < iou_thr);
      const unsigned long long m = __ballot(sup);
      if (lane == 0) s_row[r] = m;
    }
    __syncthreads();
    if (wv == 0) {                       // the sequential greedy over the tile
      const int i = t0 + lane;
      const bool live = i < n && c[i].idx >= 0;
      const unsigned long long row = s_row[lane];
      unsigned long long alive = __ballot(live), keep = 0;
      int kept = s_kept;
      while (alive && kept < max_det) {
        const int j = __builtin_ctzll(alive);
        keep |= 1ull << j;
        ++kept;
        const unsigned rlo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)row, j);
        const unsigned rhi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(row >> 32), j);
        alive &= ~(((unsigned long long)rhi << 32) | rlo) & ~(1ull << j);
      }
      const bool kp = (keep >> lane) & 1;
      if (live && !kp) c[i].idx |= NMS_DEAD;   // suppressed (or past the max_det-th: unread)
      if (kp) s_kb[tp][__popcll(keep & ((1ull << lane) - 1))] = boxat(i);
      if (lane == 0) {
        s_kn[tp] = __popcll(keep);
        s_kept = kept;
        if (keep) s_last = t0 + 63 - __builtin_clzll(keep);
      }
    }
    __syncthreads();
    if (s_kept >= max_det) break;
  }
  *last = s_last;
  const int kept = s_kept;
  __syncthreads();                       // s_* are reused by the next call
  return kept;
}

// emit(k, pos) for the k-th unsuppressed position of c[0..last], all threads at once
template <typename EmitFn>
__device__ void emit_kept(const Cand* c, int last, EmitFn emit, int& ph) {
  const int m = last + 1, T = blockDim.x;
  const int C = (m + T - 1) / T;
  const int c0 = min(m, (int)threadIdx.x * C), c1 = min(m, c0 + C);
  int cnt = 0;
  for (int i = c0; i < c1; ++i) cnt += c[i].idx >= 0;
  long long tot;
  int k = (int)block_excl_scan(cnt, &tot, ph);
  for (int i = c0; i < c1; ++i)
    if (c[i].idx >= 0) emit(k++, i);
}

// LDS of the three kernels: the candidate array, then the sort window's index arrays (reused
// as the greedy's box cache)
constexpr size_t NMS_AUX_BYTES = (size_t)XWORK_ARRAYS * (NMS_XL + 1) * sizeof(u16);
constexpr size_t NMS_LDS = (size_t)NMS_CAP * sizeof(Cand) + NMS_AUX_BYTES;
static_assert(NMS_AUX_BYTES >= NMS_XL * sizeof(float4), "box cache fits the index arrays");
static_assert(NMS_XL <= NMS_CAP && NMS_XL < 65536, "window indices are 16-bit");

struct NmsSmem {
  Cand* c;
  XW<u16> wl;
  float4* bc;
};

__device__ __forceinline__ NmsSmem nms_smem() {
  extern __shared__ __attribute__((aligned(16))) unsigned char nms_sm[];
  NmsSmem m;
  m.c = reinterpret_cast<Cand*>(nms_sm);
  u16* aux = reinterpret_cast<u16*>(nms_sm + (size_t)NMS_CAP * sizeof(Cand));
  m.wl = xw_at(aux, NMS_XL + 1);
  m.bc = reinterpret_cast<float4*>(aux);
  return m;
}

__global__ void __launch_bounds__(NMS_THREADS) k_nms_scale(const hv_nms_scale* __restrict__ scales, int nscales,
                                                           float conf_thr, float iou_thr, int max_det,
                                                           Cand* __restrict__ gcand, int* __restrict__ gx,
                                                           long seg_stride, float* sboxes, float* sscores,
                                                           int64_t* slabels, int* scount) {
  const NmsSmem sm = nms_smem();
  Cand* c = sm.c;
  __shared__ int s_n;
  const int sc = blockIdx.x % nscales, b = blockIdx.x / nscales;
  const long seg = (long)blockIdx.x;
  const hv_nms_scale S = scales[sc];
  const long cells = S.cells;
  const float* score = S.class_scores + (long)b * cells;
  Cand* g = gcand + seg * seg_stride;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  // capacity: the caller's max_cells >= every scale's cells makes it >= cells (the contract);
  // a smaller one keeps the stores in bounds (candidates past it are dropped)
  const int cap = (int)min((long)INT_MAX, seg_stride);
  for (long i = threadIdx.x; i < cells; i += blockDim.x) {
    const float v = score[i];
    if (v > conf_thr) {
      const int slot = atomicAdd(&s_n, 1);
      if (slot < NMS_BITONIC) c[slot] = Cand{v, (int)i};   // more: the exact path re-compacts
    }
  }
  __syncthreads();
  const int n = min(s_n, cap);
  const float4* boxes = reinterpret_cast<const float4*>(S.boxes) + (long)b * cells;
  const int64_t* lab = S.class_indices + (long)b * cells;
  auto box = [&](int id) { return boxes[id]; };
  auto emit_from = [&](const Cand* src) {
    return [=](int k, int pos) {
      const Cand e = src[pos];
      reinterpret_cast<float4*>(sboxes)[seg * max_det + k] = boxes[e.idx];
      sscores[seg * max_det + k] = e.score;
      slabels[seg * max_det + k] = lab[e.idx];
    };
  };
  int kept = 0, last = -1, ph = 0;         // ph: scan calls (block_excl_scan)
  bool exact = n > NMS_BITONIC;            // std::sort's order straight away
  if (!exact) {
    lds_sort(c, n);
    exact = has_ties(c, n);                // distinct scores: the one sorted order is the reference's
    if (!exact) {
      kept = greedy(c, n, iou_thr, max_det, sm.bc, box, &last);
      emit_kept(c, last, emit_from(c), ph);
    }
  }
  if (exact) {
    // the reference's order (ties included): the masked candidates in cell order, std::sort
    // restated over the prefix the greedy reads; a greedy that runs off the prefix before
    // max_det widens it 4x and starts over (deterministic)
    const XWork xw = xw_at(gx + seg * XWORK_ARRAYS * (seg_stride + 1), seg_stride + 1);
    for (int limit = min(n, NMS_PREFIX0);; limit = min(n, 4 * limit)) {
      const long C = (cells + blockDim.x - 1) / blockDim.x;
      const long c0 = min(cells, (long)threadIdx.x * C), c1 = min(cells, c0 + C);
      int cnt = 0;
      for (long i = c0; i < c1; ++i) cnt += score[i] > conf_thr;
      long long tot;
      int o = (int)block_excl_scan(cnt, &tot, ph);
      for (long i = c0; i < c1; ++i) {
        const float v = score[i];
        if (v > conf_thr && o < cap) g[o] = Cand{v, (int)i};
        o += v > conf_thr;
      }
      __syncthreads();
      Cand* src = exact_sort(g, n, xw, c, sm.wl, -1, limit, ph) ? c : g;
      if (src == g && limit <= NMS_CAP) {  // the greedy reads the prefix from LDS
        for (int i = threadIdx.x; i < limit; i += blockDim.x) c[i] = g[i];
        __syncthreads();
        src = c;
      }
      kept = greedy(src, limit, iou_thr, max_det, sm.bc, box, &last);
      emit_kept(src, last, emit_from(src), ph);
      if (kept >= max_det || limit == n) break;
    }
  }
  if (threadIdx.x == 0) scount[seg] = kept;
}

// stage 2: per image, NMS over the concatenated per-scale survivors
__global__ void __launch_bounds__(NMS_THREADS) k_nms_final(int nscales, float iou_thr, int max_det,
                                                           const float* sboxes, const float* sscores,
                                                           const int64_t* slabels, const int* scount,
                                                           Cand* __restrict__ gcand, int* __restrict__ gx,
                                                           long img_stride, float* boxes, float* scores,
                                                           int64_t* labels, int* count) {
  const NmsSmem sm = nms_smem();
  Cand* c = sm.c;
  const int b = blockIdx.x;
  int n = 0;
  for (int s = 0; s < nscales; ++s) n += scount[b * nscales + s];
  Cand* g = gcand + (long)b * img_stride;
  // concatenation order: scale 0's survivors, then scale 1's, ... (idx = seg * max_det + k)
  auto gather = [&](Cand* dst) {
    int off = 0;
    for (int s = 0; s < nscales; ++s) {
      const int seg = b * nscales + s;
      const int cnt = scount[seg];
      for (int k = threadIdx.x; k < cnt; k += blockDim.x)
        dst[off + k] = Cand{sscores[(long)seg * max_det + k], seg * max_det + k};
      off += cnt;
    }
    __syncthreads();
  };
  const float4* sb = reinterpret_cast<const float4*>(sboxes);
  auto box = [&](int id) { return sb[id]; };
  float4* ob = reinterpret_cast<float4*>(boxes) + (long)b * max_det;
  auto emit_from = [&](const Cand* src) {
    return [=](int k, int pos) {
      const int from = src[pos].idx;
      ob[k] = sb[from];
      scores[(long)b * max_det + k] = sscores[from];
      labels[(long)b * max_det + k] = slabels[from];
    };
  };
  int kept = 0, last = -1, ph = 0;
  bool exact = n > NMS_BITONIC;
  if (!exact) {
    gather(c);
    lds_sort(c, n);       // idx grows with the concatenation order
    exact = has_ties(c, n);
    if (!exact) {
      kept = greedy(c, n, iou_thr, max_det, sm.bc, box, &last);
      emit_kept(c, last, emit_from(c), ph);
    }
  }
  if (exact) {            // as stage 1: std::sort's order over the prefix the greedy reads
    const XWork xw = xw_at(gx + (long)b * XWORK_ARRAYS * (img_stride + 1), img_stride + 1);
    for (int limit = min(n, NMS_PREFIX0);; limit = min(n, 4 * limit)) {
      gather(g);
      Cand* src = exact_sort(g, n, xw, c, sm.wl, -1, limit, ph) ? c : g;
      if (src == g && limit <= NMS_CAP) {
        for (int i = threadIdx.x; i < limit; i += blockDim.x) c[i] = g[i];
        __syncthreads();
        src = c;
      }
      kept = greedy(src, limit, iou_thr, max_det, sm.bc, box, &last);
      emit_kept(src, last, emit_from(src), ph);
      if (kept >= max_det || limit == n) break;
    }
  }
  // rows past `count` are zero, so the fixed-size outputs are a function of the inputs alone
  for (int k = kept + threadIdx.x; k < max_det; k += blockDim.x) {
    ob[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    scores[(long)b * max_det + k] = 0.f;
    labels[(long)b * max_det + k] = 0;
  }
  if (threadIdx.x == 0) count[b] = kept;
}

// torch.sort(vals, descending=True).indices on the CPU, exactly (one workgroup)
__global__ void __launch_bounds__(NMS_THREADS) k_sort_desc_exact(const float* vals, int n, int depth, int* out_idx,
                                                                 Cand* A, int* gx) {
  const NmsSmem sm = nms_smem();
  for (int i = threadIdx.x; i < n; i += blockDim.x) A[i] = Cand{vals[i], i};
  __syncthreads();
  int ph = 0;
  const Cand* src = exact_sort(A, n, xw_at(gx, (long)n + 1), sm.c, sm.wl, depth, n, ph) ? sm.c : A;
  for (int i = threadIdx.x; i < n; i += blockDim.x) out_idx[i] = src[i].idx;
}

// workspace layout: [stage-1 Cand regions][stage-1 sort scratch][stage-2 Cand regions]
//                   [stage-2 sort scratch][slabels int64][sboxes float4][sscores float][scount int]
struct NmsLayout {
  long seg_stride, img_stride;           // Cand elements per region (>= pow2ceil of the count)
  size_t cand1, x1, cand2, x2, labels, boxes, scores, counts, total;
};

size_t pow2ceil_host(long n) {
  size_t m = 1;
  while ((long)m < n) m <<= 1;
  return m;
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

NmsLayout nms_layout(int batch, int nscales, int max_det, long max_cells) {
  NmsLayout L{};
  const size_t segs = (size_t)batch * nscales;
  L.seg_stride = (long)pow2ceil_host(max_cells);
  L.img_stride = (long)pow2ceil_host((long)nscales * max_det);
  L.cand1 = 0;
  L.x1 = align256(L.cand1 + segs * L.seg_stride * sizeof(Cand));
  L.cand2 = align256(L.x1 + segs * XWORK_ARRAYS * (L.seg_stride + 1) * sizeof(int));
  L.x2 = align256(L.cand2 + (size_t)batch * L.img_stride * sizeof(Cand));
  L.labels = align256(L.x2 + (size_t)batch * XWORK_ARRAYS * (L.img_stride + 1) * sizeof(int));
  L.boxes = align256(L.labels + segs * max_det * sizeof(int64_t));
  L.scores = align256(L.boxes + segs * max_det * 4 * sizeof(float));
  L.counts = align256(L.scores + segs * max_det * sizeof(float));
  L.total = L.counts + segs * sizeof(int) + 256;
  return L;
}

bool nms_args_ok(int batch, int nscales, int max_det, long max_cells) {
  // candidate indices are int (stage 2: seg * max_det + k), and pow2 sort extents must fit too
  return batch > 0 && nscales > 0 && max_det > 0 && max_cells > 0 && max_cells <= (1L << 30) &&
         (long)batch * nscales * max_det <= (1L << 30);
}

void nms_lds_attrs() {
  static const bool done = [] {
    (void)hipFuncSetAttribute((const void*)k_nms_scale, hipFuncAttributeMaxDynamicSharedMemorySize, NMS_LDS);
    (void)hipFuncSetAttribute((const void*)k_nms_final, hipFuncAttributeMaxDynamicSharedMemorySize, NMS_LDS);
    (void)hipFuncSetAttribute((const void*)k_sort_desc_exact, hipFuncAttributeMaxDynamicSharedMemorySize, NMS_LDS);
    return true;
  }();
  (void)done;
}

}  // namespace

extern "C" size_t hv_nms_work_bytes(int batch, int nscales, int max_det, long max_cells) {
  if (!nms_args_ok(batch, nscales, max_det, max_cells)) return 0;
  return nms_layout(batch, nscales, max_det, max_cells).total;
}

extern "C" int hv_nms(const hv_nms_scale* dev_scales, int nscales, int batch, float conf_thr, float iou_thr,
                      int max_det, long max_cells, float* boxes, float* scores, int64_t* labels, int* count,
                      void* work, hv_stream_t stream) {
  if (!dev_scales || !nms_args_ok(batch, nscales, max_det, max_cells) || !boxes || !scores || !labels || !count ||
      !work)
    return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const NmsLayout L = nms_layout(batch, nscales, max_det, max_cells);
  unsigned char* w = (unsigned char*)work;
  const size_t segs = (size_t)batch * nscales;
  nms_lds_attrs();
  k_nms_scale<<<(unsigned)segs, NMS_THREADS, NMS_LDS, s>>>(dev_scales, nscales, conf_thr, iou_thr, max_det,
                                                      (Cand*)(w + L.cand1), (int*)(w + L.x1), L.seg_stride,
                                                      (float*)(w + L.boxes), (float*)(w + L.scores),
                                                      (int64_t*)(w + L.labels), (int*)(w + L.counts));
  HV_CHECK_LAUNCH();
  k_nms_final<<<batch, NMS_THREADS, NMS_LDS, s>>>(nscales, iou_thr, max_det, (const float*)(w + L.boxes),
                                              (const float*)(w + L.scores), (const int64_t*)(w + L.labels),
                                              (const int*)(w + L.counts), (Cand*)(w + L.cand2), (int*)(w + L.x2),
                                              L.img_stride, boxes, scores, labels, count);
  HV_CHECK_LAUNCH();
  return HV_OK;
}

extern "C" size_t hv_sort_desc_exact_work_bytes(int n) {
  if (n <= 0 || n > (1 << 28)) return 0;
  return align256((size_t)n * sizeof(Cand)) + (size_t)XWORK_ARRAYS * (n + 1) * sizeof(int);
}

extern "C" int hv_sort_desc_exact(const float* vals, int n, int depth_limit, int* out_idx, void* work,
                                  hv_stream_t stream) {
  if (!vals || !out_idx || !work || n <= 0 || n > (1 << 28)) return HV_EINVAL;
  unsigned char* w = (unsigned char*)work;
  nms_lds_attrs();
  k_sort_desc_exact<<<1, NMS_THREADS, NMS_LDS, (hipStream_t)stream>>>(
      vals, n, depth_limit, out_idx, (Cand*)w, (int*)(w + align256((size_t)n * sizeof(Cand))));
  HV_CHECK_LAUNCH();
  return HV_OK;
}
