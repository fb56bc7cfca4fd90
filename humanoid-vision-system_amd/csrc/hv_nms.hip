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
// The order.  Up to NMS_CAP candidates are compacted into LDS (any order) and bitonic-sorted by
// (score, index); with no two scores equal that is the only sorted order, so it is the
// reference's.  With ties, or more than NMS_CAP candidates, the reference's UNSTABLE order is
// rebuilt: the candidates in cell order go through a restatement of libstdc++'s introsort
// (exact_sort below) -- only over the prefix the greedy reads, widened 4x whenever the greedy
// runs off it before max_det.  The greedy reads the prefix from LDS when it fits.  Suppressed
// candidates are marked in place (the index's sign bit) and the sweep that suppresses also finds
// the next survivor (one barrier per kept box).  Kept boxes are written as they are found, so
// neither the candidate count nor max_det has a cap.
#include "hv_common.h"
#include <climits>

namespace {

constexpr int NMS_CAP = 8192;       // candidates sorted in LDS per segment (64 KiB)
constexpr int NMS_THREADS = 1024;
constexpr int NMS_DEAD = INT_MIN;   // sign bit of Cand::idx: suppressed
constexpr int NMS_PREFIX0 = 2048;   // first prefix of the exact sort the greedy reads (widened 4x)

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

// bitonic sort of c[0..n) in LDS (n <= NMS_CAP), best first; pads to a power of two
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
// All arrays live in the workspace (global memory, coherent within the workgroup across its
// barriers).
struct XWork {
  int *lo, *hi, *PL, *SR, *Lp, *Rp, *cut, *fl;   // each >= n + 1 ints
};
constexpr int XWORK_ARRAYS = 8;

__device__ __forceinline__ XWork xwork_at(int* base, long stride) {
  XWork w;
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

// exclusive scan of one int per thread in thread order; *total = the sum
__device__ int block_excl_scan(int v, int* total) {
  __shared__ int s_w[NMS_THREADS / 64 + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < nw; ++i) { const int t = s_w[i]; s_w[i] = acc; acc += t; }
    s_w[nw] = acc;
  }
  __syncthreads();
  const int r = s_w[wv] + x - v;
  *total = s_w[nw];
  __syncthreads();                       // s_w is reused by the next call
  return r;
}

// A[0..n) (global) in its ORIGINAL order -> std::sort's permutation of positions [0, limit): a
// segment lying wholly at or past `limit` is never partitioned further (what std::sort does there
// cannot move anything into the prefix: every element left of a cut is >= every element right of
// it), so the greedy NMS -- which reads the sorted order front to back and usually stops at
// max_det long before the end -- only pays for the top levels over all n plus the prefix.  Each
// level sweeps [0, end) with end = the last active segment's bound.  depth < 0: std::sort's own
// limit 2 * floor(log2 n); otherwise forced (tests reach the heap-sort fallback with it).
__device__ void exact_sort(Cand* A, int n, const XWork w, int depth, int limit) {
  __shared__ int s_any, s_end;
  const int T = blockDim.x, t = threadIdx.x;
  if (depth < 0) depth = n > 0 ? 2 * (31 - __clz(n)) : 0;
  for (int i = t; i < n; i += T) { w.lo[i] = 0; w.hi[i] = n; }
  if (t == 0) { s_any = n > 16 && limit > 0; s_end = n; }
  __syncthreads();
  while (s_any) {
    const int E = s_end;                 // positions past E belong to no active segment
    __syncthreads();                     // every thread has read s_any / s_end
    auto active = [&](int l, int h) { return h - l > 16 && l < limit; };
    if (depth == 0) {
      for (int i = t; i < E; i += T) {
        const int l = w.lo[i], h = w.hi[i];
        if (l == i && active(l, h)) heap_sort(A + l, h - l);
      }
      __syncthreads();
      break;
    }
    --depth;
    for (int i = t; i < E; i += T) {     // pivots: __unguarded_partition_pivot
      const int l = w.lo[i], h = w.hi[i];
      if (l == i && active(l, h)) median_to_first(A, l, l + 1, l + (h - l) / 2, h - 1);
    }
    if (t == 0) w.SR[E] = 0;
    __syncthreads();
    const int C = (E + T - 1) / T;
    const int c0 = min(E, t * C), c1 = min(E, c0 + C);
    int cL = 0, cR = 0;                  // stopper flags over this thread's chunk
    for (int i = c0; i < c1; ++i) {
      const int l = w.lo[i], h = w.hi[i];
      int f = 0;
      if (active(l, h) && i > l) {
        const float p = A[l].score, v = A[i].score;
        f = (!(v > p) ? 1 : 0) | (!(p > v) ? 2 : 0);
      }
      w.fl[i] = f;
      cL += f & 1;
      cR += f >> 1;
    }
    int totL, totR;
    const int exL = block_excl_scan(cL, &totL);
    const int exR = block_excl_scan(cR, &totR);
    int run = exL;                       // PL[i] = left stoppers in [0, i]
    for (int i = c0; i < c1; ++i) { run += w.fl[i] & 1; w.PL[i] = run; }
    run = totR - exR - cR;               // SR[i] = right stoppers in [i, E)
    for (int i = c1 - 1; i >= c0; --i) { run += w.fl[i] >> 1; w.SR[i] = run; }
    __syncthreads();
    for (int i = t; i < E; i += T) {     // l_k, r_k by rank within the segment
      const int f = w.fl[i];
      if (!f) continue;
      const int l = w.lo[i], h = w.hi[i];
      if (f & 1) w.Lp[l + w.PL[i] - w.PL[l]] = i;
      if (f & 2) w.Rp[l + w.SR[i] - w.SR[h]] = i;
    }
    __syncthreads();
    for (int i = t; i < E; i += T) {     // the swaps (disjoint pairs) and each segment's cut
      if (!(w.fl[i] & 1)) continue;
      const int l = w.lo[i], h = w.hi[i];
      const int k = w.PL[i] - w.PL[l];
      const int cntL = w.PL[h - 1] - w.PL[l], cntR = w.SR[l + 1] - w.SR[h];
      const int r = k <= cntR ? w.Rp[l + k] : -1;
      if (r > i) {
        xswap(A, i, r);
        const bool next = k + 1 <= cntL && k + 1 <= cntR && w.Lp[l + k + 1] < w.Rp[l + k + 1];
        if (!next) w.cut[l] = k + 1 <= cntL ? min(w.Lp[l + k + 1], r) : r;
      } else if (k == 1) {
        w.cut[l] = i;                    // no swap at all: cut = l_1
      }
    }
    if (t == 0) { s_any = 0; s_end = 0; }
    __syncthreads();
    for (int i = t; i < E; i += T) {     // [first, cut) and [cut, last), one level deeper
      const int l = w.lo[i], h = w.hi[i];
      if (!active(l, h)) continue;
      const int c = w.cut[l];
      const int nl = i < c ? l : c, nh = i < c ? c : h;
      w.lo[i] = nl;
      w.hi[i] = nh;
      if (i == nl && active(nl, nh)) {   // one thread per new active segment
        s_any = 1;
        atomicMax(&s_end, nh);
      }
    }
    __syncthreads();
  }
  const int P = min(n, limit);
  for (int i = t; i < P; i += T) {       // __final_insertion_sort = stable sort of every leaf
    const int l = w.lo[i], h = w.hi[i];
    if (l == i && h - l <= 16) insertion_sort(A + l, h - l);
  }
  __syncthreads();
}

// any equal neighbours among sorted c[0..n)?  (n <= 16: std::sort is then stable anyway)
__device__ bool has_ties(const Cand* c, int n) {
  int tie = 0;
  if (n > 16)
    for (int i = 1 + threadIdx.x; i < n; i += blockDim.x) tie |= c[i].score == c[i - 1].score;
  return __syncthreads_or(tie);
}

__device__ __forceinline__ int wave_min(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// greedy NMS over sorted c[0..n) (LDS or global).  box(idx) -> the candidate's xyxy box;
// emit(k, pos) writes output row k from c[pos] (called by thread 0).  Returns the kept count.
template <typename BoxFn, typename EmitFn>
__device__ int greedy(Cand* c, int n, float iou_thr, int max_det, BoxFn box, EmitFn emit) {
  __shared__ int s_next[3];
  if (n <= 0) return 0;
  if (threadIdx.x < 3) s_next[threadIdx.x] = INT_MAX;
  __syncthreads();
  int cur = 0, kept = 0;
  for (int it = 0;; ++it) {
    if (threadIdx.x == 0) emit(kept, cur);
    if (++kept >= max_det) break;
    const float4 cb = box(c[cur].idx);
    int first = INT_MAX;                 // this thread's first surviving position after cur
    for (int i = cur + 1 + threadIdx.x; i < n; i += blockDim.x) {
      const int id = c[i].idx;
      if (id < 0) continue;
      if (!(iou(cb, box(id)) < iou_thr)) c[i].idx = id | NMS_DEAD;
      else first = min(first, i);
    }
    first = wave_min(first);
    if ((threadIdx.x & 63) == 0 && first != INT_MAX) atomicMin(&s_next[it % 3], first);
    // the buffer of the next iteration was last read before the previous barrier
    if (threadIdx.x == 0) s_next[(it + 1) % 3] = INT_MAX;
    __syncthreads();
    cur = s_next[it % 3];
    if (cur == INT_MAX) break;
  }
  __syncthreads();
  return kept;
}

__global__ void __launch_bounds__(NMS_THREADS) k_nms_scale(const hv_nms_scale* __restrict__ scales, int nscales,
                                                           float conf_thr, float iou_thr, int max_det,
                                                           Cand* __restrict__ gcand, int* __restrict__ gx,
                                                           long seg_stride, float* sboxes, float* sscores,
                                                           int64_t* slabels, int* scount) {
  __shared__ Cand c[NMS_CAP];              // 64 KiB
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
      if (slot < NMS_CAP) c[slot] = Cand{v, (int)i};
      else if (slot < cap) g[slot] = Cand{v, (int)i};   // past the LDS capacity
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
  int kept = 0;
  bool exact = n > NMS_CAP;                // past the LDS: std::sort's order straight away
  if (!exact) {
    lds_sort(c, n);
    exact = has_ties(c, n);                // distinct scores: the one sorted order is the reference's
    if (!exact) kept = greedy(c, n, iou_thr, max_det, box, emit_from(c));
  }
  if (exact) {
    // the reference's order (ties included): the masked candidates in cell order, std::sort
    // restated over the prefix the greedy reads; a greedy that runs off the prefix before
    // max_det widens it 4x and starts over (deterministic)
    const XWork xw = xwork_at(gx + seg * XWORK_ARRAYS * (seg_stride + 1), seg_stride + 1);
    for (int limit = min(n, NMS_PREFIX0);; limit = min(n, 4 * limit)) {
      const long C = (cells + blockDim.x - 1) / blockDim.x;
      const long c0 = min(cells, (long)threadIdx.x * C), c1 = min(cells, c0 + C);
      int cnt = 0;
      for (long i = c0; i < c1; ++i) cnt += score[i] > conf_thr;
      int tot;
      int o = block_excl_scan(cnt, &tot);
      for (long i = c0; i < c1; ++i) {
        const float v = score[i];
        if (v > conf_thr && o < cap) g[o] = Cand{v, (int)i};
        o += v > conf_thr;
      }
      __syncthreads();
      exact_sort(g, n, xw, -1, limit);
      if (limit <= NMS_CAP) {              // the greedy reads the prefix from LDS
        for (int i = threadIdx.x; i < limit; i += blockDim.x) c[i] = g[i];
        __syncthreads();
        kept = greedy(c, limit, iou_thr, max_det, box, emit_from(c));
      } else {
        kept = greedy(g, limit, iou_thr, max_det, box, emit_from(g));
      }
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
  __shared__ Cand c[NMS_CAP];
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
  int kept = 0;
  bool exact = n > NMS_CAP;
  if (!exact) {
    gather(c);
    lds_sort(c, n);       // idx grows with the concatenation order
    exact = has_ties(c, n);
    if (!exact) kept = greedy(c, n, iou_thr, max_det, box, emit_from(c));
  }
  if (exact) {            // as stage 1: std::sort's order over the prefix the greedy reads
    const XWork xw = xwork_at(gx + (long)b * XWORK_ARRAYS * (img_stride + 1), img_stride + 1);
    for (int limit = min(n, NMS_PREFIX0);; limit = min(n, 4 * limit)) {
      gather(g);
      exact_sort(g, n, xw, -1, limit);
      if (limit <= NMS_CAP) {
        for (int i = threadIdx.x; i < limit; i += blockDim.x) c[i] = g[i];
        __syncthreads();
        kept = greedy(c, limit, iou_thr, max_det, box, emit_from(c));
      } else {
        kept = greedy(g, limit, iou_thr, max_det, box, emit_from(g));
      }
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
  for (int i = threadIdx.x; i < n; i += blockDim.x) A[i] = Cand{vals[i], i};
  __syncthreads();
  exact_sort(A, n, xwork_at(gx, (long)n + 1), depth, n);
  for (int i = threadIdx.x; i < n; i += blockDim.x) out_idx[i] = A[i].idx;
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
  k_nms_scale<<<(unsigned)segs, NMS_THREADS, 0, s>>>(dev_scales, nscales, conf_thr, iou_thr, max_det,
                                                      (Cand*)(w + L.cand1), (int*)(w + L.x1), L.seg_stride,
                                                      (float*)(w + L.boxes), (float*)(w + L.scores),
                                                      (int64_t*)(w + L.labels), (int*)(w + L.counts));
  HV_CHECK_LAUNCH();
  k_nms_final<<<batch, NMS_THREADS, 0, s>>>(nscales, iou_thr, max_det, (const float*)(w + L.boxes),
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
  k_sort_desc_exact<<<1, NMS_THREADS, 0, (hipStream_t)stream>>>(
      vals, n, depth_limit, out_idx, (Cand*)w, (int*)(w + align256((size_t)n * sizeof(Cand))));
  HV_CHECK_LAUNCH();
  return HV_OK;
}
