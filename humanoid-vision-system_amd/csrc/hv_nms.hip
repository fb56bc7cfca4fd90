// Detection post-processing on the GPU: YOLODetectionHead.post_process +
// non_max_suppression (reference yolo_head.py:571-731), the whole batch in two launches with no
// host round trip per box (the reference does one .item() per kept box).
//
// Stage 1, one workgroup per (image, scale): candidates with class_score > conf_thr are
// compacted into LDS in flattened [A, H, W] order, bitonic-sorted by score (descending, ties by
// index), then greedy NMS: the best remaining box is kept and every remaining box with
// IoU >= iou_thr (the reference keeps IoU < thr) is suppressed, until max_det are kept or none
// remain.  Stage 2, one workgroup per image: the same greedy NMS over the concatenation of
// the per-scale survivors (scale 0 first, each in kept order), as the reference's final
// cross-scale pass.  IoU is computed exactly as compute_iou (yolo_head.py:711-725 helper):
// inter / (area1 + area2 - inter + 1e-6).
#include "hv_common.h"

namespace {

constexpr int NMS_CAP = 8192;       // candidates held in LDS per (image, scale)
constexpr int NMS_THREADS = 1024;
constexpr int NMS_MAXDET = 1024;

struct Cand {
  float score;
  int idx;                          // index into the segment's flattened cells
};

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
  return a.score > b.score || (a.score == b.score && a.idx < b.idx);
}

__device__ __forceinline__ float iou(const float* a, const float* b) {
  const float ix1 = fmaxf(a[0], b[0]), iy1 = fmaxf(a[1], b[1]);
  const float ix2 = fminf(a[2], b[2]), iy2 = fminf(a[3], b[3]);
  const float inter = fmaxf(ix2 - ix1, 0.f) * fmaxf(iy2 - iy1, 0.f);
  const float a1 = (a[2] - a[0]) * (a[3] - a[1]);
  const float a2 = (b[2] - b[0]) * (b[3] - b[1]);
  return inter / (a1 + a2 - inter + 1e-6f);
}

// bitonic sort of c[0..n) (n <= NMS_CAP) descending by (score, -idx); pads to a power of two
__device__ void block_sort(Cand* c, int n) {
  int m = 1;
  while (m < n) m <<= 1;
  for (int i = n + threadIdx.x; i < m; i += blockDim.x) c[i] = Cand{-INFINITY, 0x7fffffff};
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & k) == 0;
          const Cand a = c[i], b = c[l];
          if (desc ? better(b, a) : better(a, b)) { c[i] = b; c[l] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// greedy NMS over the sorted candidates; box(i) gives the 4 coords of candidate i.
// alive[] flags in LDS; writes kept candidate positions to keep[], returns the count.
template <typename BoxFn>
__device__ int greedy(const Cand* c, int n, unsigned char* alive, int* keep, float iou_thr, int max_det, BoxFn box) {
  __shared__ int s_next;
  for (int i = threadIdx.x; i < n; i += blockDim.x) alive[i] = 1;
  __syncthreads();
  int kept = 0, start = 0;
  while (kept < max_det) {
    if (threadIdx.x == 0) {
      int nx = -1;
      for (int i = start; i < n; ++i)
        if (alive[i]) { nx = i; break; }
      s_next = nx;
    }
    __syncthreads();
    const int cur = s_next;
    __syncthreads();
    if (cur < 0) break;
    if (threadIdx.x == 0) keep[kept] = cur;
    ++kept;
    start = cur + 1;
    if (kept >= max_det) break;
    float cb[4];
    box(cur, cb);
    for (int i = start + threadIdx.x; i < n; i += blockDim.x) {
      if (!alive[i]) continue;
      float ob[4];
      box(i, ob);
      if (!(iou(cb, ob) < iou_thr)) alive[i] = 0;
    }
    __syncthreads();
  }
  __syncthreads();
  return kept;
}

__global__ void __launch_bounds__(NMS_THREADS) k_nms_scale(const hv_nms_scale* __restrict__ scales, int nscales,
                                                           float conf_thr, float iou_thr, int max_det,
                                                           float* sboxes, float* sscores, int64_t* slabels,
                                                           int* scount) {
  __shared__ Cand c[NMS_CAP];              // 64 KiB
  __shared__ unsigned char alive[NMS_CAP];
  __shared__ int keep[NMS_MAXDET];
  __shared__ int s_n;
  const int sc = blockIdx.x % nscales, b = blockIdx.x / nscales;
  const hv_nms_scale S = scales[sc];
  const long cells = S.cells;
  const float* score = S.class_scores + (long)b * cells;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  for (long i = threadIdx.x; i < cells; i += blockDim.x) {
    const float v = score[i];
    if (v > conf_thr) {
      const int slot = atomicAdd(&s_n, 1);
      if (slot < NMS_CAP) c[slot] = Cand{v, (int)i};
    }
  }
  __syncthreads();
  const int n = min(s_n, NMS_CAP);
  block_sort(c, n);
  const float* boxes = S.boxes + (long)b * cells * 4;
  auto box = [&](int i, float* o) {
    const float* p = boxes + (long)c[i].idx * 4;
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3];
  };
  const int kept = greedy(c, n, alive, keep, iou_thr, max_det, box);
  const long seg = (long)blockIdx.x;
  for (int k = threadIdx.x; k < kept; k += blockDim.x) {
    const int ci = keep[k];
    const long cell = c[ci].idx;
    for (int j = 0; j < 4; ++j) sboxes[(seg * max_det + k) * 4 + j] = boxes[cell * 4 + j];
    sscores[seg * max_det + k] = c[ci].score;
    slabels[seg * max_det + k] = S.class_indices[(long)b * cells + cell];
  }
  if (threadIdx.x == 0) scount[seg] = kept;
}

// stage 2: per image, NMS over the concatenated per-scale survivors
__global__ void __launch_bounds__(NMS_THREADS) k_nms_final(int nscales, float iou_thr, int max_det,
                                                           const float* sboxes, const float* sscores,
                                                           const int64_t* slabels, const int* scount, float* boxes,
                                                           float* scores, int64_t* labels, int* count) {
  __shared__ Cand c[NMS_CAP];
  __shared__ unsigned char alive[NMS_CAP];
  __shared__ int keep[NMS_MAXDET];
  const int b = blockIdx.x;
  int n = 0;
  // concatenation order: scale 0's survivors, then scale 1's, ... (index = seg * max_det + k)
  for (int s = 0; s < nscales; ++s) {
    const int seg = b * nscales + s;
    const int cnt = scount[seg];
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) c[n + k] = Cand{sscores[seg * max_det + k], seg * max_det + k};
    n += cnt;
  }
  __syncthreads();
  block_sort(c, n);       // idx = seg * max_det + k grows with the concatenation order: ties keep it
  auto box = [&](int i, float* o) {
    const float* p = sboxes + (long)c[i].idx * 4;
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3];
  };
  const int kept = greedy(c, n, alive, keep, iou_thr, max_det, box);
  for (int k = threadIdx.x; k < kept; k += blockDim.x) {
    const int src = c[keep[k]].idx;
    for (int j = 0; j < 4; ++j) boxes[((long)b * max_det + k) * 4 + j] = sboxes[(long)src * 4 + j];
    scores[(long)b * max_det + k] = sscores[src];
    labels[(long)b * max_det + k] = slabels[src];
  }
  // rows past `count` are zero, so the fixed-size outputs are a function of the inputs alone
  for (int k = kept + threadIdx.x; k < max_det; k += blockDim.x) {
    for (int j = 0; j < 4; ++j) boxes[((long)b * max_det + k) * 4 + j] = 0.f;
    scores[(long)b * max_det + k] = 0.f;
    labels[(long)b * max_det + k] = 0;
  }
  if (threadIdx.x == 0) count[b] = kept;
}

}  // namespace

extern "C" size_t hv_nms_work_bytes(int batch, int nscales, int max_det) {
  const size_t segs = (size_t)batch * nscales;
  return segs * max_det * (4 * sizeof(float) + sizeof(float) + sizeof(int64_t)) + segs * sizeof(int) + 256;
}

extern "C" int hv_nms(const hv_nms_scale* dev_scales, int nscales, int batch, float conf_thr, float iou_thr,
                      int max_det, float* boxes, float* scores, int64_t* labels, int* count, void* work,
                      hv_stream_t stream) {
  if (!dev_scales || nscales <= 0 || batch <= 0 || max_det <= 0 || max_det > 1024 || !boxes || !scores ||
      !labels || !count || !work || nscales * max_det > NMS_CAP)
    return HV_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const size_t segs = (size_t)batch * nscales;
  unsigned char* w = (unsigned char*)work;
  int64_t* slabels = (int64_t*)w;
  float* sboxes = (float*)(slabels + segs * max_det);
  float* sscores = sboxes + segs * max_det * 4;
  int* scount = (int*)(sscores + segs * max_det);
  k_nms_scale<<<(unsigned)segs, NMS_THREADS, 0, s>>>(dev_scales, nscales, conf_thr, iou_thr, max_det, sboxes, sscores,
                                                      slabels, scount);
  HV_CHECK_LAUNCH();
  k_nms_final<<<batch, NMS_THREADS, 0, s>>>(nscales, iou_thr, max_det, sboxes, sscores, slabels, scount, boxes,
                                              scores, labels, count);
  HV_CHECK_LAUNCH();
  return HV_OK;
}
