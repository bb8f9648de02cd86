// Validation-side matching of NMS detections to ground-truth labels (mAP TP matrix) on the device.
//
// Restates DetectionValidator._process_batch (U/models/yolo/detect/val.py:209-227) =
// box_iou (U/utils/metrics.py:52-71) + BaseValidator.match_predictions non-scipy branch
// (U/engine/validator.py:222-262).  That routine, per IoU threshold t, takes every
// (label, detection) pair with class-masked IoU >= t, sorts them by IoU descending, keeps the
// first pair per detection (its highest-IoU label) and then, in detection order, the first pair
// per label.  Hence, for one image:
//   best(d)   = argmax over labels of the class-masked IoU (exact ties -> larger label index, the
//               order numpy's reversed stable argsort gives for small match arrays),
//   correct[d][t] = maxIoU(d) >= t  and  no d' < d with best(d') == best(d) and maxIoU(d') >= t.
// The second condition is a per-(label, threshold) atomicMin of the detection index.
//
// One 256-thread workgroup per image.  IoU is evaluated in fp32 with the reference's operation
// order and no FMA contraction, so it is bitwise the torch CPU value and the threshold compares
// agree exactly.
#include <climits>

#include "common.hpp"

#pragma clang fp contract(off)

namespace ydbl {

constexpr int MATCH_THREADS = 256;
constexpr int MATCH_MAX_IOU = 32;

struct MatchArgs {
  const float* det; const int* det_count;
  int n, max_det;
  const float* gt_box; const float* gt_cls; const int* gt_ofs;
  const float* iouv; int n_iou;
  int single_cls;
  int* min_det;  // [n_gt][n_iou]
  int* best;     // [n][max_det]
  int* valid;    // [n][max_det] bitmask over thresholds
  uint8_t* correct;
};

// box_iou (U/utils/metrics.py:52-71) for one pair, same rounding sequence as the torch CPU op.
__device__ __forceinline__ float pair_iou(const float* a, const float* b) {
  const float iw = fmaxf(fminf(a[2], b[2]) - fmaxf(a[0], b[0]), 0.0f);
  const float ih = fmaxf(fminf(a[3], b[3]) - fmaxf(a[1], b[1]), 0.0f);
  const float inter = iw * ih;
  const float area_a = (a[2] - a[0]) * (a[3] - a[1]);
  const float area_b = (b[2] - b[0]) * (b[3] - b[1]);
  return inter / (((area_a + area_b) - inter) + 1e-7f);
}

__global__ __launch_bounds__(MATCH_THREADS) void match_kernel(MatchArgs p) {
  const int b = blockIdx.x;
  const int g0 = p.gt_ofs[b], nl = p.gt_ofs[b + 1] - g0;
  const int nd = min(p.det_count[b], p.max_det);
  const float* det = p.det + (int64_t)b * p.max_det * 6;
  uint8_t* out = p.correct + (int64_t)b * p.max_det * p.n_iou;

  for (int i = threadIdx.x; i < nl * p.n_iou; i += MATCH_THREADS)
    __hip_atomic_store(p.min_det + (int64_t)g0 * p.n_iou + i, INT_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence();
  __syncthreads();

  for (int d = threadIdx.x; d < nd; d += MATCH_THREADS) {
    const float* db = det + d * 6;
    const float dc = p.single_cls ? 0.0f : db[5];
    int best = -1;
    float bi = 0.0f;
    for (int l = 0; l < nl; ++l) {
      // iou * (true_cls == pred_cls): a class mismatch contributes an IoU of exactly 0
      const float v = p.gt_cls[g0 + l] == dc ? pair_iou(p.gt_box + (int64_t)(g0 + l) * 4, db) : 0.0f;
      if (best < 0 || v >= bi) { bi = v; best = l; }
    }
    int mask = 0;
    if (best >= 0)
      for (int t = 0; t < p.n_iou; ++t)
        if (bi >= p.iouv[t]) {
          mask |= 1 << t;
          atomicMin(p.min_det + (int64_t)(g0 + best) * p.n_iou + t, d);
        }
    p.best[(int64_t)b * p.max_det + d] = best;
    p.valid[(int64_t)b * p.max_det + d] = mask;
  }
  __threadfence();
  __syncthreads();

  for (int d = threadIdx.x; d < p.max_det; d += MATCH_THREADS) {
    const int best = d < nd ? p.best[(int64_t)b * p.max_det + d] : -1;
    const int mask = d < nd ? p.valid[(int64_t)b * p.max_det + d] : 0;
    for (int t = 0; t < p.n_iou; ++t) {
      bool ok = false;
      if ((mask >> t) & 1)
        ok = __hip_atomic_load(p.min_det + (int64_t)(g0 + best) * p.n_iou + t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) == d;
      out[d * p.n_iou + t] = ok;
    }
  }
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int64_t ydbl_match_workspace(int32_t n, int32_t max_det, int32_t n_gt, int32_t n_iou) {
  if (n < 0 || max_det < 0 || n_gt < 0 || n_iou < 0) return -1;
  return 4 * ((int64_t)n_gt * n_iou + 2 * (int64_t)n * max_det) + 16;
}

extern "C" int ydbl_match_predictions(const ydbl_match_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "match: null descriptor");
  if (!d->det || !d->det_count || !d->gt_ofs || !d->iouv || !d->correct || !d->workspace)
    return fail(YDBL_EINVAL, "match: null buffer");
  if (d->n < 1 || d->max_det < 1) return fail(YDBL_EINVAL, "match: empty batch");
  if (d->n_gt < 0 || (d->n_gt > 0 && (!d->gt_box || !d->gt_cls)))
    return fail(YDBL_EINVAL, "match: labels missing");
  if (d->n_iou < 1 || d->n_iou > MATCH_MAX_IOU) return fail(YDBL_EINVAL, "match: n_iou must be in [1, 32]");
  MatchArgs a;
  a.det = d->det; a.det_count = d->det_count; a.n = d->n; a.max_det = d->max_det;
  a.gt_box = d->gt_box; a.gt_cls = d->gt_cls; a.gt_ofs = d->gt_ofs;
  a.iouv = d->iouv; a.n_iou = d->n_iou; a.single_cls = d->single_cls;
  a.min_det = reinterpret_cast<int*>(d->workspace);
  a.best = a.min_det + (int64_t)d->n_gt * d->n_iou;
  a.valid = a.best + (int64_t)d->n * d->max_det;
  a.correct = d->correct;
  match_kernel<<<d->n, MATCH_THREADS, 0, as_stream(stream)>>>(a);
  return check_launch("ydbl_match_predictions");
}
