/* Oracle (TEST INFRASTRUCTURE ONLY): torchvision's CPU NMS kernel restated in C, the op the reference's
 * non_max_suppression calls (U/utils/ops.py:296, torchvision.ops.nms; torchvision is not installed here and
 * is not vendored: its published nms_kernel_impl, torchvision/csrc/ops/cpu/nms_kernel.cpp, is restated).
 * Same float32 arithmetic per (i, j) pair as oracle/ops.py:nms_torchvision (built with -ffp-contract=off):
 * xx1 = max, yy1 = max, xx2 = min, yy2 = min, w = max(0, xx2 - xx1), h = max(0, yy2 - yy1), inter = w * h,
 * ovr = inter / (area_i + area_j - inter), suppressed when (double)ovr > iou_threshold.
 * Order: scores descending, ties in input order (a stable sort, as oracle/ops.py uses). */
#include <stdint.h>
#include <stdlib.h>

static const float* g_scores;

static int cmp_desc(const void* a, const void* b) {
  const int64_t i = *(const int64_t*)a, j = *(const int64_t*)b;
  const float si = g_scores[i], sj = g_scores[j];
  if (si > sj) return -1;
  if (si < sj) return 1;
  return (i > j) - (i < j); /* stable: input order among equal scores */
}

/* boxes [n, 4] xyxy float32, scores [n]; writes keep indices (score order) to keep[]; returns their count,
 * or -1 when out of memory. Not thread-safe (qsort comparator state). */
int64_t ydbl_oracle_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep) {
  if (n <= 0) return 0;
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * n);
  float* x1 = (float*)malloc(sizeof(float) * n * 5);
  char* sup = (char*)calloc(n, 1);
  if (!order || !x1 || !sup) { free(order); free(x1); free(sup); return -1; }
  float *y1 = x1 + n, *x2 = x1 + 2 * n, *y2 = x1 + 3 * n, *area = x1 + 4 * n;
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  g_scores = scores;
  qsort(order, (size_t)n, sizeof(int64_t), cmp_desc);
  for (int64_t k = 0; k < n; ++k) {
    const float* b = boxes + 4 * order[k];
    x1[k] = b[0]; y1[k] = b[1]; x2[k] = b[2]; y2[k] = b[3];
    area[k] = (x2[k] - x1[k]) * (y2[k] - y1[k]);
  }
  int64_t nk = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (sup[i]) continue;
    keep[nk++] = order[i];
    const float ix1 = x1[i], iy1 = y1[i], ix2 = x2[i], iy2 = y2[i], ia = area[i];
    for (int64_t j = i + 1; j < n; ++j) {
      if (sup[j]) continue;
      const float xx1 = ix1 > x1[j] ? ix1 : x1[j];
      const float yy1 = iy1 > y1[j] ? iy1 : y1[j];
      const float xx2 = ix2 < x2[j] ? ix2 : x2[j];
      const float yy2 = iy2 < y2[j] ? iy2 : y2[j];
      const float w = xx2 - xx1 > 0.f ? xx2 - xx1 : 0.f;
      const float h = yy2 - yy1 > 0.f ? yy2 - yy1 : 0.f;
      const float inter = w * h;
      const float ovr = inter / (ia + area[j] - inter);
      if ((double)ovr > iou_threshold) sup[j] = 1;
    }
  }
  free(order); free(x1); free(sup);
  return nk;
}
