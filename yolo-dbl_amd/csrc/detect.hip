// Detect decode (DFL + dist2bbox + sigmoid + candidate filter) and batched class-offset NMS.
//
// decode : one thread per (image, anchor).  Writes the reference's y[b][4+nc][A] when asked
//          (U/nn/modules/head.py:143-181) and appends NMS candidates (U/utils/ops.py:234-276) with
//          a per-image atomic counter; candidate order is irrelevant because NMS sorts by
//          (score desc, original index asc), which is exactly the order torchvision's stable sort
//          gives the reference (anchor order, or torch.where's (anchor, class) row-major order).
// nms    : per-image bitonic key/value sort (LDS chunks of 4096 + global merge steps), then one
//          1024-thread workgroup per image runs the greedy sweep with the suppression flags and
//          the first 4096 sorted boxes in LDS.  The sweep stops after max_det keeps, which is the
//          same as the reference's keep[:max_det] because keeps are produced in score order.
#include "common.hpp"

#pragma clang fp contract(off)

namespace ydbl {

template <typename T>
struct DecodeArgs {
  DView<const T> box[3], cls[3];
  int nl, nc, A;
  int a_end[3];
  float stride[3];
  float conf;
  int multi;
  const int* classes; int ncls;
  float* yref;
  float* cbox; float* cscore; int* ccls; int* cidx; int* ccount;
  int cap;
};

__device__ __forceinline__ bool class_ok(int j, const int* classes, int ncls) {
  if (!classes) return true;
  for (int q = 0; q < ncls; ++q)
    if (classes[q] == j) return true;
  return false;
}

template <typename T>
__global__ __launch_bounds__(256) void decode_kernel(DecodeArgs<T> p) {
  const int b = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= p.A) return;
  int l = 0;
  while (l < p.nl - 1 && a >= p.a_end[l]) ++l;
  const int a0 = l ? p.a_end[l - 1] : 0;
  const int loc = a - a0;
  const DView<const T>& bx = p.box[l];
  const int gx = loc % bx.w, gy = loc / bx.w;
  const T* bp = bx.at(b, gy, gx);
  float dist[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {  // DFL: softmax over 16 bins, expectation with weights 0..15
    float v[16];
    load_f<8>(bp + s * 16, v);
    load_f<8>(bp + s * 16 + 8, v + 8);
    float m = v[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) m = fmaxf(m, v[k]);
    float e[16], sum = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      e[k] = expf(v[k] - m);
      sum += e[k];
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += float(k) * (e[k] / sum);
    dist[s] = acc;
  }
  const float ax = float(gx) + 0.5f, ay = float(gy) + 0.5f, st = p.stride[l];
  const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
  const float cx = ((x1 + x2) / 2.0f) * st, cy = ((y1 + y2) / 2.0f) * st;
  const float w = (x2 - x1) * st, h = (y2 - y1) * st;
  const int64_t A = p.A;
  if (p.yref) {
    float* yr = p.yref + (int64_t)b * (4 + p.nc) * A + a;
    yr[0] = cx; yr[A] = cy; yr[2 * A] = w; yr[3 * A] = h;
  }
  // xywh2xyxy (U/utils/ops.py:416-433)
  const float hw = w / 2.0f, hh = h / 2.0f;
  const float bx1 = cx - hw, by1 = cy - hh, bx2 = cx + hw, by2 = cy + hh;
  const T* cp = p.cls[l].at(b, gy, gx);
  float best = -1.f;
  int bj = 0;
  for (int j = 0; j < p.nc; ++j) {
    const float sc = 1.0f / (1.0f + expf(-float(cp[j])));
    if (p.yref) p.yref[((int64_t)b * (4 + p.nc) + 4 + j) * A + a] = sc;
    if (p.multi) {
      if (sc > p.conf && class_ok(j, p.classes, p.ncls)) {
        const int slot = atomicAdd(p.ccount + b, 1);
        if (slot < p.cap) {
          const int64_t o = (int64_t)b * p.cap + slot;
          *reinterpret_cast<f32x4*>(p.cbox + o * 4) = f32x4{bx1, by1, bx2, by2};
          p.cscore[o] = sc; p.ccls[o] = j; p.cidx[o] = a * p.nc + j;
        }
      }
    } else if (sc > best) {  // torch.max: first index of the maximum
      best = sc;
      bj = j;
    }
  }
  if (!p.multi && best > p.conf && class_ok(bj, p.classes, p.ncls)) {
    const int slot = atomicAdd(p.ccount + b, 1);
    if (slot < p.cap) {
      const int64_t o = (int64_t)b * p.cap + slot;
      *reinterpret_cast<f32x4*>(p.cbox + o * 4) = f32x4{bx1, by1, bx2, by2};
      p.cscore[o] = best; p.ccls[o] = bj; p.cidx[o] = a;
    }
  }
}

// Candidates from a prediction tensor in the reference layout pred[b][4+nc][A] (xywh, scores).
__global__ __launch_bounds__(256) void pred_cand_kernel(ydbl_pred_cand_desc p) {
  const int b = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= p.A) return;
  const int64_t A = p.A;
  const float* pr = p.pred + (int64_t)b * (4 + p.nc) * A + a;
  const float cx = pr[0], cy = pr[A], hw = pr[2 * A] / 2.0f, hh = pr[3 * A] / 2.0f;
  const float bx1 = cx - hw, by1 = cy - hh, bx2 = cx + hw, by2 = cy + hh;
  float best = -INFINITY;
  int bj = 0;
  for (int j = 0; j < p.nc; ++j) {
    const float sc = pr[(4 + j) * A];
    if (p.multi_label) {
      if (sc > p.conf_thres && class_ok(j, p.classes, p.nclasses)) {
        const int slot = atomicAdd(p.cand_count + b, 1);
        if (slot < p.cap) {
          const int64_t o = (int64_t)b * p.cap + slot;
          *reinterpret_cast<f32x4*>(p.cand_box + o * 4) = f32x4{bx1, by1, bx2, by2};
          p.cand_score[o] = sc; p.cand_cls[o] = j; p.cand_idx[o] = a * p.nc + j;
        }
      }
    } else if (sc > best) {
      best = sc;
      bj = j;
    }
  }
  if (!p.multi_label && best > p.conf_thres && class_ok(bj, p.classes, p.nclasses)) {
    const int slot = atomicAdd(p.cand_count + b, 1);
    if (slot < p.cap) {
      const int64_t o = (int64_t)b * p.cap + slot;
      *reinterpret_cast<f32x4*>(p.cand_box + o * 4) = f32x4{bx1, by1, bx2, by2};
      p.cand_score[o] = best; p.cand_cls[o] = bj; p.cand_idx[o] = a;
    }
  }
}

// ------------------------------------------------------------------------------------ sort
constexpr int SORT_CHUNK = 4096;

__device__ __forceinline__ uint64_t make_key(float score, int idx) {
  // scores are sigmoid outputs in (0,1): their bit patterns order like the values.
  const uint32_t sb = __float_as_uint(score);
  return ((uint64_t)(0xFFFFFFFFu - sb) << 32) | (uint32_t)idx;
}

__global__ __launch_bounds__(1024) void nms_keys_kernel(const float* __restrict__ score, const int* __restrict__ idx,
                                                        const int* __restrict__ count, int cap, int L,
                                                        uint64_t* __restrict__ keys, int* __restrict__ vals) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  const int n = min(count[b], cap);
  const int64_t o = (int64_t)b * L + i;
  if (i < n) {
    keys[o] = make_key(score[(int64_t)b * cap + i], idx[(int64_t)b * cap + i]);
    vals[o] = i;
  } else {
    keys[o] = ~0ull;
    vals[o] = -1;
  }
}

// Bitonic steps (k, j) for j < SORT_CHUNK inside LDS.  If full, runs every k <= chunk.
__global__ __launch_bounds__(1024) void bitonic_local_kernel(uint64_t* __restrict__ keys, int* __restrict__ vals, int L,
                                                             int chunk, int kfixed) {
  __shared__ uint64_t sk[SORT_CHUNK];
  __shared__ int sv[SORT_CHUNK];
  const int b = blockIdx.y;
  const int64_t base = (int64_t)b * L + (int64_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
    sk[i] = keys[base + i];
    sv[i] = vals[base + i];
  }
  __syncthreads();
  const int gbase = blockIdx.x * chunk;
  auto step = [&](int k, int j) {
    for (int t = threadIdx.x; t < chunk / 2; t += blockDim.x) {
      const int i = 2 * j * (t / j) + (t % j);
      const int ixj = i + j;
      const bool up = ((gbase + i) & k) == 0;
      const uint64_t a = sk[i], c = sk[ixj];
      if ((a > c) == up) {
        sk[i] = c; sk[ixj] = a;
        const int tv = sv[i]; sv[i] = sv[ixj]; sv[ixj] = tv;
      }
    }
    __syncthreads();
  };
  if (kfixed == 0) {
    for (int k = 2; k <= chunk; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) step(k, j);
  } else {
    for (int j = chunk >> 1; j > 0; j >>= 1) step(kfixed, j);
  }
  for (int i = threadIdx.x; i < chunk; i += blockDim.x) {
    keys[base + i] = sk[i];
    vals[base + i] = sv[i];
  }
}

__global__ __launch_bounds__(256) void bitonic_global_kernel(uint64_t* __restrict__ keys, int* __restrict__ vals, int L,
                                                             int k, int j) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L / 2) return;
  const int i = 2 * j * (t / j) + (t % j);
  const int ixj = i + j;
  const bool up = (i & k) == 0;
  uint64_t* kb = keys + (int64_t)b * L;
  int* vb = vals + (int64_t)b * L;
  const uint64_t a = kb[i], c = kb[ixj];
  if ((a > c) == up) {
    kb[i] = c; kb[ixj] = a;
    const int tv = vb[i]; vb[i] = vb[ixj]; vb[ixj] = tv;
  }
}

// ------------------------------------------------------------------------------------ greedy
constexpr int NMS_LDS_BOXES = 4096;
constexpr int NMS_MAX_FLAGS = 32768;
constexpr int NMS_MAX_DET = 4096;

struct NmsArgs {
  const float* cbox; const float* cscore; const int* ccls; const int* ccount;
  const int* vals; int L, cap;
  double thr; int max_det, max_nms; float off_scale;
  float clip_w, clip_h;
  float* out; int* out_count;
};

__global__ __launch_bounds__(1024) void nms_greedy_kernel(NmsArgs p) {
  __shared__ f32x4 sbox[NMS_LDS_BOXES];
  __shared__ unsigned char removed[NMS_MAX_FLAGS];
  __shared__ int kept_slot[NMS_MAX_DET];
  __shared__ int s_next;
  const int b = blockIdx.x;
  const int n = min(min(p.ccount[b], p.cap), p.max_nms);
  const int* vb = p.vals + (int64_t)b * p.L;
  auto load_box = [&](int i) -> f32x4 {
    const int slot = vb[i];
    const int64_t o = (int64_t)b * p.cap + slot;
    const f32x4 v = *reinterpret_cast<const f32x4*>(p.cbox + o * 4);
    const float c = float(p.ccls[o]) * p.off_scale;  // boxes + cls * max_wh (0 if agnostic)
    return f32x4{v[0] + c, v[1] + c, v[2] + c, v[3] + c};
  };
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    removed[i] = 0;
    if (i < NMS_LDS_BOXES) sbox[i] = load_box(i);
  }
  __syncthreads();
  int kept = 0, cur = 0;
  const int lane = threadIdx.x & 63;
  while (true) {
    if (threadIdx.x < 64) {  // wave 0: first non-removed index >= cur
      int found = n;
      for (int base = cur; base < n; base += 64) {
        const int i = base + lane;
        const bool live = i < n && !removed[i];
        const uint64_t mask = __ballot(live);
        if (mask) {
          found = base + __ffsll((long long)mask) - 1;
          break;
        }
      }
      if (lane == 0) s_next = found;
    }
    __syncthreads();
    const int i = s_next;
    __syncthreads();
    if (i >= n || kept >= p.max_det) break;
    if (threadIdx.x == 0) kept_slot[kept] = vb[i];
    ++kept;
    cur = i + 1;
    const f32x4 bi = i < NMS_LDS_BOXES ? sbox[i] : load_box(i);
    const float area_i = (bi[2] - bi[0]) * (bi[3] - bi[1]);
    for (int j = i + 1 + threadIdx.x; j < n; j += blockDim.x) {
      if (removed[j]) continue;
      const f32x4 bj = j < NMS_LDS_BOXES ? sbox[j] : load_box(j);
      const float xx1 = fmaxf(bi[0], bj[0]), yy1 = fmaxf(bi[1], bj[1]);
      const float xx2 = fminf(bi[2], bj[2]), yy2 = fminf(bi[3], bj[3]);
      const float ww = fmaxf(0.f, xx2 - xx1), hh = fmaxf(0.f, yy2 - yy1);
      const float inter = ww * hh;
      const float area_j = (bj[2] - bj[0]) * (bj[3] - bj[1]);
      const float ovr = inter / ((area_i + area_j) - inter);
      if ((double)ovr > p.thr) removed[j] = 1;
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < kept; k += blockDim.x) {
    const int64_t o = (int64_t)b * p.cap + kept_slot[k];
    f32x4 v = *reinterpret_cast<const f32x4*>(p.cbox + o * 4);
    if (p.clip_w > 0.f) {
      v[0] = fminf(fmaxf(v[0], 0.f), p.clip_w);
      v[2] = fminf(fmaxf(v[2], 0.f), p.clip_w);
    }
    if (p.clip_h > 0.f) {
      v[1] = fminf(fmaxf(v[1], 0.f), p.clip_h);
      v[3] = fminf(fmaxf(v[3], 0.f), p.clip_h);
    }
    float* dst = p.out + ((int64_t)b * p.max_det + k) * 6;
    dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
    dst[4] = p.cscore[o];
    dst[5] = float(p.ccls[o]);
  }
  if (threadIdx.x == 0) p.out_count[b] = kept;
}

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

template <typename T>
static DView<const T> cvw(const ydbl_view& v) {
  return DView<const T>{reinterpret_cast<const T*>(v.ptr), v.n, v.h, v.w, v.c, v.cs};
}

template <typename T>
static int decode_t(const ydbl_decode_desc* d, hipStream_t s) {
  DecodeArgs<T> a{};
  int A = 0;
  for (int l = 0; l < d->nl; ++l) {
    a.box[l] = cvw<T>(d->box[l]);
    a.cls[l] = cvw<T>(d->cls[l]);
    A += d->box[l].h * d->box[l].w;
    a.a_end[l] = A;
    a.stride[l] = d->stride[l];
  }
  a.nl = d->nl; a.nc = d->nc; a.A = A;
  a.conf = d->conf_thres; a.multi = d->multi_label;
  a.classes = d->classes; a.ncls = d->nclasses;
  a.yref = d->y_ref;
  a.cbox = d->cand_box; a.cscore = d->cand_score; a.ccls = d->cand_cls; a.cidx = d->cand_idx; a.ccount = d->cand_count;
  a.cap = d->cap;
  const int B = d->box[0].n;
  if (hipMemsetAsync(d->cand_count, 0, sizeof(int) * B, s) != hipSuccess) return check_launch("decode memset");
  decode_kernel<T><<<dim3((unsigned)cdiv(A, 256), B), 256, 0, s>>>(a);
  return check_launch("ydbl_detect_decode");
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_detect_decode(const ydbl_decode_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "decode: null descriptor");
  if (d->nl < 1 || d->nl > 3) return fail(YDBL_EINVAL, "decode: 1..3 levels");
  for (int l = 0; l < d->nl; ++l) {
    if (check_view(&d->box[l], "decode.box", false) || check_view(&d->cls[l], "decode.cls", false)) return YDBL_EINVAL;
    if (d->box[l].c != 64 || d->cls[l].c != d->nc || d->box[l].h != d->cls[l].h || d->box[l].w != d->cls[l].w ||
        d->box[l].n != d->box[0].n || d->cls[l].n != d->box[0].n || d->box[l].dtype != d->box[0].dtype ||
        d->cls[l].dtype != d->box[0].dtype)
      return fail(YDBL_EINVAL, "decode: level shape mismatch");
    if (d->box[l].cs % (d->box[l].dtype == YDBL_F16 ? 8 : 4))
      return fail(YDBL_EINVAL, "decode: box channel stride must be 16-byte aligned");
  }
  if (!d->cand_box || !d->cand_score || !d->cand_cls || !d->cand_idx || !d->cand_count || d->cap < 1)
    return fail(YDBL_EINVAL, "decode: null candidate buffers");
  hipStream_t s = as_stream(stream);
  return d->box[0].dtype == YDBL_F16 ? decode_t<_Float16>(d, s) : decode_t<float>(d, s);
}

extern "C" int ydbl_pred_candidates(const ydbl_pred_cand_desc* d, void* stream) {
  if (!d || !d->pred) return fail(YDBL_EINVAL, "pred_candidates: null prediction");
  if (d->n < 1 || d->nc < 1 || d->A < 1) return fail(YDBL_EINVAL, "pred_candidates: bad shape");
  if (!d->cand_box || !d->cand_score || !d->cand_cls || !d->cand_idx || !d->cand_count || d->cap < 1)
    return fail(YDBL_EINVAL, "pred_candidates: null candidate buffers");
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(d->cand_count, 0, sizeof(int) * d->n, s) != hipSuccess) return check_launch("pred memset");
  pred_cand_kernel<<<dim3((unsigned)cdiv(d->A, 256), d->n), 256, 0, s>>>(*d);
  return check_launch("ydbl_pred_candidates");
}

extern "C" int64_t ydbl_nms_workspace(int32_t n, int32_t cap, int32_t max_nms) {
  (void)max_nms;
  const int L = next_pow2(cap < SORT_CHUNK ? SORT_CHUNK : cap);
  return (int64_t)n * L * (8 + 4);
}

extern "C" int ydbl_nms(const ydbl_nms_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "nms: null descriptor");
  if (!d->cand_box || !d->cand_score || !d->cand_cls || !d->cand_idx || !d->cand_count || !d->out || !d->out_count ||
      !d->workspace)
    return fail(YDBL_EINVAL, "nms: null buffer");
  if (d->n < 1 || d->cap < 1) return fail(YDBL_EINVAL, "nms: empty batch");
  if (d->max_det < 1 || d->max_det > NMS_MAX_DET) return fail(YDBL_EINVAL, "nms: max_det must be in [1, 4096]");
  if (d->max_nms < 1 || d->max_nms > NMS_MAX_FLAGS) return fail(YDBL_EINVAL, "nms: max_nms must be in [1, 32768]");
  if (!(d->iou_thres >= 0.0 && d->iou_thres <= 1.0)) return fail(YDBL_EINVAL, "nms: iou_thres must be in [0, 1]");
  hipStream_t s = as_stream(stream);
  const int L = next_pow2(d->cap < SORT_CHUNK ? SORT_CHUNK : d->cap);
  uint64_t* keys = reinterpret_cast<uint64_t*>(d->workspace);
  int* vals = reinterpret_cast<int*>(keys + (int64_t)d->n * L);
  nms_keys_kernel<<<dim3((unsigned)cdiv(L, 1024), d->n), 1024, 0, s>>>(d->cand_score, d->cand_idx, d->cand_count,
                                                                       d->cap, L, keys, vals);
  const int chunk = SORT_CHUNK;
  bitonic_local_kernel<<<dim3(L / chunk, d->n), 1024, 0, s>>>(keys, vals, L, chunk, 0);
  for (int k = 2 * chunk; k <= L; k <<= 1) {
    for (int j = k >> 1; j >= chunk; j >>= 1)
      bitonic_global_kernel<<<dim3((unsigned)cdiv(L / 2, 256), d->n), 256, 0, s>>>(keys, vals, L, k, j);
    bitonic_local_kernel<<<dim3(L / chunk, d->n), 1024, 0, s>>>(keys, vals, L, chunk, k);
  }
  NmsArgs a;
  a.cbox = d->cand_box; a.cscore = d->cand_score; a.ccls = d->cand_cls; a.ccount = d->cand_count;
  a.vals = vals; a.L = L; a.cap = d->cap;
  a.thr = d->iou_thres; a.max_det = d->max_det; a.max_nms = d->max_nms;
  a.off_scale = d->agnostic ? 0.f : d->max_wh;
  a.clip_w = d->clip_w; a.clip_h = d->clip_h;
  a.out = d->out; a.out_count = d->out_count;
  nms_greedy_kernel<<<d->n, 1024, 0, s>>>(a);
  return check_launch("ydbl_nms");
}
