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
#include <stdlib.h>

#include <algorithm>

#include "common.hpp"

extern "C" __device__ unsigned long long __ockl_wfred_or_u64(unsigned long long);  // DPP wave OR (ockl)

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

// Slot of this lane's candidate in image b's list: one atomic per wave (the first active lane adds the
// wave's candidate count, the others take their rank among the active lanes).  Candidates cluster on
// objects, so a wave often holds tens of them; per-lane atomics on the one counter serialize in L2.
__device__ __forceinline__ int wave_slot(int* counter, bool want) {
  const uint64_t m = __ballot(want);
  if (!want) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  return base + __popcll(m & ((1ull << lane) - 1));
}

__device__ __forceinline__ bool class_ok(int j, const int* classes, int ncls) {
  if (!classes) return true;
  for (int q = 0; q < ncls; ++q)
    if (classes[q] == j) return true;
  return false;
}

// Four lanes per anchor (a quad): lane s computes side s's DFL expectation (16 bins; the quad's four sides are
// then shared by shuffles) and the classes j = s, s + 4, ...; so a lane's dependent chain is 16 exponentials
// instead of 64, and the launch has four times the waves to hide it.  Same arithmetic per value as one lane per
// anchor: the decoded boxes, scores and candidate sets are unchanged (candidate order within an image may differ;
// every candidate carries its anchor / class index).
template <typename T>
__global__ __launch_bounds__(256) void decode_kernel(DecodeArgs<T> p) {
  const int b = blockIdx.y;
  const int tq = blockIdx.x * blockDim.x + threadIdx.x;
  const int a = tq >> 2, s = tq & 3;
  if (a >= p.A) return;  // whole quads
  int l = 0;
  while (l < p.nl - 1 && a >= p.a_end[l]) ++l;
  const int a0 = l ? p.a_end[l - 1] : 0;
  const int loc = a - a0;
  const DView<const T>& bx = p.box[l];
  const int gx = loc % bx.w, gy = loc / bx.w;
  const T* bp = bx.at(b, gy, gx);
  float mine;
  {  // DFL: softmax over 16 bins, expectation with weights 0..15
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
    // softmax weights as e * (1 / sum): one division per side instead of 16 (<= 1 ulp per weight, far
    // inside the decode tolerance; the reference's DFL conv sums the 16 products in its own order anyway)
    const float inv = 1.0f / sum;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += float(k) * (e[k] * inv);
    mine = acc;
  }
  const int q0 = (threadIdx.x & 63) & ~3;  // the quad's first lane
  float dist[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) dist[k] = __shfl(mine, q0 + k);
  const float ax = float(gx) + 0.5f, ay = float(gy) + 0.5f, st = p.stride[l];
  const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
  const float cx = ((x1 + x2) / 2.0f) * st, cy = ((y1 + y2) / 2.0f) * st;
  const float w = (x2 - x1) * st, h = (y2 - y1) * st;
  const int64_t A = p.A;
  if (p.yref) {
    float* yr = p.yref + (int64_t)b * (4 + p.nc) * A + a;
    yr[s * A] = s == 0 ? cx : s == 1 ? cy : s == 2 ? w : h;
  }
  // xywh2xyxy (U/utils/ops.py:416-433)
  const float hw = w / 2.0f, hh = h / 2.0f;
  const float bx1 = cx - hw, by1 = cy - hh, bx2 = cx + hw, by2 = cy + hh;
  const T* cp = p.cls[l].at(b, gy, gx);
  float best = -1.f;
  int bj = 0;
  for (int j = s; j < p.nc; j += 4) {
    const float sc = 1.0f / (1.0f + expf(-float(cp[j])));
    if (p.yref) p.yref[((int64_t)b * (4 + p.nc) + 4 + j) * A + a] = sc;
    if (p.multi) {
      const int slot = wave_slot(p.ccount + b, sc > p.conf && class_ok(j, p.classes, p.ncls));
      if (slot >= 0) {
        if (slot < p.cap) {
          const int64_t o = (int64_t)b * p.cap + slot;
          *reinterpret_cast<f32x4*>(p.cbox + o * 4) = f32x4{bx1, by1, bx2, by2};
          p.cscore[o] = sc; p.ccls[o] = j; p.cidx[o] = a * p.nc + j;
        }
      }
    } else if (sc > best) {  // torch.max: first index of the maximum (within this lane's classes)
      best = sc;
      bj = j;
    }
  }
  if (p.multi) return;
  // the quad's first maximum: larger score, or the same score at a smaller class index
#pragma unroll
  for (int k = 1; k < 4; k <<= 1) {
    const float ob = __shfl_xor(best, k);
    const int oj = __shfl_xor(bj, k);
    if (ob > best || (ob == best && oj < bj)) {
      best = ob;
      bj = oj;
    }
  }
  const int slot = wave_slot(p.ccount + b, s == 0 && best > p.conf && class_ok(bj, p.classes, p.ncls));
  if (slot >= 0) {
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
      const int slot = wave_slot(p.cand_count + b, sc > p.conf_thres && class_ok(j, p.classes, p.nclasses));
      if (slot >= 0) {
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
  const int slot =
      p.multi_label ? -1 : wave_slot(p.cand_count + b, best > p.conf_thres && class_ok(bj, p.classes, p.nclasses));
  if (slot >= 0) {
    if (slot < p.cap) {
      const int64_t o = (int64_t)b * p.cap + slot;
      *reinterpret_cast<f32x4*>(p.cand_box + o * 4) = f32x4{bx1, by1, bx2, by2};
      p.cand_score[o] = best; p.cand_cls[o] = bj; p.cand_idx[o] = a;
    }
  }
}

// ------------------------------------------------------------------------------------ NMS
// One 1024-thread workgroup per image does the whole post-filter path of U/utils/ops.py:278-310:
//   1. sort the image's candidates by (score desc, original index asc) -- torchvision's stable
//      descending sort over candidates that are in anchor (or torch.where) order -- bitonic in LDS
//      for n <= NMS_SORT_LDS, in the global workspace (same workgroup, barrier-separated) above;
//   2. truncate to max_nms (the reference's argsort(descending)[:max_nms] gives the same prefix);
//   3. greedy sweep in chunks of 64 sorted boxes: the 16 waves compute the chunk's 64x64 upper-
//      triangular suppression mask in parallel, wave 0 resolves the chunk serially on a wave-
//      uniform 64-bit live mask (find-first-set, readlane of the kept row's mask, and-not), then
//      all waves suppress every later box against the chunk's kept boxes (LDS byte flags).
//      Kept boxes come out in score order, so stopping at max_det == keep[:max_det].
//   IoU arithmetic is torchvision's CPU kernel in fp32: inter / (area_i + area_j - inter),
//   compared as double against iou_thres; areas without +1; boxes offset by cls * max_wh.
constexpr int NMS_SORT_LDS = 8192;   // candidates sorted in LDS (8 B key + 4 B slot each)
constexpr int NMS_MAX_FLAGS = 32768;  // max_nms limit (LDS suppression flags, 1 B each)
constexpr int NMS_MAX_DET = 4096;
constexpr int NMS_THREADS = 1024;

__device__ __forceinline__ uint64_t make_key(float score, int idx) {
  // candidate scores are > conf_thres >= 0: positive floats order like their bit patterns.
  const uint32_t sb = __float_as_uint(score);
  return ((uint64_t)(0xFFFFFFFFu - sb) << 32) | (uint32_t)idx;
}

constexpr int NMS_GROUPS = 8;  // class groups (cls % 8) swept by separate workgroups

struct NmsArgs {
  const float* cbox; const float* cscore; const int* ccls; const int* cidx; const int* ccount;
  uint64_t* gkeys; int* gvals; int L;  // global sort scratch (only when cap > NMS_SORT_LDS)
  int* gslot; uint64_t* gkey; int* gcount; int gk;  // per (image, class group) keep lists, gk entries each
  int cap;
  uint64_t* fmask; int* frank; int frows; int fast;  // pair-matrix path (nms_pair_kernel), frows rows per image
  // wide pair-matrix path (NMS_FAST < n <= NMS_WIDE): per image wrows rows of rank accumulators (zero between
  // calls: the sweep clears what nms_pair_kernel added), rank -> slot order, and the rank-space IoU rows
  // (wwords words each; only the words at and right of a row's own 64-rank block are written)
  unsigned long long* wacc; int* worder; uint64_t* wmask; int wrows; int wwords;
  double thr; int max_det, max_nms; float off_scale;
  float clip_w, clip_h;
  float* out; int* out_count;
  int64_t ostride; int64_t cstride;  // floats per image of out, int32s per image of out_count
};

// bitonic sort of P (power of two) key/value pairs; keys/vals in LDS or global, one workgroup
template <typename KP, typename VP>
__device__ void block_bitonic(KP keys, VP vals, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += NMS_THREADS) {
        const int i = 2 * j * (t / j) + (t % j);
        const int ixj = i + j;
        const bool up = (i & k) == 0;
        const uint64_t a = keys[i], c = keys[ixj];
        if ((a > c) == up) {
          keys[i] = c; keys[ixj] = a;
          const int tv = vals[i]; vals[i] = vals[ixj]; vals[ixj] = tv;
        }
      }
      __syncthreads();
    }
  }
}

// Bitonic sort of P <= NMS_THREADS (power of two) keys held one per thread (thread t: element t),
// values carried along.  Exchanges with partner t ^ j: inside the wave (j < 64) by cross-lane
// shuffles, no barrier; across waves through two LDS ping-pong buffers, one barrier per stage (a
// thread reaches stage s+1's barrier only after its stage-s read, so the buffer it overwrites two
// stages later is no longer read).  log2(P) (log2(P) + 1) / 2 stages, of which only the j >= 64 ones
// (10 at P = 1024) touch LDS.
__device__ void reg_bitonic(uint64_t& key, int& val, int P, uint64_t* xk, int* xv) {
  const int t = threadIdx.x;
  int stage = 0;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint64_t ok;
      int ov;
      if (j < 64) {
        const uint32_t lo = __shfl_xor((uint32_t)key, j), hi = __shfl_xor((uint32_t)(key >> 32), j);
        ok = ((uint64_t)hi << 32) | lo;
        ov = __shfl_xor(val, j);
      } else {
        uint64_t* bk = xk + (stage & 1) * NMS_THREADS;
        int* bv = xv + (stage & 1) * NMS_THREADS;
        bk[t] = key;
        bv[t] = val;
        __syncthreads();
        ok = bk[t ^ j];
        ov = bv[t ^ j];
        ++stage;
      }
      if (t < P) {
        const bool up = (t & k) == 0, lower = (t & j) == 0;
        const bool take = (lower == up) ? ok < key : ok > key;
        if (take) {
          key = ok;
          val = ov;
        }
      }
    }
  }
}

__device__ __forceinline__ bool iou_gt(const f32x4& a, float area_a, const f32x4& b, double thr) {
  const float xx1 = fmaxf(a[0], b[0]), yy1 = fmaxf(a[1], b[1]);
  const float xx2 = fminf(a[2], b[2]), yy2 = fminf(a[3], b[3]);
  const float ww = fmaxf(0.f, xx2 - xx1), hh = fmaxf(0.f, yy2 - yy1);
  const float inter = ww * hh;
  if (!(inter > 0.f)) return false;  // IoU 0 is never > thr (thr in [0, 1])
  const float area_b = (b[2] - b[0]) * (b[3] - b[1]);
  const float uni = (area_a + area_b) - inter;
  // The decision is torchvision's: the correctly rounded fp32 quotient inter / uni, compared in
  // double.  inter * rcp(uni) is within a few ulp of that quotient, so it decides alone unless it
  // lies within 1e-5 (relative) of the threshold; only those cases pay for the IEEE division.
  const float approx = inter * __builtin_amdgcn_rcpf(uni);
  const double ad = (double)approx;
  if (ad > thr * (1.0 + 1e-5) + 1e-30) return true;
  if (ad < thr * (1.0 - 1e-5) - 1e-30) return false;
  const float ovr = inter / uni;
  return (double)ovr > thr;
}

// Diagnostic build only (-DYDBL_NMS_STAMPS, scripts/build_stamps.sh detect, scripts/nms_stamps.py): per-workgroup phase timestamps.
#ifdef YDBL_NMS_STAMPS
__device__ unsigned long long g_nms_stamps[16 * 4096];
#define NMS_STAMP(k, v) \
  do { if (threadIdx.x == 0) g_nms_stamps[blockIdx.x * 16 + (k)] = (v); } while (0)
#define NMS_TICK(acc) \
  do { const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); acc += t_ - t_last; t_last = t_; } while (0)
#else
#define NMS_STAMP(k, v) do { } while (0)
#define NMS_TICK(acc) do { } while (0)
#endif

// ---- pair-matrix path for images with n <= NMS_FAST candidates (the common case) --------------------
// The greedy sweep of one image is serial, but everything it consumes is not: nms_pair_kernel spreads the
// n x n candidate pairs of every image over the chip (64 x 64 blocks, one per workgroup at a time, each
// wave testing 16 of the block's columns) and writes, in candidate (slot) order,
//   fmask[b][i][w] bit s = IoU(box i, box 64w+s) > thr   (torchvision's decision, iou_gt; the IoU is
//                                                         symmetric bit for bit, so row i is what box i
//                                                         suppresses whichever of the two ranks first)
//   frank[b][w][i]       = #{j in block w : key_j < key_i} (partial ranks; keys are unique)
// and nms_kernel then only sums the ranks (rank = sort position, as the stable sort), stages the rows in
// LDS and runs the sweep in rank order on one wave, 64 ranks at a time: a candidate is kept iff its bit
// in the running removed mask is clear and no kept candidate earlier in its block suppresses it, and a
// kept candidate ORs its row into the mask.  Rows of candidates ranked earlier get bits set too, which
// changes nothing: their decision is already made.
constexpr int NMS_FAST = 1024;        // candidates per image on this path (mask rows staged in LDS: 128 KiB)
constexpr int NMS_FW = NMS_FAST / 64;  // 64-bit words per mask row

// LDS slot of word w of mask row c: the words of a row are XOR-permuted by the row's low bits, so that
// 64 lanes reading the same word of 64 different rows (the rank-word build) spread over the banks, while
// the 16 words of one row (the sweep's row reads) stay one conflict-free 128-byte line.
__device__ __forceinline__ int mslot(int c, int w) { return c * NMS_FW + (w ^ (c & (NMS_FW - 1))); }

__device__ __forceinline__ float rlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

constexpr int NMS_WIDE = 8192;       // candidates per image on the wide pair-matrix path (rows in rank space)
constexpr int NMS_WIDE_COLS = 1024;  // columns per rank item of nms_pair_kernel (4 waves x 256)
constexpr int NMS_PAIR_MAXB = 1024;  // images per launch on the pair-matrix path (block offsets in LDS)
constexpr int NMS_PAIR_WGS = 512;    // workgroups, each taking 64 x 64 blocks in turn

// Persistent over all images' blocks: no workgroup is launched for an image with few candidates (a
// (32 x images) grid of one block per wave took 22 us, mostly dispatching empty workgroups and walking a
// block's 64 columns on one wave), and the blocks of a heavy image spread over the whole chip.
__global__ __launch_bounds__(256) void nms_pair_kernel(NmsArgs p, int nimg) {
  __shared__ int s_pre[NMS_PAIR_MAXB + 1];  // s_pre[b] = blocks of images < b
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave == 0) {
    int run = 0;
    for (int b0 = 0; b0 < nimg; b0 += 64) {
      const int bb = b0 + lane;
      int cnt = 0;
      if (bb < nimg) {
        const int nn = min(p.ccount[bb], p.cap);
        const int nbb = (nn + 63) >> 6;
        cnt = nn <= NMS_FAST ? nbb * nbb
              : (nn <= NMS_WIDE && p.wrows > 0 ? nbb * ((nn + NMS_WIDE_COLS - 1) / NMS_WIDE_COLS) : 0);
      }
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      if (bb < nimg) s_pre[bb + 1] = run + incl;
      run += __shfl(incl, 63);
    }
    if (lane == 0) s_pre[0] = 0;
  }
  __syncthreads();
  __shared__ uint64_t s_bits[4][64];
  __shared__ int s_cnt[4][64];
  const int total = s_pre[nimg];
  // a workgroup takes one 64 x 64 block at a time; wave w tests its rows against columns 16w .. 16w+15
  for (int g = blockIdx.x; g < total; g += gridDim.x) {
    int lo = 0, hi = nimg - 1;  // image b: s_pre[b] <= g < s_pre[b + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    const int b = lo;
    const int n = min(p.ccount[b], p.cap);
    const int nb = (n + 63) >> 6;
    const int t = g - s_pre[b];
    const float* cb = p.cbox + (int64_t)b * p.cap * 4;
    const float* sc = p.cscore + (int64_t)b * p.cap;
    const int* ix = p.cidx + (int64_t)b * p.cap;
    const int* cc = p.ccls + (int64_t)b * p.cap;
    if (n > NMS_FAST) {
      // wide image: a rank item = 64 candidates (rows) against NMS_WIDE_COLS columns, wave w taking 256 of them;
      // the item adds its count of smaller keys and one contribution into the row's 64-bit accumulator, and the
      // row's last contribution (all ng column groups in) knows the final rank = the stable-sort position and
      // writes order[rank] = slot
      const int ng = (n + NMS_WIDE_COLS - 1) / NMS_WIDE_COLS;
      const int bi = t / ng, gq = t - bi * ng;
      const int i = bi * 64 + lane, ic = min(i, n - 1);
      const uint64_t ki = make_key(sc[ic], ix[ic]);
      const int c0 = gq * NMS_WIDE_COLS + wave * 256;
      uint32_t kh[4], kl[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // the wave's 256 column keys, all loads issued first
        const int jc = min(c0 + q * 64 + lane, n - 1);
        const uint64_t k = make_key(sc[jc], ix[jc]);
        kh[q] = (uint32_t)(k >> 32);
        kl[q] = (uint32_t)k;
      }
      int below = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ns = min(64, n - (c0 + q * 64));  // wave-uniform; <= 0 past the end
        for (int s = 0; s < ns; ++s) {
          const uint64_t k = ((uint64_t)__builtin_amdgcn_readlane(kh[q], s) << 32) | __builtin_amdgcn_readlane(kl[q], s);
          below += k < ki;
        }
      }
      s_cnt[wave][lane] = below;
      __syncthreads();
      if (wave == 0 && i < n) {
        const int tot = s_cnt[0][lane] + s_cnt[1][lane] + s_cnt[2][lane] + s_cnt[3][lane];
        const unsigned long long old =
            atomicAdd(p.wacc + (int64_t)b * p.wrows + i, (1ull << 32) | (unsigned long long)(unsigned)tot);
        if ((int)(old >> 32) == ng - 1) p.worder[(int64_t)b * p.wrows + (int)(uint32_t)old + tot] = i;
      }
      __syncthreads();
      continue;
    }
    const int bi = t / nb, bj = t - bi * nb;
    auto box_of = [&](int i) -> f32x4 {  // the sweep's class-offset box (nms_kernel load_box)
      const f32x4 v = *reinterpret_cast<const f32x4*>(cb + (int64_t)i * 4);
      const float c = float(cc[i]) * p.off_scale;
      return f32x4{v[0] + c, v[1] + c, v[2] + c, v[3] + c};
    };
    const int i = bi * 64 + lane, j = bj * 64 + 16 * wave + (lane & 15);
    const int ic = min(i, n - 1), jc = min(j, n - 1);
    const f32x4 xi = box_of(ic), xj = box_of(jc);
    const float ai = (xi[2] - xi[0]) * (xi[3] - xi[1]);
    const uint64_t ki = make_key(sc[ic], ix[ic]), kj = make_key(sc[jc], ix[jc]);
    const uint32_t kjh = (uint32_t)(kj >> 32), kjl = (uint32_t)kj;
    const int ns = min(16, n - bj * 64 - 16 * wave);  // this wave's columns (may be <= 0)
    uint64_t bits = 0;
    int below = 0;
    for (int s = 0; s < ns; ++s) {
      const f32x4 y = f32x4{rlane(xj[0], s), rlane(xj[1], s), rlane(xj[2], s), rlane(xj[3], s)};
      const uint64_t k = ((uint64_t)__builtin_amdgcn_readlane(kjh, s) << 32) | __builtin_amdgcn_readlane(kjl, s);
      below += k < ki;
      if (iou_gt(xi, ai, y, p.thr)) bits |= 1ull << (16 * wave + s);
    }
    s_bits[wave][lane] = bits;
    s_cnt[wave][lane] = below;
    __syncthreads();
    if (wave == 0 && i < n) {
      p.fmask[((int64_t)b * p.frows + i) * NMS_FW + bj] = s_bits[0][lane] | s_bits[1][lane] | s_bits[2][lane] | s_bits[3][lane];
      p.frank[((int64_t)b * NMS_FW + bj) * p.frows + i] = s_cnt[0][lane] + s_cnt[1][lane] + s_cnt[2][lane] + s_cnt[3][lane];
    }
    __syncthreads();
  }
}

// Wide images, after nms_pair_kernel has ranked them: the IoU > thr bits of every pair of the first m = min(n,
// max_nms) ranks, in rank space, row r word w bit s = IoU(rank r, rank 64w + s) > thr, for the 64 x 64 blocks on
// and right of the diagonal (w >= r / 64; the sweep reads no other word).  Each wave takes one block at a time
// (lane = row, the 64 columns broadcast by readlane), no barrier; persistent over all images' blocks.
__global__ __launch_bounds__(256) void nms_wide_mask_kernel(NmsArgs p, int nimg) {
  __shared__ int s_pre[NMS_PAIR_MAXB + 1];  // s_pre[b] = blocks of images < b
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave == 0) {
    int run = 0;
    for (int b0 = 0; b0 < nimg; b0 += 64) {
      const int bb = b0 + lane;
      int cnt = 0;
      if (bb < nimg) {
        const int nn = min(p.ccount[bb], p.cap);
        const int nbm = (min(nn, p.max_nms) + 63) >> 6;
        cnt = nn > NMS_FAST && nn <= NMS_WIDE ? nbm * (nbm + 1) / 2 : 0;
      }
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      if (bb < nimg) s_pre[bb + 1] = run + incl;
      run += __shfl(incl, 63);
    }
    if (lane == 0) s_pre[0] = 0;
  }
  __syncthreads();
  const int total = s_pre[nimg];
  for (int g = blockIdx.x * 4 + wave; g < total; g += gridDim.x * 4) {
    int lo = 0, hi = nimg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    const int b = lo;
    const int n = min(p.ccount[b], p.cap);
    const int m = min(n, p.max_nms);
    const int nbm = (m + 63) >> 6;
    int t = g - s_pre[b], bi = 0;  // upper-triangular block index -> (bi, bj >= bi)
    while (t >= nbm - bi) {
      t -= nbm - bi;
      ++bi;
    }
    const int bj = bi + t;
    const float* cb = p.cbox + (int64_t)b * p.cap * 4;
    const int* cc = p.ccls + (int64_t)b * p.cap;
    const int* ord = p.worder + (int64_t)b * p.wrows;
    const int r = bi * 64 + lane;
    const int si = ord[min(r, m - 1)], sj = ord[min(bj * 64 + lane, m - 1)];
    const f32x4 vi = *reinterpret_cast<const f32x4*>(cb + (int64_t)si * 4);
    const f32x4 vj = *reinterpret_cast<const f32x4*>(cb + (int64_t)sj * 4);
    const float ci = float(cc[si]) * p.off_scale, cj = float(cc[sj]) * p.off_scale;
    const f32x4 xi = f32x4{vi[0] + ci, vi[1] + ci, vi[2] + ci, vi[3] + ci};
    const f32x4 xj = f32x4{vj[0] + cj, vj[1] + cj, vj[2] + cj, vj[3] + cj};
    const float ai = (xi[2] - xi[0]) * (xi[3] - xi[1]);
    const int ns = min(64, m - bj * 64);
    uint64_t bits = 0;
    for (int s = 0; s < ns; ++s) {
      const f32x4 y = f32x4{rlane(xj[0], s), rlane(xj[1], s), rlane(xj[2], s), rlane(xj[3], s)};
      if (iou_gt(xi, ai, y, p.thr)) bits |= 1ull << s;
    }
    if (r < m) p.wmask[((int64_t)b * p.wrows + r) * p.wwords + bj] = bits;
  }
}

// GROUPS: the class-split form (non-agnostic NMS).  Boxes are offset by cls * max_wh, so boxes of
// different classes never overlap and torchvision's greedy sweep is, class by class, independent: the
// keep set of an image is the union of the keep sets of any partition of its classes, in (score, index)
// order.  Workgroup (image b, group g) runs the sweep on the candidates with cls % NMS_GROUPS == g and
// leaves its keep list (slots + sort keys, at most max_det) in the workspace; nms_merge_kernel ranks the
// groups' lists into the final max_det rows.  An image whose candidates exceed max_nms (the reference's
// global pre-NMS truncation) or the LDS sort runs whole in group 0 (the other groups leave empty lists).
template <bool GROUPS>
__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(NmsArgs p) {
  // LDS: sort keys (64 KB) are reused for the first 4096 sorted boxes after sorting.
  // sort keys | sort slots | suppression flags, one buffer: the pair-matrix path stages its mask rows
  // (NMS_FAST x NMS_FW words = 128 KiB) over all three
  __shared__ __align__(16) unsigned char s_raw[NMS_SORT_LDS * 12 + NMS_MAX_FLAGS];
  static_assert(NMS_FAST * NMS_FW * 8 <= NMS_SORT_LDS * 12 + NMS_MAX_FLAGS, "pair-matrix rows fit the sort buffers");
  uint64_t* s_keys = reinterpret_cast<uint64_t*>(s_raw);
  int* s_vals = reinterpret_cast<int*>(s_raw + NMS_SORT_LDS * 8);
  unsigned char* removed = s_raw + NMS_SORT_LDS * 12;
  __shared__ int kept_slot[NMS_MAX_DET];
  __shared__ int s_order[NMS_FAST];
  __shared__ uint64_t s_dw[NMS_FAST];
  __shared__ int s_wsum[NMS_THREADS / 64];
  __shared__ f32x4 chunk_box[64];
  __shared__ float chunk_area[64];
  __shared__ unsigned char cmask[64][16];
  __shared__ int s_nk;
  f32x4* s_box = reinterpret_cast<f32x4*>(s_keys);
  constexpr int LDS_BOXES = NMS_SORT_LDS * 8 / 16;

  NMS_STAMP(0, __builtin_amdgcn_s_memrealtime());
  bool kept_rank = false;  // the wide path keeps ranks in kept_slot (slot = worder[rank])
  const int b = GROUPS ? blockIdx.x / NMS_GROUPS : blockIdx.x;
  const int grp = GROUPS ? blockIdx.x % NMS_GROUPS : 0;
  int n = min(p.ccount[b], p.cap);
  const float* sc = p.cscore + (int64_t)b * p.cap;
  const int* ix = p.cidx + (int64_t)b * p.cap;
  if (p.fast && n <= NMS_FAST) {
    // ---- pair-matrix path (nms_pair_kernel filled fmask / frank for this image)
    if constexpr (GROUPS) {
      if (grp != 0) {  // the whole image is group 0's
        if (threadIdx.x == 0) p.gcount[(int64_t)b * NMS_GROUPS + grp] = 0;
        return;
      }
    }
    const int m = min(n, p.max_nms);  // the reference's argsort(descending)[:max_nms]
    const int nb = (n + 63) >> 6;
    const int* rpart = p.frank + (int64_t)b * NMS_FW * p.frows;
    // every global load of this thread is issued before the first one is used (fixed trip counts)
    static_assert(NMS_FAST == NMS_THREADS, "one candidate per thread");
    {
      const int i = threadIdx.x;
      int part[NMS_FW];
#pragma unroll
      for (int w = 0; w < NMS_FW; ++w) part[w] = i < n && w < nb ? rpart[w * p.frows + i] : 0;
      int r = 0;
#pragma unroll
      for (int w = 0; w < NMS_FW; ++w) r += part[w];
      if (i < n && r < m) s_order[r] = i;
    }
    uint64_t* smask = reinterpret_cast<uint64_t*>(s_raw);  // [n][NMS_FW]
    {
      const uint64_t* gm = p.fmask + (int64_t)b * p.frows * NMS_FW;
      uint64_t v[NMS_FW];
#pragma unroll
      for (int k = 0; k < NMS_FW; ++k) {
        const int e = threadIdx.x + k * NMS_THREADS;
        v[k] = e < n * NMS_FW && (e & (NMS_FW - 1)) < nb ? gm[e] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < NMS_FW; ++k) {
        const int e = threadIdx.x + k * NMS_THREADS;
        if (e < n * NMS_FW) smask[mslot(e >> 4, e & (NMS_FW - 1))] = v[k];
      }
    }
    __syncthreads();
    NMS_STAMP(1, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(2, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(6, (unsigned long long)m);
    // within-block suppression words in rank space: s_dw[r] bit s = row of rank r suppresses rank
    // 64*(r/64) + s, for s > r%64 (wave w builds block w: the column candidates are wave-uniform)
    // (branch-free body: the 64 row reads of a lane are issued back to back)
    if ((int)(threadIdx.x & ~63) < m) {
      const int r = threadIdx.x, k0 = r & ~63, rl = r & 63;
      const int cr = r < m ? s_order[r] : 0;  // lane rl holds the candidate of rank k0 + rl (this wave's block)
      const int send = min(64, m - k0);
      uint64_t dw = 0;
#pragma unroll 8
      for (int q = 0; q < 64; ++q) {
        const int cq = __builtin_amdgcn_readlane(cr, q);
        const uint64_t bit = (smask[mslot(cr, (cq >> 6) & (NMS_FW - 1))] >> (cq & 63)) & 1ull;
        dw |= (q > rl && q < send) ? bit << q : 0ull;
      }
      if (r < m) s_dw[r] = dw;
    }
    __syncthreads();
    NMS_STAMP(4, __builtin_amdgcn_s_memrealtime());
    if (threadIdx.x < 64) {  // one wave sweeps the rank blocks in order
      const int lane = threadIdx.x;
      uint64_t rem = 0;  // lane w < nb: removed flags of candidates 64w .. 64w+63
      int nk = 0;
      for (int t0 = 0; t0 < m && nk < p.max_det; t0 += 64) {
        const bool valid = t0 + lane < m;
        const int myc = valid ? s_order[t0 + lane] : 0;
        const uint64_t dw = valid ? s_dw[t0 + lane] : 0ull;
        // alive = not removed by a kept candidate of an earlier block
        const int wsrc = myc >> 6;
        const uint32_t rlo = __shfl((uint32_t)rem, wsrc), rhi = __shfl((uint32_t)(rem >> 32), wsrc);
        const uint64_t rw = ((uint64_t)rhi << 32) | rlo;
        const uint64_t M = __ballot(valid && !((rw >> (myc & 63)) & 1));
        const int nk0 = nk;
        // greedy inside the block: K_r = M_r & !(any s < r in K with D[s] bit r).  Iterated from K = M as
        // K' = M & ~OR_{s in K} D[s] (one wave-wide OR per step) it reaches that unique fixed point: after t
        // steps the first t ranks are final, and steps stop as soon as K repeats -- a few for NMS clusters,
        // where the scalar walk paid one dependent step per kept rank
        uint64_t K = M;
        for (;;) {
          const uint64_t W = __ockl_wfred_or_u64((K >> lane) & 1 ? dw : 0ull);
          const uint64_t Kn = M & ~W;
          if (Kn == K) break;
          K = Kn;
        }
        // keep[:max_det]: the greedy stops at max_det keeps, i.e. the lowest ranks of K
        for (int extra = __popcll(K) - (p.max_det - nk0); extra > 0; --extra) K &= ~(1ull << (63 - __clzll(K)));
        nk = nk0 + __popcll(K);
        if ((K >> lane) & 1) kept_slot[nk0 + __popcll(K & ((1ull << lane) - 1))] = myc;
        // the kept candidates' rows join the removed flags (8 row reads in flight at a time)
        // (branch-free: all 8 reads are issued before the first OR)
        while (K) {
          int c[8];
          bool ok[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int t = __ffsll((long long)K) - 1;  // -1 once K is empty
            K &= K - 1;
            ok[q] = t >= 0;
            c[q] = __builtin_amdgcn_readlane(myc, t & 63);
          }
          uint64_t row[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) row[q] = smask[mslot(c[q], lane & (NMS_FW - 1))];
#pragma unroll
          for (int q = 0; q < 8; ++q) rem |= ok[q] && lane < nb ? row[q] : 0ull;
        }
      }
      if (lane == 0) s_nk = nk;
    }
    __syncthreads();
    NMS_STAMP(3, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(5, 0ull);
  } else if (p.fast && p.wrows > 0 && n <= NMS_WIDE) {
    // ---- wide pair-matrix path: the ranks and rank-space IoU rows come from nms_pair_kernel and
    // nms_wide_mask_kernel; the sweep walks the ranks in chunks of NMS_FAST.  Per chunk: the ranks not yet
    // removed by an earlier chunk's kept rows are compacted (rank order kept), their rows' words over the chunk
    // are staged in LDS and the chunk runs exactly the pair-matrix sweep above (within-block words, fixed-point
    // block greedy, kept rows ORed into the chunk's removed flags); then the rows of the chunk's new keeps are
    // ORed, over the ranks right of the chunk, into the image's removed bits -- so a chunk only ever sweeps
    // ranks nothing kept before it suppresses.
    if constexpr (GROUPS) {
      if (grp != 0) {  // the whole image is group 0's
        if (threadIdx.x == 0) p.gcount[(int64_t)b * NMS_GROUPS + grp] = 0;
        return;
      }
    }
    kept_rank = true;
    const int m = min(n, p.max_nms);
    const int W = (m + 63) >> 6;
    uint64_t* wrem = reinterpret_cast<uint64_t*>(chunk_box);  // removed bits of ranks 0 .. NMS_WIDE - 1
    static_assert(sizeof(chunk_box) >= NMS_WIDE / 8, "wide removed bits alias chunk_box");
    for (int w = threadIdx.x; w < NMS_WIDE / 64; w += NMS_THREADS) wrem[w] = 0ull;
    unsigned long long* acc = p.wacc + (int64_t)b * p.wrows;
    for (int i = threadIdx.x; i < n; i += NMS_THREADS) acc[i] = 0ull;  // ready for the next call (pair kernel done)
    const uint64_t* gm = p.wmask + (int64_t)b * p.wrows * p.wwords;
    uint64_t* smask = reinterpret_cast<uint64_t*>(s_raw);  // [compact position][NMS_FW], mslot order
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) s_nk = 0;
    __syncthreads();
    for (int R0 = 0; R0 < m; R0 += NMS_FAST) {
      const int nk_prev = s_nk;
      if (nk_prev >= p.max_det) break;
      const int L = min(NMS_FAST, m - R0);
      // (a) compaction of the chunk's live ranks: s_order[pos] = local rank (0 .. L-1)
      const int r = R0 + t;
      const bool alive = t < L && !((wrem[r >> 6] >> (r & 63)) & 1ull);
      const uint64_t bal = __ballot(alive);
      if (lane == 0) s_wsum[wave] = __popcll(bal);
      __syncthreads();
      int off = 0, cnt = 0;
#pragma unroll
      for (int w = 0; w < NMS_THREADS / 64; ++w) {
        const int v = s_wsum[w];
        off += w < wave ? v : 0;
        cnt += v;
      }
      if (alive) s_order[off + __popcll(bal & ((1ull << lane) - 1))] = t;
      __syncthreads();
      if (cnt == 0) continue;
      // (b) rows of the live ranks, words of this chunk (words left of a row's own block were not written: 0)
      const int w0 = R0 >> 6, nbw = (L + 63) >> 6;
      {
        uint64_t v[NMS_FW];
#pragma unroll
        for (int k = 0; k < NMS_FW; ++k) {
          const int e = t + k * NMS_THREADS, pos = e >> 4, w = e & (NMS_FW - 1);
          v[k] = 0ull;
          if (pos < cnt && w < nbw) {
            const int rr = R0 + s_order[pos];
            if (w0 + w >= (rr >> 6)) v[k] = gm[(int64_t)rr * p.wwords + w0 + w];
          }
        }
#pragma unroll
        for (int k = 0; k < NMS_FW; ++k) {
          const int e = t + k * NMS_THREADS;
          if ((e >> 4) < cnt) smask[mslot(e >> 4, e & (NMS_FW - 1))] = v[k];
        }
      }
      __syncthreads();
      // (c) within-block words over compact positions (columns: local ranks)
      if ((t & ~63) < cnt) {
        const int k0 = t & ~63, rl = t & 63;
        const int cr = t < cnt ? s_order[t] : 0;
        const int send = min(64, cnt - k0);
        uint64_t dw = 0;
#pragma unroll 8
        for (int q = 0; q < 64; ++q) {
          const int cq = __builtin_amdgcn_readlane(cr, q);
          const uint64_t bit = (smask[mslot(t, (cq >> 6) & (NMS_FW - 1))] >> (cq & 63)) & 1ull;
          dw |= (q > rl && q < send) ? bit << q : 0ull;
        }
        if (t < cnt) s_dw[t] = dw;
      }
      __syncthreads();
      // (d) the sweep of the pair-matrix path over the compact positions
      if (t < 64) {
        uint64_t rem = 0;  // lane w < nbw: removed flags of local ranks 64w .. 64w+63
        int nk = nk_prev;
        for (int t0 = 0; t0 < cnt && nk < p.max_det; t0 += 64) {
          const bool valid = t0 + lane < cnt;
          const int myc = valid ? s_order[t0 + lane] : 0;
          const uint64_t dw = valid ? s_dw[t0 + lane] : 0ull;
          const int wsrc = myc >> 6;
          const uint32_t rlo = __shfl((uint32_t)rem, wsrc), rhi = __shfl((uint32_t)(rem >> 32), wsrc);
          const uint64_t rw = ((uint64_t)rhi << 32) | rlo;
          const uint64_t M = __ballot(valid && !((rw >> (myc & 63)) & 1));
          const int nk0 = nk;
          uint64_t K = M;
          for (;;) {
            const uint64_t Wo = __ockl_wfred_or_u64((K >> lane) & 1 ? dw : 0ull);
            const uint64_t Kn = M & ~Wo;
            if (Kn == K) break;
            K = Kn;
          }
          for (int extra = __popcll(K) - (p.max_det - nk0); extra > 0; --extra) K &= ~(1ull << (63 - __clzll(K)));
          nk = nk0 + __popcll(K);
          if ((K >> lane) & 1) kept_slot[nk0 + __popcll(K & ((1ull << lane) - 1))] = R0 + myc;  // a rank here
          while (K) {
            int c[8];
            bool ok[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const int tt = __ffsll((long long)K) - 1;
              K &= K - 1;
              ok[q] = tt >= 0;
              c[q] = t0 + (tt & 63);  // the kept candidate's compact position = its staged row
            }
            uint64_t row[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) row[q] = smask[mslot(c[q], lane & (NMS_FW - 1))];
#pragma unroll
            for (int q = 0; q < 8; ++q) rem |= ok[q] && lane < nbw ? row[q] : 0ull;
          }
        }
        if (lane == 0) s_nk = nk;
      }
      __syncthreads();
      // (e) the new keeps' rows, right of the chunk, into the image's removed bits (8 loads in flight per thread)
      const int nk_now = s_nk, wbeg = w0 + NMS_FW;
      if (nk_now < p.max_det && wbeg < W && nk_now > nk_prev) {
        const int span = W - wbeg, tot = (nk_now - nk_prev) * span;
        for (int e0 = t; e0 < tot; e0 += 8 * NMS_THREADS) {
          uint64_t v[8];
          int wd[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int e = e0 + q * NMS_THREADS;
            const int k = e / span, w = wbeg + (e - k * span);
            wd[q] = e < tot ? w : -1;
            v[q] = e < tot ? gm[(int64_t)kept_slot[nk_prev + k] * p.wwords + w] : 0ull;
          }
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (wd[q] >= 0 && v[q]) atomicOr(reinterpret_cast<unsigned long long*>(&wrem[wd[q]]), (unsigned long long)v[q]);
        }
      }
      __syncthreads();
    }
    NMS_STAMP(3, __builtin_amdgcn_s_memrealtime());
  } else {
    bool listed = false;  // GROUPS: this group's (key, slot) list is already in s_keys / s_vals
    if constexpr (GROUPS) {
      const int64_t gi = (int64_t)b * NMS_GROUPS + grp;
      if (n > p.max_nms || n > NMS_SORT_LDS) {  // whole image in group 0
        if (grp != 0) {
          if (threadIdx.x == 0) p.gcount[gi] = 0;
          return;
        }
      } else {
        const int* cc = p.ccls + (int64_t)b * p.cap;
        if (threadIdx.x == 0) s_nk = 0;
        __syncthreads();
        for (int t = threadIdx.x; t < n; t += NMS_THREADS) {
          if (cc[t] % NMS_GROUPS == grp) {  // list order is free: the sort key orders it
            const int pos = atomicAdd(&s_nk, 1);
            s_keys[pos] = make_key(sc[t], ix[t]);
            s_vals[pos] = t;
          }
        }
        __syncthreads();
        n = s_nk;
        __syncthreads();
        listed = true;
        if (n == 0) {
          if (threadIdx.x == 0) p.gcount[gi] = 0;
          return;
        }
      }
    }
    // ---- 1. sort
    const bool in_lds = n <= NMS_SORT_LDS;
    int P = 64;
    while (P < n) P <<= 1;
    int* order;  // list position -> candidate slot
    if (in_lds && P <= NMS_THREADS) {  // the common case: one candidate per thread, sorted in registers
      const int t = threadIdx.x;
      uint64_t key = ~0ull;
      int val = -1;
      if (t < n) {
        key = listed ? s_keys[t] : make_key(sc[t], ix[t]);
        val = listed ? s_vals[t] : t;
      }
      if (n > 1) reg_bitonic(key, val, P, s_keys + 2 * NMS_THREADS, s_vals + 2 * NMS_THREADS);
      __syncthreads();
      if (t < P) {
        s_keys[t] = key;
        s_vals[t] = val;
      }
      __syncthreads();
      order = s_vals;
    } else if (in_lds) {
      for (int i = threadIdx.x; i < P; i += NMS_THREADS) {
        if (!listed || i >= n) {
          s_keys[i] = i < n ? make_key(sc[i], ix[i]) : ~0ull;
          s_vals[i] = i < n ? i : -1;
        }
      }
      __syncthreads();
      if (n > 1) block_bitonic(s_keys, s_vals, P);
      order = s_vals;
    } else {
      uint64_t* gk = p.gkeys + (int64_t)b * p.L;
      int* gv = p.gvals + (int64_t)b * p.L;
      for (int i = threadIdx.x; i < P; i += NMS_THREADS) {
        gk[i] = i < n ? make_key(sc[i], ix[i]) : ~0ull;
        gv[i] = i < n ? i : -1;
      }
      __syncthreads();
      block_bitonic(gk, gv, P);
      order = gv;
    }
    const int m = min(n, p.max_nms);
    NMS_STAMP(1, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(6, (unsigned long long)m);
    // ---- stage boxes (class-offset) of the first LDS_BOXES sorted candidates; flags
    const float* cb = p.cbox + (int64_t)b * p.cap * 4;
    const int* cc = p.ccls + (int64_t)b * p.cap;
    auto load_box = [&](int i) -> f32x4 {
      const int slot = order[i];
      const f32x4 v = *reinterpret_cast<const f32x4*>(cb + (int64_t)slot * 4);
      const float c = float(cc[slot]) * p.off_scale;  // boxes + cls * max_wh (0 if agnostic)
      return f32x4{v[0] + c, v[1] + c, v[2] + c, v[3] + c};
    };
    // s_box aliases s_keys: read every box first, then write (order[] = s_vals is separate)
    f32x4 mine[LDS_BOXES / NMS_THREADS];
#pragma unroll
    for (int r = 0; r < LDS_BOXES / NMS_THREADS; ++r) {
      const int i = threadIdx.x + r * NMS_THREADS;
      if (i < m) mine[r] = load_box(i);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LDS_BOXES / NMS_THREADS; ++r) {
      const int i = threadIdx.x + r * NMS_THREADS;
      if (i < m) s_box[i] = mine[r];
    }
    for (int i = threadIdx.x; i < m; i += NMS_THREADS) removed[i] = 0;
    if (threadIdx.x == 0) s_nk = 0;
    __syncthreads();
    auto box_at = [&](int i) -> f32x4 { return i < LDS_BOXES ? s_box[i] : load_box(i); };

    // ---- 3. chunked greedy sweep.  With the sorted list in LDS (n <= NMS_SORT_LDS) the list is
    // compacted after every chunk: the next chunk is always the 64 best boxes still alive, so the
    // number of rounds follows the boxes that survive, not the candidate count.  Above that the chunk
    // walks the sorted positions and skips suppressed ones by flag.
    const bool compact = in_lds;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;  // 16 waves
    int m_cur = m;
    NMS_STAMP(2, __builtin_amdgcn_s_memrealtime());
    int rounds = 0;
#ifdef YDBL_NMS_STAMPS
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime(), ta = 0, tb = 0, tc = 0, td = 0;
#endif
    for (int c0 = 0; c0 < m_cur;) {
      ++rounds;
      const int nk0 = s_nk;
      if (nk0 >= p.max_det) break;
      // (a) intra-chunk suppression masks: wave w tests columns c0+4w..c0+4w+3 against row c0+lane
      const int i = c0 + lane;
      const bool live = i < m_cur && !removed[i];
      f32x4 bi = f32x4{0.f, 0.f, 0.f, 0.f};
      {
        unsigned bits = 0;
        if (live) {
          bi = box_at(i);
          const float ai = (bi[2] - bi[0]) * (bi[3] - bi[1]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = c0 + 4 * wave + q;
            if (j > i && j < m_cur && !removed[j] && iou_gt(bi, ai, box_at(j), p.thr)) bits |= 1u << q;
          }
        }
        cmask[lane][wave] = (unsigned char)bits;
      }
      __syncthreads();
      NMS_TICK(ta);
      // (b) wave 0 resolves the chunk on scalar registers only (find-first-set, readlane of the kept
      // row's mask, and-not), then every lane places itself by the rank of its bit in the kept mask
      if (wave == 0) {
        uint64_t rm = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) rm |= (uint64_t)cmask[lane][w] << (4 * w);
        uint64_t M = __ballot(live), K = 0;
        int nk = nk0;
        while (M && nk < p.max_det) {
          const int t = __ffsll((long long)M) - 1;
          const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)rm, t);
          const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(rm >> 32), t);
          K |= 1ull << t;
          M &= ~((((uint64_t)hi << 32) | lo) | (1ull << t));
          ++nk;
        }
        if ((K >> lane) & 1) {
          const int rank = __popcll(K & ((1ull << lane) - 1));
          kept_slot[nk0 + rank] = order[i];
          chunk_box[rank] = bi;
          chunk_area[rank] = (bi[2] - bi[0]) * (bi[3] - bi[1]);
        }
        if (lane == 0) s_nk = nk;
      }
      __syncthreads();
      const int ck = s_nk - nk0;
      if (s_nk >= p.max_det) break;
      NMS_TICK(tb);
      // (c) suppress every later box against the chunk's kept boxes (all of which precede it).  The
      // (box, kept box) pairs are spread over the whole workgroup: G thread groups (G in 1..16) each test
      // every box against every G-th kept box, any hit sets the flag; G minimises the per-thread test
      // count ceil(R G / 1024) * ceil(ck / G) (R later boxes, ck kept boxes).
      const int R = m_cur - (c0 + 64);
      if (R > 0 && ck > 0) {
        int G = 1, best = 1 << 30;
        for (int g = 1; g <= 16; g <<= 1) {
          const int cost = ((R * g + NMS_THREADS - 1) / NMS_THREADS) * ((ck + g - 1) / g);
          if (g <= ck && cost < best) {
            best = cost;
            G = g;
          }
        }
        const int TS = NMS_THREADS / G;
        const int tg = threadIdx.x / TS, r = threadIdx.x - tg * TS;
        if (tg < G) {
          for (int j = c0 + 64 + r; j < m_cur; j += TS) {
            if (removed[j]) continue;
            const f32x4 bj = box_at(j);
            // kept boxes in batches of 8: the 8 broadcast LDS reads are in flight together and the tests
            // are independent (any hit suppresses; testing past the first hit changes nothing)
            bool sup = false;
            for (int q0 = tg; q0 < ck && !sup; q0 += 8 * G) {
              f32x4 bq[8];
              float aq[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int q = min(q0 + u * G, ck - 1);
                bq[u] = chunk_box[q];
                aq[u] = chunk_area[q];
              }
#pragma unroll
              for (int u = 0; u < 8; ++u)
                if (q0 + u * G < ck) sup |= iou_gt(bq[u], aq[u], bj, p.thr);
            }
            if (sup) removed[j] = 1;
          }
        }
      }
      __syncthreads();
      NMS_TICK(tc);
      if (!compact) {
        c0 += 64;
        continue;
      }
      // (d) compaction (c0 == 0): survivors of positions [64, m_cur) move to [0, R') in order.  Each
      // thread owns a contiguous run of E <= 8 positions held in registers (all reads before the
      // barrier, all writes after it); a wave scan + per-wave totals give the destinations.
      if (R <= 0) break;
      constexpr int EMAX = NMS_SORT_LDS / NMS_THREADS;
      const int E = (R + NMS_THREADS - 1) / NMS_THREADS;
      f32x4 kb[EMAX];
      int ks[EMAX];
      bool kv[EMAX];
      int cnt = 0;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        const int pos = 64 + threadIdx.x * E + e;
        kv[e] = e < E && pos < m_cur && !removed[pos];
        if (kv[e]) {
          kb[e] = box_at(pos);
          ks[e] = order[pos];
          ++cnt;
        }
      }
      int incl = cnt;  // inclusive scan over the wave
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      if (lane == 63) s_wsum[wave] = incl;
      __syncthreads();
      int off = incl - cnt, total = 0;
#pragma unroll
      for (int w = 0; w < NMS_THREADS / 64; ++w) {
        const int t = s_wsum[w];
        off += w < wave ? t : 0;
        total += t;
      }
      int dst = off;
#pragma unroll
      for (int e = 0; e < EMAX; ++e) {
        if (kv[e]) {
          order[dst] = ks[e];
          if (dst < LDS_BOXES) s_box[dst] = kb[e];
          removed[dst] = 0;
          ++dst;
        }
      }
      m_cur = total;
      NMS_TICK(td);
      __syncthreads();
    }
    __syncthreads();
    NMS_STAMP(3, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(5, (unsigned long long)rounds);
#ifdef YDBL_NMS_STAMPS
    NMS_STAMP(7, ta); NMS_STAMP(8, tb); NMS_STAMP(9, tc); NMS_STAMP(10, td);
#endif
  }
  const int kept = min(s_nk, p.max_det);
  if constexpr (GROUPS) {  // this group's keep list for nms_merge_kernel
    const int64_t gi = (int64_t)b * NMS_GROUPS + grp;
    for (int k = threadIdx.x; k < kept; k += NMS_THREADS) {
      const int slot = kept_rank ? p.worder[(int64_t)b * p.wrows + kept_slot[k]] : kept_slot[k];
      const int64_t o = (int64_t)b * p.cap + slot;
      p.gslot[gi * p.gk + k] = slot;
      p.gkey[gi * p.gk + k] = make_key(p.cscore[o], p.cidx[o]);
    }
    if (threadIdx.x == 0) p.gcount[gi] = kept;
    return;
  }
  for (int k = threadIdx.x; k < kept; k += NMS_THREADS) {
    const int slot = kept_rank ? p.worder[(int64_t)b * p.wrows + kept_slot[k]] : kept_slot[k];
    const int64_t o = (int64_t)b * p.cap + slot;
    f32x4 v = *reinterpret_cast<const f32x4*>(p.cbox + o * 4);
    if (p.clip_w > 0.f) {
      v[0] = fminf(fmaxf(v[0], 0.f), p.clip_w);
      v[2] = fminf(fmaxf(v[2], 0.f), p.clip_w);
    }
    if (p.clip_h > 0.f) {
      v[1] = fminf(fmaxf(v[1], 0.f), p.clip_h);
      v[3] = fminf(fmaxf(v[3], 0.f), p.clip_h);
    }
    float* dst = p.out + (int64_t)b * p.ostride + (int64_t)k * 6;
    dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
    dst[4] = p.cscore[o];
    dst[5] = float(p.ccls[o]);
  }
  // rows kept..max_det of the fixed-shape output are zeroed (the all-gather ships whole buffers)
  float* rest = p.out + (int64_t)b * p.ostride + (int64_t)kept * 6;
  for (int k = threadIdx.x; k < (p.max_det - kept) * 6; k += NMS_THREADS) rest[k] = 0.f;
  if (threadIdx.x == 0) p.out_count[(int64_t)b * p.cstride] = kept;
}

// The groups' keep lists of one image, each in (score, index) order, merged into the first max_det rows:
// an entry's final row is its position in its own list plus the number of entries of every other list
// with a smaller key (keys are unique: they carry the candidate's original index), found by binary
// search over the lists staged in LDS.  Entries ranked past max_det are dropped, the rest of the
// fixed-shape output is zeroed.
constexpr int NMS_MERGE_LDS = 8192;
__global__ __launch_bounds__(NMS_THREADS) void nms_merge_kernel(NmsArgs p) {
  __shared__ uint64_t s_key[NMS_MERGE_LDS];
  __shared__ int s_cnt[NMS_GROUPS], s_off[NMS_GROUPS + 1];
  const int b = blockIdx.x;
  const int64_t g0 = (int64_t)b * NMS_GROUPS;
  if (threadIdx.x == 0) {
    int o = 0;
    for (int g = 0; g < NMS_GROUPS; ++g) {
      s_cnt[g] = p.gcount[g0 + g];
      s_off[g] = o;
      o += s_cnt[g];
    }
    s_off[NMS_GROUPS] = o;
  }
  __syncthreads();
  const int E = s_off[NMS_GROUPS];
  const bool in_lds = E <= NMS_MERGE_LDS;
  if (in_lds) {
    for (int g = 0; g < NMS_GROUPS; ++g)
      for (int j = threadIdx.x; j < s_cnt[g]; j += NMS_THREADS) s_key[s_off[g] + j] = p.gkey[(g0 + g) * p.gk + j];
    __syncthreads();
  }
  auto key_at = [&](int g, int j) -> uint64_t {
    return in_lds ? s_key[s_off[g] + j] : p.gkey[(g0 + g) * p.gk + j];
  };
  for (int e = threadIdx.x; e < E; e += NMS_THREADS) {
    int g = 0;
    while (e >= s_off[g + 1]) ++g;
    const int j = e - s_off[g];
    const uint64_t key = key_at(g, j);
    int rank = j;
    for (int h = 0; h < NMS_GROUPS; ++h) {
      if (h == g) continue;
      int lo = 0, hi = s_cnt[h];  // number of keys of list h below `key`
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (key_at(h, mid) < key) lo = mid + 1;
        else hi = mid;
      }
      rank += lo;
    }
    if (rank >= p.max_det) continue;
    const int slot = p.gslot[(g0 + g) * p.gk + j];
    const int64_t o = (int64_t)b * p.cap + slot;
    f32x4 v = *reinterpret_cast<const f32x4*>(p.cbox + o * 4);
    if (p.clip_w > 0.f) {
      v[0] = fminf(fmaxf(v[0], 0.f), p.clip_w);
      v[2] = fminf(fmaxf(v[2], 0.f), p.clip_w);
    }
    if (p.clip_h > 0.f) {
      v[1] = fminf(fmaxf(v[1], 0.f), p.clip_h);
      v[3] = fminf(fmaxf(v[3], 0.f), p.clip_h);
    }
    float* dst = p.out + (int64_t)b * p.ostride + (int64_t)rank * 6;
    dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
    dst[4] = p.cscore[o];
    dst[5] = float(p.ccls[o]);
  }
  const int kept = min(E, p.max_det);
  float* rest = p.out + (int64_t)b * p.ostride + (int64_t)kept * 6;
  for (int k = threadIdx.x; k < (p.max_det - kept) * 6; k += NMS_THREADS) rest[k] = 0.f;
  if (threadIdx.x == 0) p.out_count[(int64_t)b * p.cstride] = kept;
}

// Zeroes the per-image candidate counters ahead of the decode's atomics.  A kernel, not
// hipMemsetAsync: a memset captured into a hipGraph was observed (ROCm 7.x) NOT to be ordered before
// the following kernel on some replays -- the counters then carried the previous replay's totals and
// NMS saw stale candidates (tests/test_gpu_model.py::test_split_session_equals_separate_sessions).
__global__ void zero_counts_kernel(int* c, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) c[i] = 0;
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
  zero_counts_kernel<<<1, 256, 0, s>>>(d->cand_count, B);
  decode_kernel<T><<<dim3((unsigned)cdiv((int64_t)A * 4, 256), B), 256, 0, s>>>(a);  // a quad per anchor
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
  zero_counts_kernel<<<1, 256, 0, s>>>(d->cand_count, d->n);
  pred_cand_kernel<<<dim3((unsigned)cdiv(d->A, 256), d->n), 256, 0, s>>>(*d);
  return check_launch("ydbl_pred_candidates");
}

// [global sort keys n*L x 8 B][sort slots n*L x 4 B][group keys n*G*gk x 8 B][group slots x 4 B][counts n*G x 4 B]
// [pad to 8 B][pair-matrix rows n*R*NMS_FW x 8 B][partial ranks n*NMS_FW*R x 4 B]
static int64_t nms_sort_len(int32_t cap) { return cap <= NMS_SORT_LDS ? 0 : next_pow2(cap); }
static int32_t nms_group_len(int32_t cap) { return cap < NMS_MAX_DET ? cap : NMS_MAX_DET; }
// rows per image of the pair-matrix workspace: candidates up to NMS_FAST, in whole 64-row blocks
static int32_t nms_fast_rows(int32_t cap) { return (std::min(cap, NMS_FAST) + 63) / 64 * 64; }
// rows per image of the wide path (0: cap <= NMS_FAST, no image can be wide)
static int32_t nms_wide_rows(int32_t cap) { return cap <= NMS_FAST ? 0 : (std::min(cap, NMS_WIDE) + 63) / 64 * 64; }

#ifdef YDBL_NMS_STAMPS
extern "C" int ydbl_nms_debug_stamps(unsigned long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nms_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t ydbl_nms_workspace(int32_t n, int32_t cap, int32_t max_nms) {
  (void)max_nms;
  if (n < 1 || cap < 1) return 16;
  const int64_t L = nms_sort_len(cap), gk = nms_group_len(cap), R = nms_fast_rows(cap), RW = nms_wide_rows(cap);
  // + pair-matrix rows (u64 x NMS_FW) and partial ranks (int x NMS_FW) per candidate row, 8-byte aligned
  // + wide rows: rank accumulator (u64), order (int), IoU row (RW / 64 u64) per row
  return (int64_t)n * L * 12 + (int64_t)n * NMS_GROUPS * (gk * 12 + 4) + 8 + (int64_t)n * R * NMS_FW * 12 + 16 +
         (int64_t)n * RW * (12 + RW / 8) + 16;
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
  if (d->out_stride < 0 || (d->out_stride && d->out_stride < (int64_t)d->max_det * 6) || d->count_stride < 0)
    return fail(YDBL_EINVAL, "nms: out_stride must be 0 or >= max_det * 6, count_stride >= 0");
  hipStream_t s = as_stream(stream);
  NmsArgs a;
  a.cbox = d->cand_box; a.cscore = d->cand_score; a.ccls = d->cand_cls; a.cidx = d->cand_idx;
  a.ccount = d->cand_count;
  a.L = (int)nms_sort_len(d->cap);
  a.gkeys = reinterpret_cast<uint64_t*>(d->workspace);
  a.gvals = reinterpret_cast<int*>(a.gkeys + (int64_t)d->n * a.L);
  a.gk = nms_group_len(d->cap);
  a.gkey = reinterpret_cast<uint64_t*>(a.gvals + (int64_t)d->n * a.L + ((int64_t)d->n * a.L & 1));  // 8-B aligned
  a.gslot = reinterpret_cast<int*>(a.gkey + (int64_t)d->n * NMS_GROUPS * a.gk);
  a.gcount = a.gslot + (int64_t)d->n * NMS_GROUPS * a.gk;
  a.cap = d->cap;
  a.thr = d->iou_thres; a.max_det = d->max_det; a.max_nms = d->max_nms;
  a.off_scale = d->agnostic ? 0.f : d->max_wh;
  a.clip_w = d->clip_w; a.clip_h = d->clip_h;
  a.out = d->out; a.out_count = d->out_count;
  a.ostride = d->out_stride ? d->out_stride : (int64_t)d->max_det * 6;
  a.cstride = d->count_stride ? d->count_stride : 1;
  a.frows = nms_fast_rows(d->cap);
  a.fmask = reinterpret_cast<uint64_t*>(a.gcount + (int64_t)d->n * NMS_GROUPS + ((int64_t)d->n * NMS_GROUPS & 1));
  a.frank = reinterpret_cast<int*>(a.fmask + (int64_t)d->n * a.frows * NMS_FW);
  a.wrows = nms_wide_rows(d->cap);
  a.wwords = a.wrows / 64;
  {
    const int64_t fr = (int64_t)d->n * NMS_FW * a.frows;  // ints of frank, then 8-byte alignment
    a.wacc = reinterpret_cast<unsigned long long*>(a.frank + fr + (fr & 1));
    a.wmask = reinterpret_cast<uint64_t*>(a.wacc + (int64_t)d->n * a.wrows);
    a.worder = reinterpret_cast<int*>(a.wmask + (int64_t)d->n * a.wrows * a.wwords);
  }
  const char* we = getenv("YDBL_NMS_WIDE");  // A/B switch (read per launch: tests): 0 = no wide pair-matrix path
  if (we && *we == '0') a.wrows = 0;
  const char* fe = getenv("YDBL_NMS_FAST");  // A/B switch (read per launch: tests): 0 = sort + chunked sweep only
  a.fast = !(fe && *fe == '0') && d->n <= NMS_PAIR_MAXB;
  if (a.fast) nms_pair_kernel<<<NMS_PAIR_WGS, 256, 0, s>>>(a, d->n);
  if (a.fast && a.wrows > 0) nms_wide_mask_kernel<<<NMS_PAIR_WGS, 256, 0, s>>>(a, d->n);
  // class-split sweep + merge (non-agnostic); the one-workgroup-per-image form for agnostic NMS or on request
  const char* ev = getenv("YDBL_NMS_GROUPS");  // A/B switch (read per launch: tests): 0 = one workgroup per image
  if (d->agnostic || d->per_image || (ev && *ev == '0')) {
    nms_kernel<false><<<d->n, NMS_THREADS, 0, s>>>(a);
  } else {
    nms_kernel<true><<<(unsigned)((int64_t)d->n * NMS_GROUPS), NMS_THREADS, 0, s>>>(a);
    nms_merge_kernel<<<d->n, NMS_THREADS, 0, s>>>(a);
  }
  return check_launch("ydbl_nms");
}
