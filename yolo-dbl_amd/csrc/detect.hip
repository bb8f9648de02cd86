// Detect decode (DFL + dist2bbox + sigmoid + candidate filter) and batched class-offset NMS.
//
// decode : one thread per (image, anchor).  Writes the reference's y[b][4+nc][A] when asked
//          (U/nn/modules/head.py:143-181) and appends NMS candidates (U/utils/ops.py:234-276) with
//          a per-image atomic counter; candidate order is irrelevant because NMS sorts by
//          (score desc, original index asc), which is exactly the order torchvision's stable sort
//          gives the reference (anchor order, or torch.where's (anchor, class) row-major order).
// nms    : images with <= 8192 candidates: chip-wide ranks (= the stable sort's positions) and rank-space
//          IoU > thr bit rows, then one 1024-thread workgroup per image sweeps 64-rank blocks (the pair-matrix
//          path below); larger images: a per-image radix select of the first max_nms sort keys, sorted in
//          8192-key buckets in LDS (nms_select_sort), and a chunked greedy sweep with the suppression flags and
//          the first 4096 sorted boxes in LDS.  Both stop after max_det keeps, which is
//          the reference's keep[:max_det] because keeps are produced in score order.
#include <stdlib.h>

#include <algorithm>
#include <cmath>

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

struct IouT {  // iou_gt's fp32 thresholds (below)
  float a, hi, lo;  // a = round-down(thr); hi / lo = a (1 +- 2e-5) +- 1e-30
};

struct NmsArgs {
  const float* cbox; const float* cscore; const int* ccls; const int* cidx; const int* ccount;
  uint64_t* gkeys; int* gvals; int L;  // global sort scratch (only when cap > NMS_SORT_LDS)
  int* gslot; uint64_t* gkey; int* gcount; int gk;  // per (image, class group) keep lists, gk entries each
  int cap;
  int fast;  // pair-matrix path (n <= NMS_WIDE): per image wrows rows of rank accumulators (zero between calls:
  // the sweep clears what nms_pair_kernel added), rank -> slot order, and the rank-space IoU rows (wwords words
  // each; only the words at and right of a row's own 64-rank block are written)
  unsigned long long* wacc; int* worder; uint64_t* wmask; int wrows; int wwords;
  double thr; IouT th; int max_det, max_nms; float off_scale;
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

// Images above NMS_SORT_LDS candidates (validation settings: conf 0.001, multi-label; the reference truncates to
// argsort(descending)[:max_nms]): the first m = min(n, max_nms) sorted (key, slot) pairs into gk / gv[0, m), by one
// workgroup and without sorting the n candidates.
//   1. radix select, 8 bits per pass from the top of the 64-bit key, for the bucket targets t_j = min(8192 (j+1), m):
//      per pass, an LDS histogram of the keys that share target j's prefix; the bin where the running count reaches
//      the target's remaining rank extends the prefix.  A target is resolved when its rank is the last of its bin
//      (bound U_j = prefix with all lower bits set: exactly t_j keys are <= U_j) or after the 8th pass (the key);
//   2. one pass scatters every key <= U_{nb-1} into bucket j (the first j with key <= U_j) at gk[8192 j + ...];
//   3. each bucket (<= 8192 pairs, key range (U_{j-1}, U_j]) is sorted in LDS and written back in place, which is
//      its final position since bucket j starts at rank t_{j-1} = 8192 j.
// Keys are unique (they carry the candidate's original index), so the m pairs and their order are those of the
// reference's stable sort.  Passes read the n scores and indices (8 B per candidate); DBL-l 1280 nc80 at conf 0.001
// with 2.6 M candidates per image: 3-4 passes.  (Before: one bitonic sort of next_pow2(n) pairs in global memory,
// 62 ms per image at that size.)
constexpr int NMS_BUCKETS = NMS_MAX_FLAGS / NMS_SORT_LDS;
constexpr int SEL_U = 2;  // candidates in flight per thread and pass

__device__ void nms_select_sort(const float* sc, const int* ix, int n, int m, uint64_t* gk, int* gv, uint64_t* s_keys,
                                int* s_vals, int* hist /* LDS, NMS_BUCKETS x 256 */) {
  __shared__ uint64_t s_pre[NMS_BUCKETS], s_ub[NMS_BUCKETS];
  __shared__ int s_need[NMS_BUCKETS], s_done[NMS_BUCKETS], s_cnt[NMS_BUCKETS];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nb = (m + NMS_SORT_LDS - 1) / NMS_SORT_LDS;
  if (t < nb) {
    s_pre[t] = 0;
    s_need[t] = min(NMS_SORT_LDS * (t + 1), m);  // 1-based rank of the target within its prefix group
    s_done[t] = t == nb - 1 && m == n;             // every key: no bound needed
    s_ub[t] = ~0ull;
    s_cnt[t] = 0;
  }
  __syncthreads();
  for (int d = 0; d < 8; ++d) {
    bool open = false;
    for (int j = 0; j < nb; ++j) open |= !s_done[j];
    if (!open) break;
    const int sh = 56 - 8 * d;
    for (int i = t; i < nb * 256; i += NMS_THREADS) hist[i] = 0;
    // targets that share a prefix share the histogram: only the first of each prefix (src) counts
    uint64_t pre[NMS_BUCKETS];
    bool opn[NMS_BUCKETS], act[NMS_BUCKETS];
    int src[NMS_BUCKETS];
#pragma unroll
    for (int j = 0; j < NMS_BUCKETS; ++j) {
      pre[j] = s_pre[j];
      opn[j] = j < nb && !s_done[j];
      src[j] = j;
#pragma unroll
      for (int q = j - 1; q >= 0; --q)
        if (opn[q] && pre[q] == pre[j]) src[j] = q;
      act[j] = opn[j] && src[j] == j;
    }
    __syncthreads();
    // keys crowd into few bins in the first passes (scores share their exponent): up to two rounds of one
    // aggregated LDS add per distinct bin of the wave, then per-lane adds for the rest
    for (int i0 = t; i0 - lane < n; i0 += SEL_U * NMS_THREADS) {
      uint64_t key[SEL_U];
#pragma unroll
      for (int u = 0; u < SEL_U; ++u) {
        const int i = i0 + u * NMS_THREADS;
        key[u] = i < n ? make_key(sc[i], ix[i]) : ~0ull;
      }
#pragma unroll
      for (int u = 0; u < SEL_U; ++u) {
        const bool valid = i0 + u * NMS_THREADS < n;
        const int dig = (int)((key[u] >> sh) & 255);
        const uint64_t kp = d == 0 ? 0ull : key[u] >> (sh + 8);
#pragma unroll
        for (int j = 0; j < NMS_BUCKETS; ++j) {
          if (!act[j]) continue;  // wave-uniform
          bool pend = valid && kp == pre[j];
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const uint64_t mm = __ballot(pend);
            if (!mm) break;
            const int leader = __ffsll((long long)mm) - 1;
            const int ld = __shfl(dig, leader);
            const uint64_t same = __ballot(pend && dig == ld);
            if (lane == leader) atomicAdd(&hist[j * 256 + ld], __popcll(same));
            pend = pend && dig != ld;
          }
          if (pend) atomicAdd(&hist[j * 256 + dig], 1);
        }
      }
    }
    __syncthreads();
    if (wave < nb && opn[wave]) {  // wave j resolves target j: lane l holds bins 4l .. 4l+3
      const int j = wave;
      int hs = j;  // the first open target with this prefix counted the histogram
#pragma unroll
      for (int q = 0; q < NMS_BUCKETS; ++q) hs = q == j ? src[q] : hs;
      int c[4], sum = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) sum += (c[q] = hist[hs * 256 + 4 * lane + q]);
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const int need = s_need[j];
      int before = incl - sum;
      if (before < need && need <= incl) {  // exactly one lane
        int q = 3, cq = c[3];  // the first bin of the lane where the count reaches need (unrolled: no scratch)
#pragma unroll
        for (int u = 2; u >= 0; --u) {
          int b4 = before;
#pragma unroll
          for (int v = 0; v <= u; ++v) b4 += c[v];
          if (b4 >= need) { q = u; cq = c[u]; }
        }
#pragma unroll
        for (int v = 0; v < 3; ++v) before += v < q ? c[v] : 0;
        const uint64_t pre2 = (s_pre[j] << 8) | (uint64_t)(4 * lane + q);
        const int need2 = need - before;
        s_pre[j] = pre2;
        s_need[j] = need2;
        if (need2 == cq || d == 7) {
          s_done[j] = 1;
          s_ub[j] = sh == 0 ? pre2 : ((pre2 << sh) | ((1ull << sh) - 1));
        }
      }
    }
    __syncthreads();
  }
  // 2. scatter into the buckets
  uint64_t ub[NMS_BUCKETS];
#pragma unroll
  for (int j = 0; j < NMS_BUCKETS; ++j) ub[j] = j < nb ? s_ub[j] : 0ull;
  for (int i0 = t - lane; i0 < n; i0 += NMS_THREADS) {  // wave-uniform trip count: one LDS add per bucket and wave
    const int i = i0 + lane;
    const uint64_t key = i < n ? make_key(sc[i], ix[i]) : ~0ull;
    const bool sel = i < n && key <= ub[nb - 1];
    int j = 0;
#pragma unroll
    for (int q = 0; q < NMS_BUCKETS - 1; ++q) j += q < nb - 1 && key > ub[q];
    int pos = 0;
#pragma unroll
    for (int q = 0; q < NMS_BUCKETS; ++q) {
      const uint64_t mm = __ballot(sel && j == q);
      if (!mm) continue;
      const int leader = __ffsll((long long)mm) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(&s_cnt[q], __popcll(mm));
      base = __shfl(base, leader);
      if (sel && j == q) pos = NMS_SORT_LDS * q + base + __popcll(mm & ((1ull << lane) - 1));
    }
    if (sel) {
      gk[pos] = key;
      gv[pos] = i;
    }
  }
  __syncthreads();
  // 3. sort each bucket in LDS, in place
  for (int j = 0; j < nb; ++j) {
    const int c = s_cnt[j], base = NMS_SORT_LDS * j;
    int P = 64;
    while (P < c) P <<= 1;
    for (int i = t; i < P; i += NMS_THREADS) {
      s_keys[i] = i < c ? gk[base + i] : ~0ull;
      s_vals[i] = i < c ? gv[base + i] : -1;
    }
    __syncthreads();
    block_bitonic(s_keys, s_vals, P);
    for (int i = t; i < c; i += NMS_THREADS) gv[base + i] = s_vals[i];
    __syncthreads();
  }
}

// torchvision's decision (double)(inter / uni) > thr, for the fp32 quotient q = inter / uni, is q > a with a the
// largest float <= thr (q > a means q >= the next float, which is > thr; q <= a <= thr is not), so every compare
// here is fp32.  inter * rcp(uni) is within a few ulp of q: it decides alone unless it lies within 2e-5
// (relative) of a; only those cases pay for the IEEE division.  (IouT: set on the host by iou_thresholds.)
__device__ __forceinline__ bool iou_gt(const f32x4& a, float area_a, const f32x4& b, float area_b, const IouT& t) {
  const float xx1 = fmaxf(a[0], b[0]), yy1 = fmaxf(a[1], b[1]);
  const float xx2 = fminf(a[2], b[2]), yy2 = fminf(a[3], b[3]);
  const float ww = fmaxf(0.f, xx2 - xx1), hh = fmaxf(0.f, yy2 - yy1);
  const float inter = ww * hh;
  if (!(inter > 0.f)) return false;  // IoU 0 is never > thr (thr in [0, 1])
  const float uni = (area_a + area_b) - inter;
  const float approx = inter * __builtin_amdgcn_rcpf(uni);
  if (approx > t.hi) return true;
  if (approx < t.lo) return false;
  return inter / uni > t.a;
}

__device__ __forceinline__ bool iou_gt(const f32x4& a, float area_a, const f32x4& b, const IouT& t) {
  return iou_gt(a, area_a, b, (b[2] - b[0]) * (b[3] - b[1]), t);
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

// ---- pair-matrix path for images with n <= NMS_WIDE candidates (every predict image) -------------------
// The greedy sweep of one image is serial, but everything it consumes is not.  Two chip-wide kernels prepare it:
//   nms_pair_kernel  ranks every candidate: its count of smaller sort keys (keys are unique: they carry the
//                    original index) = its position in the reference's stable descending sort, summed over
//                    column groups in a 64-bit accumulator whose last contribution writes order[rank] = slot;
//   nms_mask_kernel  writes, in RANK space, row r word w bit s = IoU(rank r, rank 64w+s) > thr (torchvision's
//                    decision, iou_gt), every word (the blocks right of the diagonal computed, the ones left of it
//                    their mirror images; rows of ceil(m / 64) words, packed per image).
// nms_kernel then sweeps the ranks in chunks of NMS_FAST: the chunk's rows are staged in LDS, and one wave walks
// its 64-rank blocks in order, lane = rank.  A candidate is live iff no kept rank of an earlier chunk (the image's
// removed bits) and no kept rank of an earlier block of the chunk suppresses it -- its own row's words ANDed with
// the chunk's kept bits, one row read per lane whatever the number of keeps -- and it is kept iff it is live and no
// kept candidate earlier in its block suppresses it (the rows' diagonal words; the block greedy as the fixed point
// of K' = live & ~OR_{s in K} D[s], one DPP wave-OR per step).  Between chunks the new keeps' rows are ORed, over
// the later ranks, into the image's removed bits.
constexpr int NMS_FAST = 1024;        // ranks per sweep chunk (rows staged in LDS: 128 KiB)
constexpr int NMS_FW = NMS_FAST / 64;  // 64-bit words per staged row
constexpr int NMS_WIDE = 8192;         // candidates per image on this path (rank-space rows of 1 KiB)
constexpr int NMS_RANK_COLS = 256;     // columns per rank item of nms_pair_kernel (4 waves x 64)

// LDS slot of word w of staged row c: the words of a row are XOR-permuted by the row's low bits, so that
// 64 lanes reading the same word of 64 different rows (the diagonal-word reads) spread over the banks, while
// the 16 words of one row (the sweep's row reads) stay one conflict-free 128-byte line.
__device__ __forceinline__ int mslot(int c, int w) { return c * NMS_FW + (w ^ (c & (NMS_FW - 1))); }

constexpr int NMS_PAIR_MAXB = 1024;  // images per launch on the pair-matrix path (block offsets in LDS)
constexpr int NMS_PAIR_WGS = 512;    // workgroups of the persistent rank kernel
constexpr int NMS_MASK_WGS = 1024;   // and of the mask kernel (4 per CU: its blocks are short, latency-bound chains)

// s_pre[b] = work items of images < b (wave 0 of a workgroup; items(n) per image)
template <typename F>
__device__ void nms_item_prefix(const NmsArgs& p, int nimg, int* s_pre, F items) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    int run = 0;
    for (int b0 = 0; b0 < nimg; b0 += 64) {
      const int bb = b0 + lane;
      int cnt = 0;
      if (bb < nimg) {
        const int nn = min(p.ccount[bb], p.cap);
        cnt = nn >= 1 && nn <= NMS_WIDE ? items(nn) : 0;
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
}

__device__ __forceinline__ int nms_item_image(const int* s_pre, int nimg, int g) {
  int lo = 0, hi = nimg - 1;  // image b: s_pre[b] <= g < s_pre[b + 1]
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_pre[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Rank items: 64 candidates (rows) against NMS_RANK_COLS columns, wave w taking 64 of them as LDS broadcasts;
// persistent over all images' items, so a heavy image's items spread over the whole chip.
__global__ __launch_bounds__(256) void nms_pair_kernel(NmsArgs p, int nimg) {
  __shared__ int s_pre[NMS_PAIR_MAXB + 1];
  __shared__ int s_cnt[4][64];
  __shared__ uint64_t s_ck[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  nms_item_prefix(p, nimg, s_pre, [](int nn) { return ((nn + 63) >> 6) * ((nn + NMS_RANK_COLS - 1) / NMS_RANK_COLS); });
  __syncthreads();
  const int total = s_pre[nimg];
  for (int g = blockIdx.x; g < total; g += gridDim.x) {
    const int b = nms_item_image(s_pre, nimg, g);
    const int n = min(p.ccount[b], p.cap);
    const int t = g - s_pre[b];
    const float* sc = p.cscore + (int64_t)b * p.cap;
    const int* ix = p.cidx + (int64_t)b * p.cap;
    const int ng = (n + NMS_RANK_COLS - 1) / NMS_RANK_COLS;
    const int bi = t / ng, gq = t - bi * ng;
    const int i = bi * 64 + lane, ic = min(i, n - 1);
    const int c0 = gq * NMS_RANK_COLS + wave * 64;
    const int jc = min(c0 + lane, n - 1);
    const float csc = sc[jc], isc = sc[ic];
    const int cix = ix[jc], iix = ix[ic];
    s_ck[wave][lane] = make_key(csc, cix);  // this wave's 64 column keys (wave-private)
    const uint64_t ki = make_key(isc, iix);
    __builtin_amdgcn_wave_barrier();
    const int ns = max(0, min(64, n - c0));  // wave-uniform
    int below = 0;
    if (ns == 64) {
#pragma unroll 16
      for (int s = 0; s < 64; ++s) below += s_ck[wave][s] < ki;
    } else {
      for (int s = 0; s < ns; ++s) below += s_ck[wave][s] < ki;
    }
    s_cnt[wave][lane] = below;
    __syncthreads();
    if (wave == 0 && i < n) {
      const int tot = s_cnt[0][lane] + s_cnt[1][lane] + s_cnt[2][lane] + s_cnt[3][lane];
      const int64_t o = (int64_t)b * p.wrows + i;
      if (ng == 1) {
        p.worder[(int64_t)b * p.wrows + tot] = i;  // the only contribution: no accumulator
      } else {
        const unsigned long long old = atomicAdd(p.wacc + o, (1ull << 32) | (unsigned long long)(unsigned)tot);
        if ((int)(old >> 32) == ng - 1) p.worder[(int64_t)b * p.wrows + (int)(uint32_t)old + tot] = i;
      }
    }
    __syncthreads();
  }
}

// Rank-space IoU rows of the first m = min(n, max_nms) ranks: a workgroup takes one 64 x 64 block on or right of the
// diagonal at a time -- lane = row, wave w the block's columns 16w .. 16w+15 as LDS broadcasts -- and writes it AND,
// from the same decisions gathered column by column (ballot), its mirror block left of the diagonal: every row
// complete.  Persistent over all images' blocks.
__global__ __launch_bounds__(256) void nms_mask_kernel(NmsArgs p, int nimg) {
  __shared__ int s_pre[NMS_PAIR_MAXB + 1];
  __shared__ f32x4 s_cb[4][16];
  __shared__ float s_ca[4][16];
  __shared__ uint64_t s_bits[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mx = p.max_nms;
  nms_item_prefix(p, nimg, s_pre, [mx](int nn) {
    const int nbm = (min(nn, mx) + 63) >> 6;
    return nbm * (nbm + 1) / 2;
  });
  __syncthreads();
  const int total = s_pre[nimg];
  for (int g = blockIdx.x; g < total; g += gridDim.x) {
    const int b = nms_item_image(s_pre, nimg, g);
    const int n = min(p.ccount[b], p.cap);
    const int m = min(n, p.max_nms);
    const int nbm = (m + 63) >> 6;
    // upper-triangular block index t -> (bi, bj >= bi): row bi starts at bi*nbm - bi*(bi-1)/2
    const int t = g - s_pre[b];
    const float tn = 2.f * nbm + 1.f;
    int bi = (int)((tn - sqrtf(tn * tn - 8.f * (float)t)) * 0.5f);
    bi = max(0, min(bi, nbm - 1));
    while (bi > 0 && bi * nbm - bi * (bi - 1) / 2 > t) --bi;
    while (bi + 1 < nbm && (bi + 1) * nbm - (bi + 1) * bi / 2 <= t) ++bi;
    const int bj = bi + (t - (bi * nbm - bi * (bi - 1) / 2));
    const float* cb = p.cbox + (int64_t)b * p.cap * 4;
    const int* cc = p.ccls + (int64_t)b * p.cap;
    const int* ord = p.worder + (int64_t)b * p.wrows;
    const int r = bi * 64 + lane, c = bj * 64 + 16 * wave + (lane & 15);
    const int si = ord[min(r, m - 1)], sj = ord[min(c, m - 1)];
    const f32x4 vi = *reinterpret_cast<const f32x4*>(cb + (int64_t)si * 4);
    const f32x4 vj = *reinterpret_cast<const f32x4*>(cb + (int64_t)sj * 4);
    const float ci = float(cc[si]) * p.off_scale, cj = float(cc[sj]) * p.off_scale;  // boxes + cls * max_wh
    const f32x4 xi = f32x4{vi[0] + ci, vi[1] + ci, vi[2] + ci, vi[3] + ci};
    const f32x4 xj = f32x4{vj[0] + cj, vj[1] + cj, vj[2] + cj, vj[3] + cj};
    const float ai = (xi[2] - xi[0]) * (xi[3] - xi[1]);
    if (lane < 16) {
      s_cb[wave][lane] = xj;
      s_ca[wave][lane] = (xj[2] - xj[0]) * (xj[3] - xj[1]);
    }
    __builtin_amdgcn_wave_barrier();
    const int ns = min(16, m - bj * 64 - 16 * wave);  // this wave's columns (may be <= 0)
    uint64_t bits = 0, tw = 0;  // tw: lane s's transposed word = row (64 bj + 16 wave + s), word bi
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool hit = s < ns && r < m && iou_gt(xi, ai, s_cb[wave][s], s_ca[wave][s], p.th);
      bits |= hit ? 1ull << (16 * wave + s) : 0ull;
      const uint64_t col = __ballot(hit);  // the IoU is symmetric bit for bit: column s = row s of the twin block
      tw = lane == s ? col : tw;
    }
    uint64_t* gm = p.wmask + (int64_t)b * p.wrows * p.wwords;  // rows of nbm words
    if (bi < bj && lane < ns) gm[(int64_t)(bj * 64 + 16 * wave + lane) * nbm + bi] = tw;
    s_bits[wave][lane] = bits;
    __syncthreads();
    if (wave == 0 && r < m) gm[(int64_t)r * nbm + bj] = s_bits[0][lane] | s_bits[1][lane] | s_bits[2][lane] | s_bits[3][lane];
    __syncthreads();  // the columns and partial words are not overwritten before every wave is done with them
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
  // sort keys | sort slots | suppression flags, one buffer: the pair-matrix path stages a chunk's rows
  // (NMS_FAST x NMS_FW words = 128 KiB) over all three
  __shared__ __align__(16) unsigned char s_raw[NMS_SORT_LDS * 12 + NMS_MAX_FLAGS];
  static_assert(NMS_FAST * NMS_FW * 8 <= NMS_SORT_LDS * 12 + NMS_MAX_FLAGS, "pair-matrix rows fit the sort buffers");
  uint64_t* s_keys = reinterpret_cast<uint64_t*>(s_raw);
  int* s_vals = reinterpret_cast<int*>(s_raw + NMS_SORT_LDS * 8);
  unsigned char* removed = s_raw + NMS_SORT_LDS * 12;
  __shared__ int kept_slot[NMS_MAX_DET];
  __shared__ int s_wsum[NMS_THREADS / 64];
  __shared__ f32x4 chunk_box[64];
  __shared__ float chunk_area[64];
  __shared__ unsigned char cmask[64][16];
  __shared__ int s_nk;
  __shared__ uint64_t s_kb[NMS_FW];
  f32x4* s_box = reinterpret_cast<f32x4*>(s_keys);
  constexpr int LDS_BOXES = NMS_SORT_LDS * 8 / 16;

  NMS_STAMP(0, __builtin_amdgcn_s_memrealtime());
  bool kept_rank = false;  // the pair-matrix path keeps ranks in kept_slot (slot = worder[rank])
  const int b = GROUPS ? blockIdx.x / NMS_GROUPS : blockIdx.x;
  const int grp = GROUPS ? blockIdx.x % NMS_GROUPS : 0;
  int n = min(p.ccount[b], p.cap);
  const float* sc = p.cscore + (int64_t)b * p.cap;
  const int* ix = p.cidx + (int64_t)b * p.cap;
  if (p.fast && p.wrows > 0 && n <= NMS_WIDE) {
    // ---- pair-matrix path (nms_pair_kernel ranked the image, nms_mask_kernel wrote its rank-space rows)
    if constexpr (GROUPS) {
      if (grp != 0) {  // the whole image is group 0's
        if (threadIdx.x == 0) p.gcount[(int64_t)b * NMS_GROUPS + grp] = 0;
        return;
      }
    }
    kept_rank = true;
    const int m = min(n, p.max_nms);  // the reference's argsort(descending)[:max_nms]
    const int W = (m + 63) >> 6;
    uint64_t* wrem = reinterpret_cast<uint64_t*>(chunk_box);  // removed bits of ranks 0 .. NMS_WIDE - 1
    static_assert(sizeof(chunk_box) >= NMS_WIDE / 8, "removed bits alias chunk_box");
    const int t = threadIdx.x, lane = t & 63;
    for (int w = t; w < W; w += NMS_THREADS) wrem[w] = 0ull;
    if (n > NMS_RANK_COLS) {  // the rank accumulators nms_pair_kernel used, zero again for the next call
      unsigned long long* acc = p.wacc + (int64_t)b * p.wrows;
      for (int i = t; i < n; i += NMS_THREADS) acc[i] = 0ull;
    }
    const uint64_t* gm = p.wmask + (int64_t)b * p.wrows * p.wwords;
    uint64_t* smask = reinterpret_cast<uint64_t*>(s_raw);  // [local rank][NMS_FW], mslot order
    if (t == 0) s_nk = 0;
    __syncthreads();
    NMS_STAMP(1, __builtin_amdgcn_s_memrealtime());
#ifdef YDBL_NMS_STAMPS
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime(), ta = 0, tb = 0, tc = 0;
    int rounds = 0;
#endif
    for (int R0 = 0; R0 < m; R0 += NMS_FAST) {
#ifdef YDBL_NMS_STAMPS
      ++rounds;
#endif
      const int nk_prev = s_nk;
      if (nk_prev >= p.max_det) break;
      const int L = min(NMS_FAST, m - R0), nbw = (L + 63) >> 6, w0 = R0 >> 6;
      // (a) the chunk's rows, words of this chunk; rows of ranks an earlier chunk removed stay 0 (never read)
      {
        uint64_t v[NMS_FW];
#pragma unroll
        for (int k = 0; k < NMS_FW; ++k) {
          const int e = t + k * NMS_THREADS, pos = e >> 4, w = e & (NMS_FW - 1), r = R0 + pos;
          const bool ok = pos < L && w < nbw && !((wrem[min(r, m - 1) >> 6] >> (r & 63)) & 1ull);
          v[k] = ok ? gm[(int64_t)r * W + w0 + w] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < NMS_FW; ++k) {
          const int e = t + k * NMS_THREADS;
          if ((e >> 4) < L) smask[mslot(e >> 4, e & (NMS_FW - 1))] = v[k];
        }
      }
      __syncthreads();
      NMS_TICK(ta);
      // (b) one wave sweeps the chunk's 64-rank blocks in order
      if (t < 64) {
        const uint64_t xrem = lane < nbw ? wrem[w0 + lane] : ~0ull;  // lane w: removed by earlier chunks, word w
        if (lane < NMS_FW) s_kb[lane] = 0ull;  // kept bits of the chunk's words (wave-private)
        int nk = nk_prev;
        auto row_of = [&](int blk, uint64_t (&rw)[NMS_FW]) {  // the lane's own row (rank 64 blk + lane), all words
          const int c = min(blk * 64 + lane, L - 1);
#pragma unroll
          for (int w = 0; w < NMS_FW; ++w) rw[w] = smask[mslot(c, w)];
        };
        uint64_t nrow[NMS_FW];
        row_of(0, nrow);  // read one block ahead
        for (int blk = 0; blk < nbw && nk < p.max_det; ++blk) {
          uint64_t row[NMS_FW];
#pragma unroll
          for (int w = 0; w < NMS_FW; ++w) row[w] = nrow[w];
          if (blk + 1 < nbw) row_of(blk + 1, nrow);
          const int cnt = min(64, L - blk * 64);
          const uint64_t valid = cnt == 64 ? ~0ull : ((1ull << cnt) - 1);
          // removed by a kept rank of an earlier block of this chunk: the row's words AND the kept bits (s_kb of the
          // words at and right of blk are still 0)
          uint64_t sup = 0;
#pragma unroll
          for (int w = 0; w < NMS_FW; ++w) sup |= row[w] & s_kb[w];
          const uint64_t rw = ((uint64_t)__shfl((uint32_t)(xrem >> 32), blk) << 32) | __shfl((uint32_t)xrem, blk);
          const uint64_t M = valid & ~rw & ~__ballot(sup != 0);
          if (!M) continue;
          uint64_t drow = row[0];  // the own block's word (blk is wave-uniform)
#pragma unroll
          for (int w = 1; w < NMS_FW; ++w) drow = w == blk ? row[w] : drow;
          const uint64_t dw = lane < 63 ? drow & (~0ull << (lane + 1)) : 0ull;  // later ranks of the block it suppresses
          const int nk0 = nk;
          // greedy inside the block: K_r = M_r & !(any s < r in K with D[s] bit r).  Iterated from K = M as
          // K' = M & ~OR_{s in K} D[s] (one wave-wide OR per step) it reaches that unique fixed point: after t
          // steps the first t ranks are final, and steps stop as soon as K repeats -- a few for NMS clusters,
          // where a scalar walk would pay one dependent step per kept rank
          uint64_t K = M;
          for (;;) {
            const uint64_t Wo = __ockl_wfred_or_u64((K >> lane) & 1 ? dw : 0ull);
            const uint64_t Kn = M & ~Wo;
            if (Kn == K) break;
            K = Kn;
          }
          // keep[:max_det]: the greedy stops at max_det keeps, i.e. the lowest ranks of K
          for (int extra = __popcll(K) - (p.max_det - nk0); extra > 0; --extra) K &= ~(1ull << (63 - __clzll(K)));
          nk = nk0 + __popcll(K);
          if ((K >> lane) & 1) kept_slot[nk0 + __popcll(K & ((1ull << lane) - 1))] = R0 + blk * 64 + lane;  // a rank
          if (lane == 0) s_kb[blk] = K;
        }
        if (lane == 0) s_nk = nk;
      }
      __syncthreads();
      NMS_TICK(tb);
      // (c) the new keeps' rows, right of the chunk, into the image's removed bits (8 loads in flight per thread)
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
            v[q] = e < tot ? gm[(int64_t)kept_slot[nk_prev + k] * W + w] : 0ull;
          }
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (wd[q] >= 0 && v[q]) atomicOr(reinterpret_cast<unsigned long long*>(&wrem[wd[q]]), (unsigned long long)v[q]);
        }
      }
      __syncthreads();
      NMS_TICK(tc);
    }
    NMS_STAMP(2, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(3, __builtin_amdgcn_s_memrealtime());
    NMS_STAMP(6, (unsigned long long)m);
#ifdef YDBL_NMS_STAMPS
    NMS_STAMP(5, (unsigned long long)rounds);
    NMS_STAMP(7, ta); NMS_STAMP(8, tb); NMS_STAMP(9, tc);
#endif
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
    } else {  // the first min(n, max_nms) of the sorted order only (nms_select_sort)
      int* gv = p.gvals + (int64_t)b * p.L;
      nms_select_sort(sc, ix, n, min(n, p.max_nms), p.gkeys + (int64_t)b * p.L, gv, s_keys, s_vals,
                      reinterpret_cast<int*>(removed));
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
            if (j > i && j < m_cur && !removed[j] && iou_gt(bi, ai, box_at(j), p.th)) bits |= 1u << q;
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
                if (q0 + u * G < ck) sup |= iou_gt(bq[u], aq[u], bj, p.th);
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
// [pad to 8 B][rank accumulators n*R x 8 B][rank-space rows n*R x R/64 x 8 B][order n*R x 4 B]
// (bucket space of nms_select_sort: the first max_nms <= NMS_MAX_FLAGS sorted pairs, in 8192-pair buckets)
static int64_t nms_sort_len(int32_t cap) { return cap <= NMS_SORT_LDS ? 0 : std::min(next_pow2(cap), NMS_MAX_FLAGS); }
static int32_t nms_group_len(int32_t cap) { return cap < NMS_MAX_DET ? cap : NMS_MAX_DET; }
// rows per image of the pair-matrix path: candidates up to NMS_WIDE, in whole 64-row blocks
static int32_t nms_rank_rows(int32_t cap) { return (std::min(cap, NMS_WIDE) + 63) / 64 * 64; }

#ifdef YDBL_NMS_STAMPS
extern "C" int ydbl_nms_debug_stamps(unsigned long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nms_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t ydbl_nms_workspace(int32_t n, int32_t cap, int32_t max_nms) {
  (void)max_nms;
  if (n < 1 || cap < 1) return 16;
  const int64_t L = nms_sort_len(cap), gk = nms_group_len(cap), R = nms_rank_rows(cap);
  // + per pair-matrix row: rank accumulator (u64), order entry (int), rank-space IoU row (R / 64 u64)
  return (int64_t)n * L * 12 + (int64_t)n * NMS_GROUPS * (gk * 12 + 4) + 8 + (int64_t)n * R * (12 + R / 8) + 16;
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
  {  // the fp32 thresholds of iou_gt: a = the largest float <= thr
    float f = (float)d->iou_thres;
    if ((double)f > d->iou_thres) f = std::nextafter(f, -1.f);
    a.th.a = f;
    a.th.hi = f * (1.f + 2e-5f) + 1e-30f;
    a.th.lo = f * (1.f - 2e-5f) - 1e-30f;
  }
  a.off_scale = d->agnostic ? 0.f : d->max_wh;
  a.clip_w = d->clip_w; a.clip_h = d->clip_h;
  a.out = d->out; a.out_count = d->out_count;
  a.ostride = d->out_stride ? d->out_stride : (int64_t)d->max_det * 6;
  a.cstride = d->count_stride ? d->count_stride : 1;
  a.wrows = nms_rank_rows(d->cap);
  a.wwords = a.wrows / 64;
  a.wacc = reinterpret_cast<unsigned long long*>(a.gcount + (int64_t)d->n * NMS_GROUPS + ((int64_t)d->n * NMS_GROUPS & 1));
  a.wmask = reinterpret_cast<uint64_t*>(a.wacc + (int64_t)d->n * a.wrows);
  a.worder = reinterpret_cast<int*>(a.wmask + (int64_t)d->n * a.wrows * a.wwords);
  const char* fe = getenv("YDBL_NMS_FAST");  // A/B switch (read per launch: tests): 0 = sort + chunked sweep only
  a.fast = !(fe && *fe == '0') && d->n <= NMS_PAIR_MAXB;
  if (a.fast) {
    nms_pair_kernel<<<NMS_PAIR_WGS, 256, 0, s>>>(a, d->n);
    nms_mask_kernel<<<NMS_MASK_WGS, 256, 0, s>>>(a, d->n);
  }
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
