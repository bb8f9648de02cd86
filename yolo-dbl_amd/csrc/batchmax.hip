// LoadTensor's /255 decision on the device (U/data/loaders.py:561-566: `if im.max() > 1.0 + eps: im = im / 255`)
// for predict() on an HBM-resident batch: the batch maximum feeds the plans' input binding (include/ydbl.h
// ydbl_input_bind), so the stem kernels scale the batch themselves and no staging copy or host sync is needed.
//
// One launch, HBM-bound (4 bytes per element, read once) with nontemporal loads: the batch is not in the 256 MiB
// Infinity Cache when predict() runs (the previous call's activations evicted it) and a plain load's allocation
// there evicts dirty activation lines first -- 63 vs 31 us cold, scripts/bmax_bench.py, profiles/r05/r05_nt_input.txt
// (warm, back-to-back, both 26 us).  Each workgroup reads a contiguous chunk in rounds of 16 16-byte loads per thread, the
// index clamped to the chunk's last vector instead of a masked tail (max is idempotent: a repeated element changes
// nothing), so a thread waits on two round trips.  Workgroup maxima meet in device-scope atomicMax on an
// order-preserving integer key (NaN mapped to the largest key: NaN propagates as in torch.max), in two levels:
// the blocks of each of 8 groups on the group's key and ticket, the last block of each group on the global pair;
// the block that takes the last global ticket writes amax / scale.  Every pair is reset by the block that took its
// last ticket, so the next call finds them initial.  A key's atomic and its ticket's are issued in order by one
// lane, the ticket only after the key's returned value is in hand, and both live at the device coherence point:
// no L2 write-back is needed.  work: BMAX_WORK_INTS ints, keys INT_MIN and tickets 0 before the first call.
#include "common.hpp"

namespace ydbl {

constexpr int BMAX_THREADS = 256;
constexpr int BMAX_ROUND = 16;  // 16-byte loads in flight per thread
constexpr int BMAX_MAX_BLOCKS = 2048;

__device__ __forceinline__ float nanmax(float m, float v) { return (v > m || v != v) ? v : m; }

__device__ __forceinline__ int order_key(float v) {
  if (v != v) return 0x7fffffff;
  const int i = __float_as_int(v);
  return i >= 0 ? i : i ^ 0x7fffffff;
}

__device__ __forceinline__ float key_value(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

// work layout: 8 per-XCD-group {key, ticket} pairs and one global pair, each int on its own 256-byte line so the
// groups' atomics run in parallel (1200 atomics on one address serialise: +17 us of a 40 us launch)
constexpr int BMAX_SLOT = 64;  // ints per 256-byte line
constexpr int BMAX_WORK_INTS = 18 * BMAX_SLOT;

__global__ __launch_bounds__(BMAX_THREADS) void batch_max_kernel(const float* __restrict__ x,
                                                                 const float* const* __restrict__ xword, int64_t n,
                                                                 int* __restrict__ work, float* __restrict__ amax,
                                                                 float* __restrict__ scale) {
  if (xword) x = *xword;  // ydbl_batch_max_bound: the batch pointer is read when the (captured) launch runs
  const int64_t nv = n / 4;  // whole float4 vectors (x is 16-byte aligned)
  const f32x4* xv = reinterpret_cast<const f32x4*>(x);
  float m = -__builtin_huge_valf();
  if (nv > 0) {  // block-contiguous: each round reads 64 KB in one piece (grid-stride rounds ran at 3.9 vs 6.6 TB/s)
    const int64_t chunk = (nv + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(lo + chunk, nv) - 1;
    for (int64_t base = lo + threadIdx.x; base <= hi; base += BMAX_ROUND * BMAX_THREADS) {
      f32x4 v[BMAX_ROUND];
#pragma unroll
      for (int u = 0; u < BMAX_ROUND; ++u) v[u] = __builtin_nontemporal_load(xv + min(base + u * BMAX_THREADS, hi));
#pragma unroll
      for (int u = 0; u < BMAX_ROUND; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = nanmax(m, v[u][e]);
    }
  }
  if (blockIdx.x == 0)  // the elements past the last whole vector
    for (int64_t t = nv * 4 + threadIdx.x; t < n; t += BMAX_THREADS) m = nanmax(m, x[t]);
  __shared__ float red[BMAX_THREADS / 64];
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) m = nanmax(m, __shfl_xor(m, k));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int w = 1; w < BMAX_THREADS / 64; ++w) m = nanmax(m, red[w]);
  // level 1: the blocks of group g = b % 8 (about one XCD's share) meet on the group's own key / ticket
  const int g = blockIdx.x & 7, ng = min((int)gridDim.x, 8);
  const int members = ((int)gridDim.x - g + 7) / 8;
  int* gkey = work + (2 * g) * BMAX_SLOT;
  int* gtick = work + (2 * g + 1) * BMAX_SLOT;
  int prev = atomicMax(gkey, order_key(m));
  asm volatile("" : "+v"(prev) : : "memory");  // the key's atomic has returned before the ticket is taken
  if (atomicAdd(gtick, 1) != members - 1) return;
  // the group's last block: its key is final; reset the group's pair, then level 2 over the groups
  int k = atomicExch(gkey, (int)0x80000000);
  atomicExch(gtick, 0);
  int* key = work + 16 * BMAX_SLOT;
  int* tick = work + 17 * BMAX_SLOT;
  prev = atomicMax(key, k);
  asm volatile("" : "+v"(prev) : : "memory");
  if (atomicAdd(tick, 1) != ng - 1) return;
  const float r = key_value(atomicExch(key, (int)0x80000000));
  atomicExch(tick, 0);
  amax[0] = r;
  if (scale) scale[0] = r > 1.0f + __FLT_EPSILON__ ? 1.0f / 255.0f : 1.0f;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int32_t ydbl_batch_max_work_ints(void) { return BMAX_WORK_INTS; }

extern "C" void ydbl_batch_max_work_init(int32_t* host_work) {  // keys INT_MIN, tickets 0 (host memory)
  for (int i = 0; i < BMAX_WORK_INTS; ++i) host_work[i] = (i / BMAX_SLOT) % 2 == 0 ? (int32_t)0x80000000 : 0;
}

extern "C" int ydbl_batch_max(const float* x, int64_t n, int32_t* work, float* amax, float* scale, void* stream) {
  if (!x || !work || !amax || n < 1) return fail(YDBL_EINVAL, "batch_max: null pointer or empty batch");
  if (reinterpret_cast<uintptr_t>(x) & 15) return fail(YDBL_EINVAL, "batch_max: x must be 16-byte aligned");
  // about two rounds of BMAX_ROUND loads per thread
  const int64_t want = cdiv(cdiv(n, 4), (int64_t)BMAX_THREADS * BMAX_ROUND * 2);
  const int blocks = (int)(want < 1 ? 1 : (want > BMAX_MAX_BLOCKS ? BMAX_MAX_BLOCKS : want));
  batch_max_kernel<<<blocks, BMAX_THREADS, 0, as_stream(stream)>>>(x, nullptr, n, reinterpret_cast<int*>(work), amax,
                                                                    scale);
  return check_launch("ydbl_batch_max");
}

extern "C" int ydbl_batch_max_bound(const float* const* xword, int64_t n, int32_t* work, float* amax, float* scale,
                                    void* stream) {
  if (!xword || !work || !amax || n < 1) return fail(YDBL_EINVAL, "batch_max_bound: null pointer or empty batch");
  const int64_t want = cdiv(cdiv(n, 4), (int64_t)BMAX_THREADS * BMAX_ROUND * 2);
  const int blocks = (int)(want < 1 ? 1 : (want > BMAX_MAX_BLOCKS ? BMAX_MAX_BLOCKS : want));
  batch_max_kernel<<<blocks, BMAX_THREADS, 0, as_stream(stream)>>>(nullptr, xword, n, reinterpret_cast<int*>(work),
                                                                    amax, scale);
  return check_launch("ydbl_batch_max_bound");
}
