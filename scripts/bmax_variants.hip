// Experiment only (scripts/bmax_bench.py --variants): read-order variants of batchmax.hip's max over a cold
// (HBM-resident, not in the Infinity Cache) batch.  Each variant writes the block maxima to part[]; the bench
// compares them with torch.amax.  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float nanmax(float m, float v) { return (v > m || v != v) ? v : m; }

constexpr int NT = 256;

__device__ __forceinline__ float block_reduce(float m) {
  __shared__ float red[NT / 64];
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) m = nanmax(m, __shfl_xor(m, k));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) m = nanmax(m, red[w]);
  return m;
}

__device__ __forceinline__ int order_key(float v) {
  if (v != v) return 0x7fffffff;
  const int i = __float_as_int(v);
  return i >= 0 ? i : i ^ 0x7fffffff;
}

// MODE 0: block-contiguous chunks (the library's order); 1: chunks staggered by `skew` vectors per block;
// 2: segment-interleaved (round r of block b reads segment r * grid + b); 3: mode 0 with nontemporal loads;
// 4: mode 3 + the library's two-level atomic merge over `groups` groups (work: 64 ints per slot, 2 * groups + 2
// slots, keys INT_MIN / tickets 0 initially); part[0] = the maximum
template <int MODE, int R>
__global__ __launch_bounds__(NT) void bmax_var(const f32x4* __restrict__ xv, int64_t nv, int64_t chunk,
                                               float* __restrict__ part, int* __restrict__ work, int groups) {
  float m = -__builtin_huge_valf();
  if constexpr (MODE == 2) {
    const int64_t seg = (int64_t)R * NT;
    const int64_t nseg = (nv + seg - 1) / seg;
    for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
      const int64_t base = s * seg + threadIdx.x;
      f32x4 v[R];
#pragma unroll
      for (int u = 0; u < R; ++u) v[u] = xv[min(base + u * NT, nv - 1)];
#pragma unroll
      for (int u = 0; u < R; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = nanmax(m, v[u][e]);
    }
  } else {
    const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(lo + chunk, nv) - 1;
    for (int64_t base = lo + threadIdx.x; base <= hi; base += R * NT) {
      f32x4 v[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const f32x4* a = xv + min(base + u * NT, hi);
        if constexpr (MODE >= 3) v[u] = __builtin_nontemporal_load(a);
        else v[u] = *a;
      }
#pragma unroll
      for (int u = 0; u < R; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = nanmax(m, v[u][e]);
    }
  }
  m = block_reduce(m);
  if constexpr (MODE == 4) {
    if (threadIdx.x != 0) return;
    const int g = blockIdx.x % groups, ng = min((int)gridDim.x, groups);
    const int members = ((int)gridDim.x - g + groups - 1) / groups;
    int* gkey = work + (2 * g) * 64;
    int* gtick = work + (2 * g + 1) * 64;
    int prev = atomicMax(gkey, order_key(m));
    asm volatile("" : "+v"(prev) : : "memory");
    if (atomicAdd(gtick, 1) != members - 1) return;
    int k = atomicExch(gkey, (int)0x80000000);
    atomicExch(gtick, 0);
    int* key = work + (2 * groups) * 64;
    int* tick = work + (2 * groups + 1) * 64;
    prev = atomicMax(key, k);
    asm volatile("" : "+v"(prev) : : "memory");
    if (atomicAdd(tick, 1) != ng - 1) return;
    const int r = atomicExch(key, (int)0x80000000);
    atomicExch(tick, 0);
    part[0] = __int_as_float(r >= 0 ? r : r ^ 0x7fffffff);
  } else if constexpr (MODE == 5) {
    // non-returning atomicMax into `groups` keys (64 ints apart), keys of the other parity (work + 8192) reset
    if (threadIdx.x == 0) atomicMax(work + (blockIdx.x % groups) * 64, order_key(m));
    if (blockIdx.x == 0 && threadIdx.x < groups) work[8192 + threadIdx.x * 64] = (int)0x80000000;
  } else {
    if (threadIdx.x == 0) part[blockIdx.x] = m;
  }
}

template <int MODE, int R>
static void launch(const float* x, int64_t n, int blocks, int64_t skew, float* part, int* work, hipStream_t s) {
  const int64_t nv = n / 4;
  int64_t chunk = (nv + blocks - 1) / blocks;
  if (MODE == 1) chunk += skew;
  const int groups = MODE >= 4 ? (int)skew : 1;
  const int64_t need = (nv + chunk - 1) / chunk;
  const int grid = MODE == 1 ? (int)need : blocks;
  bmax_var<MODE, R><<<grid, NT, 0, s>>>(reinterpret_cast<const f32x4*>(x), nv, chunk, part, work, groups);
}

extern "C" int bmax_variant(int mode, int rounds, const float* x, int64_t n, int blocks, int64_t skew, float* part,
                            int* work, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define BMAX_CASE(M)                                                     \
  if (mode == M) {                                                      \
    if (rounds == 32) launch<M, 32>(x, n, blocks, skew, part, work, s); \
    else if (rounds == 16) launch<M, 16>(x, n, blocks, skew, part, work, s); \
    else if (rounds == 8) launch<M, 8>(x, n, blocks, skew, part, work, s); \
    else launch<M, 4>(x, n, blocks, skew, part, work, s);               \
  }
  BMAX_CASE(0)
  BMAX_CASE(1)
  BMAX_CASE(2)
  BMAX_CASE(3)
  BMAX_CASE(4)
  BMAX_CASE(5)
  return (int)hipGetLastError();
}
