// Read-bandwidth probe: what one CU can pull through vector loads when the data is an L2 hit, a MALL hit or
// an HBM miss, at the occupancy and loads-in-flight of the halo conv kernel (256-thread workgroups, 2 per CU,
// 8 x 16-byte loads per thread per round) and at higher ones.  Standalone diagnostic (not part of libydbl).
//   hipcc --offload-arch=gfx950 -O3 scripts/l2_probe.hip -o build_dbg/l2_probe && build_dbg/l2_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

using f4 = float __attribute__((ext_vector_type(4)));

template <int INFLIGHT>
__global__ __launch_bounds__(256) void probe(const f4* __restrict__ buf, size_t nvec, int rounds, f4* out) {
  // each workgroup walks its own window of the buffer (windows wrap): rounds x INFLIGHT loads per thread,
  // all INFLIGHT issued before any is consumed
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  size_t base = ((size_t)blockIdx.x * 256 * INFLIGHT * 7) % nvec;
  for (int r = 0; r < rounds; ++r) {
    f4 v[INFLIGHT];
#pragma unroll
    for (int i = 0; i < INFLIGHT; ++i) v[i] = buf[(base + (size_t)i * 256 + threadIdx.x) % nvec];
#pragma unroll
    for (int i = 0; i < INFLIGHT; ++i) acc += v[i];
    base = (base + 256 * INFLIGHT) % nvec;
  }
  if (acc.x == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int INFLIGHT>
static void run(const f4* buf, size_t bytes, int wgs_per_cu, f4* out, const char* what) {
  const int cus = 256, rounds = 64;
  const size_t nvec = bytes / 16;
  const int grid = cus * wgs_per_cu;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<INFLIGHT><<<grid, 256>>>(buf, nvec, rounds, out);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int it = 0; it < 5; ++it) {
    hipEventRecord(a);
    probe<INFLIGHT><<<grid, 256>>>(buf, nvec, rounds, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  const double moved = (double)grid * 256 * rounds * INFLIGHT * 16;
  const double gbs = moved / (best * 1e-3) / 1e9;
  printf("%-5s %8.1f MB window, %d WG/CU, %2d x 16B in flight/thread: %8.1f GB/s  = %5.1f B/clk/CU @2.1GHz (%.1f us)\n",
         what, bytes / 1e6, wgs_per_cu, INFLIGHT, gbs, gbs * 1e9 / 256 / 2.1e9, best * 1e3);
}

int main() {
  const size_t big = (size_t)2 << 30;
  f4 *buf, *out;
  hipMalloc(&buf, big);
  hipMemset(buf, 0, big);
  hipMalloc(&out, 256 * 16 * 256 * 16);
  const size_t sizes[3] = {(size_t)1 << 20, (size_t)96 << 20, big};
  const char* names[3] = {"L2", "MALL", "HBM"};
  for (int s = 0; s < 3; ++s) {
    for (int w : {2, 4, 8}) {
      run<8>(buf, sizes[s], w, out, names[s]);
      run<16>(buf, sizes[s], w, out, names[s]);
    }
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
