// DSConv (U/nn/modules/conv.py:91-108: SiLU(BN(pw1x1(dw_kxk(x))))) and the Detect head's DWConv -> Conv1x1
// pairs (U/nn/modules/head.py:93-101) for the small maps of the neck and head (20^2..80^2 at 640), laid
// out for latency instead of streaming.
//
// At DBL-n's bs16 sub-batch sizes a DSConv layer moves 3-7 MB: one launch of dsconv.hip's chunked kernel
// (halo of 32 channels at a time, three barriers and one global round trip per chunk, residual loaded in
// the epilogue) spends most of its 10-15 us waiting on serial global latencies.  Here a workgroup owns an
// 8x8 (or 4x8) output tile and ALL input channels:
//   1. one round trip: the whole fp16 halo (every channel), the fp32 taps, then the pointwise weights'
//      MFMA A fragments and the residual tile are issued together; the halo and taps land in LDS
//      (fp16 halo: half the LDS bytes of an fp32 staging), the A fragments and residual stay in VGPRs;
//   2. depthwise: thread = (channel quad, output row, CSEG-pixel segment) with a sliding register
//      window per input row, fp32 FMAs in the reference's (ky, kx) tap order, optional DWConv bias +
//      activation, rounded to fp16 into the MFMA B tile of all channels;
//   3. pointwise on MFMA 16x16x32 over all k-steps, + bias, activation, residual, NHWC store (and the
//      Detect class conv tail of conv_common.hpp when one wave holds all 64 output channels).
// Two barriers per launch.  Every rounding and every accumulation order is dsconv.hip's (taps and halo
// rounded to the activation dtype, k-steps in channel order), so the outputs are bit-identical to it
// (tests/test_gpu_ops.py::test_dsconv_lean_bit_identical).
#include <stdlib.h>

#include "dsc_lean.hpp"

namespace ydbl {

template <int C, int CO, int K, int S, int TH, int TW, int NT, bool TG = false, bool TAIL = false, bool PRE = false>
__global__ __launch_bounds__(NT, 1) void dsc_lean_kernel(ConvArgs<_Float16> p, const float* __restrict__ dww,
                                                          const float* __restrict__ dwb, int dw_act, int tiles_x,
                                                          int tiles_y, int ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LeanLds<C, CO, K, S, TH, TW, NT, TG, PRE, TAIL>::BYTES];
  lean_tile<C, CO, K, S, TH, TW, NT, TG, TAIL, PRE>(p, dww, dwb, dw_act, xcd_remap(blockIdx.x, ntiles), tiles_x,
                                                          tiles_y, smem);
}

template <int C, int CO, int K, int S, int TH, int TW, int NT, bool TG, bool TAIL, bool PRE = false>
static void lean_go2(const ConvArgs<_Float16>& a, const float* dww, const float* dwb, int dw_act, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, TW), tiles_y = (int)cdiv(a.Ho, TH);
  const int ntiles = a.N * tiles_y * tiles_x;
  // (measured and not kept: a persistent walk with the next tile's halo prefetched -- 2-3 workgroups per CU,
  // VGPR-bound, slower or even on every DBL-n shape but the 80^2 stride-2 one, which the chunked kernel takes)
  dsc_lean_kernel<C, CO, K, S, TH, TW, NT, TG, TAIL, PRE><<<(unsigned)ntiles, NT, 0, s>>>(a, dww, dwb, dw_act, tiles_x,
                                                                                     tiles_y, ntiles);
}

// the Detect class-conv tail (p.t3w, CO 64 only) as its own instance: its 64 tail weights per lane would
// otherwise set the register budget of every launch of the shape
template <int C, int CO, int K, int S, int TH, int TW, int NT, bool TG = false>
static void lean_go(const ConvArgs<_Float16>& a, const float* dww, const float* dwb, int dw_act, hipStream_t s) {
  if constexpr (CO == 64 && !TG) {
    if (a.t3w) return lean_go2<C, CO, K, S, TH, TW, NT, TG, true>(a, dww, dwb, dw_act, s);
  }
  if constexpr (C == 64 && CO == 64 && K == 3 && S == 1 && !TG) {
    if (a.g0w) return lean_go2<C, CO, K, S, TH, TW, NT, TG, false, true>(a, dww, dwb, dw_act, s);
  }
  lean_go2<C, CO, K, S, TH, TW, NT, TG, false>(a, dww, dwb, dw_act, s);
}

constexpr int64_t LEAN_MAX_TILES_WIDE = 160;
static int64_t lean_tiles8(const ConvArgs<_Float16>& a) { return (int64_t)a.N * cdiv(a.Ho, 8) * cdiv(a.Wo, 8); }

// Shapes built (DBL-n / DBL-s neck and head, fp16): DSBottleneck's k3 / k7 DSConvs at 64 / 128 channels, the
// stride-2 DSConvs 128 -> 128 / 256, and the Detect DWConv -> Conv1x1 pairs (c_in 64 / 128 / 256 -> 64).
bool try_dsc_lean(const ConvArgs<_Float16>& a, const float* dww, const float* dwb, int dw_act, int k, int st, int dil,
                  hipStream_t s) {
  const char* off = getenv("YDBL_DS_LEAN");  // A/B switch (read per launch: tests): 0 = dsconv.hip chunked kernel
  if ((off && *off == '0') || dil != 1 || a.y2) return false;
  if (a.xcs % 8 || a.ycs % 4 || (a.res && a.rcs % 4) || a.KPAD != a.Cin) return false;
  const int c = a.Cin, co = a.Cout;
  if (a.t3w && co != 64) return false;
  if (a.g0w && !(st == 1 && k == 3 && c == 64 && co == 64)) return false;  // the leading 1x1 (ydbl.h g0)
  // 128+ input channels only while the map is small enough that the chunked kernel cannot fill the chip
  // (<= 160 8x8 tiles: DBL-n's 20^2 maps at bs16).  On DBL-s bs64 (800 tiles at 40^2) and DBL-l 1280
  // (400 tiles at 80^2) the lean kernel's 512-thread one-round-trip tiles lost to the chunked kernel:
  // +43 / +35 ms over the bench's profile run (profiles/r03/r03rec_c{3,4}_*).  Must agree with
  // ydbl.nn.modules.C3._cv3_fusable (the trailing GEMM exists only here).
  if (c >= 128 && lean_tiles8(a) > LEAN_MAX_TILES_WIDE) return false;
  if (a.g2w) {  // DSC3k's last bottleneck k7 DSConv + its cv3 (ydbl.h: g2)
    if (st != 1 || k != 7 || c != co || a.g2xcs % 8 || a.g2ycs % 4) return false;
    if (c == 64) return lean_go<64, 64, 7, 1, 8, 8, 256, true>(a, dww, dwb, dw_act, s), true;
    if (c == 128) return lean_go<128, 128, 7, 1, 8, 8, 512, true>(a, dww, dwb, dw_act, s), true;
    return false;
  }
  if (st == 1 && k == 3) {
    if (c == 64 && co == 64) return lean_go<64, 64, 3, 1, 8, 8, 256>(a, dww, dwb, dw_act, s), true;
    if (c == 128 && co == 128) return lean_go<128, 128, 3, 1, 8, 8, 512>(a, dww, dwb, dw_act, s), true;
    // 128 -> 64 (Detect P4 pair): the chunked kernel is faster (bs16 @40^2: 12.0 vs 17.4 us, scripts/kbench.py)
    if (c == 256 && co == 64) return lean_go<256, 64, 3, 1, 8, 8, 512>(a, dww, dwb, dw_act, s), true;
  }
  if (st == 1 && k == 7) {
    if (c == 64 && co == 64) return lean_go<64, 64, 7, 1, 8, 8, 256>(a, dww, dwb, dw_act, s), true;
    if (c == 128 && co == 128) return lean_go<128, 128, 7, 1, 8, 8, 512>(a, dww, dwb, dw_act, s), true;
  }
  // stride 2: the lean tile only below 12800 output pixels (bs16 80^2 -> 40^2: chunked 17.4 vs lean 28.4 us;
  // 40^2 -> 20^2: lean 13.4 vs chunked 17.9 us per bs16 graph)
  if (st == 2 && k == 3 && c == 128 && a.P <= 12800) {
    if (co == 128) return lean_go<128, 128, 3, 2, 4, 8, 512>(a, dww, dwb, dw_act, s), true;
    if (co == 256) return lean_go<128, 256, 3, 2, 4, 8, 512>(a, dww, dwb, dw_act, s), true;
  }
  return false;
}

}  // namespace ydbl
