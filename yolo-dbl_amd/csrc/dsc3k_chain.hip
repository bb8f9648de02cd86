// DSC3k (U/nn/modules/block.py:1447-1503: C3 whose m is two DSBottlenecks, block.py:1408-1444) in ONE launch:
// its four DSConvs as four stages of lean 8x8 tiles (dsc_lean.hpp), the merged cv2 | cv1 1x1 as stage 0's
// leading GEMM and cv3 as stage 3's trailing GEMM, exactly as the four ydbl_dsconv_nhwc launches of the plan
// builder compute them (bit-identical: same tile function, same arithmetic):
//   stage 0  t1 = DSConv_k3(cv1 | cv2 = 1x1(x))     (writes cv2 | cv1 and t1)
//   stage 1  y1 = DSConv_k7(t1) + cv1               (DSBottleneck 1)
//   stage 2  t2 = DSConv_k3(y1)
//   stage 3  out = cv3([DSConv_k7(t2) + y1 ; cv2])  (DSBottleneck 2 + cv3)
// At DBL-n's 40^2 x 64-channel maps each of those launches is latency-bound (7-16 us for 3-7 MB, bs16 in graph:
// the launch gap, the ramp and the two-round tail of 400 workgroups); here the stages overlap.
//
// Workgroup b runs item b: stage b / ntiles, tile b % ntiles (image-major, row-major).  A stage-s tile reads its
// 3x3 neighbourhood of stage-(s-1) tiles (k <= 7 halo <= 3 px < one 8-px tile) and the residual / second GEMM input
// of its own pixels, which stages s-1 / s-2 wrote earlier in the chain (complete once the neighbourhood is: each
// of those tiles waited for its own neighbourhood).  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility,
// Valid forms table row 1): every activation byte is stored sc1 (write-through) and loaded sc1 (L1 bypassed);
// every storing wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, then one lane stores the tile's flag sc1;
// the consumer's wave 0 polls its <= 9 producer flags with sc1 loads, then a workgroup barrier.
//
// Progress: a workgroup only waits for items with smaller indices.  With in-order dispatch per XCD the smallest
// waiting item always has its producers resident or done, so the chain drains; HIP does not promise that order,
// so every wait is bounded (HO_SPIN_LIMIT polls) -- on a timeout the workgroup records the error in the control
// block (ydbl_dsc3k_chain_status) and goes on, so a broken assumption gives wrong numbers and a loud error, never
// a hung GPU.
//
// Flags carry the launch's epoch + 1 (control word 1, read by every workgroup at its start); the workgroup that
// completes last bumps the epoch and resets the completion count, so graph replays need no reset launch.
#include "dsc_lean.hpp"

namespace ydbl {

constexpr int CH_TH = 8, CH_TW = 8;
constexpr int CH_HDR = 16;                 // control block: [0] completed items, [1] epoch, [2] error; flags at 16
constexpr int HO_SPIN_LIMIT = 1 << 20;     // flag polls (each >= ~0.1 us) before a wait is declared broken

struct ChainArgs {
  ConvArgs<_Float16> st[4];
  const float* dww[4];
  const float* dwb[4];
  int dw_act[4];
  int* ctrl;
  int tiles_x, tiles_y, ntiles;
};

// C = 64: 256 threads, the leading 1x1 in stage 0 (PRE); C = 128: 512 threads (the lean kernel's tiles), the merged
// 1x1 ran in an earlier launch.
template <int C, int NT, bool PRE>
__global__ __launch_bounds__(NT, 1) void dsc3k_chain_kernel(ChainArgs q) {
  using L0 = LeanLds<C, C, 3, 1, CH_TH, CH_TW, NT, false, PRE>;
  using L1 = LeanLds<C, C, 7, 1, CH_TH, CH_TW, NT, false, false>;
  using L3 = LeanLds<C, C, 7, 1, CH_TH, CH_TW, NT, true, false>;
  constexpr int LDS = L0::BYTES > L1::BYTES ? (L0::BYTES > L3::BYTES ? L0::BYTES : L3::BYTES)
                                            : (L1::BYTES > L3::BYTES ? L1::BYTES : L3::BYTES);
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  __shared__ int s_epoch;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x, stage = item / q.ntiles, t = item - stage * q.ntiles;
  const __amdgpu_buffer_rsrc_t rc = ho_rsrc(q.ctrl);
  if (tid == 0) s_epoch = ho_ld32(rc, 4);
  if (stage > 0 && wave == 0) {  // wait for the 3x3 neighbourhood of stage-1 tiles
    const int epoch = ho_ld32(rc, 4);
    const int tx = t % q.tiles_x, ty = (t / q.tiles_x) % q.tiles_y, img = t / (q.tiles_x * q.tiles_y);
    const int ny = ty + lane / 3 - 1, nx = tx + lane % 3 - 1;
    const bool need = lane < 9 && ny >= 0 && ny < q.tiles_y && nx >= 0 && nx < q.tiles_x;
    const unsigned off = (unsigned)(CH_HDR + (stage - 1) * q.ntiles + (img * q.tiles_y + ny) * q.tiles_x + nx) * 4;
    for (int spin = 0;; ++spin) {
      const bool ok = !need || ho_ld32(rc, off) == epoch + 1;
      if (__ballot(!ok) == 0) break;
      if (spin == HO_SPIN_LIMIT) {
        if (lane == 0) ho_st32(rc, 8, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  const int want = s_epoch + 1;
  switch (stage) {
    case 0:
      lean_tile<C, C, 3, 1, CH_TH, CH_TW, NT, false, false, PRE, true>(q.st[0], q.dww[0], q.dwb[0], q.dw_act[0], t,
                                                                            q.tiles_x, q.tiles_y, smem);
      break;
    case 1:
      lean_tile<C, C, 7, 1, CH_TH, CH_TW, NT, false, false, false, true>(q.st[1], q.dww[1], q.dwb[1], q.dw_act[1], t,
                                                                             q.tiles_x, q.tiles_y, smem);
      break;
    case 2:
      lean_tile<C, C, 3, 1, CH_TH, CH_TW, NT, false, false, false, true>(q.st[2], q.dww[2], q.dwb[2], q.dw_act[2], t,
                                                                             q.tiles_x, q.tiles_y, smem);
      break;
    default:
      lean_tile<C, C, 7, 1, CH_TH, CH_TW, NT, true, false, false, true>(q.st[3], q.dww[3], q.dwb[3], q.dw_act[3], t,
                                                                            q.tiles_x, q.tiles_y, smem);
      break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its sc1 stores
  __syncthreads();
  if (tid == 0) {
    if (stage < 3) ho_st32(rc, (unsigned)(CH_HDR + stage * q.ntiles + t) * 4, want);
    const int done = __hip_atomic_fetch_add(q.ctrl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == 4 * q.ntiles - 1) {  // the last item: ready for the next launch (graph replay)
      __hip_atomic_store(q.ctrl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q.ctrl + 1, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static bool same_view(const ydbl_view& a, const ydbl_view& b) {
  return a.ptr == b.ptr && a.n == b.n && a.h == b.h && a.w == b.w && a.c == b.c && a.cs == b.cs && a.dtype == b.dtype;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int64_t ydbl_dsc3k_chain_workspace(int32_t n, int32_t h, int32_t w) {
  if (n < 1 || h < 1 || w < 1) return -1;
  const int64_t ntiles = (int64_t)n * ((h + CH_TH - 1) / CH_TH) * ((w + CH_TW - 1) / CH_TW);
  return (CH_HDR + 3 * ntiles) * 4;
}

extern "C" int ydbl_dsc3k_chain_status(const void* ctrl, void* stream) {
  // the error word, read back on the host (synchronises the stream)
  if (!ctrl) return fail(YDBL_EINVAL, "dsc3k_chain: null control block");
  int err = 0;
  hipStream_t s = as_stream(stream);
  if (hipMemcpyAsync(&err, static_cast<const int*>(ctrl) + 2, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(YDBL_ELAUNCH, "dsc3k_chain: status read failed");
  return err ? fail(YDBL_ECAPACITY, "dsc3k_chain: a stage wait timed out (dispatch-order assumption broken)") : YDBL_OK;
}

extern "C" int ydbl_dsc3k_chain(const ydbl_dsc3k_chain_desc* d, void* stream) {
  if (!d || !d->ctrl) return fail(YDBL_EINVAL, "dsc3k_chain: null descriptor / control block");
  const ydbl_dsconv_desc* s = d->st;
  for (int i = 0; i < 4; ++i)
    if (const int rc = ds_check(&s[i])) return rc;
  const ydbl_view& x = s[0].x;
  const int c = x.c;
  const bool pre = s[0].g0_w != nullptr;  // the merged cv2 | cv1 1x1 in stage 0 (c 64) or in an earlier launch
  bool ok = x.dtype == YDBL_F16 && (c == 64 || (c == 128 && !pre));
  for (int i = 0; i < 4 && ok; ++i) {
    const ydbl_dsconv_desc& e = s[i];
    const int k = i % 2 ? 7 : 3;
    ok = e.k == k && e.stride == 1 && e.dil == 1 && e.pad == k / 2 && e.x.c == c && e.y.c == c && e.x.n == x.n &&
         e.x.h == x.h && e.x.w == x.w && e.kpad == c && !e.tail_w && (i == 0 && pre) == (e.g0_w != nullptr) &&
         (i == 3) == (e.g2_w != nullptr) && (e.res_mode == YDBL_RES_ADD) == (i % 2 == 1) &&
         (e.res_mode == YDBL_RES_NONE || e.res_mode == YDBL_RES_ADD) && e.y.cs % 4 == 0;
  }
  if (!ok)
    return fail(YDBL_EINVAL, "dsc3k_chain: stages must be fp16 DSConvs k3 (g0 at 64 channels) / k7 + residual / "
                             "k3 / k7 + residual (g2), 64 channels or 128 without g0, stride 1, one map size, no tail");
  // the chain's data flow, which the in-launch dependencies assume (dsc3k_chain.hip header): cv2 | cv1 adjacent
  // channel slices of one buffer (cv1 = stage 0's x), each stage's x the previous stage's y
  const int es = 2;
  ydbl_view cv2 = s[0].x;
  cv2.ptr = (char*)s[0].x.ptr - (int64_t)c * es;
  if (!same_view(s[1].x, s[0].y) || !same_view(s[1].r, s[0].x) || !same_view(s[2].x, s[1].y) ||
      !same_view(s[3].x, s[2].y) || !same_view(s[3].r, s[1].y) || !same_view(s[3].g2_x, cv2))
    return fail(YDBL_EINVAL, "dsc3k_chain: stage inputs must be the previous stages' outputs (x, residuals, cv2)");
  const void* outs[5] = {s[0].y.ptr, s[1].y.ptr, s[2].y.ptr, s[3].g2_y.ptr, pre ? s[0].g0_y.ptr : s[0].x.ptr};
  for (int i = 0; i < 5; ++i)
    for (int j = i + 1; j < 5; ++j)
      if (outs[i] == outs[j]) return fail(YDBL_EINVAL, "dsc3k_chain: stage outputs must not alias");
  if (s[3].g2_y.c != c || s[3].g2_x.c != c) return fail(YDBL_EINVAL, "dsc3k_chain: cv3 must map 2c -> c");
  ChainArgs q{};
  for (int i = 0; i < 4; ++i) {
    q.st[i] = ds_args_f16(&s[i]);
    q.dww[i] = s[i].dw_w;
    q.dwb[i] = s[i].dw_bias;
    q.dw_act[i] = s[i].dw_act;
  }
  q.ctrl = static_cast<int*>(d->ctrl);
  q.tiles_x = (x.w + CH_TW - 1) / CH_TW;
  q.tiles_y = (x.h + CH_TH - 1) / CH_TH;
  q.ntiles = x.n * q.tiles_x * q.tiles_y;
  if ((int64_t)q.ntiles * 4 > 0x7fffffff / 4) return fail(YDBL_EINVAL, "dsc3k_chain: too many tiles");
  if (c == 64 && pre) dsc3k_chain_kernel<64, 256, true><<<(unsigned)(4 * q.ntiles), 256, 0, as_stream(stream)>>>(q);
  else if (c == 64) dsc3k_chain_kernel<64, 256, false><<<(unsigned)(4 * q.ntiles), 256, 0, as_stream(stream)>>>(q);
  else dsc3k_chain_kernel<128, 512, false><<<(unsigned)(4 * q.ntiles), 512, 0, as_stream(stream)>>>(q);
  return check_launch("ydbl_dsc3k_chain");
}
