// Stem: BasePredictor.preprocess (U/engine/predictor.py:116-134: /255 scale, .half()) fused with the
// first Conv(+folded BN)+SiLU of the backbone (U/nn/modules/conv.py:39-63), reading the NCHW fp32
// image batch directly and writing the NHWC activation: the layout change costs no extra pass.
//
// One workgroup = STEM_ROWS output rows of one image.  The (STEM_ROWS-1)*S+3 input rows they
// need are staged in LDS as one 4-channel record per pixel, (c0, c1, c2, 0) in the activation
// dtype (8 B f16 / 16 B f32; rounded once: the reference feeds the conv a .half() tensor in fp16
// mode), from 16-byte float4 loads of the three NCHW planes when W % 4 == 0.
// K is ordered tap-major over the record, k = (ky*3 + kx)*4 + c (36 slots, c = 3 zero-weighted),
// so a lane's slice of one MFMA k-step is whole records: f16 (16x16x32): lane g holds taps
// 2g, 2g+1 of k-step m (two ds_read_b64); f32 (exact 16x16x4 x4 per 16-k step): lane g holds tap
// 4m+g (one ds_read_b128).  A = weights [16 couts][k] in registers, loaded once.
// Epilogue: + bias, SiLU, 4 consecutive couts of one pixel per lane -> NHWC.
#include "conv_common.hpp"

namespace ydbl {

constexpr int STEM_ROWS = 4;

template <typename T> struct Rec;  // one staged pixel: 4 channels of T
template <> struct Rec<_Float16> { using type = h4; };
template <> struct Rec<float> { using type = f32x4; };

template <typename T, int NT, int S, bool V4>
__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ x, int H, int W, float scale,
                                                   const float* __restrict__ wt, const float* __restrict__ bias,
                                                   int act, DView<T> y, InputBind ib) {
  x = bound_x(ib, x);
  scale = bound_scale(ib, scale);
  using rec = typename Rec<T>::type;
  constexpr bool F16 = sizeof(T) == 2;
  constexpr int KS = F16 ? 2 : 3;          // k-steps: 36 slots -> 2 x 32 (f16) / 3 x 16 (f32)
  constexpr int TPL = F16 ? 2 : 1;         // taps per lane per k-step
  constexpr int ROWS_IN = (STEM_ROWS - 1) * S + 3;
  extern __shared__ __align__(16) unsigned char smem[];
  rec* tile = reinterpret_cast<rec*>(smem);  // [ROWS_IN][W + 2]
  const int wpad = W + 2;
  const int b = blockIdx.y;
  const int oy0 = blockIdx.x * STEM_ROWS;
  const int iy0 = oy0 * S - 1;
  const int64_t plane = (int64_t)H * W;
  const float* xb = x + (int64_t)b * 3 * plane;
  auto pack = [&](float c0, float c1, float c2) {
    rec r;
    r[0] = T(round_to<T>(c0 * scale)); r[1] = T(round_to<T>(c1 * scale)); r[2] = T(round_to<T>(c2 * scale)); r[3] = T(0.f);
    return r;
  };
  if constexpr (V4) {
    // lane task = (input row, 4-pixel group): three float4 loads (one per plane) -> 4 records
    const int groups = W >> 2;
    const int total = ROWS_IN * groups;
    for (int t0 = 0; t0 < total; t0 += 4 * 256) {
      f32x4 v[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = min(t0 + u * 256 + (int)threadIdx.x, total - 1);
        const int r = t / groups, gx = t - r * groups;
        const int iy = iy0 + r;
        const int iyc = min(max(iy, 0), H - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c)  // the batch, read once: nontemporal (batchmax.hip)
          v[u][c] = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>(xb + c * plane + (int64_t)iyc * W + 4 * gx));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * 256 + threadIdx.x;
        if (t >= total) continue;
        const int r = t / groups, gx = t - r * groups;
        const int iy = iy0 + r;
        const bool ok = iy >= 0 && iy < H;
        rec* d = tile + r * wpad + 1 + 4 * gx;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          d[e] = ok ? pack(v[u][0][e], v[u][1][e], v[u][2][e]) : pack(0.f, 0.f, 0.f);
      }
    }
    for (int t = threadIdx.x; t < ROWS_IN * 2; t += 256)  // left / right zero pad columns
      tile[(t >> 1) * wpad + ((t & 1) ? W + 1 : 0)] = pack(0.f, 0.f, 0.f);
  } else {
    const int total = ROWS_IN * wpad;
    for (int t = threadIdx.x; t < total; t += 256) {
      const int r = t / wpad, xx = t - r * wpad;
      const int iy = iy0 + r, ix = xx - 1;
      const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
      const int64_t o = (int64_t)min(max(iy, 0), H - 1) * W + min(max(ix, 0), W - 1);
      const float c0 = xb[o], c1 = xb[plane + o], c2 = xb[2 * plane + o];
      tile[t] = ok ? pack(c0, c1, c2) : pack(0.f, 0.f, 0.f);
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // A fragments: k-step m, lane g, element j -> slot k = m*16*TPL*... (tap, c) = (k / 4, k % 4)
  using vec = typename Vec<T>::type;
  vec afrag[NT][KS];
  int toff[KS][TPL];  // LDS record offset of each of this lane's taps relative to the pixel's (0,0)
#pragma unroll
  for (int m = 0; m < KS; ++m) {
#pragma unroll
    for (int u = 0; u < TPL; ++u) {
      const int tap = min((m * 4 + g) * TPL + u, 8);  // taps >= 9 carry zero weights
      toff[m][u] = (tap / 3) * wpad + tap % 3;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int co = min(16 * t + r16, y.c - 1);
#pragma unroll
      for (int j = 0; j < Vec<T>::N; ++j) {
        const int tap = (m * 4 + g) * TPL + j / 4, c = j % 4;
        const bool live = tap < 9 && c < 3 && 16 * t + r16 < y.c;
        const float wv = wt[(co * 3 + min(c, 2)) * 9 + min(tap, 8)];
        afrag[t][m][j] = live ? T(wv) : T(0.f);
      }
    }
  }
  float bv[NT][4];  // bias of this lane's output channels, loaded once
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[t][q] = bias[min(16 * t + 4 * g + q, y.c - 1)];
  const int Wo = y.w;
  const int tiles_per_row = (Wo + 15) / 16;
  for (int tt = wave; tt < STEM_ROWS * tiles_per_row; tt += 4) {
    const int r = tt / tiles_per_row;
    const int ox0 = (tt - r * tiles_per_row) * 16;
    const int oy = oy0 + r;
    if (oy >= y.h) break;
    const int ox = min(ox0 + r16, Wo - 1);
    const rec* base = tile + (r * S) * wpad + ox * S;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < KS; ++m) {
      vec bf;
      if constexpr (F16) {
        const h4 lo = base[toff[m][0]], hi = base[toff[m][1]];
        bf = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      } else {
        bf = base[toff[m][0]];
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma_chunk<T>(afrag[t][m], bf, acc[t]);
    }
    if (ox0 + r16 >= Wo) continue;
    T* yp = y.at(b, oy, ox0 + r16);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int co = 16 * t + 4 * g;
      if (co >= y.c) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[t][q] + bv[t][q], act);
      store_f<4>(yp + co, v);
    }
  }
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_conv_stem(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, float scale,
                              const float* wt, const float* bias, int32_t k, int32_t stride, int32_t act,
                              const ydbl_view* y, const ydbl_input_bind* bind, void* stream) {
  if (bind && !bind->x != !bind->amax) return fail(YDBL_EINVAL, "stem: input binding with a null pointer");
  if (!x || !wt || !bias) return fail(YDBL_EINVAL, "stem: null input/weights");
  if (check_view(y, "stem.y", true)) return YDBL_EINVAL;
  if (cin != 3) return fail(YDBL_EINVAL, "stem: cin must be 3 (RGB; K = 27 = one MFMA k-step)");
  if (k != 3 || (stride != 1 && stride != 2)) return fail(YDBL_EINVAL, "stem: k=3, stride 1 or 2 only");
  const int ho = (h + 2 * (k / 2) - k) / stride + 1, wo = (w + 2 * (k / 2) - k) / stride + 1;
  if (y->n != n || y->h != ho || y->w != wo) return fail(YDBL_EINVAL, "stem: output shape mismatch");
  const int cout = y->c;
  if (cout > 64 || cout % 4) return fail(YDBL_EINVAL, "stem: cout must be a multiple of 4, <= 64");
  const int rs = y->dtype == YDBL_F16 ? 8 : 16;  // bytes per staged 4-channel pixel record
  const size_t lds = (size_t)((STEM_ROWS - 1) * stride + k) * (w + 2) * rs;
  if (lds > 160 * 1024) return fail(YDBL_EINVAL, "stem: image row too wide for the LDS tile");
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)cdiv(ho, STEM_ROWS), (unsigned)n);
  const int nt = (cout + 15) / 16;
  const bool v4 = w % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  auto go = [&](auto kern, auto yv) {
    kern<<<grid, 256, lds, s>>>(x, h, w, scale, wt, bias, act, yv, input_bind(bind));
    return check_launch("ydbl_conv_stem");
  };
#define YDBL_STEM_CASE(T, NT)                                                                        \
  if (nt == NT) {                                                                                   \
    if (v4) return stride == 1 ? go(stem_kernel<T, NT, 1, true>, dview<T>(*y)) : go(stem_kernel<T, NT, 2, true>, dview<T>(*y)); \
    return stride == 1 ? go(stem_kernel<T, NT, 1, false>, dview<T>(*y)) : go(stem_kernel<T, NT, 2, false>, dview<T>(*y)); \
  }
  if (y->dtype == YDBL_F16) {
    YDBL_STEM_CASE(_Float16, 1)
    YDBL_STEM_CASE(_Float16, 2)
    YDBL_STEM_CASE(_Float16, 3)
    YDBL_STEM_CASE(_Float16, 4)
  } else {
    YDBL_STEM_CASE(float, 1)
    YDBL_STEM_CASE(float, 2)
    YDBL_STEM_CASE(float, 3)
    YDBL_STEM_CASE(float, 4)
  }
#undef YDBL_STEM_CASE
  return fail(YDBL_EINVAL, "stem: unsupported cout");
}
