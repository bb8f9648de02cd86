// Stem: BasePredictor.preprocess (U/engine/predictor.py:116-134: /255 scale, .half()) fused with the
// first Conv(+folded BN)+SiLU of the backbone (U/nn/modules/conv.py:39-63), reading the NCHW fp32
// image batch directly and writing the NHWC activation: the layout change costs no extra pass.
//
// One workgroup = STEM_ROWS output rows of one image.  The input rows those need (x Cin planes,
// zero halo) are staged in LDS with coalesced row loads (NCHW rows are contiguous), rounded once
// to the activation dtype (the reference feeds the conv a .half() tensor in fp16 mode).
// The contraction K = Cin*3*3 <= 36 is one MFMA k-step of 32 (Cin <= 3) padded with zero weights:
//   A = weights [16 couts][32 k] (registers, loaded once), B = im2col [32 k][16 pixels] gathered
//   from the LDS tile, f16: one v_mfma_f32_16x16x32_f16; f32: eight exact v_mfma_f32_16x16x4_f32.
// k = c*9 + ky*3 + kx.  Lane l holds k = kidx(l>>4, j), j = 0..7, for pixel / cout l&15.
// Epilogue: + bias, SiLU, 4 consecutive couts of one pixel per lane -> NHWC.
#include "common.hpp"

namespace ydbl {

constexpr int STEM_ROWS = 2;

template <typename T>
__device__ __forceinline__ int stem_kidx(int g, int j) {
  return sizeof(T) == 2 ? 8 * g + j : 4 * j + g;
}

template <typename T, int NT, int S>
__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ x, int cin, int H, int W, float scale,
                                                   const float* __restrict__ wt, const float* __restrict__ bias,
                                                   int act, DView<T> y) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* tile = reinterpret_cast<T*>(smem);  // [rows_in][cin][wpad]
  const int wpad = W + 2;
  const int b = blockIdx.y;
  const int oy0 = blockIdx.x * STEM_ROWS;
  const int iy0 = oy0 * S - 1;
  // stage: for each of the ROWS_IN x 3 input lines, threads cover the padded row in 256-wide
  // chunks; the loads of all lines of a chunk are issued before any store (no integer division,
  // clamped addresses, zero padding by select).
  constexpr int ROWS_IN = (STEM_ROWS - 1) * S + 3;
  for (int x0 = 0; x0 < wpad; x0 += 256) {
    const int xx = x0 + threadIdx.x;
    const int ix = xx - 1;
    const bool okx = xx < wpad && ix >= 0 && ix < W;
    const int ixc = min(max(ix, 0), W - 1);
    float v[ROWS_IN][3];
#pragma unroll
    for (int r = 0; r < ROWS_IN; ++r) {
      const int iy = iy0 + r;
      const bool ok = okx && iy >= 0 && iy < H;
      const int iyc = min(max(iy, 0), H - 1);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = x[(((int64_t)b * 3 + c) * H + iyc) * W + ixc];
        v[r][c] = ok ? t * scale : 0.f;
      }
    }
    if (xx < wpad) {
#pragma unroll
      for (int r = 0; r < ROWS_IN; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) tile[(r * 3 + c) * wpad + xx] = T(v[r][c]);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int K = cin * 9;
  // per-lane im2col offsets (relative to the pixel's top-left tap) and A fragments
  int boff[8];
  float afrag[NT][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = stem_kidx<T>(g, j);
    const int kk = k < K ? k : 0;  // padded k: any finite tap, weight is zero
    const int c = kk / 9, ky = (kk % 9) / 3, kx = kk % 3;
    boff[j] = (ky * cin + c) * wpad + kx;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int co = 16 * t + r16;
      const float wv = wt[(min(co, y.c - 1) * cin + c) * 9 + ky * 3 + kx];  // unconditional, then select
      afrag[t][j] = (k < K && co < y.c) ? float(T(wv)) : 0.f;
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
    const T* base = tile + (r * S) * cin * wpad + ox * S;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 2) {
      h8 bf;
#pragma unroll
      for (int j = 0; j < 8; ++j) bf[j] = base[boff[j]];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        h8 af;
#pragma unroll
        for (int j = 0; j < 8; ++j) af[j] = (_Float16)afrag[t][j];
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, acc[t], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float bv = base[boff[j]];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(afrag[t][j], bv, acc[t], 0, 0, 0);
      }
    }
    if (ox0 + r16 >= Wo) continue;
    T* yp = y.at(b, oy, ox0 + r16);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int co = 16 * t + 4 * g;
      if (co >= y.c) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act(acc[t][q] + bv[t][q], act);
      store_f<4>(yp + co, v);
    }
  }
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_conv_stem(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, float scale,
                              const float* wt, const float* bias, int32_t k, int32_t stride, int32_t act,
                              const ydbl_view* y, void* stream) {
  if (!x || !wt || !bias) return fail(YDBL_EINVAL, "stem: null input/weights");
  if (check_view(y, "stem.y", true)) return YDBL_EINVAL;
  if (cin != 3) return fail(YDBL_EINVAL, "stem: cin must be 3 (RGB; K = 27 = one MFMA k-step)");
  if (k != 3 || (stride != 1 && stride != 2)) return fail(YDBL_EINVAL, "stem: k=3, stride 1 or 2 only");
  const int ho = (h + 2 * (k / 2) - k) / stride + 1, wo = (w + 2 * (k / 2) - k) / stride + 1;
  if (y->n != n || y->h != ho || y->w != wo) return fail(YDBL_EINVAL, "stem: output shape mismatch");
  const int cout = y->c;
  if (cout > 64 || cout % 4) return fail(YDBL_EINVAL, "stem: cout must be a multiple of 4, <= 64");
  const int es = y->dtype == YDBL_F16 ? 2 : 4;
  const size_t lds = (size_t)cin * ((STEM_ROWS - 1) * stride + k) * (w + 2) * es;
  if (lds > 160 * 1024) return fail(YDBL_EINVAL, "stem: image row too wide for the LDS tile");
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)cdiv(ho, STEM_ROWS), (unsigned)n);
  const int nt = (cout + 15) / 16;
  auto go = [&](auto kern, auto yv) {
    kern<<<grid, 256, lds, s>>>(x, cin, h, w, scale, wt, bias, act, yv);
    return check_launch("ydbl_conv_stem");
  };
#define YDBL_STEM_CASE(T, NT)                                                                      \
  if (nt == NT)                                                                                   \
    return stride == 1 ? go(stem_kernel<T, NT, 1>, dview<T>(*y)) : go(stem_kernel<T, NT, 2>, dview<T>(*y));
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
