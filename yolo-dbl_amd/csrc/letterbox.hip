// LetterBox + BGR->RGB + HWC->CHW + uint8->fp32 /255 for a batch of camera frames, one kernel.
//
// Restates what BasePredictor.preprocess (U/engine/predictor.py:116-134) does to a list of HWC
// uint8 BGR frames: LetterBox.__call__ (U/data/augment.py:1535-1597; cv2.resize INTER_LINEAR into
// the unpadded size, cv2.copyMakeBorder with 114), then im[..., ::-1].transpose(0, 3, 1, 2),
// .float() and /255.  The resize is OpenCV 4.x's uint8 INTER_LINEAR (imgproc/src/resize.cpp,
// opencv-python >= 4.6 as the reference requires; not vendored, not installed here):
//   * exact 2x downscale in both axes switches to INTER_AREA fast: (a+b+c+d+2)>>2;
//   * otherwise fixed-point separable bilinear: per column sx = floor(fx), fx in float from the
//     double (dx+0.5)*scale-0.5, edge columns clamp with fx=0, coefficients round(w*2048) each;
//     rows sy, sy+1 clamped to the image with unclamped fy; horizontal pass exact in int32;
//     vertical pass as the 128-bit SIMD kernel VResizeLinearVec_32s8u computes it
//     (((S0>>4)*b0>>16) + ((S1>>4)*b1>>16) + 2) >> 2 for the leading row elements it covers and
//     the scalar FixedPtCast (S0*b0 + S1*b1 + 2^21) >> 22 for the row tail.
// One thread per output pixel (3 channels); a workgroup covers 256 pixels of one canvas row.
// HBM-bound: 3 B read (x ~4 source texels, cached) + 12 B written per pixel.
#include <cmath>

#include "common.hpp"

#pragma clang fp contract(off)

namespace ydbl {

constexpr int LB_THREADS = 256;

struct LbArgs {
  const uint8_t* src; const int64_t* src_off; const int32_t* meta;  // meta[i] = h, w, uh, uw, top, left
  int out_h, out_w;
  float pad;
  float* out;
};

struct AxisTap {
  int s0, s1;   // source indices of the two taps
  int a0, a1;   // fixed-point weights (sum ~2048)
};

// Column taps: resize.cpp's xofs/ialpha table entry for destination column dx.
__device__ __forceinline__ AxisTap col_tap(int dx, int dw, int sw) {
  const double inv = (double)dw / sw;
  const double scale = 1.0 / inv;
  float fx = (float)((dx + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { fx = 0.f; sx = 0; }
  if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
  AxisTap t;
  t.s0 = sx;
  t.s1 = min(sx + 1, sw - 1);
  t.a0 = (int)rintf((1.f - fx) * 2048.f);
  t.a1 = (int)rintf(fx * 2048.f);
  if (sx + 1 >= sw) t.a1 = 0;  // single-tap columns past xmax
  return t;
}

// Row taps: yofs/ibeta (no coefficient clamp), rows clipped into the image by the invoker.
__device__ __forceinline__ AxisTap row_tap(int dy, int dh, int sh) {
  const double inv = (double)dh / sh;
  const double scale = 1.0 / inv;
  float fy = (float)((dy + 0.5) * scale - 0.5);
  int sy = (int)floorf(fy);
  fy -= (float)sy;
  AxisTap t;
  t.s0 = min(max(sy, 0), sh - 1);
  t.s1 = min(max(sy + 1, 0), sh - 1);
  t.a0 = (int)rintf((1.f - fy) * 2048.f);
  t.a1 = (int)rintf(fy * 2048.f);
  return t;
}

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }

__global__ __launch_bounds__(LB_THREADS) void letterbox_kernel(LbArgs p) {
  const int img = blockIdx.z, oy = blockIdx.y;
  const int ox = blockIdx.x * LB_THREADS + threadIdx.x;
  if (ox >= p.out_w) return;
  const int* m = p.meta + img * 6;
  const int sh = m[0], sw = m[1], uh = m[2], uw = m[3], top = m[4], left = m[5];
  const int64_t plane = (int64_t)p.out_h * p.out_w;
  float* o = p.out + (int64_t)img * 3 * plane + (int64_t)oy * p.out_w + ox;
  const int dy = oy - top, dx = ox - left;
  if (dy < 0 || dy >= uh || dx < 0 || dx >= uw) {
    o[0] = p.pad; o[plane] = p.pad; o[2 * plane] = p.pad;
    return;
  }
  const uint8_t* s = p.src + p.src_off[img];
  const int64_t rs = (int64_t)sw * 3;
  int v[3];
  if (uh == sh && uw == sw) {
    const uint8_t* q = s + dy * rs + dx * 3;
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2];
  } else if (sw == 2 * uw && sh == 2 * uh) {
    const uint8_t* q0 = s + (2 * dy) * rs + 2 * dx * 3;
    const uint8_t* q1 = q0 + rs;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (q0[c] + q0[c + 3] + q1[c] + q1[c + 3] + 2) >> 2;
  } else {
    const AxisTap cx = col_tap(dx, uw, sw), ry = row_tap(dy, uh, sh);
    const uint8_t* r0 = s + ry.s0 * rs;
    const uint8_t* r1 = s + ry.s1 * rs;
    // leading elements of the uw*3-wide row done by the 16/8-lane SIMD loops, the rest scalar
    const int width = uw * 3;
    int simd_end = width >= 16 ? (width / 16) * 16 : 0;
    while (simd_end < width - 8) simd_end += 8;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int S0 = r0[cx.s0 * 3 + c] * cx.a0 + r0[cx.s1 * 3 + c] * cx.a1;
      const int S1 = r1[cx.s0 * 3 + c] * cx.a0 + r1[cx.s1 * 3 + c] * cx.a1;
      if (dx * 3 + c < simd_end) {
        const int h0 = ((S0 >> 4) * ry.a0) >> 16;
        const int h1 = ((S1 >> 4) * ry.a1) >> 16;
        v[c] = sat_u8((h0 + h1 + 2) >> 2);
      } else {
        v[c] = sat_u8((S0 * ry.a0 + S1 * ry.a1 + (1 << 21)) >> 22);
      }
    }
  }
  // BGR -> RGB planes, uint8 -> float, / 255
  o[0] = (float)v[2] / 255.0f;
  o[plane] = (float)v[1] / 255.0f;
  o[2 * plane] = (float)v[0] / 255.0f;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_letterbox(const ydbl_letterbox_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "letterbox: null descriptor");
  if (!d->src || !d->src_off || !d->meta || !d->out) return fail(YDBL_EINVAL, "letterbox: null buffer");
  if (d->n < 1 || d->out_h < 1 || d->out_w < 1) return fail(YDBL_EINVAL, "letterbox: empty batch");
  if (d->n > 65535 || d->out_h > 65535) return fail(YDBL_EINVAL, "letterbox: batch / canvas too large");
  LbArgs a;
  a.src = d->src; a.src_off = d->src_off; a.meta = d->meta;
  a.out_h = d->out_h; a.out_w = d->out_w;
  a.pad = d->pad_value / 255.0f;
  a.out = d->out;
  dim3 grid((unsigned)cdiv(d->out_w, LB_THREADS), (unsigned)d->out_h, (unsigned)d->n);
  letterbox_kernel<<<grid, LB_THREADS, 0, as_stream(stream)>>>(a);
  return check_launch("ydbl_letterbox");
}
