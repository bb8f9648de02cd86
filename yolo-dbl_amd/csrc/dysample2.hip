// DySample ('lp', scale 2, groups 4, no scope: U/nn/modules_upsample/DySample.py:20-81) in ONE launch: the offset
// 1x1 conv (0.25 and init_pos folded into its weights / bias on the host) and the bilinear border grid_sample.
//
// misc.hip's dysample_kernel reads the offsets of a separate ydbl_conv2d_nhwc launch and gathers the four
// corners of every output sample straight from L2 (a source pixel is read by ~16 sample taps; PMC: 1.47x the
// algorithmic bytes).  Here a workgroup owns a TH x TW low-resolution tile and all C channels:
//   1. the tile plus a 2-pixel halo, all channels, goes to LDS (one round trip);
//   2. the 32 offset channels of the tile's pixels on MFMA from that LDS window: two 16-channel A tiles (the x
//      and the y offsets) in the standalone conv's row order, k-steps in channel order -- the same instruction
//      sequence per output as conv.hip's, so the offsets, rounded to the activation dtype as that conv stores
//      them, are bit-identical;
//   3. every output sample of the tile (2TH x 2TW pixels x C/V channel vectors, vector fastest: whole pixels
//      per wave store) computes its source coordinates (misc.hip's formula) and blends the four corners from
//      LDS, or from global memory for the rare corner outside the staged window; optional fused FullPAD
//      second output.
// Outputs are bit-identical to the offset conv + dysample_ex pair (tests/test_gpu_ops.py).
#include <stdlib.h>

#include "conv_common.hpp"

namespace ydbl {

constexpr int DS2_HALO = 2;

template <typename T, int C, int TH, int TW>
__global__ __launch_bounds__(256) void dysample2_kernel(DView<const T> x, const T* __restrict__ woff,
                                                        const float* __restrict__ boff, DView<T> y, DView<T> y2,
                                                        DView<const T> r2, float a2, float b2, int tiles_x, int tiles_y) {
  constexpr int G = 4;
  constexpr int V = Vec<T>::N;
  constexpr int CV = C / V;                                   // vectors per pixel
  constexpr int SH = TH + 2 * DS2_HALO, SW = TW + 2 * DS2_HALO;
  constexpr int NPX = TH * TW, NPT = NPX / 16;                // 16-pixel MFMA tiles
  static_assert(NPX % 16 == 0 && NPT <= 8, "tile");
  constexpr int TPW = (NPT + 3) / 4;                          // pixel tiles per wave
  constexpr int HV = SH * SW * CV, HIT = (HV + 255) / 256;
  constexpr int NKS = C / (4 * V);                            // offset-conv k-steps
  using vec = typename Vec<T>::type;
  __shared__ vec s_x[SH * SW * CV];
  __shared__ float s_off[NPX][8 * G];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int H = x.h, W = x.w;
  const int ly0 = ty * TH - DS2_HALO, lx0 = tx * TW - DS2_HALO;  // staged window origin

  // ---- 1. window -> LDS
  {
    vec xr[HIT];
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = min(tid + it * 256, HV - 1);
      const int cv = i % CV, px = i / CV;
      const int yy = ly0 + px / SW, xx = lx0 + px % SW;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      xr[it] = vload_sel(x.at(b, ok ? yy : 0, ok ? xx : 0) + cv * V, x.p, ok);
    }
#pragma unroll
    for (int it = 0; it < HIT; ++it)
      if (tid + it * 256 < HV) s_x[tid + it * 256] = xr[it];
  }
  const int g = lane >> 4, r16 = lane & 15;
  vec af[2][NKS];  // offset weights: tile t = output channels 16t .. 16t+15 (t 0: x offsets, 1: y offsets)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int m = 0; m < NKS; ++m) af[t][m] = vload(woff + (int64_t)(16 * t + r16) * C + m * 4 * V + g * V);
  float bq[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[t][q] = boff[16 * t + 4 * g + q];
  __syncthreads();

  // ---- 2. offsets on MFMA from the window's interior
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int pt = wave + 4 * j;
    if (pt < NPT) {
      const int p = pt * 16 + r16;
      const vec* src = &s_x[((p / TW + DS2_HALO) * SW + p % TW + DS2_HALO) * CV + g];
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int m = 0; m < NKS; ++m) {
        const vec bf = src[m * 4];
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma_chunk<T>(af[t][m], bf, acc[t]);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) s_off[p][16 * t + 4 * g + q] = round_to<T>(acc[t][q] + bq[t][q]);
    }
  }
  __syncthreads();

  // ---- 3. samples: task = (output pixel, channel vector), vector fastest
  constexpr int NT = 4 * NPX * CV;
  constexpr int CVG = CV / G;  // vectors per group
  for (int t = tid; t < NT; t += 256) {
    const int cv = t % CV, op = t / CV;
    const int oy2 = 2 * ty * TH + op / (2 * TW), ox2 = 2 * tx * TW + op % (2 * TW);
    if (oy2 >= y.h || ox2 >= y.w) continue;
    const int gi = cv / CVG;
    const int h = oy2 >> 1, w = ox2 >> 1, si = oy2 & 1, sj = ox2 & 1;
    const int lp = (h - ty * TH) * TW + (w - tx * TW);
    const float offx = s_off[lp][gi * 4 + si * 2 + sj];
    const float offy = s_off[lp][4 * G + gi * 4 + si * 2 + sj];
    // misc.hip dysample_kernel's coordinate arithmetic, op for op
    const float gx = 2.0f * ((float(w) + 0.5f) + offx) / float(W) - 1.0f;
    const float gy = 2.0f * ((float(h) + 0.5f) + offy) / float(H) - 1.0f;
    float ix = ((gx + 1.0f) * float(W) - 1.0f) / 2.0f;
    float iy = ((gy + 1.0f) * float(H) - 1.0f) / 2.0f;
    ix = fminf(float(W - 1), fmaxf(ix, 0.0f));
    iy = fminf(float(H - 1), fmaxf(iy, 0.0f));
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    const int x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = (float(x1) - ix) * (float(y1) - iy);
    const float wne = (ix - float(x0)) * (float(y1) - iy);
    const float wsw = (float(x1) - ix) * (iy - float(y0));
    const float wse = (ix - float(x0)) * (iy - float(y0));
    const bool xin = x1 < W, yin = y1 < H;
    const int x1c = xin ? x1 : x0, y1c = yin ? y1 : y0;
    float vnw[V], vne[V], vsw[V], vse[V];
    const int wy0 = y0 - ly0, wy1 = y1c - ly0, wx0 = x0 - lx0, wx1 = x1c - lx0;
    if (wy0 >= 0 && wy1 < SH && wx0 >= 0 && wx1 < SW) {
      const vec a = s_x[(wy0 * SW + wx0) * CV + cv], bb = s_x[(wy0 * SW + wx1) * CV + cv];
      const vec cc = s_x[(wy1 * SW + wx0) * CV + cv], dd = s_x[(wy1 * SW + wx1) * CV + cv];
#pragma unroll
      for (int q = 0; q < V; ++q) {
        vnw[q] = float(a[q]); vne[q] = float(bb[q]); vsw[q] = float(cc[q]); vse[q] = float(dd[q]);
      }
    } else {
      load_f<V>(x.at(b, y0, x0) + cv * V, vnw);
      load_f<V>(x.at(b, y0, x1c) + cv * V, vne);
      load_f<V>(x.at(b, y1c, x0) + cv * V, vsw);
      load_f<V>(x.at(b, y1c, x1c) + cv * V, vse);
    }
    const float kne = xin ? wne : 0.f, ksw = yin ? wsw : 0.f, kse = xin && yin ? wse : 0.f;
    float o[V];
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = blend4(vnw[q], wnw, vne[q], kne, vsw[q], ksw, vse[q], kse);
    store_f<V>(y.at(b, oy2, ox2) + cv * V, o);
    if (y2.p) {  // fused FullPAD_Tunnel (block.py:1954-1956): y2 = a2 * T(y) + b2 * r2
      float rv[V], o2[V];
      load_f<V>(r2.at(b, oy2, ox2) + cv * V, rv);
#pragma unroll
      for (int q = 0; q < V; ++q) o2[q] = pad_mix(a2, round_to<T>(o[q]), b2, rv[q]);
      store_f<V>(y2.at(b, oy2, ox2) + cv * V, o2);
    }
  }
}

template <typename T>
static DView<const T> cdv(const ydbl_view& v) {
  return DView<const T>{reinterpret_cast<const T*>(v.ptr), v.n, v.h, v.w, v.c, v.cs};
}

template <typename T, int C, int TH, int TW>
static int ds2_go(const ydbl_dysample2_desc* d, hipStream_t s) {
  const int tiles_x = (int)cdiv(d->x.w, TW), tiles_y = (int)cdiv(d->x.h, TH);
  const int64_t nb = (int64_t)d->x.n * tiles_y * tiles_x;
  const bool two = d->y2.ptr != nullptr;
  dysample2_kernel<T, C, TH, TW><<<(unsigned)nb, 256, 0, s>>>(
      cdv<T>(d->x), reinterpret_cast<const T*>(d->off_w), d->off_b, dview<T>(d->y),
      two ? dview<T>(d->y2) : DView<T>{nullptr, 0, 0, 0, 0, 0}, two ? cdv<T>(d->r2) : DView<const T>{nullptr, 0, 0, 0, 0, 0},
      d->a2, d->b2, tiles_x, tiles_y);
  return check_launch("ydbl_dysample2");
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dysample2(const ydbl_dysample2_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "dysample2: null descriptor");
  if (check_view(&d->x, "dysample2.x", true) || check_view(&d->y, "dysample2.y", true)) return YDBL_EINVAL;
  if (!d->off_w || !d->off_b) return fail(YDBL_EINVAL, "dysample2: null offset weights");
  const int C = d->x.c;
  if (d->groups != 4) return fail(YDBL_EINVAL, "dysample2: groups must be 4");
  if (d->y.c != C || d->y.n != d->x.n || d->y.h != 2 * d->x.h || d->y.w != 2 * d->x.w || d->y.dtype != d->x.dtype)
    return fail(YDBL_EINVAL, "dysample2: y must be [n, 2h, 2w, c] of x's dtype");
  if (d->y2.ptr) {
    if (check_view(&d->y2, "dysample2.y2", true) || check_view(&d->r2, "dysample2.r2", true)) return YDBL_EINVAL;
    auto same = [&](const ydbl_view& v) {
      return v.n == d->y.n && v.h == d->y.h && v.w == d->y.w && v.c == d->y.c && v.dtype == d->y.dtype;
    };
    if (!same(d->y2) || !same(d->r2)) return fail(YDBL_EINVAL, "dysample2: y2/r2 must match y");
  }
  hipStream_t s = as_stream(stream);
  // 2 x 8 tiles (kbench bs16, in graph: 128@40 20.4 us as offset conv + dysample_ex -> 18.2 with 8 x 8 tiles,
  // 16.4 with 4 x 8, 15.4 with 2 x 8; 256@20 15.6 -> 13.8 / 13.8 / 11.3): the halo re-read costs less than
  // the parallelism small tiles buy.
  if (d->x.dtype == YDBL_F16) {
    if (C == 64) return ds2_go<_Float16, 64, 2, 8>(d, s);
    if (C == 128) return ds2_go<_Float16, 128, 2, 8>(d, s);
    if (C == 256) return ds2_go<_Float16, 256, 2, 8>(d, s);
  } else {
    if (C == 64) return ds2_go<float, 64, 8, 8>(d, s);
    if (C == 128) return ds2_go<float, 128, 4, 8>(d, s);
    if (C == 256) return ds2_go<float, 256, 4, 4>(d, s);
  }
  return fail(YDBL_EINVAL, "dysample2: channels must be 64, 128 or 256");
}
