// DSBottleneck in one launch (U/nn/modules/block.py:1408-1444): y = x + cv2(cv1(x)) with
//   cv1 = DSConv(c, c, k=3): t = SiLU(pw1(dw3(x)) + b1)   (BN folded into pw1)
//   cv2 = DSConv(c, c, k=7): u = SiLU(pw2(dw7(t)) + b2)
// The intermediate t never leaves the CU.  A workgroup owns an 8x8 output tile and all C = NTN*16
// channels; it computes t on the 14x14 region the 7x7 depthwise needs (halo 3, recomputed by the
// neighbouring tiles), so it reads x on a 16x16 region.  Per 32-channel chunk (one MFMA k-step):
//   phase 1  x halo chunk -> LDS (fp32, the dsconv.hip layout) -> dw3 over the 14x14 region (fp32
//            FMAs in the reference's (ky, kx) order) -> rounded to fp16 into the B tile -> pw1 MFMA
//            into 13 16-pixel accumulator tiles spread over the 4 waves;
//   t        = SiLU(acc1 + b1) rounded to fp16, ZERO outside the image (cv2's zero padding), kept
//            in LDS as [196 px][C] fp16;
//   phase 2  t chunk -> LDS (fp32) -> dw7 over the 8x8 outputs -> fp16 B tile -> pw2 MFMA;
//   epilogue = conv.hip's (bias, SiLU, residual add of x, channel-slice store).
// Every rounding step and accumulation order is the one of the two ydbl_dsconv_nhwc launches it
// replaces, so the result is bit-identical to them (tests/test_gpu_ops.py::test_dsbottleneck_fused).
#include <stdlib.h>

#include "conv_common.hpp"

namespace ydbl {

namespace {
constexpr int TH = 8, TW = 8;            // output tile
constexpr int RT = 3;                    // dw7 halo
constexpr int TTH = TH + 2 * RT, TTW = TW + 2 * RT;  // t region 14 x 14
constexpr int NTP = TTH * TTW;           // 196 t pixels
constexpr int NT1 = (NTP + 15) / 16;     // 13 MFMA pixel tiles of t
constexpr int TMW1 = (NT1 + 3) / 4;      // per wave
constexpr int XH = TTH + 2, XW = TTW + 2;  // x region 16 x 16 (dw3 halo 1)
constexpr int XWP = XW | 1;              // odd row pitch (bank spread, as dsconv.hip)
constexpr int NQ = 8;                    // fp32 quads of a 32-channel chunk
constexpr int SB_VEC = NT1 * 16 * 4;     // B-tile slots (16-byte, 8 fp16 channels)
}  // namespace

__device__ __forceinline__ int bslot(int row, int kv) { return row * 4 + (kv ^ (((row >> 2) & 1) << 1)); }

template <int NTN>
__global__ __launch_bounds__(256, 2) void dsbneck_kernel(ConvArgs<_Float16> p, const float* __restrict__ dw1,
                                                         const _Float16* __restrict__ pw1, const float* __restrict__ b1,
                                                         const float* __restrict__ dw2, int tiles_x, int tiles_y) {
  constexpr int C = NTN * 16;
  constexpr int NCH = C / 32;
  __shared__ f32x4 s_x[XH * XWP * NQ];  // fp32 window of the current chunk (x in phase 1, t in phase 2)
  __shared__ f32x4 s_w[49 * NQ];        // depthwise taps of the current chunk (9 or 49)
  __shared__ h8 s_b[SB_VEC];            // pointwise B tile (fp16)
  __shared__ h4 s_t[NTP * C / 4];       // t, [px][C] fp16

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = p.N * tiles_y * tiles_x;
  int bid = xcd_remap(blockIdx.x, ntiles);
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int xy0 = oy0 - RT - 1, xx0 = ox0 - RT - 1;  // x region origin
  const int ty0 = oy0 - RT, tx0 = ox0 - RT;          // t region origin

  // ---------------------------------------------------------------- phase 1: t = cv1(x) on 14x14
  constexpr int XV = XH * XW * 4;  // 16-byte x vectors per chunk (1024)
  constexpr int XIT = XV / 256;
  h8 xr[XIT];
  f32x4 wr;
  auto load_x = [&](int c0) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      const int cv = i & 3, px = i >> 2;
      const int hy = px / XW, hx = px - hy * XW;
      const int iy = xy0 + hy, ix = xx0 + hx;
      const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      xr[it] = vload_sel(p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + c0 + cv * 8, p.x, ok);
    }
    if (tid < 9 * NQ) {  // taps rounded to fp16 (the reference's .half() weights), as dsconv.hip
      const f32x4 w = *reinterpret_cast<const f32x4*>(dw1 + (tid / NQ) * C + c0 + (tid % NQ) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) wr[e] = float(_Float16(w[e]));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int i = tid + it * 256;
      const int cv = i & 3, px = i >> 2;
      const int hy = px / XW, hx = px - hy * XW;
      f32x4* d = &s_x[(hy * XWP + hx) * NQ + cv * 2];
      d[0] = f32x4{float(xr[it][0]), float(xr[it][1]), float(xr[it][2]), float(xr[it][3])};
      d[1] = f32x4{float(xr[it][4]), float(xr[it][5]), float(xr[it][6]), float(xr[it][7])};
    }
    if (tid < 9 * NQ) s_w[tid] = wr;
  };

  f32x4 acc1[NTN][TMW1];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < TMW1; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < SB_VEC; i += 256) s_b[i] = h8{};  // pixels 196..207 of the last tile: zeros

  load_x(0);
  store_x();
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const int c0 = ch * 32;
    if (ch + 1 < NCH) load_x(c0 + 32);
    h8 af[NTN];
#pragma unroll
    for (int i = 0; i < NTN; ++i) af[i] = *reinterpret_cast<const h8*>(pw1 + (int64_t)(i * 16 + r16) * p.KPAD + c0 + g * 8);
    // dw3 over the t region: task = (quad, row, 2-px segment), quad fastest
    constexpr int NTASK = NQ * TTH * (TTW / 2);
    for (int task = tid; task < NTASK; task += 256) {
      const int q = task % NQ;
      const int r = (task / NQ) % TTH;
      const int sg = task / (NQ * TTH);
      float a[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const f32x4* xrow = &s_x[((r + ky) * XWP + sg * 2) * NQ + q];
        f32x4 xs[4], wv[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) xs[i] = xrow[i * NQ];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) wv[kx] = s_w[(ky * 3 + kx) * NQ + q];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c + kx][e], wv[kx][e], a[c][e]);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int px = r * TTW + sg * 2 + c;
        *(reinterpret_cast<h4*>(&s_b[bslot(px, q >> 1)]) + (q & 1)) =
            to_h4_rne(a[c]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TMW1; ++j) {
      const int t = wave + 4 * j;
      if (t < NT1) {
        const h8 bf = s_b[bslot(t * 16 + r16, g)];
#pragma unroll
        for (int i = 0; i < NTN; ++i) acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf, acc1[i][j], 0, 0, 0);
      }
    }
    if (ch + 1 < NCH) {
      __syncthreads();  // every wave is past this chunk's window, taps and B tile
      store_x();
      __syncthreads();
    }
  }
  // t = SiLU(acc1 + b1) -> fp16, zero outside the image
#pragma unroll
  for (int i = 0; i < NTN; ++i) {
    const int co = i * 16 + 4 * g;
    const f32x4 bq = *reinterpret_cast<const f32x4*>(b1 + co);
#pragma unroll
    for (int j = 0; j < TMW1; ++j) {
      const int t = wave + 4 * j;
      const int px = t * 16 + r16;
      if (t < NT1 && px < NTP) {
        const int gy = ty0 + px / TTW, gx = tx0 + px % TTW;
        const bool in = gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
        float sv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) sv[e] = in ? silu_fast(acc1[i][j][e] + bq[e]) : 0.f;
        s_t[(px * C + co) / 4] = to_h4_rne(sv);
      }
    }
  }

  // ---------------------------------------------------------------- phase 2: u = cv2(t) on 8x8
  constexpr int TWP = TTW | 1;
  constexpr int TAPV = 49 * NQ;  // 392 fp32 tap quads
  f32x4 acc2[NTN][1];
#pragma unroll
  for (int i = 0; i < NTN; ++i) acc2[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ch = 0; ch < NCH; ++ch) {
    const int c0 = ch * 32;
    f32x4 w2r[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = min(tid + it * 256, TAPV - 1);
      const f32x4 w = *reinterpret_cast<const f32x4*>(dw2 + (i / NQ) * C + c0 + (i % NQ) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) w2r[it][e] = float(_Float16(w[e]));
    }
    h8 af[NTN];
#pragma unroll
    for (int i = 0; i < NTN; ++i) af[i] = vload(p.w + (int64_t)(i * 16 + r16) * p.KPAD + c0 + g * 8);
    __syncthreads();  // t complete (first chunk) / previous chunk's window, taps, B tile consumed
    for (int i = tid; i < NTP * NQ; i += 256) {  // t chunk -> fp32 window (row pitch TWP)
      const int px = i / NQ, q = i % NQ;
      const h4 v = s_t[(px * C + c0) / 4 + q];
      s_x[((px / TTW) * TWP + px % TTW) * NQ + q] = f32x4{float(v[0]), float(v[1]), float(v[2]), float(v[3])};
    }
#pragma unroll
    for (int it = 0; it < 2; ++it)
      if (tid + it * 256 < TAPV) s_w[tid + it * 256] = w2r[it];
    __syncthreads();
    {  // dw7: one task per thread = (quad, row, 2-px segment)
      const int q = tid % NQ;
      const int r = (tid / NQ) % TH;
      const int sg = tid / (NQ * TH);
      float a[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll 1
      for (int ky = 0; ky < 7; ++ky) {
        const f32x4* xrow = &s_x[((r + ky) * TWP + sg * 2) * NQ + q];
        f32x4 xs[8], wv[7];
#pragma unroll
        for (int i = 0; i < 8; ++i) xs[i] = xrow[i * NQ];
#pragma unroll
        for (int kx = 0; kx < 7; ++kx) wv[kx] = s_w[(ky * 7 + kx) * NQ + q];
#pragma unroll
        for (int kx = 0; kx < 7; ++kx)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c + kx][e], wv[kx][e], a[c][e]);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int px = r * TW + sg * 2 + c;
        *(reinterpret_cast<h4*>(&s_b[bslot(px, q >> 1)]) + (q & 1)) =
            to_h4_rne(a[c]);
      }
    }
    __syncthreads();
    const h8 bf = s_b[bslot(wave * 16 + r16, g)];
#pragma unroll
    for (int i = 0; i < NTN; ++i) acc2[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf, acc2[i][0], 0, 0, 0);
  }

  const int op = wave * 16 + r16;
  const int oy = oy0 + op / TW, ox = ox0 + op % TW;
  const bool pv[1] = {oy < p.Ho && ox < p.Wo};
  const int64_t pp[1] = {((int64_t)b * p.Ho + oy) * p.Wo + ox};
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = i * 16 + 4 * g;
  conv_epilogue<_Float16, NTN, 1>(p, acc2, pp, pv, co);
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dsbottleneck_nhwc(const ydbl_dsbneck_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "dsbottleneck: null descriptor");
  if (check_view(&d->x, "dsbottleneck.x", true) || check_view(&d->y, "dsbottleneck.y", true)) return YDBL_EINVAL;
  if (d->x.dtype != YDBL_F16 || d->y.dtype != YDBL_F16) return fail(YDBL_EINVAL, "dsbottleneck: fp16 views only");
  const int c = d->x.c;
  if (c != 64) return fail(YDBL_EINVAL, "dsbottleneck: C must be 64");
  if (d->y.c != c || d->y.n != d->x.n || d->y.h != d->x.h || d->y.w != d->x.w)
    return fail(YDBL_EINVAL, "dsbottleneck: y must have x's shape");
  if (d->kpad != c) return fail(YDBL_EINVAL, "dsbottleneck: kpad must equal C");
  if (!d->dw1_w || !d->pw1_w || !d->b1 || !d->dw2_w || !d->pw2_w || !d->b2)
    return fail(YDBL_EINVAL, "dsbottleneck: null weights");
  if (d->y.ptr == d->x.ptr) return fail(YDBL_EINVAL, "dsbottleneck: y must not alias x (halo reads)");
  ConvArgs<_Float16> a{};
  a.x = reinterpret_cast<const _Float16*>(d->x.ptr);
  a.xcs = d->x.cs; a.N = d->x.n; a.H = d->x.h; a.W = d->x.w; a.Cin = c;
  a.y = reinterpret_cast<_Float16*>(d->y.ptr);
  a.ycs = d->y.cs; a.Ho = d->y.h; a.Wo = d->y.w; a.Cout = c;
  a.r = d->add ? a.x : nullptr; a.rcs = d->x.cs;
  a.w = reinterpret_cast<const _Float16*>(d->pw2_w); a.bias = d->b2;
  a.KW = 7; a.S = 1; a.PAD = 3; a.DIL = 1; a.K = c; a.KPAD = d->kpad;
  a.act = YDBL_ACT_SILU; a.res = d->add ? YDBL_RES_ADD : YDBL_RES_NONE;
  a.P = d->y.n * d->y.h * d->y.w;
  const int tiles_x = (int)cdiv(a.Wo, TW), tiles_y = (int)cdiv(a.Ho, TH);
  const int64_t n = (int64_t)a.N * tiles_x * tiles_y;
  dsbneck_kernel<4><<<(unsigned)n, 256, 0, as_stream(stream)>>>(
      a, d->dw1_w, reinterpret_cast<const _Float16*>(d->pw1_w), d->b1, d->dw2_w, tiles_x, tiles_y);
  return check_launch("ydbl_dsbottleneck_nhwc");
}
