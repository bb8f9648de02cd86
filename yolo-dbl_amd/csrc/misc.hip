// Memory-bound NHWC kernels: depthwise conv, input layout, FullPAD gate, pool/upsample concat,
// DySample bilinear gather, LSKblock spatial gate.  One thread = one pixel x one 16-byte channel
// vector (8 x f16 / 4 x f32), fp32 arithmetic, coalesced along channels.
#include "common.hpp"

namespace ydbl {

// ------------------------------------------------------------------ depthwise convolution
template <typename T>
__global__ __launch_bounds__(256) void dwconv_kernel(DView<const T> x, DView<T> y, DView<const T> r,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     int KH, int KW, int S, int PAD, int DIL, int act) {
  constexpr int V = Vec<T>::N;
  const int cg = y.c / V;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)y.n * y.h * y.w * cg;
  if (idx >= total) return;
  const int c0 = (int)(idx % cg) * V;
  int64_t pix = idx / cg;
  const int ox = (int)(pix % y.w);
  const int64_t t = pix / y.w;
  const int oy = (int)(t % y.h);
  const int b = (int)(t / y.h);
  float acc[V];
#pragma unroll
  for (int q = 0; q < V; ++q) acc[q] = 0.f;
  for (int ky = 0; ky < KH; ++ky) {
    const int iy = oy * S - PAD + ky * DIL;
    if (iy < 0 || iy >= x.h) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int ix = ox * S - PAD + kx * DIL;
      if (ix < 0 || ix >= x.w) continue;
      float xv[V], wv[V];
      load_f<V>(x.at(b, iy, ix) + c0, xv);
      load_f<V>(w + (ky * KW + kx) * y.c + c0, wv);
#pragma unroll
      for (int q = 0; q < V; ++q) acc[q] = fmaf(xv[q], wv[q], acc[q]);
    }
  }
  if (bias) {
    float bv[V];
    load_f<V>(bias + c0, bv);
#pragma unroll
    for (int q = 0; q < V; ++q) acc[q] += bv[q];
  }
#pragma unroll
  for (int q = 0; q < V; ++q) acc[q] = apply_act<T>(acc[q], act);
  if (r.p) {
    float rv[V];
    load_f<V>(r.at(b, oy, ox) + c0, rv);
#pragma unroll
    for (int q = 0; q < V; ++q) acc[q] = rv[q] + acc[q];
  }
  store_f<V>(y.at(b, oy, ox) + c0, acc);
}

// LDS-tiled variant for the fixed geometries of the DBL graphs.  A workgroup owns a TH x TW output
// tile x CV channel vectors (16 B each); the input tile it needs, halo included, is staged in LDS
// once with coalesced 16-byte loads (one global read per input element instead of one per tap), then
// every thread computes its outputs from LDS.  Accumulation order per output is the reference's tap
// order (ky, kx) with padded taps skipped, identical to dwconv_kernel.
template <typename T, int K, int S, int DIL, int CV, int TH, int TW>
__global__ __launch_bounds__(256) void dwconv_lds_kernel(DView<const T> x, DView<T> y, DView<const T> r,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         int PAD, int act, int tiles_x, int tiles_y) {
  constexpr int V = Vec<T>::N;
  constexpr int IH = (TH - 1) * S + (K - 1) * DIL + 1;
  constexpr int IW = (TW - 1) * S + (K - 1) * DIL + 1;
  constexpr int LANES = 256 / CV;             // pixel lanes
  constexpr int NPX = (TH * TW) / LANES;      // outputs per thread, computed jointly
  static_assert(NPX * LANES == TH * TW, "tile must split evenly over the pixel lanes");
  using vec = typename Vec<T>::type;
  __shared__ vec tile[IH * IW * CV];
  __shared__ f32x4 wts[K * K * CV * V / 4];   // fp32 taps of this workgroup's channel slice
  const int cgroups = y.c / (CV * V);
  int bid = blockIdx.x;
  const int cgi = bid % cgroups; bid /= cgroups;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int c0 = cgi * CV * V;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  {  // stage the halo tile: all loads of a thread in flight before the first LDS store
    constexpr int TOT = IH * IW * CV, IT = (TOT + 255) / 256;
    vec tmp[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = min((int)threadIdx.x + it * 256, TOT - 1);
      const int cv = i % CV, px = i / CV;
      const int iy = iy0 + px / IW, ix = ix0 + px % IW;
      const bool ok = iy >= 0 && iy < x.h && ix >= 0 && ix < x.w;
      tmp[it] = vload_sel(x.at(b, iy, ix) + c0 + cv * V, x.p + c0, ok);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i < TOT) tile[i] = tmp[it];
    }
  }
  for (int i = threadIdx.x; i < K * K * CV * V / 4; i += 256) {
    const int tap = i / (CV * V / 4), q = i % (CV * V / 4);
    wts[i] = *reinterpret_cast<const f32x4*>(w + tap * y.c + c0 + 4 * q);
  }
  __syncthreads();
  const int cv = threadIdx.x % CV, pl = threadIdx.x / CV;
  const int cc = c0 + cv * V;
  int py[NPX], px[NPX];
  bool ok[NPX];
#pragma unroll
  for (int u = 0; u < NPX; ++u) {
    const int p = pl + u * LANES;
    py[u] = p / TW; px[u] = p % TW;
    ok[u] = oy0 + py[u] < y.h && ox0 + px[u] < y.w;
  }
  float acc[NPX][V];
#pragma unroll
  for (int u = 0; u < NPX; ++u)
#pragma unroll
    for (int q = 0; q < V; ++q) acc[u][q] = 0.f;
#pragma unroll 1
  for (int ky = 0; ky < K; ++ky) {
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      float wv[V];
#pragma unroll
      for (int h = 0; h < V / 4; ++h) {
        const f32x4 t4 = wts[((ky * K + kx) * CV + cv) * (V / 4) + h];
        wv[4 * h] = t4[0]; wv[4 * h + 1] = t4[1]; wv[4 * h + 2] = t4[2]; wv[4 * h + 3] = t4[3];
      }
#pragma unroll
      for (int u = 0; u < NPX; ++u) {
        const int iy = (oy0 + py[u]) * S - PAD + ky * DIL;
        const int ix = (ox0 + px[u]) * S - PAD + kx * DIL;
        if (iy < 0 || iy >= x.h || ix < 0 || ix >= x.w) continue;  // the reference has no padded-tap terms
        const vec xv = tile[((py[u] * S + ky * DIL) * IW + px[u] * S + kx * DIL) * CV + cv];
#pragma unroll
        for (int q = 0; q < V; ++q) acc[u][q] = fmaf(float(xv[q]), wv[q], acc[u][q]);
      }
    }
  }
  float bv[V];
#pragma unroll
  for (int q = 0; q < V; ++q) bv[q] = 0.f;
  if (bias) load_f<V>(bias + cc, bv);
#pragma unroll
  for (int u = 0; u < NPX; ++u) {
    if (!ok[u]) continue;
    const int oy = oy0 + py[u], ox = ox0 + px[u];
    float o[V];
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = apply_act<T>(bias ? acc[u][q] + bv[q] : acc[u][q], act);
    if (r.p) {
      float rv[V];
      load_f<V>(r.at(b, oy, ox) + cc, rv);
#pragma unroll
      for (int q = 0; q < V; ++q) o[q] = rv[q] + o[q];
    }
    store_f<V>(y.at(b, oy, ox) + cc, o);
  }
}

template <typename T>
static bool launch_dw_lds(const ydbl_dwconv_desc* d, DView<const T> x, DView<T> y, DView<const T> r, hipStream_t s) {
  constexpr int V = Vec<T>::N;
  const int k = d->kw, st = d->stride, dl = d->dil;
  auto go = [&](auto kern, int cv, int th, int tw) {
    if (d->y.c % (cv * V)) return false;
    const int tiles_x = (int)cdiv(d->y.w, tw), tiles_y = (int)cdiv(d->y.h, th);
    const int64_t blocks = (int64_t)d->y.n * tiles_y * tiles_x * (d->y.c / (cv * V));
    kern<<<(unsigned)blocks, 256, 0, s>>>(x, y, r, d->w, d->bias, d->pad, d->act, tiles_x, tiles_y);
    return true;
  };
  // f16: 8 vectors = 64 channels per workgroup; f32: 8 vectors = 32 channels
  if (k == 3 && st == 1 && dl == 1) return go(dwconv_lds_kernel<T, 3, 1, 1, 8, 8, 8>, 8, 8, 8);
  if (k == 3 && st == 2 && dl == 1) return go(dwconv_lds_kernel<T, 3, 2, 1, 8, 8, 8>, 8, 8, 8);
  if (k == 5 && st == 1 && dl == 1) return go(dwconv_lds_kernel<T, 5, 1, 1, 8, 8, 8>, 8, 8, 8);
  if (k == 7 && st == 1 && dl == 1) return go(dwconv_lds_kernel<T, 7, 1, 1, 8, 8, 8>, 8, 8, 8);
  if (k == 7 && st == 1 && dl == 3) return go(dwconv_lds_kernel<T, 7, 1, 3, 2, 8, 16>, 2, 8, 16);
  return false;
}

// ------------------------------------------------------------------ chained depthwise pair (LSK)
// LSKA.py:40-41: a1 = conv0(x) (dw 5x5), a2 = conv_spatial(a1) (dw 7x7 dil 3).  On the small P5 maps
// (20^2 at 640) the dilated 7x7 needs a 9-px halo, so an output tile drags in 3-6x its pixels and the
// two launches cost 17 + 27 us (DBL-n bs32).  Here a workgroup owns one image x CV channel vectors
// with the WHOLE map in LDS: x is staged once, a1 is computed into LDS (and stored, conv1 reads it),
// a2 is computed from that.  Tap order (ky, kx) with padded taps skipped and fp32 FMAs as in
// dwconv_lds_kernel, and a1 is rounded to T before phase 2 exactly as the two-launch path stores and
// reloads it, so the outputs are bit-identical to it.
constexpr int DWP_HWMAX = 512;
// one phase: every thread owns channel vector cv of pixels pl, pl + LANES, ...  (Measured on DBL-n
// bs32: this plain form, 36-38 us for both LSK depthwise convs, beat tap-unrolled variants with
// 2-4 independent pixels in flight, 42-53 us: their LDS reads and code size cost more than the ILP
// they bought.)
template <typename T, int K, int D, int CV, int NT>
__device__ __forceinline__ void dw_pair_phase(const typename Vec<T>::type* src, const f32x4* wts, const float* bias,
                                              int pad, int act, DView<T> out, typename Vec<T>::type* keep, int b,
                                              int cc, int cv, int pl, int H, int W) {
  constexpr int V = Vec<T>::N, LANES = NT / CV;
  using vec = typename Vec<T>::type;
  float bv[V];
#pragma unroll
  for (int q = 0; q < V; ++q) bv[q] = 0.f;
  if (bias) load_f<V>(bias + cc, bv);
  for (int p = pl; p < H * W; p += LANES) {
    const int oy = p / W, ox = p % W;
    float acc[V];
#pragma unroll
    for (int q = 0; q < V; ++q) acc[q] = 0.f;
#pragma unroll 1
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy - pad + ky * D;
      if (iy < 0 || iy >= H) continue;
#pragma unroll 1
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox - pad + kx * D;
        if (ix < 0 || ix >= W) continue;  // padded taps contribute no term
        const vec xv = src[(iy * W + ix) * CV + cv];
#pragma unroll
        for (int h = 0; h < V / 4; ++h) {
          const f32x4 t4 = wts[((ky * K + kx) * CV + cv) * (V / 4) + h];
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[4 * h + q] = fmaf(float(xv[4 * h + q]), t4[q], acc[4 * h + q]);
        }
      }
    }
    float o[V];
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = apply_act<T>(bias ? acc[q] + bv[q] : acc[q], act);
    store_f<V>(out.at(b, oy, ox) + cc, o);
    if (keep) {
      vec t;
#pragma unroll
      for (int q = 0; q < V; ++q) t[q] = (T)round_to<T>(o[q]);  // the same pinned rounding as the stored y0
      keep[p * CV + cv] = t;
    }
  }
}

// NT = 1024 threads: a pixel's taps are a chain of dependent LDS reads, and at one workgroup per CU (16
// images x 256 channels / 16 = 256 workgroups) four waves per SIMD hide that latency where one did not
// (DBL-n bs16 LSK pair 39.5 -> 20.9 us, bit-identical).
template <typename T, int K0, int D0, int K1, int D1, int CV, int NT>
__global__ __launch_bounds__(NT) void dw_pair_kernel(DView<const T> x, DView<T> y0, DView<T> y1,
                                                      const float* __restrict__ w0, const float* __restrict__ b0,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      int pad0, int pad1, int act0, int act1) {
  constexpr int V = Vec<T>::N;
  using vec = typename Vec<T>::type;
  __shared__ vec tx[DWP_HWMAX * CV], ta[DWP_HWMAX * CV];
  __shared__ f32x4 ws0[K0 * K0 * CV * V / 4], ws1[K1 * K1 * CV * V / 4];
  const int C = y0.c, H = x.h, W = x.w, HW = H * W;
  const int cgroups = C / (CV * V);
  const int b = blockIdx.x / cgroups, c0 = (blockIdx.x % cgroups) * CV * V;
  {  // all of a thread's map loads in flight before the first LDS store
    constexpr int IT = (DWP_HWMAX * CV + NT - 1) / NT;
    vec tmp[IT];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int i = threadIdx.x + u * NT, cv = i % CV, px = min(i / CV, HW - 1);
      tmp[u] = vload(x.at(b, px / W, px % W) + c0 + cv * V);
    }
#pragma unroll
    for (int u = 0; u < IT; ++u)
      if (threadIdx.x + u * NT < HW * CV) tx[threadIdx.x + u * NT] = tmp[u];
  }
  for (int i = threadIdx.x; i < K0 * K0 * CV * V / 4; i += NT) {
    const int tap = i / (CV * V / 4), q = i % (CV * V / 4);
    ws0[i] = *reinterpret_cast<const f32x4*>(w0 + tap * C + c0 + 4 * q);
  }
  for (int i = threadIdx.x; i < K1 * K1 * CV * V / 4; i += NT) {
    const int tap = i / (CV * V / 4), q = i % (CV * V / 4);
    ws1[i] = *reinterpret_cast<const f32x4*>(w1 + tap * C + c0 + 4 * q);
  }
  __syncthreads();
  const int cv = threadIdx.x % CV, pl = threadIdx.x / CV;
  const int cc = c0 + cv * V;
  dw_pair_phase<T, K0, D0, CV, NT>(tx, ws0, b0, pad0, act0, y0, ta, b, cc, cv, pl, H, W);
  __syncthreads();
  dw_pair_phase<T, K1, D1, CV, NT>(ta, ws1, b1, pad1, act1, y1, nullptr, b, cc, cv, pl, H, W);
}

// ------------------------------------------------------------------ input NCHW fp32 -> NHWC
template <typename T>
__global__ __launch_bounds__(256) void input_kernel(const float* __restrict__ x, int n, int c, int h, int w,
                                                    float scale, DView<T> y, InputBind ib) {
  x = bound_x(ib, x);
  scale = bound_scale(ib, scale);
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t hw = (int64_t)h * w;
  if (pix >= (int64_t)n * hw) return;
  const int64_t b = pix / hw, off = pix % hw;
  T* yp = y.pix(pix);
  for (int c0 = 0; c0 < y.c; c0 += Vec<T>::N) {
    float v[Vec<T>::N];
#pragma unroll
    for (int q = 0; q < Vec<T>::N; ++q) {
      const int ch = c0 + q;
      v[q] = ch < c ? __builtin_nontemporal_load(x + (b * c + ch) * hw + off) * scale : 0.f;
    }
    store_f<Vec<T>::N>(yp + c0, v);
  }
}

// ------------------------------------------------------------------ FullPAD: y = a + g * b
template <typename T>
__global__ __launch_bounds__(256) void gate_add_kernel(DView<const T> a, DView<const T> bv, float gate, DView<T> y) {
  constexpr int V = Vec<T>::N;
  const int cg = y.c / V;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)y.n * y.h * y.w * cg) return;
  const int c0 = (int)(idx % cg) * V;
  const int64_t pix = idx / cg;
  float av[V], b2[V], o[V];
  load_f<V>(a.pix(pix) + c0, av);
  load_f<V>(bv.pix(pix) + c0, b2);
#pragma unroll
  for (int q = 0; q < V; ++q) o[q] = __builtin_fmaf(gate, b2[q], av[q]);
  store_f<V>(y.pix(pix) + c0, o);
}

// ------------------------------------------------------------------ FuseModule / DownsampleConv input
template <typename T>
__global__ __launch_bounds__(256) void pool_up_concat_kernel(DView<const T> lo, DView<const T> mid,
                                                             DView<const T> hi, DView<T> y) {
  // Work items are numbered segment by segment (all pool items, then all copies, then all
  // upsamples), channel vector fastest: a wave takes one branch, instead of every wave (one output
  // pixel = 64 vectors) running all three branches one after the other.
  constexpr int V = Vec<T>::N;
  const int clo = lo.p ? lo.c : 0, cmid = mid.p ? mid.c : 0;
  const int64_t npix = (int64_t)y.n * y.h * y.w;
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npix * (y.c / V)) return;
  int seg_c0 = 0, seg_cg = clo / V;
  if (idx >= npix * seg_cg) {
    idx -= npix * seg_cg;
    seg_c0 = clo;
    seg_cg = cmid / V;
    if (idx >= npix * seg_cg) {
      idx -= npix * seg_cg;
      seg_c0 = clo + cmid;
      seg_cg = (y.c - clo - cmid) / V;
    }
  }
  const int c = seg_c0 + (int)(idx % seg_cg) * V;
  const int64_t pix = idx / seg_cg;
  const int ox = (int)(pix % y.w);
  const int64_t t = pix / y.w;
  const int oy = (int)(t % y.h);
  const int b = (int)(t / y.h);
  float o[V];
  if (c < clo) {  // nn.AvgPool2d(2): mean of the 2x2 window (sum then / 4)
    float s[V], v[V];
    load_f<V>(lo.at(b, 2 * oy, 2 * ox) + c, s);
    load_f<V>(lo.at(b, 2 * oy, 2 * ox + 1) + c, v);
#pragma unroll
    for (int q = 0; q < V; ++q) s[q] += v[q];
    load_f<V>(lo.at(b, 2 * oy + 1, 2 * ox) + c, v);
#pragma unroll
    for (int q = 0; q < V; ++q) s[q] += v[q];
    load_f<V>(lo.at(b, 2 * oy + 1, 2 * ox + 1) + c, v);
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = (s[q] + v[q]) / 4.0f;
  } else if (c < clo + cmid) {
    load_f<V>(mid.at(b, oy, ox) + (c - clo), o);
  } else {  // nn.Upsample(scale_factor=2, mode='nearest')
    load_f<V>(hi.at(b, oy >> 1, ox >> 1) + (c - clo - cmid), o);
  }
  store_f<V>(y.at(b, oy, ox) + c, o);
}

// ------------------------------------------------------------------ DySample (style lp, scale 2)
// offset channel k = coord*4G + group*4 + i*2 + j (i,j = sub-pixel row/col of the x2 output).
// Coordinates follow DySample.py:48-61 and ATen grid_sampler (align_corners=False, border).
template <typename T>
__global__ __launch_bounds__(256) void dysample_kernel(DView<const T> x, DView<const T> off, int G, DView<T> y,
                                                       DView<T> y2, DView<const T> r2, float a2, float b2) {
  constexpr int V = Vec<T>::N;
  const int cpg = x.c / G;
  const int cgv = cpg / V;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)y.n * y.h * y.w * G * cgv;
  if (idx >= total) return;
  const int cv = (int)(idx % cgv);
  int64_t t = idx / cgv;
  const int gi = (int)(t % G);
  t /= G;
  const int ox2 = (int)(t % y.w);
  t /= y.w;
  const int oy2 = (int)(t % y.h);
  const int b = (int)(t / y.h);
  const int H = x.h, W = x.w;
  const int h = oy2 >> 1, w = ox2 >> 1, si = oy2 & 1, sj = ox2 & 1;
  const T* op = off.at(b, h, w);
  const float offx = float(op[gi * 4 + si * 2 + sj]);
  const float offy = float(op[4 * G + gi * 4 + si * 2 + sj]);
  // normalized grid coordinate, then grid_sampler_unnormalize + border clip
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
  const int c0 = gi * cpg + cv * V;
  // The four corner loads are unconditional (clamped addresses, the out-of-range corner's weight
  // zeroed: acc + v * 0 = acc exactly, v finite), so they are in flight together instead of each
  // behind its own branch and wait.  Terms are added in grid_sample's nw, ne, sw, se order.
  const bool xin = x1 < W, yin = y1 < H;
  const int x1c = xin ? x1 : x0, y1c = yin ? y1 : y0;
  float vnw[V], vne[V], vsw[V], vse[V];
  load_f<V>(x.at(b, y0, x0) + c0, vnw);
  load_f<V>(x.at(b, y0, x1c) + c0, vne);
  load_f<V>(x.at(b, y1c, x0) + c0, vsw);
  load_f<V>(x.at(b, y1c, x1c) + c0, vse);
  const float kne = xin ? wne : 0.f, ksw = yin ? wsw : 0.f, kse = xin && yin ? wse : 0.f;
  float acc[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    acc[q] = blend4(vnw[q], wnw, vne[q], kne, vsw[q], ksw, vse[q], kse);
  }
  store_f<V>(y.at(b, oy2, ox2) + c0, acc);
  if (y2.p) {  // fused FullPAD_Tunnel (block.py:1954-1956) on this output: y2 = a2 * T(y) + b2 * r2
    float rv[V], o2[V];
    load_f<V>(r2.at(b, oy2, ox2) + c0, rv);
#pragma unroll
    for (int q = 0; q < V; ++q) o2[q] = pad_mix(a2, round_to<T>(acc[q]), b2, rv[q]);
    store_f<V>(y2.at(b, oy2, ox2) + c0, o2);
  }
}

// ------------------------------------------------------------------ LSKblock gate
// LSKA.py:46-52.  Stats: 32 lanes per pixel walk its channel vectors (coalesced 16-byte loads, 512 B
// per pixel per wave instruction) and reduce sum / max over the 32 lanes; one launch of N*H*W*32
// threads (a thread per pixel looping over all channels gave 50 workgroups at 20^2 bs32).
template <typename T>
__global__ __launch_bounds__(256) void lsk_stats_kernel(DView<const T> attn, float* __restrict__ agg) {
  constexpr int V = Vec<T>::N, L = 32;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pix = t / L;
  const int sub = (int)(t % L);
  const bool live = pix < (int64_t)attn.n * attn.h * attn.w;  // whole 32-lane groups share `live`
  const T* p = attn.pix(live ? pix : 0);
  float s = 0.f, m = -INFINITY;
  for (int c = sub * V; c < attn.c; c += L * V) {
    float v[V];
    load_f<V>(p + c, v);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s += v[q];
      m = fmaxf(m, v[q]);
    }
  }
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    m = fmaxf(m, __shfl_xor(m, o));
  }
  if (live && sub == 0) {
    agg[pix * 2 + 0] = s / float(attn.c);
    agg[pix * 2 + 1] = m;
  }
}

// Gate: thread per (pixel, channel vector).  When a pixel's vectors fill whole 16-lane groups
// (half % (16 V) == 0: every DBL config) the 2 x 49 taps of the 7x7 squeeze conv are split over
// the 16 lanes and summed by xor-shuffles, instead of every thread redoing all 98.
template <typename T>
__global__ __launch_bounds__(256) void lsk_gate_kernel(DView<const T> attn, const float* __restrict__ agg,
                                                       const float* __restrict__ sw, const float* __restrict__ sb,
                                                       DView<T> out) {
  constexpr int V = Vec<T>::N;
  const int half = out.c;
  const int cg = half / V;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)out.n * out.h * out.w * cg) return;  // 16-lane groups leave together (split path)
  const int c0 = (int)(idx % cg) * V;
  const int64_t pix = idx / cg;
  const int ox = (int)(pix % out.w);
  const int64_t t = pix / out.w;
  const int oy = (int)(t % out.h);
  const int b = (int)(t / out.h);
  const bool split = cg % 16 == 0;  // uniform
  const int t0 = split ? (int)(idx & 15) : 0, ts = split ? 16 : 1;
  float s0 = 0.f, s1 = 0.f;
  for (int tap = t0; tap < 98; tap += ts) {
    const int ci = tap / 49, ky = (tap % 49) / 7, kx = tap % 7;
    const int iy = oy - 3 + ky, ix = ox - 3 + kx;
    if (iy < 0 || iy >= out.h || ix < 0 || ix >= out.w) continue;
    const float a = agg[(((int64_t)b * out.h + iy) * out.w + ix) * 2 + ci];
    s0 = fmaf(sw[((0 * 2 + ci) * 7 + ky) * 7 + kx], a, s0);
    s1 = fmaf(sw[((1 * 2 + ci) * 7 + ky) * 7 + kx], a, s1);
  }
  if (split) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
  }
  s0 = sigmoidf_(s0 + sb[0]);
  s1 = sigmoidf_(s1 + sb[1]);
  float a1[V], a2[V], o[V];
  load_f<V>(attn.pix(pix) + c0, a1);
  load_f<V>(attn.pix(pix) + half + c0, a2);
#pragma unroll
  for (int q = 0; q < V; ++q) o[q] = gate_mix(a1[q], s0, a2[q], s1);
  store_f<V>(out.pix(pix) + c0, o);
}

template <typename T>
static DView<const T> cview(const ydbl_view* v) {
  if (!v) return DView<const T>{nullptr, 0, 0, 0, 0, 0};
  return DView<const T>{reinterpret_cast<const T*>(v->ptr), v->n, v->h, v->w, v->c, v->cs};
}

static unsigned nblk(int64_t n) { return (unsigned)cdiv(n, 256); }

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dwconv2d_nhwc(const ydbl_dwconv_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "dwconv: null descriptor");
  if (check_view(&d->x, "dwconv.x", true) || check_view(&d->y, "dwconv.y", true)) return YDBL_EINVAL;
  if (d->x.c != d->y.c || d->x.n != d->y.n || d->x.dtype != d->y.dtype) return fail(YDBL_EINVAL, "dwconv: x/y mismatch");
  const int ho = (d->x.h + 2 * d->pad - d->dil * (d->kh - 1) - 1) / d->stride + 1;
  const int wo = (d->x.w + 2 * d->pad - d->dil * (d->kw - 1) - 1) / d->stride + 1;
  if (ho != d->y.h || wo != d->y.w) return fail(YDBL_EINVAL, "dwconv: output spatial size mismatch");
  if (!d->w) return fail(YDBL_EINVAL, "dwconv: null weights");
  const bool res = d->res_mode == YDBL_RES_ADD;
  if (d->res_mode != YDBL_RES_NONE && !res) return fail(YDBL_EINVAL, "dwconv: only residual ADD is supported");
  if (res && (check_view(&d->r, "dwconv.r", true) || d->r.c != d->y.c || d->r.n != d->y.n || d->r.h != d->y.h ||
              d->r.w != d->y.w || d->r.dtype != d->y.dtype))
    return fail(YDBL_EINVAL, "dwconv: residual shape mismatch");
  hipStream_t s = as_stream(stream);
  const int V = d->x.dtype == YDBL_F16 ? 8 : 4;
  const int64_t total = (int64_t)d->y.n * d->y.h * d->y.w * (d->y.c / V);
  if (d->kh == d->kw) {
    const bool done = d->x.dtype == YDBL_F16
                          ? launch_dw_lds<_Float16>(d, cview<_Float16>(&d->x), dview<_Float16>(d->y),
                                                   cview<_Float16>(res ? &d->r : nullptr), s)
                          : launch_dw_lds<float>(d, cview<float>(&d->x), dview<float>(d->y),
                                                cview<float>(res ? &d->r : nullptr), s);
    if (done) return check_launch("ydbl_dwconv2d_nhwc");
  }
  if (d->x.dtype == YDBL_F16)
    dwconv_kernel<_Float16><<<nblk(total), 256, 0, s>>>(cview<_Float16>(&d->x), dview<_Float16>(d->y),
                                                        cview<_Float16>(res ? &d->r : nullptr), d->w, d->bias,
                                                        d->kh, d->kw, d->stride, d->pad, d->dil, d->act);
  else
    dwconv_kernel<float><<<nblk(total), 256, 0, s>>>(cview<float>(&d->x), dview<float>(d->y),
                                                     cview<float>(res ? &d->r : nullptr), d->w, d->bias, d->kh, d->kw,
                                                     d->stride, d->pad, d->dil, d->act);
  return check_launch("ydbl_dwconv2d_nhwc");
}

extern "C" int ydbl_dwconv2d_pair_nhwc(const ydbl_dwconv_desc* d0, const ydbl_dwconv_desc* d1, void* stream) {
  if (!d0 || !d1) return fail(YDBL_EINVAL, "dw_pair: null descriptor");
  if (d1->x.ptr != d0->y.ptr || d1->x.cs != d0->y.cs || d1->x.c != d0->y.c)
    return fail(YDBL_EINVAL, "dw_pair: d1.x must be d0.y");
  const bool pair = d0->kh == 5 && d0->kw == 5 && d0->dil == 1 && d1->kh == 7 && d1->kw == 7 && d1->dil == 3 &&
                    d0->stride == 1 && d1->stride == 1 && d0->res_mode == YDBL_RES_NONE &&
                    d1->res_mode == YDBL_RES_NONE && d0->x.h == d0->y.h && d0->x.w == d0->y.w &&
                    d1->y.h == d0->y.h && d1->y.w == d0->y.w && d0->x.h * d0->x.w <= DWP_HWMAX &&
                    d0->x.dtype == d0->y.dtype && d1->y.dtype == d0->y.dtype && d0->x.c == d0->y.c &&
                    d1->y.c == d0->y.c && d0->x.n == d0->y.n && d1->y.n == d0->y.n;
  const int V = d0->x.dtype == YDBL_F16 ? 8 : 4;
  constexpr int CV = 2;  // 16 (f16) / 8 (f32) channels per workgroup (CV = 1: 42 vs 38 us)
  if (!pair || d0->y.c % (CV * V) || !d0->w || !d1->w || check_view(&d0->x, "dw_pair.x", true) ||
      check_view(&d0->y, "dw_pair.y0", true) || check_view(&d1->y, "dw_pair.y1", true)) {
    // not the fused geometry: the two launches
    const int r = ydbl_dwconv2d_nhwc(d0, stream);
    return r ? r : ydbl_dwconv2d_nhwc(d1, stream);
  }
  hipStream_t s = as_stream(stream);
  const unsigned blocks = (unsigned)(d0->y.n * (d0->y.c / (CV * V)));
  constexpr int NT = 1024;
  if (d0->x.dtype == YDBL_F16)
    dw_pair_kernel<_Float16, 5, 1, 7, 3, CV, NT><<<blocks, NT, 0, s>>>(
        cview<_Float16>(&d0->x), dview<_Float16>(d0->y), dview<_Float16>(d1->y), d0->w, d0->bias, d1->w, d1->bias,
        d0->pad, d1->pad, d0->act, d1->act);
  else
    dw_pair_kernel<float, 5, 1, 7, 3, CV, NT><<<blocks, NT, 0, s>>>(
        cview<float>(&d0->x), dview<float>(d0->y), dview<float>(d1->y), d0->w, d0->bias, d1->w, d1->bias, d0->pad,
        d1->pad, d0->act, d1->act);
  return check_launch("ydbl_dwconv2d_pair_nhwc");
}

extern "C" int ydbl_input_nchw_to_nhwc(const float* x, int32_t n, int32_t c, int32_t h, int32_t w, float scale,
                                       const ydbl_view* y, const ydbl_input_bind* bind, void* stream) {
  if (!x) return fail(YDBL_EINVAL, "input: null x");
  if (check_view(y, "input.y", true)) return YDBL_EINVAL;
  if (y->n != n || y->h != h || y->w != w || y->c < c) return fail(YDBL_EINVAL, "input: shape mismatch");
  hipStream_t s = as_stream(stream);
  const int64_t total = (int64_t)n * h * w;
  if (y->dtype == YDBL_F16)
    input_kernel<_Float16><<<nblk(total), 256, 0, s>>>(x, n, c, h, w, scale, dview<_Float16>(*y), input_bind(bind));
  else
    input_kernel<float><<<nblk(total), 256, 0, s>>>(x, n, c, h, w, scale, dview<float>(*y), input_bind(bind));
  return check_launch("ydbl_input_nchw_to_nhwc");
}

extern "C" int ydbl_gate_add(const ydbl_view* a, const ydbl_view* b, float gate, const ydbl_view* y, void* stream) {
  if (check_view(a, "gate.a", true) || check_view(b, "gate.b", true) || check_view(y, "gate.y", true)) return YDBL_EINVAL;
  if (a->c != y->c || b->c != y->c || a->n * a->h * a->w != y->n * y->h * y->w ||
      b->n * b->h * b->w != y->n * y->h * y->w || a->dtype != y->dtype || b->dtype != y->dtype)
    return fail(YDBL_EINVAL, "gate_add: shape mismatch");
  hipStream_t s = as_stream(stream);
  const int V = y->dtype == YDBL_F16 ? 8 : 4;
  const int64_t total = (int64_t)y->n * y->h * y->w * (y->c / V);
  if (y->dtype == YDBL_F16)
    gate_add_kernel<_Float16><<<nblk(total), 256, 0, s>>>(cview<_Float16>(a), cview<_Float16>(b), gate, dview<_Float16>(*y));
  else
    gate_add_kernel<float><<<nblk(total), 256, 0, s>>>(cview<float>(a), cview<float>(b), gate, dview<float>(*y));
  return check_launch("ydbl_gate_add");
}

extern "C" int ydbl_pool_up_concat(const ydbl_view* lo, const ydbl_view* mid, const ydbl_view* hi, const ydbl_view* y,
                                   void* stream) {
  if (check_view(y, "concat.y", true)) return YDBL_EINVAL;
  int ctot = 0;
  if (lo) {
    if (check_view(lo, "concat.lo", true)) return YDBL_EINVAL;
    if (lo->h != 2 * y->h || lo->w != 2 * y->w || lo->n != y->n) return fail(YDBL_EINVAL, "concat: lo must be 2x output");
    ctot += lo->c;
  }
  if (mid) {
    if (check_view(mid, "concat.mid", true)) return YDBL_EINVAL;
    if (mid->h != y->h || mid->w != y->w || mid->n != y->n) return fail(YDBL_EINVAL, "concat: mid must match output");
    ctot += mid->c;
  }
  if (hi) {
    if (check_view(hi, "concat.hi", true)) return YDBL_EINVAL;
    if (2 * hi->h != y->h || 2 * hi->w != y->w || hi->n != y->n) return fail(YDBL_EINVAL, "concat: hi must be 1/2 output");
    ctot += hi->c;
  }
  if (ctot != y->c) return fail(YDBL_EINVAL, "concat: channel sum mismatch");
  hipStream_t s = as_stream(stream);
  const int V = y->dtype == YDBL_F16 ? 8 : 4;
  const int64_t total = (int64_t)y->n * y->h * y->w * (y->c / V);
  if (y->dtype == YDBL_F16)
    pool_up_concat_kernel<_Float16><<<nblk(total), 256, 0, s>>>(cview<_Float16>(lo), cview<_Float16>(mid),
                                                                 cview<_Float16>(hi), dview<_Float16>(*y));
  else
    pool_up_concat_kernel<float><<<nblk(total), 256, 0, s>>>(cview<float>(lo), cview<float>(mid), cview<float>(hi),
                                                              dview<float>(*y));
  return check_launch("ydbl_pool_up_concat");
}

static int dysample_go(const ydbl_view* x, const ydbl_view* off, int32_t groups, const ydbl_view* y,
                       const ydbl_view* y2, const ydbl_view* r2, float a2, float b2, void* stream) {
  if (check_view(x, "dysample.x", true) || check_view(off, "dysample.off", false) || check_view(y, "dysample.y", true))
    return YDBL_EINVAL;
  const int V = y->dtype == YDBL_F16 ? 8 : 4;
  if (groups < 1 || x->c % groups || (x->c / groups) % V) return fail(YDBL_EINVAL, "dysample: bad groups");
  if (off->c != 8 * groups || off->h != x->h || off->w != x->w || y->h != 2 * x->h || y->w != 2 * x->w ||
      y->c != x->c || off->dtype != x->dtype || y->dtype != x->dtype)
    return fail(YDBL_EINVAL, "dysample: shape mismatch");
  const bool two = y2 && y2->ptr;
  if (two) {
    if (check_view(y2, "dysample.y2", true) || check_view(r2, "dysample.r2", true)) return YDBL_EINVAL;
    auto same = [&](const ydbl_view* v) {
      return v->n == y->n && v->h == y->h && v->w == y->w && v->c == y->c && v->dtype == y->dtype;
    };
    if (!same(y2) || !same(r2)) return fail(YDBL_EINVAL, "dysample: y2/r2 must match y");
  }
  hipStream_t s = as_stream(stream);
  const int64_t total = (int64_t)y->n * y->h * y->w * groups * (x->c / groups / V);
  if (y->dtype == YDBL_F16)
    dysample_kernel<_Float16><<<nblk(total), 256, 0, s>>>(
        cview<_Float16>(x), cview<_Float16>(off), groups, dview<_Float16>(*y),
        two ? dview<_Float16>(*y2) : DView<_Float16>{nullptr, 0, 0, 0, 0, 0}, cview<_Float16>(two ? r2 : nullptr), a2, b2);
  else
    dysample_kernel<float><<<nblk(total), 256, 0, s>>>(
        cview<float>(x), cview<float>(off), groups, dview<float>(*y),
        two ? dview<float>(*y2) : DView<float>{nullptr, 0, 0, 0, 0, 0}, cview<float>(two ? r2 : nullptr), a2, b2);
  return check_launch("ydbl_dysample");
}

extern "C" int ydbl_dysample(const ydbl_view* x, const ydbl_view* off, int32_t groups, const ydbl_view* y,
                             void* stream) {
  return dysample_go(x, off, groups, y, nullptr, nullptr, 0.f, 0.f, stream);
}

extern "C" int ydbl_dysample_ex(const ydbl_dysample_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "dysample: null descriptor");
  return dysample_go(&d->x, &d->off, d->groups, &d->y, &d->y2, &d->r2, d->a2, d->b2, stream);
}

extern "C" int64_t ydbl_lsk_gate_workspace(int32_t n, int32_t h, int32_t w) { return (int64_t)n * h * w * 2 * 4; }

extern "C" int ydbl_lsk_gate(const ydbl_view* attn, const float* sw, const float* sb, const ydbl_view* out,
                             void* workspace, void* stream) {
  if (check_view(attn, "lsk.attn", true) || check_view(out, "lsk.out", true)) return YDBL_EINVAL;
  if (attn->c != 2 * out->c || attn->n != out->n || attn->h != out->h || attn->w != out->w ||
      attn->dtype != out->dtype)
    return fail(YDBL_EINVAL, "lsk: shape mismatch");
  if (!sw || !sb || !workspace) return fail(YDBL_EINVAL, "lsk: null weights/workspace");
  hipStream_t s = as_stream(stream);
  float* agg = reinterpret_cast<float*>(workspace);
  const int64_t npix = (int64_t)out->n * out->h * out->w;
  const int V = out->dtype == YDBL_F16 ? 8 : 4;
  if (out->dtype == YDBL_F16) {
    lsk_stats_kernel<_Float16><<<nblk(npix * 32), 256, 0, s>>>(cview<_Float16>(attn), agg);
    lsk_gate_kernel<_Float16><<<nblk(npix * (out->c / V)), 256, 0, s>>>(cview<_Float16>(attn), agg, sw, sb,
                                                                         dview<_Float16>(*out));
  } else {
    lsk_stats_kernel<float><<<nblk(npix * 32), 256, 0, s>>>(cview<float>(attn), agg);
    lsk_gate_kernel<float><<<nblk(npix * (out->c / V)), 256, 0, s>>>(cview<float>(attn), agg, sw, sb,
                                                                      dview<float>(*out));
  }
  return check_launch("ydbl_lsk_gate");
}
