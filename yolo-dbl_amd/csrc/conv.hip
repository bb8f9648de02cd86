// Dense NHWC convolution as an implicit GEMM on MFMA (gfx950).
//
// GEMM mapping (one wave = NT x MT MFMA tiles of 16x16):
//   rows    = output channels (A operand = weights [cout][kh*kw*cin], K-contiguous)
//   columns = output pixels   (B operand = im2col patches, gathered on the fly, K-contiguous in NHWC)
// The accumulator C/D map (col = lane&15, row = 4*(lane>>4)+r) gives every lane 4 CONSECUTIVE
// output channels of one pixel, so the epilogue stores 8 B (f16) / 16 B (f32) per lane in NHWC.
// Every lane loads 16 B per operand per K-chunk: f16 -> one v_mfma_f32_16x16x32_f16,
// f32 -> four exact-f32 v_mfma_f32_16x16x4_f32 (parity mode; same fmaf-chain numerics as VALU).
// Fused epilogue: + bias, activation (SiLU/GELU/sigmoid), residual add or multiply, write into a
// channel slice of a wider buffer (concat without copies).
#include "common.hpp"

namespace ydbl {

template <typename T>
struct ConvArgs {
  const T* x; int xcs; int N, H, W, Cin;
  T* y; int ycs; int Ho, Wo, Cout;
  const T* r; int rcs;
  const T* w; const float* bias;
  int KW, S, PAD, DIL, K, KPAD;
  int act, res;
  int P;
};

template <typename T>
__device__ __forceinline__ f32x4 mfma_chunk(const typename Vec<T>::type& a, const typename Vec<T>::type& b, f32x4 c);

template <>
__device__ __forceinline__ f32x4 mfma_chunk<_Float16>(const h8& a, const h8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma_chunk<float>(const f32x4& a, const f32x4& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

// POINTWISE: 1x1, stride 1, pad 0 (x is a dense [P][xcs] matrix).
template <typename T, int MT, int NT, bool POINTWISE>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs<T> p) {
  constexpr int VEC = Vec<T>::N;
  constexpr int KCH = 4 * VEC;
  using vec = typename Vec<T>::type;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int r16 = lane & 15;
  const int px0 = (blockIdx.x * 4 + wave) * (MT * 16);
  const int co0 = blockIdx.y * (NT * 16);

  // Per pixel-tile B-operand coordinates for this lane.
  int pb[MT], piy[MT], pix[MT];
  bool pv[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    int pp = px0 + 16 * j + r16;
    pv[j] = pp < p.P;
    pp = pv[j] ? pp : 0;
    int ox = pp % p.Wo;
    int t = pp / p.Wo;
    int oy = t % p.Ho;
    pb[j] = t / p.Ho;
    piy[j] = oy * p.S - p.PAD;
    pix[j] = ox * p.S - p.PAD;
  }
  const T* wrow[NT];
  bool wv[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    int co = co0 + 16 * i + r16;
    wv[i] = co < p.Cout;
    wrow[i] = p.w + (int64_t)(wv[i] ? co : 0) * p.KPAD;
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < p.K; k0 += KCH) {
    const int k = k0 + g * VEC;
    const bool kv = k < p.K;
    vec a[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) a[i] = wv[i] ? vload(wrow[i] + k) : vzero<T>();
    vec b[MT];
    if constexpr (POINTWISE) {
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int64_t pp = px0 + 16 * j + r16;
        b[j] = (pv[j] && kv) ? vload(p.x + pp * p.xcs + k) : vzero<T>();
      }
    } else {
      const int tap = k / p.Cin;
      const int ci = k - tap * p.Cin;
      const int ky = tap / p.KW;
      const int kx = tap - ky * p.KW;
      const int dy = ky * p.DIL, dx = kx * p.DIL;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int iy = piy[j] + dy, ix = pix[j] + dx;
        const bool ok = pv[j] && kv && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        b[j] = ok ? vload(p.x + ((int64_t)(pb[j] * p.H + iy) * p.W + ix) * p.xcs + ci) : vzero<T>();
      }
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = mfma_chunk<T>(a[i], b[j], acc[i][j]);
  }

  // Epilogue: lane owns channels co..co+3 of pixel px0+16j+r16.
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    if (!pv[j]) continue;
    const int64_t pp = px0 + 16 * j + r16;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int co = co0 + 16 * i + 4 * g;
      if (co >= p.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const bool full = co + 4 <= p.Cout;
      if (p.bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += (full || co + q < p.Cout) ? p.bias[co + q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], p.act);
      if (p.res != YDBL_RES_NONE) {
        float rv[4];
        const T* rp = p.r + pp * p.rcs + co;
        if (full) {
          load_f<4>(rp, rv);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) rv[q] = (co + q < p.Cout) ? float(rp[q]) : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (p.res == YDBL_RES_ADD) ? rv[q] + v[q] : rv[q] * v[q];
      }
      T* yp = p.y + pp * p.ycs + co;
      if (full) {
        store_f<4>(yp, v);
      } else {
        for (int q = 0; q < 4 && co + q < p.Cout; ++q) yp[q] = (T)v[q];
      }
    }
  }
}

template <typename T, int MT, int NT>
static void launch_conv(const ConvArgs<T>& a, bool pointwise, hipStream_t s) {
  dim3 grid((unsigned)cdiv(a.P, 4 * MT * 16), (unsigned)cdiv(a.Cout, NT * 16));
  if (pointwise)
    conv_mfma_kernel<T, MT, NT, true><<<grid, 256, 0, s>>>(a);
  else
    conv_mfma_kernel<T, MT, NT, false><<<grid, 256, 0, s>>>(a);
}

template <typename T>
static void dispatch_conv(const ConvArgs<T>& a, bool pointwise, hipStream_t s) {
  // Tile choice: cover Cout with 1/2/4 16-row tiles per wave; shrink the pixel tile until the
  // grid has enough workgroups to fill 256 CUs.
  const int nt = a.Cout <= 16 ? 1 : (a.Cout <= 32 ? 2 : 4);
  auto blocks = [&](int mt) { return cdiv(a.P, 4 * mt * 16) * cdiv(a.Cout, nt * 16); };
  if (nt == 1) {
    if (blocks(8) >= 1024) return launch_conv<T, 8, 1>(a, pointwise, s);
    if (blocks(4) >= 512) return launch_conv<T, 4, 1>(a, pointwise, s);
    return launch_conv<T, 2, 1>(a, pointwise, s);
  }
  if (nt == 2) {
    if (blocks(4) >= 512) return launch_conv<T, 4, 2>(a, pointwise, s);
    return launch_conv<T, 2, 2>(a, pointwise, s);
  }
  if (blocks(4) >= 512) return launch_conv<T, 4, 4>(a, pointwise, s);
  if (blocks(2) >= 512) return launch_conv<T, 2, 4>(a, pointwise, s);
  return launch_conv<T, 1, 4>(a, pointwise, s);
}

template <typename T>
static int run_conv(const ydbl_conv_desc* d, hipStream_t s) {
  ConvArgs<T> a;
  a.x = reinterpret_cast<const T*>(d->x.ptr);
  a.xcs = d->x.cs; a.N = d->x.n; a.H = d->x.h; a.W = d->x.w; a.Cin = d->x.c;
  a.y = reinterpret_cast<T*>(d->y.ptr);
  a.ycs = d->y.cs; a.Ho = d->y.h; a.Wo = d->y.w; a.Cout = d->y.c;
  a.r = reinterpret_cast<const T*>(d->r.ptr); a.rcs = d->r.cs;
  a.w = reinterpret_cast<const T*>(d->w); a.bias = d->bias;
  a.KW = d->kw; a.S = d->stride; a.PAD = d->pad; a.DIL = d->dil;
  a.K = d->kh * d->kw * d->x.c; a.KPAD = d->kpad;
  a.act = d->act; a.res = d->res_mode;
  a.P = d->y.n * d->y.h * d->y.w;
  const bool pw = d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && d->x.h == d->y.h && d->x.w == d->y.w;
  dispatch_conv<T>(a, pw, s);
  return check_launch("ydbl_conv2d_nhwc");
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_conv2d_nhwc(const ydbl_conv_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "conv: null descriptor");
  if (check_view(&d->x, "conv.x", true) || check_view(&d->y, "conv.y", false)) return YDBL_EINVAL;
  if (d->x.dtype != d->y.dtype) return fail(YDBL_EINVAL, "conv: x/y dtype mismatch");
  if (d->x.c % 8) return fail(YDBL_EINVAL, "conv: input channels must be a multiple of 8");
  if (d->x.n != d->y.n) return fail(YDBL_EINVAL, "conv: batch mismatch");
  if (d->kh < 1 || d->kw < 1 || d->stride < 1 || d->dil < 1 || d->pad < 0)
    return fail(YDBL_EINVAL, "conv: bad kernel geometry");
  const int ho = (d->x.h + 2 * d->pad - d->dil * (d->kh - 1) - 1) / d->stride + 1;
  const int wo = (d->x.w + 2 * d->pad - d->dil * (d->kw - 1) - 1) / d->stride + 1;
  if (ho != d->y.h || wo != d->y.w) return fail(YDBL_EINVAL, "conv: output spatial size mismatch");
  const int K = d->kh * d->kw * d->x.c;
  if (d->kpad < K || d->kpad % 32) return fail(YDBL_EINVAL, "conv: kpad must be >= K and a multiple of 32");
  if (!d->w) return fail(YDBL_EINVAL, "conv: null weights");
  if (d->y.cs % 4) return fail(YDBL_EINVAL, "conv: output channel stride must be a multiple of 4");
  if (d->res_mode != YDBL_RES_NONE) {
    if (check_view(&d->r, "conv.r", false)) return YDBL_EINVAL;
    if (d->r.cs % 4 || d->r.dtype != d->y.dtype) return fail(YDBL_EINVAL, "conv: residual stride/dtype");
    if (d->r.n != d->y.n || d->r.h != d->y.h || d->r.w != d->y.w || d->r.c < d->y.c)
      return fail(YDBL_EINVAL, "conv: residual shape mismatch");
  }
  const hipStream_t s = as_stream(stream);
  return d->x.dtype == YDBL_F16 ? run_conv<_Float16>(d, s) : run_conv<float>(d, s);
}
