// DSConv fused into one kernel (U/nn/modules/conv.py:91-108: SiLU(BN(pw1x1(dw_kxk(x))))), BN
// folded into the pointwise weights.  The depthwise output never touches HBM:
//   for each 4-vector channel chunk of Cin (32 f16 / 16 f32 = one MFMA k-step of the pointwise):
//     1. stage the chunk's input halo tile and depthwise taps in LDS,
//     2. 256 threads = 64 tile pixels x 4 channel vectors compute the depthwise outputs (fp32
//        accumulate in the reference's tap order, padded taps skipped), round to the activation
//        dtype (the reference's fp16 dw output) and write them as the MFMA B tile [64 px][k],
//     3. wave w multiplies its 16 pixels by the chunk's pointwise weights (A fragments straight
//        from the L2-resident [Cout][KPAD] matrix) into NTN 16x16 accumulators.
// Fused epilogue (bias, SiLU, residual add of DSBottleneck, channel-slice store) as conv.hip.
#include "conv_common.hpp"

namespace ydbl {

template <typename T, int K, int S, int DIL, int NTN>
__global__ __launch_bounds__(256) void dsconv_kernel(ConvArgs<T> p, const float* __restrict__ dww, int tiles_x,
                                                     int tiles_y) {
  constexpr int VEC = Vec<T>::N;
  constexpr int CC = 4 * VEC;  // channels per chunk = one MFMA k-step
  constexpr int TH = 8, TW = 8;
  constexpr int IH = (TH - 1) * S + (K - 1) * DIL + 1, IW = (TW - 1) * S + (K - 1) * DIL + 1;
  constexpr int HALO = IH * IW * 4;  // vectors
  constexpr int HIT = (HALO + 255) / 256;
  using vec = typename Vec<T>::type;
  __shared__ vec s_halo[HALO];
  __shared__ vec s_w[K * K * 4];  // taps in the activation dtype (the reference's .half() weights)
  __shared__ vec s_b[64 * 4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - p.PAD, ix0 = ox0 * S - p.PAD;
  const int co0 = blockIdx.y * NTN * 16;

  // dw-phase role: pixel dpx of the tile, channel vector dcv of the chunk
  const int dpx = tid >> 2, dcv = tid & 3;
  const int dpy = dpx / TW, dpxx = dpx % TW;
  const int doy = oy0 + dpy, dox = ox0 + dpxx;

  f32x4 acc[NTN][1];
#pragma unroll
  for (int i = 0; i < NTN; ++i) acc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.Cin / CC;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = ch * CC;
    {  // 1. stage halo (all loads in flight, then stores) and the chunk's depthwise taps
      vec t[HIT];
#pragma unroll
      for (int it = 0; it < HIT; ++it) {
        const int i = min(tid + it * 256, HALO - 1);
        const int cv = i & 3, px = i >> 2;
        const int iy = iy0 + px / IW, ix = ix0 + px % IW;
        const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        t[it] = vload_sel(p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + c0 + cv * VEC, p.x, ok);
      }
      for (int i = tid; i < K * K * 4; i += 256) {
        const int tap = i >> 2, q = i & 3;
        float wf[VEC];
        load_f<VEC>(dww + tap * p.Cin + c0 + q * VEC, wf);
        vec wv;
#pragma unroll
        for (int e = 0; e < VEC; ++e) wv[e] = T(wf[e]);
        s_w[i] = wv;
      }
#pragma unroll
      for (int it = 0; it < HIT; ++it) {
        const int i = tid + it * 256;
        if (i < HALO) s_halo[i] = t[it];
      }
    }
    __syncthreads();
    {  // 2. depthwise outputs of this chunk -> B tile
      float a[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) a[q] = 0.f;
#pragma unroll 1
      for (int ky = 0; ky < K; ++ky) {
        const int iy = doy * S - p.PAD + ky * DIL;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int ix = dox * S - p.PAD + kx * DIL;
          if (iy < 0 || iy >= p.H || ix < 0 || ix >= p.W) continue;
          const vec xv = s_halo[((dpy * S + ky * DIL) * IW + dpxx * S + kx * DIL) * 4 + dcv];
          const vec wv = s_w[(ky * K + kx) * 4 + dcv];
#pragma unroll
          for (int q = 0; q < VEC; ++q) a[q] = fmaf(float(xv[q]), float(wv[q]), a[q]);  // fp32 accumulate
        }
      }
      vec o;
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = T(a[q]);
      s_b[dpx * 4 + (dcv ^ (((dpx >> 2) & 1) << 1))] = o;
    }
    __syncthreads();
    {  // 3. pointwise MFMA: wave's 16 pixels x NTN*16 output channels, one k-step
      const int row = wave * 16 + r16;
      const vec bf = s_b[row * 4 + (g ^ (((row >> 2) & 1) << 1))];
#pragma unroll
      for (int i = 0; i < NTN; ++i) {
        const int co = co0 + i * 16 + r16;
        const vec af = vload_sel(p.w + (int64_t)co * p.KPAD + c0 + g * VEC, p.w, co < p.Cout);
        acc[i][0] = mfma_chunk<T>(af, bf, acc[i][0]);
      }
    }
    __syncthreads();
  }
  const int op = wave * 16 + r16;
  const int oy = oy0 + op / TW, ox = ox0 + op % TW;
  const bool pv[1] = {oy < p.Ho && ox < p.Wo};
  const int64_t pp[1] = {((int64_t)b * p.Ho + oy) * p.Wo + ox};
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = co0 + i * 16 + 4 * g;
  conv_epilogue<T, NTN, 1>(p, acc, pp, pv, co);
}

template <typename T, int K, int S, int DIL>
static int launch_ds(const ConvArgs<T>& a, const float* dww, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, 8), tiles_y = (int)cdiv(a.Ho, 8);
  const unsigned gx = (unsigned)(a.N * tiles_y * tiles_x);
  if (a.Cout <= 32) {
    dsconv_kernel<T, K, S, DIL, 2><<<dim3(gx, 1), 256, 0, s>>>(a, dww, tiles_x, tiles_y);
  } else {
    dsconv_kernel<T, K, S, DIL, 4><<<dim3(gx, (unsigned)cdiv(a.Cout, 64)), 256, 0, s>>>(a, dww, tiles_x, tiles_y);
  }
  return check_launch("ydbl_dsconv_nhwc");
}

template <typename T>
static int run_ds(const ydbl_dsconv_desc* d, hipStream_t s) {
  ConvArgs<T> a;
  a.x = reinterpret_cast<const T*>(d->x.ptr);
  a.xcs = d->x.cs; a.N = d->x.n; a.H = d->x.h; a.W = d->x.w; a.Cin = d->x.c;
  a.y = reinterpret_cast<T*>(d->y.ptr);
  a.ycs = d->y.cs; a.Ho = d->y.h; a.Wo = d->y.w; a.Cout = d->y.c;
  a.r = reinterpret_cast<const T*>(d->r.ptr); a.rcs = d->r.cs;
  a.w = reinterpret_cast<const T*>(d->pw_w); a.bias = d->bias;
  a.KW = d->k; a.S = d->stride; a.PAD = d->pad; a.DIL = d->dil;
  a.K = d->x.c; a.KPAD = d->kpad;
  a.act = d->act; a.res = d->res_mode;
  a.P = d->y.n * d->y.h * d->y.w;
  if (d->k == 3 && d->stride == 1 && d->dil == 1) return launch_ds<T, 3, 1, 1>(a, d->dw_w, s);
  if (d->k == 3 && d->stride == 2 && d->dil == 1) return launch_ds<T, 3, 2, 1>(a, d->dw_w, s);
  if (d->k == 5 && d->stride == 1 && d->dil == 1) return launch_ds<T, 5, 1, 1>(a, d->dw_w, s);
  if (d->k == 7 && d->stride == 1 && d->dil == 1) return launch_ds<T, 7, 1, 1>(a, d->dw_w, s);
  return fail(YDBL_EINVAL, "dsconv: supported (k, stride, dil): (3,1,1) (3,2,1) (5,1,1) (7,1,1)");
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dsconv_nhwc(const ydbl_dsconv_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "dsconv: null descriptor");
  if (check_view(&d->x, "dsconv.x", true) || check_view(&d->y, "dsconv.y", false)) return YDBL_EINVAL;
  if (d->x.dtype != d->y.dtype || d->x.n != d->y.n) return fail(YDBL_EINVAL, "dsconv: x/y mismatch");
  const int cc = d->x.dtype == YDBL_F16 ? 32 : 16;
  if (d->x.c % cc) return fail(YDBL_EINVAL, "dsconv: Cin must be a multiple of 32 (f16) / 16 (f32)");
  const int ho = (d->x.h + 2 * d->pad - d->dil * (d->k - 1) - 1) / d->stride + 1;
  const int wo = (d->x.w + 2 * d->pad - d->dil * (d->k - 1) - 1) / d->stride + 1;
  if (ho != d->y.h || wo != d->y.w) return fail(YDBL_EINVAL, "dsconv: output spatial size mismatch");
  if (!d->dw_w || !d->pw_w) return fail(YDBL_EINVAL, "dsconv: null weights");
  if (d->kpad < d->x.c || d->kpad % 32) return fail(YDBL_EINVAL, "dsconv: kpad must be >= Cin and a multiple of 32");
  if (d->y.cs % 4) return fail(YDBL_EINVAL, "dsconv: output channel stride must be a multiple of 4");
  if (d->res_mode != YDBL_RES_NONE) {
    if (check_view(&d->r, "dsconv.r", false)) return YDBL_EINVAL;
    if (d->r.cs % 4 || d->r.dtype != d->y.dtype || d->r.n != d->y.n || d->r.h != d->y.h || d->r.w != d->y.w ||
        d->r.c < d->y.c)
      return fail(YDBL_EINVAL, "dsconv: residual shape mismatch");
  }
  const hipStream_t s = as_stream(stream);
  return d->x.dtype == YDBL_F16 ? run_ds<_Float16>(d, s) : run_ds<float>(d, s);
}
