// DSConv fused into one kernel (U/nn/modules/conv.py:91-108: SiLU(BN(pw1x1(dw_kxk(x))))), BN
// folded into the pointwise weights.  The depthwise output never touches HBM.
//
// A workgroup owns a TH x TW output tile and NTN*16 output channels.  For each chunk of
// CC = 4*VEC input channels (= one MFMA k-step of the pointwise):
//   1. the chunk's input halo tile and depthwise taps sit in LDS as fp32 (converted once per
//      element at staging; the next chunk's halo is loaded into registers before this chunk's
//      arithmetic and stored after it, into a second buffer or the refilled single one),
//   2. depthwise phase: a thread owns CSEG consecutive outputs of one row and one fp32 quad of
//      channels; it slides a (CSEG-1)*S + K register window along each input row, so every LDS
//      element it reads feeds up to K outputs (fp32 accumulate in the reference's (ky, kx) tap
//      order; padded taps read staged zeros, fma(0, w, a) == a), rounds to the activation dtype
//      (the reference's fp16 dw output) and writes the MFMA B tile [TH*TW px][CC],
//   3. pointwise phase: wave w multiplies its 16-pixel tiles w, w+4, ... by the chunk's
//      pointwise weights (A fragments loaded from the L2-resident [Cout][KPAD] matrix at the top
//      of the chunk) into NTN x TMW 16x16 accumulators.
// Fused epilogue (bias, SiLU, residual add of DSBottleneck, channel-slice store) as conv.hip.
#include "conv_common.hpp"

namespace ydbl {

template <int R>
__device__ __forceinline__ int bswz(int row, int kv) {  // B-tile slot: 16 consecutive rows -> distinct banks
  return row * 4 + (kv ^ (((row >> 2) & 1) << 1));
}

// 4 consecutive activation-dtype channels from 4 fp32 values (8 B f16 / 16 B f32).
__device__ __forceinline__ void store4(_Float16* d, const float* a) { *reinterpret_cast<h4*>(d) = to_h4_rne(a); }
__device__ __forceinline__ void store4(float* d, const float* a) {
  *reinterpret_cast<f32x4*>(d) = f32x4{a[0], a[1], a[2], a[3]};
}

template <typename T, int K, int S, int DIL, int TH, int TW, int CSEG, int NTN, bool DBUF>
__global__ __launch_bounds__(256, 2) void dsconv_kernel(ConvArgs<T> p, const float* __restrict__ dww,
                                                        const float* __restrict__ dwb, int dw_act, int tiles_x,
                                                        int tiles_y, int co_splits) {
  constexpr int VEC = Vec<T>::N;
  constexpr int CC = 4 * VEC;    // channels per chunk (one pointwise MFMA k-step)
  constexpr int NQ = CC / 4;     // fp32 quads per staged pixel
  constexpr int QV = VEC / 4;    // quads per 16-byte activation vector
  constexpr int IH = (TH - 1) * S + (K - 1) * DIL + 1, IW = (TW - 1) * S + (K - 1) * DIL + 1;
  constexpr int IWP = IW | 1;    // odd row pitch: the rows of a half-wave hit distinct bank quarters
  constexpr int NSEG = TW / CSEG;
  static_assert(TW % CSEG == 0, "segments");
  constexpr int NTASK = NQ * TH * NSEG;  // (quad, row, segment), quad fastest
  constexpr int SEGW = (CSEG - 1) * S + (K - 1) * DIL + 1;
  constexpr int HALO = IH * IW * 4;      // 16-byte activation vectors to stage per chunk
  constexpr int HIT = (HALO + 255) / 256;
  constexpr int NT = TH * TW / 16;       // 16-pixel MFMA tiles
  static_assert(TH * TW % 16 == 0, "tile");
  constexpr int TMW = (NT + 3) / 4;
  using vec = typename Vec<T>::type;
  // the halo and the taps are staged as fp32 (converted once per element, not once per tap use)
  constexpr int NB = DBUF ? 2 : 1;  // double-buffered halo, or one buffer refilled between barriers
  __shared__ f32x4 s_x[NB][IH * IWP * NQ];
  __shared__ f32x4 s_w[NB][K * K * NQ];
  __shared__ vec s_b[TH * TW * 4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = p.N * tiles_y * tiles_x;
  int bid = xcd_remap(blockIdx.x, ntiles * co_splits);
  const int cs = bid % co_splits;
  bid /= co_splits;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - p.PAD, ix0 = ox0 * S - p.PAD;
  const int co0 = cs * NTN * 16;
  __shared__ __align__(16) float s_bias[NTN * 16];
  BiasStage<NTN * 16> bst;
  bst.fetch(p.bias, co0, p.Cout);

  constexpr int TAPV = K * K * NQ;  // fp32 tap quads per chunk (392 for k7 f16: > one per thread)
  constexpr int TIT = (TAPV + 255) / 256;
  // raw loads now, zero selects / tap rounding at the LDS store: the next chunk's loads stay in flight through
  // this chunk's depthwise and pointwise phases (a select or conversion next to its load waits for it there)
  vec xr[HIT];
  bool xok[HIT];
  f32x4 wr[TIT];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = min(tid + it * 256, HALO - 1);
      const int cv = i & 3, px = i >> 2;
      const int hy = px / IW, hx = px - hy * IW;
      const int iy = iy0 + hy, ix = ix0 + hx;
      xok[it] = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      xr[it] = vload_clamped(p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + c0 + cv * VEC, p.x, xok[it]);
    }
#pragma unroll
    for (int it = 0; it < TIT; ++it) {
      const int i = min(tid + it * 256, TAPV - 1);
      const int tap = i / NQ, q = i % NQ;
      wr[it] = *reinterpret_cast<const f32x4*>(dww + tap * p.Cin + c0 + q * 4);
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = tid + it * 256;
      if (i < HALO) {
        const int cv = i & 3, px = i >> 2;
        const int hy = px / IW, hx = px - hy * IW;
        f32x4* d = &s_x[buf][(hy * IWP + hx) * NQ + cv * QV];
        const vec xv = vsel(xr[it], xok[it]);
#pragma unroll
        for (int u = 0; u < QV; ++u)
          d[u] = f32x4{float(xv[4 * u]), float(xv[4 * u + 1]), float(xv[4 * u + 2]), float(xv[4 * u + 3])};
      }
    }
#pragma unroll
    for (int it = 0; it < TIT; ++it)  // taps rounded to the activation dtype (the reference's .half() weights)
      if (tid + it * 256 < TAPV)
        s_w[buf][tid + it * 256] = f32x4{float(T(wr[it][0])), float(T(wr[it][1])), float(T(wr[it][2])), float(T(wr[it][3]))};
  };

  f32x4 acc[NTN][TMW];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < TMW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.Cin / CC;
  load_chunk(0);
  store_chunk(0);
  bst.commit(s_bias);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = DBUF ? (ch & 1) : 0;
    const int c0 = ch * CC;
    // this chunk's pointwise A fragments first (loads complete in order: waiting for them later does not wait
    // for the next chunk's), zero rows past Cout selected at the MFMAs
    vec af[NTN];
#pragma unroll
    for (int i = 0; i < NTN; ++i) {
      const int co = co0 + i * 16 + r16;
      af[i] = vload_clamped(p.w + (int64_t)co * p.KPAD + c0 + g * VEC, p.w, co < p.Cout);
    }
    if (ch + 1 < nchunks) load_chunk(c0 + CC);
    // ---- depthwise phase
    for (int task = tid; task < NTASK; task += 256) {
      const int q = task % NQ;
      const int r = (task / NQ) % TH;
      const int sg = task / (NQ * TH);
      float a[CSEG][4];
#pragma unroll
      for (int c = 0; c < CSEG; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[c][e] = 0.f;
#pragma unroll 1
      for (int ky = 0; ky < K; ++ky) {  // rolled: one input row's window + taps live at a time
        const f32x4* xrow = &s_x[buf][((r * S + ky * DIL) * IWP + sg * CSEG * S) * NQ + q];
        f32x4 xs[SEGW], wv[K];
#pragma unroll
        for (int i = 0; i < SEGW; ++i) xs[i] = xrow[i * NQ];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) wv[kx] = s_w[buf][(ky * K + kx) * NQ + q];
#pragma unroll
        for (int kx = 0; kx < K; ++kx)
#pragma unroll
          for (int c = 0; c < CSEG; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c * S + kx * DIL][e], wv[kx][e], a[c][e]);
      }
      if (dwb) {  // uniform: DWConv (+ folded BN) bias and activation before the pointwise
        const f32x4 bq = *reinterpret_cast<const f32x4*>(dwb + c0 + q * 4);
#pragma unroll
        for (int c = 0; c < CSEG; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) a[c][e] = apply_act<T>(a[c][e] + bq[e], dw_act);
      }
#pragma unroll
      for (int c = 0; c < CSEG; ++c) {
        const int px = r * TW + sg * CSEG + c;
        store4(reinterpret_cast<T*>(&s_b[bswz<0>(px, q / QV)]) + (q % QV) * 4, a[c]);
      }
    }
    __syncthreads();
    // ---- pointwise phase
#pragma unroll
    for (int j = 0; j < TMW; ++j) {
      const int t = wave + 4 * j;
      if (t < NT) {
        const vec bf = s_b[bswz<0>(t * 16 + r16, g)];
#pragma unroll
        for (int i = 0; i < NTN; ++i) acc[i][j] = mfma_chunk<T>(vsel(af[i], co0 + i * 16 + r16 < p.Cout), bf, acc[i][j]);
      }
    }
    if constexpr (DBUF) {
      if (ch + 1 < nchunks) store_chunk(buf ^ 1);
    } else {
      if (ch + 1 < nchunks) {
        __syncthreads();  // every wave is past this chunk's depthwise reads
        store_chunk(0);
      }
    }
    __syncthreads();
  }

  int64_t pp[TMW];
  bool pv[TMW];
#pragma unroll
  for (int j = 0; j < TMW; ++j) {
    const int t = wave + 4 * j;
    const int op = t * 16 + r16;
    const int oy = oy0 + op / TW, ox = ox0 + op % TW;
    pv[j] = t < NT && oy < p.Ho && ox < p.Wo;
    pp[j] = ((int64_t)b * p.Ho + oy) * p.Wo + ox;
  }
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = co0 + i * 16 + 4 * g;
  conv_epilogue<T, NTN, TMW>(p, acc, pp, pv, co, s_bias, co0);
  if constexpr (NTN == 4) {  // the tail is only launched with Cout 64 = NTN * 16 (host-checked)
    if (p.t3w) conv_tail_1x1<T, NTN, TMW>(p, acc, pp, pv, co, g);
  }
}

template <typename T, int K, int S, int DIL, int TH, int TW, int CSEG, bool DBUF = true>
static void launch_ds_tile(const ConvArgs<T>& a, const float* dww, const float* dwb, int dw_act, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, TW), tiles_y = (int)cdiv(a.Ho, TH);
  const int64_t ntiles = (int64_t)a.N * tiles_y * tiles_x;
  auto go = [&](auto kern, int ntn) {
    const int cs = (int)cdiv(a.Cout, ntn * 16);
    kern<<<(unsigned)(ntiles * cs), 256, 0, s>>>(a, dww, dwb, dw_act, tiles_x, tiles_y, cs);
  };
  if (a.Cout <= 32) go(dsconv_kernel<T, K, S, DIL, TH, TW, CSEG, 2, DBUF>, 2);
  // k3 s1 with < 512 tiles: two 64-channel column workgroups per tile (the cheap depthwise phase is
  // recomputed; 128->128 @20^2 bs32 15.0 -> 11.8 us; k7 loses: 19.7 -> 25.4)
  else if (a.Cout <= 64 || ntiles < 256 || (K == 3 && S == 1 && ntiles < 512))
    go(dsconv_kernel<T, K, S, DIL, TH, TW, CSEG, 4, DBUF>, 4);
  else go(dsconv_kernel<T, K, S, DIL, TH, TW, CSEG, 8, DBUF>, 8);
}

// Tile shape (measured on the DBL-n/s shapes, fp16 bs 32): maps wider than 20 px take a 16x8 tile
// with 4-output row segments and one refilled LDS buffer (small footprint: 3-4 workgroups per CU
// hide each other's halo loads; 40^2 k7 64ch 25.8 -> 15.1 us); 20-px and smaller maps take an 8x8
// double-buffered tile (more workgroups on the few pixels).
template <typename T, int K, int S, int DIL>
static int launch_ds(const ConvArgs<T>& a, const float* dww, const float* dwb, int dw_act, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    if (try_dsc_lean(a, dww, dwb, dw_act, K, S, DIL, s)) return check_launch("ydbl_dsconv_nhwc");
  }
  // Fewer than 400 16x8 tiles (the bench's bs16 sub-batch graphs at 40^2: 240): 8x8 single-buffered
  // tiles, 1.7x the workgroups (DBL-n bs32 on two streams 13.98 k -> 14.45 k img/s; at bs32 / 480 tiles
  // the two are even, and the 16x8 tile stays ahead on DBL-s bs64 and DBL-l 1280)
  const int64_t t168 = (int64_t)a.N * cdiv(a.Ho, 16) * cdiv(a.Wo, 8);
  if (a.Wo > 20 && t168 < 400) launch_ds_tile<T, K, S, DIL, 8, 8, 2, false>(a, dww, dwb, dw_act, s);
  else if (a.Wo > 20) launch_ds_tile<T, K, S, DIL, 16, 8, 4, false>(a, dww, dwb, dw_act, s);
  else launch_ds_tile<T, K, S, DIL, 8, 8, 2, true>(a, dww, dwb, dw_act, s);
  return check_launch("ydbl_dsconv_nhwc");
}

template <typename T>
static ConvArgs<T> ds_args(const ydbl_dsconv_desc* d) {
  ConvArgs<T> a{};
  a.x = reinterpret_cast<const T*>(d->x.ptr);
  a.xcs = d->x.cs; a.N = d->x.n; a.H = d->x.h; a.W = d->x.w; a.Cin = d->x.c;
  a.y = reinterpret_cast<T*>(d->y.ptr);
  a.ycs = d->y.cs; a.Ho = d->y.h; a.Wo = d->y.w; a.Cout = d->y.c;
  a.r = reinterpret_cast<const T*>(d->r.ptr); a.rcs = d->r.cs;
  a.w = reinterpret_cast<const T*>(d->pw_w); a.bias = d->bias;
  a.KW = d->k; a.S = d->stride; a.PAD = d->pad; a.DIL = d->dil;
  a.K = d->x.c; a.KPAD = d->kpad;
  a.act = d->act; a.res = d->res_mode;
  if (d->tail_w) {
    a.t3w = d->tail_w; a.t3b = d->tail_b; a.nt3 = d->tail_n;
    a.y3 = reinterpret_cast<T*>(d->tail_y.ptr); a.y3cs = d->tail_y.cs;
  }
  a.P = d->y.n * d->y.h * d->y.w;
  if (d->g2_w) {
    a.g2w = reinterpret_cast<const T*>(d->g2_w); a.g2b = d->g2_b;
    a.g2x = reinterpret_cast<const T*>(d->g2_x.ptr); a.g2xcs = d->g2_x.cs;
    a.g2y = reinterpret_cast<T*>(d->g2_y.ptr); a.g2ycs = d->g2_y.cs; a.g2act = d->g2_act;
  }
  if (d->g0_w) {
    a.g0w = reinterpret_cast<const T*>(d->g0_w); a.g0b = d->g0_b;
    a.g0x = reinterpret_cast<const T*>(d->g0_x.ptr); a.g0xcs = d->g0_x.cs;
    a.g0y = reinterpret_cast<T*>(d->g0_y.ptr); a.g0ycs = d->g0_y.cs; a.g0act = d->g0_act;
  }
  return a;
}

ConvArgs<_Float16> ds_args_f16(const ydbl_dsconv_desc* d) { return ds_args<_Float16>(d); }

template <typename T>
static int run_ds(const ydbl_dsconv_desc* d, hipStream_t s) {
  const ConvArgs<T> a = ds_args<T>(d);
  if (d->g2_w) {  // trailing GEMM: only the lean kernel has it (ydbl.h: fp16, k 7 s 1, C 64 / 128)
    if constexpr (sizeof(T) == 2) {
      if (d->k == 7 && d->stride == 1 && d->dil == 1 &&
          try_dsc_lean(a, d->dw_w, d->dw_bias, d->dw_act, 7, 1, 1, s))
        return check_launch("ydbl_dsconv_nhwc");
    }
    return fail(YDBL_EINVAL, "dsconv: the trailing GEMM (g2) needs fp16, k 7 stride 1, C 64 or 128 (lean kernel)");
  }
  if (d->g0_w) {  // leading 1x1: only the lean kernel has it (ydbl.h: fp16, k 3 s 1, C 64, g0_y 128)
    if constexpr (sizeof(T) == 2) {
      if (d->k == 3 && d->stride == 1 && d->dil == 1 &&
          try_dsc_lean(a, d->dw_w, d->dw_bias, d->dw_act, 3, 1, 1, s))
        return check_launch("ydbl_dsconv_nhwc");
    }
    return fail(YDBL_EINVAL, "dsconv: the leading 1x1 (g0) needs fp16, k 3 stride 1, C 64 (lean kernel)");
  }
  if (d->k == 3 && d->stride == 1 && d->dil == 1) return launch_ds<T, 3, 1, 1>(a, d->dw_w, d->dw_bias, d->dw_act, s);
  if (d->k == 3 && d->stride == 2 && d->dil == 1) return launch_ds<T, 3, 2, 1>(a, d->dw_w, d->dw_bias, d->dw_act, s);
  if (d->k == 5 && d->stride == 1 && d->dil == 1) return launch_ds<T, 5, 1, 1>(a, d->dw_w, d->dw_bias, d->dw_act, s);
  if (d->k == 7 && d->stride == 1 && d->dil == 1) return launch_ds<T, 7, 1, 1>(a, d->dw_w, d->dw_bias, d->dw_act, s);
  return fail(YDBL_EINVAL, "dsconv: supported (k, stride, dil): (3,1,1) (3,2,1) (5,1,1) (7,1,1)");
}

// The descriptor rules of ydbl_dsconv_nhwc (include/ydbl.h).
int ds_check(const ydbl_dsconv_desc* d) {
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
  if (d->g2_w) {
    if (!d->g2_b || check_view(&d->g2_x, "dsconv.g2_x", true) || check_view(&d->g2_y, "dsconv.g2_y", false) ||
        d->g2_x.c != d->y.c || d->g2_y.c != d->y.c || d->x.c != d->y.c || d->tail_w || d->g2_x.dtype != d->y.dtype ||
        d->g2_y.dtype != d->y.dtype || d->g2_y.cs % 4 || d->g2_x.n != d->y.n || d->g2_x.h != d->y.h ||
        d->g2_x.w != d->y.w || d->g2_y.n != d->y.n || d->g2_y.h != d->y.h || d->g2_y.w != d->y.w)
      return fail(YDBL_EINVAL, "dsconv: g2 needs g2_x/g2_y of y's shape and dtype, x.c == y.c, no class tail");
  }
  if (d->g0_w) {
    const int es = d->y.dtype == YDBL_F16 ? 2 : 4;
    if (!d->g0_b || check_view(&d->g0_x, "dsconv.g0_x", true) || check_view(&d->g0_y, "dsconv.g0_y", false) ||
        d->g0_x.c != d->x.c || d->g0_y.c != 2 * d->x.c || d->x.c != d->y.c || d->g2_w || d->tail_w ||
        d->g0_x.dtype != d->x.dtype || d->g0_y.dtype != d->x.dtype || d->g0_y.cs % 4 || d->g0_x.cs % 8 ||
        d->res_mode != YDBL_RES_NONE || d->g0_x.n != d->x.n || d->g0_x.h != d->x.h || d->g0_x.w != d->x.w ||
        d->g0_y.n != d->x.n || d->g0_y.h != d->x.h || d->g0_y.w != d->x.w || d->x.cs != d->g0_y.cs ||
        (const char*)d->x.ptr != (const char*)d->g0_y.ptr + (int64_t)d->x.c * es)
      return fail(YDBL_EINVAL, "dsconv: g0 needs g0_x [n,h,w,x.c], g0_y [n,h,w,2 x.c] whose last x.c channels are x, "
                               "x.c == y.c, no residual / tail / g2");
  }
  if (d->tail_w) {
    if (!d->tail_b || d->tail_n < 1 || d->tail_n > 4 || d->y.c != 64 || d->res_mode != YDBL_RES_NONE ||
        check_view(&d->tail_y, "dsconv.tail_y", false) || d->tail_y.c != d->tail_n || d->tail_y.dtype != d->y.dtype ||
        d->tail_y.n != d->y.n || d->tail_y.h != d->y.h || d->tail_y.w != d->y.w)
      return fail(YDBL_EINVAL, "dsconv: tail needs y.c 64, 1 <= tail_n <= 4, tail_y [n,h,w,tail_n] of y's dtype, no residual");
  }
  return YDBL_OK;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dsconv_nhwc(const ydbl_dsconv_desc* d, void* stream) {
  if (const int rc = ds_check(d)) return rc;
  const hipStream_t s = as_stream(stream);
  return d->x.dtype == YDBL_F16 ? run_ds<_Float16>(d, s) : run_ds<float>(d, s);
}
