// DSBottleneck (U/nn/modules/block.py:1408-1444: y = x + DSConv_k7(DSConv_k3(x)), DSConv = SiLU(BN(pw1x1(dw(x)))),
// conv.py:91-108) in ONE launch, 64 or 128 channels, fp16 -- the two DSConvs of DSC3k2's blocks (block.py:1447-1580;
// DBL-n's 40^2 maps at 64, DBL-s's 40^2 / DBL-n's 20^2 at 128), which dsc_lean.hip runs as two launches with the
// intermediate going through HBM.
//
// A workgroup owns an 8x8 output tile and keeps the whole bottleneck in LDS, recomputing the k7 stage's 3-px halo of
// the intermediate (k3 over 14x14 pixels for 8x8 outputs: 1.3x the depthwise work of the two launches, not the 4x of
// a whole-DSC3k chain):
//   1. one round trip: the 16x16 input halo (all 64 channels, fp16) -> LDS, both stages' fp32 taps -> LDS, the k3
//      pointwise A fragments -> VGPRs (PRE: instead of the halo, the leading 1x1's operands: its B fragments straight
//      from global, 16 input pixels per halo row, and its A fragments; TG: the trailing GEMM's second input tile);
//   PRE. C3's merged cv2 | cv1 1x1 (ydbl_dsconv_desc.g0) on MFMA: the cv1 half over the 16x16 halo into LDS (zero
//      outside the image: the k3 padding), both halves written to g0_y at the output pixels as the unfused launch does;
//   2. k3 depthwise over the 14x14 intermediate region (the reference's (ky, kx) fp32 FMA order, rounded to fp16) into
//      the pointwise B tile; the residual (the bottleneck's input at the 64 output pixels) read from the halo;
//   3. k3 pointwise on MFMA, bias, SiLU, rounded; zero outside the image (the k7 padding); written over the B tile it
//      was computed from after a barrier -> the k7 stage's input in LDS;
//   4. k7 depthwise over the 8x8 outputs into a B tile in the halo's place;
//   5. k7 pointwise on MFMA, bias, SiLU, + residual -> y (or, TG, the trailing GEMM's B tile);
//   TG. C3's cv3 over [y ; g2_x] (ydbl_dsconv_desc.g2) -> g2_y.
// 77 KB of LDS at 64 channels (4 waves): two workgroups per CU; 151 KB at 128 (8 waves): one.  Every rounding point and accumulation order is dsc_lean.hip's, so the outputs
// are bit-identical to the two ydbl_dsconv_nhwc launches it replaces (tests/test_gpu_ops.py::test_dsb_pair_bit_identical).
#include <stdlib.h>

#include "dsc_lean.hpp"

namespace ydbl {

template <int C_>
struct DsbGeo {
  static constexpr int C = C_, NQ = C / 4, CV = C / 8, NKS = C / 32;
  static constexpr int WAVES = C / 16, NT = 64 * WAVES;            // 4 waves at 64 channels, 8 at 128
  static constexpr int TH = 8, TW = 8, NPX = TH * TW, NTP = NPX / 16;  // output tile
  static constexpr int XH = TH + 8, XW = TW + 8, XP = XW + 1;      // k3 input region (halo 4), odd pitch
  static constexpr int RH = TH + 6, RW = TW + 6, RP = RW + 1;      // k3 output = k7 input region (halo 3)
  static constexpr int NR = RH * RW, NRP = (NR + 15) / 16 * 16, NRT = NRP / 16;
  static constexpr int OX = 0;                                     // h4 [XH][XP][NQ]; later the k7 B tile + TG tile
  static constexpr int OS = OX + XH * XP * NQ * 8;                 // k3 B tile h8 [NKS][NRP][4], then h4 [RH][RP][NQ]
  static constexpr int SB = RH * RP * NQ * 8 > NKS * NRP * 4 * 16 ? RH * RP * NQ * 8 : NKS * NRP * 4 * 16;
  static constexpr int OW3 = OS + SB;                              // f32x4 [9][NQ]
  static constexpr int OW7 = OW3 + 9 * NQ * 16;                    // f32x4 [49][NQ]
  static constexpr int OB = OW7 + 49 * NQ * 16;                    // f32 [3][C]: k3 pw, k7 pw, TG biases
  static constexpr int BYTES = OB + 3 * C * 4;
  static_assert(C == 64 ? BYTES <= 80 * 1024 : BYTES <= 160 * 1024, "two workgroups per CU at 64 channels, one at 128");
  static_assert(3 * NKS * NPX * 4 * 16 <= XH * XP * NQ * 8, "k7 B tile + TG tile inside the halo");
  static_assert(NQ * TH * 2 == NT, "k7 depthwise tasks");
};

template <int C_, bool PRE, bool TG>
__global__ __launch_bounds__(DsbGeo<C_>::NT, C_ == 64 ? 2 : 1) void dsb_pair_kernel(
    ConvArgs<_Float16> p1, ConvArgs<_Float16> p2, const float* __restrict__ dw1, const float* __restrict__ dw2,
    int tiles_x, int tiles_y, int ntiles) {
  using G = DsbGeo<C_>;
  constexpr int C = G::C, NQ = G::NQ, CV = G::CV, NKS = G::NKS, NT = G::NT;
  constexpr int TH = G::TH, TW = G::TW, NPX = G::NPX;
  constexpr int XH = G::XH, XW = G::XW, XP = G::XP, RH = G::RH, RW = G::RW, RP = G::RP;
  constexpr int NR = G::NR, NRP = G::NRP, NRT = G::NRT;
  constexpr int OX = G::OX, OS = G::OS, OW3 = G::OW3, OW7 = G::OW7, OB = G::OB, BYTES = G::BYTES;
  static_assert(!PRE || C == 64, "the leading 1x1 is built for 64 channels");
  using T = _Float16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[BYTES];
  h4* s_x = reinterpret_cast<h4*>(smem + OX);
  h8* s_b3 = reinterpret_cast<h8*>(smem + OS);
  h4* s_t = reinterpret_cast<h4*>(smem + OS);
  h8* s_b7 = reinterpret_cast<h8*>(smem + OX);
  h8* s_g = reinterpret_cast<h8*>(smem + OX + NKS * NPX * 4 * 16);
  f32x4* s_w3 = reinterpret_cast<f32x4*>(smem + OW3);
  f32x4* s_w7 = reinterpret_cast<f32x4*>(smem + OW7);
  float* s_bias = reinterpret_cast<float*>(smem + OB);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int t = xcd_remap(blockIdx.x, ntiles);
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int b = t / tiles_y;
  const int H = p1.H, W = p1.W;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int xy0 = oy0 - 4, xx0 = ox0 - 4;  // halo origin
  // pointwise stages: wave = (64-channel group cg, 16-pixel tile group wp); lane's 4 epilogue channels per 16-channel tile
  const int cg = wave / 4, wp = wave % 4;
  int co[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) co[i] = (cg * 4 + i) * 16 + 4 * g;
  // this lane's output pixel in the k7 pointwise of the 8x8 tile (wp = its 16-pixel tile)
  const int op = wp * 16 + r16;
  const int ooy = oy0 + op / TW, oox = ox0 + op % TW;
  const bool opv = ooy < H && oox < W;
  const int64_t opp = opv ? ((int64_t)b * H + ooy) * W + oox : 0;

  // ---- 1. one round trip
  constexpr int HV = XH * XW * CV, HIT = HV / NT;
  static_assert(HV % NT == 0, "halo vectors per thread");
  h8 xr[PRE ? 1 : HIT];
  if constexpr (!PRE) {
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = tid + it * NT;
      const int cv = i % CV, px = i / CV;
      const int iy = xy0 + px / XW, ix = xx0 + px % XW;
      const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
      xr[it] = vload_sel(p1.x + ((int64_t)(b * H + iy) * W + ix) * p1.xcs + cv * 8, p1.x, ok);
    }
  }
  // PRE operands: B fragments of g0_x for halo rows wave + 4u (16 pixels each) and for this wave's output pixels;
  // A fragments of the cv1 half (rows C..2C-1 of g0_w) and of the cv2 half (rows 0..C-1)
  h8 gb[PRE ? 4 : 1][NKS], gc[NKS], a0[PRE ? 4 : 1][NKS], a0c[PRE ? 4 : 1][NKS];
  float b0v[PRE ? 4 : 1][4], b0c[PRE ? 4 : 1][4];
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int iy = xy0 + wave + 4 * u, ix = xx0 + r16;
      const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
      for (int m = 0; m < NKS; ++m)
        gb[u][m] = vload_sel(p1.g0x + ((int64_t)(b * H + iy) * W + ix) * p1.g0xcs + m * 32 + g * 8, p1.g0x, ok);
    }
#pragma unroll
    for (int m = 0; m < NKS; ++m) gc[m] = vload_sel(p1.g0x + opp * p1.g0xcs + m * 32 + g * 8, p1.g0x, opv);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int m = 0; m < NKS; ++m) {
        a0[i][m] = vload(p1.g0w + (int64_t)(C + i * 16 + r16) * C + m * 32 + g * 8);
        a0c[i][m] = vload(p1.g0w + (int64_t)(i * 16 + r16) * C + m * 32 + g * 8);
      }
      load_f<4>(p1.g0b + C + co[i], b0v[i]);
      load_f<4>(p1.g0b + co[i], b0c[i]);
    }
  }
  constexpr int TAPV = (9 + 49) * NQ, TIT = (TAPV + NT - 1) / NT;
  f32x4 wr[TIT];
#pragma unroll
  for (int it = 0; it < TIT; ++it) {
    const int i = min(tid + it * NT, TAPV - 1);
    const f32x4 w = i < 9 * NQ ? *reinterpret_cast<const f32x4*>(dw1 + (i / NQ) * C + (i % NQ) * 4)
                               : *reinterpret_cast<const f32x4*>(dw2 + ((i - 9 * NQ) / NQ) * C + (i % NQ) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[it][e] = float(T(w[e]));  // the reference's .half() weights
  }
  float bias_r = 0.f;  // tid < 3C: one bias each (k3 pw, k7 pw, TG)
  if (tid < C) bias_r = p1.bias[tid];
  else if (tid < 2 * C) bias_r = p2.bias[tid - C];
  else if (TG && tid < 3 * C) bias_r = p2.g2b[tid - 2 * C];
  h8 af1[4][NKS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int m = 0; m < NKS; ++m) af1[i][m] = vload(p1.w + (int64_t)((cg * 4 + i) * 16 + r16) * p1.KPAD + m * 32 + g * 8);
  // TG's second input (C3's cv2 branch), or with PRE the cv2 half this launch computes itself (rounded as stored)
  constexpr int X2IT = TG && !PRE ? NPX * CV / NT : 1;
  h8 x2r[X2IT];
  h4 c2h[PRE && TG ? 4 : 1];
#pragma unroll
  for (int i = 0; i < (PRE && TG ? 4 : 1); ++i) c2h[i] = h4{0, 0, 0, 0};
  if constexpr (TG && !PRE) {
#pragma unroll
    for (int it = 0; it < X2IT; ++it) {
      const int i = tid + it * NT;
      const int px = i / CV, cv = i % CV;
      const int oy = oy0 + px / TW, ox = ox0 + px % TW;
      const bool ok = oy < H && ox < W;
      x2r[it] = vload_sel(p2.g2x + (((int64_t)b * H + oy) * W + ox) * p2.g2xcs + cv * 8, p2.g2x, ok);
    }
  }

  if constexpr (PRE) {
    // ---- PRE. cv1 half over the halo (halo row wave + 4u = one 16-pixel MFMA tile), zero outside the image
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NKS; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i][m], gb[u][m], acc[i], 0, 0, 0);
      const int hy = wave + 4 * u, hx = r16;
      const int iy = xy0 + hy, ix = xx0 + hx;
      const bool inimg = iy >= 0 && iy < H && ix >= 0 && ix < W;
      const bool outpx = inimg && hy >= 4 && hy < 4 + TH && hx >= 4 && hx < 4 + TW;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][q] + b0v[i][q], p1.g0act);
        const h4 o = to_h4_rne(v);
        if (outpx) *reinterpret_cast<h4*>(p1.g0y + ((int64_t)(b * H + iy) * W + ix) * p1.g0ycs + C + co[i]) = o;
        s_x[(hy * XP + hx) * NQ + i * 4 + g] = inimg ? o : h4{0, 0, 0, 0};
      }
    }
    // cv2 half at this wave's output pixels -> g0_y (C3's cv2 branch, read by the trailing GEMM of the block's end)
    {
      f32x4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NKS; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0c[i][m], gc[m], acc[i], 0, 0, 0);
      if (opv) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][q] + b0c[i][q], p1.g0act);
          store_f<4>(p1.g0y + opp * p1.g0ycs + co[i], v);
          if constexpr (TG) c2h[i] = to_h4_rne(v);
        }
      }
    }
  } else {
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = tid + it * NT;
      const int cv = i % CV, px = i / CV;
      *reinterpret_cast<h8*>(&s_x[((px / XW) * XP + px % XW) * NQ + cv * 2]) = xr[it];
    }
  }
#pragma unroll
  for (int it = 0; it < TIT; ++it) {
    const int i = tid + it * NT;
    if (i < 9 * NQ) s_w3[i] = wr[it];
    else if (i < TAPV) s_w7[i - 9 * NQ] = wr[it];
  }
  if (tid < (TG ? 3 : 2) * C) s_bias[tid] = bias_r;
  // the k3 B tile's pad pixels (NR..NRP-1): finite zeros for the last MFMA tile
  for (int i = tid; i < NKS * (NRP - NR) * 4; i += NT) {
    const int ks = i / ((NRP - NR) * 4), rem = i % ((NRP - NR) * 4);
    s_b3[ks * NRP * 4 + lean_bswz(NR + rem / 4, rem % 4)] = h8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();

  // ---- 2. k3 depthwise over the 14x14 region -> B tile; the residual from the halo
  h4 rv[4];
  if (p2.res == YDBL_RES_ADD) {
    const int hy = op / TW + 4, hx = op % TW + 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) rv[i] = s_x[(hy * XP + hx) * NQ + co[i] / 4];
  }
  {
    constexpr int SEG = RW / 2, SEGW = SEG + 2, NTASK = NQ * RH * 2;
    for (int tk = tid; tk < NTASK; tk += NT) {
      const int q = tk % NQ, r = (tk / NQ) % RH, sg = tk / (NQ * RH);
      float a[SEG][4];
#pragma unroll
      for (int c = 0; c < SEG; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[c][e] = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const h4* xrow = &s_x[((r + ky) * XP + sg * SEG) * NQ + q];
        float xs[SEGW][4];
#pragma unroll
        for (int i = 0; i < SEGW; ++i) {
          const h4 v = xrow[i * NQ];
#pragma unroll
          for (int e = 0; e < 4; ++e) xs[i][e] = float(v[e]);
        }
        f32x4 wv[3];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) wv[kx] = s_w3[(ky * 3 + kx) * NQ + q];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int c = 0; c < SEG; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c + kx][e], wv[kx][e], a[c][e]);
      }
      const int ks = q / 8, ql = q % 8;
#pragma unroll
      for (int c = 0; c < SEG; ++c) {
        const int px = r * RW + sg * SEG + c;
        *(reinterpret_cast<h4*>(&s_b3[ks * NRP * 4 + lean_bswz(px, ql >> 1)]) + (ql & 1)) = to_h4_rne(a[c]);
      }
    }
  }
  // the k7 pointwise A fragments: issued here, used in stage 5
  h8 af2[4][NKS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int m = 0; m < NKS; ++m) af2[i][m] = vload(p2.w + (int64_t)((cg * 4 + i) * 16 + r16) * p2.KPAD + m * 32 + g * 8);
  __syncthreads();

  // ---- 3. k3 pointwise over the region's 16-pixel tiles wave + 4u, rounded, zero outside the image
  {
    constexpr int TU = (NRT + 3) / 4;
    f32x4 acc[4][TU];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < TU; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < NKS; ++m)
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int pt = wp + 4 * u;
        if (pt < NRT) {
          const h8 bf = s_b3[m * NRP * 4 + lean_bswz(pt * 16 + r16, g)];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af1[i][m], bf, acc[i][u], 0, 0, 0);
        }
      }
    h4 th[4][TU];
    float bv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(s_bias + co[i]);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = b4[q];
    }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int px = (wp + 4 * u) * 16 + r16;
      const int iy = oy0 - 3 + px / RW, ix = ox0 - 3 + px % RW;
      const bool inimg = px < NR && iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][u][q] + bv[i][q], p1.act);
        th[i][u] = inimg ? to_h4_rne(v) : h4{0, 0, 0, 0};
      }
    }
    __syncthreads();  // every wave is done reading the B tile
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int px = (wp + 4 * u) * 16 + r16;
      if (px < NR) {
#pragma unroll
        for (int i = 0; i < 4; ++i) s_t[((px / RW) * RP + px % RW) * NQ + co[i] / 4] = th[i][u];
      }
    }
  }
  __syncthreads();

  // ---- 4. k7 depthwise over the 8x8 outputs -> B tile (in the halo's place)
  {
    constexpr int SEG = 4, SEGW = SEG + 6;
    const int q = tid % NQ, r = (tid / NQ) % TH, sg = tid / (NQ * TH);
    float a[SEG][4];
#pragma unroll
    for (int c = 0; c < SEG; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[c][e] = 0.f;
#pragma unroll 1
    for (int ky = 0; ky < 7; ++ky) {
      const h4* trow = &s_t[((r + ky) * RP + sg * SEG) * NQ + q];
      float xs[SEGW][4];
#pragma unroll
      for (int i = 0; i < SEGW; ++i) {
        const h4 v = trow[i * NQ];
#pragma unroll
        for (int e = 0; e < 4; ++e) xs[i][e] = float(v[e]);
      }
      f32x4 wv[7];
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) wv[kx] = s_w7[(ky * 7 + kx) * NQ + q];
#pragma unroll
      for (int kx = 0; kx < 7; ++kx)
#pragma unroll
        for (int c = 0; c < SEG; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c + kx][e], wv[kx][e], a[c][e]);
    }
    const int ks = q / 8, ql = q % 8;
#pragma unroll
    for (int c = 0; c < SEG; ++c) {
      const int px = r * TW + sg * SEG + c;
      *(reinterpret_cast<h4*>(&s_b7[ks * NPX * 4 + lean_bswz(px, ql >> 1)]) + (ql & 1)) = to_h4_rne(a[c]);
    }
  }
  if constexpr (TG && PRE) {  // the trailing GEMM's second input: this launch's own cv2 half (k-steps NKS..)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = co[i];
      *(reinterpret_cast<h4*>(&s_g[(NKS + (c >> 5)) * NPX * 4 + lean_bswz(op, (c >> 3) & 3)]) + ((c >> 2) & 1)) = c2h[i];
    }
  } else if constexpr (TG) {  // the trailing GEMM's second input (C3's cv2 branch): k-steps NKS.. of its B tile
#pragma unroll
    for (int it = 0; it < X2IT; ++it) {
      const int i = tid + it * NT;
      const int px = i / CV, cv = i % CV;
      s_g[(NKS + cv / 4) * NPX * 4 + lean_bswz(px, cv & 3)] = x2r[it];
    }
  }
  __syncthreads();

  // ---- 5. k7 pointwise, bias, SiLU, + residual
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NKS; ++m) {
    const h8 bf = s_b7[m * NPX * 4 + lean_bswz(op, g)];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af2[i][m], bf, acc[i], 0, 0, 0);
  }
  h8 a2[TG ? 4 : 1][TG ? 2 * NKS : 1];
  if constexpr (TG) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int m = 0; m < 2 * NKS; ++m) a2[i][m] = vload(p2.g2w + (int64_t)((cg * 4 + i) * 16 + r16) * (2 * C) + m * 32 + g * 8);
  }
  if (opv) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(s_bias + C + co[i]);
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][q] + b4[q], p2.act);
      if (p2.res == YDBL_RES_ADD) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = float(rv[i][q]) + v[q];
      }
      if constexpr (TG) {
        const int c = co[i];
        *(reinterpret_cast<h4*>(&s_g[(c >> 5) * NPX * 4 + lean_bswz(op, (c >> 3) & 3)]) + ((c >> 2) & 1)) = to_h4_rne(v);
      } else {
        store_f<4>(p2.y + opp * p2.ycs + co[i], v);
      }
    }
  }
  if constexpr (TG) {
    // ---- TG. g2_y = act(g2_w [y ; g2_x] + g2_b), k-steps in channel order
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 2 * NKS; ++m) {
      const h8 bf = s_g[m * NPX * 4 + lean_bswz(op, g)];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i][m], bf, acc[i], 0, 0, 0);
    }
    if (opv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(s_bias + 2 * C + co[i]);
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][q] + b4[q], p2.g2act);
        store_f<4>(p2.g2y + opp * p2.g2ycs + co[i], v);
      }
    }
  }
}

int ds_check(const ydbl_dsconv_desc* d);                 // dsconv.hip
ConvArgs<_Float16> ds_args_f16(const ydbl_dsconv_desc* d);  // dsconv.hip

static bool same_view(const ydbl_view& a, const ydbl_view& b) {
  return a.ptr == b.ptr && a.n == b.n && a.h == b.h && a.w == b.w && a.c == b.c && a.cs == b.cs && a.dtype == b.dtype;
}

constexpr int64_t DSB_MAX_TILES_128 = 160;

// The pair this kernel is built for (include/ydbl.h ydbl_dsbottleneck_nhwc); anything else runs as the two launches.
static bool dsb_pair_fusable(const ydbl_dsconv_desc* d1, const ydbl_dsconv_desc* d2) {
  const char* e = getenv("YDBL_DSB_PAIR");  // A/B switch (read per launch: tests): 0 = two ydbl_dsconv_nhwc launches
  if (e && *e == '0') return false;
  if (d1->x.dtype != YDBL_F16) return false;
  const int c = d1->x.c;
  if ((c != 64 && c != 128) || d1->y.c != c || d2->y.c != c || (c == 128 && d1->g0_w)) return false;
  // 128 channels (one workgroup per CU) only on the small maps where the lean kernel runs too (dsc_lean.hip
  // LEAN_MAX_TILES_WIDE: DBL-s's 40^2 blocks at bs4, DBL-n's 20^2 at bs16)
  if (c == 128 && (int64_t)d1->x.n * cdiv(d1->x.h, 8) * cdiv(d1->x.w, 8) > DSB_MAX_TILES_128) return false;
  if (d1->k != 3 || d1->stride != 1 || d1->pad != 1 || d1->dil != 1 || d1->kpad != c) return false;
  if (d2->k != 7 || d2->stride != 1 || d2->pad != 3 || d2->dil != 1 || d2->kpad != c) return false;
  if (d1->dw_bias || d2->dw_bias || d1->tail_w || d2->tail_w || d1->g2_w || d2->g0_w) return false;
  if (d1->res_mode != YDBL_RES_NONE) return false;
  if (d2->res_mode != YDBL_RES_NONE && (d2->res_mode != YDBL_RES_ADD || d2->r.ptr != d1->x.ptr || d2->r.cs != d1->x.cs))
    return false;
  if (d1->x.cs % 8 || reinterpret_cast<uintptr_t>(d1->x.ptr) % 16) return false;
  if (d2->g2_w && (d2->g2_x.cs % 8 || reinterpret_cast<uintptr_t>(d2->g2_x.ptr) % 16)) return false;
  if (d1->g0_w && reinterpret_cast<uintptr_t>(d1->g0_x.ptr) % 16) return false;
  return true;
}

template <int C, bool PRE, bool TG>
static void dsb_go(const ConvArgs<_Float16>& a1, const ConvArgs<_Float16>& a2, const ydbl_dsconv_desc* d1,
                   const ydbl_dsconv_desc* d2, hipStream_t s) {
  using G = DsbGeo<C>;
  const int tiles_x = (int)cdiv(a1.W, G::TW), tiles_y = (int)cdiv(a1.H, G::TH);
  const int ntiles = a1.N * tiles_x * tiles_y;
  dsb_pair_kernel<C, PRE, TG><<<(unsigned)ntiles, G::NT, 0, s>>>(a1, a2, d1->dw_w, d2->dw_w, tiles_x, tiles_y, ntiles);
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_dsbottleneck_nhwc(const ydbl_dsconv_desc* d1, const ydbl_dsconv_desc* d2, void* stream) {
  if (const int rc = ds_check(d1)) return rc;
  if (const int rc = ds_check(d2)) return rc;
  if (!same_view(d1->y, d2->x)) return fail(YDBL_EINVAL, "dsbottleneck: d2.x must be d1.y (the intermediate)");
  const hipStream_t s = as_stream(stream);
  if (dsb_pair_fusable(d1, d2)) {
    const ConvArgs<_Float16> a1 = ds_args_f16(d1), a2 = ds_args_f16(d2);
    if (d1->x.c == 128) {
      if (d2->g2_w) dsb_go<128, false, true>(a1, a2, d1, d2, s);
      else dsb_go<128, false, false>(a1, a2, d1, d2, s);
    } else if (d1->g0_w && d2->g2_w) dsb_go<64, true, true>(a1, a2, d1, d2, s);
    else if (d1->g0_w) dsb_go<64, true, false>(a1, a2, d1, d2, s);
    else if (d2->g2_w) dsb_go<64, false, true>(a1, a2, d1, d2, s);
    else dsb_go<64, false, false>(a1, a2, d1, d2, s);
    return check_launch("ydbl_dsbottleneck_nhwc");
  }
  if (const int rc = ydbl_dsconv_nhwc(d1, stream)) return rc;
  return ydbl_dsconv_nhwc(d2, stream);
}
