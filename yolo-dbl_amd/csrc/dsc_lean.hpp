// The lean DSConv tile (dsc_lean.hip) as a device function.  See dsc_lean.hip for the design.
#pragma once
#include "conv_common.hpp"

namespace ydbl {

__device__ __forceinline__ int lean_bswz(int row, int kv) { return row * 4 + (kv ^ (((row >> 2) & 1) << 1)); }

// LDS carve-up of one lean tile
template <int C, int CO, int K, int S, int TH, int TW, int NT, bool TG, bool PRE, bool TAIL = false>
struct LeanLds {
  static constexpr int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K, IWP = IW | 1, NQ = C / 4;
  static constexpr int NPX = TH * TW, NKS = C / 32, PNP = PRE ? (IH * IW + 15) / 16 * 16 : 16;
  static constexpr int X = 0;                                              // h4 [IH * IWP * NQ]
  static constexpr int W = (X + IH * IWP * NQ * 8 + 15) / 16 * 16;          // f32x4 [K * K * NQ]
  static constexpr int B = W + K * K * NQ * 16;                             // h8 [NKS * NPX * 4]
  static constexpr int P = B + NKS * NPX * 4 * 16;                          // h8 [2 * PNP * 4] (PRE)
  static constexpr int T = P + (PRE ? 2 * PNP * 4 * 16 : 16);               // f32 [4][CO] class-conv weights (TAIL)
  static constexpr int BI = T + (TAIL ? 4 * CO * 4 : 0);                    // f32 [CO] pointwise bias
  static constexpr int BI2 = BI + CO * 4;                                   // f32 [CO] trailing-GEMM bias (TG)
  static constexpr int BYTES = BI2 + (TG ? CO * 4 : 0);
};

// One TH x TW output tile (linear tile index `tile`: image-major, then tile row, tile column).
// smem: LeanLds::BYTES of LDS, 16-byte aligned.
template <int C, int CO, int K, int S, int TH, int TW, int NT, bool TG, bool TAIL, bool PRE>
__device__ __forceinline__ void lean_tile(const ConvArgs<_Float16>& p, const float* __restrict__ dww,
                                          const float* __restrict__ dwb, int dw_act, int tile, int tiles_x,
                                          int tiles_y, unsigned char* smem) {
  using T = _Float16;
  constexpr int WAVES = NT / 64;
  constexpr int CV = C / 8;                          // 16-byte vectors per pixel
  constexpr int NQ = C / 4;                          // channel quads
  constexpr int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K;
  constexpr int IWP = IW | 1;                        // odd pixel pitch: rows r, r+1 in opposite bank halves
  constexpr int HV = IH * IW * CV;
  constexpr int HIT = (HV + NT - 1) / NT;
  constexpr int CSEG = NQ * TH * TW / NT;            // outputs per depthwise task
  static_assert(CSEG >= 1 && TW % CSEG == 0 && NQ * TH * (TW / CSEG) == NT, "depthwise task split");
  constexpr int SEGW = (CSEG - 1) * S + K;
  constexpr int TAPV = K * K * NQ;
  constexpr int TIT = (TAPV + NT - 1) / NT;
  constexpr int NPX = TH * TW, NTP = NPX / 16;       // 16-pixel MFMA tiles
  static_assert(NPX % 16 == 0, "tile");
  constexpr int NKS = C / 32;                        // pointwise k-steps
  constexpr int NTC = CO / 16;                       // output-channel tiles
  // per wave: a group of TN output-channel tiles (<= 64 channels; fewer for deep inputs, whose A fragments
  // [TN][NKS] would not fit the VGPRs); all 64 when CO = 64 and C <= 128 (the Detect class-conv tail needs them)
  constexpr int TNA = 16 / NKS < 1 ? 1 : 16 / NKS;
  constexpr int TN = NTC < (TNA < 4 ? TNA : 4) ? NTC : (TNA < 4 ? TNA : 4);
  constexpr int NCG = NTC / TN;
  static_assert(NTC % TN == 0 && WAVES % NCG == 0, "channel groups over waves");
  constexpr int WPG = WAVES / NCG;
  constexpr int TM = (NTP + WPG - 1) / WPG;          // pixel tiles per wave
  // TG: trailing GEMM over [y ; g2x] (2*CO channels, CO/16 output tiles as the pointwise): its B tile
  // [2*CO/32 k-steps][pixel][slot] reuses the halo's LDS once the depthwise phase is over
  constexpr int NKS2 = TG ? 2 * CO / 32 : 0;
  static_assert(!TG || (C == CO && NKS2 * NPX * 4 * 16 <= IH * IWP * NQ * 8), "trailing GEMM layout");
  constexpr int X2V = TG ? NPX * CO / 8 : 1, X2IT = (X2V + NT - 1) / NT;
  // PRE: leading 1x1 g0y = act(W0 g0x + b0) (2C outputs: C3's cv2 | cv1) over the whole halo, its last C channels
  // are this DSConv's input; B tile [2 k-steps][halo pixel, padded to 16][slot], one 16-channel tile pair per wave
  static_assert(!PRE || (C == 64 && CO == 64 && S == 1 && !TG && !TAIL && WAVES == 4), "leading 1x1 layout");
  constexpr int PNP = PRE ? (IH * IW + 15) / 16 * 16 : 16, PNT = PNP / 16;
  using L = LeanLds<C, CO, K, S, TH, TW, NT, TG, PRE, TAIL>;
  h4* s_x = reinterpret_cast<h4*>(smem + L::X);      // fp16 halo, [row][col][quad]
  f32x4* s_w = reinterpret_cast<f32x4*>(smem + L::W);  // fp32 taps (rounded to fp16), [tap][quad]
  h8* s_b = reinterpret_cast<h8*>(smem + L::B);      // pointwise B tile, [k-step][pixel][slot]
  h8* s_g = reinterpret_cast<h8*>(s_x);              // TG: trailing GEMM B tile (after the depthwise phase)
  h8* s_p = reinterpret_cast<h8*>(smem + L::P);      // PRE: the leading 1x1's B tile (g0x halo)
  // activation accessors (element offsets from each view's base)
  auto ld16 = [&](const T* base, int64_t off, bool ok) -> h8 { return vload_sel(base + off, base, ok); };
  auto ld8 = [&](const T* base, int64_t off) -> h4 { return *reinterpret_cast<const h4*>(base + off); };
  auto st8 = [&](T* base, int64_t off, const float* v) { store_f<4>(base + off, v); };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int cg = wave % NCG, wp = wave / NCG;
  int co[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) co[i] = (cg * TN + i) * 16 + 4 * g;  // this lane's 4 epilogue channels

  struct Tile {
    int b, oy0, ox0, iy0, ix0;
  };
  auto tile_of = [&](int t) {
    int bid = t;
    const int tx = bid % tiles_x;
    bid /= tiles_x;
    const int ty = bid % tiles_y;
    Tile tl;
    tl.b = bid / tiles_y;
    tl.oy0 = ty * TH;
    tl.ox0 = tx * TW;
    tl.iy0 = tl.oy0 * S - p.PAD;
    tl.ix0 = tl.ox0 * S - p.PAD;
    return tl;
  };
  h8 xr[HIT];
  const T* xsrc = PRE ? p.g0x : p.x;
  const int xscs = PRE ? p.g0xcs : p.xcs;
  auto load_halo = [&](const Tile& tl) {
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = min(tid + it * NT, HV - 1);
      const int cv = i % CV, px = i / CV;
      const int hy = px / IW, hx = px - hy * IW;
      const int iy = tl.iy0 + hy, ix = tl.ix0 + hx;
      const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      xr[it] = ld16(xsrc, ((int64_t)(tl.b * p.H + iy) * p.W + ix) * xscs + cv * 8, ok);
    }
  };

  // ---- 1. one round trip: halo + taps (-> LDS), then A fragments (+ residual, second GEMM input) (-> VGPRs)
  const Tile tl = tile_of(tile);
  load_halo(tl);
  f32x4 wr[TIT];
#pragma unroll
  for (int it = 0; it < TIT; ++it) {
    const int i = min(tid + it * NT, TAPV - 1);
    const f32x4 w = *reinterpret_cast<const f32x4*>(dww + (i / NQ) * C + (i % NQ) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[it][e] = float(T(w[e]));  // the reference's .half() weights
  }
  // the pointwise bias (+ TG's g2b, + TAIL's class-conv weights [k][CO]) for LDS: loaded here, in the first round
  // trip, and stored just before its barrier (a store right after its load waits on every load issued before it).
  // Read from global after the MFMAs they cost one more round trip at the very end; kept in VGPRs from the start
  // they cost 16 registers and a wave per SIMD.
  constexpr int BIT = (CO + NT - 1) / NT, TLT = TAIL ? (4 * CO + NT - 1) / NT : 0;
  float bir[BIT], b2r[TG ? BIT : 1], tlr[TLT > 0 ? TLT : 1];
#pragma unroll
  for (int it = 0; it < BIT; ++it) {
    const int i = min(tid + it * NT, CO - 1);
    bir[it] = p.bias[i];
    if constexpr (TG) b2r[it] = p.g2b[i];
  }
#pragma unroll
  for (int it = 0; it < TLT; ++it) {
    const int i = min(tid + it * NT, 4 * CO - 1);
    tlr[it] = i / CO < p.nt3 ? p.t3w[i] : 0.f;
  }
  h8 af[TN][NKS];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int row = (cg * TN + i) * 16 + r16;  // A rows: output channel of this lane
#pragma unroll
    for (int m = 0; m < NKS; ++m) af[i][m] = vload(p.w + (int64_t)row * p.KPAD + m * 32 + g * 8);
  }

  // PRE: tile i = 0 of this wave = 16 channels of the cv1 half (C + 16 wave.., over the whole halo, before the
  // depthwise), i = 1 = 16 channels of the cv2 half (16 wave.., over the output pixels only, after the pointwise)
  h8 a0[2][2];
  float b0v[2][4];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ct = i == 0 ? C / 16 + wave : wave;
      const int row = ct * 16 + r16;
#pragma unroll
      for (int m = 0; m < 2; ++m) a0[i][m] = vload(p.g0w + (int64_t)row * C + m * 32 + g * 8);
      load_f<4>(p.g0b + ct * 16 + 4 * g, b0v[i]);
    }
  }
#pragma unroll
  for (int it = 0; it < TIT; ++it)
    if (tid + it * NT < TAPV) s_w[tid + it * NT] = wr[it];
  {
    int64_t pp[TM];
    bool pv[TM];
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int pt = wp + WPG * j;
      const int op = pt * 16 + r16;
      const int oy = tl.oy0 + op / TW, ox = tl.ox0 + op % TW;
      pv[j] = pt < NTP && oy < p.Ho && ox < p.Wo;
      pp[j] = pv[j] ? ((int64_t)tl.b * p.Ho + oy) * p.Wo + ox : 0;
    }
    h8 x2r[X2IT];  // TG: the second GEMM input's tile (C3's cv2 branch), [pixel][8-channel vector]
    if constexpr (TG) {
#pragma unroll
      for (int it = 0; it < X2IT; ++it) {
        const int i = min(tid + it * NT, X2V - 1);
        const int px = i / (CO / 8), cv = i % (CO / 8);
        const int oy = tl.oy0 + px / TW, ox = tl.ox0 + px % TW;
        const bool ok = oy < p.Ho && ox < p.Wo;
        x2r[it] = ld16(p.g2x, (((int64_t)tl.b * p.Ho + oy) * p.Wo + ox) * p.g2xcs + cv * 8, ok);
      }
    }
    h4 rv[TN][TM];
    if (p.res != YDBL_RES_NONE) {
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int i = 0; i < TN; ++i) rv[i][j] = ld8(p.r, pp[j] * p.rcs + co[i]);
    }
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int i = tid + it * NT;
      if (i < HV) {
        const int cv = i % CV, px = i / CV;
        if constexpr (PRE) {
          s_p[(cv >> 2) * PNP * 4 + lean_bswz(px, cv & 3)] = xr[it];
        } else {
          const int hy = px / IW, hx = px - hy * IW;
          *reinterpret_cast<h8*>(&s_x[(hy * IWP + hx) * NQ + cv * 2]) = xr[it];
        }
      }
    }
    if constexpr (PRE) {  // the pad pixels of the last 16-pixel tile: finite zeros (never stored)
      for (int i = tid; i < (PNP - IH * IW) * CV; i += NT) {
        const int cv = i % CV, px = IH * IW + i / CV;
        s_p[(cv >> 2) * PNP * 4 + lean_bswz(px, cv & 3)] = h8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int it = 0; it < BIT; ++it)
      if (tid + it * NT < CO) {
        reinterpret_cast<float*>(smem + L::BI)[tid + it * NT] = bir[it];
        if constexpr (TG) reinterpret_cast<float*>(smem + L::BI2)[tid + it * NT] = b2r[it];
      }
#pragma unroll
    for (int it = 0; it < TLT; ++it)
      if (tid + it * NT < 4 * CO) reinterpret_cast<float*>(smem + L::T)[tid + it * NT] = tlr[it];
    __syncthreads();
    if constexpr (PRE) {
      // ---- 1b. leading 1x1 over the halo on MFMA (k-steps in channel order, epilogue as conv_epilogue's):
      // every output pixel's 2C values -> g0y; the last C channels (zero outside the image: the depthwise
      // padding) -> the fp16 halo in LDS, exactly what the unfused DSConv would read back
      const int c = C + wave * 16 + 4 * g;
#pragma unroll
      for (int j = 0; j < PNT; ++j) {
        f32x4 pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 2; ++m)
          pa = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[0][m], s_p[m * PNP * 4 + lean_bswz(j * 16 + r16, g)], pa, 0, 0, 0);
        const int px = j * 16 + r16;
        const int hy = px / IW, hx = px - hy * IW;
        const int iy = tl.iy0 + hy, ix = tl.ix0 + hx;
        const bool live = px < IH * IW;
        const bool inimg = live && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        const bool outpx = inimg && hy >= p.PAD && hy < p.PAD + TH && hx >= p.PAD && hx < p.PAD + TW;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(pa[q] + b0v[0][q], p.g0act);
        const h4 o = to_h4_rne(v);
        if (outpx) *reinterpret_cast<h4*>(p.g0y + ((int64_t)(tl.b * p.H + iy) * p.W + ix) * p.g0ycs + c) = o;
        if (live) s_x[(hy * IWP + hx) * NQ + (c - C) / 4] = inimg ? o : h4{0, 0, 0, 0};
      }
      __syncthreads();
    }

    // ---- 2. depthwise: task = (quad q, output row r, segment sg), quad fastest
    {
      const int q = tid % NQ;
      const int r = (tid / NQ) % TH;
      const int sg = tid / (NQ * TH);
      float a[CSEG][4];
#pragma unroll
      for (int c = 0; c < CSEG; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[c][e] = 0.f;
      constexpr int KU = K <= 3 ? K : 1;  // the 7x7: one input row's window + taps live at a time
#pragma unroll KU
      for (int ky = 0; ky < K; ++ky) {
        const h4* xrow = &s_x[((r * S + ky) * IWP + sg * CSEG * S) * NQ + q];
        float xs[SEGW][4];
#pragma unroll
        for (int i = 0; i < SEGW; ++i) {
          const h4 v = xrow[i * NQ];
#pragma unroll
          for (int e = 0; e < 4; ++e) xs[i][e] = float(v[e]);
        }
        f32x4 wv[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) wv[kx] = s_w[(ky * K + kx) * NQ + q];
#pragma unroll
        for (int kx = 0; kx < K; ++kx)
#pragma unroll
          for (int c = 0; c < CSEG; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[c][e] = fmaf(xs[c * S + kx][e], wv[kx][e], a[c][e]);
      }
      if (dwb) {  // uniform: DWConv (+ folded BN) bias and activation before the pointwise
        const f32x4 bq = *reinterpret_cast<const f32x4*>(dwb + q * 4);
#pragma unroll
        for (int c = 0; c < CSEG; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) a[c][e] = apply_act<T>(a[c][e] + bq[e], dw_act);
      }
      const int ks = q / 8, ql = q % 8;  // k-step and 4-channel slot of this quad
#pragma unroll
      for (int c = 0; c < CSEG; ++c) {
        const int px = r * TW + sg * CSEG + c;
        *(reinterpret_cast<h4*>(&s_b[ks * NPX * 4 + lean_bswz(px, ql >> 1)]) + (ql & 1)) = to_h4_rne(a[c]);
      }
    }
    __syncthreads();

    // ---- 3. pointwise MFMA over all k-steps, epilogue
    f32x4 acc[TN][TM];
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < NKS; ++m)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int pt = wp + WPG * j;
        if (TM * WPG == NTP || pt < NTP) {
          const h8 bf = s_b[m * NPX * 4 + lean_bswz(pt * 16 + r16, g)];
#pragma unroll
          for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][m], bf, acc[i][j], 0, 0, 0);
        }
      }
    float bv[TN][4];
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(smem + L::BI + co[i] * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = b4[q];
    }
    float ys[TAIL ? TN : 1][TAIL ? TM : 1][4];  // TAIL: the stored y values for the class conv
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      if (!pv[j]) continue;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][j][q] + bv[i][q], p.act);
        if (p.res == YDBL_RES_ADD) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = float(rv[i][j][q]) + v[q];
        } else if (p.res == YDBL_RES_MUL) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = float(rv[i][j][q]) * v[q];
        }
        if constexpr (TG) {  // y (rounded as the unfused path stores it) -> the trailing GEMM's B tile
          const int px = (wp + WPG * j) * 16 + r16, c = co[i];
          *(reinterpret_cast<h4*>(&s_g[(c >> 5) * NPX * 4 + lean_bswz(px, (c >> 3) & 3)]) + ((c >> 2) & 1)) =
              to_h4_rne(v);
        } else {
          st8(p.y, pp[j] * p.ycs + co[i], v);
          if constexpr (TAIL) {
#pragma unroll
            for (int q = 0; q < 4; ++q) ys[i][j][q] = round_to<T>(v[q]);
          }
        }
      }
    }
    if constexpr (PRE) {
      // ---- 3b. the cv2 half of the leading 1x1 over the output pixels (s_p is read-only since the first barrier)
      const int c = wave * 16 + 4 * g;
#pragma unroll
      for (int j = 0; j < NTP; ++j) {
        const int op = j * 16 + r16;
        const int hpx = (op / TW + p.PAD) * IW + op % TW + p.PAD;
        f32x4 pa = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < 2; ++m)
          pa = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[1][m], s_p[m * PNP * 4 + lean_bswz(hpx, g)], pa, 0, 0, 0);
        const int oy = tl.oy0 + op / TW, ox = tl.ox0 + op % TW;
        if (oy < p.Ho && ox < p.Wo) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(pa[q] + b0v[1][q], p.g0act);
          st8(p.g0y, (((int64_t)tl.b * p.Ho + oy) * p.Wo + ox) * p.g0ycs + c, v);
        }
      }
    }
    if constexpr (TAIL && NCG == 1 && TN == 4 && !TG) {  // Detect class conv over the 64 output channels (CO == 64)
      conv_tail_1x1_vals<T, TN, TM>(p, ys, pp, pv, co, g, reinterpret_cast<const float*>(smem + L::T));
    }
    if constexpr (TG) {
      // ---- 4. trailing GEMM: g2y = act(W2 [y ; g2x] + b2), K = 2*CO in channel order (the unfused cv3's k-steps)
#pragma unroll
      for (int it = 0; it < X2IT; ++it) {
        const int i = tid + it * NT;
        if (i < X2V) {
          const int px = i / (CO / 8), cv = i % (CO / 8);
          s_g[(CO / 32 + cv / 4) * NPX * 4 + lean_bswz(px, cv & 3)] = x2r[it];
        }
      }
      h8 a2[TN][NKS2];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = (cg * TN + i) * 16 + r16;
#pragma unroll
        for (int m = 0; m < NKS2; ++m) a2[i][m] = vload(p.g2w + (int64_t)row * (2 * CO) + m * 32 + g * 8);
      }
      float b2v[TN][4];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(smem + L::BI2 + co[i] * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) b2v[i][q] = b4[q];
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NKS2; ++m)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int pt = wp + WPG * j;
          if (TM * WPG == NTP || pt < NTP) {
            const h8 bf = s_g[m * NPX * 4 + lean_bswz(pt * 16 + r16, g)];
#pragma unroll
            for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i][m], bf, acc[i][j], 0, 0, 0);
          }
        }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        if (!pv[j]) continue;
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][j][q] + b2v[i][q], p.g2act);
          st8(p.g2y, pp[j] * p.g2ycs + co[i], v);
        }
      }
    }
  }
}

}  // namespace ydbl
