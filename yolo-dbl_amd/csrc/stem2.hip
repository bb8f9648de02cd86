// Stem pair: preprocess + the backbone's first two Convs in one kernel (fp16 path).
//
// The DBL backbones open with Conv(3, C0, 3, 1) at full resolution followed by Conv(C0, 2*C0, 3, 2)
// (U/cfg/models/DBL/yolov13*-DBL*.yaml layers 0-1; Conv = conv + folded BN + SiLU,
// U/nn/modules/conv.py:39-63).  Run separately, the full-resolution C0-channel map is written and
// read back once (at 640x640, bs32, C0 = 8: 210 MB each way) — more HBM traffic than the input and
// the output together.  Here each workgroup produces a TH x TW tile of the second conv's output and
// keeps the (2TH+1) x (2TW+1) first-conv tile it needs in LDS only:
//   1. stage the (2TH+3) x (2TW+3) input window from the NCHW fp32 batch as one (c0,c1,c2,0) fp16
//      record per pixel (x * scale rounded to fp16 once, as .half() does), from float4 plane loads
//      all issued before the first LDS write (one memory round trip per workgroup);
//   2. first conv on MFMA 16x16x32 f16 (K = 9 taps x 4 record slots = 36 per pixel; M = 16 rows =
//      C0 couts, or for C0 = 8 two 16-pixel sets x 8 couts via a block-diagonal A, 3 k-steps per 32 px),
//      + bias + SiLU, rounded to fp16 (the precision the reference stores it in), zero where the
//      pixel lies outside the image (the second conv's zero padding) -> LDS tile;
//   3. second conv on MFMA (K = 9 taps x C0, k-steps of 32), + bias + SiLU -> NHWC fp16.
// The first-conv tile is stored as 16-byte records of 8 channels, split by column parity
// ([chunk][row][parity][col/2]) so that the stride-2 second conv reads consecutive records across a
// 16-lane pixel group: every ds_read_b128 is conflict-free.  The halo rows/cols of the first conv
// (one extra row and column per tile, 6-8 % extra MFMA work) are recomputed instead of exchanged.
// HBM traffic is the input once (+ halo re-reads, mostly L2 hits) and the output once.
#include <stdlib.h>

#include <type_traits>

#include "conv_common.hpp"

namespace ydbl {

template <int C0, int TW, int TH>
struct Stem2Cfg {
  static constexpr int C1 = 2 * C0;
  // first conv: M = 16 rows = PS pixel sets x C0M couts.  C0 = 8 fills the rows with two 16-pixel
  // sets through a block-diagonal A (rows 0-7 see only set 0's K slots, rows 8-15 only set 1's)
  static constexpr int PS = C0 == 8 ? 2 : 1;
  static constexpr int C0M = 16 / PS;
  static constexpr int KS0 = (PS * 36 + 31) / 32;   // first conv k-steps (36 slots per pixel set)
  static constexpr int NT1 = C1 / 16;               // second conv: 16-cout MFMA tiles
  static constexpr int KS1 = (9 * C0 + 31) / 32;    // second conv k-steps
  static constexpr int CH = C0 / 8;                 // 8-channel chunks of a first-conv pixel
  static constexpr int INH = 2 * TH + 3, INW = 2 * TW + 3;
  static constexpr int L0H = 2 * TH + 1, L0W = 2 * TW + 1;
  static constexpr int L0P = TW + 1;                // records per parity plane row
  // + slack: the virtual first-conv grid's last MFMA group reads up to 16 * PS + 2 records past the
  // window (results discarded); keep those reads inside the tile
  static constexpr int IN_BYTES = (INH * INW + 16 * PS + 16) * 8;
  static constexpr int L0_BYTES = CH * L0H * 2 * L0P * 16;
  static constexpr int LDS = IN_BYTES + L0_BYTES;
  // packed parameter blob: MFMA A fragments (h8 per lane) of both convs, then fp32 biases
  static constexpr int W0F = KS0 * 64;              // h8 entries
  static constexpr int W1F = NT1 * KS1 * 64;
  static constexpr int64_t BYTES = (int64_t)(W0F + W1F) * 16 + (16 + C1) * 4;
};

// Host: pack conv weights (fp32, PyTorch layouts) into the kernel's fragment order.
template <int C0>
void stem2_pack(const float* w0, const float* b0, const float* w1, const float* b1, unsigned char* out) {
  using Cfg = Stem2Cfg<C0, 32, 8>;
  _Float16* f0 = reinterpret_cast<_Float16*>(out);
  _Float16* f1 = f0 + Cfg::W0F * 8;
  float* fb0 = reinterpret_cast<float*>(f1 + Cfg::W1F * 8);
  float* fb1 = fb0 + 16;
  // A[row][k]: row -> (pixel set row / C0M, cout row % C0M); slot k -> record q = k / 4 (set q / 9,
  // tap q % 9), channel k % 4
  for (int m = 0; m < Cfg::KS0; ++m)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        const int g = lane >> 4, row = lane & 15;
        const int k = 32 * m + 8 * g + j, q = k / 4, c = k % 4;
        const bool live = q < 9 * Cfg::PS && q / 9 == row / Cfg::C0M;
        const int co = row % Cfg::C0M, tap = q % 9;
        // slot 3 of a record is 1 for pixels inside the image: the centre tap's slot-3 weight is the bias
        const float wv = !live ? 0.f : c < 3 ? w0[(co * 3 + c) * 9 + tap] : tap == 4 ? b0[co] : 0.f;
        f0[(m * 64 + lane) * 8 + j] = (_Float16)wv;
      }
  for (int t = 0; t < Cfg::NT1; ++t)
    for (int m = 0; m < Cfg::KS1; ++m)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int g = lane >> 4, co = 16 * t + (lane & 15);
          const int k0 = 32 * m + 8 * g, tap = k0 / C0, c = k0 % C0 + j;
          f1[((t * Cfg::KS1 + m) * 64 + lane) * 8 + j] = (_Float16)(tap < 9 ? w1[(co * C0 + c) * 9 + tap] : 0.f);
        }
  for (int i = 0; i < 16; ++i) fb0[i] = b0[i % Cfg::C0M];
  for (int i = 0; i < Cfg::C1; ++i) fb1[i] = b1[i];
}

// Diagnostic build only (-DYDBL_STEM2_STAMPS, scripts/build_stamps.sh stem2): per-workgroup s_memrealtime stamps
// (100 MHz) when wave 0 starts, has staged the window, has finished the first conv, has stored; + hardware ids.
#ifdef YDBL_STEM2_STAMPS
__device__ unsigned long long g_st_stamps[8 * 16384];
#define ST_STAMP(k)                                                                                         \
  do {                                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_st_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ST_STAMP(k) \
  do {              \
  } while (0)
#endif

// One workgroup per tile.  (Measured and not kept: a persistent walk over 2-8 tiles per CU with the next
// tile's window prefetched during the current tile's convs -- 140-166 vs 136 us at bs32: the kernel is VALU-
// issue-bound on the first conv's SiLU, not latency-bound.)
// BOUND (a template flag, so the session's own unbound launch carries no binding code): x and scale from the input
// binding (include/ydbl.h ydbl_input_bind), read once at the start.
template <int C0, int TW, int TH, bool V4, bool BOUND>
__global__ __launch_bounds__(256, 2) void stem2_kernel(const float* __restrict__ x, int H, int W, float scale,
                                                       const unsigned char* __restrict__ params,
                                                       DView<_Float16> y, int tiles_x, int tiles_y, int nblocks,
                                                       InputBind ib) {
  if constexpr (BOUND) {
    x = *ib.x;
    scale = *ib.amax > 1.0f + __FLT_EPSILON__ ? 1.0f / 255.0f : 1.0f;
  }
  using Cfg = Stem2Cfg<C0, TW, TH>;
  const h8* w0f = reinterpret_cast<const h8*>(params);
  const h8* w1f = w0f + Cfg::W0F;
  const float* b0 = reinterpret_cast<const float*>(w1f + Cfg::W1F);
  const float* b1 = b0 + 16;
  extern __shared__ __align__(16) unsigned char smem[];
  h4* in = reinterpret_cast<h4*>(smem);                        // [INH][INW] records
  unsigned char* l0 = smem + Cfg::IN_BYTES;                     // [CH][L0H][2][L0P] x 16 B
  const int64_t plane = (int64_t)H * W;

  struct Tile {
    int img, oy0, ox0, Y0, X0;
  };
  auto tile_of = [&](int t) {
    const int bid = xcd_remap(t, nblocks);
    const int tx = bid % tiles_x;
    const int ty = (bid / tiles_x) % tiles_y;
    Tile tl;
    tl.img = bid / (tiles_x * tiles_y);
    tl.oy0 = ty * TH;
    tl.ox0 = tx * TW;
    tl.Y0 = 2 * tl.oy0 - 1;  // first-conv tile origin (image coords)
    tl.X0 = 2 * tl.ox0 - 1;
    return tl;
  };

  // ---- 1. input window, origin (Y0 - 1, X0 - 1); the slack past it is zeroed once (a block-diagonal
  // MFMA multiplies the other set's records by 0, which must not meet a NaN)
  if (threadIdx.x < Cfg::IN_BYTES / 8 - Cfg::INH * Cfg::INW) in[Cfg::INH * Cfg::INW + threadIdx.x] = h4{0, 0, 0, 0};
  // V4 tasks = (row, 16-byte column group): three float4 loads (one per plane) -> 4 records.
  // Group k covers image columns A + 4k .. A + 4k + 3 = record columns 4k - 2 .. 4k + 1, with
  // A = X0 - 3 a multiple of 4, so with W % 4 == 0 a group is wholly inside or outside the image.
  constexpr int NG = (Cfg::INW + 5) / 4;
  constexpr int TASKS = V4 ? Cfg::INH * NG : Cfg::INH * Cfg::INW;
  constexpr int IT = (TASKS + 255) / 256;
  f32x4 v[IT][3];
  bool okv[IT];  // the task's pixels lie inside the image (record slot 3 = 1: the folded bias)
  // A bound input (predict() reading the caller's batch in place, include/ydbl.h ydbl_input_bind) arrives cold and is
  // read once: nontemporal loads, which skip the Infinity-Cache allocation that would evict dirty activation lines
  // (batchmax.hip).  The session's own staging buffer (no binding: the bench path) is read with plain loads: in the
  // graph it was just written by the copy in, and nontemporal loads cost it 3-4 us per bs16 launch
  // (profiles/r06/r06_stem2_nt_ab.txt).
  auto ld = [](const auto* ptr, auto nt) {
    if constexpr (decltype(nt)::value) return __builtin_nontemporal_load(ptr);
    else return *ptr;
  };
  auto load_window = [&](const Tile& tl, auto nt) {
    const float* xb = x + (int64_t)tl.img * 3 * plane;
    if constexpr (V4) {
      const int A = tl.X0 - 3;
#pragma unroll
      for (int u = 0; u < IT; ++u) {
        const int t = threadIdx.x + u * 256;
        const int r = t / NG, k = t - r * NG;
        const int iy = tl.Y0 - 1 + r, ix = A + 4 * k;
        const bool ok = t < TASKS && iy >= 0 && iy < H && ix >= 0 && ix < W;
        okv[u] = ok;
        const int64_t o = ok ? (int64_t)iy * W + ix : 0;
#pragma unroll
        for (int c = 0; c < 3; ++c)
          v[u][c] = ok ? ld(reinterpret_cast<const f32x4*>(xb + c * plane + o), nt)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int u = 0; u < IT; ++u) {
        const int t = threadIdx.x + u * 256;
        const int r = t / Cfg::INW, c = t - r * Cfg::INW;
        const int iy = tl.Y0 - 1 + r, ix = tl.X0 - 1 + c;
        const bool ok = t < TASKS && iy >= 0 && iy < H && ix >= 0 && ix < W;
        okv[u] = ok;
        const int64_t o = ok ? (int64_t)iy * W + ix : 0;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) v[u][ch][0] = ok ? ld(xb + ch * plane + o, nt) : 0.f;
      }
    }
  };
  auto store_window = [&]() {
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int t = threadIdx.x + u * 256;
      if (t >= TASKS) continue;
      if constexpr (V4) {
        const int r = t / NG, k = t - r * NG;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 4 * k - 2 + e;
          if (col < 0 || col >= Cfg::INW) continue;
          in[r * Cfg::INW + col] = h4{f16_rne(v[u][0][e] * scale), f16_rne(v[u][1][e] * scale),
                                      f16_rne(v[u][2][e] * scale), (_Float16)(okv[u] ? 1.f : 0.f)};
        }
      } else {
        in[t] = h4{f16_rne(v[u][0][0] * scale), f16_rne(v[u][1][0] * scale), f16_rne(v[u][2][0] * scale),
                   (_Float16)(okv[u] ? 1.f : 0.f)};
      }
    }
  };

  const int lane = threadIdx.x & 63, wave = wave_id();
  const int g = lane >> 4, r16 = lane & 15;

  // First conv over a virtual grid of L0H rows x INW columns (the input tile's pitch; the last two
  // columns of each row are dead): pixel p then sits at input record p, so a lane's B address is
  // its pixel index plus a per-lane constant and no per-pixel division is needed until the store.
  // A fragments and this lane's two B records per k-step: record q = 8m + 2g + u of the K layout
  // [set 0: 9 taps][set 1: 9 taps] (slots past the last set carry zero weights).
  constexpr int PS = Cfg::PS, KS0 = Cfg::KS0;
  h8 a0[KS0];
  int boff[KS0][2];  // byte offset from this lane's set-0 pixel record
#pragma unroll
  for (int m = 0; m < KS0; ++m) {
    a0[m] = w0f[m * 64 + lane];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = 8 * m + 2 * g + u;
      const int tap = q < 9 * PS ? q % 9 : 8;
      const int set = q < 9 * PS ? q / 9 : PS - 1;
      boff[m][u] = (set * 16 + (tap / 3) * Cfg::INW + tap % 3) * 8;
    }
  }
  const int my_set = (4 * g) / Cfg::C0M, cbase = (4 * g) % Cfg::C0M;  // rows of D this lane holds
  unsigned char* l0w = l0 + ((cbase >> 3) * Cfg::L0H * 2 * Cfg::L0P) * 16 + (cbase & 7) * 2;
  // second-conv weights: k = tap*C0 + c; lane g of k-step m holds k = 32m + 8g .. +7
  h8 a1[Cfg::NT1][Cfg::KS1];
  int roff[Cfg::KS1];  // LDS byte offset of this lane's 8-channel chunk relative to pixel (0, 0)
#pragma unroll
  for (int m = 0; m < Cfg::KS1; ++m) {
    const int k0 = 32 * m + 8 * g;
    const int tap = k0 / C0, c = k0 % C0;
    const int tp = min(tap, 8), ky = tp / 3, kx = tp % 3;
    // pixel (j, i) tap (ky, kx) -> row 2j + ky, column 2i + kx -> parity kx & 1, index i + (kx >> 1)
    roff[m] = (((c >> 3) * Cfg::L0H + ky) * 2 * Cfg::L0P + (kx & 1) * Cfg::L0P + (kx >> 1)) * 16;
#pragma unroll
    for (int t = 0; t < Cfg::NT1; ++t) a1[t][m] = w1f[(t * Cfg::KS1 + m) * 64 + lane];
  }
  float bias1[Cfg::NT1][4];
#pragma unroll
  for (int t = 0; t < Cfg::NT1; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) bias1[t][q] = b1[16 * t + 4 * g + q];

  ST_STAMP(0);
#ifdef YDBL_STEM2_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_st_stamps[blockIdx.x * 8 + 4] = hw;
    g_st_stamps[blockIdx.x * 8 + 5] = xcc;
  }
#endif
  const Tile tl = tile_of(blockIdx.x);
  load_window(tl, std::integral_constant<bool, BOUND>{});
  {
    store_window();
    __syncthreads();
    ST_STAMP(1);
    // workgroups whose first-conv window lies inside the image skip the per-pixel padding test
    const bool interior = tl.Y0 >= 0 && tl.X0 >= 0 && tl.Y0 + Cfg::L0H <= H && tl.X0 + Cfg::L0W <= W;

    // ---- 2. first conv, 16 * PS pixels per MFMA group (bias folded into the MFMA: record slot 3); interior tiles
    // run a copy of the loop without the per-pixel padding test
    constexpr int P0V = Cfg::L0H * Cfg::INW;
    const unsigned char* inb = reinterpret_cast<const unsigned char*>(in);
    auto conv1 = [&](auto interior_c) {
      constexpr bool INTERIOR = decltype(interior_c)::value;
      // this lane's output pixel p = pt * 16 * PS + 16 * my_set + r16 of the virtual grid, its (row, column) and
      // record row base walked incrementally (one division before the loop, none in it)
      constexpr int STEP = 4 * 16 * PS, DR = STEP / Cfg::INW, DC = STEP % Cfg::INW;
      static_assert(STEP < 2 * Cfg::INW, "one row wrap per step at most");
      int p = wave * 16 * PS + my_set * 16 + r16;
      int lr = p / Cfg::INW, lc = p - lr * Cfg::INW;
      int rb = lr * 2 * Cfg::L0P;
      for (int pt = wave; pt * 16 * PS < P0V; pt += 4) {
        const int p0 = pt * 16 * PS + r16;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < KS0; ++m) {
          const h4 lo = *reinterpret_cast<const h4*>(inb + p0 * 8 + boff[m][0]);
          const h4 hi = *reinterpret_cast<const h4*>(inb + p0 * 8 + boff[m][1]);
          const h8 bf = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[m], bf, acc, 0, 0, 0);
        }
        if (p < P0V && lc < Cfg::L0W) {
          h4 hv;
          if constexpr (INTERIOR) {
#pragma unroll
            for (int q = 0; q < 4; ++q) hv[q] = f16_rne(silu_fast(acc[q]));
          } else {
            const int iy = tl.Y0 + lr, ix = tl.X0 + lc;
            const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float sv = silu_fast(acc[q]);
              hv[q] = f16_rne(inside ? sv : 0.f);
            }
          }
          const int rec = rb + (lc & 1) * Cfg::L0P + (lc >> 1);
          *reinterpret_cast<h4*>(l0w + rec * 16) = hv;
        }
        p += STEP;
        lc += DC;
        lr += DR;
        rb += DR * 2 * Cfg::L0P;
        const bool wrap = lc >= Cfg::INW;
        lc -= wrap ? Cfg::INW : 0;
        lr += wrap ? 1 : 0;
        rb += wrap ? 2 * Cfg::L0P : 0;
      }
    };
    if (interior) conv1(std::true_type{});
    else conv1(std::false_type{});
    __syncthreads();
    ST_STAMP(2);

    // ---- 3. second conv: TH rows x TW cols, 16-pixel row segments
    constexpr int SEG = TW / 16;
    const int64_t lane_px = (int64_t)r16 * y.cs;
    for (int st = wave; st < TH * SEG; st += 4) {
      const int j = st / SEG, i = (st - j * SEG) * 16 + r16;
      const unsigned char* pbase = l0 + ((2 * j) * 2 * Cfg::L0P + i) * 16;
      f32x4 acc[Cfg::NT1];
#pragma unroll
      for (int q = 0; q < Cfg::NT1; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < Cfg::KS1; ++m) {
        const h8 bf = *reinterpret_cast<const h8*>(pbase + roff[m]);
#pragma unroll
        for (int q = 0; q < Cfg::NT1; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[q][m], bf, acc[q], 0, 0, 0);
      }
      const int oy = tl.oy0 + j, ox = tl.ox0 + i;
      if (oy >= y.h || ox >= y.w) continue;
      // segment base wave-uniform (scalar address arithmetic) + this lane's pixel
      _Float16* yp = y.at(tl.img, oy, tl.ox0 + (st - j * SEG) * 16) + lane_px;
#pragma unroll
      for (int q = 0; q < Cfg::NT1; ++q) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = silu_fast(acc[q][e] + bias1[q][e]);
        store_f<4>(yp + 16 * q + 4 * g, o);
      }
    }
  }
  ST_STAMP(3);
}

}  // namespace ydbl

using namespace ydbl;

#ifdef YDBL_STEM2_STAMPS
extern "C" int ydbl_stem2_debug_stamps(unsigned long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_st_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
extern "C" int ydbl_stem2_debug_reset() {
  static unsigned long long zeros[8 * 16384];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_st_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t ydbl_conv_stem2_params_size(int32_t c0) {
  if (c0 == 8) return Stem2Cfg<8, 32, 8>::BYTES;
  if (c0 == 16) return Stem2Cfg<16, 32, 8>::BYTES;
  return -1;
}

extern "C" int ydbl_conv_stem2_pack(const float* w0, const float* b0, const float* w1, const float* b1, int32_t c0,
                                    void* out) {
  if (!w0 || !b0 || !w1 || !b1 || !out) return fail(YDBL_EINVAL, "stem2_pack: null pointer");
  auto* o = reinterpret_cast<unsigned char*>(out);
  if (c0 == 8) { stem2_pack<8>(w0, b0, w1, b1, o); return 0; }
  if (c0 == 16) { stem2_pack<16>(w0, b0, w1, b1, o); return 0; }
  return fail(YDBL_EINVAL, "stem2_pack: c0 must be 8 or 16");
}

extern "C" int ydbl_conv_stem2(const ydbl_stem2_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "stem2: null descriptor");
  if (!d->x || !d->params) return fail(YDBL_EINVAL, "stem2: null input/parameters");
  if (!d->bind.x != !d->bind.amax) return fail(YDBL_EINVAL, "stem2: input binding with a null pointer");
  if (check_view(&d->y, "stem2.y", true)) return YDBL_EINVAL;
  if (d->y.dtype != YDBL_F16) return fail(YDBL_EINVAL, "stem2: fp16 activations only");
  if (d->cin != 3) return fail(YDBL_EINVAL, "stem2: cin must be 3");
  const int c0 = d->c0, c1 = d->y.c;
  if (c1 != 2 * c0) return fail(YDBL_EINVAL, "stem2: second conv must have 2 * c0 output channels");
  if (d->n < 1 || d->h < 1 || d->w < 1) return fail(YDBL_EINVAL, "stem2: empty input");
  const int ho = (d->h - 1) / 2 + 1, wo = (d->w - 1) / 2 + 1;
  if (d->y.n != d->n || d->y.h != ho || d->y.w != wo) return fail(YDBL_EINVAL, "stem2: output shape mismatch");
  hipStream_t s = as_stream(stream);
  auto go = [&](auto kern, int tw, int th, int lds) {
    const int tiles_x = (wo + tw - 1) / tw, tiles_y = (ho + th - 1) / th;
    const int64_t nb = (int64_t)tiles_x * tiles_y * d->n;
    if (nb > 0x7fffffff) return fail(YDBL_EINVAL, "stem2: grid too large");
    kern<<<(unsigned)nb, 256, lds, s>>>(d->x, d->h, d->w, d->scale, reinterpret_cast<const unsigned char*>(d->params),
                                        dview<_Float16>(d->y), tiles_x, tiles_y, (int)nb, input_bind(&d->bind));
    return check_launch("ydbl_conv_stem2");
  };
  const bool v4 = d->w % 4 == 0 && (reinterpret_cast<uintptr_t>(d->x) & 15) == 0;
  const bool bound = d->bind.x != nullptr;
#define YDBL_STEM2_GO(C0_, TH_)                                                                                     \
  {                                                                                                                  \
    if (bound)                                                                                                       \
      return v4 ? go(stem2_kernel<C0_, 32, TH_, true, true>, 32, TH_, Stem2Cfg<C0_, 32, TH_>::LDS)                 \
                : go(stem2_kernel<C0_, 32, TH_, false, true>, 32, TH_, Stem2Cfg<C0_, 32, TH_>::LDS);               \
    return v4 ? go(stem2_kernel<C0_, 32, TH_, true, false>, 32, TH_, Stem2Cfg<C0_, 32, TH_>::LDS)                  \
              : go(stem2_kernel<C0_, 32, TH_, false, false>, 32, TH_, Stem2Cfg<C0_, 32, TH_>::LDS);                \
  }
  if (c0 == 8) YDBL_STEM2_GO(8, 8)
  if (c0 == 16) YDBL_STEM2_GO(16, 8)
#undef YDBL_STEM2_GO
  return fail(YDBL_EINVAL, "stem2: c0 must be 8 or 16");
}
