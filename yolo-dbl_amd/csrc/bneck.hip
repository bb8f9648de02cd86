// Fused Bottleneck (fp16): y = x + SiLU(conv3x3(SiLU(conv3x3(x) + b1)) + b2)   (add = shortcut && c1 == c2)
// U/nn/modules/block.py:344-357 with Conv = conv + folded BN + SiLU (U/nn/modules/conv.py:39-63).
//
// The DBL backbones run chains of Bottleneck(C, C, e=0.5) at high resolution (DBL-n: C=16 @320^2,
// 32 @160^2, 4x 64 @80^2).  As two launches the C/2-channel intermediate is written to HBM and read
// back, and each 3x3 conv stages its own input; the pair is ~0.45 ms of DBL-n's 2.8 ms step.  Here a
// workgroup owns a TH x 16 output tile and all C output channels:
//   1. the (TH+4) x 20 input window, all C channels, is staged once in LDS (16-byte records, one plane
//      per 8-channel chunk; the lane -> (pixel, chunk) order gives 1 KiB contiguous global reads per
//      wave and conflict-free ds_write_b128 groups);
//   2. cv1 over the (TH+2) x 18 intermediate window on MFMA 16x16x32 f16, walked as a virtual grid with
//      the input's 20-record pitch (the two dead columns per row cost 11 %, and a lane's B address is
//      its pixel index plus a per-k-step constant), + bias + SiLU, zero outside the image (cv2's
//      padding), rounded to fp16 exactly as the unfused path stores it -> LDS;
//   3. cv2 over the TH x 16 tile from that LDS window, + bias + SiLU, + x (read back from the staged
//      input window), -> NHWC fp16.
// Weights never touch LDS: each wave keeps the MFMA A fragments of its output-channel tile in VGPRs
// (one 1 KiB coalesced load per k-step, every weight read once per workgroup).
// K order per 32-wide k-step (lane group g = lane / 16 supplies k = 8g..8g+7): chosen per channel
// count so that the two lane groups a ds_read_b128 services together ({g0, g1}, {g2, g3}) read from
// addresses 256 B apart (same bank quad offset): for >= 32 channels a k-step is one tap x 4 chunks, for
// 16 channels two taps x 2 chunks, for 8 channels four taps paired by equal dx (planes/pitches are
// multiples of 16 records).  Pack (host) and kernel share kslot().
// HBM traffic: x once (+ the 4-row halo, mostly L2 hits), y once; the intermediate never leaves LDS.
#include <algorithm>

#include "common.hpp"

namespace ydbl {

struct KSlot {
  int tap, chunk;
  bool live;
};

// k-step m, lane group g -> (tap = dy*3 + dx, 8-channel chunk, live); dead slots carry zero weights
// and point at a live address (finite data, broadcast reads)
template <int CH>
__host__ __device__ constexpr KSlot kslot(int m, int g) {
  if constexpr (CH >= 4) {
    return KSlot{m / (CH / 4), (m % (CH / 4)) * 4 + g, true};
  } else if constexpr (CH == 2) {
    const int tap = 2 * m + (g >> 1);
    return KSlot{tap < 9 ? tap : 8, g & 1, tap < 9};
  } else {
    // {g0,g1} and {g2,g3} share dx: (0,0)(1,0)|(0,1)(1,1), (0,2)(1,2)|(2,0)(2,0)', (2,1)(2,1)'|(2,2)(2,2)'
    constexpr int taps[3][4] = {{0, 3, 1, 4}, {2, 5, 6, 6}, {7, 7, 8, 8}};
    constexpr bool live[3][4] = {{true, true, true, true}, {true, true, true, false}, {true, false, true, false}};
    return KSlot{taps[m][g], 0, live[m][g]};
  }
}
template <int CH>
constexpr int ksteps() {
  return CH >= 4 ? 9 * CH / 4 : (CH == 2 ? 5 : 3);
}
constexpr int rup16(int v) { return (v + 15) / 16 * 16; }

template <int C, int CMID, int TH, int CIN = C>
struct BneckCfg {
  static constexpr int CM = CMID, CH = CIN / 8, CHM = (CM + 7) / 8;  // CH: 8-channel chunks of the input
  static constexpr int NT1 = (CM + 15) / 16, NT2 = C / 16;
  // BD (8-channel intermediate of a 16-channel input): cv1's 16 MFMA rows are two pixel sets x 8 channels through a
  // block-diagonal A (rows 0-7 see set 0's K slots, rows 8-15 set 1's), so no D row is dead; k-step m = tap m,
  // lane group g = (set g / 2, chunk g % 2)
  static constexpr bool BD = CM == 8 && CH == 2;
  static constexpr int KS1 = BD ? 9 : ksteps<CH>(), KS2 = ksteps<CHM>();
  static constexpr int TW = 16;
  static constexpr int IP = TW + 4;                  // input window pitch (records) = its width
  static constexpr int IR = TH + 5;                  // + 1 slack row for the virtual grid's tail
  static constexpr int NPX = IR * IP;
  static constexpr int PIN = rup16(NPX);             // chunk plane, records (multiple of 16: 256 B)
  static constexpr int MR = TH + 2;
  static constexpr int MP = CHM == 1 ? 32 : IP;      // 8-channel intermediate: pitch a multiple of 16
  static constexpr int PMID = rup16(MR * MP);
  static constexpr int G1 = (MR * IP + 15) / 16;     // 16-pixel groups of the cv1 virtual grid
  static constexpr int IN_BYTES = CH * PIN * 16, MID_BYTES = CHM * PMID * 16;
  static constexpr int LDS = IN_BYTES + MID_BYTES;
  static constexpr int W1F = NT1 * KS1 * 64, W2F = NT2 * KS2 * 64;  // h8 fragments
  static constexpr int64_t BYTES = (int64_t)(W1F + W2F) * 16 + (NT1 * 16 + C) * 4;
  static_assert(CH >= 2, "input needs >= 16 channels");
  static_assert((G1 * 16 - 1) + 2 * IP + 2 < NPX, "virtual grid tail must stay inside the window");
};

// Host: fp32 PyTorch-layout weights (BN folded) -> fragment blob.  A[row][k]: row = output channel of
// the 16-channel tile, k = 32m + 8g + j -> (kslot(m, g), channel chunk*8 + j).
template <int C, int CMID, int CIN = C>
void bneck_pack(const float* w1, const float* b1, const float* w2, const float* b2, unsigned char* out) {
  using Cfg = BneckCfg<C, CMID, 16, CIN>;
  constexpr int CM = Cfg::CM;
  _Float16* f1 = reinterpret_cast<_Float16*>(out);
  _Float16* f2 = f1 + Cfg::W1F * 8;
  float* fb1 = reinterpret_cast<float*>(f2 + Cfg::W2F * 8);
  float* fb2 = fb1 + Cfg::NT1 * 16;
  if constexpr (Cfg::BD) {
    for (int m = 0; m < Cfg::KS1; ++m)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int g = lane >> 4, row = lane & 15;
          const int co = row % 8, ci = (g & 1) * 8 + j;
          f1[(m * 64 + lane) * 8 + j] = (_Float16)((row / 8) == (g >> 1) ? w1[(co * CIN + ci) * 9 + m] : 0.f);
        }
  } else
  for (int t = 0; t < Cfg::NT1; ++t)
    for (int m = 0; m < Cfg::KS1; ++m)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const KSlot s = kslot<Cfg::CH>(m, lane >> 4);
          const int co = 16 * t + (lane & 15), ci = s.chunk * 8 + j;
          const bool ok = s.live && co < CM;
          f1[((t * Cfg::KS1 + m) * 64 + lane) * 8 + j] = (_Float16)(ok ? w1[(co * CIN + ci) * 9 + s.tap] : 0.f);
        }
  for (int t = 0; t < Cfg::NT2; ++t)
    for (int m = 0; m < Cfg::KS2; ++m)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const KSlot s = kslot<Cfg::CHM>(m, lane >> 4);
          const int co = 16 * t + (lane & 15), ci = s.chunk * 8 + j;
          const bool ok = s.live && ci < CM;
          f2[((t * Cfg::KS2 + m) * 64 + lane) * 8 + j] = (_Float16)(ok ? w2[(co * CM + ci) * 9 + s.tap] : 0.f);
        }
  for (int i = 0; i < Cfg::NT1 * 16; ++i) fb1[i] = i < CM ? b1[i] : 0.f;
  for (int i = 0; i < C; ++i) fb2[i] = b2[i];
}

// per-k-step LDS byte offset of lane group g's slot relative to its pixel record (PL = chunk plane,
// P = pitch, both in records); g-independent except for the lane base chunk when CH >= 4
template <int CH, int PL, int P>
__device__ __forceinline__ int koff(int m, int g) {
  const KSlot s = kslot<CH>(m, CH >= 4 ? 0 : g);
  return (s.chunk * PL + (s.tap / 3) * P + s.tap % 3) * 16;
}
template <int CH, int PL>
__device__ __forceinline__ int kbase(int g) {
  return CH >= 4 ? g * PL * 16 : 0;
}

// Diagnostic build only (-DYDBL_BNECK_STAMPS, scripts/phase_stamps.py): per-workgroup s_memrealtime stamps (100 MHz)
// when wave 0 starts, has staged the window, has finished cv1, has stored cv2; plus the hardware ids.
#ifdef YDBL_BNECK_STAMPS
__device__ unsigned long long g_bn_stamps[8 * 16384];
#define BN_STAMP(k)                                                                                         \
  do {                                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_bn_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define BN_STAMP(k) \
  do {              \
  } while (0)
#endif

template <int C, int CMID, int TH, bool ADD, bool PW = false, int CIN = C>
__global__ __launch_bounds__(256, 2) void bneck_kernel(DView<const _Float16> x, DView<_Float16> y,
                                                       const unsigned char* __restrict__ params, int tiles_x,
                                                       int tiles_y, int ntiles) {
  using Cfg = BneckCfg<C, CMID, TH, CIN>;
  constexpr int CH = Cfg::CH, CHM = Cfg::CHM, CM = Cfg::CM;
  static_assert(CIN == C || !ADD, "the residual needs c_in == c");
  constexpr bool LATE_A2 = CIN > C;  // deep input: cv2's A fragments are loaded after cv1 (VGPR budget)
  constexpr int IP = Cfg::IP, MP = Cfg::MP, PIN = Cfg::PIN, PMID = Cfg::PMID;
  constexpr int NT1 = Cfg::NT1, NT2 = Cfg::NT2, KS1 = Cfg::KS1, KS2 = Cfg::KS2;
  const h8* w1f = reinterpret_cast<const h8*>(params);
  const h8* w2f = w1f + Cfg::W1F;
  const float* b1 = reinterpret_cast<const float*>(w2f + Cfg::W2F);
  const float* b2 = b1 + NT1 * 16;
  __shared__ __align__(16) unsigned char smem[Cfg::LDS];
  unsigned char* s_in = smem;                    // [CH][PIN] records
  unsigned char* s_mid = smem + Cfg::IN_BYTES;   // [CHM][PMID] records

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int g = lane >> 4, r16 = lane & 15;
  BN_STAMP(0);
#ifdef YDBL_BNECK_STAMPS
  if (tid == 0 && blockIdx.x < 16384) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_bn_stamps[blockIdx.x * 8 + 4] = hw;
    g_bn_stamps[blockIdx.x * 8 + 5] = xcc;
  }
#endif
  const int t = (ntiles & 7) ? (int)blockIdx.x : xcd_remap(blockIdx.x, ntiles);
  const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y;
  const int img = t / (tiles_x * tiles_y);
  const int oy0 = ty * TH, ox0 = tx * Cfg::TW;

  // ---- 1. input window (image rows oy0-2.., cols ox0-2..).  Item i = u*256 + tid -> chunk
  // (i >> 3) % CH (the same for every u: CH divides 32), pixel px0 + u * 256/CH: each wave reads
  // 1 KiB of contiguous NHWC pixels per instruction, each 8-lane ds_write_b128 group 8 records
  static_assert(32 % CH == 0, "staging pattern assumes CH | 32");
  constexpr int PXU = 256 / CH;
  constexpr int IT = (Cfg::NPX + PXU - 1) / PXU;
  const int s_chunk = (tid >> 3) % CH, px0 = ((tid >> 3) / CH) * 8 + (tid & 7);
  h8 xr[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int px = px0 + u * PXU;
    const int r = px / IP, c = px - r * IP;
    const int iy = oy0 - 2 + r, ix = ox0 - 2 + c;
    const bool ok = px < Cfg::NPX && iy >= 0 && iy < x.h && ix >= 0 && ix < x.w;
    const _Float16* src = ok ? x.at(img, iy, ix) + s_chunk * 8 : x.p;
    const h8 v = *reinterpret_cast<const h8*>(src);
    xr[u] = ok ? v : h8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  // this wave's weight tiles, VGPR-resident
  const int t1 = wave % NT1, t2 = wave % NT2;
  h8 a1[KS1], a2[KS2];
#pragma unroll
  for (int m = 0; m < KS1; ++m) a1[m] = w1f[(t1 * KS1 + m) * 64 + lane];
  if constexpr (!LATE_A2) {
#pragma unroll
    for (int m = 0; m < KS2; ++m) a2[m] = w2f[(t2 * KS2 + m) * 64 + lane];
  }
  unsigned char* s_dst = s_in + (s_chunk * PIN + px0) * 16;
#pragma unroll
  for (int u = 0; u < IT; ++u)
    if (px0 + u * PXU < Cfg::NPX) *reinterpret_cast<h8*>(s_dst + u * PXU * 16) = xr[u];
  float bias1[4], bias2[4];
  const int c1 = Cfg::BD ? 4 * (g & 1) : 16 * t1 + 4 * g;  // first intermediate channel of this lane's cv1 D rows
  const int c2 = 16 * t2 + 4 * g;  // first output channel of this lane's cv2 D rows
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bias1[q] = b1[c1 + q];
    bias2[q] = b2[c2 + q];
  }
  unsigned char* mid_w = s_mid + ((c1 >> 3) * PMID) * 16 + (c1 & 7) * 2;
  const unsigned char* in_b = s_in + kbase<CH, PIN>(g);
  const bool interior = oy0 >= 1 && ox0 >= 1 && oy0 + TH + 1 <= y.h && ox0 + Cfg::TW + 1 <= y.w;
  __syncthreads();
  BN_STAMP(1);

  // ---- 2. cv1 over the virtual grid: MR rows x IP columns, mid pixel v reads input record v + tap.
  // Two 16-pixel groups per iteration (independent accumulators: the LDS reads of one overlap the
  // MFMAs of the other, and the two SiLU epilogues interleave)
  auto epi1 = [&](const f32x4& acc, int vr, int vc, int rb) {
    if (vr >= Cfg::MR || c1 >= CM) return;
    bool inside = true;
    if (!interior) {
      const int my = oy0 - 1 + vr, mx = ox0 - 1 + vc;
      inside = my >= 0 && my < y.h && mx >= 0 && mx < y.w;
    }
    h4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float sv = silu_fast(acc[q] + bias1[q]);  // computed unconditionally: a select, not a branch per value
      o[q] = f16_rne(inside ? sv : 0.f);
    }
    *reinterpret_cast<h4*>(mid_w + (rb + vc) * 16) = o;
  };
  constexpr int WPT1 = 4 / NT1;
  // the two groups' virtual-grid (row, column) and intermediate row base, walked incrementally (no division
  // or 32-bit multiply in the loop): group 0 advances S0 pixels per iteration, group 1 sits H1 pixels after it
  constexpr int S0 = 2 * WPT1 * 16, H1 = WPT1 * 16;
  int r0, c0, rb0;
  {
    const int v = (wave / NT1) * 16 + r16;
    r0 = v / IP;
    c0 = v - r0 * IP;
    rb0 = r0 * MP;
  }
  for (int gi = wave / NT1; gi < Cfg::G1; gi += 2 * WPT1) {
    const int v0 = gi * 16 + r16;
    const bool two = gi + WPT1 < Cfg::G1;  // wave-uniform
    const int v1 = two ? v0 + 16 * WPT1 : v0;
    if constexpr (Cfg::BD) {
      // one accumulator for both groups: lane group g reads set g / 2's pixel, chunk g % 2, at tap m
      const int set = g >> 1;
      const unsigned char* pb = s_in + ((g & 1) * PIN + (set ? v1 : v0)) * 16;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < KS1; ++m) {
        const h8 bf = *reinterpret_cast<const h8*>(pb + ((m / 3) * IP + m % 3) * 16);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[m], bf, acc, 0, 0, 0);
      }
      // one epilogue for both sets (per-lane position select, not a branch per set); set 1 of a single-group
      // iteration duplicates group 0 and is skipped through an out-of-range row
      const bool w1 = c0 + H1 % IP >= IP;
      const int dr = set ? H1 / IP + (w1 ? 1 : 0) : 0;
      epi1(acc, set && !two ? Cfg::MR : r0 + dr, set ? c0 + H1 % IP - (w1 ? IP : 0) : c0, rb0 + dr * MP);
    } else {
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      const unsigned char* p0 = in_b + v0 * 16;
      const unsigned char* p1 = in_b + v1 * 16;
#pragma unroll
      for (int m = 0; m < KS1; ++m) {
        const int o = koff<CH, PIN, IP>(m, g);
        const h8 bf0 = *reinterpret_cast<const h8*>(p0 + o);
        const h8 bf1 = *reinterpret_cast<const h8*>(p1 + o);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[m], bf0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[m], bf1, acc1, 0, 0, 0);
      }
      epi1(acc0, r0, c0, rb0);
      if (two) {
        const bool w1 = c0 + H1 % IP >= IP;
        const int dr = H1 / IP + (w1 ? 1 : 0);
        epi1(acc1, r0 + dr, c0 + H1 % IP - (w1 ? IP : 0), rb0 + dr * MP);
      }
    }
    const bool w0 = c0 + S0 % IP >= IP;
    const int dr = S0 / IP + (w0 ? 1 : 0);
    c0 += S0 % IP - (w0 ? IP : 0);
    r0 += dr;
    rb0 += dr * MP;
  }

  const unsigned char* res_r = s_in + ((c2 >> 3) * PIN + 2 * IP + 2) * 16 + (c2 & 7) * 2;
  const unsigned char* mid_b = s_mid + kbase<CHM, PMID>(g);
  if constexpr (LATE_A2) {
#pragma unroll
    for (int m = 0; m < KS2; ++m) a2[m] = w2f[(t2 * KS2 + m) * 64 + lane];
  }
  __syncthreads();
  BN_STAMP(2);

  // ---- 3. cv2: output rows j, j + WPT2 of the tile, 16 columns = the 16 lanes
  const int64_t lane_px = (int64_t)r16 * y.cs;  // this lane's pixel offset from the row's first column
  auto epi2 = [&](const f32x4& acc, int j) {
    const int oy = oy0 + j, ox = ox0 + r16;
    if (oy >= y.h || ox >= y.w) return;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = silu_fast(acc[q] + bias2[q]);
    if constexpr (ADD) {
      const h4 rv = *reinterpret_cast<const h4*>(res_r + (j * IP + r16) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = float(rv[q]) + v[q];
    }
    if constexpr (PW) {  // cv2 output, rounded to fp16 as the unfused path stores it, -> LDS for the 1x1
      h4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = f16_rne(v[q]);
      *reinterpret_cast<h4*>(s_in + ((c2 >> 3) * (TH * 16) + j * 16 + r16) * 16 + (c2 & 7) * 2) = o;
    } else {
      store_f<4>(y.at(img, oy, ox0) + lane_px + c2, v);  // row base wave-uniform (scalar address arithmetic)
    }
  };
  constexpr int WPT2 = 4 / NT2;
  for (int j = wave / NT2; j < TH; j += 2 * WPT2) {
    const bool two = j + WPT2 < TH;
    const int j1 = two ? j + WPT2 : j;
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const unsigned char* p0 = mid_b + (j * MP + r16) * 16;
    const unsigned char* p1 = mid_b + (j1 * MP + r16) * 16;
#pragma unroll
    for (int m = 0; m < KS2; ++m) {
      const int o = koff<CHM, PMID, MP>(m, g);
      const h8 bf0 = *reinterpret_cast<const h8*>(p0 + o);
      const h8 bf1 = *reinterpret_cast<const h8*>(p1 + o);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[m], bf0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[m], bf1, acc1, 0, 0, 0);
    }
    epi2(acc0, j);
    if (two) epi2(acc1, j1);
  }
  BN_STAMP(3);

  if constexpr (PW) {
    // ---- 4. trailing 1x1 conv C -> C + bias (Detect box branch cv2[i][2], head.py:86-90) over the
    // TH x 16 cv2 tile now in LDS (C/8 planes of TH*16 records, in the input window's space)
    static_assert(ADD == false && C % 32 == 0 && (C / 8) * TH * 16 * 16 <= Cfg::IN_BYTES, "pw stage layout");
    constexpr int NT3 = C / 16, KS3 = C / 32, WPT3 = 4 / NT3;
    const h8* w3f = reinterpret_cast<const h8*>(b2 + C);
    const float* b3 = reinterpret_cast<const float*>(w3f + NT3 * KS3 * 64);
    const int t3 = wave % NT3, c3 = 16 * t3 + 4 * g;
    h8 a3[KS3];
#pragma unroll
    for (int m = 0; m < KS3; ++m) a3[m] = w3f[(t3 * KS3 + m) * 64 + lane];
    float bias3[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bias3[q] = b3[c3 + q];
    __syncthreads();
    for (int j = wave / NT3; j < TH; j += WPT3) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < KS3; ++m) {
        const h8 bf = *reinterpret_cast<const h8*>(s_in + ((m * 4 + g) * (TH * 16) + j * 16 + r16) * 16);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3[m], bf, acc, 0, 0, 0);
      }
      const int oy = oy0 + j, ox = ox0 + r16;
      if (oy < y.h && ox < y.w) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = acc[q] + bias3[q];
        store_f<4>(y.at(img, oy, ox) + c3, v);
      }
    }
  }
}

}  // namespace ydbl

using namespace ydbl;

// (c, c_mid) pairs built: the backbone Bottleneck(c, c, e=0.5) chains and the Detect head's box
// branch cv2[i][0:2] = Conv(64, 64, 3) -> Conv(64, 64, 3) (head.py:86-90, no shortcut).
static int64_t pair_bytes(int c, int cm) {
  if (c == 16 && cm == 8) return BneckCfg<16, 8, 16>::BYTES;
  if (c == 32 && cm == 16) return BneckCfg<32, 16, 16>::BYTES;
  if (c == 64 && cm == 32) return BneckCfg<64, 32, 16>::BYTES;
  if (c == 64 && cm == 64) return BneckCfg<64, 64, 16>::BYTES;
  return -1;
}

#ifdef YDBL_BNECK_STAMPS
extern "C" int ydbl_bneck_debug_stamps(unsigned long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bn_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
extern "C" int ydbl_bneck_debug_reset() {
  static unsigned long long zeros[8 * 16384];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_bn_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t ydbl_bottleneck_params_size(int32_t c) { return pair_bytes(c, c / 2); }
extern "C" int64_t ydbl_conv3x3_pair_params_size(int32_t c, int32_t c_mid) { return pair_bytes(c, c_mid); }

extern "C" int ydbl_conv3x3_pair_pack(const float* w1, const float* b1, const float* w2, const float* b2, int32_t c,
                                      int32_t c_mid, void* out) {
  if (!w1 || !b1 || !w2 || !b2 || !out) return fail(YDBL_EINVAL, "bottleneck_pack: null pointer");
  auto* o = reinterpret_cast<unsigned char*>(out);
  if (c == 16 && c_mid == 8) { bneck_pack<16, 8>(w1, b1, w2, b2, o); return 0; }
  if (c == 32 && c_mid == 16) { bneck_pack<32, 16>(w1, b1, w2, b2, o); return 0; }
  if (c == 64 && c_mid == 32) { bneck_pack<64, 32>(w1, b1, w2, b2, o); return 0; }
  if (c == 64 && c_mid == 64) { bneck_pack<64, 64>(w1, b1, w2, b2, o); return 0; }
  return fail(YDBL_EINVAL, "bottleneck_pack: (c, c_mid) must be (16, 8), (32, 16), (64, 32) or (64, 64)");
}

// Detect box branch: the (c_in -> 64 -> 64) pair blob + the trailing 1x1's A fragments (k = 32m + 8g + j
// -> input channel, row = output channel) and its fp32 bias.  c_in 64 (P3 of DBL-n), 128 (P4).
template <int CIN>
static int64_t box_bytes() {
  return BneckCfg<64, 64, 16, CIN>::BYTES + (64 / 16) * (64 / 32) * 64 * 16 + 64 * 4;
}

extern "C" int64_t ydbl_detect_box_params_size(int32_t c_in, int32_t c) {
  if (c != 64) return -1;
  if (c_in == 64) return box_bytes<64>();
  if (c_in == 128) return box_bytes<128>();
  return -1;
}

template <int CIN>
static void box_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                     const float* b3, unsigned char* out) {
  bneck_pack<64, 64, CIN>(w1, b1, w2, b2, out);
  _Float16* f3 = reinterpret_cast<_Float16*>(out + BneckCfg<64, 64, 16, CIN>::BYTES);
  constexpr int NT3 = 4, KS3 = 2;
  for (int t = 0; t < NT3; ++t)
    for (int m = 0; m < KS3; ++m)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int co = 16 * t + (lane & 15), ci = (m * 4 + (lane >> 4)) * 8 + j;
          f3[((t * KS3 + m) * 64 + lane) * 8 + j] = (_Float16)w3[co * 64 + ci];
        }
  float* fb3 = reinterpret_cast<float*>(f3 + NT3 * KS3 * 64 * 8);
  for (int i = 0; i < 64; ++i) fb3[i] = b3[i];
}

extern "C" int ydbl_detect_box_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                                    const float* b3, int32_t c_in, int32_t c, void* out) {
  if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !out) return fail(YDBL_EINVAL, "detect_box_pack: null pointer");
  if (c != 64 || (c_in != 64 && c_in != 128)) return fail(YDBL_EINVAL, "detect_box_pack: (c_in, c) must be (64|128, 64)");
  auto* o = reinterpret_cast<unsigned char*>(out);
  if (c_in == 64) box_pack<64>(w1, b1, w2, b2, w3, b3, o);
  else box_pack<128>(w1, b1, w2, b2, w3, b3, o);
  return 0;
}

extern "C" int ydbl_bottleneck_pack(const float* w1, const float* b1, const float* w2, const float* b2, int32_t c,
                                    void* out) {
  return ydbl_conv3x3_pair_pack(w1, b1, w2, b2, c, c / 2, out);
}

template <int C, int CMID, int TH, bool PW = false, int CIN = C>
static int bneck_go(const ydbl_bottleneck_desc* d, hipStream_t s) {
  using Cfg = BneckCfg<C, CMID, TH, CIN>;
  const int tiles_x = (int)cdiv(d->y.w, Cfg::TW), tiles_y = (int)cdiv(d->y.h, TH);
  const int64_t nt = (int64_t)tiles_x * tiles_y * d->y.n;
  if (nt > 0x7fffffff) return fail(YDBL_EINVAL, "bottleneck: grid too large");
  auto x = dview<const _Float16>(d->x);
  auto y = dview<_Float16>(d->y);
  auto* p = reinterpret_cast<const unsigned char*>(d->params);
  if constexpr (PW)
    bneck_kernel<C, CMID, TH, false, true, CIN><<<(unsigned)nt, 256, 0, s>>>(x, y, p, tiles_x, tiles_y, (int)nt);
  else if (d->add)
    bneck_kernel<C, CMID, TH, true><<<(unsigned)nt, 256, 0, s>>>(x, y, p, tiles_x, tiles_y, (int)nt);
  else
    bneck_kernel<C, CMID, TH, false><<<(unsigned)nt, 256, 0, s>>>(x, y, p, tiles_x, tiles_y, (int)nt);
  return check_launch("ydbl_bottleneck_nhwc");
}

// workgroups of a bneck_kernel instantiation resident per CU x the CUs (queried once per instantiation)
template <int C, int CMID, int TH>
static int64_t bneck_slots() {
  static int64_t slots = [] {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, bneck_kernel<C, CMID, TH, true>, 256, 0) != hipSuccess)
      return (int64_t)0;
    return (int64_t)cus * per;
  }();
  return slots;
}

template <int C, int CMID>
static int bneck_dispatch(const ydbl_bottleneck_desc* d, hipStream_t s) {
  // 16-row tiles halve the halo recompute; 8-row tiles when 16-row ones leave the chip under-filled
  // (and always for c_mid = 64: its 16-row tile would need 102 KB of LDS, one workgroup per CU)
  const int64_t t16 = cdiv(d->y.h, 16) * cdiv(d->y.w, 16) * (int64_t)d->y.n;
  int th = d->tile_h ? d->tile_h : (t16 >= 1024 && CMID < 64 ? 16 : 8);
  if constexpr (C == 64 && CMID == 32) {
    // 9-row tiles (51 KB of LDS: still 3 workgroups per CU) when they take fewer rounds of the resident
    // workgroups: DBL-n's 80^2 Bottlenecks at bs16 are 800 8-row tiles on 768 slots -- a second round of 32 --
    // and 720 9-row ones in one (a round priced by its cv1 rows, TH + 2)
    if (!d->tile_h && th == 8) {
      const int64_t s8 = bneck_slots<C, CMID, 8>(), s9 = bneck_slots<C, CMID, 9>();
      const int64_t t8 = cdiv(d->y.h, 8) * cdiv(d->y.w, 16) * (int64_t)d->y.n;
      const int64_t t9 = cdiv(d->y.h, 9) * cdiv(d->y.w, 16) * (int64_t)d->y.n;
      if (s8 > 0 && s9 > 0 && cdiv(t9, s9) * 11 < cdiv(t8, s8) * 10) th = 9;
    }
    if (th == 9) return bneck_go<C, CMID, 9>(d, s);
  }
  return th == 16 ? bneck_go<C, CMID, 16>(d, s) : bneck_go<C, CMID, 8>(d, s);
}

extern "C" int ydbl_bottleneck_nhwc(const ydbl_bottleneck_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "bottleneck: null descriptor");
  if (!d->params) return fail(YDBL_EINVAL, "bottleneck: null parameters");
  if (check_view(&d->x, "bottleneck.x", true) || check_view(&d->y, "bottleneck.y", true)) return YDBL_EINVAL;
  if (d->x.dtype != YDBL_F16 || d->y.dtype != YDBL_F16) return fail(YDBL_EINVAL, "bottleneck: fp16 views only");
  const int c = d->c, cm = d->c_mid ? d->c_mid : d->c / 2;
  const int cin = d->x.c;
  if (d->y.c != c || (cin != c && !(d->pw && cin == 128)))
    return fail(YDBL_EINVAL, "bottleneck: y.c must equal c, and x.c too (except x.c 128 with pw)");
  if (d->x.n != d->y.n || d->x.h != d->y.h || d->x.w != d->y.w)
    return fail(YDBL_EINVAL, "bottleneck: x and y shapes differ");
  if (d->y.n < 1 || d->y.h < 1 || d->y.w < 1) return fail(YDBL_EINVAL, "bottleneck: empty input");
  if (d->tile_h != 0 && d->tile_h != 8 && d->tile_h != 16 && !(d->tile_h == 9 && c == 64 && cm == 32))
    return fail(YDBL_EINVAL, "bottleneck: tile_h must be 0, 8 or 16 (or 9 for (c, c_mid) = (64, 32))");
  if (d->x.ptr == d->y.ptr) return fail(YDBL_EINVAL, "bottleneck: in-place is not supported (halo reads)");
  hipStream_t s = as_stream(stream);
  if (c == 16 && cm == 8) return bneck_dispatch<16, 8>(d, s);
  if (c == 32 && cm == 16) return bneck_dispatch<32, 16>(d, s);
  if (c == 64 && cm == 32) return bneck_dispatch<64, 32>(d, s);
  if (c == 64 && cm == 64) {
    if (d->tile_h == 16) return fail(YDBL_EINVAL, "bottleneck: c_mid 64 takes 8-row tiles only");
    if (d->pw) {
      if (d->add) return fail(YDBL_EINVAL, "bottleneck: pw (trailing 1x1) excludes the residual add");
      return cin == 128 ? bneck_go<64, 64, 8, true, 128>(d, s) : bneck_go<64, 64, 8, true>(d, s);
    }
    return bneck_go<64, 64, 8>(d, s);
  }
  if (d->pw) return fail(YDBL_EINVAL, "bottleneck: pw needs (c, c_mid) = (64, 64)");
  return fail(YDBL_EINVAL, "bottleneck: (c, c_mid) must be (16, 8), (32, 16), (64, 32) or (64, 64)");
}
