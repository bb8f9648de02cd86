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
#include <stdlib.h>

#include "conv_common.hpp"

namespace ydbl {

// LDS-staged implicit GEMM.  Workgroup tile = BM output pixels x BN output channels, 4 waves as
// WM x WN, each wave TM x TN MFMA tiles of 16x16.  K (= taps x Cin, tap-major, NHWC-contiguous
// within a tap) advances in steps of BK = four 16-byte vectors per row (32 f16 / 16 f32):
//   global -> registers (step s+1, issued before the MFMAs of step s) -> LDS (double buffer)
//   -> fragments (ds_read_b128, XOR-swizzled rows: conflict-free for the 16x16 fragment pattern)
// A = weights [cout][KPAD] (rows shared by the WM waves of a column), B = im2col rows gathered
// on the fly (shared by the WN waves of a row); one barrier per k-step.
// Operand-slot swizzle within a row of 4 slots: 16-byte slots (f16/f32) flip by row bit 2, 8-byte
// fp8 slots by row bit 3, so the 16x16 fragment reads (ds_read_b128 / ds_read_b64 lane groups)
// are conflict-free.
template <bool Q8>
__device__ __forceinline__ int swz(int row, int kv) {
  if constexpr (Q8) return row * 4 + (kv ^ (((row >> 3) & 1) << 1));
  else return row * 4 + (kv ^ (((row >> 2) & 1) << 1));
}

template <typename T, int BM, int BN, int WM, int WN, bool POINTWISE, bool Q8, int PF = 1>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs<T> p) {
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = 4 * VEC;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "tile config");
  static_assert(PF >= 1 && PF <= 4, "prefetch depth");
  constexpr int A_IT = (BN * 4 + 255) / 256, B_IT = (BM * 4 + 255) / 256;
  using vec = typename Vec<T>::type;
  using opv = typename Op<T, Q8>::lds;
  __shared__ opv sA[2][BN * 4];
  __shared__ opv sB[2][BM * 4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wm = wave % WM, wn = wave / WM;
  int mb, nb;
  xcd_tile2(mb, nb);
  const int m0 = mb * BM;
  const int n0 = nb * BN;
  __shared__ __align__(16) float s_bias[BN];
  BiasStage<BN> bst;
  bst.fetch(p.bias, n0, p.Cout);

  // ---- per-thread staging coordinates (vector v = tid + it*256: row v>>2, k-vector v&3)
  int64_t arow[A_IT];  // element offset of this thread's weight k-vector
  bool aval[A_IT];
#pragma unroll
  for (int it = 0; it < A_IT; ++it) {
    const int v = tid + it * 256;
    const int co = n0 + (v >> 2);
    aval[it] = v < BN * 4 && co < p.Cout;
    arow[it] = (int64_t)(aval[it] ? co : 0) * p.KPAD + (v & 3) * VEC;
  }
  int bb[B_IT], biy[B_IT], bix[B_IT];
  int64_t bpix[B_IT];
  bool bval[B_IT];
#pragma unroll
  for (int it = 0; it < B_IT; ++it) {
    const int v = tid + it * 256;
    int pp = m0 + (v >> 2);
    bval[it] = v < BM * 4 && pp < p.P;
    pp = bval[it] ? pp : 0;
    bpix[it] = pp;
    const int ox = pp % p.Wo;
    const int t = pp / p.Wo;
    const int oy = t % p.Ho;
    bb[it] = t / p.Ho;
    biy[it] = oy * p.S - p.PAD;
    bix[it] = ox * p.S - p.PAD;
  }
  // PF register slots: step s lives in slot s % PF from its load (issued PF steps before it is computed,
  // so PF - 1 steps of MFMA work cover its latency) until its LDS store
  opv ra[PF][A_IT];
  vec rb[PF][B_IT];
  bool rok[PF][B_IT], aok[PF][A_IT];
  // k-walk state: every staging vector of this thread has k-vector tid&3, so one (ky, kx, ci)
  // cursor serves all of them; it advances by BK per step with no integer division (loads are issued
  // in step order, so one cursor serves the prefetch ring too).
  int cur_ci = (tid & 3) * VEC, cur_kx = 0, cur_ky = 0;
  if constexpr (!POINTWISE) {
    const int tap = cur_ci / p.Cin;
    cur_ci -= tap * p.Cin;
    cur_ky = tap / p.KW;
    cur_kx = tap - cur_ky * p.KW;
  }
  auto advance = [&]() {
    if constexpr (!POINTWISE) {
      cur_ci += BK;
      while (cur_ci >= p.Cin) {
        cur_ci -= p.Cin;
        if (++cur_kx == p.KW) { cur_kx = 0; ++cur_ky; }
      }
    }
  };
  // raw loads now, zero selects at the LDS store (vload_clamped): a slot's loads stay in flight until then
  // Steps past the end (the ring's tail) load nothing: k >= K masks B, k >= KPAD masks A (clamped addresses).
  auto load_step = [&](int ks, opv (&a)[A_IT], bool (&aok)[A_IT], vec (&b)[B_IT], bool (&bok)[B_IT]) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      aok[it] = aval[it] && ks * BK < p.KPAD;
      a[it] = load_wop_raw<T, Q8>(p.w, arow[it] + ks * BK, aok[it]);
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int v = tid + it * 256;
      const int k = ks * BK + (v & 3) * VEC;
      const bool kin = k < p.K;
      if constexpr (POINTWISE) {
        bok[it] = bval[it] && kin;
        b[it] = vload_clamped(p.x + bpix[it] * p.xcs + k, p.x, bok[it]);
      } else {
        const int iy = biy[it] + cur_ky * p.DIL, ix = bix[it] + cur_kx * p.DIL;
        bok[it] = bval[it] && kin && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        b[it] = vload_clamped(p.x + ((int64_t)(bb[it] * p.H + iy) * p.W + ix) * p.xcs + cur_ci, p.x, bok[it]);
      }
    }
    advance();
  };
  auto store_step = [&](int buf, const opv (&a)[A_IT], const bool (&aok)[A_IT], const vec (&b)[B_IT],
                        const bool (&bok)[B_IT]) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int v = tid + it * 256;
      if (v < BN * 4) sA[buf][swz<Q8>(v >> 2, v & 3)] = vsel(a[it], aok[it]);
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int v = tid + it * 256;
      if (v < BM * 4) sB[buf][swz<Q8>(v >> 2, v & 3)] = to_op<T, Q8>(vsel(b[it], bok[it]), p.qs);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (p.K + BK - 1) / BK;
#pragma unroll
  for (int u = 0; u < PF; ++u) load_step(u, ra[u], aok[u], rb[u], rok[u]);
  store_step(0, ra[0], aok[0], rb[0], rok[0]);
  bst.commit(s_bias);
  __syncthreads();
  // The loads are unconditional (past the end they are masked no-ops), so the waitcnt pass sees one fixed
  // order of outstanding loads and waits only for the slot being stored.
  for (int k0 = 0; k0 < nsteps; k0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int ks = k0 + u;
      if (PF > 1 || ks + PF < nsteps) load_step(ks + PF, ra[u], aok[u], rb[u], rok[u]);  // slot u's step is in LDS
      if (ks < nsteps) {  // uniform
        const int buf = ks & 1;
        opv af[TN], bf[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i) af[i] = sA[buf][swz<Q8>(wn * TN * 16 + i * 16 + r16, g)];
#pragma unroll
        for (int j = 0; j < TM; ++j) bf[j] = sB[buf][swz<Q8>(wm * TM * 16 + j * 16 + r16, g)];
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = mfma_op<T, Q8>(af[i], bf[j], acc[i][j]);
        const int nx = (u + 1) % PF;
        if (ks + 1 < nsteps) store_step(buf ^ 1, ra[nx], aok[nx], rb[nx], rok[nx]);
        __syncthreads();
      }
    }
  }

  // ---- epilogue
  int64_t pp[TM];
  bool pv[TM];
  int co[TN];
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    pp[j] = m0 + wm * TM * 16 + j * 16 + r16;
    pv[j] = pp[j] < p.P;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) co[i] = n0 + wn * TN * 16 + i * 16 + 4 * g;
  conv_epilogue<T, TN, TM, Q8>(p, acc, pp, pv, co, s_bias, n0);
}

// Spatial-tile 3x3 conv for thin inputs (Cin <= 32, the high-resolution backbone layers).
// A workgroup owns a TH x TW output tile of one image and ALL output channels (NTN x 16 <= 64):
// the input halo tile (IH x IW pixels x Cin) and the whole weight matrix [Cout][KPAD] are staged
// in LDS once, so each input element leaves HBM/L2 about once instead of once per tap (the 9x
// im2col amplification of conv_igemm_kernel).  B fragments are gathered from the LDS tile:
// lane (pixel r16, k-vector g) reads the 8 channels of tap k/Cin at (py*S+ky, px*S+kx).
// Channel-vector slots are XOR-swizzled by pixel so 16 consecutive pixels hit distinct banks.
template <int CV>
__device__ __forceinline__ int tswz(int pix, int cv) {
  if constexpr (CV == 1) return pix;
  else return pix * CV + (cv ^ ((pix / (16 / CV)) & (CV - 1)));
}

template <typename T, int CIN, int S, int TH, int TW, int NTN>
__global__ __launch_bounds__(256) void conv3x3_tile_kernel(ConvArgs<T> p, int tiles_x, int tiles_y) {
  constexpr int VEC = Vec<T>::N;
  constexpr int CV = CIN / VEC;                 // 16-byte channel vectors per pixel
  constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  constexpr int K = 9 * CIN;
  constexpr int BK = 4 * VEC;
  constexpr int KPAD = (K + 31) / 32 * 32;
  constexpr int NSTEP = (K + BK - 1) / BK;
  constexpr int WROW = KPAD / VEC + 1;          // weight row in 16B vectors (+1 pad: bank spread)
  constexpr int TM = TH * TW / 64;              // 16-pixel tiles per wave
  using vec = typename Vec<T>::type;
  __shared__ vec sx[IH * IW * CV];
  __shared__ vec sw[NTN * 16 * WROW];

  const int tid = threadIdx.x;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - p.PAD, ix0 = ox0 * S - p.PAD;
  __shared__ __align__(16) float s_bias[NTN * 16];
  BiasStage<NTN * 16> bst;
  bst.fetch(p.bias, 0, p.Cout);
  {  // stage the input tile (loads batched 4 deep before their LDS stores)
    constexpr int TOT = IH * IW * CV;
    for (int base = 0; base < TOT; base += 4 * 256) {
      vec t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = min(base + u * 256 + tid, TOT - 1);
        const int pix = i / CV, cv = i - pix * CV;
        const int iy = iy0 + pix / IW, ix = ix0 + pix % IW;
        const bool ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        t[u] = vload_sel(p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + cv * VEC, p.x, ok);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = base + u * 256 + tid;
        if (i < TOT) sx[tswz<CV>(i / CV, i % CV)] = t[u];
      }
    }
    constexpr int WTOT = NTN * 16 * (KPAD / VEC);
    for (int base = 0; base < WTOT; base += 4 * 256) {
      vec t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = min(base + u * 256 + tid, WTOT - 1);
        const int co = i / (KPAD / VEC), kv = i % (KPAD / VEC);
        t[u] = vload_sel(p.w + (int64_t)co * p.KPAD + kv * VEC, p.w, co < p.Cout);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = base + u * 256 + tid;
        if (i < WTOT) sw[(i / (KPAD / VEC)) * WROW + i % (KPAD / VEC)] = t[u];
      }
    }
  }
  bst.commit(s_bias);
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int lbase[TM];  // LDS pixel index of each 16-pixel tile's top-left tap for this lane
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int op = wave * TM * 16 + j * 16 + r16;
    const int py = op / TW, px = op % TW;
    lbase[j] = (py * S) * IW + px * S;
  }
  f32x4 acc[NTN][TM];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NSTEP; ++ks) {
    const int k = ks * BK + g * VEC;
    const bool kin = k < K;
    const int tap = kin ? k / CIN : 0, cv = kin ? (k % CIN) / VEC : 0;
    const int ky = tap / 3, kx = tap % 3;
    const int toff = ky * IW + kx;
    vec af[NTN], bf[TM];
#pragma unroll
    for (int i = 0; i < NTN; ++i) af[i] = sw[(i * 16 + r16) * WROW + ks * 4 + g];  // zero beyond K
#pragma unroll
    for (int j = 0; j < TM; ++j) bf[j] = sx[tswz<CV>(lbase[j] + toff, cv)];
#pragma unroll
    for (int i = 0; i < NTN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = mfma_chunk<T>(af[i], bf[j], acc[i][j]);
  }

  int64_t pp[TM];
  bool pv[TM];
  int co[NTN];
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int op = wave * TM * 16 + j * 16 + r16;
    const int oy = oy0 + op / TW, ox = ox0 + op % TW;
    pv[j] = oy < p.Ho && ox < p.Wo;
    pp[j] = ((int64_t)b * p.Ho + oy) * p.Wo + ox;
  }
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = i * 16 + 4 * g;
  conv_epilogue<T, NTN, TM>(p, acc, pp, pv, co, s_bias, 0);
}

template <typename T, int CIN, int S, int TH, int TW, int NTN>
static void launch_tile(const ConvArgs<T>& a, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, TW), tiles_y = (int)cdiv(a.Ho, TH);
  conv3x3_tile_kernel<T, CIN, S, TH, TW, NTN><<<(unsigned)(a.N * tiles_y * tiles_x), 256, 0, s>>>(a, tiles_x, tiles_y);
}

// 3x3 / pad 1 / dil 1, Cin in {8,16,32}, Cout <= 64 and a multiple of 4: the spatial-tile kernel.
template <typename T, int CIN, int NTN>
static void launch_tile_s(const ConvArgs<T>& a, hipStream_t s) {
  if (a.S == 1) launch_tile<T, CIN, 1, 8, 32, NTN>(a, s);
  else launch_tile<T, CIN, 2, 8, 16, NTN>(a, s);
}

template <typename T, int CIN>
static bool tile_ntn(const ConvArgs<T>& a, hipStream_t s) {
  switch ((a.Cout + 15) / 16) {
    case 1: launch_tile_s<T, CIN, 1>(a, s); return true;
    case 2: launch_tile_s<T, CIN, 2>(a, s); return true;
    case 3: launch_tile_s<T, CIN, 3>(a, s); return true;
    case 4: launch_tile_s<T, CIN, 4>(a, s); return true;
    default: return false;
  }
}

template <typename T>
static bool try_tile(const ConvArgs<T>& a, int kh, hipStream_t s) {
  if (kh != 3 || a.KW != 3 || a.DIL != 1 || a.PAD != 1 || a.Cout > 64 || a.Cout % 4) return false;
  if (a.S != 1 && a.S != 2) return false;
  if ((int64_t)a.Ho * a.Wo < 4096) return false;  // small maps: the GEMM kernel has more parallelism
  if (a.xcs % Vec<T>::N) return false;
  switch (a.Cin) {
    case 8: return tile_ntn<T, 8>(a, s);
    case 16: return tile_ntn<T, 16>(a, s);
    case 32: return tile_ntn<T, 32>(a, s);
    default: return false;
  }
}

// Wave-split-K implicit GEMM for large K (3x3 with Cin >= 64, wide 1x1): every wave computes the
// whole BM x BN tile (TM x TN = up to 16 MFMA tiles) over its quarter of each 4*BK-deep k-block,
// so a barrier is amortised over TM*TN MFMAs per wave instead of (TM*TN)/4; the four partial
// tiles are summed through LDS in fixed wave order before the fused epilogue.
// LDS rows are 16 vectors (4*BK elements), slot-swizzled with (kv ^ row) so both the staging
// stores and the 16x16 fragment reads are bank-conflict-free.
template <typename T, int BM, int BN, bool POINTWISE, bool Q8, int PF = 1, bool SPLIT = false>
__global__ __launch_bounds__(256) void conv_wsk_kernel(ConvArgs<T> p) {
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = 4 * VEC;    // per wave
  constexpr int BKB = 4 * BK;    // per block step
  constexpr int TM = BM / 16, TN = BN / 16;
  constexpr int A_IT = BN * 16 / 256, B_IT = BM * 16 / 256;
  static_assert(A_IT >= 1 && B_IT >= 1, "tile");
  using vec = typename Vec<T>::type;
  using opv = typename Op<T, Q8>::lds;
  constexpr int STAGE = 2 * (BN + BM) * 16 * (int)sizeof(opv);  // bytes, double-buffered operands
  constexpr int RED = 4 * TN * TM * 64 * 16;                      // bytes of f32x4 partials
  __shared__ f32x4 smem[(STAGE > RED ? STAGE : RED) / 16];
  opv* sA = reinterpret_cast<opv*>(smem);                         // [2][BN*16]
  opv* sB = sA + 2 * BN * 16;                                     // [2][BM*16]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int mb, nb;
  xcd_tile2(mb, nb);
  const int m0 = mb * BM, n0 = nb * BN;
  const int kv = tid & 15;
  // (no LDS-staged bias here: the extra bytes cost a workgroup per CU at 80 KB of staging)  // every staging vector of this thread has k-vector kv

  int64_t arow[A_IT];  // element offset of this thread's weight k-vector
  bool aval[A_IT];
#pragma unroll
  for (int it = 0; it < A_IT; ++it) {
    const int co = n0 + ((tid + it * 256) >> 4);
    aval[it] = co < p.Cout;
    arow[it] = (int64_t)(aval[it] ? co : 0) * p.KPAD + kv * VEC;
  }
  int bb[B_IT], biy[B_IT], bix[B_IT];
  int64_t bpix[B_IT];
  bool bval[B_IT];
#pragma unroll
  for (int it = 0; it < B_IT; ++it) {
    int pp = m0 + ((tid + it * 256) >> 4);
    bval[it] = pp < p.P;
    pp = bval[it] ? pp : 0;
    bpix[it] = pp;
    const int ox = pp % p.Wo;
    const int t = pp / p.Wo;
    bb[it] = t / p.Ho;
    biy[it] = (t % p.Ho) * p.S - p.PAD;
    bix[it] = ox * p.S - p.PAD;
  }
  // split-K: workgroup z of ksplit takes k-block steps [s0, s1) (ksplit 1: all of them)
  // (a template flag: the runtime start step cost the unsplit kernels up to 86 VGPRs -- 2 -> 1 waves per SIMD on
  // the 32 x 128 tiles, DBL-l 1280's deep 3x3s 142 -> 272 us)
  const int nsteps_all = (p.K + BKB - 1) / BKB;
  const int z = SPLIT ? (int)blockIdx.z : 0;
  const int s0 = SPLIT ? (int)((int64_t)z * nsteps_all / p.ksplit) : 0;
  const int s1 = SPLIT ? (int)((int64_t)(z + 1) * nsteps_all / p.ksplit) : nsteps_all;
  int cur_ci = s0 * BKB + kv * VEC, cur_kx = 0, cur_ky = 0;
  if constexpr (!POINTWISE) {
    const int tap = cur_ci / p.Cin;
    cur_ci -= tap * p.Cin;
    cur_ky = tap / p.KW;
    cur_kx = tap - cur_ky * p.KW;
  }
  // PF register slots as in conv_igemm_kernel: raw loads, zero selects at the LDS store, loads unconditional
  opv ra[PF][A_IT];
  vec rb[PF][B_IT];
  bool aok[PF], bok[PF][B_IT];
  auto load_step = [&](int kb, opv (&a)[A_IT], bool& ak, vec (&b)[B_IT], bool (&bk)[B_IT]) {
    const int k = kb * BKB + kv * VEC;
    const bool kin = k < p.K;
    ak = kin;
#pragma unroll
    for (int it = 0; it < A_IT; ++it) a[it] = load_wop_raw<T, Q8>(p.w, arow[it] + kb * BKB, aval[it] && kin);
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      if constexpr (POINTWISE) {
        bk[it] = bval[it] && kin;
        b[it] = vload_clamped(p.x + bpix[it] * p.xcs + k, p.x, bk[it]);
      } else {
        const int iy = biy[it] + cur_ky * p.DIL, ix = bix[it] + cur_kx * p.DIL;
        bk[it] = bval[it] && kin && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        b[it] = vload_clamped(p.x + ((int64_t)(bb[it] * p.H + iy) * p.W + ix) * p.xcs + cur_ci, p.x, bk[it]);
      }
    }
    if constexpr (!POINTWISE) {
      cur_ci += BKB;
      while (cur_ci >= p.Cin) {
        cur_ci -= p.Cin;
        if (++cur_kx == p.KW) { cur_kx = 0; ++cur_ky; }
      }
    }
  };
  auto store_step = [&](int buf, const opv (&a)[A_IT], bool ak, const vec (&b)[B_IT], const bool (&bk)[B_IT]) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int row = (tid + it * 256) >> 4;
      sA[buf * BN * 16 + row * 16 + (kv ^ (row & 15))] = vsel(a[it], aval[it] && ak);
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int row = (tid + it * 256) >> 4;
      sB[buf * BM * 16 + row * 16 + (kv ^ (row & 15))] = to_op<T, Q8>(vsel(b[it], bk[it]), p.qs);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // local step l = global step s0 + l (the loads past s1 are in bounds and never stored)
  const int nsteps = s1 - s0;
#pragma unroll
  for (int u = 0; u < PF; ++u) load_step(s0 + u, ra[u], aok[u], rb[u], bok[u]);
  store_step(0, ra[0], aok[0], rb[0], bok[0]);
  __syncthreads();
  const int myk = wave * 4 + g;  // k-vector this lane reads inside a block step
  for (int k0 = 0; k0 < nsteps; k0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int kb = k0 + u;
      if (PF > 1 || kb + PF < nsteps) load_step(s0 + kb + PF, ra[u], aok[u], rb[u], bok[u]);
      if (kb < nsteps) {  // uniform
        const int buf = kb & 1;
        opv af[TN], bf[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int row = i * 16 + r16;
          af[i] = sA[buf * BN * 16 + row * 16 + (myk ^ (row & 15))];
        }
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int row = j * 16 + r16;
          bf[j] = sB[buf * BM * 16 + row * 16 + (myk ^ (row & 15))];
        }
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = mfma_op<T, Q8>(af[i], bf[j], acc[i][j]);
        const int nx = (u + 1) % PF;
        if (kb + 1 < nsteps) store_step(buf ^ 1, ra[nx], aok[nx], rb[nx], bok[nx]);
        __syncthreads();
      }
    }
  }

  // cross-wave reduction: partial tile (i, j) of wave w at red[((w * TN + i) * TM + j) * 64 + lane]
  f32x4* red = reinterpret_cast<f32x4*>(smem);
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) red[((wave * TN + i) * TM + j) * 64 + lane] = acc[i][j];
  __syncthreads();
  for (int t = wave; t < TN * TM; t += 4) {
    const int i = t / TM, j = t % TM;
    f32x4 sum = red[((0 * TN + i) * TM + j) * 64 + lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const f32x4 o = red[((w * TN + i) * TM + j) * 64 + lane];
      sum = f32x4{sum[0] + o[0], sum[1] + o[1], sum[2] + o[2], sum[3] + o[3]};
    }
    const f32x4 one[1][1] = {{sum}};
    const int64_t pp[1] = {m0 + j * 16 + r16};
    const bool pv[1] = {pp[0] < p.P};
    const int co[1] = {n0 + i * 16 + 4 * g};
    if constexpr (SPLIT) {  // this split's partial tile, summed by splitk_epilogue_kernel
      if (pv[0] && co[0] < p.Cout)
        *reinterpret_cast<f32x4*>(p.ws + ((int64_t)z * p.P + pp[0]) * ((p.Cout + 3) & ~3) + co[0]) = sum;
    } else {
      conv_epilogue<T, 1, 1, Q8>(p, one, pp, pv, co);
    }
  }
}

// Split-K epilogue: one thread per (pixel, 4 output channels) sums the ksplit partial tiles in split order and runs
// the same fused epilogue (bias, activation, residual, channel-slice store, second output) as the unsplit kernel.
template <typename T, bool Q8>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(ConvArgs<T> p) {
  const int c4 = (p.Cout + 3) >> 2, cs = c4 * 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t pix = t / c4;
  const int co = (int)(t - pix * c4) * 4;
  const bool ok = pix < p.P;
  const int64_t pc = ok ? pix : 0;
  f32x4 v[4];
#pragma unroll
  for (int z = 0; z < 4; ++z)  // all loads issued first (ksplit <= 4)
    v[z] = z < p.ksplit ? *reinterpret_cast<const f32x4*>(p.ws + ((int64_t)z * p.P + pc) * cs + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 sum = v[0];
#pragma unroll
  for (int z = 1; z < 4; ++z)
    if (z < p.ksplit) sum = f32x4{sum[0] + v[z][0], sum[1] + v[z][1], sum[2] + v[z][2], sum[3] + v[z][3]};
  const f32x4 one[1][1] = {{sum}};
  const int64_t pp[1] = {pix};
  const bool pv[1] = {ok};
  const int cc[1] = {co};
  conv_epilogue<T, 1, 1, Q8>(p, one, pp, pv, cc);
}

template <typename T, bool Q8>
void launch_splitk_epilogue(const ConvArgs<T>& a, hipStream_t s) {
  splitk_epilogue_kernel<T, Q8><<<(unsigned)cdiv((int64_t)a.P * ((a.Cout + 3) >> 2), 256), 256, 0, s>>>(a);
}
template void launch_splitk_epilogue<_Float16, false>(const ConvArgs<_Float16>&, hipStream_t);
template void launch_splitk_epilogue<_Float16, true>(const ConvArgs<_Float16>&, hipStream_t);
template void launch_splitk_epilogue<float, false>(const ConvArgs<float>&, hipStream_t);

// Split of the wave-split-K k-loop for a BM x BN tiling: the serial k-block chain is what a deep-K conv on a small
// map waits on (DBL-s bs4 sub-batch: 768->128 3x3 @40^2, 400 tiles of 54 k-block steps, about 1 us each: 53.7 us in
// graph), so below 768 tiles (3 workgroups per CU) the loop is split over up to 4 workgroups, each keeping >= 8
// steps.  YDBL_SPLITK=0 (read per launch): no split (A/B switch).
constexpr int WSK_SPLIT_BELOW = 768;
template <typename T>
static int wsk_ksplit(const ConvArgs<T>& a, int bm, int bn) {
  const char* e = getenv("YDBL_SPLITK");
  if (sizeof(T) != 2 || (e && *e == '0')) return 1;  // fp16 only: the fp32 parity mode keeps one summation order
  const int64_t tiles = cdiv(a.P, bm) * cdiv(a.Cout, bn);
  const int nsteps = (int)cdiv(a.K, 16 * Vec<T>::N);  // BKB
  if (tiles >= WSK_SPLIT_BELOW || nsteps < 16) return 1;
  int k = (int)std::min<int64_t>(4, (WSK_SPLIT_BELOW + tiles - 1) / tiles);
  while (k > 1 && nsteps / k < 8) --k;
  return k;
}
template <typename T>
static int64_t wsk_ws_bytes(const ConvArgs<T>& a, int ksplit) {
  return ksplit > 1 ? (int64_t)ksplit * a.P * ((a.Cout + 3) & ~3) * 4 : 0;
}

// Two k-block steps in flight (kbench bs16: 256->64 3x3 @20^2 18.8 -> 17.4 us; three or four: no better)
constexpr int WSK_PF = 2;

template <typename T, bool Q8, int BM, int BN>
static void launch_wsk(const ConvArgs<T>& a0, bool pointwise, hipStream_t s) {
  ConvArgs<T> a = a0;
  a.ksplit = wsk_ksplit(a, BM, BN);
  if (a.ksplit > 1 && (!a.ws || a.ws_bytes < wsk_ws_bytes(a, a.ksplit))) a.ksplit = 1;  // no room: unsplit
  dim3 grid((unsigned)cdiv(a.P, BM), (unsigned)cdiv(a.Cout, BN), (unsigned)a.ksplit);
  if (a.ksplit > 1) {
    if (pointwise) conv_wsk_kernel<T, BM, BN, true, Q8, WSK_PF, true><<<grid, 256, 0, s>>>(a);
    else conv_wsk_kernel<T, BM, BN, false, Q8, WSK_PF, true><<<grid, 256, 0, s>>>(a);
    launch_splitk_epilogue<T, Q8>(a, s);
  } else if (pointwise) {
    conv_wsk_kernel<T, BM, BN, true, Q8, WSK_PF><<<grid, 256, 0, s>>>(a);
  } else {
    conv_wsk_kernel<T, BM, BN, false, Q8, WSK_PF><<<grid, 256, 0, s>>>(a);
  }
}

// The wave-split-K tiling try_wsk picks (BM, BN), without launching.
template <typename T>
static void wsk_tiles(const ConvArgs<T>& a, int& bm, int& bn) {
  auto blocks = [&](int m, int n) { return cdiv(a.P, m) * cdiv(a.Cout, n); };
  const int64_t want = 768;
  const char* eh = getenv("YDBL_WSK_HALF");  // A/B switch (read per launch): 0 = no half-height tiles
  if (a.Cout <= 128 && blocks(32, a.Cout <= 64 ? 64 : 128) < 256 && !(eh && *eh == '0')) {
    bm = a.Cout <= 64 ? 16 : 32;
    bn = 64;
    return;
  }
  if (a.Cout <= 32) { bm = blocks(128, 32) >= want ? 128 : 64; bn = 32; return; }
  if (a.Cout <= 64) { bm = blocks(64, 64) >= want ? 64 : 32; bn = 64; return; }
  bm = 32;
  bn = blocks(32, 128) >= want || a.Cout % 128 == 0 ? 128 : 64;
}

// Wave-split-K where the block-tiled GEMM runs out of parallelism or k-depth per barrier:
// K >= 1024, or K >= 512 on small maps (measured on DBL-n: 384->64 3x3 @40^2 112 -> 82 us,
// 256->64 3x3 @20^2 47 -> 27 us; 64->64 3x3 @80^2 stays on conv_igemm_kernel, 47 vs 74 us).
template <typename T>
static bool wsk_applies(const ConvArgs<T>& a) { return a.K >= 1024 || (a.K >= 512 && a.P <= 16384); }

template <typename T, bool Q8>
static bool try_wsk(const ConvArgs<T>& a, bool pointwise, hipStream_t s) {
  if (!wsk_applies(a)) return false;
  // Tiles (wsk_tiles): under 256 workgroups with the usual tiles (the 20^2 maps of a bs16 sub-batch): half-height
  // tiles, 16 pixels for Cout <= 64 and 64-wide columns for Cout 128 -- twice the workgroups for the same k-loop
  // (bs16 graphs: 128->128 3x3 s2 @20^2 17.4 -> 14.4 us, 64->64 3x3 @20^2 9.5 -> 8.6, 256->64 18.4 -> 17.7; DBL-n
  // bs32 even to +0.5 % over two boxes, DBL-s bs64 even: profiles/r04/r04_wsk_small_tiles_ab.txt); then the
  // k-loop split where the tiles are still few (wsk_ksplit)
  int bm, bn;
  wsk_tiles(a, bm, bn);
  if (bm == 16) launch_wsk<T, Q8, 16, 64>(a, pointwise, s);
  else if (bm == 32 && bn == 64) launch_wsk<T, Q8, 32, 64>(a, pointwise, s);
  else if (bm == 32) launch_wsk<T, Q8, 32, 128>(a, pointwise, s);
  else if (bm == 64 && bn == 64) launch_wsk<T, Q8, 64, 64>(a, pointwise, s);
  else if (bm == 64) launch_wsk<T, Q8, 64, 32>(a, pointwise, s);
  else launch_wsk<T, Q8, 128, 32>(a, pointwise, s);
  return true;
}

// One k-step in flight: with the zero selects at the LDS store the loads of step s+1 overlap step s's MFMAs
// (kbench bs16: 512->128 1x1 @40^2 16.9 -> 13.2 us, 128->64 @80^2 19.4 -> 11.1); deeper rings (2-4 steps,
// the kernel's PF parameter) measured slower on every 1x1 shape (512->128: 13.4 / 14.6 / 14.2 us).
template <typename T, bool Q8, int BM, int BN, int WM, int WN>
static void launch_igemm(const ConvArgs<T>& a, bool pointwise, hipStream_t s) {
  dim3 grid((unsigned)cdiv(a.P, BM), (unsigned)cdiv(a.Cout, BN));
  if (pointwise)
    conv_igemm_kernel<T, BM, BN, WM, WN, true, Q8><<<grid, 256, 0, s>>>(a);
  else
    conv_igemm_kernel<T, BM, BN, WM, WN, false, Q8><<<grid, 256, 0, s>>>(a);
}

template <typename T, bool Q8>
static void dispatch_conv(const ConvArgs<T>& a, bool pointwise, hipStream_t s) {
  // BN covers Cout <= 64 in one column of workgroups (the input tile is then read once; wider Cout: below);
  // BM is the largest pixel tile that still gives >= `want` workgroups: 512 (2 per CU) for small
  // maps whose Cout fits one 128-wide column (bigger pixel tiles re-read the weights less:
  // 512->128 1x1 @40^2 bs32 31.3 -> 23.0 us, 384->128 25.6 -> 19.4 us), 1024 otherwise
  // (128->192: 16.4 vs 21.4 us; DBL-s bs64 end to end 0.8 % faster at 1024).
  // Shallow K (<= 128) on large maps: 2048 (8 per CU; each tile is a short k-loop, so more workgroups
  // hide each other's load latency: 64->128 @80^2 bs32 35.3 -> 28.1 us, 64->64 17.5 -> 16.4,
  // 128->64 22.2 -> 21.2).
  // (bs16 sub-batch graphs, scripts/kbench.py: for K 128, 2048 only above 131072 pixels -- 128->64 1x1 @80^2
  // 12.6 -> 11.3 us at 1024; K 64 keeps 2048 there, 64->128 @80^2 14.4 vs 15.6 us -- and 64x64 tiles for the
  // deep-K (>= 512) 3x3 convs with >= 16384 output pixels: 64->64 s2 @80^2 14.6 -> 13.1 us; DBL-n bs32 on two
  // streams 16.20 -> 16.30 k img/s over three pairs with the halo kernel's n2_below 512, DBL-s bs64 even)
  const int64_t want = a.Cout <= 128 && a.P <= 65536 ? 512
                       : (a.K <= 128 && a.P > (a.K <= 64 ? 65536 : 131072) ? 2048 : 1024);
  auto blocks = [&](int bm, int bn) { return cdiv(a.P, bm) * cdiv(a.Cout, bn); };
  if (a.Cout <= 16) {
    if (blocks(256, 16) >= want) return launch_igemm<T, Q8, 256, 16, 4, 1>(a, pointwise, s);
    if (blocks(128, 16) >= want) return launch_igemm<T, Q8, 128, 16, 4, 1>(a, pointwise, s);
    return launch_igemm<T, Q8, 64, 16, 4, 1>(a, pointwise, s);
  }
  if (a.Cout <= 32) {
    if (blocks(256, 32) >= want) return launch_igemm<T, Q8, 256, 32, 4, 1>(a, pointwise, s);
    if (blocks(128, 32) >= want) return launch_igemm<T, Q8, 128, 32, 4, 1>(a, pointwise, s);
    return launch_igemm<T, Q8, 64, 32, 4, 1>(a, pointwise, s);
  }
  if (a.Cout <= 64) {
    if (blocks(128, 64) >= want) return launch_igemm<T, Q8, 128, 64, 2, 2>(a, pointwise, s);
    if (blocks(64, 64) >= want || (!pointwise && a.K >= 512 && a.P >= 16384))
      return launch_igemm<T, Q8, 64, 64, 2, 2>(a, pointwise, s);
    return launch_igemm<T, Q8, 32, 64, 2, 2>(a, pointwise, s);
  }
  // Cout > 64: 64-wide column blocks (each workgroup stages half the weight rows; the input tile is read
  // once per column block, from L2/MALL at these map sizes).  Measured against 128-wide blocks on the
  // bench workloads: DBL-n bs32 14.82 -> 14.91 k img/s (bs16 graphs: 64->128 @80^2 22.6 -> 19.8 us,
  // 128->192 @40^2 15.6 -> 12.1 us), DBL-s bs64 7.52 -> 7.57 k, DBL-l 1280 bs8 467 -> 466 (noise).
  if (blocks(128, 64) >= want) return launch_igemm<T, Q8, 128, 64, 2, 2>(a, pointwise, s);
  if (blocks(64, 64) >= want) return launch_igemm<T, Q8, 64, 64, 2, 2>(a, pointwise, s);
  return launch_igemm<T, Q8, 32, 64, 2, 2>(a, pointwise, s);
}

// Kernel choice: thin-input spatial tile (f16/f32 only), halo tile, wave-split-K, block GEMM.
template <typename T>
int halo_ksplit(const ConvArgs<T>& a, int64_t wgs);  // conv3x3.hip

template <typename T, bool Q8>
static void route(const ConvArgs<T>& a, int kh, bool pw, hipStream_t s) {
  if constexpr (sizeof(T) == 2 && !Q8) {
    if (try_conv3x3_vw(a, kh, s)) return;
  }
  if (!Q8 && try_tile<T>(a, kh, s)) return;
  if (try_conv3x3_halo<T, Q8>(a, kh, s)) return;
  if (try_wsk<T, Q8>(a, pw, s)) return;
  dispatch_conv<T, Q8>(a, pw, s);
}

template <typename T>
static ConvArgs<T> conv_args(const ydbl_conv_desc* d) {
  ConvArgs<T> a{};
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
  a.y2 = reinterpret_cast<T*>(d->y2.ptr); a.y2cs = d->y2.cs;
  a.r2 = reinterpret_cast<const T*>(d->r2.ptr); a.r2cs = d->r2.cs;
  a.a2 = d->a2; a.b2 = d->b2;
  a.dq = d->dq; a.qs = d->qscale;
  a.ws = reinterpret_cast<float*>(d->workspace); a.ws_bytes = d->workspace ? d->workspace_bytes : 0;
  a.ksplit = 1;
  return a;
}

ConvArgs<_Float16> conv_args_f16(const ydbl_conv_desc* d) { return conv_args<_Float16>(d); }

template <typename T>
static int run_conv(const ydbl_conv_desc* d, hipStream_t s) {
  const ConvArgs<T> a = conv_args<T>(d);
  const bool pw = d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && d->x.h == d->y.h && d->x.w == d->y.w;
  if constexpr (sizeof(T) == 2) {
    if (d->dq) {
      route<T, true>(a, d->kh, pw, s);
      return check_launch("ydbl_conv2d_nhwc");
    }
  }
  route<T, false>(a, d->kh, pw, s);
  return check_launch("ydbl_conv2d_nhwc");
}

// The descriptor rules of ydbl_conv2d_nhwc (include/ydbl.h).
int conv_check(const ydbl_conv_desc* d) {
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
  if (d->dq && d->x.dtype != YDBL_F16) return fail(YDBL_EINVAL, "conv: fp8 operands need f16 activations");
  if (d->y2.ptr) {
    if (check_view(&d->y2, "conv.y2", false) || check_view(&d->r2, "conv.r2", false)) return YDBL_EINVAL;
    auto same = [&](const ydbl_view& v) {
      return v.n == d->y.n && v.h == d->y.h && v.w == d->y.w && v.c == d->y.c && v.dtype == d->y.dtype && v.cs % 4 == 0;
    };
    if (!same(d->y2) || !same(d->r2)) return fail(YDBL_EINVAL, "conv: y2/r2 must match y (shape, dtype, cs % 4)");
  }
  return YDBL_OK;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_conv2d_nhwc(const ydbl_conv_desc* d, void* stream) {
  if (const int rc = conv_check(d)) return rc;
  const hipStream_t s = as_stream(stream);
  return d->x.dtype == YDBL_F16 ? run_conv<_Float16>(d, s) : run_conv<float>(d, s);
}

// Split-K scratch the wave-split-K path would use for this descriptor (0: it would not split).  Computed as if the
// conv took that path; a conv routed to another kernel ignores its workspace.
template <typename T>
static int64_t conv_ws_t(const ydbl_conv_desc* d) {
  const ConvArgs<T> a = conv_args<T>(d);
  int64_t need = 0;
  if (wsk_applies(a)) {
    int bm, bn;
    wsk_tiles(a, bm, bn);
    need = wsk_ws_bytes(a, wsk_ksplit(a, bm, bn));
  }
  if (d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad == 1 && d->dil == 1 && (int64_t)a.P < 25600) {
    const int64_t wgs = (int64_t)a.N * cdiv(a.Ho, 8) * cdiv(a.Wo, 16) * cdiv(a.Cout, 32);
    need = std::max(need, wsk_ws_bytes(a, halo_ksplit(a, wgs)));
  }
  return need;
}
extern "C" int64_t ydbl_conv_workspace(const ydbl_conv_desc* d) {
  if (conv_check(d)) return -1;
  return d->x.dtype == YDBL_F16 ? conv_ws_t<_Float16>(d) : conv_ws_t<float>(d);
}
