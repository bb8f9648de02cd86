// Halo-tiled 3x3 convolution on MFMA for 64 <= Cin <= 256 on large maps (head and backbone 3x3s; U/nn/modules/conv.py:39-63 after fuse, U/nn/modules/block.py:344-357 Bottleneck).
//
// conv_igemm_kernel gathers im2col rows on the fly, so every input element is fetched once per
// tap (9x from L2/MALL); at 40x40 / 80x80 with Cout <= 128 that re-read traffic, not the MFMAs,
// sets the time.  Here a workgroup owns a TH x 16 output tile and NTN*16 output channels and
// walks Cin in chunks of BK (32 f16 / 16 f32) channels:
//   - the chunk's input halo ((TH-1)*S+3) x (15*S+3) pixels and its weights [co][9 taps][BK]
//     are staged in LDS once (the next chunk is loaded into registers during this chunk's MFMAs,
//     the single buffer is refilled between two barriers: a small footprint, 2-3 workgroups/CU),
//   - each wave takes 16-pixel tiles (one output row of the tile each) and multiplies them by all
//     NTN weight tiles for each of the 9 taps: B fragments are read from the halo at the tap's
//     offset, so the input leaves L2 about (TH+2)/TH times instead of 9 times.
// LDS layouts are "planar per 16-lane run": halo vector (pixel p, k-vector g) lives at
//   (p / 16S) * 64S + g * 16S + (p % S) * 16 + (p / S) % 16
// so the 16 lanes of a B-fragment read (16 pixels at stride S, one g) hit 16 distinct 16-byte
// bank quads for any starting pixel, and the mixed-g lane groups of ds_read_b128
// ({0-3,12-15,20-27}, ...) stay conflict-free; weights are [co/16][tap][g][co%16] for the same
// reason.  Fused epilogue (bias, SiLU, residual add, channel-slice store) from conv_common.hpp.
#include "conv_common.hpp"

namespace ydbl {

template <int S>
__device__ __forceinline__ int hslot(int pix, int g) {
  return (pix / (16 * S)) * (64 * S) + g * (16 * S) + (pix % S) * 16 + ((pix / S) & 15);
}

template <typename T, int S, int TH, int NTN, bool Q8>
__global__ __launch_bounds__(256, 2) void conv3x3_halo_kernel(ConvArgs<T> p, int tiles_x, int tiles_y,
                                                              int co_splits) {
  constexpr int TW = 16;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = 4 * VEC;
  constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  constexpr int NPIX = IH * IW;
  constexpr int XSLOTS = (NPIX + 16 * S - 1) / (16 * S) * (64 * S);
  constexpr int WV = NTN * 16 * 36;  // weight vectors per chunk
  constexpr int XIT = (XSLOTS + 255) / 256, WIT = (WV + 255) / 256;
  constexpr int TMW = (TH + 3) / 4;  // 16-pixel tiles (= output rows) per wave
  using vec = typename Vec<T>::type;
  using opv = typename Op<T, Q8>::lds;  // 8-byte e4m3 groups in fp8 mode (same slot layout)
  __shared__ opv s_x[XSLOTS];
  __shared__ opv s_w[WV];

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
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const int co0 = cs * NTN * 16;

  // Staging walks LDS slots linearly (consecutive lanes -> consecutive 16-byte slots, so the
  // ds_write_b128s are conflict-free) and gathers the matching global vectors: a wave still
  // covers 16 pixels x 64 B (halo) / 16 rows x 64 B (weights) of global memory.  The per-lane
  // source offsets are chunk-invariant and computed once.
  const T* xsrc[XIT];
  bool xok[XIT];
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int slot = min(it * 256 + tid, XSLOTS - 1);
    const int blk = slot / (64 * S), rem = slot % (64 * S);
    const int gv = rem / (16 * S), r2 = rem % (16 * S);
    const int px = blk * 16 * S + (r2 & 15) * S + r2 / 16;
    const int hy = px / IW, hx = px - hy * IW;
    const int iy = iy0 + hy, ix = ix0 + hx;
    xok[it] = px < NPIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    xsrc[it] = p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + gv * VEC;
  }
  int64_t wsrc[WIT];  // element offsets into the weight matrix
  bool wok[WIT];
#pragma unroll
  for (int it = 0; it < WIT; ++it) {  // slot = ((cb*9 + tap)*4 + g)*16 + r  ->  row cb*16 + r
    const int slot = min(it * 256 + tid, WV - 1);
    const int r = slot & 15, gv = (slot >> 4) & 3, t2 = slot >> 6;
    const int tap = t2 % 9, cb = t2 / 9;
    const int co = co0 + cb * 16 + r;
    wok[it] = co < p.Cout;
    wsrc[it] = (int64_t)min(co, p.Cout - 1) * p.KPAD + tap * p.Cin + gv * VEC;
  }
  vec xr[XIT];
  opv wr[WIT];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) xr[it] = vload_sel(xsrc[it] + c0, p.x, xok[it]);
#pragma unroll
    for (int it = 0; it < WIT; ++it) wr[it] = load_wop<T, Q8>(p.w, wsrc[it] + c0, wok[it]);
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int it = 0; it < XIT; ++it)
      if (it * 256 + tid < XSLOTS) s_x[it * 256 + tid] = to_op<T, Q8>(xr[it], p.qs);
#pragma unroll
    for (int it = 0; it < WIT; ++it)
      if (it * 256 + tid < WV) s_w[it * 256 + tid] = wr[it];
  };

  f32x4 acc[NTN][TMW];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < TMW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one LDS buffer, refilled between barriers; the next chunk is in registers during the MFMAs
  const int nchunks = p.Cin / BK;
  load_chunk(0);
  store_chunk();
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    if (ch + 1 < nchunks) load_chunk((ch + 1) * BK);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      opv af[NTN], bf[TMW];
#pragma unroll
      for (int i = 0; i < NTN; ++i) af[i] = s_w[((i * 9 + tap) * 4 + g) * 16 + r16];
#pragma unroll
      for (int j = 0; j < TMW; ++j) {
        const int row = min(wave + 4 * j, TH - 1);  // clamped rows of a short last round are masked
        bf[j] = s_x[hslot<S>((row * S + ky) * IW + r16 * S + kx, g)];
      }
#pragma unroll
      for (int j = 0; j < TMW; ++j)
#pragma unroll
        for (int i = 0; i < NTN; ++i) acc[i][j] = mfma_op<T, Q8>(af[i], bf[j], acc[i][j]);
    }
    if (ch + 1 < nchunks) {
      __syncthreads();  // every wave is done reading this chunk
      store_chunk();
      __syncthreads();
    }
  }

  int64_t pp[TMW];
  bool pv[TMW];
#pragma unroll
  for (int j = 0; j < TMW; ++j) {
    const int row = wave + 4 * j;
    const int oy = oy0 + row, ox = ox0 + r16;
    pv[j] = row < TH && oy < p.Ho && ox < p.Wo;
    pp[j] = ((int64_t)b * p.Ho + oy) * p.Wo + ox;
  }
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = co0 + i * 16 + 4 * g;
  conv_epilogue<T, NTN, TMW, Q8>(p, acc, pp, pv, co);
}

template <typename T, bool Q8, int S, int TH>
static void launch_halo(const ConvArgs<T>& a, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, 16), tiles_y = (int)cdiv(a.Ho, TH);
  const int64_t ntiles = (int64_t)a.N * tiles_y * tiles_x;
  if (a.Cout <= 32) {
    conv3x3_halo_kernel<T, S, TH, 2, Q8><<<(unsigned)ntiles, 256, 0, s>>>(a, tiles_x, tiles_y, 1);
  } else {
    const int cs = (int)cdiv(a.Cout, 64);
    conv3x3_halo_kernel<T, S, TH, 4, Q8><<<(unsigned)(ntiles * cs), 256, 0, s>>>(a, tiles_x, tiles_y, cs);
  }
}

// 3x3, pad 1, dil 1, stride 1/2, Cin a multiple of BK and >= 2 chunks.  Returns false when the
// shape is not this kernel's (the caller falls back to the implicit-GEMM kernels).
// Where the halo tile beats the implicit GEMM (scripts/conv_bench.py, fp16, MI355X): stride 1 on
// >= 51200 output pixels, except deep-K convs with few output columns (384->64 @40^2 bs32 stays
// on conv_wsk_kernel, 79 vs 86 us).  Measured: 256->32 @80^2 bs32 132 -> 62 us, 512->64 @80^2 bs64
// 714 -> 382 us, 768->128 @40^2 bs64 534 -> 348 us, 1024->128 @160^2 bs8 1371 -> 688 us.
// 16-row tiles where the map allows (weights staged once per 256 pixels instead of 128),
// 4-row tiles when 8-row tiles would leave fewer than 512 workgroups.
template <typename T, bool Q8>
bool try_conv3x3_halo(const ConvArgs<T>& a, int kh, hipStream_t s) {
  constexpr int BK = 4 * Vec<T>::N;
  if (kh != 3 || a.KW != 3 || a.PAD != 1 || a.DIL != 1 || a.S != 1) return false;
  if (a.Cin % BK || a.Cin < 2 * BK || a.xcs % Vec<T>::N) return false;
  if ((int64_t)a.P < 51200) return false;
  if (a.Cin > 256 && (int64_t)a.P * a.Cout <= 51200LL * 64) return false;
  const int64_t csplit = cdiv(a.Cout, 64);
  const int64_t tiles8 = (int64_t)a.N * cdiv(a.Ho, 8) * cdiv(a.Wo, 16) * csplit;
  const int64_t tiles16 = (int64_t)a.N * cdiv(a.Ho, 16) * cdiv(a.Wo, 16) * csplit;
  if (a.Ho % 16 == 0 && a.Cout > 32 && tiles16 >= 512) launch_halo<T, Q8, 1, 16>(a, s);
  else if (tiles8 < 512) launch_halo<T, Q8, 1, 4>(a, s);
  else launch_halo<T, Q8, 1, 8>(a, s);
  return true;
}

template bool try_conv3x3_halo<_Float16, false>(const ConvArgs<_Float16>&, int, hipStream_t);
template bool try_conv3x3_halo<_Float16, true>(const ConvArgs<_Float16>&, int, hipStream_t);
template bool try_conv3x3_halo<float, false>(const ConvArgs<float>&, int, hipStream_t);

}  // namespace ydbl
