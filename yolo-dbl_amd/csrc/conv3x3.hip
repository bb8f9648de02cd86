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
#include <stdlib.h>

#include <algorithm>

#include "conv_common.hpp"

namespace ydbl {


// NB > 1 (N-blocking): the workgroup takes the same tile of NB consecutive images, so every staged weight chunk feeds NB
// times the MFMAs (the weights are most of a deep-K chunk's bytes: 384->64 @40^2, 8-row tile, 64 channels: 36.9 KB
// of weights against 11.5 KB of halo per 32-channel chunk).
template <typename T, int S, int TH, int NTN, bool Q8, int NB = 1>
__global__ __launch_bounds__(256, 2) void conv3x3_halo_kernel(ConvArgs<T> p, int tiles_x, int tiles_y,
                                                              int co_splits) {
  constexpr int TW = 16;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = 4 * VEC;
  constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3;
  constexpr int NPIX = IH * IW;
  constexpr int XSLOTS = (NPIX + 16 * S - 1) / (16 * S) * (64 * S);
  constexpr int WV = NTN * 16 * 36;  // weight vectors per k-step
  constexpr int XIT = (XSLOTS + 255) / 256, WIT = (WV + 255) / 256;
  constexpr int TMW = (TH + 3) / 4;  // 16-pixel tiles (= output rows) per wave
  using vec = typename Vec<T>::type;
  using opv = typename Op<T, Q8>::lds;  // 8-byte e4m3 groups in fp8 mode (same slot layout)
  __shared__ opv s_x[NB * XSLOTS];
  __shared__ opv s_w[WV];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = (p.N + NB - 1) / NB * tiles_y * tiles_x;
  int bid = xcd_remap(blockIdx.x, ntiles * co_splits);
  const int cs = bid % co_splits;
  bid /= co_splits;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b0 = bid / tiles_y * NB;  // first image of the block
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const int co0 = cs * NTN * 16;
  __shared__ __align__(16) float s_bias[NTN * 16];
  BiasStage<NTN * 16> bst;
  bst.fetch(p.bias, co0, p.Cout);

  // Staging walks LDS slots linearly (consecutive lanes -> consecutive 16-byte slots, so the
  // ds_write_b128s are conflict-free) and gathers the matching global vectors: a wave still
  // covers 16 pixels x 64 B (halo) / 16 rows x 64 B (weights) of global memory.  The per-lane
  // source offsets are chunk-invariant and computed once.  (Lane maps that read whole 64-byte pieces per
  // lane quad cut the TCP accesses 3.2x and TD busy 1.7x but not the time: 384->64 @40^2 bs16 29.6 vs 30.2 us,
  // profiles/r05/r05_halo_lane_map_ab.txt.)
  const T* xsrc[NB][XIT];
  bool xok[NB][XIT];
#pragma unroll
  for (int it = 0; it < XIT; ++it) {
    const int slot = min(it * 256 + tid, XSLOTS - 1);
    const int blk = slot / (64 * S), rem = slot % (64 * S);
    const int gv = rem / (16 * S), r2 = rem % (16 * S);
    const int px = blk * 16 * S + (r2 & 15) * S + r2 / 16;
    const int hy = px / IW, hx = px - hy * IW;
    const int iy = iy0 + hy, ix = ix0 + hx;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int b = min(b0 + nb, p.N - 1);
      xok[nb][it] = b0 + nb < p.N && px < NPIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      xsrc[nb][it] = p.x + ((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + gv * VEC;
    }
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
  // raw loads, zero selects at the LDS store (vload_clamped): the next chunk stays in flight during the MFMAs
  vec xr[NB][XIT];
  opv wr[WIT];
  bool cok = true;
  auto load_chunk = [&](int c0) {
    cok = c0 < p.Cin;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int it = 0; it < XIT; ++it) xr[nb][it] = vload_clamped(xsrc[nb][it] + c0, p.x, xok[nb][it] && cok);
#pragma unroll
    for (int it = 0; it < WIT; ++it) wr[it] = load_wop_raw<T, Q8>(p.w, wsrc[it] + c0, wok[it] && cok);
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int it = 0; it < XIT; ++it)
        if (it * 256 + tid < XSLOTS)
          s_x[nb * XSLOTS + it * 256 + tid] = to_op<T, Q8>(vsel(xr[nb][it], xok[nb][it] && cok), p.qs);
#pragma unroll
    for (int it = 0; it < WIT; ++it)
      if (it * 256 + tid < WV) s_w[it * 256 + tid] = vsel(wr[it], wok[it] && cok);
  };

  f32x4 acc[NTN][NB * TMW];  // [channel tile][image nb * TMW + row round j]
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < NB * TMW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one LDS buffer, refilled between barriers; the next chunk is in registers during the MFMAs (two buffers and
  // one barrier per chunk measured even or slower: kbench bs16 384->64 @40^2 27.0 vs 26.7 us, 64->128 13.2 vs 15.7;
  // two k-steps per chunk, fewer barriers: 384->64 26.6 -> 28.2 us; timing split with the staging or the MFMAs
  // switched off: staging holds 24.7 of 26.6 us; an LDS-DMA chunk ring (buffer_load ... lds, 2-4 chunks in flight,
  // bit-identical) 26.4-27.1 us -- profiles/r05/r05_halo_*.txt)
  // split-K (ksplit > 1, launch_halo): workgroup z of the tile takes input-channel chunks [c0, c1)
  const int nchunks_all = p.Cin / BK;
  const int z = blockIdx.y;
  const int c0 = z * nchunks_all / p.ksplit, c1 = (z + 1) * nchunks_all / p.ksplit;
  load_chunk(c0 * BK);
  store_chunk();
  bst.commit(s_bias);
  __syncthreads();
  const int nchunks = c1;
  for (int ch = c0; ch < nchunks; ++ch) {
    if (ch + 1 < nchunks) load_chunk((ch + 1) * BK);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      opv af[NTN], bf[NB * TMW];
#pragma unroll
      for (int i = 0; i < NTN; ++i) af[i] = s_w[((i * 9 + tap) * 4 + g) * 16 + r16];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int j = 0; j < TMW; ++j) {
          const int row = min(wave + 4 * j, TH - 1);  // clamped rows of a short last round are masked
          bf[nb * TMW + j] = s_x[nb * XSLOTS + hslot<S>((row * S + ky) * IW + r16 * S + kx, g)];
        }
#pragma unroll
      for (int j = 0; j < NB * TMW; ++j)
#pragma unroll
        for (int i = 0; i < NTN; ++i) acc[i][j] = mfma_op<T, Q8>(af[i], bf[j], acc[i][j]);
    }
    if (ch + 1 < nchunks) {
      __syncthreads();  // every wave is done reading this chunk
      store_chunk();
      __syncthreads();
    }
  }

  int64_t pp[NB * TMW];
  bool pv[NB * TMW];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int j = 0; j < TMW; ++j) {
      const int row = wave + 4 * j;
      const int oy = oy0 + row, ox = ox0 + r16;
      pv[nb * TMW + j] = b0 + nb < p.N && row < TH && oy < p.Ho && ox < p.Wo;
      pp[nb * TMW + j] = ((int64_t)(b0 + nb) * p.Ho + oy) * p.Wo + ox;
    }
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = co0 + i * 16 + 4 * g;
  if (p.ksplit > 1) {  // this split's partial tile (f32), summed + epilogue by splitk_epilogue_kernel (conv.hip)
    const int cs4 = (p.Cout + 3) & ~3;
#pragma unroll
    for (int j = 0; j < NB * TMW; ++j)
#pragma unroll
      for (int i = 0; i < NTN; ++i)
        if (pv[j] && co[i] < p.Cout) *reinterpret_cast<f32x4*>(p.ws + ((int64_t)z * p.P + pp[j]) * cs4 + co[i]) = acc[i][j];
    return;
  }
  conv_epilogue<T, NTN, NB * TMW, Q8>(p, acc, pp, pv, co, s_bias, co0);
}

template <typename T, bool Q8>
void launch_splitk_epilogue(const ConvArgs<T>& a, hipStream_t s);  // conv.hip

// Split-K of the halo kernel for the deep-K stride-1 convs on small maps (fewer than 25600 output pixels: the 40^2
// maps of a bs4 sub-batch), where a workgroup per tile leaves the chip idle behind a long serial chunk chain
// (DBL-s 768->128 @40^2 bs4: 24 chunks; on the wave-split-K kernel it took 53.7 us, its 32-pixel tiles re-reading the
// whole weight slice 200 times): up to 4 workgroups per tile over the input-channel chunks, >= 3 chunks each,
// toward 512 workgroups; the partials summed in split order by the epilogue kernel.
constexpr int HALO_SPLIT_MIN_CHUNKS = 8;
template <typename T>
int halo_ksplit(const ConvArgs<T>& a, int64_t wgs) {
  const char* e = getenv("YDBL_SPLITK");
  if (sizeof(T) != 2 || (e && *e == '0') || (int64_t)a.P >= 25600) return 1;  // fp16 only (conv.hip wsk_ksplit)
  const int nch = a.Cin / (4 * Vec<T>::N);
  if (nch < HALO_SPLIT_MIN_CHUNKS) return 1;
  int k = (int)std::min<int64_t>(4, (512 + wgs - 1) / wgs);
  while (k > 1 && nch / k < 3) --k;
  return k;
}

template <typename T, bool Q8, int S, int TH>
static void launch_halo(const ConvArgs<T>& a0, hipStream_t s) {
  ConvArgs<T> a = a0;
  const int tiles_x = (int)cdiv(a.Wo, 16), tiles_y = (int)cdiv(a.Ho, TH);
  const int64_t ntiles = (int64_t)a.N * tiles_y * tiles_x;
  a.ksplit = 1;
  if (S == 1 && (int64_t)a.P < 25600) {  // (the split's own tiling: 32-channel slices below)
    a.ksplit = halo_ksplit(a, ntiles * cdiv(a.Cout, 32));
    if (a.ksplit > 1 && (!a.ws || a.ws_bytes < (int64_t)a.ksplit * a.P * ((a.Cout + 3) & ~3) * 4)) a.ksplit = 1;
    if (a.ksplit > 1) {
      const int cs = (int)cdiv(a.Cout, 32);
      conv3x3_halo_kernel<T, S, TH, 2, Q8><<<dim3((unsigned)(ntiles * cs), (unsigned)a.ksplit), 256, 0, s>>>(
          a, tiles_x, tiles_y, cs);
      launch_splitk_epilogue<T, Q8>(a, s);
      return;
    }
  }
  // Fewer than 400 64-channel workgroups (the 40^2 head convs of a bs16 sub-batch graph: 240) leave
  // most CUs with one workgroup; 32-channel slices double the grid (conv_bench.py bs16: 384->64 @40^2
  // 40.5 -> 29.5 us, 192->64 22.8 -> 17.3 us; at bs32, 480 workgroups, they lose: 49.2 -> 52.1 us)
  // (512: the 64->128 @40^2 head convs of a bs16 graph, 480 workgroups, also gain: 14.3 -> 13.2 us, kbench;
  // 16-channel slices and 4-row tiles lose on every head shape: profiles/r05/r05_halo_tile_ab.txt)
  constexpr int64_t n2_below = 512;
  // 8-row stride-1 tiles of two images per workgroup (N-blocking), 32-channel slices: half the weight staging per
  // output; each launch takes longer, but with less CU time the two sub-batch branches overlap better -- DBL-n bs32
  // +0.8 %, DBL-s bs64 / DBL-l 1280 bs8 +0.4 %, DBL-s bs8 even (profiles/r06/r06_fusion_switch_sweep.txt,
  // r06_sweep2.txt; per launch in graph at bs16: 384->64 @40^2 28.3 -> 33.5 us, 192->64 17.6 -> 20.2).
  // YDBL_HALO_NB=1 (read per launch; A/B switch): one image per workgroup.
  if constexpr (S == 1 && TH == 8 && !Q8) {
    // (four images per workgroup, or two in 64-channel slices: DBL-n bs32 -3.1 / -2.3 %, r06_sweep3_cumask.txt)
    const char* e = getenv("YDBL_HALO_NB");
    if (!(e && *e == '1') && a.N >= 2) {
      const int64_t nt2 = (int64_t)(a.N + 1) / 2 * tiles_y * tiles_x;
      const int cs = (int)cdiv(a.Cout, 32);
      conv3x3_halo_kernel<T, S, TH, 2, Q8, 2><<<(unsigned)(nt2 * cs), 256, 0, s>>>(a, tiles_x, tiles_y, cs);
      return;
    }
  }
  if (a.Cout <= 32) {
    conv3x3_halo_kernel<T, S, TH, 2, Q8><<<(unsigned)ntiles, 256, 0, s>>>(a, tiles_x, tiles_y, 1);
  } else if (ntiles * cdiv(a.Cout, 64) < n2_below) {
    const int cs = (int)cdiv(a.Cout, 32);
    conv3x3_halo_kernel<T, S, TH, 2, Q8><<<(unsigned)(ntiles * cs), 256, 0, s>>>(a, tiles_x, tiles_y, cs);
  } else {
    const int cs = (int)cdiv(a.Cout, 64);
    conv3x3_halo_kernel<T, S, TH, 4, Q8><<<(unsigned)(ntiles * cs), 256, 0, s>>>(a, tiles_x, tiles_y, cs);
  }
}

// (One chunk in flight: a register ring of two or three was slower on every head shape, kbench bs16 1 / 2 / 3
// chunks: 384->64 @40^2 26.6 / 28.8 / 31.3 us, 256->32 @80^2 28.4 / 32.8 / 47.1, 64->128 @40^2 12.9 / 17.1 / 19.9.)

// 3x3, pad 1, dil 1, stride 1/2, Cin a multiple of BK and >= 2 chunks.  Returns false when the
// shape is not this kernel's (the caller falls back to the implicit-GEMM kernels).
// Where the halo tile beats the implicit GEMM (scripts/conv_bench.py, fp16, MI355X): stride 1 on
// >= 51200 output pixels.  Measured: 256->32 @80^2 bs32 132 -> 62 us, 512->64 @80^2 bs64
// 714 -> 382 us, 768->128 @40^2 bs64 534 -> 348 us, 1024->128 @160^2 bs8 1371 -> 688 us.
// 16-row tiles where the map allows (weights staged once per 256 pixels instead of 128),
// 4-row tiles when 8-row tiles would leave fewer than 512 workgroups.
template <typename T, bool Q8>
bool try_conv3x3_halo(const ConvArgs<T>& a, int kh, hipStream_t s) {
  constexpr int BK = 4 * Vec<T>::N;
  // Stride 2 on >= 204800 output pixels: 8-row tiles over a (2*8+1) x 33 halo (A/B against the block
  // GEMM: DBL-l 128->256 @320 bs8 442 -> 341 us).  Smaller maps stay on the block GEMM: 128->128 @40 bs32
  // 17.8 vs 24.7 us, and DBL-n's 64->64 @80 bs32 (18.8 vs 17.5 us alone) cost the whole step ~40 us.
  if (kh == 3 && a.KW == 3 && a.PAD == 1 && a.DIL == 1 && a.S == 2 && a.Cin % BK == 0 &&
      a.Cin >= 2 * BK && a.xcs % Vec<T>::N == 0 && (int64_t)a.P >= 204800)
    return launch_halo<T, Q8, 2, 8>(a, s), true;
  if (kh != 3 || a.KW != 3 || a.PAD != 1 || a.DIL != 1 || a.S != 1) return false;
  if (a.Cin % BK || a.Cin < 2 * BK || a.xcs % Vec<T>::N) return false;
  // 51200 output pixels (40^2 x 32) was the measured crossover at bs32; the bench's two bs16 sub-batch
  // graphs put the 40^2 head convs at 25600, where the halo tile still wins (DBL-n bs32 on two streams
  // 13.7 k -> 14.1 k img/s; 12800 loses again: 14.0 k)
  if ((int64_t)a.P < 25600) {  // small maps: only as the split-K form (halo_ksplit), with room for its partials
    const int64_t wgs = (int64_t)a.N * cdiv(a.Ho, 8) * cdiv(a.Wo, 16) * cdiv(a.Cout, 32);
    const int k = halo_ksplit(a, wgs);
    if ((int64_t)a.P < 4096) return false;
    if (k >= 2 && a.ws && a.ws_bytes >= (int64_t)k * a.P * ((a.Cout + 3) & ~3) * 4) return launch_halo<T, Q8, 1, 8>(a, s), true;
    // Too few chunks to split (Cin < 256) and wide Cout: the wave-split-K kernel's 32x128 tiles would re-read the
    // whole weight matrix once per 32 pixels (DBL-s bs4: 128->256 @40^2, 200 tile rows x 590 KB); the halo tile in
    // 32-channel slices reads it once per 128 pixels
    // (YDBL_HALO_SMALL=0, read per launch: the wave-split-K route, A/B switch)
    const char* e = getenv("YDBL_HALO_SMALL");
    if (k < 2 && a.Cout >= 128 && !(e && *e == '0')) return launch_halo<T, Q8, 1, 8>(a, s), true;
    return false;
  }
  const int64_t csplit = cdiv(a.Cout, 64);
  const int64_t tiles8 = (int64_t)a.N * cdiv(a.Ho, 8) * cdiv(a.Wo, 16) * csplit;
  const int64_t tiles16 = (int64_t)a.N * cdiv(a.Ho, 16) * cdiv(a.Wo, 16) * csplit;
  // No 4-row tiles by default: every workgroup re-reads all of its channels' weights, so at 480
  // 8-row tiles (40^2 bs32, Cout 64) the doubled grid lost (A/B: 384->64 88.9 vs
  // 49.6 us, 192->64 45.9 vs 28.0 us); 384->64 @40^2 also beats the wave-split-K kernel it used to
  // take (78.8 us).  (P >= 51200 already guarantees >= 400 8-row tiles.)
  (void)tiles8;
  // Cout <= 32 (one 32-channel slice: the weights are as many bytes per chunk as the halo): 16-row tiles from
  // 256 of them (DBL-n's 256->32 @80^2 at bs16, 400 tiles: 34.6 -> 31.8 us in graph, scripts/kbench.py)
  // 16-row tiles only with YDBL_HALO_T16=1 (read per launch): the N-blocked 8-row tiles measured even to +0.7 % against
  // them in the two-branch layout (profiles/r06/r06_conv_route_sweep.txt)
  const char* e16 = getenv("YDBL_HALO_T16");
  if (a.Ho % 16 == 0 && (a.Cout > 32 ? tiles16 >= 512 : tiles16 >= 256) && e16 && *e16 == '1')
    launch_halo<T, Q8, 1, 16>(a, s);
  else launch_halo<T, Q8, 1, 8>(a, s);
  return true;
}

// ---- VGPR-weight 3x3 (fp16, stride 1, Cin 32..128): the bneck.hip layout for a single conv ----------
// The halo kernel above reads both MFMA operands from LDS (a ds_read_b128 per 1.3 MFMAs) and walks Cin
// in chunks behind two barriers each; on the head's 64/128-channel convs (Detect cv2, Bottleneck cv2)
// that held it at 10-15 % of the MFMA rate, against ~30 % for the fused Bottleneck kernel.  Here, as
// there: the whole (TH+2) x 18 input window with all Cin channels is staged once (one plane of 16-byte
// records per 8-channel chunk, 1 KiB contiguous global reads per wave), one barrier, and each wave
// keeps the A fragments of its TPW output-channel tiles in VGPRs for the whole launch, loaded straight
// from the [Cout][KPAD] tap-major weight matrix (lane (co, g) at k-step m reads 8 consecutive input
// channels of one tap: 16 contiguous bytes, no repacking).  Every B fragment read from LDS feeds TPW
// MFMAs.  K order per 32-wide k-step: one tap x 4 chunks (lane group g = chunk 4i+g), so the lane
// groups of a ds_read_b128 hit bank quads PIN*16 bytes apart (PIN a multiple of 16 records): conflict-free.
// Fused epilogue (bias, act, residual, second output) from conv_common.hpp.
template <int CIN, int TPW, int NWG, int TH, int ROWS>
__global__ __launch_bounds__(256, 2) void conv3x3_vw_kernel(ConvArgs<_Float16> p, int tiles_x, int tiles_y, int ntiles,
                                                            int co_splits) {
  constexpr int CH = CIN / 8, KS = 9 * CH / 4, CPT = CH / 4;  // chunks, k-steps, k-steps per tap
  constexpr int TW = 16, IP = TW + 2, IR = TH + 2, NPX = IR * IP, PIN = (NPX + 15) / 16 * 16;
  constexpr int RW = 4 / NWG;  // waves sharing one output-channel group split the rows
  static_assert(CH >= 4 && 32 % CH == 0 && TH % (RW * ROWS) == 0, "conv3x3_vw shape");
  __shared__ __align__(16) unsigned char s_in[CH * PIN * 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int t = xcd_remap(blockIdx.x, ntiles * co_splits);
  const int cs = t % co_splits;  // output-channel slice of NWG * TPW * 16 channels
  t /= co_splits;
  __shared__ __align__(16) float s_bias[NWG * TPW * 16];
  BiasStage<NWG * TPW * 16> bst;
  bst.fetch(p.bias, cs * NWG * TPW * 16, p.Cout);
  const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y, img = t / (tiles_x * tiles_y);
  const int oy0 = ty * TH, ox0 = tx * TW;

  // 1. input window rows oy0-1.., cols ox0-1..: item u*256 + tid -> chunk (tid >> 3) % CH,
  // pixel px0 + u * PXU (8 consecutive pixels x CH chunks per wave instruction)
  constexpr int PXU = 256 / CH, IT = (NPX + PXU - 1) / PXU;
  const int s_chunk = (tid >> 3) % CH, px0 = ((tid >> 3) / CH) * 8 + (tid & 7);
  h8 xr[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int px = px0 + u * PXU;
    const int r = px / IP, c = px - r * IP;
    const int iy = oy0 - 1 + r, ix = ox0 - 1 + c;
    const bool ok = px < NPX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    const _Float16* src = ok ? p.x + ((int64_t)(img * p.H + iy) * p.W + ix) * p.xcs + s_chunk * 8 : p.x;
    const h8 v = *reinterpret_cast<const h8*>(src);
    xr[u] = ok ? v : h8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  // this wave's A fragments: tiles cg*TPW .. +TPW-1 (16 output channels each)
  const int cg = cs * NWG + wave % NWG;
  h8 a[TPW][KS];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const _Float16* wrow = p.w + (int64_t)((cg * TPW + tt) * 16 + r16) * p.KPAD + g * 8;
#pragma unroll
    for (int m = 0; m < KS; ++m)
      a[tt][m] = *reinterpret_cast<const h8*>(wrow + (m / CPT) * CIN + (m % CPT) * 32);
  }
  unsigned char* s_dst = s_in + (s_chunk * PIN + px0) * 16;
#pragma unroll
  for (int u = 0; u < IT; ++u)
    if (px0 + u * PXU < NPX) *reinterpret_cast<h8*>(s_dst + u * PXU * 16) = xr[u];
  int co[TPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) co[tt] = (cg * TPW + tt) * 16 + 4 * g;
  const unsigned char* in_b = s_in + (g * PIN + r16) * 16;
  bst.commit(s_bias);
  __syncthreads();

  // 2. rows j0, j0+1 of the tile per pass; B for (row j, column r16, tap) at record (j+dy)*IP + r16+dx
#pragma nounroll
  for (int j0 = (wave / NWG) * ROWS; j0 < TH; j0 += RW * ROWS) {
    f32x4 acc[TPW][ROWS];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int r = 0; r < ROWS; ++r) acc[tt][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < KS; ++m) {
      const int tap = m / CPT;
      const int o = (((m % CPT) * 4) * PIN + (tap / 3) * IP + tap % 3) * 16;
      h8 bf[ROWS];
#pragma unroll
      for (int r = 0; r < ROWS; ++r) bf[r] = *reinterpret_cast<const h8*>(in_b + (j0 + r) * IP * 16 + o);
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt)
          acc[tt][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[tt][m], bf[r], acc[tt][r], 0, 0, 0);
    }
    int64_t pp[ROWS];
    bool pv[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const int oy = oy0 + j0 + r, ox = ox0 + r16;
      pv[r] = oy < p.Ho && ox < p.Wo;
      pp[r] = ((int64_t)img * p.Ho + oy) * p.Wo + ox;
    }
    conv_epilogue<_Float16, TPW, ROWS, false>(p, acc, pp, pv, co, s_bias, cs * NWG * TPW * 16);
  }
}

// TH16 > 0: 16-row tiles (ROWS16 rows per pass) when the map gives >= 1024 of them (half the halo
// re-reads of 8-row tiles); only configurations that stay spill-free at 16 rows have one.
template <int CIN, int TPW, int NWG, int ROWS8, int ROWS16 = 0>
static void launch_vw(const ConvArgs<_Float16>& a, int cs, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, 16);
  const int64_t t16 = (int64_t)a.N * cdiv(a.Ho, 16) * tiles_x;
  if constexpr (ROWS16 > 0) {
    if (t16 >= 1024) {
      const int tiles_y = (int)cdiv(a.Ho, 16), nt = a.N * tiles_y * tiles_x;
      conv3x3_vw_kernel<CIN, TPW, NWG, 16, ROWS16><<<(unsigned)(nt * cs), 256, 0, s>>>(a, tiles_x, tiles_y, nt, cs);
      return;
    }
  }
  const int tiles_y = (int)cdiv(a.Ho, 8), nt = a.N * tiles_y * tiles_x;
  conv3x3_vw_kernel<CIN, TPW, NWG, 8, ROWS8><<<(unsigned)(nt * cs), 256, 0, s>>>(a, tiles_x, tiles_y, nt, cs);
}

// fp16 3x3 stride-1 pad-1 convs routed to the VGPR-weight kernel; false when the shape is not one of
// them.  TPW output-channel tiles per wave, NWG wave groups over the channels (4 / NWG waves split the
// rows): combinations that fit 256 VGPRs without scratch (scripts/kres.py).
// Only the shapes where it measured faster than the halo / block-GEMM / tile kernels (conv_bench.py,
// bs32, MI355X): 128->64 @40^2 32.3 -> 21.3 us, 64->64 @40^2 20.0 -> 16.5 us.  Every workgroup loads
// all of its channels' weights into VGPRs, so on 80^2 maps (1600 workgroups) and for Cout 32/128 the
// re-read loses (measured with the kernel open to Cin/Cout 32..128: 64->64 @80^2 41.7 -> 47.9,
// 64->32 @80^2 22.5 -> 39.5, 64->128 @40^2 26.0 -> 29.4, 64->64 @20^2 8.9 -> 10.0 us).
bool try_conv3x3_vw(const ConvArgs<_Float16>& a, int kh, hipStream_t s) {
  if (kh != 3 || a.KW != 3 || a.PAD != 1 || a.DIL != 1 || a.S != 1) return false;
  // Round 6: off by default -- the N-blocked halo tile takes these shapes (DBL-n bs32 +0.4 %, DBL-s bs8 +0.7 %, bs64
  // +1.5 %, profiles/r06/r06_conv_route_sweep.txt: less CU time per image in the two-branch layout, though each launch
  // is longer).  YDBL_VW=1 (read per launch) routes them here.
  const char* e = getenv("YDBL_VW");
  if (!(e && *e == '1')) return false;
  if (a.xcs % 8 || a.H != a.Ho || a.W != a.Wo || (int64_t)a.N * a.Ho * a.Wo >= (1LL << 31)) return false;
  if (a.Cin == 128 && a.Cout == 64) return launch_vw<128, 1, 4, 2>(a, 1, s), true;
  constexpr int64_t vw_min = 25601;
  if (a.Cin == 64 && a.Cout == 64 && a.P >= vw_min && a.P <= 65536) return launch_vw<64, 2, 2, 4>(a, 1, s), true;
  return false;
}

template int halo_ksplit<_Float16>(const ConvArgs<_Float16>&, int64_t);
template int halo_ksplit<float>(const ConvArgs<float>&, int64_t);
template bool try_conv3x3_halo<_Float16, false>(const ConvArgs<_Float16>&, int, hipStream_t);
template bool try_conv3x3_halo<_Float16, true>(const ConvArgs<_Float16>&, int, hipStream_t);
template bool try_conv3x3_halo<float, false>(const ConvArgs<float>&, int, hipStream_t);

}  // namespace ydbl
