// Deep-K 3x3 stride-1 convolution (fp16) with an LDS-DMA ring: the head's 384->64 / 256->32 / 192->64 / 64->128
// convs (U/nn/modules/block.py:344-357 Bottleneck cv1/cv2, head.py:84-90 Detect cv2; conv.py:39-63 after fuse).
//
// What bounds the register-staged halo kernel (conv3x3.hip) on these shapes, measured with its timing-only switch
// (scripts/gpu_r05_diag.sh, kbench bs16, 384->64 @40^2): the whole launch 26.6 us, its chunk staging alone (no
// MFMAs) 24.7 us, its MFMAs alone (no restaging) 16.2 us -- the per-chunk global round trips and the
// store-barrier-compute-barrier sequence do not overlap, and at two workgroups per CU nothing else fills the gap.
// Here the staging never passes through registers: every 32-channel chunk (the (TH+2) x 18 input halo and the
// chunk's [co][9 taps][32] weights, in the halo kernel's LDS slot layouts) is copied global -> LDS by
// buffer_load_dwordx4 ... lds (one KiB per wave instruction, lane-linear in the slot order; out-of-image pixels and
// rows past Cout read as zero through the buffer range check), R chunks deep, so chunk c+R-1 is in flight while
// chunk c is multiplied: one raw barrier per chunk, counted vmcnt waits, no vmcnt(0) in the loop.  One workgroup
// per CU (the ring is ~135 KiB of LDS) with taller tiles (TH rows x 16 columns), so each staged weight chunk
// serves more pixels.  The MFMA part is the halo kernel's (same fragments, same accumulation order per output:
// bit-identical results).
#include <stdlib.h>
#include <string.h>

#include "conv_common.hpp"

namespace ydbl {

namespace {

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt[5:4] at
// bits 15:14)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

}  // namespace

constexpr uint32_t RING_OOB = 0x80000000u;  // a voffset past every buffer's num_records: the load returns zeros

template <int TH, int NTN, int R, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void conv3x3_ring_kernel(ConvArgs<_Float16> p, int tiles_x, int tiles_y,
                                                                     int co_splits, uint32_t xbytes) {
  constexpr int TW = 16, IH = TH + 2, IW = TW + 2, NPIX = IH * IW;
  constexpr int XG = (NPIX + 15) / 16;                     // halo slot groups: 16 pixels x 4 k-vectors = 1 KiB
  constexpr int WGR = NTN * 9;                             // weight slot groups: 16 rows x 4 k-vectors of one tap
  constexpr int XPW = (XG + WAVES - 1) / WAVES, WPW = (WGR + WAVES - 1) / WAVES;
  constexpr int PER = XPW + WPW;                           // LDS-DMA instructions per wave per chunk
  constexpr int STAGE = (XG + WGR) * 1024;                 // bytes per ring slot
  constexpr int TMW = (TH + WAVES - 1) / WAVES;            // output rows (16-pixel MFMA tiles) per wave
  static_assert(R >= 2 && (R - 2) * PER < 64, "ring depth");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[R * STAGE + WAVES * 1024];  // + a junk KiB per wave

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = wave_id();
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = p.N * tiles_y * tiles_x;
  int bid = xcd_remap(blockIdx.x, ntiles * co_splits);
  const int cs = bid % co_splits;
  bid /= co_splits;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 - 1, ix0 = ox0 - 1;
  const int co0 = cs * NTN * 16;

  // per-lane byte offsets of the 16-byte vectors this lane copies for each of its wave's slot groups (chunk 0;
  // a chunk adds its channel offset as the scalar soffset).  Group c, lane L: k-vector L / 16, pixel / row L % 16 --
  // slot c * 64 + L of the halo kernel's layouts (hslot<1>, weights [(cb*9 + tap)*4 + g]*16 + r).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.Cout * p.KPAD * 2, 0x00020000);
  uint32_t xoff[XPW], woff[WPW];
#pragma unroll
  for (int j = 0; j < XPW; ++j) {
    const int c = j * WAVES + wave;
    const int px = c * 16 + r16;
    const int hy = px / IW, hx = px - hy * IW;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = c < XG && px < NPIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    xoff[j] = ok ? (uint32_t)((((int64_t)(b * p.H + iy) * p.W + ix) * p.xcs + g * 8) * 2) : RING_OOB;
  }
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int c = j * WAVES + wave;
    const int tap = c % 9, cb = c / 9;
    const int co = co0 + cb * 16 + r16;
    const bool ok = c < WGR && co < p.Cout;
    woff[j] = ok ? (uint32_t)(((int64_t)co * p.KPAD + tap * p.Cin + g * 8) * 2) : RING_OOB;
  }
  unsigned char* junk = smem + R * STAGE + wave * 1024;
  auto issue = [&](int chunk, int slot) {  // chunk's 32 channels -> ring slot `slot`, PER instructions per wave
    unsigned char* st = smem + slot * STAGE;
    const uint32_t so = (uint32_t)chunk * 64;  // 32 channels x 2 bytes
#pragma unroll
    for (int j = 0; j < XPW; ++j) {
      const int c = j * WAVES + wave;
      glds16(xr, c < XG ? st + c * 1024 : junk, xoff[j], so);
    }
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int c = j * WAVES + wave;
      glds16(wr, c < WGR ? st + (XG + c) * 1024 : junk, woff[j], so);
    }
  };

  f32x4 acc[NTN][TMW];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < TMW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.Cin / 32;
#pragma unroll
  for (int c = 0; c < R - 1; ++c)
    if (c < nchunks) issue(c, c);
  for (int ch = 0; ch < nchunks; ++ch) {
    // this wave's copies of chunk ch have landed once at most (chunks issued after it) x PER are outstanding
    const int after = min(R - 2, nchunks - 1 - ch);
    if (after >= R - 2) wait_vm<(R - 2) * PER>();
    else if (R > 3 && after == 1) wait_vm<PER>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's copies of chunk ch are in; every wave is done with chunk ch - 1
    if (ch + R - 1 < nchunks) issue(ch + R - 1, (ch + R - 1) % R);  // into the slot chunk ch - 1 used
    const h8* s_x = reinterpret_cast<const h8*>(smem + (ch % R) * STAGE);
    const h8* s_w = reinterpret_cast<const h8*>(smem + (ch % R) * STAGE + XG * 1024);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      h8 af[NTN], bf[TMW];
#pragma unroll
      for (int i = 0; i < NTN; ++i) af[i] = s_w[((i * 9 + tap) * 4 + g) * 16 + r16];
#pragma unroll
      for (int j = 0; j < TMW; ++j) {
        const int row = min(wave + WAVES * j, TH - 1);  // clamped rows of a short last round are masked
        bf[j] = s_x[hslot<1>((row + ky) * IW + r16 + kx, g)];
      }
#pragma unroll
      for (int j = 0; j < TMW; ++j)
#pragma unroll
        for (int i = 0; i < NTN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  int64_t pp[TMW];
  bool pv[TMW];
#pragma unroll
  for (int j = 0; j < TMW; ++j) {
    const int row = wave + WAVES * j;
    const int oy = oy0 + row, ox = ox0 + r16;
    pv[j] = row < TH && oy < p.Ho && ox < p.Wo;
    pp[j] = ((int64_t)b * p.Ho + oy) * p.Wo + ox;
  }
  int co[NTN];
#pragma unroll
  for (int i = 0; i < NTN; ++i) co[i] = co0 + i * 16 + 4 * g;
  conv_epilogue<_Float16, NTN, TMW, false>(p, acc, pp, pv, co);
}

template <int TH, int NTN, int R, int WAVES>
static void launch_ring(const ConvArgs<_Float16>& a, uint32_t xbytes, hipStream_t s) {
  const int tiles_x = (int)cdiv(a.Wo, 16), tiles_y = (int)cdiv(a.Ho, TH);
  const int cs = (int)cdiv(a.Cout, NTN * 16);
  const int64_t grid = (int64_t)a.N * tiles_y * tiles_x * cs;
  conv3x3_ring_kernel<TH, NTN, R, WAVES><<<(unsigned)grid, WAVES * 64, 0, s>>>(a, tiles_x, tiles_y, cs, xbytes);
}

// fp16 3x3, pad 1, dil 1, stride 1, Cin a multiple of 32 with >= 2 chunks, the input's byte extent within the
// buffer range check's 31 bits.  YDBL_HALO_RING=TH[,WAVES] (experiment switch): route such convs here.
bool try_conv3x3_ring(const ConvArgs<_Float16>& a, int kh, hipStream_t s) {
  const char* e = getenv("YDBL_HALO_RING");
  if (!e) return false;
  if (kh != 3 || a.KW != 3 || a.PAD != 1 || a.DIL != 1 || a.S != 1) return false;
  if (a.Cin % 32 || a.Cin < 64 || a.xcs % 8) return false;
  const int64_t xbytes = ((int64_t)(a.N * a.H * a.W - 1) * a.xcs + a.Cin) * 2;
  if (xbytes + (int64_t)a.Cin * 2 >= (int64_t)RING_OOB || (int64_t)a.Cout * a.KPAD * 2 >= (int64_t)RING_OOB) return false;
  const int th = atoi(e);
  const char* c = strchr(e, ',');
  const int waves = c ? atoi(c + 1) : 4;
  const uint32_t xb = (uint32_t)xbytes;
  if (waves == 8) {
    if (th == 16) return launch_ring<16, 2, 3, 8>(a, xb, s), true;
    if (th == 20) return launch_ring<20, 2, 3, 8>(a, xb, s), true;
    return launch_ring<8, 2, 3, 8>(a, xb, s), true;
  }
  if (th == 16) return launch_ring<16, 2, 3, 4>(a, xb, s), true;
  if (th == 20) return launch_ring<20, 2, 3, 4>(a, xb, s), true;
  return launch_ring<8, 2, 3, 4>(a, xb, s), true;
}

}  // namespace ydbl
