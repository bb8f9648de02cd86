// LSKblock (U/nn/modules_attention/LSKA.py:28-52) after its depthwise pair, in two launches instead of five
// (conv1, conv2, the gate's stats and gating kernels, conv):
//
//   ydbl_lsk_attn  attn = [conv1(a1) | conv2(a2)] (+ bias): one workgroup owns 16*TM pixels and ALL dim output
//                  channels (waves 0-1 conv1 over a1, waves 2-3 conv2 over a2), MFMA operands straight from
//                  global (the weights are L2-resident, each wave's A rows are its own), one-deep register
//                  prefetch.  The rounded attn tile also goes to LDS, where 32 lanes per pixel reduce it to
//                  agg = (mean, max) in lsk_stats_kernel's order -- the stats launch is gone.
//   ydbl_lsk_out   per pixel the 7x7 squeeze of agg (16 lanes share the 98 taps as lsk_gate_kernel does),
//                  sigmoid, gated = a1' * s0 + a2' * s1 rounded into the MFMA B tile in LDS, then
//                  y = x * (conv(gated) + b) -- the gated map never leaves the CU.
//
// Every rounding point and accumulation order is that of the kernels it replaces (conv_igemm_kernel's k-step
// MFMA chain and epilogue, lsk_stats_kernel, lsk_gate_kernel with gate_mix), so the result is bit-identical to
// the five launches whenever those run the block GEMM (tests/test_gpu_ops.py::test_lsk_fused_bit_identical).
#include "conv_common.hpp"

namespace ydbl {

__device__ __forceinline__ int lsk_bswz(int row, int kv) { return row * 4 + (kv ^ (((row >> 2) & 1) << 1)); }

template <int DIM, int TM>
__global__ __launch_bounds__(256) void lsk_attn_kernel(DView<const _Float16> a1, DView<const _Float16> a2,
                                                       const _Float16* __restrict__ w12, const float* __restrict__ b12,
                                                       DView<_Float16> attn, float* __restrict__ agg, int P) {
  constexpr int TN = DIM / 64;  // 16-channel tiles per wave (a wave owns DIM/4 output channels)
  constexpr int NK = DIM / 32;  // k-steps
  constexpr int NPX = 16 * TM;
  constexpr int RP = DIM + 8;  // padded row pitch: the 16 pixels of a store hit distinct banks
  __shared__ _Float16 s_at[NPX * RP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * NPX;
  const DView<const _Float16> src = wave < 2 ? a1 : a2;  // wave-uniform: conv1 over a1, conv2 over a2
  const int cw = wave * (DIM / 4);

  const _Float16* bp[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) bp[j] = src.pix(min(m0 + j * 16 + r16, P - 1)) + g * 8;
  const _Float16* ap[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) ap[i] = w12 + (int64_t)(cw + i * 16 + r16) * DIM + g * 8;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  h8 af[2][TN], bf[2][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i) af[0][i] = vload(ap[i]);
#pragma unroll
  for (int j = 0; j < TM; ++j) bf[0][j] = vload(bp[j]);
#pragma unroll 2
  for (int ks = 0; ks < NK; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < NK) {
#pragma unroll
      for (int i = 0; i < TN; ++i) af[cur ^ 1][i] = vload(ap[i] + (ks + 1) * 32);
#pragma unroll
      for (int j = 0; j < TM; ++j) bf[cur ^ 1][j] = vload(bp[j] + (ks + 1) * 32);
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0);
  }

  // epilogue (conv_epilogue's arithmetic: + bias, no activation), attn to HBM and to the LDS tile
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int co = cw + i * 16 + 4 * g;
    float bv[4];
    load_f<4>(b12 + co, bv);
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q] + bv[q];
      const h4 hv = to_h4_rne(v);
      const int pl = j * 16 + r16;
      *reinterpret_cast<h4*>(&s_at[pl * RP + co]) = hv;
      if (m0 + pl < P) *reinterpret_cast<h4*>(attn.pix(m0 + pl) + co) = hv;
    }
  }
  __syncthreads();

  // stats: 32 lanes per pixel, lane `sub` walks the 8-channel vectors sub, sub + 32, ... (lsk_stats_kernel)
  constexpr int L = 32;
#pragma unroll
  for (int it = 0; it < NPX * L / 256; ++it) {
    const int t = tid + it * 256;
    const int pl = t / L, sub = t % L;
    float s = 0.f, m = -INFINITY;
#pragma unroll
    for (int c = sub * 8; c < DIM; c += L * 8) {
      const h8 v = *reinterpret_cast<const h8*>(&s_at[pl * RP + c]);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s += float(v[q]);
        m = fmaxf(m, float(v[q]));
      }
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) {
      s += __shfl_xor(s, o);
      m = fmaxf(m, __shfl_xor(m, o));
    }
    if (sub == 0 && m0 + pl < P) {
      agg[(int64_t)(m0 + pl) * 2 + 0] = s / float(DIM);
      agg[(int64_t)(m0 + pl) * 2 + 1] = m;
    }
  }
}

template <int DIM, int TM>
__global__ __launch_bounds__(256) void lsk_out_kernel(DView<const _Float16> attn, const float* __restrict__ agg,
                                                      const float* __restrict__ sw, const float* __restrict__ sb,
                                                      const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                      DView<const _Float16> x, DView<_Float16> y, int P) {
  constexpr int HALF = DIM / 2;
  constexpr int NV = HALF / 8;    // 8-channel vectors of the gated map per pixel
  constexpr int NKS = HALF / 32;  // k-steps of conv
  constexpr int TN = DIM / 64;
  constexpr int NPX = 16 * TM;
  static_assert(NV % 16 == 0, "16 lanes per pixel");
  __shared__ h8 s_g[NKS * NPX * 4];  // gated B tile [k-step][pixel][slot]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * NPX;
  const int cw = wave * (DIM / 4);

  // A fragments of the first k-step early (L2 latency under the gate phase)
  const _Float16* ap[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) ap[i] = w + (int64_t)(cw + i * 16 + r16) * HALF + g * 8;
  h8 af[2][TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) af[0][i] = vload(ap[i]);

  // ---- gate: 16 lanes per pixel
  const int l16 = tid & 15;
#pragma unroll
  for (int pass = 0; pass < TM; ++pass) {
    const int pl = pass * 16 + (tid >> 4);
    const int px = m0 + pl;
    const bool ok = px < P;
    const int pc = ok ? px : P - 1;
    const int ox = pc % y.w;
    const int t = pc / y.w;
    const int oy = t % y.h, b = t / y.h;
    float s0 = 0.f, s1 = 0.f;
    for (int tap = l16; tap < 98; tap += 16) {
      const int ci = tap / 49, ky = (tap % 49) / 7, kx = tap % 7;
      const int iy = oy - 3 + ky, ix = ox - 3 + kx;
      if (iy < 0 || iy >= y.h || ix < 0 || ix >= y.w) continue;
      const float a = agg[(((int64_t)b * y.h + iy) * y.w + ix) * 2 + ci];
      s0 = fmaf(sw[((0 * 2 + ci) * 7 + ky) * 7 + kx], a, s0);
      s1 = fmaf(sw[((1 * 2 + ci) * 7 + ky) * 7 + kx], a, s1);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
    s0 = sigmoidf_(s0 + sb[0]);
    s1 = sigmoidf_(s1 + sb[1]);
    const _Float16* ar = attn.pix(pc);
#pragma unroll
    for (int cv = l16; cv < NV; cv += 16) {
      const h8 va = *reinterpret_cast<const h8*>(ar + cv * 8);
      const h8 vb = *reinterpret_cast<const h8*>(ar + HALF + cv * 8);
      h8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = ok ? f16_rne(gate_mix(float(va[q]), s0, float(vb[q]), s1)) : _Float16(0);
      s_g[(cv >> 2) * NPX * 4 + lsk_bswz(pl, cv & 3)] = o;
    }
  }
  __syncthreads();

  // ---- conv (1x1, HALF -> DIM) on MFMA, then y = x * (acc + b)
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int ks = 0; ks < NKS; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < NKS) {
#pragma unroll
      for (int i = 0; i < TN; ++i) af[cur ^ 1][i] = vload(ap[i] + (ks + 1) * 32);
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const h8 bf = s_g[ks * NPX * 4 + lsk_bswz(j * 16 + r16, g)];
#pragma unroll
      for (int i = 0; i < TN; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[cur][i], bf, acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int px = m0 + j * 16 + r16;
    const int pc = px < P ? px : P - 1;
    float rv[TN][4];
#pragma unroll
    for (int i = 0; i < TN; ++i) load_f<4>(x.pix(pc) + cw + i * 16 + 4 * g, rv[i]);
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int co = cw + i * 16 + 4 * g;
      float bv[4], v[4];
      load_f<4>(bias + co, bv);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = rv[i][q] * (acc[i][j][q] + bv[q]);
      if (px < P) store_f<4>(y.pix(px) + co, v);
    }
  }
}

template <int DIM>
static void lsk_go(const ydbl_lsk_desc* d, bool out, hipStream_t s) {
  constexpr int TM = 2;
  const int P = d->x.n * d->x.h * d->x.w;
  const unsigned blocks = (unsigned)cdiv(P, 16 * TM);
  auto cv = [](const ydbl_view& v) { return DView<const _Float16>{reinterpret_cast<const _Float16*>(v.ptr), v.n, v.h, v.w, v.c, v.cs}; };
  if (!out)
    lsk_attn_kernel<DIM, TM><<<blocks, 256, 0, s>>>(cv(d->a1), cv(d->a2), reinterpret_cast<const _Float16*>(d->w12),
                                                    d->b12, dview<_Float16>(d->attn), d->agg, P);
  else
    lsk_out_kernel<DIM, TM><<<blocks, 256, 0, s>>>(cv(d->attn), d->agg, d->sw, d->sb,
                                                   reinterpret_cast<const _Float16*>(d->w), d->b, cv(d->x),
                                                   dview<_Float16>(d->y), P);
}

static int lsk_check(const ydbl_lsk_desc* d, const char* what) {
  if (!d) return fail(YDBL_EINVAL, std::string(what) + ": null descriptor");
  const ydbl_view* vs[5] = {&d->x, &d->a1, &d->a2, &d->attn, &d->y};
  const char* names[5] = {"lsk.x", "lsk.a1", "lsk.a2", "lsk.attn", "lsk.y"};
  for (int i = 0; i < 5; ++i) {
    if (check_view(vs[i], names[i], true)) return YDBL_EINVAL;
    const ydbl_view& v = *vs[i];
    if (v.dtype != YDBL_F16 || v.n != d->x.n || v.h != d->x.h || v.w != d->x.w || v.c != d->x.c)
      return fail(YDBL_EINVAL, std::string(what) + ": x, a1, a2, attn, y must be fp16 views of one [n,h,w,dim] shape");
  }
  if (d->x.c != 256 && d->x.c != 512) return fail(YDBL_EINVAL, std::string(what) + ": dim must be 256 or 512");
  if (!d->w12 || !d->b12 || !d->sw || !d->sb || !d->w || !d->b || !d->agg)
    return fail(YDBL_EINVAL, std::string(what) + ": null weights / workspace");
  return 0;
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int ydbl_lsk_attn(const ydbl_lsk_desc* d, void* stream) {
  if (int e = lsk_check(d, "lsk_attn")) return e;
  if (d->x.c == 256) lsk_go<256>(d, false, as_stream(stream));
  else lsk_go<512>(d, false, as_stream(stream));
  return check_launch("ydbl_lsk_attn");
}

extern "C" int ydbl_lsk_out(const ydbl_lsk_desc* d, void* stream) {
  if (int e = lsk_check(d, "lsk_out")) return e;
  if (d->x.c == 256) lsk_go<256>(d, true, as_stream(stream));
  else lsk_go<512>(d, true, as_stream(stream));
  return check_launch("ydbl_lsk_out");
}
