// AdaHGConv in ONE launch per call (U/nn/modules/block.py:1582-1708: AdaHyperedgeGen + AdaHGConv), for token
// counts whose N x E logits fit in LDS (every DBL-n / DBL-s call at 640: N = 1600 tokens, D = 64 / 128,
// E = 4 / 8, head_dim 16).  hg.hip runs the same math as seven launches (stats, proto, the pre_head_proj
// 1x1 conv, logits, gather, edge, out) of a few microseconds of work each; here one workgroup of 1024
// threads owns one image and keeps everything between the passes on the CU:
//   pass 1  ctx = [mean_N X | max_N X]: threads (8-channel vector, token lane) sweep X, wave shuffles +
//           a 16-wave LDS combine; proto = base + Wc ctx + bc  -> LDS [E][D] fp32;
//   pass 2  xp = X Wp^T + bp on MFMA, one 16-token tile per wave step with the B fragments loaded straight
//           from X (no LDS staging, no barrier), rounded to the activation dtype as the unfused conv stores
//           it; logits[n][e] = mean_h (xp_h[n] . proto_h[e]) / sqrt(16) -> LDS [N][E] fp32 (each 16-channel
//           output tile of the MFMA is one head);
//   softmax over N per hyperedge (max, sum of exp) -> A[n][e] in place;
//   pass 3  He = A^T X (threads as pass 1, per-thread accumulators, shuffle + LDS combine in fixed order);
//           He2 = GELU(He We^T + be), He3 = He2 Wn^T (node_proj re-associated as in hg.hip);
//   pass 4  y[n] = GELU(A[n] He3 + bn) + X[n].
// X is read four times, from L2 (one image is 200-400 KB); the workgroup runs beside the other sub-batch
// stream's kernels on the remaining CUs.  All arithmetic fp32; reduction orders differ from hg.hip's
// (tests/test_gpu_ops.py compares both with the oracle, and with each other).
#include "conv_common.hpp"

namespace ydbl {

constexpr int HGF_NT = 1024, HGF_WAVES = HGF_NT / 64;
constexpr int64_t HGF_LDS_MAX = 160 * 1024 - 1024;  // dynamic LDS cap (the kernel's static s_stat stays inside)

template <typename T, int D, int E>
struct HgfCfg {
  static constexpr int V = Vec<T>::N;           // channels per 16-byte vector
  static constexpr int CV = D / V;              // vectors per token
  static constexpr int TL = HGF_NT / CV;        // token lanes
  static constexpr int TLW = 64 / CV;           // token lanes per wave
  static constexpr int NTC = D / 16;            // 16-channel tiles = heads (head_dim 16)
  static constexpr int KS = D / (4 * V);        // MFMA k-steps over D (32 f16 / 16 f32 channels each)
};

// LDS bytes: logits [N][E] + Wp [D][D] (T) + proto, He, He2/He3 [E][D] + combine scratch [16][max(2D, 4D)]
template <typename T, int D, int E>
constexpr int64_t hgf_lds(int N) {
  return (int64_t)N * E * 4 + (int64_t)D * D * sizeof(T) + 3LL * E * D * 4 + (int64_t)HGF_WAVES * 4 * D * 4 + 256;
}

template <typename T, int D, int E>
__global__ __launch_bounds__(HGF_NT, 1) void hg_fused_kernel(DView<const T> x, DView<T> y, int N, int H,
                                                              const float* __restrict__ base,
                                                              const float* __restrict__ wc, const float* __restrict__ bc,
                                                              const T* __restrict__ wp, const float* __restrict__ bp,
                                                              const float* __restrict__ we, const float* __restrict__ be,
                                                              const float* __restrict__ wn,
                                                              const float* __restrict__ bn) {
  using C = HgfCfg<T, D, E>;
  constexpr int V = C::V, CV = C::CV, TL = C::TL, TLW = C::TLW, NTC = C::NTC, KS = C::KS;
  using vec = typename Vec<T>::type;
  extern __shared__ __align__(16) unsigned char smem[];
  float* s_l = reinterpret_cast<float*>(smem);                    // [N][E] logits, then A
  T* s_wp = reinterpret_cast<T*>(s_l + (int64_t)N * E);           // [D][D] pre_head_proj weight
  float* s_p = reinterpret_cast<float*>(s_wp + D * D);            // [E][D] proto
  float* s_he = s_p + E * D;                                      // [E][D] He, then He3
  float* s_h2 = s_he + E * D;                                     // [E][D] He2
  float* s_red = s_h2 + E * D;                                    // [16 waves][4 * D] combine scratch
  __shared__ float s_stat[2][E];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const T* xb = x.p + (int64_t)b * N * x.cs;
  const int cv = tid % CV, tl = tid / CV;  // pass 1 / 3 / 4 thread roles

  for (int i = tid; i < D * D / V; i += HGF_NT) reinterpret_cast<vec*>(s_wp)[i] = reinterpret_cast<const vec*>(wp)[i];

  // ---------------------------------------------------------------- pass 1: context + prototypes
  {
    float s[V], m[V];
#pragma unroll
    for (int q = 0; q < V; ++q) { s[q] = 0.f; m[q] = -INFINITY; }
#pragma unroll 4
    for (int n = tl; n < N; n += TL) {
      float v[V];
      load_f<V>(xb + (int64_t)n * x.cs + cv * V, v);
#pragma unroll
      for (int q = 0; q < V; ++q) { s[q] += v[q]; m[q] = fmaxf(m[q], v[q]); }
    }
#pragma unroll
    for (int off = CV; off < 64; off <<= 1)
#pragma unroll
      for (int q = 0; q < V; ++q) { s[q] += __shfl_xor(s[q], off); m[q] = fmaxf(m[q], __shfl_xor(m[q], off)); }
    if (lane < CV)
#pragma unroll
      for (int q = 0; q < V; ++q) {
        s_red[wave * 4 * D + cv * V + q] = s[q];
        s_red[wave * 4 * D + D + cv * V + q] = m[q];
      }
    __syncthreads();
    float* ctx = s_h2;  // [2D] (E >= 2: fits in He2's slot until pass 3)
    if (tid < 2 * D) {
      float v = s_red[tid];
      for (int w = 1; w < HGF_WAVES; ++w) v = tid < D ? v + s_red[w * 4 * D + tid] : fmaxf(v, s_red[w * 4 * D + tid]);
      ctx[tid] = tid < D ? v / float(N) : v;
    }
    __syncthreads();
    for (int o = tid; o < E * D; o += HGF_NT) {  // proto[o] = base[o] + (Wc[o] . ctx + bc[o])
      const float* wr = wc + (int64_t)o * 2 * D;
      float acc = 0.f;
#pragma unroll 8
      for (int k = 0; k < 2 * D; k += 4) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(wr + k);
        acc = fmaf(w4[0], ctx[k], acc);
        acc = fmaf(w4[1], ctx[k + 1], acc);
        acc = fmaf(w4[2], ctx[k + 2], acc);
        acc = fmaf(w4[3], ctx[k + 3], acc);
      }
      s_p[o] = base[o] + (acc + bc[o]);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- pass 2: xp (MFMA) -> logits
  {
    const int g = lane >> 4, r16 = lane & 15;
    const float inv_scale = 0.25f;  // 1 / sqrt(head_dim 16)
    float bq[NTC][4], pq[NTC][E][4];  // this lane's 4 output channels of each tile: bias and prototype values
#pragma unroll
    for (int ct = 0; ct < NTC; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = ct * 16 + 4 * g + q;
        bq[ct][q] = bp[c];
#pragma unroll
        for (int e = 0; e < E; ++e) pq[ct][e][q] = s_p[e * D + c];
      }
    float lmax[E];
#pragma unroll
    for (int e = 0; e < E; ++e) lmax[e] = -INFINITY;
    const int ntt = (N + 15) / 16;
    for (int tt = wave; tt < ntt; tt += HGF_WAVES) {
      const int tok = tt * 16 + r16;
      const bool ok = tok < N;
      vec bf[KS];
#pragma unroll
      for (int m = 0; m < KS; ++m) bf[m] = vload_sel(xb + (int64_t)tok * x.cs + m * 4 * V + g * V, xb, ok);
      f32x4 acc[NTC];
#pragma unroll
      for (int ct = 0; ct < NTC; ++ct) {
        acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < KS; ++m) {
          const vec af = *reinterpret_cast<const vec*>(s_wp + (ct * 16 + r16) * D + m * 4 * V + g * V);
          acc[ct] = mfma_chunk<T>(af, bf[m], acc[ct]);
        }
      }
      float tot[E];
#pragma unroll
      for (int e = 0; e < E; ++e) tot[e] = 0.f;
#pragma unroll
      for (int ct = 0; ct < NTC; ++ct) {  // tile ct = head ct: its 16 channels are the 4 lanes g x 4 regs
        float hd[E];
#pragma unroll
        for (int e = 0; e < E; ++e) hd[e] = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float xv = round_to<T>(acc[ct][q] + bq[ct][q]);  // xp as the unfused conv stores it
#pragma unroll
          for (int e = 0; e < E; ++e) hd[e] = fmaf(xv, pq[ct][e][q], hd[e]);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          hd[e] += __shfl_xor(hd[e], 16);
          hd[e] += __shfl_xor(hd[e], 32);
          tot[e] += hd[e] * inv_scale;
        }
      }
      if (g == 0 && ok) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float l = tot[e] / float(H);
          s_l[tok * E + e] = l;
          lmax[e] = fmaxf(lmax[e], l);
        }
      }
    }
    // softmax over tokens: max, then sum exp(l - max)
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) lmax[e] = fmaxf(lmax[e], __shfl_xor(lmax[e], off));
    if (lane == 0)
#pragma unroll
      for (int e = 0; e < E; ++e) s_red[wave * E + e] = lmax[e];
    __syncthreads();
    if (tid < E) {
      float m = s_red[tid];
      for (int w = 1; w < HGF_WAVES; ++w) m = fmaxf(m, s_red[w * E + tid]);
      s_stat[0][tid] = m;
    }
    __syncthreads();
    float ps[E];
#pragma unroll
    for (int e = 0; e < E; ++e) ps[e] = 0.f;
    for (int n = tid; n < N; n += HGF_NT)
#pragma unroll
      for (int e = 0; e < E; ++e) ps[e] += expf(s_l[n * E + e] - s_stat[0][e]);
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) ps[e] += __shfl_xor(ps[e], off);
    __syncthreads();  // s_red's max partials consumed
    if (lane == 0)
#pragma unroll
      for (int e = 0; e < E; ++e) s_red[wave * E + e] = ps[e];
    __syncthreads();
    if (tid < E) {
      float sum = s_red[tid];
      for (int w = 1; w < HGF_WAVES; ++w) sum += s_red[w * E + tid];
      s_stat[1][tid] = 1.0f / sum;
    }
    __syncthreads();
    for (int i = tid; i < N * E; i += HGF_NT) {
      const int e = i % E;
      s_l[i] = expf(s_l[i] - s_stat[0][e]) * s_stat[1][e];
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- pass 3: He = A^T X, He2, He3
  {
    float acc[E][V];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int q = 0; q < V; ++q) acc[e][q] = 0.f;
#pragma unroll 2
    for (int n = tl; n < N; n += TL) {
      float v[V];
      load_f<V>(xb + (int64_t)n * x.cs + cv * V, v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float a = s_l[n * E + e];
#pragma unroll
        for (int q = 0; q < V; ++q) acc[e][q] = fmaf(a, v[q], acc[e][q]);
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int off = CV; off < 64; off <<= 1)
#pragma unroll
        for (int q = 0; q < V; ++q) acc[e][q] += __shfl_xor(acc[e][q], off);
    for (int e0 = 0; e0 < E; e0 += 4) {  // combine the 16 waves' partials, 4 hyperedges at a time
      if (lane < CV)
#pragma unroll
        for (int e = 0; e < 4 && e0 + e < E; ++e)
#pragma unroll
          for (int q = 0; q < V; ++q) s_red[wave * 4 * D + e * D + cv * V + q] = acc[e0 + e][q];
      __syncthreads();
      for (int i = tid; i < 4 * D && e0 + i / D < E; i += HGF_NT) {
        float v = s_red[i];
        for (int w = 1; w < HGF_WAVES; ++w) v += s_red[w * 4 * D + i];
        s_he[e0 * D + i] = v;
      }
      __syncthreads();
    }
    // He2 = GELU(He We^T + be), then He3 = He2 Wn^T: a wave per weight row d (coalesced row loads, lanes over k),
    // the E dot products reduced across the wave
    auto rows = [&](const float* __restrict__ in, const float* __restrict__ w, float* out, const float* bias) {
      for (int d = wave; d < D; d += HGF_WAVES) {
        float sv[E];
#pragma unroll
        for (int e = 0; e < E; ++e) sv[e] = 0.f;
#pragma unroll
        for (int k = lane; k < D; k += 64) {
          const float wv = w[(int64_t)d * D + k];
#pragma unroll
          for (int e = 0; e < E; ++e) sv[e] = fmaf(in[e * D + k], wv, sv[e]);
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) sv[e] += __shfl_xor(sv[e], off);
        if (lane < E) {
          float v = sv[0];
#pragma unroll
          for (int e = 1; e < E; ++e) v = lane == e ? sv[e] : v;
          out[lane * D + d] = bias ? gelu_erf(v + bias[d]) : v;
        }
      }
    };
    rows(s_he, we, s_h2, be);
    __syncthreads();
    rows(s_h2, wn, s_he, nullptr);  // He3 over He's slot (He is dead)
    __syncthreads();
  }

  // ---------------------------------------------------------------- pass 4: y = GELU(A He3 + bn) + X
  {
    float h3[E][V], bv[V];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int q = 0; q < V; ++q) h3[e][q] = s_he[e * D + cv * V + q];
    load_f<V>(bn + cv * V, bv);
    T* yb = y.p + (int64_t)b * N * y.cs;
#pragma unroll 2
    for (int n = tl; n < N; n += TL) {
      float v[V], o[V];
      load_f<V>(xb + (int64_t)n * x.cs + cv * V, v);
#pragma unroll
      for (int q = 0; q < V; ++q) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) s = fmaf(s_l[n * E + e], h3[e][q], s);
        o[q] = gelu_erf(s + bv[q]) + v[q];
      }
      store_f<V>(yb + (int64_t)n * y.cs + cv * V, o);
    }
  }
}

template <typename T, int D, int E>
static int hgf_go(const ydbl_hg_desc* d, hipStream_t s) {
  const int N = d->x.h * d->x.w;
  const int64_t lds = hgf_lds<T, D, E>(N);
  // Dynamic LDS up to the CU's 160 KiB launches without an opt-in on ROCm (measured: the 128-dim / 8-edge fp32
  // instantiation at N = 1600 takes 158 KiB); hipFuncSetAttribute(MaxDynamicSharedMemorySize) returns an error
  // there, which would otherwise surface in check_launch below, so it is not called.
  hg_fused_kernel<T, D, E><<<d->x.n, HGF_NT, (size_t)lds, s>>>(
      DView<const T>{reinterpret_cast<const T*>(d->x.ptr), d->x.n, d->x.h, d->x.w, d->x.c, d->x.cs}, dview<T>(d->y), N,
      d->num_heads, d->proto_base, d->ctx_w, d->ctx_b, reinterpret_cast<const T*>(d->pre_w), d->pre_b, d->edge_w,
      d->edge_b, d->node_w, d->node_b);
  return check_launch("ydbl_hg_fused");
}

template <typename F>
static int hgf_dispatch(int dim, int e, bool f16, F&& f) {
  auto pick = [&](auto T0) -> int {
    using T = decltype(T0);
    if (dim == 64 && e == 4) return f(T{}, std::integral_constant<int, 64>{}, std::integral_constant<int, 4>{});
    if (dim == 64 && e == 8) return f(T{}, std::integral_constant<int, 64>{}, std::integral_constant<int, 8>{});
    if (dim == 128 && e == 4) return f(T{}, std::integral_constant<int, 128>{}, std::integral_constant<int, 4>{});
    if (dim == 128 && e == 8) return f(T{}, std::integral_constant<int, 128>{}, std::integral_constant<int, 8>{});
    return -1;
  };
  return f16 ? pick(_Float16{}) : pick(float{});
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int64_t ydbl_hg_fused_lds(int32_t tokens, int32_t dim, int32_t edges, int32_t dtype) {
  if (tokens < 1) return -1;
  const int64_t r = hgf_dispatch(dim, edges, dtype == YDBL_F16, [&](auto T0, auto D0, auto E0) -> int {
    return (int)hgf_lds<decltype(T0), decltype(D0)::value, decltype(E0)::value>(tokens);
  });
  return r;
}

extern "C" int ydbl_hg_fused(const ydbl_hg_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "hg_fused: null descriptor");
  if (check_view(&d->x, "hg_fused.x", true) || check_view(&d->y, "hg_fused.y", true)) return YDBL_EINVAL;
  if (d->y.c != d->x.c || d->y.n != d->x.n || d->y.h * d->y.w != d->x.h * d->x.w || d->y.dtype != d->x.dtype)
    return fail(YDBL_EINVAL, "hg_fused: y shape mismatch");
  if (!d->proto_base || !d->ctx_w || !d->ctx_b || !d->pre_w || !d->pre_b || !d->edge_w || !d->edge_b || !d->node_w ||
      !d->node_b)
    return fail(YDBL_EINVAL, "hg_fused: null weights");
  if (d->num_heads < 1 || d->x.c != 16 * d->num_heads) return fail(YDBL_EINVAL, "hg_fused: head_dim must be 16");
  const int64_t lds = ydbl_hg_fused_lds(d->x.h * d->x.w, d->x.c, d->num_edges, d->x.dtype);
  if (lds < 0) return fail(YDBL_EINVAL, "hg_fused: (dim, edges) must be (64|128, 4|8)");
  if (lds > HGF_LDS_MAX) return fail(YDBL_EINVAL, "hg_fused: tokens x edges too large for LDS (use hg_context/propagate)");
  hipStream_t s = as_stream(stream);
  return hgf_dispatch(d->x.c, d->num_edges, d->x.dtype == YDBL_F16, [&](auto T0, auto D0, auto E0) -> int {
    return hgf_go<decltype(T0), decltype(D0)::value, decltype(E0)::value>(d, s);
  });
}
