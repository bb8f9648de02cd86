// AdaHGConv (U/nn/modules/block.py:1582-1708: AdaHyperedgeGen + AdaHGConv, pre_head_proj included) in five
// plain launches spread over the chip (every DBL call: N = 1600 tokens at 640, D = 64 / 128, E = 4 / 8,
// head_dim 16).  The math has three reductions over all N tokens of an image (context stats, softmax over N,
// He = A^T X); the token-parallel launches split the tokens into slices of HG3_TS, one 256-thread workgroup
// per (slice, image), write per-slice partials to the workspace, and the next launch merges them (stream
// order is the only synchronisation: no counters, nothing to zero):
//   hg3_ctx   partial [sum | max] of X per slice;
//   hg3_proto merges the slices' [sum | max] into ctx, then proto = base + Wc ctx + bc (16 rows per workgroup:
//             the 2D x E*D weight is read by many CUs at once);
//   hg3_edge  xp = X Wp^T + bp (MFMA, rounded as the unfused conv stores it), logits = mean_h(xp_h . proto_h) / 4
//             (kept in the workspace), per-slice online-softmax partials (max m_s, sum of exp, He'_s =
//             sum exp(l - m_s) X);
//   hg3_merge per (image, hyperedge): m, 1/S, He = sum_s e^(m_s - m) He'_s / S, He2 = GELU(He We^T + be),
//             He3 = He2 Wn^T (node_proj re-associated);
//   hg3_out   y = GELU(A He3 + bn) + X, A = exp(l - m) / S.
// (One 1024-thread workgroup per image doing all of it -- the round-2 form -- kept 16 CUs busy for 58 us per
// call at bs16 while the rest of the chip waited.)  All arithmetic fp32; slices merge in slice order.
#include "conv_common.hpp"

namespace ydbl {

constexpr int HG3_TS = 64;  // tokens per slice (a 16-token MFMA tile per wave)
constexpr int HG3_ZB = 8;   // slab loads issued together by a merging thread
constexpr int HG3_NSMAX = 128;  // slices per image the merge handles (N <= 8192 tokens)

template <typename T, int D, int E>
struct Hg3 {
  static constexpr int V = Vec<T>::N;  // channels per 16-byte vector
  static constexpr int CV = D / V;     // vectors per token
  static constexpr int TL = 256 / CV;  // token lanes of a workgroup
  static constexpr int NTC = D / 16;   // 16-channel output tiles = heads (head_dim 16)
  static constexpr int KS = D / (4 * V);
  static constexpr int R2 = (2 * E + E * D + 3) / 4 * 4;  // floats of a slice's edge-stage partial
};

// workspace carve-up (bytes, 256-aligned sections)
struct Hg3Ws {
  int64_t slab1, ctx, proto, logits, slab2, he3, stat, total;
};
static Hg3Ws hg3_ws(int B, int N, int D, int E) {
  auto up = [](int64_t v) { return (v + 255) & ~255ll; };
  const int NS = (N + HG3_TS - 1) / HG3_TS, R2 = (2 * E + E * D + 3) / 4 * 4;
  Hg3Ws w;
  w.slab1 = 0;
  w.ctx = up(w.slab1 + (int64_t)B * NS * 2 * D * 4);
  w.proto = up(w.ctx + (int64_t)B * 2 * D * 4);
  w.logits = up(w.proto + (int64_t)B * E * D * 4);
  w.slab2 = up(w.logits + (int64_t)B * N * E * 4);
  w.he3 = up(w.slab2 + (int64_t)B * NS * R2 * 4);
  w.stat = up(w.he3 + (int64_t)B * E * D * 4);
  w.total = up(w.stat + (int64_t)B * 2 * E * 4);
  return w;
}

// ---- 1. context [mean_N X | max_N X] and the prototypes
template <typename T, int D, int E>
__global__ __launch_bounds__(256) void hg3_ctx_kernel(DView<const T> x, int N, unsigned char* __restrict__ ws, Hg3Ws o) {
  using C = Hg3<T, D, E>;
  constexpr int V = C::V, CV = C::CV, TL = C::TL;
  __shared__ float s_red[4 * 2 * D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sl = blockIdx.x, b = blockIdx.y, NS = gridDim.x;
  const int cv = tid % CV, tl = tid / CV;
  const T* xb = x.p + (int64_t)b * N * x.cs;
  const int n0 = sl * HG3_TS, n1 = min(N, n0 + HG3_TS);
  float sm[V], mx[V];
#pragma unroll
  for (int q = 0; q < V; ++q) sm[q] = 0.f, mx[q] = -INFINITY;
  for (int n = n0 + tl; n < n1; n += TL) {
    float v[V];
    load_f<V>(xb + (int64_t)n * x.cs + cv * V, v);
#pragma unroll
    for (int q = 0; q < V; ++q) sm[q] += v[q], mx[q] = fmaxf(mx[q], v[q]);
  }
#pragma unroll
  for (int off = CV; off < 64; off <<= 1)
#pragma unroll
    for (int q = 0; q < V; ++q) sm[q] += __shfl_xor(sm[q], off), mx[q] = fmaxf(mx[q], __shfl_xor(mx[q], off));
  if (lane < CV)
#pragma unroll
    for (int q = 0; q < V; ++q) s_red[wave * 2 * D + cv * V + q] = sm[q], s_red[wave * 2 * D + D + cv * V + q] = mx[q];
  __syncthreads();
  f32x4* slab = reinterpret_cast<f32x4*>(ws + o.slab1) + ((int64_t)b * NS + sl) * (2 * D / 4);
  if (tid < 2 * D / 4) {  // 4 channels of [sum | max] per thread, the 4 waves combined in order
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * tid + e;
      float a = s_red[c];
      for (int w = 1; w < 4; ++w) a = c < D ? a + s_red[w * 2 * D + c] : fmaxf(a, s_red[w * 2 * D + c]);
      v[e] = a;
    }
    slab[tid] = v;
  }
}

// ---- 1b. ctx = [mean | max] of the image's slice partials (slice order), then proto[e][d] = base + (Wc[e*D+d] .
// ctx + bc): 16 rows per workgroup, 4 per wave, every row's weights loaded in one round trip together with the
// partials (lane l holds k = l*KL .. +KL-1), reduced across the wave
template <int D, int E>
__global__ __launch_bounds__(256) void hg3_proto_kernel(int N, int NS, const unsigned char* __restrict__ ws, Hg3Ws o,
                                                        const float* __restrict__ base, const float* __restrict__ wc,
                                                        const float* __restrict__ bc, unsigned char* __restrict__ wsw) {
  constexpr int KL = 2 * D / 64;  // ctx entries per lane (2 or 4)
  constexpr int C4 = 2 * D / 4;   // f32x4 columns of a slice partial
  constexpr int ZG = 256 / C4;    // slice groups
  __shared__ f32x4 s_part[ZG][C4];
  __shared__ float s_ctx[2 * D];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, b = blockIdx.y;
  float wv[4][KL];
#pragma unroll
  for (int r = 0; r < 4; ++r) load_f<KL>(wc + (int64_t)(blockIdx.x * 16 + wave * 4 + r) * 2 * D + lane * KL, wv[r]);
  const f32x4* slab = reinterpret_cast<const f32x4*>(ws + o.slab1) + (int64_t)b * NS * C4;
  const int col = tid % C4, zg = tid / C4;
  const bool sum = 4 * col < D;
  f32x4 acc = sum ? f32x4{0.f, 0.f, 0.f, 0.f} : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int z0 = zg; z0 < NS; z0 += ZG * HG3_ZB) {
    f32x4 v[HG3_ZB];
#pragma unroll
    for (int u = 0; u < HG3_ZB; ++u) v[u] = slab[(int64_t)min(z0 + u * ZG, NS - 1) * C4 + col];
#pragma unroll
    for (int u = 0; u < HG3_ZB; ++u) {
      if (z0 + u * ZG >= NS) break;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = sum ? acc[e] + v[u][e] : fmaxf(acc[e], v[u][e]);
    }
  }
  s_part[zg][col] = acc;
  __syncthreads();
  if (tid < C4) {
    f32x4 a = s_part[0][tid];
    for (int g = 1; g < ZG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = sum ? a[e] + s_part[g][tid][e] : fmaxf(a[e], s_part[g][tid][e]);
#pragma unroll
    for (int e = 0; e < 4; ++e) s_ctx[4 * tid + e] = sum ? a[e] / float(N) : a[e];
  }
  __syncthreads();
  float cv[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) cv[k] = s_ctx[lane * KL + k];
  float* proto = reinterpret_cast<float*>(wsw + o.proto) + (int64_t)b * E * D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < KL; ++k) a = fmaf(wv[r][k], cv[k], a);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
    const int i = blockIdx.x * 16 + wave * 4 + r;
    if (lane == 0) proto[i] = base[i] + (a + bc[i]);
  }
}

// ---- 2. logits, online-softmax partials, He = A^T X, He2, He3
template <typename T, int D, int E>
__global__ __launch_bounds__(256) void hg3_edge_kernel(DView<const T> x, int N, int H, unsigned char* __restrict__ ws,
                                                       Hg3Ws o, const T* __restrict__ wp, const float* __restrict__ bp,
                                                       const float* __restrict__ we, const float* __restrict__ be,
                                                       const float* __restrict__ wn) {
  using C = Hg3<T, D, E>;
  constexpr int V = C::V, CV = C::CV, TL = C::TL, NTC = C::NTC, KS = C::KS, R2 = C::R2;
  using vec = typename Vec<T>::type;
  __shared__ T s_wp[D * D];            // pre_head_proj weight [D][D]
  __shared__ float s_l[HG3_TS * E];    // this slice's logits, then exp(l - m_s)
  __shared__ float s_red[E * D];       // He'_s
  __shared__ T s_xt[HG3_TS * D];       // the slice's tokens (B operand of the He' MFMA)
  __shared__ float s_p[E * D];         // the image's prototypes
  __shared__ float s_m[2][E];          // slice max, sum
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int sl = blockIdx.x, b = blockIdx.y, NS = gridDim.x;
  const T* xb = x.p + (int64_t)b * N * x.cs;
  const int n0 = sl * HG3_TS, ntok = min(N - n0, HG3_TS);
  // every global load of the workgroup is issued before the first barrier: the weight tile, this wave's MFMA
  // operands, this thread's He' token vectors, the prototypes
  for (int i = tid; i < D * D / V; i += 256) reinterpret_cast<vec*>(s_wp)[i] = reinterpret_cast<const vec*>(wp)[i];
  const int tok = wave * 16 + r16;  // HG3_TS = 4 waves x 16 tokens
  const bool tok_ok = tok < ntok;
  vec bf[KS];
#pragma unroll
  for (int m = 0; m < KS; ++m) bf[m] = vload_sel(xb + (int64_t)(n0 + tok) * x.cs + m * 4 * V + g * V, xb, tok_ok);
  constexpr int XT = HG3_TS / TL;  // He' tokens per thread
  const int hcv = tid % CV, htl = tid / CV;
  vec xh[XT];
#pragma unroll
  for (int u = 0; u < XT; ++u) {
    const int t = htl + u * TL;
    xh[u] = vload_sel(xb + (int64_t)(n0 + t) * x.cs + hcv * V, xb, t < ntok);
  }
  const float* proto = reinterpret_cast<const float*>(ws + o.proto) + (int64_t)b * E * D;
#pragma unroll
  for (int u = 0; u < XT; ++u) *reinterpret_cast<vec*>(&s_xt[(htl + u * TL) * D + hcv * V]) = xh[u];
  for (int i = tid; i < E * D / 4; i += 256) reinterpret_cast<f32x4*>(s_p)[i] = reinterpret_cast<const f32x4*>(proto)[i];
  float bq[NTC][4];
#pragma unroll
  for (int ct = 0; ct < NTC; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[ct][q] = bp[ct * 16 + 4 * g + q];
  __syncthreads();

  // xp tile of wave `wave` (16 tokens) -> logits
  {
    const bool ok = tok_ok;
    float tot[E];
#pragma unroll
    for (int e = 0; e < E; ++e) tot[e] = 0.f;
#pragma unroll
    for (int ct = 0; ct < NTC; ++ct) {  // tile ct = head ct: its 16 channels are the 4 lanes g x 4 regs
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < KS; ++m) {
        const vec af = *reinterpret_cast<const vec*>(s_wp + (ct * 16 + r16) * D + m * 4 * V + g * V);
        acc = mfma_chunk<T>(af, bf[m], acc);
      }
      float hd[E];
#pragma unroll
      for (int e = 0; e < E; ++e) hd[e] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float xv = round_to<T>(acc[q] + bq[ct][q]);  // xp as the unfused conv stores it
#pragma unroll
        for (int e = 0; e < E; ++e) hd[e] = fmaf(xv, s_p[e * D + ct * 16 + 4 * g + q], hd[e]);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        hd[e] += __shfl_xor(hd[e], 16);
        hd[e] += __shfl_xor(hd[e], 32);
        tot[e] += hd[e] * 0.25f;  // 1 / sqrt(head_dim 16)
      }
    }
    float* lg = reinterpret_cast<float*>(ws + o.logits) + ((int64_t)b * N + n0) * E;
    if (g == 0 && ok) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float l = tot[e] / float(H);
        s_l[tok * E + e] = l;
        lg[tok * E + e] = l;
      }
    }
  }
  __syncthreads();
  // slice max and sum of exp per hyperedge: a wave per hyperedge, a lane per token (HG3_TS = 64), butterflies
  for (int e = wave; e < E; e += 4) {
    const float l = lane < ntok ? s_l[lane * E + e] : -INFINITY;
    float m = l;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    const float pe = lane < ntok ? expf(l - m) : 0.f;
    if (lane < ntok) s_l[lane * E + e] = pe;
    float sum = pe;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    if (lane == 0) s_m[0][e] = m, s_m[1][e] = sum;
  }
  __syncthreads();
  // He'_s[e][d] = sum_t exp(l_t - m_s) X_t[d] on the exact-f32 MFMA (16x16x4: the sequential fmaf chain over
  // tokens, bitwise): A[e][t] = the slice's probabilities (rows e >= E zero), B[t][d] = X from the LDS tile; a
  // wave per 16-channel column tile
  {
    constexpr int NCT = D / 16;  // column tiles
    for (int ct = wave; ct < NCT; ct += 4) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int t0 = 0; t0 < HG3_TS; t0 += 4) {
        const int t = t0 + g;
        const float av = (r16 < E && t < ntok) ? s_l[t * E + r16] : 0.f;
        const float bv = t < ntok ? float(s_xt[t * D + ct * 16 + r16]) : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * g + q < E) s_red[(4 * g + q) * D + ct * 16 + r16] = acc[q];
    }
  }
  __syncthreads();
  f32x4* rec = reinterpret_cast<f32x4*>(ws + o.slab2) + ((int64_t)b * NS + sl) * (R2 / 4);
  for (int i = tid; i < R2 / 4; i += 256) {  // record: [m_s (E) | S_s (E) | He'_s (E*D)]
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = 4 * i + e;
      float a = 0.f;
      if (f < E) a = s_m[0][f];
      else if (f < 2 * E) a = s_m[1][f - E];
      else if (f < 2 * E + E * D) {
        a = s_red[f - 2 * E];
      }
      v[e] = a;
    }
    rec[i] = v;
  }
}

// ---- 2b. per (image, hyperedge e): merge the slices (slice order) into He[e], then He2[e] = GELU(We He[e] + be),
// He3[e] = Wn He2[e] (row e of each product depends on row e only).  Every load is issued before the first use:
// a thread's two weight rows (output d = tid % D), the slices' (max, sum) of e, this thread's He' entries.
template <int D, int E>
__global__ __launch_bounds__(256) void hg3_merge_kernel(int NS, unsigned char* __restrict__ ws, Hg3Ws o,
                                                        const float* __restrict__ we, const float* __restrict__ be,
                                                        const float* __restrict__ wn) {
  constexpr int R2 = (2 * E + E * D + 3) / 4 * 4;
  constexpr int ZG = 256 / D;  // slice groups of the He' merge (4 at D 64, 2 at D 128)
  constexpr int ZB = (HG3_NSMAX + ZG - 1) / ZG;
  __shared__ float s_ms[2][HG3_NSMAX];
  __shared__ float s_part[ZG][D];
  __shared__ float s_v[2][D];
  __shared__ float s_st[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e = blockIdx.x, b = blockIdx.y;
  const int d = tid % D, zg = tid / D;
  const float* recs = reinterpret_cast<const float*>(ws + o.slab2) + (int64_t)b * NS * R2;
  f32x4 w1[D / 4 / ZG], w2[D / 4 / ZG];  // this thread's quarter/half of weight rows d (k split over the ZG groups)
#pragma unroll
  for (int i = 0; i < D / 4 / ZG; ++i) {
    w1[i] = reinterpret_cast<const f32x4*>(we + (int64_t)d * D)[zg * (D / 4 / ZG) + i];
    w2[i] = reinterpret_cast<const f32x4*>(wn + (int64_t)d * D)[zg * (D / 4 / ZG) + i];
  }
  for (int z = tid; z < NS; z += 256) s_ms[0][z] = recs[(int64_t)z * R2 + e], s_ms[1][z] = recs[(int64_t)z * R2 + E + e];
  float hv[ZB];
#pragma unroll
  for (int u = 0; u < ZB; ++u) {
    const int z = min(zg + u * ZG, NS - 1);
    hv[u] = recs[(int64_t)z * R2 + 2 * E + e * D + d];
  }
  __syncthreads();
  if (wave == 0) {  // m, 1/S over the slices: lanes over slices, butterflies
    float m = -INFINITY;
    for (int z = lane; z < NS; z += 64) m = fmaxf(m, s_ms[0][z]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    float S = 0.f;
    for (int z = lane; z < NS; z += 64) S += s_ms[1][z] * expf(s_ms[0][z] - m);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) S += __shfl_xor(S, off);
    if (lane == 0) s_st[0] = m, s_st[1] = 1.0f / S;
  }
  __syncthreads();
  {
    float a = 0.f;
#pragma unroll
    for (int u = 0; u < ZB; ++u) {
      const int z = zg + u * ZG;
      if (z < NS) a = fmaf(hv[u], expf(s_ms[0][z] - s_st[0]), a);
    }
    s_part[zg][d] = a;
  }
  __syncthreads();
  if (tid < D) {
    float a = s_part[0][tid];
    for (int g = 1; g < ZG; ++g) a += s_part[g][tid];
    s_v[0][tid] = a * s_st[1];  // He[e]
  }
  __syncthreads();
  // the two GEMVs: thread (d, zg) dots its k range, the ZG partials summed in group order
  auto gemv = [&](const f32x4 (&w)[D / 4 / ZG], const float* in) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < D / 4 / ZG; ++i) {
      const int k = (zg * (D / 4 / ZG) + i) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) a = fmaf(w[i][q], in[k + q], a);
    }
    s_part[zg][d] = a;
    __syncthreads();
    float r = 0.f;
    if (tid < D) {
      r = s_part[0][tid];
      for (int g = 1; g < ZG; ++g) r += s_part[g][tid];
    }
    __syncthreads();
    return r;
  };
  const float h2 = gemv(w1, s_v[0]);
  if (tid < D) s_v[1][tid] = gelu_erf(h2 + be[tid]);
  __syncthreads();
  const float h3 = gemv(w2, s_v[1]);
  if (tid < D) reinterpret_cast<float*>(ws + o.he3)[((int64_t)b * E + e) * D + tid] = h3;
  float* st = reinterpret_cast<float*>(ws + o.stat) + (int64_t)b * 2 * E;
  if (tid == 0) st[e] = s_st[0], st[E + e] = s_st[1];
}

// ---- 3. y = GELU(A He3 + bn) + X, A = exp(l - m) / S
template <typename T, int D, int E>
__global__ __launch_bounds__(256) void hg3_out_kernel(DView<const T> x, DView<T> y, int N,
                                                      const unsigned char* __restrict__ ws, Hg3Ws o,
                                                      const float* __restrict__ bn) {
  using C = Hg3<T, D, E>;
  constexpr int V = C::V, CV = C::CV, TL = C::TL;
  const int tid = threadIdx.x, cv = tid % CV, tl = tid / CV;
  const int b = blockIdx.y, n0 = blockIdx.x * HG3_TS, n1 = min(N, n0 + HG3_TS);
  const float* he3 = reinterpret_cast<const float*>(ws + o.he3) + (int64_t)b * E * D;
  const float* st = reinterpret_cast<const float*>(ws + o.stat) + (int64_t)b * 2 * E;
  const float* lg = reinterpret_cast<const float*>(ws + o.logits) + (int64_t)b * N * E;
  float h3[E][V], bv[V], m[E], inv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    load_f<V>(he3 + e * D + cv * V, h3[e]);
    m[e] = st[e];
    inv[e] = st[E + e];
  }
  load_f<V>(bn + cv * V, bv);
  const T* xb = x.p + (int64_t)b * N * x.cs;
  T* yb = y.p + (int64_t)b * N * y.cs;
  for (int n = n0 + tl; n < n1; n += TL) {
    float v[V], ov[V], a[E];
    load_f<V>(xb + (int64_t)n * x.cs + cv * V, v);
#pragma unroll
    for (int e = 0; e < E; ++e) a[e] = expf(lg[(int64_t)n * E + e] - m[e]) * inv[e];
#pragma unroll
    for (int q = 0; q < V; ++q) {
      float sacc = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) sacc = fmaf(a[e], h3[e][q], sacc);
      ov[q] = gelu_erf(sacc + bv[q]) + v[q];
    }
    store_f<V>(yb + (int64_t)n * y.cs + cv * V, ov);
  }
}

template <typename T, int D, int E>
static int hgf_go(const ydbl_hg_desc* d, hipStream_t s) {
  const int N = d->x.h * d->x.w, B = d->x.n;
  const int NS = (N + HG3_TS - 1) / HG3_TS;
  const Hg3Ws o = hg3_ws(B, N, D, E);
  unsigned char* ws = reinterpret_cast<unsigned char*>(d->workspace);
  const DView<const T> xv{reinterpret_cast<const T*>(d->x.ptr), d->x.n, d->x.h, d->x.w, d->x.c, d->x.cs};
  hg3_ctx_kernel<T, D, E><<<dim3(NS, B), 256, 0, s>>>(xv, N, ws, o);
  hg3_proto_kernel<D, E><<<dim3(E * D / 16, B), 256, 0, s>>>(N, NS, ws, o, d->proto_base, d->ctx_w, d->ctx_b, ws);
  hg3_edge_kernel<T, D, E><<<dim3(NS, B), 256, 0, s>>>(xv, N, d->num_heads, ws, o, reinterpret_cast<const T*>(d->pre_w),
                                                       d->pre_b, d->edge_w, d->edge_b, d->node_w);
  hg3_merge_kernel<D, E><<<dim3(E, B), 256, 0, s>>>(NS, ws, o, d->edge_w, d->edge_b, d->node_w);
  hg3_out_kernel<T, D, E><<<dim3(NS, B), 256, 0, s>>>(xv, dview<T>(d->y), N, ws, o, d->node_b);
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

extern "C" int64_t ydbl_hg_fused_workspace(int32_t n, int32_t tokens, int32_t dim, int32_t edges, int32_t dtype) {
  if (n < 1 || tokens < 1) return -1;
  const int64_t ok = hgf_dispatch(dim, edges, dtype == YDBL_F16, [&](auto, auto, auto) -> int { return 1; });
  if (ok < 0) return -1;
  if ((tokens + HG3_TS - 1) / HG3_TS > HG3_NSMAX) return -1;  // the merge's LDS holds <= HG3_NSMAX slices
  return hg3_ws(n, tokens, dim, edges).total;
}

extern "C" int ydbl_hg_fused(const ydbl_hg_desc* d, void* stream) {
  if (!d) return fail(YDBL_EINVAL, "hg_fused: null descriptor");
  if (check_view(&d->x, "hg_fused.x", true) || check_view(&d->y, "hg_fused.y", true)) return YDBL_EINVAL;
  if (d->y.c != d->x.c || d->y.n != d->x.n || d->y.h * d->y.w != d->x.h * d->x.w || d->y.dtype != d->x.dtype)
    return fail(YDBL_EINVAL, "hg_fused: y shape mismatch");
  if (!d->proto_base || !d->ctx_w || !d->ctx_b || !d->pre_w || !d->pre_b || !d->edge_w || !d->edge_b || !d->node_w ||
      !d->node_b)
    return fail(YDBL_EINVAL, "hg_fused: null weights");
  if (!d->workspace) return fail(YDBL_EINVAL, "hg_fused: null workspace (ydbl_hg_fused_workspace bytes, zeroed once)");
  if (d->num_heads < 1 || d->x.c != 16 * d->num_heads) return fail(YDBL_EINVAL, "hg_fused: head_dim must be 16");
  if (ydbl_hg_fused_workspace(d->x.n, d->x.h * d->x.w, d->x.c, d->num_edges, d->x.dtype) < 0)
    return fail(YDBL_EINVAL, "hg_fused: (dim, edges) must be (64|128, 4|8)");
  hipStream_t s = as_stream(stream);
  return hgf_dispatch(d->x.c, d->num_edges, d->x.dtype == YDBL_F16, [&](auto T0, auto D0, auto E0) -> int {
    return hgf_go<decltype(T0), decltype(D0)::value, decltype(E0)::value>(d, s);
  });
}
