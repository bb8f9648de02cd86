// Adaptive hypergraph convolution (AdaHyperedgeGen + AdaHGConv, U/nn/modules/block.py:1627-1708).
// Tokens are the NHWC pixels of one image (N = h*w, D = channels), so the reference's
// flatten(2).transpose(1,2) is free.  Stages (all fp32 arithmetic, f16/f32 token storage):
//   context : ctx = [mean_N X | max_N X];  proto = base + ctx @ Wc^T + bc              (per image)
//   [xp = X @ Wp^T + bp runs as a 1x1 conv through ydbl_conv2d_nhwc]
//   logits  : l[n,e] = mean_h (xp_h[n] . proto_h[e]) / sqrt(head_dim)
//   softmax : over tokens N, per (image, hyperedge)  -> (max_e, 1/sum_e)
//   edge    : He = A^T X;  He2 = GELU(He @ We^T + be);  He3 = He2 @ Wn^T
//   out     : y[n] = GELU(A[n] @ He3 + bn) + X[n]
// The last stage re-associates node_proj(A @ He2) = A @ (He2 @ Wn^T) + bn, so the D x D node
// projection runs on E rows per image instead of N (exact in real arithmetic).
#include "common.hpp"

#include <algorithm>

namespace ydbl {

// Token slices: image b's N tokens are split into NS slices so that B*NS workgroups fill the chip;
// every reduction over N writes per-slice partials that the next stage combines in fixed order.
static int hg_splits(int B, int N) {
  // ~256 workgroups: enough to fill the chip, few enough partials that every combine (proto,
  // edge) reads at most a few dozen of them per value
  int ns = (256 + B - 1) / B;
  const int max_ns = (N + 31) / 32;
  if (ns > max_ns) ns = max_ns;
  return ns < 1 ? 1 : ns;
}
constexpr int HG_LOGIT_TOK = 256;  // tokens per logits workgroup (one per thread)

struct HgWs {
  float* ctxp;    // [B][NS][2D]   partial (sum, max) over a token slice
  float* proto;   // [B][E][D]
  float* logits;  // [B][N][E]
  float* lstat;   // [B][NL][E][2] partial (max, sum exp) per logits workgroup
  float* stats;   // [B][E][2]     (max, 1/sum)
  float* hep;     // [B][NS][E][D] partial A^T X
  float* he3;     // [B][E][D]
  int ns, nl;
};

static HgWs carve(void* ws, int B, int N, int D, int E) {
  float* p = reinterpret_cast<float*>(ws);
  HgWs w;
  w.ns = hg_splits(B, N);
  w.nl = (N + HG_LOGIT_TOK - 1) / HG_LOGIT_TOK;
  w.ctxp = p; p += (int64_t)B * w.ns * 2 * D;
  w.proto = p; p += (int64_t)B * E * D;
  w.logits = p; p += (int64_t)B * N * E;
  w.lstat = p; p += (int64_t)B * w.nl * E * 2;
  w.stats = p; p += (int64_t)B * E * 2;
  w.hep = p; p += (int64_t)B * w.ns * E * D;
  w.he3 = p;
  return w;
}

static int64_t hg_ws_floats(int B, int N, int D, int E) {
  const int ns = hg_splits(B, N), nl = (N + HG_LOGIT_TOK - 1) / HG_LOGIT_TOK;
  return (int64_t)B * ns * 2 * D + (int64_t)B * E * D + (int64_t)B * N * E + (int64_t)B * nl * E * 2 +
         (int64_t)B * E * 2 + (int64_t)B * ns * E * D + (int64_t)B * E * D;
}

// partial context over one token slice: threads = (channel vector cv, token lane tl)
template <typename T>
__global__ __launch_bounds__(256) void hg_stats_kernel(DView<const T> x, float* __restrict__ ctxp, int ns) {
  constexpr int V = Vec<T>::N;
  __shared__ float ssum[256][V], smax[256][V];
  const int b = blockIdx.y, k = blockIdx.x;
  const int N = x.h * x.w, D = x.c;
  const int ncv = D / V;
  const int lanes = 256 / ncv;  // token lanes (D <= 2048)
  const int cv = threadIdx.x % ncv, tl = threadIdx.x / ncv;
  const int n0 = (int)((int64_t)N * k / ns), n1 = (int)((int64_t)N * (k + 1) / ns);
  float s[V], m[V];
#pragma unroll
  for (int q = 0; q < V; ++q) { s[q] = 0.f; m[q] = -INFINITY; }
  if (tl < lanes) {
    const T* base = x.p + (int64_t)b * N * x.cs + cv * V;
    for (int n = n0 + tl; n < n1; n += lanes) {
      float v[V];
      load_f<V>(base + (int64_t)n * x.cs, v);
#pragma unroll
      for (int q = 0; q < V; ++q) { s[q] += v[q]; m[q] = fmaxf(m[q], v[q]); }
    }
  }
#pragma unroll
  for (int q = 0; q < V; ++q) { ssum[threadIdx.x][q] = s[q]; smax[threadIdx.x][q] = m[q]; }
  __syncthreads();
  if (threadIdx.x < ncv) {
    for (int t = 1; t < lanes; ++t) {
#pragma unroll
      for (int q = 0; q < V; ++q) {
        s[q] += ssum[t * ncv + cv][q];
        m[q] = fmaxf(m[q], smax[t * ncv + cv][q]);
      }
    }
    float* o = ctxp + ((int64_t)b * ns + k) * 2 * D;
#pragma unroll
    for (int q = 0; q < V; ++q) { o[cv * V + q] = s[q]; o[D + cv * V + q] = m[q]; }
  }
}

// proto[b][e][d] = base + ctx @ Wc^T + bc; ctx = [sum/N | max] combined from the slice partials.
// one wave per output row o = e*D + d; lanes split the 2D inputs
__global__ __launch_bounds__(256) void hg_proto_kernel(const float* __restrict__ ctxp, int ns, int N,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       const float* __restrict__ base, float* __restrict__ proto,
                                                       int D, int E) {
  extern __shared__ float sctx[];  // [2D]
  const int b = blockIdx.x;
  const int K = 2 * D;
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    const float* c = ctxp + (int64_t)b * ns * K + i;
    float v = c[0];
    if (i < D) {
#pragma unroll 8
      for (int k = 1; k < ns; ++k) v += c[(int64_t)k * K];
      v /= float(N);
    } else {
#pragma unroll 8
      for (int k = 1; k < ns; ++k) v = fmaxf(v, c[(int64_t)k * K]);
    }
    sctx[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = blockIdx.y * 4 + wave; o < E * D; o += gridDim.y * 4) {
    const float* wr = w + (int64_t)o * K;
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s = fmaf(wr[k], sctx[k], s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) proto[(int64_t)b * E * D + o] = base[o] + (s + bias[o]);
  }
}

// logits[n][e] = mean_h (xp_h[n] . proto_h[e]) / sqrt(head_dim), plus per-workgroup softmax partials
template <typename T, int E>
__global__ __launch_bounds__(HG_LOGIT_TOK) void hg_logits_kernel(DView<const T> xp, const float* __restrict__ proto,
                                                                 float* __restrict__ logits, float* __restrict__ lstat,
                                                                 int H, float inv_scale) {
  extern __shared__ float sp[];  // [E][D]
  __shared__ float red[E][HG_LOGIT_TOK / 64];
  __shared__ float smx[E];
  const int b = blockIdx.y;
  const int D = xp.c, N = xp.h * xp.w;
  for (int i = threadIdx.x; i < E * D; i += blockDim.x) sp[i] = proto[(int64_t)b * E * D + i];
  __syncthreads();
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int V = Vec<T>::N;
  const int hd = D / H;
  float tot[E];
#pragma unroll
  for (int e = 0; e < E; ++e) tot[e] = -INFINITY;
  if (n < N) {
    const T* row = xp.p + ((int64_t)b * N + n) * xp.cs;
    float head[E];
#pragma unroll
    for (int e = 0; e < E; ++e) tot[e] = head[e] = 0.f;
#pragma unroll 4
    for (int d0 = 0; d0 < D; d0 += V) {
      float v[V];
      load_f<V>(row + d0, v);
#pragma unroll
      for (int q = 0; q < V; ++q) {
        const int d = d0 + q;
#pragma unroll
        for (int e = 0; e < E; ++e) head[e] = fmaf(v[q], sp[e * D + d], head[e]);
        if ((d + 1) % hd == 0) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            tot[e] += head[e] * inv_scale;
            head[e] = 0.f;
          }
        }
      }
    }
    float* lo = logits + ((int64_t)b * N + n) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      tot[e] = tot[e] / float(H);
      lo[e] = tot[e];
    }
  }
  // workgroup partial softmax stats: max, then sum exp(l - max)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float m = tot[e];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if (lane == 0) red[e][wave] = m;
  }
  __syncthreads();
  if (threadIdx.x < E) {
    float m = red[threadIdx.x][0];
    for (int w2 = 1; w2 < HG_LOGIT_TOK / 64; ++w2) m = fmaxf(m, red[threadIdx.x][w2]);
    smx[threadIdx.x] = m;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float v = n < N ? expf(tot[e] - smx[e]) : 0.f;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[e][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < E) {
    float sum = red[threadIdx.x][0];
    for (int w2 = 1; w2 < HG_LOGIT_TOK / 64; ++w2) sum += red[threadIdx.x][w2];
    float* o = lstat + (((int64_t)b * gridDim.x + blockIdx.x) * E + threadIdx.x) * 2;
    o[0] = smx[threadIdx.x];
    o[1] = sum;
  }
}

// partial He[b][k][e][d] = sum_{n in slice k} A[n][e] * X[n][d].  The softmax weights A[n][e] of a
// 64-token chunk are computed once into LDS (not once per channel-vector thread).
constexpr int HG_CHUNK = 64;
template <typename T, int E>
__global__ __launch_bounds__(256) void hg_gather_kernel(DView<const T> x, const float* __restrict__ logits,
                                                        const float* __restrict__ lstat, int nl,
                                                        float* __restrict__ hep, int ns) {
  constexpr int V = Vec<T>::N;
  __shared__ float s_mx[E], s_inv[E];
  __shared__ float s_a[HG_CHUNK][E];
  __shared__ float red[256][V];
  const int b = blockIdx.y, k = blockIdx.x;
  const int N = x.h * x.w, D = x.c;
  if (threadIdx.x < E) {
    const int e = threadIdx.x;
    float m = -INFINITY;
#pragma unroll 8
    for (int j = 0; j < nl; ++j) m = fmaxf(m, lstat[(((int64_t)b * nl + j) * E + e) * 2]);
    float sum = 0.f;
#pragma unroll 8
    for (int j = 0; j < nl; ++j) {
      const float* st = lstat + (((int64_t)b * nl + j) * E + e) * 2;
      sum += st[1] * expf(st[0] - m);
    }
    s_mx[e] = m;
    s_inv[e] = 1.0f / sum;
  }
  const int ncv = D / V;
  const int lanes = 256 / ncv;
  const int cv = threadIdx.x % ncv, tl = threadIdx.x / ncv;
  const int n0 = (int)((int64_t)N * k / ns), n1 = (int)((int64_t)N * (k + 1) / ns);
  float acc[E][V];
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int q = 0; q < V; ++q) acc[e][q] = 0.f;
  const T* xb = x.p + (int64_t)b * N * x.cs + cv * V;
  const float* l = logits + (int64_t)b * N * E;
  for (int c0 = n0; c0 < n1; c0 += HG_CHUNK) {
    const int cn = min(HG_CHUNK, n1 - c0);
    __syncthreads();  // s_mx/s_inv ready; previous chunk's s_a consumed
    for (int i = threadIdx.x; i < cn * E; i += 256) {
      const int t = i / E, e = i - t * E;
      s_a[t][e] = expf(l[(int64_t)(c0 + t) * E + e] - s_mx[e]) * s_inv[e];
    }
    __syncthreads();
    if (tl < lanes) {
      for (int t = tl; t < cn; t += lanes) {
        float xv[V];
        load_f<V>(xb + (int64_t)(c0 + t) * x.cs, xv);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float a = s_a[t][e];
#pragma unroll
          for (int q = 0; q < V; ++q) acc[e][q] = fmaf(a, xv[q], acc[e][q]);
        }
      }
    }
  }
  float* o = hep + ((int64_t)b * ns + k) * E * D;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < V; ++q) red[threadIdx.x][q] = acc[e][q];
    __syncthreads();
    if (threadIdx.x < ncv) {
      float v[V];
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = red[cv][q];
      for (int t = 1; t < lanes; ++t)
#pragma unroll
        for (int q = 0; q < V; ++q) v[q] += red[t * ncv + cv][q];
#pragma unroll
      for (int q = 0; q < V; ++q) o[e * D + cv * V + q] = v[q];
    }
  }
}

// He2 = GELU(He @ We^T + be); He3 = He2 @ Wn^T   (per image, E rows).  1024 threads per image:
// a wave owns output rows d, its lanes stride the coalesced weight row d[k] and the E dot
// products are reduced across the wave.
constexpr int HG_EDGE_THREADS = 1024;
template <int E>
__device__ __forceinline__ void hg_rows(const float* __restrict__ in, const float* __restrict__ w, int D,
                                        float* out, const float* __restrict__ bias, bool gelu, float* gout,
                                        int64_t gstride) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = HG_EDGE_THREADS / 64;
#pragma unroll 4  // weight-row loads of 4 rows in flight together
  for (int d = wave; d < D; d += NW) {
    const float* wr = w + (int64_t)d * D;
    float s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) s[e] = 0.f;
    for (int k = lane; k < D; k += 64) {
      const float wv = wr[k];
#pragma unroll
      for (int e = 0; e < E; ++e) s[e] = fmaf(in[e * D + k], wv, s[e]);
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s[e] += __shfl_xor(s[e], off, 64);
    if (lane < E) {
      float v = s[0];
#pragma unroll
      for (int e = 1; e < E; ++e) v = lane == e ? s[e] : v;
      if (gelu) v = gelu_erf(v + bias[d]);
      if (out) out[lane * D + d] = v;
      if (gout) gout[lane * gstride + d] = v;
    }
  }
}

template <int E>
__global__ __launch_bounds__(HG_EDGE_THREADS) void hg_edge_kernel(const float* __restrict__ hep, int ns,
                                                                  const float* __restrict__ lstat, int nl,
                                                                  float* __restrict__ stats, const float* __restrict__ we,
                                                                  const float* __restrict__ be,
                                                                  const float* __restrict__ wn,
                                                                  float* __restrict__ he3, int D) {
  extern __shared__ float sm[];  // he [E][D], he2 [E][D]
  float* sh = sm;
  float* sh2 = sm + E * D;
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < E * D; i += blockDim.x) {
    const float* p = hep + (int64_t)b * ns * E * D + i;
    float v = p[0];
#pragma unroll 8  // the partial loads are independent: keep 8 in flight (same summation order)
    for (int k = 1; k < ns; ++k) v += p[(int64_t)k * E * D];
    sh[i] = v;
  }
  if (threadIdx.x < E) {
    const int e = threadIdx.x;
    float m = -INFINITY;
#pragma unroll 8
    for (int j = 0; j < nl; ++j) m = fmaxf(m, lstat[(((int64_t)b * nl + j) * E + e) * 2]);
    float sum = 0.f;
#pragma unroll 8
    for (int j = 0; j < nl; ++j) {
      const float* st = lstat + (((int64_t)b * nl + j) * E + e) * 2;
      sum += st[1] * expf(st[0] - m);
    }
    stats[((int64_t)b * E + e) * 2] = m;
    stats[((int64_t)b * E + e) * 2 + 1] = 1.0f / sum;
  }
  __syncthreads();
  hg_rows<E>(sh, we, D, sh2, be, true, nullptr, 0);
  __syncthreads();
  hg_rows<E>(sh2, wn, D, nullptr, nullptr, false, he3 + (int64_t)b * E * D, D);
}

// y[n] = GELU(A[n] @ He3 + bn) + X[n].  A workgroup takes HG_CHUNK tokens of one image: He3[b] and
// the chunk's softmax weights are staged in LDS once, then threads sweep (token, channel vector).
template <typename T, int E>
__global__ __launch_bounds__(256) void hg_out_kernel(DView<const T> x, const float* __restrict__ logits,
                                                     const float* __restrict__ stats, const float* __restrict__ he3,
                                                     const float* __restrict__ bn, DView<T> y) {
  constexpr int V = Vec<T>::N;
  extern __shared__ float s_he[];  // [E][D]
  __shared__ float s_a[HG_CHUNK][E];
  const int D = x.c, N = x.h * x.w;
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * HG_CHUNK;
  const int cn = min(HG_CHUNK, N - c0);
  for (int i = threadIdx.x; i < E * D; i += 256) s_he[i] = he3[(int64_t)b * E * D + i];
  for (int i = threadIdx.x; i < cn * E; i += 256) {
    const int t = i / E, e = i - t * E;
    const float* st = stats + ((int64_t)b * E + e) * 2;
    s_a[t][e] = expf(logits[((int64_t)b * N + c0 + t) * E + e] - st[0]) * st[1];
  }
  __syncthreads();
  const int cg = D / V;
  for (int i = threadIdx.x; i < cn * cg; i += 256) {
    const int t = i / cg, d0 = (i - t * cg) * V;
    const int64_t tok = (int64_t)b * N + c0 + t;
    float xv[V], o[V];
    load_f<V>(x.pix(tok) + d0, xv);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) s = fmaf(s_a[t][e], s_he[e * D + d0 + q], s);
      o[q] = gelu_erf(s + bn[d0 + q]) + xv[q];
    }
    store_f<V>(y.pix(tok) + d0, o);
  }
}

template <typename T>
static DView<const T> cv(const ydbl_view& v) {
  return DView<const T>{reinterpret_cast<const T*>(v.ptr), v.n, v.h, v.w, v.c, v.cs};
}

template <typename T, int E>
static int hg_context_t(const ydbl_hg_desc* d, hipStream_t s) {
  const int B = d->x.n, N = d->x.h * d->x.w, D = d->x.c;
  HgWs w = carve(d->workspace, B, N, D, E);
  hg_stats_kernel<T><<<dim3(w.ns, B), 256, 0, s>>>(cv<T>(d->x), w.ctxp, w.ns);
  const int rows_blocks = (int)std::min<int64_t>(cdiv(E * D, 4), std::max<int64_t>(1, cdiv(1024, B)));
  hg_proto_kernel<<<dim3(B, rows_blocks), 256, 2 * D * sizeof(float), s>>>(w.ctxp, w.ns, N, d->ctx_w, d->ctx_b,
                                                                           d->proto_base, w.proto, D, E);
  return check_launch("ydbl_hg_context");
}

template <typename T, int E>
static int hg_propagate_t(const ydbl_hg_desc* d, hipStream_t s) {
  const int B = d->x.n, N = d->x.h * d->x.w, D = d->x.c, H = d->num_heads;
  HgWs w = carve(d->workspace, B, N, D, E);
  const float inv_scale = 1.0f / sqrtf(float(D / H));
  hg_logits_kernel<T, E><<<dim3(w.nl, B), HG_LOGIT_TOK, E * D * sizeof(float), s>>>(cv<T>(d->xp), w.proto, w.logits,
                                                                                     w.lstat, H, inv_scale);
  hg_gather_kernel<T, E><<<dim3(w.ns, B), 256, 0, s>>>(cv<T>(d->x), w.logits, w.lstat, w.nl, w.hep, w.ns);
  hg_edge_kernel<E><<<B, HG_EDGE_THREADS, 2 * E * D * sizeof(float), s>>>(
      w.hep, w.ns, w.lstat, w.nl, w.stats, d->edge_w, d->edge_b, d->node_w, w.he3, D);
  hg_out_kernel<T, E><<<dim3((unsigned)cdiv(N, HG_CHUNK), B), 256, E * D * sizeof(float), s>>>(
      cv<T>(d->x), w.logits, w.stats, w.he3, d->node_b, dview<T>(d->y));
  return check_launch("ydbl_hg_propagate");
}

static int hg_check(const ydbl_hg_desc* d, bool need_xp) {
  if (!d) return fail(YDBL_EINVAL, "hg: null descriptor");
  if (check_view(&d->x, "hg.x", true)) return YDBL_EINVAL;
  if (need_xp) {
    if (check_view(&d->xp, "hg.xp", true) || check_view(&d->y, "hg.y", true)) return YDBL_EINVAL;
    if (d->xp.c != d->x.c || d->y.c != d->x.c || d->xp.n != d->x.n || d->y.n != d->x.n ||
        d->xp.h * d->xp.w != d->x.h * d->x.w || d->y.h * d->y.w != d->x.h * d->x.w || d->xp.dtype != d->x.dtype ||
        d->y.dtype != d->x.dtype)
      return fail(YDBL_EINVAL, "hg: xp/y shape mismatch");
    if (d->num_heads < 1 || d->x.c % d->num_heads) return fail(YDBL_EINVAL, "hg: heads must divide dim");
    if (!d->edge_w || !d->edge_b || !d->node_w || !d->node_b) return fail(YDBL_EINVAL, "hg: null weights");
    if (2 * d->num_edges * d->x.c * 4 > 64 * 1024) return fail(YDBL_EINVAL, "hg: edges*dim too large");
  } else if (!d->proto_base || !d->ctx_w || !d->ctx_b) {
    return fail(YDBL_EINVAL, "hg: null context weights");
  }
  if (!d->workspace) return fail(YDBL_EINVAL, "hg: null workspace");
  if (d->num_edges != 4 && d->num_edges != 8 && d->num_edges != 12 && d->num_edges != 16)
    return fail(YDBL_EINVAL, "hg: num_edges must be 4, 8, 12 or 16");
  return YDBL_OK;
}

template <typename F>
static int by_edges(int e, F&& f) {
  switch (e) {
    case 4: return f(std::integral_constant<int, 4>{});
    case 8: return f(std::integral_constant<int, 8>{});
    case 12: return f(std::integral_constant<int, 12>{});
    default: return f(std::integral_constant<int, 16>{});
  }
}

}  // namespace ydbl

using namespace ydbl;

extern "C" int64_t ydbl_hg_workspace(int32_t n, int32_t tokens, int32_t dim, int32_t edges) {
  return 4 * hg_ws_floats(n, tokens, dim, edges);
}

extern "C" int ydbl_hg_context(const ydbl_hg_desc* d, void* stream) {
  if (int rc = hg_check(d, false)) return rc;
  hipStream_t s = as_stream(stream);
  return by_edges(d->num_edges, [&](auto E) {
    return d->x.dtype == YDBL_F16 ? hg_context_t<_Float16, decltype(E)::value>(d, s)
                                  : hg_context_t<float, decltype(E)::value>(d, s);
  });
}

extern "C" int ydbl_hg_propagate(const ydbl_hg_desc* d, void* stream) {
  if (int rc = hg_check(d, true)) return rc;
  hipStream_t s = as_stream(stream);
  return by_edges(d->num_edges, [&](auto E) {
    return d->x.dtype == YDBL_F16 ? hg_propagate_t<_Float16, decltype(E)::value>(d, s)
                                  : hg_propagate_t<float, decltype(E)::value>(d, s);
  });
}
