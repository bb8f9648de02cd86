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

namespace ydbl {

struct HgWs {
  float* ctx;     // [B][2D]
  float* proto;   // [B][E][D]
  float* logits;  // [B][N][E]
  float* stats;   // [B][E][2]  (max, 1/sum)
  float* he;      // [B][E][D]
  float* he3;     // [B][E][D]
};

static HgWs carve(void* ws, int B, int N, int D, int E) {
  float* p = reinterpret_cast<float*>(ws);
  HgWs w;
  w.ctx = p; p += (int64_t)B * 2 * D;
  w.proto = p; p += (int64_t)B * E * D;
  w.logits = p; p += (int64_t)B * N * E;
  w.stats = p; p += (int64_t)B * E * 2;
  w.he = p; p += (int64_t)B * E * D;
  w.he3 = p;
  return w;
}

template <typename T>
__global__ __launch_bounds__(256) void hg_stats_kernel(DView<const T> x, float* __restrict__ ctx) {
  __shared__ float ssum[4][64], smax[4][64];
  const int b = blockIdx.x;
  const int tx = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int d = blockIdx.y * 64 + tx;
  const int N = x.h * x.w, D = x.c;
  float s = 0.f, m = -INFINITY;
  if (d < D) {
    const T* base = x.p + (int64_t)b * N * x.cs + d;
    for (int n = part; n < N; n += 4) {
      const float v = float(base[(int64_t)n * x.cs]);
      s += v;
      m = fmaxf(m, v);
    }
  }
  ssum[part][tx] = s;
  smax[part][tx] = m;
  __syncthreads();
  if (part == 0 && d < D) {
    const float st = (ssum[0][tx] + ssum[1][tx]) + (ssum[2][tx] + ssum[3][tx]);
    const float mt = fmaxf(fmaxf(smax[0][tx], smax[1][tx]), fmaxf(smax[2][tx], smax[3][tx]));
    ctx[(int64_t)b * 2 * D + d] = st / float(N);
    ctx[(int64_t)b * 2 * D + D + d] = mt;
  }
}

// one wave per output row o = e*D + d of the context Linear; lanes split the 2D inputs
__global__ __launch_bounds__(256) void hg_proto_kernel(const float* __restrict__ ctx, const float* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ base,
                                                       float* __restrict__ proto, int D, int E) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int o = blockIdx.y * 4 + wave;
  if (o >= E * D) return;
  const int K = 2 * D;
  const float* c = ctx + (int64_t)b * K;
  const float* wr = w + (int64_t)o * K;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s = fmaf(wr[k], c[k], s);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) proto[(int64_t)b * E * D + o] = base[o] + (s + bias[o]);
}

template <typename T, int E>
__global__ __launch_bounds__(256) void hg_logits_kernel(DView<const T> xp, const float* __restrict__ proto,
                                                        float* __restrict__ logits, int H, float inv_scale) {
  extern __shared__ float sp[];  // [E][D]
  const int b = blockIdx.y;
  const int D = xp.c, N = xp.h * xp.w;
  for (int i = threadIdx.x; i < E * D; i += blockDim.x) sp[i] = proto[(int64_t)b * E * D + i];
  __syncthreads();
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  constexpr int V = Vec<T>::N;
  const int hd = D / H;
  const T* row = xp.p + ((int64_t)b * N + n) * xp.cs;
  float tot[E], head[E];
#pragma unroll
  for (int e = 0; e < E; ++e) tot[e] = head[e] = 0.f;
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
  for (int e = 0; e < E; ++e) lo[e] = tot[e] / float(H);
}

template <int E>
__global__ __launch_bounds__(256) void hg_softmax_kernel(const float* __restrict__ logits, float* __restrict__ stats,
                                                         int N) {
  __shared__ float red[E][256];
  const int b = blockIdx.x;
  const float* l = logits + (int64_t)b * N * E;
  float m[E];
#pragma unroll
  for (int e = 0; e < E; ++e) m[e] = -INFINITY;
  for (int n = threadIdx.x; n < N; n += 256)
#pragma unroll
    for (int e = 0; e < E; ++e) m[e] = fmaxf(m[e], l[(int64_t)n * E + e]);
#pragma unroll
  for (int e = 0; e < E; ++e) red[e][threadIdx.x] = m[e];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int e = 0; e < E; ++e) red[e][threadIdx.x] = fmaxf(red[e][threadIdx.x], red[e][threadIdx.x + s]);
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < E; ++e) m[e] = red[e][0];
  __syncthreads();
  float sum[E];
#pragma unroll
  for (int e = 0; e < E; ++e) sum[e] = 0.f;
  for (int n = threadIdx.x; n < N; n += 256)
#pragma unroll
    for (int e = 0; e < E; ++e) sum[e] += expf(l[(int64_t)n * E + e] - m[e]);
#pragma unroll
  for (int e = 0; e < E; ++e) red[e][threadIdx.x] = sum[e];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int e = 0; e < E; ++e) red[e][threadIdx.x] += red[e][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < E) {
    stats[((int64_t)b * E + threadIdx.x) * 2 + 0] = m[threadIdx.x];
    stats[((int64_t)b * E + threadIdx.x) * 2 + 1] = 1.0f / red[threadIdx.x][0];
  }
}

// He[b][e][d] = sum_n A[n][e] * X[n][d]
template <typename T, int E>
__global__ __launch_bounds__(256) void hg_gather_kernel(DView<const T> x, const float* __restrict__ logits,
                                                        const float* __restrict__ stats, float* __restrict__ he) {
  __shared__ float red[4][E][64];
  const int b = blockIdx.x;
  const int tx = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int d = blockIdx.y * 64 + tx;
  const int N = x.h * x.w, D = x.c;
  float mx[E], inv[E], acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    mx[e] = stats[((int64_t)b * E + e) * 2];
    inv[e] = stats[((int64_t)b * E + e) * 2 + 1];
    acc[e] = 0.f;
  }
  const float* l = logits + (int64_t)b * N * E;
  const T* xb = x.p + (int64_t)b * N * x.cs;
  if (d < D) {
    for (int n = part; n < N; n += 4) {
      const float xv = float(xb[(int64_t)n * x.cs + d]);
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = fmaf(expf(l[(int64_t)n * E + e] - mx[e]) * inv[e], xv, acc[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) red[part][e][tx] = acc[e];
  __syncthreads();
  if (part == 0 && d < D) {
#pragma unroll
    for (int e = 0; e < E; ++e)
      he[((int64_t)b * E + e) * D + d] = (red[0][e][tx] + red[1][e][tx]) + (red[2][e][tx] + red[3][e][tx]);
  }
}

// He2 = GELU(He @ We^T + be); He3 = He2 @ Wn^T   (per image, E rows)
template <int E>
__global__ __launch_bounds__(256) void hg_edge_kernel(const float* __restrict__ he, const float* __restrict__ we,
                                                      const float* __restrict__ be, const float* __restrict__ wn,
                                                      float* __restrict__ he3, int D) {
  extern __shared__ float sm[];  // he [E][D], he2 [E][D]
  float* sh = sm;
  float* sh2 = sm + E * D;
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < E * D; i += blockDim.x) sh[i] = he[(int64_t)b * E * D + i];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float* wr = we + (int64_t)d * D;
    float s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) s[e] = 0.f;
    for (int k = 0; k < D; ++k) {
      const float wv = wr[k];
#pragma unroll
      for (int e = 0; e < E; ++e) s[e] = fmaf(sh[e * D + k], wv, s[e]);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) sh2[e * D + d] = gelu_erf(s[e] + be[d]);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float* wr = wn + (int64_t)d * D;
    float s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) s[e] = 0.f;
    for (int k = 0; k < D; ++k) {
      const float wv = wr[k];
#pragma unroll
      for (int e = 0; e < E; ++e) s[e] = fmaf(sh2[e * D + k], wv, s[e]);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) he3[((int64_t)b * E + e) * D + d] = s[e];
  }
}

template <typename T, int E>
__global__ __launch_bounds__(256) void hg_out_kernel(DView<const T> x, const float* __restrict__ logits,
                                                     const float* __restrict__ stats, const float* __restrict__ he3,
                                                     const float* __restrict__ bn, DView<T> y) {
  constexpr int V = Vec<T>::N;
  const int D = x.c, N = x.h * x.w;
  const int cg = D / V;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)x.n * N * cg) return;
  const int d0 = (int)(idx % cg) * V;
  const int64_t tok = idx / cg;
  const int b = (int)(tok / N);
  float a[E];
  const float* l = logits + tok * E;
#pragma unroll
  for (int e = 0; e < E; ++e)
    a[e] = expf(l[e] - stats[((int64_t)b * E + e) * 2]) * stats[((int64_t)b * E + e) * 2 + 1];
  float xv[V], o[V];
  load_f<V>(x.pix(tok) + d0, xv);
#pragma unroll
  for (int q = 0; q < V; ++q) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) s = fmaf(a[e], he3[((int64_t)b * E + e) * D + d0 + q], s);
    o[q] = gelu_erf(s + bn[d0 + q]) + xv[q];
  }
  store_f<V>(y.pix(tok) + d0, o);
}

template <typename T>
static DView<const T> cv(const ydbl_view& v) {
  return DView<const T>{reinterpret_cast<const T*>(v.ptr), v.n, v.h, v.w, v.c, v.cs};
}

template <typename T, int E>
static int hg_context_t(const ydbl_hg_desc* d, hipStream_t s) {
  const int B = d->x.n, N = d->x.h * d->x.w, D = d->x.c;
  HgWs w = carve(d->workspace, B, N, D, E);
  hg_stats_kernel<T><<<dim3(B, (unsigned)cdiv(D, 64)), 256, 0, s>>>(cv<T>(d->x), w.ctx);
  hg_proto_kernel<<<dim3(B, (unsigned)cdiv(E * D, 4)), 256, 0, s>>>(w.ctx, d->ctx_w, d->ctx_b, d->proto_base, w.proto,
                                                                     D, E);
  return check_launch("ydbl_hg_context");
}

template <typename T, int E>
static int hg_propagate_t(const ydbl_hg_desc* d, hipStream_t s) {
  const int B = d->x.n, N = d->x.h * d->x.w, D = d->x.c, H = d->num_heads;
  HgWs w = carve(d->workspace, B, N, D, E);
  const float inv_scale = 1.0f / sqrtf(float(D / H));
  hg_logits_kernel<T, E><<<dim3((unsigned)cdiv(N, 256), B), 256, E * D * sizeof(float), s>>>(cv<T>(d->xp), w.proto,
                                                                                               w.logits, H, inv_scale);
  hg_softmax_kernel<E><<<B, 256, 0, s>>>(w.logits, w.stats, N);
  hg_gather_kernel<T, E><<<dim3(B, (unsigned)cdiv(D, 64)), 256, 0, s>>>(cv<T>(d->x), w.logits, w.stats, w.he);
  hg_edge_kernel<E><<<B, 256, 2 * E * D * sizeof(float), s>>>(w.he, d->edge_w, d->edge_b, d->node_w, w.he3, D);
  const int V = Vec<T>::N;
  hg_out_kernel<T, E><<<(unsigned)cdiv((int64_t)B * N * (D / V), 256), 256, 0, s>>>(
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
  return 4 * ((int64_t)n * 2 * dim + 3LL * n * edges * dim + (int64_t)n * tokens * edges + 2LL * n * edges);
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
