// Shared device/host helpers for libydbl (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

#include "../../include/ydbl.h"

namespace ydbl {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using h8 = __attribute__((ext_vector_type(8))) _Float16;
using h4 = __attribute__((ext_vector_type(4))) _Float16;

// ---- error plumbing (thread-local message, int status) -----------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

// ---- 16-byte vector of T (8 x f16 or 4 x f32) ---------------------------------------------
template <typename T> struct Vec;
template <> struct Vec<_Float16> {
  static constexpr int N = 8;
  using type = h8;
};
template <> struct Vec<float> {
  static constexpr int N = 4;
  using type = f32x4;
};

template <typename T>
__device__ __forceinline__ typename Vec<T>::type vload(const T* p) {
  return *reinterpret_cast<const typename Vec<T>::type*>(p);
}
template <typename T>
__device__ __forceinline__ void vstore(T* p, const typename Vec<T>::type& v) {
  *reinterpret_cast<typename Vec<T>::type*>(p) = v;
}
template <typename T>
__device__ __forceinline__ typename Vec<T>::type vzero() {
  typename Vec<T>::type v;
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) v[i] = T(0);
  return v;
}

// ---- 8-byte half vector of T (4 x f16 or 2 x f32): the depthwise phases' channel group --------
using f32x2 = __attribute__((ext_vector_type(2))) float;
template <typename T> struct HVec;
template <> struct HVec<_Float16> {
  static constexpr int N = 4;
  using type = h4;
};
template <> struct HVec<float> {
  static constexpr int N = 2;
  using type = f32x2;
};

// XCD-aware block order.  Workgroups are dealt round-robin over the 8 XCDs (block b runs on XCD
// b % 8), each with its own L2; remapping so that XCD x walks a contiguous logical range keeps
// neighbouring tiles (shared halo rows, shared input tile of several output-channel splits) in one
// L2.  Any n: XCD x receives the blocks x, x+8, ... (q + (x < r) of them for n = 8q + r) and takes
// the logical range starting at x*q + min(x, r).
__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int x = b & 7, q = n >> 3, r = n & 7;
  return x * q + min(x, r) + (b >> 3);
}

// (pixel tile, column block) of a 2-D conv grid (gridDim.x pixel tiles x gridDim.y column blocks) in XCD-aware
// order: the logical order is pixel-major, column-minor, so the column blocks of one pixel tile and the
// neighbouring pixel tiles (the 3x3 halo rows) share one L2 instead of being dealt to different XCDs.
__device__ __forceinline__ void xcd_tile2(int& mb, int& nb) {
  const int gy = gridDim.y;
  const int f = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gy);  // dispatch order: x fastest
  mb = f / gy;
  nb = f - mb * gy;
}

// Input binding (include/ydbl.h ydbl_input_bind): batch pointer and LoadTensor scale read when the kernel runs.
struct InputBind {
  const float* const* x;
  const float* amax;
};
__device__ __forceinline__ const float* bound_x(const InputBind& ib, const float* x) { return ib.x ? *ib.x : x; }
__device__ __forceinline__ float bound_scale(const InputBind& ib, float scale) {
  return ib.x ? (*ib.amax > 1.0f + __FLT_EPSILON__ ? 1.0f / 255.0f : 1.0f) : scale;
}
__host__ inline InputBind input_bind(const ydbl_input_bind* b) {
  return b ? InputBind{b->x, b->amax} : InputBind{nullptr, nullptr};
}

// This lane's wave within the workgroup, as a scalar: hipcc's divergence analysis treats threadIdx.x >> 6 as
// per-lane, which puts every loop over a wave's share of the work (and its exec-mask bookkeeping) on the VALU.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Unconditional load + select: `ok ? *p : 0` without a branch around the load.  hipcc turns a
// per-lane "load or zero" into a branch with its own s_waitcnt vmcnt(0), which serialises every
// load of an unrolled staging loop; loading from a clamped, always-valid address and selecting
// afterwards keeps all loads in flight together.  `safe` must be a readable address.
template <typename T>
__device__ __forceinline__ typename Vec<T>::type vload_sel(const T* p, const T* safe, bool ok) {
  typename Vec<T>::type v = vload(ok ? p : safe);
  return ok ? v : vzero<T>();
}
// The same split in two for prefetch pipelines: the load from the clamped address now, the zero select where
// the value is consumed (a select next to its load makes the compiler wait for that load right there: one full
// memory round trip per prefetched vector instead of one per pipeline stage).
template <typename T>
__device__ __forceinline__ typename Vec<T>::type vload_clamped(const T* p, const T* safe, bool ok) {
  return vload(ok ? p : safe);
}
template <typename V>
__device__ __forceinline__ V vsel(const V& v, bool ok) {
  return ok ? v : V{};
}

// Load/store VEC elements as fp32.
template <typename T, int N>
__device__ __forceinline__ void load_f(const T* p, float* o) {
#pragma unroll
  for (int i = 0; i < N; ++i) o[i] = float(p[i]);
}
template <int N>
__device__ __forceinline__ void load_f(const _Float16* p, float* o) {
  if constexpr (N == 8) {
    h8 v = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = float(v[i]);
  } else if constexpr (N == 4) {
    h4 v = *reinterpret_cast<const h4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = float(v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = float(p[i]);
  }
}
template <int N>
__device__ __forceinline__ void load_f(const float* p, float* o) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(p + i);
      o[i] = v[0]; o[i + 1] = v[1]; o[i + 2] = v[2]; o[i + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = p[i];
  }
}
// fp32 -> fp16 as its own rounding step (round-to-nearest-even of the fp32 value).  hipcc otherwise
// folds the op that produced the fp32 value (a multiply, an fmaf) into v_fma_mixlo_f16, which
// rounds the EXACT result once to fp16: in rare near-tie cases 1 ulp away from the fp32 result
// rounded to fp16 (the reference's accumulate-in-fp32-then-store), and chosen differently per
// kernel, so two launch plans of the same arithmetic would not agree bit for bit.  The empty asm
// pins the fp32 value in a VGPR.
__device__ __forceinline__ _Float16 f16_rne(float v) {
  asm volatile("" : "+v"(v));
  return (_Float16)v;
}
__device__ __forceinline__ h4 to_h4_rne(const float* a) {
  float v0 = a[0], v1 = a[1], v2 = a[2], v3 = a[3];
  asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
  return h4{(_Float16)v0, (_Float16)v1, (_Float16)v2, (_Float16)v3};
}

// Explicit-contraction arithmetic for results two kernels must agree on bit for bit.  Under hipcc's
// default fp-contract=fast the backend fuses a*b + c into an fma or not per kernel and even per
// element (register pressure, v_fma_mix selection), so the same source expression in two kernels
// can differ by an ulp.  These fix the rounding points.
// FullPAD_Tunnel mix y2 = a2 * y + b2 * r, equal to ydbl_gate_add's fmaf(gate, b, a) when one of the
// two coefficients is 1 (the only way the fused second outputs use it: a2 = 1 or b2 = 1).
__device__ __forceinline__ float pad_mix(float a2, float y, float b2, float r) {
  if (b2 == 1.0f) return __builtin_fmaf(a2, y, r);
  if (a2 == 1.0f) return __builtin_fmaf(b2, r, y);
  return __builtin_fmaf(a2, y, b2 * r);
}
// LSKblock gate attn1 * s0 + attn2 * s1 (LSKA.py:50): the first product rounded, the second fused
__device__ __forceinline__ float gate_mix(float a1, float s0, float a2, float s1) {
  float o = a1 * s0;
  asm volatile("" : "+v"(o));
  return __builtin_fmaf(a2, s1, o);
}
// bilinear blend in grid_sample's nw, ne, sw, se order, one rounding per term
__device__ __forceinline__ float blend4(float vnw, float wnw, float vne, float wne, float vsw, float wsw, float vse,
                                        float wse) {
  float o = vnw * wnw;
  asm volatile("" : "+v"(o));  // keep the first product a plain multiply
  o = __builtin_fmaf(vne, wne, o);
  o = __builtin_fmaf(vsw, wsw, o);
  return __builtin_fmaf(vse, wse, o);
}

// v as a stored T would hold it, back in fp32 (T = _Float16: f16_rne; T = float: v)
template <typename T>
__device__ __forceinline__ float round_to(float v) {
  if constexpr (std::is_same<T, float>::value) return v;
  else return float(f16_rne(v));
}

template <int N>
__device__ __forceinline__ void store_f(_Float16* p, const float* v) {
  if constexpr (N == 8) {
    h8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f16_rne(v[i]);
    *reinterpret_cast<h8*>(p) = o;
  } else if constexpr (N == 4) {
    *reinterpret_cast<h4*>(p) = to_h4_rne(v);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = f16_rne(v[i]);
  }
}
template <int N>
__device__ __forceinline__ void store_f(float* p, const float* v) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) *reinterpret_cast<f32x4*>(p + i) = f32x4{v[i], v[i + 1], v[i + 2], v[i + 3]};
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = v[i];
  }
}

// ---- activations (fp32) ---------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// SiLU in the fp16 / fp8 epilogues: hardware exp2 + reciprocal (v_exp_f32 / v_rcp_f32, ~1 ulp
// each) instead of the IEEE expf + division sequence; 4-5 VALU ops per element, far below fp16
// rounding.  The fp32 (parity) path keeps ATen's CPU op sequence x / (1 + exp(-x)) with IEEE
// division, so its only deviation from the reference is the accumulation order of the convs.
__device__ __forceinline__ float silu_fast(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
}
__device__ __forceinline__ float silu_exact(float v) { return v / (1.0f + expf(-v)); }
template <typename T>
__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case YDBL_ACT_SILU:
      if constexpr (std::is_same<T, float>::value) return silu_exact(v);
      else return silu_fast(v);
    case YDBL_ACT_GELU: return gelu_erf(v);
    case YDBL_ACT_SIGMOID: return sigmoidf_(v);
    default: return v;
  }
}

// Plain-struct view passed by value to kernels.
template <typename T>
struct DView {
  T* p;
  int n, h, w, c, cs;
  __device__ __forceinline__ T* at(int b, int y, int x) const { return p + ((int64_t)(b * h + y) * w + x) * cs; }
  __device__ __forceinline__ T* pix(int64_t pixel) const { return p + pixel * cs; }
};
template <typename T>
inline DView<T> dview(const ydbl_view& v) {
  return DView<T>{reinterpret_cast<T*>(v.ptr), v.n, v.h, v.w, v.c, v.cs};
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

int check_view(const ydbl_view* v, const char* name, bool need_vec_align);

}  // namespace ydbl
