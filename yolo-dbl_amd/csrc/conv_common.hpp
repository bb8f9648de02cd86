// Shared pieces of the MFMA convolution kernels (conv.hip, dsconv.hip): argument block,
// MFMA k-chunk (f16 16x16x32 / exact f32 4x 16x16x4) and the fused epilogue.
#pragma once
#include "common.hpp"

namespace ydbl {

template <typename T>
struct ConvArgs {
  const T* x; int xcs; int N, H, W, Cin;
  T* y; int ycs; int Ho, Wo, Cout;
  const T* r; int rcs;
  const T* w; const float* bias;
  int KW, S, PAD, DIL, K, KPAD;
  int act, res;
  int P;
  T* y2; int y2cs;  // optional second output y2 = a2 * T(v) + b2 * r2 (fused FullPAD)
  const T* r2; int r2cs;
  float a2, b2;
  // fp8 operand mode (dq != nullptr): w holds OCP e4m3 bytes [Cout][KPAD] (per-output-channel
  // scale sw), activations are quantized to e4m3 with the per-tensor scale qs as they are staged,
  // and the accumulator is dequantized by dq[co] = 1 / (sw[co] * qs) before bias / activation.
  const float* dq;
  float qs;
  // optional trailing 1x1 conv of nt3 (<= 4) outputs over all Cout channels (dsconv.hip, Detect cls):
  // y3[p][k] = sum_c t3w[k][c] * T(y[p][c]) + t3b[k]
  const float* t3w; const float* t3b;
  T* y3; int y3cs; int nt3;
  // optional trailing GEMM over [y ; g2x] (dsc_lean.hip, C3's cv3): g2y = g2act(g2w [y ; g2x] + g2b), y not stored
  const T* g2w; const float* g2b;
  const T* g2x; int g2xcs;
  T* g2y; int g2ycs; int g2act;
  // optional leading 1x1 (dsc_lean.hip, C3's merged cv2|cv1): g0y = g0act(g0w g0x + g0b), x = g0y's last Cin channels
  const T* g0w; const float* g0b;
  const T* g0x; int g0xcs;
  T* g0y; int g0ycs; int g0act;
  // split-K (conv_wsk_kernel): ksplit > 1 -> fp32 partial tiles ws[z][P][round_up(Cout, 4)], summed + epilogue by
  // splitk_epilogue_kernel
  float* ws; int64_t ws_bytes; int ksplit;
};

// ---- operand policy: f16/f32 vectors, or 8-byte groups of 8 e4m3 values (fp8 MFMA) -----------
template <typename T, bool Q8> struct Op {
  using lds = typename Vec<T>::type;
};
template <> struct Op<_Float16, true> {
  using lds = uint64_t;
};

// 8 activations -> 8 OCP e4m3 bytes (k order kept: byte i = element i), scaled and saturated
__device__ __forceinline__ uint64_t quant_e4m3(const h8& v, float s) {
  float f[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = fminf(fmaxf(float(v[i]) * s, -448.f), 448.f);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}

template <typename T, bool Q8>
__device__ __forceinline__ typename Op<T, Q8>::lds to_op(const typename Vec<T>::type& v, float s) {
  if constexpr (Q8) return quant_e4m3(v, s);
  else return v;
}

// weight (A operand) load of one k-vector: VEC elements of T, or 8 e4m3 bytes at the same
// element offset (the fp8 matrix is [Cout][KPAD] bytes); load_wop_raw leaves the zero select to the consumer
template <typename T, bool Q8>
__device__ __forceinline__ typename Op<T, Q8>::lds load_wop_raw(const T* w, int64_t off, bool ok) {
  if constexpr (Q8) {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
    return *reinterpret_cast<const uint64_t*>(b + (ok ? off : 0));
  } else {
    return vload_clamped(w + off, w, ok);
  }
}
template <typename T, bool Q8>
__device__ __forceinline__ typename Op<T, Q8>::lds load_wop(const T* w, int64_t off, bool ok) {
  if constexpr (Q8) {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
    const uint64_t v = *reinterpret_cast<const uint64_t*>(b + (ok ? off : 0));
    return ok ? v : 0ull;
  } else {
    return vload_sel(w + off, w, ok);
  }
}


// LDS slot of halo pixel `pix` (row-major over the halo tile), k-vector g, in the halo kernels' "planar per 16-lane
// run" layout (conv3x3.hip)
template <int S>
__device__ __forceinline__ int hslot(int pix, int g) {
  return (pix / (16 * S)) * (64 * S) + g * (16 * S) + (pix % S) * 16 + ((pix / S) & 15);
}

// conv3x3.hip: halo-tiled 3x3 kernel for Cin >= 2 k-steps; false when the shape is not its own.
template <typename T, bool Q8>
bool try_conv3x3_halo(const ConvArgs<T>& a, int kh, hipStream_t s);
// conv3x3.hip: fp16 3x3 stride-1 convs with Cin 32..128 and VGPR-resident weights.
bool try_conv3x3_vw(const ConvArgs<_Float16>& a, int kh, hipStream_t s);
// dsc_lean.hip: one-round-trip DSConv / DWConv->Conv1x1 for the small-map shapes it is built for.
// dsconv.hip: a ydbl_dsconv_desc's kernel arguments (fp16) and its descriptor rules (YDBL_OK or the error code).
ConvArgs<_Float16> ds_args_f16(const ydbl_dsconv_desc* d);
int ds_check(const ydbl_dsconv_desc* d);
bool try_dsc_lean(const ConvArgs<_Float16>& a, const float* dww, const float* dwb, int dw_act, int k, int st, int dil,
                  hipStream_t s);

template <typename T>
__device__ __forceinline__ f32x4 mfma_chunk(const typename Vec<T>::type& a, const typename Vec<T>::type& b, f32x4 c);

template <>
__device__ __forceinline__ f32x4 mfma_chunk<_Float16>(const h8& a, const h8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma_chunk<float>(const f32x4& a, const f32x4& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

// one MFMA k-step on policy operands (fp8: v_mfma_f32_16x16x32_fp8_fp8, 8 e4m3 per lane)
template <typename T, bool Q8>
__device__ __forceinline__ f32x4 mfma_op(const typename Op<T, Q8>::lds& a, const typename Op<T, Q8>::lds& b, f32x4 c) {
  if constexpr (Q8) return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8((long)a, (long)b, c, 0, 0, 0);
  else return mfma_chunk<T>(a, b, c);
}

// The workgroup's N output channels' bias from c0 on, for the epilogue to read from LDS (conv_epilogue's sb):
// read from global memory after the k-loop, the bias cost every launch one more dependent round trip at its very
// end.  fetch() issues the loads at the start of the first round trip, commit() stores them into LDS just before
// that round trip's barrier (a store right after its load would wait on every load issued before it).  256-thread
// workgroups; clamped like the epilogue's own loads.
template <int N>
struct BiasStage {
  static constexpr int IT = (N + 255) / 256;
  float v[IT];
  __device__ __forceinline__ void fetch(const float* bias, int c0, int cout) {
#pragma unroll
    for (int it = 0; it < IT; ++it) v[it] = bias ? bias[min(c0 + (int)threadIdx.x + it * 256, cout - 1)] : 0.f;
  }
  __device__ __forceinline__ void commit(float* s) const {
#pragma unroll
    for (int it = 0; it < IT; ++it)
      if ((int)threadIdx.x + it * 256 < N) s[threadIdx.x + it * 256] = v[it];
  }
};

// Epilogue of one wave's TN x TM accumulator tiles: lane owns output channels co[i]..co[i]+3 of
// pixel pp[j].  Every load is unconditional from a clamped address (bias once; the residual of a
// pixel for all TN tiles at once) so the loads overlap; only the stores are predicated.
// sb: the bias staged in LDS for channels sb0.. (16-byte aligned), or nullptr to load it here.
template <typename T, int TN, int TM, bool Q8 = false>
__device__ __forceinline__ void conv_epilogue(const ConvArgs<T>& p, const f32x4 (&acc)[TN][TM],
                                              const int64_t (&pp)[TM], const bool (&pv)[TM], const int (&co)[TN],
                                              const float* sb = nullptr, int sb0 = 0) {
  const bool c4 = (p.Cout & 3) == 0;  // uniform: co..co+3 in range whenever co < Cout
  float bv[TN][4];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    if (sb) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(sb + co[i] - sb0);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = b4[q];
    } else if (p.bias) {
      if (c4) {
        load_f<4>(p.bias + min(co[i], p.Cout - 4), bv[i]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[i][q] = p.bias[min(co[i] + q, p.Cout - 1)];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = 0.f;
    }
  }
  float dqv[TN][4];  // fp8 dequant factors (constant 1 folds away in the f16/f32 paths)
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) dqv[i][q] = Q8 ? p.dq[min(co[i] + q, p.Cout - 1)] : 1.f;
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int64_t pc = pv[j] ? pp[j] : 0;
    float rv[TN][4];
    if (p.res != YDBL_RES_NONE) {
      const T* rp = p.r + pc * p.rcs;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        if (c4) {
          load_f<4>(rp + min(co[i], p.Cout - 4), rv[i]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) rv[i][q] = float(rp[min(co[i] + q, p.Cout - 1)]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act<T>(acc[i][j][q] * dqv[i][q] + bv[i][q], p.act);
      if (p.res == YDBL_RES_ADD) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = rv[i][q] + v[q];
      } else if (p.res == YDBL_RES_MUL) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = rv[i][q] * v[q];
      }
      if (!pv[j] || co[i] >= p.Cout) continue;
      T* yp = p.y + pc * p.ycs + co[i];
      if (co[i] + 4 <= p.Cout) {
        store_f<4>(yp, v);
      } else {
        for (int q = 0; q < 4 && co[i] + q < p.Cout; ++q) store_f<1>(yp + q, v + q);
      }
      if (p.y2) {  // uniform
        const T* r2p = p.r2 + pc * p.r2cs + co[i];
        T* y2p = p.y2 + pc * p.y2cs + co[i];
        if (co[i] + 4 <= p.Cout) {
          float r2v[4];
          load_f<4>(r2p, r2v);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            r2v[q] = pad_mix(p.a2, round_to<T>(v[q]), p.b2, r2v[q]);  // y as stored (rounded to T)
          }
          store_f<4>(y2p, r2v);
        } else {
          for (int q = 0; q < 4 && co[i] + q < p.Cout; ++q) {
            const float o = pad_mix(p.a2, round_to<T>(v[q]), p.b2, float(r2p[q]));
            store_f<1>(y2p + q, &o);
          }
        }
      }
    }
  }
}

// Trailing 1x1 conv with <= 4 outputs over all Cout channels of a pixel, for kernels whose wave holds
// every channel of its pixels (TN * 16 == Cout): the Detect head's class conv cv3[i][2] (head.py:93-101)
// after its DWConv -> Conv1x1 pair.  Lane (r16, g) holds channels co[i]..co[i]+3 of pixel pp[j]; the
// rounded activations (T, as the unfused path stores them) are dotted with the weights per lane and the
// four lane groups are summed by xor-shuffles (fixed order); lane group 0 stores.
template <typename T, int TN, int TM>
__device__ __forceinline__ void conv_tail_1x1(const ConvArgs<T>& p, const f32x4 (&acc)[TN][TM], const int64_t (&pp)[TM],
                                              const bool (&pv)[TM], const int (&co)[TN], int g) {
  float bv[TN][4], wv[TN][4][4];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bv[i][q] = p.bias ? p.bias[co[i] + q] : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) wv[i][q][k] = k < p.nt3 ? p.t3w[k * p.Cout + co[i] + q] : 0.f;
    }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float u = round_to<T>(apply_act<T>(acc[i][j][q] + bv[i][q], p.act));  // y as stored
#pragma unroll
        for (int k = 0; k < 4; ++k) part[k] = fmaf(u, wv[i][q][k], part[k]);
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      part[k] += __shfl_xor(part[k], 16);
      part[k] += __shfl_xor(part[k], 32);
    }
    if (g == 0 && pv[j]) {
      T* o = p.y3 + pp[j] * p.y3cs;
      for (int k = 0; k < p.nt3; ++k) o[k] = T(part[k] + p.t3b[k]);
    }
  }
}

// The same tail from the values the epilogue stored (ys = y rounded to T, per lane [TN][TM][4]): no activation
// recomputed.  Lanes of one pixel share pv, so the xor-shuffles only mix lanes of the same pixel.
// s_t: the weights [4][Cout] staged in LDS (rows past nt3 zero), or nullptr to read them from global memory (a
// late round trip of 16 x nt3 scalar loads per lane at the very end of the launch: kbench pair 64+tail @80^2 bs16 24.8 vs 20.5 us, profiles/r05/r05_bias_lds_ab.txt).
template <typename T, int TN, int TM>
__device__ __forceinline__ void conv_tail_1x1_vals(const ConvArgs<T>& p, const float (&ys)[TN][TM][4],
                                                   const int64_t (&pp)[TM], const bool (&pv)[TM], const int (&co)[TN],
                                                   int g, const float* s_t = nullptr) {
  float wv[TN][4][4];
  if (s_t) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(s_t + k * p.Cout + co[i]);
#pragma unroll
        for (int q = 0; q < 4; ++q) wv[i][q][k] = w4[q];
      }
  } else {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) wv[i][q][k] = k < p.nt3 ? p.t3w[k * p.Cout + co[i] + q] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) part[k] = fmaf(ys[i][j][q], wv[i][q][k], part[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      part[k] += __shfl_xor(part[k], 16);
      part[k] += __shfl_xor(part[k], 32);
    }
    if (g == 0 && pv[j]) {
      T* o = p.y3 + pp[j] * p.y3cs;
      for (int k = 0; k < p.nt3; ++k) o[k] = T(part[k] + p.t3b[k]);
    }
  }
}

}  // namespace ydbl
