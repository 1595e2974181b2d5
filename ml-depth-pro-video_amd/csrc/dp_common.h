// Shared device helpers for the Depth Pro MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dp_mi355x.h"

typedef uint16_t u16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(2))) short i16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

// 16-bit element kinds.  Activations and weights are carried as raw u16 bits;
// the kind only decides the MFMA opcode and the float<->16-bit conversions.
struct KBF16 {
  static constexpr int id = DP_BF16;
  static constexpr int lo8_shift = 7 + 9;      // split residual (lo8_*): 2^(e - 16) = ulp(hi) / 256
  static __device__ __forceinline__ float to_f(u16 v) {
    return __uint_as_float(((uint32_t)v) << 16);
  }
  static __device__ __forceinline__ u16 from_f(float f) {
    return __builtin_bit_cast(u16, (__bf16)f);
  }
  // two floats -> packed pair (a in the low half), one v_cvt_pk_bf16_f32 (RNE)
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
  }
  static __device__ __forceinline__ f32x4_t mfma16(uint4 a, uint4 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x16_t mfma32(uint4 a, uint4 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
};

struct KF16 {
  static constexpr int id = DP_F16;
  static constexpr int lo8_shift = 10 + 9;     // 2^(e - 19) = ulp(hi) / 256
  static __device__ __forceinline__ float to_f(u16 v) {
    return (float)__builtin_bit_cast(_Float16, v);
  }
  static __device__ __forceinline__ u16 from_f(float f) {
    return __builtin_bit_cast(u16, (_Float16)f);
  }
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
  }
  static __device__ __forceinline__ f32x4_t mfma16(uint4 a, uint4 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x16_t mfma32(uint4 a, uint4 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  }
};

// The split residual's 8-bit low part (dp_gemm_args.ln_xl, ABI 12): x = hi + q * 2^(e - S), hi = x
// rounded to 16 bits, e = frexp exponent of hi (hi = m 2^e, m in [0.5, 1)), S = K_::lo8_shift, so
// the step is ulp(hi) / 256 and q = rint((x - hi) / step) in [-128, 127] (|x - hi| <= ulp / 2: only
// an exact tie reaches 128, clamped).  x - hi, the scaling and hi + q step are exact in fp32, so
// host code reproduces both directions bit for bit.  About 16 significant bits of x.
template <typename K_>
__device__ __forceinline__ int lo8_encode(float x, float hf) {
  const int e = __builtin_amdgcn_frexp_expf(hf);
  const float q = __builtin_rintf(__builtin_amdgcn_ldexpf(x - hf, K_::lo8_shift - e));
  return (int)__builtin_amdgcn_fmed3f(q, -128.f, 127.f);
}
template <typename K_>
__device__ __forceinline__ float lo8_decode(float hf, int q) {
  return hf + __builtin_amdgcn_ldexpf((float)q, __builtin_amdgcn_frexp_expf(hf) - K_::lo8_shift);
}
// 4 signed bytes <-> 4 ints (byte r = value r)
__device__ __forceinline__ uint32_t pack_i8x4(int a, int b, int c, int d) {
  return (uint32_t)(a & 0xff) | ((uint32_t)(b & 0xff) << 8) | ((uint32_t)(c & 0xff) << 16) | ((uint32_t)d << 24);
}
__device__ __forceinline__ int unpack_i8(uint32_t w, int r) { return (int)(w << (24 - 8 * r)) >> 24; }

// ReLU on packed 16-bit floats (bf16 or f16): a negative value has its sign bit
// set, i.e. is a negative int16, so max_i16(x, 0) zeroes it (-0 and negative
// NaNs included) and leaves every non-negative value bit-identical.
__device__ __forceinline__ uint32_t relu_pk16(uint32_t v) {
  i16x2_t x = __builtin_bit_cast(i16x2_t, v);
  i16x2_t z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, z));
}
__device__ __forceinline__ uint4 relu_pk16(uint4 v) {
  return make_uint4(relu_pk16(v.x), relu_pk16(v.y), relu_pk16(v.z), relu_pk16(v.w));
}

// nn.GELU() (exact erf form, timm Mlp.act).  Evaluated as x * sigmoid(x * P(x^2))
// with P a quadratic fitted (weighted minimax, scipy) to 0.5*x*(1+erf(x/sqrt2)):
// max |error| 2.6e-5 over all x (fp32 evaluation, checked on [-12, 12]; x^2 is
// clamped at 25, beyond which the result is x or -0 to < 2e-6) -- 100x below the
// bf16 rounding of the value it feeds.  7 VALU + 2 transcendental, vs ~35 for erff.
__device__ __forceinline__ float gelu_erf(float x) {
  const float t = fminf(x * x, 25.0f);
  const float q = x * fmaf(fmaf(t, 1.0142713e-03f, -1.0677578e-01f), t, -2.3011212e+00f);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(q));
}
// The same GELU on 4 values in the f32x4 vector form, so that the multiplies, FMAs and adds
// become packed-f32 VALU ops (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: two values per
// instruction) -- the epilogues run it with no MFMA beside it, where the packed forms halve
// the VALU issue time.  Same operations in the same order per value: bit-identical to gelu_erf.
__device__ __forceinline__ f32x4_t gelu_erf4(f32x4_t x) {
  f32x4_t t = x * x;
  t.x = fminf(t.x, 25.0f); t.y = fminf(t.y, 25.0f); t.z = fminf(t.z, 25.0f); t.w = fminf(t.w, 25.0f);
  const f32x4_t a = 1.0142713e-03f, b = -1.0677578e-01f, c = -2.3011212e+00f;
  const f32x4_t q = x * __builtin_elementwise_fma(__builtin_elementwise_fma(t, a, b), t, c);
  f32x4_t e;
  e.x = __builtin_amdgcn_exp2f(q.x); e.y = __builtin_amdgcn_exp2f(q.y);
  e.z = __builtin_amdgcn_exp2f(q.z); e.w = __builtin_amdgcn_exp2f(q.w);
  e = e + 1.0f;
  f32x4_t r;
  r.x = __builtin_amdgcn_rcpf(e.x); r.y = __builtin_amdgcn_rcpf(e.y);
  r.z = __builtin_amdgcn_rcpf(e.z); r.w = __builtin_amdgcn_rcpf(e.w);
  return x * r;
}

#define DP_CHECK_LAUNCH()                                        \
  do {                                                           \
    hipError_t e__ = hipGetLastError();                          \
    if (e__ != hipSuccess) return (int)e__;                      \
  } while (0)
