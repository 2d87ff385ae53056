// Shared types for the ViT / DPT kernels (bf16 MFMA path, gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

// OCP fp8 e4m3 (gfx950 v_cvt_pk_fp8_f32, RNE), inputs saturated to the finite range ±448
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

__device__ __forceinline__ float bf2f(bf16_t v) { return (float)v; }
__device__ __forceinline__ bf16_t f2bf(float v) { return (bf16_t)v; }  // RNE (v_cvt_pk_bf16_f32)

// erf by Abramowitz & Stegun 7.1.26 (|error| ≤ 1.5e-7, i.e. f32 rounding level): one rcp,
// one exp2 and six FMAs, branch-free.  The library erff takes two polynomial paths selected
// per lane; at one wave per SIMD the GEMM's GELU epilogue was ≈ 40 % of an M = 768 fc1
// launch with it (tools/gemm_depth.py).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-(ax * ax) * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.0f), x);
}

__device__ __forceinline__ float gelu_erf(float x) {
  // nn.GELU() default (approximate='none'): 0.5 x (1 + erf(x / sqrt(2)))
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}
