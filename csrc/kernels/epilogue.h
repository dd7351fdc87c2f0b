// Elementwise GEMM epilogue ops shared by the NT GEMM kernels (gemm_conv.hip, gemm256.hip).
#pragma once
#include "common.h"

// erf(z) without branches (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 -- far below the bf16
// output's 2^-9 relative rounding): one reciprocal, one exp, five FMAs.  The device library's erff
// is a multi-range routine that made the GELU epilogues of the ViT GEMMs VALU-bound (fc1 +0.22 ms,
// fc2 data gradient +0.22 ms per layer over the plain GEMM; tools/bench_vit_layer_gemms.py).
// e_out = exp(-z*z), which the GELU derivative reuses (exp(-x^2/2) at z = x/sqrt(2)).
__device__ __forceinline__ float erf_fast(float z, float& e_out) {
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * az);
  const float e = __expf(-az * az);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  e_out = e;
  return copysignf(1.f - p * e, z);
}

// erf-form GELU (nn.GELU default) and its derivative
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return 0.5f * x * (1.f + erf_fast(x * 0.70710678f, e));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float e;  // exp(-x^2 / 2)
  const float r = erf_fast(x * 0.70710678f, e);
  return 0.5f * (1.f + r) + x * 0.39894228f * e;
}

// GELU and its derivative at one point, from one erf / exp: the forward epilogue stores the
// derivative for the backward instead of the pre-activation (see epilogue_op_v, epi 1 / 2)
__device__ __forceinline__ float gelu_fg(float x, float& d) {
  float e;  // exp(-x^2 / 2)
  const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678f, e));
  d = cdf + x * 0.39894228f * e;
  return x * cdf;
}

// elementwise op on one 16-byte chunk (8 bf16) of the bf16 epilogue; aux has C's layout.
//   epi 1 (GELU):          C <- gelu(u), aux <- gelu'(u)   (u = acc + bias, rounded to bf16)
//   epi 2 (GELU backward): C <- acc * aux                  (aux = the derivative epi 1 stored)
//   epi 3 (residual):      C <- acc + aux
// Storing gelu'(u) rather than u moves the derivative's erf / exp from the backward GEMM's
// epilogue (where it cost 0.16 ms per ViT-B/16 layer over the plain GEMM) into the forward one,
// which evaluates the same erf / exp for gelu(u) anyway.
// epi 2 / 3 read aux: callers that batch their loads pass the chunk already loaded (aux_v).
__device__ __forceinline__ uint4 epilogue_op_v(int epi, uint4 v, bf16_t* aux, uint4 aux_v) {
  float f[8];
  unpack8(v, f);
  if (epi == 1) {
    float d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = gelu_fg(f[q], d[q]);
    *(uint4*)aux = pack8(d);
  } else {
    float g[8];
    unpack8(aux_v, g);
    if (epi == 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] *= g[q];
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] += g[q];
    }
  }
  return pack8(f);
}

__device__ __forceinline__ uint4 epilogue_op(int epi, uint4 v, bf16_t* aux) {
  return epilogue_op_v(epi, v, aux, epi == 1 ? v : *(const uint4*)aux);
}
