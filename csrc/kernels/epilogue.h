// Elementwise GEMM epilogue ops shared by the NT GEMM kernels (gemm_conv.hip, gemm256.hip).
#pragma once
#include "common.h"

// erf-form GELU (nn.GELU default) and its derivative
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678f)) + x * 0.39894228f * __expf(-0.5f * x * x);
}

// elementwise op on one 16-byte chunk (8 bf16) of the bf16 epilogue; aux has C's layout.
// epi 2 / 3 read aux: callers that batch their loads pass the chunk already loaded (aux_v).
__device__ __forceinline__ uint4 epilogue_op_v(int epi, uint4 v, bf16_t* aux, uint4 aux_v) {
  float f[8];
  unpack8(v, f);
  if (epi == 1) {
    *(uint4*)aux = v;
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = gelu_f(f[q]);
  } else {
    float g[8];
    unpack8(aux_v, g);
    if (epi == 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] *= gelu_grad_f(g[q]);
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
