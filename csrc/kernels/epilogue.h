// Elementwise GEMM epilogue ops shared by the NT GEMM kernels (gemm_conv.hip, gemm256.hip).
#pragma once
#include "common.h"

// erf-form GELU (nn.GELU default) and its derivative
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678f)) + x * 0.39894228f * __expf(-0.5f * x * x);
}

// elementwise op on one 16-byte chunk (8 bf16) of the bf16 epilogue; aux has C's layout
__device__ __forceinline__ uint4 epilogue_op(int epi, uint4 v, bf16_t* aux) {
  float f[8];
  unpack8(v, f);
  if (epi == 1) {
    *(uint4*)aux = v;
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = gelu_f(f[q]);
  } else {
    float g[8];
    unpack8(*(const uint4*)aux, g);
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
