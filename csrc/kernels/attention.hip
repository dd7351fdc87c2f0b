// Exact softmax attention for short sequences (ViT-B/16: T = 197 tokens, head dim 64) on gfx950
// MFMA, reading the packed QKV projection [B*T][3*H*64] and writing O [B*T][H*64] / dQKV
// [B*T][3*H*64] in place -- no head split / merge copies around the kernel.
//
// One workgroup (4 waves) per (batch, head); the head's whole K and V (or Q and dO) live in LDS
// (T <= 256 keys: <= 72 KB), so softmax is exact in one pass (no online rescaling).  Every
// product is a v_mfma_f32_16x16x32_bf16 in "transposed" form so that an accumulator feeds the
// next MFMA as its B operand straight from registers:
//
//   S^T[key][q] = K Q^T          lane: q = lane&15, keys 4g..4g+3 of the tile (g = lane>>4)
//   O^T[dh][q]  = V^T P^T        B = P^T with the k index permuted: k-slot 8g+j <-> key
//                                 4g+j (j<4, tile 2s) / 16+4g+j-4 (j>=4, tile 2s+1) -- exactly the
//                                 four keys x two tiles the lane already holds; A = V^T fetched
//                                 with the same permutation by ds_read_b64_tr_b16 (4 rows x 16 cols
//                                 transposed per 16-lane group) from the row-major V tile.
//
// backward: (1) dQ kernel per q tile: P^T, dP^T = V dO^T, dS^T = P^T (dP^T - D), dQ^T = K^T dS^T,
//               D = rowsum(dO * O) written for (2);
//           (2) dK/dV kernel per key tile: P, dP = dO V^T in [q][key] form, dV^T += dO^T P,
//               dK^T += Q^T dS, reduction over q in registers (no atomics).
#include "common.h"

#include <cstdlib>

namespace {

constexpr int HD = 64;     // head dim
constexpr int KSTR = 72;   // LDS row stride (elements): 144 B -> conflict-free 16-B row reads
                           // and 4-row transposed reads
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ bf16x8 g16(const bf16_t* p) { return __builtin_bit_cast(bf16x8, *(const uint4*)p); }

__device__ __forceinline__ bf16x8 zero8() { return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0)); }

// A^T fragment for an MFMA whose k index is permuted as above: rows r_lo + q4 and r_hi + q4
// (q4 = (lane&15)>>2) of a row-major [rows][KSTR] LDS tile, column block col0 + 4*(lane&3).
__device__ __forceinline__ bf16x8 tr8(const bf16_t* t, int r_lo, int r_hi, int col) {
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, t + r_lo * KSTR + col));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, t + r_hi * KSTR + col));
  short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v8);
}

__device__ __forceinline__ bf16x8 pack_perm(f32x4 a, f32x4 b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4bf(bf16_t* p, f32x4 v, float s) {
  *(uint2*)p = make_uint2(pack2bf(v[0] * s, v[1] * s), pack2bf(v[2] * s, v[3] * s));
}

// rows [0, TP) of two [T][ld] bf16 matrices (64 columns each) -> LDS [TP][KSTR], zero rows >= T.
// All of a thread's global loads are issued before any LDS store (fully unrolled, fixed trip
// count), so the staging costs one memory latency instead of one per 16-byte chunk.
// softmax exponentials: every argument is <= 0 (scores minus the row max / the saved LSE), so
// the hardware v_exp_f32 is exact enough and its flush of results below 2^-126 to zero is
// harmless; the library exp2f wraps it in denormal range scaling (~10 VALU per call, 56 calls
// per 16-query tile and wave in the forward)
__device__ __forceinline__ float att_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// First 16-row tile of wave wv (it then takes every NW-th).  13 tiles (T = 197) cannot be dealt
// evenly over a workgroup's 4 SIMDs (waves w and w + 4 share SIMD w % 4): one SIMD carries 4 tiles,
// the others 3.  Rotating the deal by the (batch, head) index moves that heavy SIMD from workgroup
// to workgroup, so two workgroups sharing a CU would mostly load different SIMDs (rot = 3,
// MI355X_DP_ATT_ROTATE=1).  Measured: forward 0.115 ms either way, backward 0.263 vs 0.255 ms per
// layer, ViT-B/16 6,999 / 6,998 vs 7,014 / 7,002 img/s (profiles/raw/r5/att_rot/) -- the fixed deal
// (rot = 0) stays the default: the hardware does not place co-resident workgroups' waves as assumed.
template <int NW>
__device__ __forceinline__ int tile_start(int wv, int bh, int rot) {
  return (wv + (bh & rot)) % NW;
}

template <int TP, int NW>
__device__ __forceinline__ void stage_rows2(bf16_t* dst0, const bf16_t* src0, int ld0, bf16_t* dst1,
                                            const bf16_t* src1, int ld1, int T) {
  constexpr int NT = 64 * NW;
  constexpr int PER = (TP * 8 + NT - 1) / NT;
  uint4 v0[PER], v1[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, part = c & 7;
    v0[i] = make_uint4(0, 0, 0, 0);
    v1[i] = make_uint4(0, 0, 0, 0);
    if (c < TP * 8 && row < T) {
      v0[i] = *(const uint4*)(src0 + (size_t)row * ld0 + part * 8);
      v1[i] = *(const uint4*)(src1 + (size_t)row * ld1 + part * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, part = c & 7;
    if (c < TP * 8) {
      *(uint4*)&dst0[row * KSTR + part * 8] = v0[i];
      *(uint4*)&dst1[row * KSTR + part * 8] = v1[i];
    }
  }
}

// NW waves per (batch, head) workgroup.  Backward: 8 (default) puts 4 waves on each SIMD at 2
// workgroups per CU (the LDS holds two heads' operands; ~100 VGPRs), so one wave's LDS reads, exp
// and MFMA-result latencies hide behind the others' MFMAs; MI355X_DP_ATT_WAVES=4 selects one wave
// per SIMD per workgroup.  Forward: always 4 (~210 VGPRs).
template <int NK2, int NW>  // keys padded to 32 * NK2 >= T
__global__ __launch_bounds__(64 * NW, NW / 2) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                          float* __restrict__ lse, int T, int H, float sl2,
                                                          int rot) {
  constexpr int TP = 32 * NK2, NKT = 2 * NK2;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[TP * KSTR];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[TP * KSTR];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + (size_t)b * T * ld + h * HD;
  stage_rows2<TP, NW>(Ks, base + D, ld, Vs, base + 2 * D, ld, T);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int nqt = (T + 15) >> 4;
  for (int qt = tile_start<NW>(wv, bh, rot); qt < nqt; qt += NW) {
    const int q = qt * 16 + li;
    const bool qv = q < T;
    bf16x8 qf[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) qf[h2] = qv ? g16(base + (size_t)q * ld + 32 * h2 + 8 * g) : zero8();
    f32x4 s[NKT];
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) acc = mfma(*(const bf16x8*)&Ks[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], qf[h2], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (kt * 16 + 4 * g + r >= T) acc[r] = -INFINITY;
        m = fmaxf(m, acc[r]);
      }
      s[kt] = acc;
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float ms = m * sl2;
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = att_exp2(s[kt][r] * sl2 - ms);
        s[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    f32x4 oa[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oa[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NK2; ++ks) {
      const bf16x8 pb = pack_perm(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        oa[dt] = mfma(tr8(Vs, ks * 32 + 4 * g + q4, ks * 32 + 16 + 4 * g + q4, (dt * 4 + p4) * 4), pb, oa[dt]);
    }
    if (qv) {
      const float inv = 1.f / l;
      bf16_t* orow = o + ((size_t)b * T + q) * D + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4bf(orow + dt * 16 + 4 * g, oa[dt], inv);
      if (g == 0) lse[(size_t)bh * T + q] = (ms + log2f(l)) * LN2;
    }
  }
}

// Forward at 8 waves per (batch, head) workgroup: the scores of a 16-query tile are taken in
// chunks of CP key-tile pairs with an online softmax (running max / sum, O rescaled when the max
// grows), so a wave holds 4 score tiles instead of all 2 * NK2 -- <= 128 VGPRs, 4 waves per SIMD at
// two workgroups per CU -- and one wave's Q-load and exp latencies hide behind the others' MFMAs
// (the backward's 4 -> 8 wave step).  Every chunk holds a valid key (chunk c starts at key
// 32 * CP * c < T), so the running max is finite after the first chunk.
template <int NK2>
__global__ __launch_bounds__(512, 4) void attn_fwd8_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                          float* __restrict__ lse, int T, int H, float sl2) {
  constexpr int NW = 8, TP = 32 * NK2, NKT = 2 * NK2;
  constexpr int CP = 2;  // key-tile pairs per chunk (4 pairs: 0.097 vs 0.095 ms per ViT layer, and spills at NK2 = 4)
  __shared__ __attribute__((aligned(16))) bf16_t Ks[TP * KSTR];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[TP * KSTR];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + (size_t)b * T * ld + h * HD;
  stage_rows2<TP, NW>(Ks, base + D, ld, Vs, base + 2 * D, ld, T);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int nqt = (T + 15) >> 4;
  for (int qt = wv; qt < nqt; qt += NW) {
    const int q = qt * 16 + li;
    const bool qv = q < T;
    bf16x8 qf[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) qf[h2] = qv ? g16(base + (size_t)q * ld + 32 * h2 + 8 * g) : zero8();
    float m = -INFINITY, l = 0.f;
    f32x4 oa[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oa[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c0 = 0; c0 < NK2; c0 += CP) {
      f32x4 sc[2 * CP];
      float cm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2 * CP; ++t) {
        const int kt = 2 * c0 + t;
        if (kt >= NKT) break;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          acc = mfma(*(const bf16x8*)&Ks[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], qf[h2], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (kt * 16 + 4 * g + r >= T) acc[r] = -INFINITY;
          cm = fmaxf(cm, acc[r]);
        }
        sc[t] = acc;
      }
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      const float mn = fmaxf(m, cm);
      const float alpha = att_exp2((m - mn) * sl2);  // first chunk: exp2(-inf) = 0 (oa, l are 0)
      m = mn;
      const float ms = mn * sl2;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) oa[dt] *= alpha;
#pragma unroll
      for (int t = 0; t < 2 * CP; ++t) {
        if (2 * c0 + t >= NKT) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = att_exp2(sc[t][r] * sl2 - ms);
          sc[t][r] = p;
          l += p;
        }
      }
#pragma unroll
      for (int kp = 0; kp < CP; ++kp) {
        const int ks = c0 + kp;
        if (ks >= NK2) break;
        const bf16x8 pb = pack_perm(sc[2 * kp], sc[2 * kp + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          oa[dt] = mfma(tr8(Vs, ks * 32 + 4 * g + q4, ks * 32 + 16 + 4 * g + q4, (dt * 4 + p4) * 4), pb, oa[dt]);
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qv) {
      const float inv = 1.f / l;
      bf16_t* orow = o + ((size_t)b * T + q) * D + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4bf(orow + dt * 16 + 4 * g, oa[dt], inv);
      if (g == 0) lse[(size_t)bh * T + q] = (m * sl2 + log2f(l)) * LN2;
    }
  }
}

template <int NK2, int NW>
__global__ __launch_bounds__(64 * NW, NW / 2) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv,
                                                             const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             float* __restrict__ dvec, bf16_t* __restrict__ dqkv,
                                                             int T, int H, float sl2, float scale, int rot) {
  constexpr int TP = 32 * NK2;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[TP * KSTR];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[TP * KSTR];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + (size_t)b * T * ld + h * HD;
  stage_rows2<TP, NW>(Ks, base + D, ld, Vs, base + 2 * D, ld, T);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int nqt = (T + 15) >> 4;
  for (int qt = tile_start<NW>(wv, bh, rot); qt < nqt; qt += NW) {
    const int q = qt * 16 + li;
    const bool qv = q < T;
    const size_t orow = ((size_t)b * T + q) * D + h * HD;
    // the row's LSE is loaded with its operands (clamped index, discarded past T), not after the
    // dd reduction: issued there under `qv ?` it was a second memory round trip per query tile
    const float lse_q = lse[(size_t)bh * T + min(q, T - 1)];
    bf16x8 qf[2], df[2];
    float dd = 0.f;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      qf[h2] = qv ? g16(base + (size_t)q * ld + 32 * h2 + 8 * g) : zero8();
      df[h2] = qv ? g16(dout + orow + 32 * h2 + 8 * g) : zero8();
      const bf16x8 of = qv ? g16(o + orow + 32 * h2 + 8 * g) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) dd += (float)df[h2][j] * (float)of[j];
    }
    dd += __shfl_xor(dd, 16, 64);
    dd += __shfl_xor(dd, 32, 64);
    const float l2 = qv ? lse_q * LOG2E : 0.f;
    if (qv && g == 0) dvec[(size_t)bh * T + q] = dd;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // dQ^T = K^T dS^T accumulated one 32-key step at a time (P comes from the saved LSE)
#pragma unroll 1
    for (int ks = 0; ks < NK2; ++ks) {
      f32x4 ds[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = 2 * ks + t;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s = mfma(*(const bf16x8*)&Ks[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], qf[h2], s);
          dp = mfma(*(const bf16x8*)&Vs[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], df[h2], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // exp evaluated unconditionally and selected: a conditional exp2f compiled to an
          // exec-masked branch inside the key loop
          const bool valid = qv && (kt * 16 + 4 * g + r < T);
          const float e = att_exp2(s[r] * sl2 - l2);
          const float p = valid ? e : 0.f;
          ds[t][r] = p * (dp[r] - dd);
        }
      }
      const bf16x8 sb = pack_perm(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        dq[dt] = mfma(tr8(Ks, ks * 32 + 4 * g + q4, ks * 32 + 16 + 4 * g + q4, (dt * 4 + p4) * 4), sb, dq[dt]);
    }
    if (qv) {
      bf16_t* drow = dqkv + ((size_t)b * T + q) * ld + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4bf(drow + dt * 16 + 4 * g, dq[dt], scale);
    }
  }
}

template <int NK2, int NW>
__global__ __launch_bounds__(64 * NW, NW / 2) void attn_bwd_dkv_kernel(const bf16_t* __restrict__ qkv,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ dvec,
                                                              bf16_t* __restrict__ dqkv, int T, int H, float sl2,
                                                              float scale, int rot) {
  constexpr int TP = 32 * NK2;
  __shared__ __attribute__((aligned(16))) bf16_t Qs[TP * KSTR];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[TP * KSTR];
  __shared__ float Ls[TP], Dv[TP];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + (size_t)b * T * ld + h * HD;
  stage_rows2<TP, NW>(Qs, base, ld, Ds, dout + (size_t)b * T * D + h * HD, D, T);
  for (int i = threadIdx.x; i < TP; i += 64 * NW) {
    Ls[i] = i < T ? lse[(size_t)bh * T + i] * LOG2E : INFINITY;  // padded queries: P = 0
    Dv[i] = i < T ? dvec[(size_t)bh * T + i] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int nkt = (T + 15) >> 4;
  for (int kt = tile_start<NW>(wv, bh, rot); kt < nkt; kt += NW) {
    const int key = kt * 16 + li;
    const bool kv = key < T;
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      kf[h2] = kv ? g16(base + (size_t)key * ld + D + 32 * h2 + 8 * g) : zero8();
      vf[h2] = kv ? g16(base + (size_t)key * ld + 2 * D + 32 * h2 + 8 * g) : zero8();
    }
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }
#pragma unroll 1
    for (int qs = 0; qs < NK2; ++qs) {
      f32x4 P[2], S[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int row = (2 * qs + t) * 16 + li;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s = mfma(*(const bf16x8*)&Qs[row * KSTR + 32 * h2 + 8 * g], kf[h2], s);
          dp = mfma(*(const bf16x8*)&Ds[row * KSTR + 32 * h2 + 8 * g], vf[h2], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = (2 * qs + t) * 16 + 4 * g + r;
          const float e = att_exp2(s[r] * sl2 - Ls[qq]);  // unconditional + select (see the dQ kernel)
          const float p = kv ? e : 0.f;
          P[t][r] = p;
          S[t][r] = p * (dp[r] - Dv[qq]);
        }
      }
      const bf16x8 pb = pack_perm(P[0], P[1]), sb = pack_perm(S[0], S[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int r0 = qs * 32 + 4 * g + q4, r1 = r0 + 16, col = (dt * 4 + p4) * 4;
        dv[dt] = mfma(tr8(Ds, r0, r1, col), pb, dv[dt]);
        dk[dt] = mfma(tr8(Qs, r0, r1, col), sb, dk[dt]);
      }
    }
    if (kv) {
      bf16_t* drow = dqkv + ((size_t)b * T + key) * ld + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store4bf(drow + D + dt * 16 + 4 * g, dk[dt], scale);
        store4bf(drow + 2 * D + dt * 16 + 4 * g, dv[dt], 1.f);
      }
    }
  }
}

// Backward in ONE kernel per (batch, head): the dQ pass and the dK/dV pass of the two kernels above
// share a workgroup, so every operand is read from HBM once instead of twice.
//   stage K, V (LDS X0, X1) and the LSE
//   pass 1 (per q tile, as attn_bwd_dq_kernel): Q / dO / O fragments from global, D = rowsum(dO*O)
//          into LDS (never to global), dQ
//   each wave copies the K / V fragments of its (<= 2) key tiles from LDS into registers, then
//   X0, X1 are restaged with Q, dO (the rows pass 1 just read: L2 / MALL hits)
//   pass 2 (per key tile, as attn_bwd_dkv_kernel): dK, dV
// 8 waves, 66 KB of LDS at T <= 224, <= 128 VGPRs (launch bound: 4 waves per SIMD): two workgroups
// per CU, one's staging under the other's MFMAs.
template <int NK2>
__global__ __launch_bounds__(512, 4) void attn_bwd_fused_kernel(const bf16_t* __restrict__ qkv,
                                                              const bf16_t* __restrict__ o,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              bf16_t* __restrict__ dqkv, int T, int H, float sl2,
                                                              float scale) {
  constexpr int NW = 8;
  constexpr int TP = 32 * NK2;
  __shared__ __attribute__((aligned(16))) bf16_t X0[TP * KSTR];
  __shared__ __attribute__((aligned(16))) bf16_t X1[TP * KSTR];
  __shared__ float Ls[TP], Dv[TP];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + (size_t)b * T * ld + h * HD;
  const bf16_t* dbase = dout + (size_t)b * T * D + h * HD;
  stage_rows2<TP, NW>(X0, base + D, ld, X1, base + 2 * D, ld, T);
  for (int i = threadIdx.x; i < TP; i += 64 * NW) {
    Ls[i] = i < T ? lse[(size_t)bh * T + i] * LOG2E : INFINITY;  // padded queries: P = 0
    Dv[i] = 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int nt = (T + 15) >> 4;

  // ---- pass 1: dQ (K = X0, V = X1)
  for (int qt = wv; qt < nt; qt += NW) {
    const int q = qt * 16 + li;
    const bool qv = q < T;
    const size_t orow = ((size_t)b * T + q) * D + h * HD;
    bf16x8 qf[2], df[2];
    float dd = 0.f;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      qf[h2] = qv ? g16(base + (size_t)q * ld + 32 * h2 + 8 * g) : zero8();
      df[h2] = qv ? g16(dout + orow + 32 * h2 + 8 * g) : zero8();
      const bf16x8 of = qv ? g16(o + orow + 32 * h2 + 8 * g) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) dd += (float)df[h2][j] * (float)of[j];
    }
    dd += __shfl_xor(dd, 16, 64);
    dd += __shfl_xor(dd, 32, 64);
    const float l2 = Ls[q];  // q < nt * 16 <= TP
    if (qv && g == 0) Dv[q] = dd;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ks = 0; ks < NK2; ++ks) {
      f32x4 ds[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = 2 * ks + t;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s = mfma(*(const bf16x8*)&X0[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], qf[h2], s);
          dp = mfma(*(const bf16x8*)&X1[(kt * 16 + li) * KSTR + 32 * h2 + 8 * g], df[h2], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool valid = qv && (kt * 16 + 4 * g + r < T);
          const float e = att_exp2(s[r] * sl2 - l2);
          ds[t][r] = (valid ? e : 0.f) * (dp[r] - dd);
        }
      }
      const bf16x8 sb = pack_perm(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        dq[dt] = mfma(tr8(X0, ks * 32 + 4 * g + q4, ks * 32 + 16 + 4 * g + q4, (dt * 4 + p4) * 4), sb, dq[dt]);
    }
    if (qv) {
      bf16_t* drow = dqkv + ((size_t)b * T + q) * ld + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4bf(drow + dt * 16 + 4 * g, dq[dt], scale);
    }
  }

  // ---- hand-over: this wave's key tiles (wv, wv + NW; nt <= 16) to registers, then Q / dO staged
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int row = min(wv + NW * j, nt - 1) * 16 + li;  // rows >= T are zero in the staged tiles
      kf[j][h2] = *(const bf16x8*)&X0[row * KSTR + 32 * h2 + 8 * g];
      vf[j][h2] = *(const bf16x8*)&X1[row * KSTR + 32 * h2 + 8 * g];
    }
  __syncthreads();
  stage_rows2<TP, NW>(X0, base, ld, X1, dbase, D, T);
  __syncthreads();

  // ---- pass 2: dK, dV (Q = X0, dO = X1)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kt = wv + NW * j;
    if (kt >= nt) break;
    const int key = kt * 16 + li;
    const bool kv = key < T;
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }
#pragma unroll 1
    for (int qs = 0; qs < NK2; ++qs) {
      f32x4 P[2], S[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int row = (2 * qs + t) * 16 + li;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s = mfma(*(const bf16x8*)&X0[row * KSTR + 32 * h2 + 8 * g], kf[j][h2], s);
          dp = mfma(*(const bf16x8*)&X1[row * KSTR + 32 * h2 + 8 * g], vf[j][h2], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = (2 * qs + t) * 16 + 4 * g + r;
          const float e = att_exp2(s[r] * sl2 - Ls[qq]);
          const float p = kv ? e : 0.f;
          P[t][r] = p;
          S[t][r] = p * (dp[r] - Dv[qq]);
        }
      }
      const bf16x8 pb = pack_perm(P[0], P[1]), sb = pack_perm(S[0], S[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int r0 = qs * 32 + 4 * g + q4, r1 = r0 + 16, col = (dt * 4 + p4) * 4;
        dv[dt] = mfma(tr8(X1, r0, r1, col), pb, dv[dt]);
        dk[dt] = mfma(tr8(X0, r0, r1, col), sb, dk[dt]);
      }
    }
    if (kv) {
      bf16_t* drow = dqkv + ((size_t)b * T + key) * ld + h * HD;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store4bf(drow + D + dt * 16 + 4 * g, dk[dt], scale);
        store4bf(drow + 2 * D + dt * 16 + 4 * g, dv[dt], 1.f);
      }
    }
  }
}

}  // namespace

#define MI_ATT_SWITCH(NK2, LAUNCH)                                                                       \
  switch (NK2) {                                                                                         \
    case 1: LAUNCH(1); break;                                                                            \
    case 2: LAUNCH(2); break;                                                                            \
    case 3: LAUNCH(3); break;                                                                            \
    case 4: LAUNCH(4); break;                                                                            \
    case 5: LAUNCH(5); break;                                                                            \
    case 6: LAUNCH(6); break;                                                                            \
    case 7: LAUNCH(7); break;                                                                            \
    case 8: LAUNCH(8); break;                                                                            \
    default: return (int)hipErrorInvalidValue;                                                          \
  }

MI_API int mi_attn_max_seq() { return 256; }

static int g_att_waves = 0;
static int att_waves() {
  if (!g_att_waves) {
    const char* e = std::getenv("MI355X_DP_ATT_WAVES");
    g_att_waves = (e && e[0] == '4') ? 4 : 8;
  }
  return g_att_waves;
}

static int g_att_rot = -1;
static int att_rot() {
  if (g_att_rot < 0) {
    const char* e = std::getenv("MI355X_DP_ATT_ROTATE");
    g_att_rot = (e && e[0] == '1') ? 3 : 0;
  }
  return g_att_rot;
}

MI_API int mi_set_att_rotate(int on) {
  g_att_rot = on ? 3 : 0;
  return 0;
}

// backward workgroup size in waves (4 or 8): A/B runs in one process
MI_API int mi_set_att_waves(int w) {
  g_att_waves = w == 4 ? 4 : 8;
  return 0;
}

static int g_att_fwd_waves = 0;
static int att_fwd_waves() {
  if (!g_att_fwd_waves) {
    const char* e = std::getenv("MI355X_DP_ATT_FWD_WAVES");
    g_att_fwd_waves = (e && e[0] == '4') ? 4 : 8;
  }
  return g_att_fwd_waves;
}

// forward workgroup size in waves: 8 (online softmax over key chunks, default) or 4 (A/B)
MI_API int mi_set_att_fwd_waves(int w) {
  g_att_fwd_waves = w == 4 ? 4 : 8;
  return 0;
}

// qkv [B*T][3*H*64] bf16 (q | k | v, heads contiguous), o [B*T][H*64] bf16, lse [B*H][T] fp32
MI_API int mi_attn_fwd(const void* qkv, void* o, float* lse, int B, int T, int H, float scale, hipStream_t st) {
  if (T <= 0 || T > 256 || B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const float sl2 = scale * LOG2E;
  if (att_fwd_waves() == 8) {
#define L(N)                                                                                             \
  hipLaunchKernelGGL((attn_fwd8_kernel<N>), dim3(B * H), dim3(512), 0, st, (const bf16_t*)qkv, (bf16_t*)o, lse, T, \
                     H, sl2)
    MI_ATT_SWITCH((T + 31) / 32, L)
#undef L
    return (int)hipGetLastError();
  }
  // forward: 4 waves (its 14 score tiles per q tile need ~210 VGPRs: 2 waves per SIMD)
#define L(N)                                                                                             \
  hipLaunchKernelGGL((attn_fwd_kernel<N, 4>), dim3(B * H), dim3(256), 0, st, (const bf16_t*)qkv, (bf16_t*)o, \
                     lse, T, H, sl2, att_rot())
  MI_ATT_SWITCH((T + 31) / 32, L)
#undef L
  return (int)hipGetLastError();
}

static int g_att_fused = -1;
static int att_fused() {
  if (g_att_fused < 0) {
    const char* e = std::getenv("MI355X_DP_ATT_FUSED_BWD");
    g_att_fused = (e && e[0] == '0') ? 0 : 1;
  }
  return g_att_fused;
}

// backward schedule: 1 = one fused kernel (default), 0 = the dQ and dK/dV kernels (A/B runs)
MI_API int mi_set_att_fused_bwd(int on) {
  g_att_fused = on ? 1 : 0;
  return 0;
}

// dout [B*T][H*64]; dqkv [B*T][3*H*64] fully written; dvec [B*H][T] fp32 scratch (two-kernel path)
MI_API int mi_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse, float* dvec, void* dqkv,
                       int B, int T, int H, float scale, hipStream_t st) {
  if (T <= 0 || T > 256 || B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const float sl2 = scale * LOG2E;
  if (att_fused() && T <= 224) {  // 2 x 66 KB of LDS per CU at T <= 224
#define L(N)                                                                                             \
  hipLaunchKernelGGL((attn_bwd_fused_kernel<N>), dim3(B * H), dim3(512), 0, st, (const bf16_t*)qkv,        \
                     (const bf16_t*)o, (const bf16_t*)dout, lse, (bf16_t*)dqkv, T, H, sl2, scale)
    MI_ATT_SWITCH((T + 31) / 32, L)
#undef L
    return (int)hipGetLastError();
  }
#define L(N)                                                                                             \
  if (att_waves() == 8)                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<N, 8>), dim3(B * H), dim3(512), 0, st, (const bf16_t*)qkv,    \
                       (const bf16_t*)o, (const bf16_t*)dout, lse, dvec, (bf16_t*)dqkv, T, H, sl2, scale, att_rot()); \
  else                                                                                                   \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<N, 4>), dim3(B * H), dim3(256), 0, st, (const bf16_t*)qkv,    \
                       (const bf16_t*)o, (const bf16_t*)dout, lse, dvec, (bf16_t*)dqkv, T, H, sl2, scale,  \
                       att_rot())
  MI_ATT_SWITCH((T + 31) / 32, L)
#undef L
#define L(N)                                                                                             \
  if (att_waves() == 8)                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<N, 8>), dim3(B * H), dim3(512), 0, st, (const bf16_t*)qkv,   \
                       (const bf16_t*)dout, lse, dvec, (bf16_t*)dqkv, T, H, sl2, scale, att_rot());       \
  else                                                                                                   \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<N, 4>), dim3(B * H), dim3(256), 0, st, (const bf16_t*)qkv,   \
                       (const bf16_t*)dout, lse, dvec, (bf16_t*)dqkv, T, H, sl2, scale, att_rot())
  MI_ATT_SWITCH((T + 31) / 32, L)
#undef L
  return (int)hipGetLastError();
}
