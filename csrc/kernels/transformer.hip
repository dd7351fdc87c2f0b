// Transformer (ViT-B/16) support kernels for gfx950: LayerNorm forward / backward with the
// residual-gradient add fused, and the bias-gradient column reduction.  All bf16 activations,
// fp32 statistics / parameters / gradients.  The GEMMs themselves (QKV, projections, MLP with
// fused GELU and residual epilogues) are the MFMA kernels of gemm_conv.hip.
#include "common.h"
#include <map>
#include <mutex>
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int LN_MAXV = 8;  // 4-element (8-byte) vectors per lane: D <= 64 * 4 * 8 = 2048
constexpr int kLnReplicas = 32;  // LayerNorm parameter-gradient replicas (0: atomics straight into dw / db)
constexpr int kLnBwdRW = 2;      // LayerNorm backward rows in flight per wave (D <= 1024)

__device__ __forceinline__ void load4(const bf16_t* p, float* f) {
  const uint2 v = *(const uint2*)p;
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}

__device__ __forceinline__ void store4(bf16_t* p, const float* f) {
  *(uint2*)p = make_uint2(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]));
}

// One wave per row; lane owns 4-element vectors v = lane + 64 i (coalesced 512-B wave accesses).
// y = (x - mean) * rstd * w + b; the row stays in registers between the two reduction passes.
template <int LN_V>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = D >> 2;
  const bf16_t* xr = x + (size_t)row * D;
  // every load of the row (x, and the affine parameters the store loop needs) issued up front,
  // branch-free (chunks past D read a clamped address and are discarded): one memory latency
  // per row instead of one for x and another for w / b after the reductions
  float v[LN_V][4];
  float4 wv[LN_V], bv[LN_V];
#pragma unroll
  for (int i = 0; i < LN_V; ++i) {
    const int c = min(lane + 64 * i, nv - 1);
    load4(xr + 4 * c, v[i]);
    wv[i] = *(const float4*)(w + 4 * c);
    bv[i] = *(const float4*)(b + 4 * c);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_V; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_V; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
  bf16_t* yr = y + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < LN_V; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      float o[4] = {(v[i][0] - mean) * rstd * wv[i].x + bv[i].x, (v[i][1] - mean) * rstd * wv[i].y + bv[i].y,
                    (v[i][2] - mean) * rstd * wv[i].z + bv[i].z, (v[i][3] - mean) * rstd * wv[i].w + bv[i].w};
      store4(yr + 4 * c, o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// dx = dres + rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
// dw += sum_rows dy * xhat, db += sum_rows dy: per-lane register partials over the rows this
// wave visits (grid-stride), reduced across the block's 4 waves in LDS, then one atomic per column
// into replica (block mod R) of a [R][2][D] workspace -- every block of a resident-sized grid (768
// at D = 768) adding into the same 6 KB of dw / db serialised the kernel's tail on atomic
// contention (MI355X_MICROARCH.md: one shared row ~14x slower); ln_rep_reduce_kernel then sums the
// R replicas into dw / db and re-zeroes them.  rep == nullptr: atomics straight into dw / db.
template <int LN_V>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                     float* __restrict__ dw, float* __restrict__ db, int M, int D,
                                                     float* __restrict__ rep, int R) {
  extern __shared__ float red[];  // [4][D]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = D >> 2;
  float pw[LN_V][4], pb[LN_V][4];
#pragma unroll
  for (int i = 0; i < LN_V; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) { pw[i][e] = 0.f; pb[i][e] = 0.f; }

  // A wave owns RW adjacent rows per iteration and issues every load of them (dy, x and the
  // residual gradient, kept packed) before the first cross-lane reduction.  The loads are
  // branch-free -- rows past M and chunks past D read a clamped in-range address and are
  // discarded -- so all of them are in flight together: issued under `if`s, the compiler put a
  // vmcnt wait between every group and the row's ~20 loads paid their latency one group at a
  // time (3.4 TB/s at D = 768).  The weight chunks are loaded once, before the row loop.
  constexpr int RW = LN_V <= 4 ? kLnBwdRW : 1;
  float wr[LN_V][4];
#pragma unroll
  for (int i = 0; i < LN_V; ++i) {
    const int c = min(lane + 64 * i, nv - 1);
    const float4 wq = *(const float4*)(w + 4 * c);
    wr[i][0] = wq.x; wr[i][1] = wq.y; wr[i][2] = wq.z; wr[i][3] = wq.w;
  }
  const bf16_t* rsrc = dres ? dres : dy;  // no residual gradient: loaded, then ignored
  for (int row0 = (blockIdx.x * 4 + wv) * RW; row0 < M; row0 += gridDim.x * 4 * RW) {
    uint2 qd[RW][LN_V], qx[RW][LN_V], qr[RW][LN_V];
    float mean[RW], rstd[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const size_t row = (size_t)min(row0 + r, M - 1);
      mean[r] = mean_in[row];
      rstd[r] = rstd_in[row];
#pragma unroll
      for (int i = 0; i < LN_V; ++i) {
        const int c = min(lane + 64 * i, nv - 1);
        qd[r][i] = *(const uint2*)(dy + row * D + 4 * c);
        qx[r][i] = *(const uint2*)(x + row * D + 4 * c);
        qr[r][i] = *(const uint2*)(rsrc + row * D + 4 * c);
      }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int row = row0 + r;
      if (row >= M) break;
      float xh[LN_V][4], g[LN_V][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < LN_V; ++i) {
        const int c = lane + 64 * i;
        if (c < nv) {
          float d[4];
          load4((const bf16_t*)&qd[r][i], d);
          load4((const bf16_t*)&qx[r][i], xh[i]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            xh[i][e] = (xh[i][e] - mean[r]) * rstd[r];
            g[i][e] = d[e] * wr[i][e];
            s1 += g[i][e];
            s2 += g[i][e] * xh[i][e];
            pw[i][e] += d[e] * xh[i][e];
            pb[i][e] += d[e];
          }
        }
      }
      const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
      bf16_t* dxr = dx + (size_t)row * D;
#pragma unroll
      for (int i = 0; i < LN_V; ++i) {
        const int c = lane + 64 * i;
        if (c < nv) {
          float o[4], rv[4] = {0.f, 0.f, 0.f, 0.f};
          if (dres) load4((const bf16_t*)&qr[r][i], rv);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = rv[e] + rstd[r] * (g[i][e] - m1 - xh[i][e] * m2);
          store4(dxr + 4 * c, o);
        }
      }
    }
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();
#pragma unroll
    for (int i = 0; i < LN_V; ++i) {
      const int c = lane + 64 * i;
      if (c < nv) {
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wv * D + 4 * c + e] = pass ? pb[i][e] : pw[i][e];
      }
    }
    __syncthreads();
    float* dst = rep ? rep + ((size_t)(blockIdx.x % R) * 2 + pass) * D : (pass ? db : dw);
    for (int col = threadIdx.x; col < D; col += 256)
      atomicAdd(dst + col, red[col] + red[D + col] + red[2 * D + col] + red[3 * D + col]);
  }
}

// The same backward with 16-byte accesses, for D % 256 == 0 (D = 256 or 768): a row is one
// HALF-wave -- lane hl = lane & 31 of half hf owns the 8-element chunks hl + 32 i -- so a wave works
// on 2 rows at a time (RW16 row pairs in flight), every load / store is a 16-byte access (half the
// memory instructions of the 8-byte, full-wave-row kernel), and the row reductions are 5-step
// half-wave xor shuffles.  dw / db partials as ln_bwd_kernel, over 8 half-waves per block.
constexpr int kLn16RW = 2;  // row pairs in flight per wave

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int V>
__global__ __launch_bounds__(256) void ln_bwd16_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                       const float* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       float* __restrict__ dw, float* __restrict__ db, int M, int D,
                                                       float* __restrict__ rep, int R) {
  extern __shared__ float red[];  // [8 half-waves][D]
  constexpr int RW = kLn16RW;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hf = lane >> 5, hl = lane & 31;
  float pw[V][8], pb[V][8], wr[V][8];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * (hl + 32 * i);
    const float4 a = *(const float4*)(w + c), b = *(const float4*)(w + c + 4);
    wr[i][0] = a.x; wr[i][1] = a.y; wr[i][2] = a.z; wr[i][3] = a.w;
    wr[i][4] = b.x; wr[i][5] = b.y; wr[i][6] = b.z; wr[i][7] = b.w;
#pragma unroll
    for (int e = 0; e < 8; ++e) { pw[i][e] = 0.f; pb[i][e] = 0.f; }
  }
  const bf16_t* rsrc = dres ? dres : dy;  // no residual gradient: loaded, then ignored
  const float invD = 1.f / (float)D;
  for (int row0 = (blockIdx.x * 4 + wv) * 2 * RW; row0 < M; row0 += gridDim.x * 8 * RW) {
    // every load of the RW row pairs first (rows past M read row M - 1 and are discarded)
    uint4 qd[RW][V], qx[RW][V], qr[RW][V];
    float mean[RW], rstd[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const size_t row = (size_t)min(row0 + 2 * r + hf, M - 1);
      mean[r] = mean_in[row];
      rstd[r] = rstd_in[row];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const size_t off = row * D + 8 * (hl + 32 * i);
        qd[r][i] = *(const uint4*)(dy + off);
        qx[r][i] = *(const uint4*)(x + off);
        qr[r][i] = *(const uint4*)(rsrc + off);
      }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int row = row0 + 2 * r + hf;
      const bool live = row < M;  // both halves take part in the shuffles; only live rows count
      float xh[V][8], g[V][8];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        float d[8];
        unpack8(qd[r][i], d);
        unpack8(qx[r][i], xh[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[i][e] = (xh[i][e] - mean[r]) * rstd[r];
          g[i][e] = d[e] * wr[i][e];
          s1 += g[i][e];
          s2 += g[i][e] * xh[i][e];
          if (live) {
            pw[i][e] += d[e] * xh[i][e];
            pb[i][e] += d[e];
          }
        }
      }
      const float m1 = half_sum(s1) * invD, m2 = half_sum(s2) * invD;
      if (live) {
        bf16_t* dxr = dx + (size_t)row * D;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          float o[8], rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if (dres) unpack8(qr[r][i], rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = rv[e] + rstd[r] * (g[i][e] - m1 - xh[i][e] * m2);
          *(uint4*)(dxr + 8 * (hl + 32 * i)) = pack8(o);
        }
      }
    }
  }
  const int hw = wv * 2 + hf;  // half-wave index 0..7
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();
#pragma unroll
    for (int i = 0; i < V; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[hw * D + 8 * (hl + 32 * i) + e] = pass ? pb[i][e] : pw[i][e];
    __syncthreads();
    float* dst = rep ? rep + ((size_t)(blockIdx.x % R) * 2 + pass) * D : (pass ? db : dw);
    for (int col = threadIdx.x; col < D; col += 256) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += red[k * D + col];
      atomicAdd(dst + col, t);
    }
  }
}

// ---------------------------------------------------------------- ViT token embedding
// out[n][0][:] = cls + pos[0], out[n][1 + p][:] = patches[n][p][:] + pos[1 + p]: the class-token
// concatenation and the position-embedding add in one pass (fp32 math, one bf16 rounding).
// 8 channels per thread; T = tokens (patches + 1), D % 8 == 0.
__global__ __launch_bounds__(256) void vit_embed_fwd_kernel(const bf16_t* __restrict__ patches,
                                                            const float* __restrict__ cls,
                                                            const float* __restrict__ pos, bf16_t* __restrict__ out,
                                                            int64_t total8, int T, int D) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const int64_t e = i * 8;
  const int64_t per = (int64_t)T * D;
  const int64_t n = e / per;
  const int64_t r = e - n * per;  // token * D + channel
  const int t = (int)(r / D), c = (int)(r - (int64_t)t * D);
  float f[8];
  if (t == 0) {
    *(float4*)&f[0] = *(const float4*)(cls + c);
    *(float4*)&f[4] = *(const float4*)(cls + c + 4);
  } else {
    unpack8(*(const uint4*)(patches + (n * (T - 1) + (t - 1)) * D + c), f);
  }
  const float4 p0 = *(const float4*)(pos + r), p1 = *(const float4*)(pos + r + 4);
  f[0] += p0.x; f[1] += p0.y; f[2] += p0.z; f[3] += p0.w;
  f[4] += p1.x; f[5] += p1.y; f[6] += p1.z; f[7] += p1.w;
  *(uint4*)(out + e) = pack8(f);
}

// Patchify for a stride = kernel = p patch embedding: x NHWC [N][H][W][Cs] bf16 -> out [N * (H/p) *
// (W/p)][p * p * C] bf16, row = patch, columns in (r, s, c) order -- the flat engine's conv weight
// layout [K][R][S][C] -- for the C <= Cs real channels.  The patch embedding is then one plain GEMM
// with K = p * p * C (768 for ViT-B/16) instead of an 8-channel-padded implicit-GEMM conv (2048).
// One thread per 16-byte output chunk (8 columns, from up to 4 input pixels).
__global__ __launch_bounds__(256) void vit_patchify_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                           int64_t chunks, int H, int W, int Cs, int C, int p,
                                                           int Qn, int PQ) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= chunks) return;
  const int row_len = p * p * C;
  const int64_t e0 = i * 8;
  const int64_t patch = e0 / row_len;
  const int col0 = (int)(e0 - patch * row_len);
  const int n = (int)(patch / PQ), pq = (int)(patch - (int64_t)n * PQ);
  const int py = pq / Qn, px = pq - (pq / Qn) * Qn;
  const bf16_t* img = x + (size_t)n * H * W * Cs;
  bf16_t v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int col = col0 + q;
    const int pix = col / C, c = col - pix * C;
    const int r = pix / p, sx = pix - r * p;
    v[q] = img[((size_t)(py * p + r) * W + (px * p + sx)) * Cs + c];
  }
  uint4 o;
  o.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16); o.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
  o.z = (uint32_t)v[4] | ((uint32_t)v[5] << 16); o.w = (uint32_t)v[6] | ((uint32_t)v[7] << 16);
  *(uint4*)(out + e0) = o;
}

// backward, pass 1: dpatches[n][p] = dout[n][1 + p] (the patch conv's dense output gradient) and
// per image-group partial sums part[g][t * D + c] = sum over the group's images of dout[n][t][c]
// (fixed order).  Block (x, g): 256 threads x 8 channels of the T * D positions, images
// [g * per_g, (g + 1) * per_g).
__global__ __launch_bounds__(256) void vit_embed_bwd_kernel(const bf16_t* __restrict__ dout,
                                                            bf16_t* __restrict__ dpatches, float* __restrict__ part,
                                                            int N, int T, int D, int per_g) {
  const int64_t TD = (int64_t)T * D;
  const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (r >= TD) return;
  const int t = (int)(r / D);
  const int n0 = blockIdx.y * per_g, n1 = min(N, n0 + per_g);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int n = n0; n < n1; n += 4) {  // 4 images' loads in flight, summed in image order
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = n + u < n1 ? *(const uint4*)(dout + (n + u) * TD + r) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (n + u >= n1) break;
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += f[q];
      if (t > 0) *(uint4*)(dpatches + (n + u) * (TD - D) + (r - D)) = v[u];
    }
  }
  float* o = part + (size_t)blockIdx.y * TD + r;
  *(float4*)o = make_float4(s[0], s[1], s[2], s[3]);
  *(float4*)(o + 4) = make_float4(s[4], s[5], s[6], s[7]);
}

// pass 2: dpos[r] += sum_g part[g][r]; dcls[c] += the same sum for token 0 (the class token's
// gradient is the position embedding's row 0)
__global__ __launch_bounds__(256) void vit_embed_bwd_sum_kernel(const float* __restrict__ part, int G, int64_t TD,
                                                                int D, float* __restrict__ dpos,
                                                                float* __restrict__ dcls) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= TD) return;
  float s = 0.f;
  for (int g = 0; g < G; g += 8) {  // 8 partial rows' loads in flight, summed in order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = g + u < G ? part[(size_t)(g + u) * TD + r] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  if (dpos) dpos[r] += s;
  if (dcls && r < D) dcls[r] += s;
}

// dw[c] += sum_r rep[r][0][c], db[c] += sum_r rep[r][1][c] (fixed order), replicas zeroed again
__global__ __launch_bounds__(256) void ln_rep_reduce_kernel(float* __restrict__ rep, int R, int D,
                                                            float* __restrict__ dw, float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * D) return;
  const int pass = i / D, col = i - pass * D;
  constexpr int RMAX = kLnReplicas > 0 ? kLnReplicas : 1;
  float v[RMAX];  // every replica's load in flight at once, then the fixed-order sum
#pragma unroll
  for (int r = 0; r < RMAX; ++r) v[r] = r < R ? rep[((size_t)r * 2 + pass) * D + col] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) s += v[r];
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
    if (r < R) rep[((size_t)r * 2 + pass) * D + col] = 0.f;
  float* dst = pass ? db : dw;
  if (dst) dst[col] += s;
}

// out[n] += sum_m X[m][n] (bf16 X, row stride ld): lane owns an 8-column chunk, the block's 4
// waves split the rows of a row slab, LDS reduction, one fp32 atomic per column per block.
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ X, float* __restrict__ out,
                                                     int M, int N, int ld, int rows_per_block) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = (blockIdx.x * 64 + lane) * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (n < N) {
    for (int m = r0 + wv; m < r1; m += 4) {
      float f[8];
      unpack8(*(const uint4*)(X + (size_t)m * ld + n), f);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += f[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[wv][lane * 8 + q] = acc[q];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int col = blockIdx.x * 512 + c;
    if (col < N) atomicAdd(out + col, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
  }
}

// [LN_REPLICAS][2][D] zeroed fp32 replicas of the LayerNorm parameter gradients, one per (device,
// stream), grown on demand (the first call of a shape allocates and zeroes: never inside a graph
// capture -- a warm-up step runs first); ln_rep_reduce_kernel leaves them zeroed for the next call.
constexpr int LN_REPLICAS = kLnReplicas;
struct LnRep { float* p = nullptr; int D = 0; };
static std::mutex g_lnrep_mu;
static std::map<std::pair<int, hipStream_t>, LnRep> g_lnrep;
static float* ln_rep_workspace(int D, hipStream_t st) {
  if (LN_REPLICAS <= 0) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_lnrep_mu);
  LnRep& w = g_lnrep[{dev, st}];
  if (w.D < D) {
    if (mi_stream_capturing(st)) {  // common.h: never allocate inside a capture
      mi_ws_capture_warn("LayerNorm replica");
      return nullptr;  // -> the replica-free parameter-gradient path
    }
    float* p = nullptr;
    const size_t bytes = sizeof(float) * LN_REPLICAS * 2 * (size_t)D;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, bytes) != hipSuccess) return nullptr;
    (void)hipDeviceSynchronize();  // the zeroing is complete before any stream uses the replicas
    mi_ws_retire(w.p);       // graphs captured earlier may still replay into it (common.h)
    w.p = p;
    w.D = D;
  }
  return w.p;
}

}  // namespace

// test hook (tests/test_graph_workspaces_gpu.py): grow this stream's LayerNorm replicas to width D
MI_API int mi_ln_ws_reserve(int D, hipStream_t st) { return ln_rep_workspace(D, st) ? 0 : 1; }

MI_API int mi_layernorm_fwd(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                            int M, int D, float eps, hipStream_t st) {
  if (D % 4 != 0 || D > 64 * 4 * LN_MAXV || M <= 0) return (int)hipErrorInvalidValue;
#define MI_LN_FWD(V)                                                                                    \
  case V:                                                                                               \
    hipLaunchKernelGGL(ln_fwd_kernel<V>, dim3(cdiv(M, 4)), dim3(256), 0, st, (const bf16_t*)x, w, b,     \
                       (bf16_t*)y, mean, rstd, M, D, eps);                                              \
    break;
  switch (cdiv(D, 256)) {
    MI_LN_FWD(1) MI_LN_FWD(2) MI_LN_FWD(3) MI_LN_FWD(4) MI_LN_FWD(5) MI_LN_FWD(6) MI_LN_FWD(7) MI_LN_FWD(8)
  }
#undef MI_LN_FWD
  return (int)hipGetLastError();
}

MI_API int mi_layernorm_bwd(const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                            const void* dres, void* dx, float* dw, float* db, int M, int D, hipStream_t st) {
  if (D % 4 != 0 || D > 64 * 4 * LN_MAXV || M <= 0) return (int)hipErrorInvalidValue;
  // Grid-stride kernel: launch at most one resident wave of blocks (CUs x occupancy, per LN_V
  // instantiation), so no block waits for a slot while the others already stride past its rows.
  // MI355X_DP_LN_BWD_BLOCKS overrides (rows in flight vs dW/dB atomics per block).
  static int env_blocks = -2;
  // resident-block count per (device, dynamic LDS bytes): the occupancy depends on the LDS size
  // (4 * D floats), which differs between D values of one LN_V instantiation (e.g. 640 vs 768)
  static std::mutex res_mu;
  static std::map<std::pair<int, size_t>, int> resident;
  if (env_blocks == -2) {
    const char* e = std::getenv("MI355X_DP_LN_BWD_BLOCKS");
    env_blocks = e ? std::max(1, std::atoi(e)) : -1;
  }
  const size_t lds = (size_t)4 * D * sizeof(float);
  const int nvec = cdiv(D, 256);
  auto cap = [&](const void* fn) {
    if (env_blocks > 0) return env_blocks;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(res_mu);
    auto it = resident.find({dev, lds});
    if (it != resident.end()) return it->second;
    int cus = 256, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu <= 0) per_cu = 2;
    resident[{dev, lds}] = cus * per_cu;
    return cus * per_cu;
  };
  const int rw = nvec <= 4 ? kLnBwdRW : 1;
  float* rep = (dw && db) ? ln_rep_workspace(D, st) : nullptr;
  const int R = LN_REPLICAS;
  static int ln16 = -1;  // MI355X_DP_LN_BWD16=0: always the full-wave-row kernel (A/B)
  if (ln16 < 0) {
    const char* e = std::getenv("MI355X_DP_LN_BWD16");
    ln16 = (e && e[0] == '0') ? 0 : 1;
  }
  // the 16-byte kernel at D = 256 / 768 (the V = 2 instantiation spills, V = 4 runs one wave per SIMD)
  if (ln16 && D % 256 == 0 && (nvec == 1 || nvec == 3) && dw && db) {
    const size_t lds16 = (size_t)8 * D * sizeof(float);
    static std::map<std::pair<int, size_t>, int> resident16;
    auto cap16 = [&](const void* fn) {
      if (env_blocks > 0) return env_blocks;
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
      std::lock_guard<std::mutex> lk(res_mu);
      auto it = resident16.find({dev, lds16});
      if (it != resident16.end()) return it->second;
      int cus = 256, per_cu = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds16) != hipSuccess || per_cu <= 0)
        per_cu = 2;
      resident16[{dev, lds16}] = cus * per_cu;
      return cus * per_cu;
    };
#define MI_LN_BWD16_CASE(V)                                                                              \
  case V:                                                                                                \
    hipLaunchKernelGGL(ln_bwd16_kernel<V>,                                                               \
                       dim3(min(cdiv(M, 8 * kLn16RW), cap16((const void*)ln_bwd16_kernel<V>))), dim3(256), \
                       lds16, st, (const bf16_t*)dy, (const bf16_t*)x, w, mean, rstd, (const bf16_t*)dres,    \
                       (bf16_t*)dx, dw, db, M, D, rep, R);                                               \
    break;
    switch (nvec) { MI_LN_BWD16_CASE(1) MI_LN_BWD16_CASE(3) }
#undef MI_LN_BWD16_CASE
    // a separate reduce: in the last-arriving block the same 2 x D x 32 replica reads ran ~10x
    // longer than this 6-block launch (ViT-B/16 -7 %, profiles/raw/r4_l38_*)
    if (rep) hipLaunchKernelGGL(ln_rep_reduce_kernel, dim3(cdiv(2 * D, 256)), dim3(256), 0, st, rep, R, D, dw, db);
    return (int)hipGetLastError();
  }
#define MI_LN_BWD(V)                                                                                    \
  case V:                                                                                               \
    hipLaunchKernelGGL(ln_bwd_kernel<V>, dim3(min(cdiv(M, 4 * rw), cap((const void*)ln_bwd_kernel<V>))),  \
                       dim3(256), lds, st, (const bf16_t*)dy,                                            \
                       (const bf16_t*)x, w, mean, rstd, (const bf16_t*)dres, (bf16_t*)dx, dw, db, M, D,  \
                       rep, R);                                                                          \
    break;
  switch (cdiv(D, 256)) {
    MI_LN_BWD(1) MI_LN_BWD(2) MI_LN_BWD(3) MI_LN_BWD(4) MI_LN_BWD(5) MI_LN_BWD(6) MI_LN_BWD(7) MI_LN_BWD(8)
  }
#undef MI_LN_BWD
  if (rep) hipLaunchKernelGGL(ln_rep_reduce_kernel, dim3(cdiv(2 * D, 256)), dim3(256), 0, st, rep, R, D, dw, db);
  return (int)hipGetLastError();
}

MI_API int mi_vit_patchify(const void* x, void* out, int N, int H, int W, int Cs, int C, int p, hipStream_t st) {
  if (p <= 0 || H % p || W % p || C <= 0 || C > Cs || (p * p * C) % 8 != 0) return (int)hipErrorInvalidValue;
  const int Pn = H / p, Qn = W / p;
  const int64_t chunks = (int64_t)N * Pn * Qn * p * p * C / 8;
  hipLaunchKernelGGL(vit_patchify_kernel, dim3((unsigned)cdiv(chunks, 256)), dim3(256), 0, st, (const bf16_t*)x,
                     (bf16_t*)out, chunks, H, W, Cs, C, p, Qn, Pn * Qn);
  return (int)hipGetLastError();
}

// ViT embedding: out [N][T][D] bf16 from patches [N][T-1][D] bf16, cls [D] and pos [T][D] fp32.
MI_API int mi_vit_embed_fwd(const void* patches, const float* cls, const float* pos, void* out, int N, int T, int D,
                            hipStream_t st) {
  if (D % 8 != 0 || N <= 0 || T < 2) return (int)hipErrorInvalidValue;
  const int64_t total8 = (int64_t)N * T * D / 8;
  hipLaunchKernelGGL(vit_embed_fwd_kernel, dim3((unsigned)cdiv(total8, 256)), dim3(256), 0, st,
                     (const bf16_t*)patches, cls, pos, (bf16_t*)out, total8, T, D);
  return (int)hipGetLastError();
}

// backward: dpatches [N][T-1][D] bf16 = dout[:, 1:], dpos [T][D] += sum_n dout[n], dcls [D] += sum_n
// dout[n][0] (fp32, fixed-order sums; dpos / dcls may be null).  part: fp32 workspace of
// mi_vit_embed_bwd_part_floats(N, T, D) floats.
MI_API int64_t mi_vit_embed_bwd_part_floats(int N, int T, int D) {
  const int G = std::min(N, 16);
  return (int64_t)G * T * D;
}

MI_API int mi_vit_embed_bwd(const void* dout, void* dpatches, float* dpos, float* dcls, float* part, int N, int T,
                            int D, hipStream_t st) {
  if (D % 8 != 0 || N <= 0 || T < 2) return (int)hipErrorInvalidValue;
  const int G = std::min(N, 16), per_g = cdiv(N, G);
  const int G_used = cdiv(N, per_g);
  const int64_t TD = (int64_t)T * D;
  hipLaunchKernelGGL(vit_embed_bwd_kernel, dim3((unsigned)cdiv(TD / 8, 256), G_used), dim3(256), 0, st,
                     (const bf16_t*)dout, (bf16_t*)dpatches, part, N, T, D, per_g);
  if (dpos || dcls)
    hipLaunchKernelGGL(vit_embed_bwd_sum_kernel, dim3((unsigned)cdiv(TD, 256)), dim3(256), 0, st, part, G_used,
                       TD, D, dpos, dcls);
  return (int)hipGetLastError();
}

// fp32 X [M][N] -> bf16 Y (the GEMM operand) and, when out != nullptr, out[n] += sum_m X[m][n] from
// the fp32 values (a classifier head's bias gradient from fp32 logit gradients): one pass, same
// blocking as colsum_kernel.
__global__ __launch_bounds__(256) void cast_colsum_f32_kernel(const float* __restrict__ X, bf16_t* __restrict__ Y,
                                                              float* __restrict__ out, int M, int N,
                                                              int rows_per_block) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = (blockIdx.x * 64 + lane) * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (n < N) {
    for (int m = r0 + wv; m < r1; m += 4) {
      const float4 a = *(const float4*)(X + (size_t)m * N + n), b = *(const float4*)(X + (size_t)m * N + n + 4);
      const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      *(uint4*)(Y + (size_t)m * N + n) = pack8(f);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += f[q];
    }
  }
  if (!out) return;
#pragma unroll
  for (int q = 0; q < 8; ++q) red[wv][lane * 8 + q] = acc[q];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int col = blockIdx.x * 512 + c;
    if (col < N) atomicAdd(out + col, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
  }
}

MI_API int mi_cast_colsum_f32(const float* X, void* Y, float* out, int M, int N, hipStream_t st) {
  if (N % 8 != 0 || M <= 0) return (int)hipErrorInvalidValue;
  const int bx = cdiv(N, 512);
  int by = max(1, min(cdiv(M, 64), 2048 / bx));
  const int rpb = cdiv(M, by);
  by = cdiv(M, rpb);
  hipLaunchKernelGGL(cast_colsum_f32_kernel, dim3(bx, by), dim3(256), 0, st, X, (bf16_t*)Y, out, M, N, rpb);
  return (int)hipGetLastError();
}

MI_API int mi_colsum_bf16(const void* X, float* out, int M, int N, int ld, hipStream_t st) {
  if (N % 8 != 0 || ld % 8 != 0 || M <= 0) return (int)hipErrorInvalidValue;
  const int bx = cdiv(N, 512);
  int by = max(1, min(cdiv(M, 64), 2048 / bx));
  const int rpb = cdiv(M, by);
  by = cdiv(M, rpb);
  hipLaunchKernelGGL(colsum_kernel, dim3(bx, by), dim3(256), 0, st, (const bf16_t*)X, out, M, N, ld, rpb);
  return (int)hipGetLastError();
}
