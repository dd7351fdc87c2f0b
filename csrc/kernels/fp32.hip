// fp32 compute mode for the reference workload: the reference trains in fp32
// (cifar10-distributed-smddp-gpu.py:145-158, PyTorch fp32 on A100; nb2:2611-2612), so a like-for-like
// comparison of its job needs an fp32 path.  gfx950 has no xf32/TF32: the matrix core's f32-operand
// form v_mfma_f32_16x16x4_f32 computes exact fp32 products with fp32 accumulation (an fmaf chain,
// bitwise) at the fp32 vector rate -- that is the engine here.  Selected by
// MI355X_DP_COMPUTE_DTYPE=fp32 (mi355x_dp/ops/fp32.py); NHWC fp32 activations, conv weights read as
// [K][R][S][C] fp32 (the flat engine's master layout), channels a multiple of 4 (16-byte vectors;
// the 3-channel stem input is zero-padded to 4).
//
//   * conv_f32_kernel<MODE>: one implicit-GEMM tile kernel for the forward (MODE 0), data gradient
//     (1) and weight gradient (2): 64x64 output tiles, 4 waves of 32x32 (2x2 MFMA 16x16x4 tiles),
//     16-deep k-tiles staged through LDS (k-major, 16-float row skew: conflict-free fragment reads),
//     next k-tile's global loads issued before the current one's MFMAs; operands gathered on the fly
//     (padding / stride / parity by bounds checks, no im2col); small grids split K over blockIdx.z
//     into an fp32 slab summed in split order by a second launch (deterministic).
//   * BatchNorm train forward / backward with fused ReLU and residual (two-stage deterministic
//     reductions, fp64 finalize), max pool with a 1-byte arg-max tap and a gather backward (no
//     atomics), global average pool, Linear bias gradient.
#include "common.h"
#include <algorithm>

namespace {

constexpr int FT = 256;            // threads per block (4 waves)
constexpr int TM = 64, TN = 64;    // output tile
constexpr int TK = 16;             // k-tile depth
constexpr int LDS_LD = TM + 16;    // row stride of the k-major LDS tiles (floats)

struct F32Geom {
  int Nb, H, W, C, K, R, S, stride, pad, P, Q;
  int M, N, Kr;  // GEMM dims of the mode
};

typedef float f32x4v __attribute__((ext_vector_type(4)));

// ---- operand gathers: one float4 per thread per k-tile, zero outside the problem
// A tile (TM rows m x TK k), B tile (TN cols n x TK k); `la` / `lb` say along which dimension the
// thread's 4 floats run (0: along k, 1: along m / n)
template <int MODE>
__device__ __forceinline__ float4 load_a(const float* __restrict__ a, const F32Geom& g, int m, int kk) {
  float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (MODE == 0) {  // X[n][h][w][c], m = (n,p,q), kk = (r,s,c): 4 consecutive c
    if (m >= g.M || kk >= g.Kr) return z;
    const int c = kk % g.C, rs = kk / g.C, s = rs % g.S, r = rs / g.S;
    const int q = m % g.Q, np = m / g.Q, p = np % g.P, n = np / g.P;
    const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
    if (h < 0 || h >= g.H || w < 0 || w >= g.W) return z;
    return *(const float4*)(a + (((int64_t)n * g.H + h) * g.W + w) * g.C + c);
  } else if (MODE == 1) {  // dY[n][p][q][k], m = (n,h,w), kk = (r,s,k): 4 consecutive k
    if (m >= g.M || kk >= g.Kr) return z;
    const int k = kk % g.K, rs = kk / g.K, s = rs % g.S, r = rs / g.S;
    const int w = m % g.W, nh = m / g.W, h = nh % g.H, n = nh / g.H;
    const int ph = h + g.pad - r, pw = w + g.pad - s;
    if (ph < 0 || pw < 0 || ph % g.stride || pw % g.stride) return z;
    const int p = ph / g.stride, q = pw / g.stride;
    if (p >= g.P || q >= g.Q) return z;
    return *(const float4*)(a + (((int64_t)n * g.P + p) * g.Q + q) * g.K + k);
  } else {  // dY^T: m = k_out (4 consecutive), kk = (n,p,q)
    if (m >= g.M || kk >= g.Kr) return z;
    return *(const float4*)(a + (int64_t)kk * g.K + m);
  }
}

template <int MODE>
__device__ __forceinline__ float4 load_b(const float* __restrict__ b, const F32Geom& g, int n, int kk) {
  float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (MODE == 0) {  // W[k_out][rsc]: n = k_out, 4 consecutive kk
    if (n >= g.N || kk >= g.Kr) return z;
    return *(const float4*)(b + (int64_t)n * g.Kr + kk);
  } else if (MODE == 1) {  // W[k][r][s][c]: n = c (4 consecutive), kk = (r,s,k)
    if (n >= g.N || kk >= g.Kr) return z;
    const int k = kk % g.K, rs = kk / g.K;
    return *(const float4*)(b + ((int64_t)k * g.R * g.S + rs) * g.C + n);
  } else {  // X gathered: n = (r,s,c) (4 consecutive c), kk = (n,p,q)
    if (n >= g.N || kk >= g.Kr) return z;
    const int c = n % g.C, rs = n / g.C, s = rs % g.S, r = rs / g.S;
    const int q = kk % g.Q, np = kk / g.Q, p = np % g.P, nn = np / g.P;
    const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
    if (h < 0 || h >= g.H || w < 0 || w >= g.W) return z;
    return *(const float4*)(b + (((int64_t)nn * g.H + h) * g.W + w) * g.C + c);
  }
}

// which dimension a thread's float4 runs along: A -- along k for modes 0/1, along m for mode 2;
// B -- along k for mode 0, along n for modes 1/2
template <int MODE> struct Lay {
  static constexpr bool a_along_k = MODE != 2;
  static constexpr bool b_along_k = MODE == 0;
};

__device__ __forceinline__ void tile_coord(bool along_k, int t, int& mn, int& kq) {
  if (along_k) { mn = t >> 2; kq = (t & 3) * 4; }     // 64 rows x 4 quads of k
  else { mn = (t & 15) * 4; kq = t >> 4; }             // 16 quads of rows x 16 k
}

__device__ __forceinline__ void tile_store(float (*s)[LDS_LD], bool along_k, int mn, int kq, float4 v) {
  if (along_k) {
    s[kq + 0][mn] = v.x; s[kq + 1][mn] = v.y; s[kq + 2][mn] = v.z; s[kq + 3][mn] = v.w;
  } else {
    *(float4*)&s[kq][mn] = v;
  }
}

// out (splits == 1): out[m][n] (= or +=, + bias[n]); else ws[split][m][n] partials
template <int MODE>
__global__ __launch_bounds__(FT) void conv_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ out, float* __restrict__ ws,
                                                      const float* __restrict__ bias, F32Geom g, int accumulate,
                                                      int ktiles_per_split) {
  __shared__ float As[TK][LDS_LD];
  __shared__ float Bs[TK][LDS_LD];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  const int kt_total = (g.Kr + TK - 1) / TK;
  const int kt0 = blockIdx.z * ktiles_per_split, kt1 = min(kt_total, kt0 + ktiles_per_split);
  int am, ak, bn, bk;
  tile_coord(Lay<MODE>::a_along_k, t, am, ak);
  tile_coord(Lay<MODE>::b_along_k, t, bn, bk);
  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
  if (kt0 < kt1) {
    ra = load_a<MODE>(a, g, m0 + am, kt0 * TK + ak);
    rb = load_b<MODE>(b, g, n0 + bn, kt0 * TK + bk);
  }
  for (int kt = kt0; kt < kt1; ++kt) {
    __syncthreads();  // the previous k-tile's fragment reads are done
    tile_store(As, Lay<MODE>::a_along_k, am, ak, ra);
    tile_store(Bs, Lay<MODE>::b_along_k, bn, bk, rb);
    __syncthreads();
    if (kt + 1 < kt1) {  // next k-tile in flight under this one's MFMAs
      ra = load_a<MODE>(a, g, m0 + am, (kt + 1) * TK + ak);
      rb = load_b<MODE>(b, g, n0 + bn, (kt + 1) * TK + bk);
    }
#pragma unroll
    for (int ks = 0; ks < TK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[kr][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  // C/D map: col = lane & 15, row = 4 * (lane >> 4) + r
  float* dst = ws ? ws + (int64_t)blockIdx.z * g.M * g.N : out;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        float v = acc[i][j][r];
        float* o = dst + (int64_t)m * g.N + n;
        if (ws) {
          *o = v;
        } else {
          if (bias) v += bias[n];
          *o = accumulate ? *o + v : v;
        }
      }
    }
}

// out[i] (= or +=) sum over splits of ws[s][i] in split order (+ bias[i % N])
__global__ __launch_bounds__(FT) void splitk_sum_f32_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                            const float* __restrict__ bias, int64_t MN, int N,
                                                            int splits, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)FT + threadIdx.x; i < MN; i += (int64_t)gridDim.x * FT) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += ws[(int64_t)s * MN + i];
    if (bias) v += bias[i % N];
    out[i] = accumulate ? out[i] + v : v;
  }
}

F32Geom make_f32_geom(int mode, int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad, int P,
                      int Q) {
  F32Geom g{Nb, H, W, C, K, R, S, stride, pad, P, Q, 0, 0, 0};
  if (mode == 0) { g.M = Nb * P * Q; g.N = K; g.Kr = R * S * C; }
  else if (mode == 1) { g.M = Nb * H * W; g.N = C; g.Kr = R * S * K; }
  else { g.M = K; g.N = R * S * C; g.Kr = Nb * P * Q; }
  return g;
}

int f32_splits(const F32Geom& g) {
  const int tiles = cdiv(g.M, TM) * cdiv(g.N, TN);
  const int kt = cdiv(g.Kr, TK);
  int s = 1;
  // fill the 256 CUs (>= ~512 blocks) while every split keeps >= 8 k-tiles
  while (s < 64 && tiles * s < 512 && kt / (2 * s) >= 8) s *= 2;
  return s;
}

// ----------------------------------------------------------------------- BatchNorm (fp32)
// partial slab rows [nblk][2][C]: block x covers rows [x * rpb, ..), block y a 4*tpr channel slab
__device__ __forceinline__ void slab_geom4(int C, int& tpr, int& rp) {
  tpr = min(C / 4, FT);
  rp = FT / tpr;
}

// mv (forward statistics): the sums are of x - k with k = x[rb] (the block's first row, per channel)
// and the block writes its (mean, M2) instead -- shifted sums keep E[x^2] - mean^2 from cancelling
// when |mean| >> std; the finalize merges the blocks with Chan's formula
__device__ __forceinline__ void block_reduce4(float4 s, float4 q, float* part, int C, int cb,
                                              const float* mv_x = nullptr, int mv_rb = 0, int mv_n = 0) {
  __shared__ float red[2][FT * 4];
  int tpr, rp;
  slab_geom4(C, tpr, rp);
  const int t = threadIdx.x, c4 = t % tpr, r0 = t / tpr, cw = tpr * 4;
  *(float4*)&red[0][r0 * cw + c4 * 4] = s;
  *(float4*)&red[1][r0 * cw + c4 * 4] = q;
  __syncthreads();
  for (int c = t; c < cw; c += FT) {
    float x = 0.f, y = 0.f;
    for (int r = 0; r < rp; ++r) { x += red[0][r * cw + c]; y += red[1][r * cw + c]; }
    if (mv_x && cb + c < C) {
      const float k = mv_x[(int64_t)mv_rb * C + cb + c], n = (float)mv_n;
      const float d = x / n;                 // mean of x - k
      const float m2 = fmaxf(y - x * d, 0.f);  // sum (x - k)^2 - n d^2 = sum (x - mean)^2
      x = k + d;
      y = m2;
    }
    part[(int64_t)(blockIdx.x * 2) * C + cb + c] = x;
    part[(int64_t)(blockIdx.x * 2 + 1) * C + cb + c] = y;
  }
}

// fwd: (sum x, sum x^2); bwd: (sum dz, sum dz * (x - mean)), dz = dy * [y > 0] when relu
template <bool BWD>
__global__ __launch_bounds__(FT) void bnf_stats_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       const float* __restrict__ y, const float* __restrict__ mean,
                                                       float* __restrict__ part, int M, int C, int rpb, int relu) {
  int tpr, rp;
  slab_geom4(C, tpr, rp);
  const int t = threadIdx.x, c4 = t % tpr, r0 = t / tpr;
  const int cb = blockIdx.y * tpr * 4, c = cb + c4 * 4;
  const int rb = blockIdx.x * rpb, re = min(M, rb + rpb);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  float4 mu = s;
  if (BWD) mu = *(const float4*)(mean + c);
  else if (rb < re) mu = *(const float4*)(x + (int64_t)rb * C + c);  // forward: the shift k
  for (int r = rb + r0; r < re; r += rp) {
    const int64_t off = (int64_t)r * C + c;
    float4 xv = *(const float4*)(x + off);
    if (!BWD) {
      xv.x -= mu.x; xv.y -= mu.y; xv.z -= mu.z; xv.w -= mu.w;
      s.x += xv.x; s.y += xv.y; s.z += xv.z; s.w += xv.w;
      q.x += xv.x * xv.x; q.y += xv.y * xv.y; q.z += xv.z * xv.z; q.w += xv.w * xv.w;
    } else {
      float4 d = *(const float4*)(dy + off);
      if (relu) {
        const float4 yv = *(const float4*)(y + off);
        d.x = yv.x > 0.f ? d.x : 0.f; d.y = yv.y > 0.f ? d.y : 0.f;
        d.z = yv.z > 0.f ? d.z : 0.f; d.w = yv.w > 0.f ? d.w : 0.f;
      }
      s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
      q.x += d.x * (xv.x - mu.x); q.y += d.y * (xv.y - mu.y);
      q.z += d.z * (xv.z - mu.z); q.w += d.w * (xv.w - mu.w);
    }
  }
  if (BWD) block_reduce4(s, q, part, C, cb);
  else block_reduce4(s, q, part, C, cb, x, rb, max(re - rb, 1));
}

struct BnF32Fin {
  int M, C, nblk, rpb;
  float eps, momentum;
  const float* gamma; const float* beta;
  float* rmean; float* rvar; int64_t* nbt;
  float* save_mean; float* save_invstd; float* scale; float* shift;   // fwd
  const float* mean; const float* invstd;                               // bwd
  float* dgamma; float* dbeta; float* coef;                             // bwd
};

// one thread per channel, the block partials summed in fp64 in block order (deterministic)
template <bool BWD>
__global__ void bnf_finalize_kernel(const float* __restrict__ part, BnF32Fin f) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (!BWD && c == 0 && f.nbt) f.nbt[0] += 1;
  if (c >= f.C) return;
  double s = 0.0, q = 0.0;
  if (BWD) {
    for (int b = 0; b < f.nblk; ++b) {
      s += part[(int64_t)(2 * b) * f.C + c];
      q += part[(int64_t)(2 * b + 1) * f.C + c];
    }
  } else {
    // Chan's parallel merge of the blocks' (count, mean, M2), in block order, fp64
    double n = 0.0;
    for (int b = 0; b < f.nblk; ++b) {
      const double nb = (double)(min(f.M, (b + 1) * f.rpb) - b * f.rpb);
      if (nb <= 0) continue;
      const double mb = part[(int64_t)(2 * b) * f.C + c], m2b = part[(int64_t)(2 * b + 1) * f.C + c];
      const double d = mb - s, nn = n + nb;
      s += d * nb / nn;
      q += m2b + d * d * n * nb / nn;
      n = nn;
    }
  }
  if (!BWD) {
    const double mean = s;
    double var = q / f.M;
    if (var < 0) var = 0;
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    f.save_mean[c] = (float)mean;
    f.save_invstd[c] = invstd;
    const float gm = f.gamma ? f.gamma[c] : 1.f, bt = f.beta ? f.beta[c] : 0.f;
    f.scale[c] = gm * invstd;
    f.shift[c] = bt;  // the apply centres x on save_mean (bnf_apply_kernel)
    if (f.rmean) {
      const double unbiased = f.M > 1 ? var * f.M / (f.M - 1) : var;
      f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * (float)mean;
      f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * (float)unbiased;
    }
  } else {
    const float is = f.invstd[c];
    const float sum_dz = (float)s, sum_dz_xhat = (float)(q * is);
    if (f.dgamma) f.dgamma[c] += sum_dz_xhat;
    if (f.dbeta) f.dbeta[c] += sum_dz;
    const float gm = f.gamma ? f.gamma[c] : 1.f;
    const float k0 = gm * is;
    const float mdz = sum_dz / f.M, mdzx = sum_dz_xhat / f.M;
    const float k1 = -k0 * is * mdzx;  // dx = k0 (dz - mean dz - xhat mean(dz xhat))
    f.coef[c] = k0;
    f.coef[f.C + c] = k1;
    f.coef[2 * f.C + c] = -k0 * mdz - k1 * f.mean[c];
  }
}

// y = act(x * scale + shift (+ res)); center (training forward, the batch mean): y = act((x - center) *
// scale + shift (+ res)) with shift = beta -- the centred form keeps fp32 accuracy when |mean| >> std,
// where x * scale and beta - mean * scale would cancel (as PyTorch's (x - mean) * invstd * w + b)
__global__ __launch_bounds__(FT) void bnf_apply_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                       float* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const float* __restrict__ center,
                                                       int64_t nvec, int C, int relu) {
  for (int64_t v = blockIdx.x * (int64_t)FT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * FT) {
    const int c = (int)((v * 4) % C);
    float4 a = ((const float4*)x)[v];
    const float4 sc = *(const float4*)(scale + c), sh = *(const float4*)(shift + c);
    if (center) {
      const float4 mu = *(const float4*)(center + c);
      a.x -= mu.x; a.y -= mu.y; a.z -= mu.z; a.w -= mu.w;
    }
    a.x = a.x * sc.x + sh.x; a.y = a.y * sc.y + sh.y; a.z = a.z * sc.z + sh.z; a.w = a.w * sc.w + sh.w;
    if (res) {
      const float4 r = ((const float4*)res)[v];
      a.x += r.x; a.y += r.y; a.z += r.z; a.w += r.w;
    }
    if (relu) { a.x = fmaxf(a.x, 0.f); a.y = fmaxf(a.y, 0.f); a.z = fmaxf(a.z, 0.f); a.w = fmaxf(a.w, 0.f); }
    ((float4*)y)[v] = a;
  }
}

// dz = dy * [y > 0] (relu); dx = k0 dz + k1 x + k2; dres = dz
__global__ __launch_bounds__(FT) void bnf_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                           const float* __restrict__ x, const float* __restrict__ coef,
                                                           float* __restrict__ dx, float* __restrict__ dres,
                                                           int64_t nvec, int C, int relu) {
  for (int64_t v = blockIdx.x * (int64_t)FT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * FT) {
    const int c = (int)((v * 4) % C);
    float4 d = ((const float4*)dy)[v];
    if (relu) {
      const float4 yv = ((const float4*)y)[v];
      d.x = yv.x > 0.f ? d.x : 0.f; d.y = yv.y > 0.f ? d.y : 0.f;
      d.z = yv.z > 0.f ? d.z : 0.f; d.w = yv.w > 0.f ? d.w : 0.f;
    }
    if (dres) ((float4*)dres)[v] = d;
    const float4 xv = ((const float4*)x)[v];
    const float4 k0 = *(const float4*)(coef + c), k1 = *(const float4*)(coef + C + c),
                 k2 = *(const float4*)(coef + 2 * C + c);
    float4 o;
    o.x = k0.x * d.x + k1.x * xv.x + k2.x; o.y = k0.y * d.y + k1.y * xv.y + k2.y;
    o.z = k0.z * d.z + k1.z * xv.z + k2.z; o.w = k0.w * d.w + k1.w * xv.w + k2.w;
    ((float4*)dx)[v] = o;
  }
}

// ----------------------------------------------------------------------- pooling (fp32)
// max pool k x k / stride / pad; tap = kh * k + kw of the first maximum in scan order (PyTorch's rule)
__global__ __launch_bounds__(FT) void maxpoolf_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          uint8_t* __restrict__ tap, int Nb, int H, int W, int C,
                                                          int P, int Q, int k, int s, int pad) {
  const int64_t total = (int64_t)Nb * P * Q * C;
  for (int64_t i = blockIdx.x * (int64_t)FT + threadIdx.x; i < total; i += (int64_t)gridDim.x * FT) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int q = (int)(r % Q); r /= Q;
    const int p = (int)(r % P);
    const int n = (int)(r / P);
    float best = -INFINITY;
    int bt = 0;
    for (int kh = 0; kh < k; ++kh) {
      const int h = p * s - pad + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = q * s - pad + kw;
        if (w < 0 || w >= W) continue;
        const float v = x[(((int64_t)n * H + h) * W + w) * C + c];
        if (v > best || v != v) { best = v; bt = kh * k + kw; }
      }
    }
    y[i] = best;
    tap[i] = (uint8_t)bt;
  }
}

// dx[n,h,w,c] = sum of dy over the windows whose arg-max tap is (h, w): a gather, no atomics
__global__ __launch_bounds__(FT) void maxpoolf_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ tap,
                                                          float* __restrict__ dx, int Nb, int H, int W, int C, int P,
                                                          int Q, int k, int s, int pad) {
  const int64_t total = (int64_t)Nb * H * W * C;
  for (int64_t i = blockIdx.x * (int64_t)FT + threadIdx.x; i < total; i += (int64_t)gridDim.x * FT) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    const int p0 = max(0, (h + pad - k + s) / s), p1 = min(P - 1, (h + pad) / s);
    const int q0 = max(0, (w + pad - k + s) / s), q1 = min(Q - 1, (w + pad) / s);
    float acc = 0.f;
    for (int p = p0; p <= p1; ++p) {
      const int kh = h + pad - p * s;
      if (kh < 0 || kh >= k) continue;
      for (int q = q0; q <= q1; ++q) {
        const int kw = w + pad - q * s;
        if (kw < 0 || kw >= k) continue;
        const int64_t o = (((int64_t)n * P + p) * Q + q) * C + c;
        if (tap[o] == kh * k + kw) acc += dy[o];
      }
    }
    dx[i] = acc;
  }
}

// y[n][c] = mean over HW of x[n][hw][c]; one thread per (n, c), HW summed in order
__global__ __launch_bounds__(FT) void gapf_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int Nb,
                                                      int HW, int C) {
  const int i = blockIdx.x * FT + threadIdx.x;
  if (i >= Nb * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int j = 0; j < HW; ++j) s += x[((int64_t)n * HW + j) * C + c];
  y[i] = s / HW;
}

__global__ __launch_bounds__(FT) void gapf_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, int Nb,
                                                      int HW, int C) {
  const int64_t total = (int64_t)Nb * HW * C;
  for (int64_t i = blockIdx.x * (int64_t)FT + threadIdx.x; i < total; i += (int64_t)gridDim.x * FT) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((int64_t)HW * C));
    dx[i] = dy[(int64_t)n * C + c] / HW;
  }
}

// g[n] (+)= sum over rows of dy[row][n], rows in order (Linear bias gradient)
__global__ __launch_bounds__(FT) void colsum_f32_kernel(const float* __restrict__ dy, float* __restrict__ g, int rows,
                                                        int N, int accumulate) {
  const int n = blockIdx.x * FT + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += dy[(int64_t)r * N + n];
  g[n] = accumulate ? g[n] + s : s;
}

int ew_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + FT - 1) / FT, 8192)); }

int bnf_rows_per_block(int M, int C) {
  int tpr = std::min(C / 4, FT), rp = FT / tpr;
  // ~1024 blocks over rows, each block's row count a multiple of the rows it processes at once
  int rpb = std::max(rp, cdiv(M, 1024));
  return cdiv(rpb, rp) * rp;
}

}  // namespace

// ------------------------------------------------------------------------------------------ API
// mode 0: out[Nb*P*Q][K] = conv(x, w); 1: out[Nb*H*W][C] = dgrad(dy, w); 2: out[K][R*S*C] (+)= wgrad(dy, x)
// a / b: mode 0 (x, w), 1 (dy, w), 2 (dy, x).  Split-K workspace: mi_f32_conv_ws_floats() floats.
MI_API int mi_f32_conv_splits(int mode, int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad, int P,
                              int Q) {
  return f32_splits(make_f32_geom(mode, Nb, H, W, C, K, R, S, stride, pad, P, Q));
}

MI_API int64_t mi_f32_conv_ws_floats(int mode, int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad,
                                     int P, int Q) {
  const F32Geom g = make_f32_geom(mode, Nb, H, W, C, K, R, S, stride, pad, P, Q);
  const int s = f32_splits(g);
  return s > 1 ? (int64_t)s * g.M * g.N : 0;
}

MI_API int mi_f32_conv(int mode, const float* a, const float* b, float* out, float* ws, const float* bias,
                       int accumulate, int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad, int P,
                       int Q, hipStream_t st) {
  if (mode < 0 || mode > 2 || C % 4 || K % 4 || stride < 1 || (bias && mode != 0)) return (int)hipErrorInvalidValue;
  if (P != (H + 2 * pad - R) / stride + 1 || Q != (W + 2 * pad - S) / stride + 1) return (int)hipErrorInvalidValue;
  const F32Geom g = make_f32_geom(mode, Nb, H, W, C, K, R, S, stride, pad, P, Q);
  if ((int64_t)g.M * g.N > 0x7FFFFFFF || (int64_t)g.Kr > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  const int splits = f32_splits(g);
  if (splits > 1 && !ws) return (int)hipErrorInvalidValue;
  const int kt = cdiv(g.Kr, TK);
  const int per = cdiv(kt, splits);
  dim3 grid(cdiv(g.M, TM), cdiv(g.N, TN), splits);
  float* w = splits > 1 ? ws : nullptr;
  if (mode == 0) hipLaunchKernelGGL(conv_f32_kernel<0>, grid, dim3(FT), 0, st, a, b, out, w, bias, g, accumulate, per);
  else if (mode == 1) hipLaunchKernelGGL(conv_f32_kernel<1>, grid, dim3(FT), 0, st, a, b, out, w, bias, g, accumulate, per);
  else hipLaunchKernelGGL(conv_f32_kernel<2>, grid, dim3(FT), 0, st, a, b, out, w, bias, g, accumulate, per);
  if (splits > 1) {
    const int64_t mn = (int64_t)g.M * g.N;
    hipLaunchKernelGGL(splitk_sum_f32_kernel, dim3(ew_grid(mn)), dim3(FT), 0, st, ws, out, bias, mn, g.N, splits,
                       accumulate);
  }
  return (int)hipGetLastError();
}

// partial-slab rows of the fp32 BN statistics passes
MI_API int mi_f32_bn_partial_rows(int M, int C) { return cdiv(M, bnf_rows_per_block(M, C)); }

// training forward: batch statistics -> running stats, nbt, save_mean / save_invstd, scale / shift,
// then y = act(x * scale + shift (+ res)) (y may be null: statistics only)
MI_API int mi_f32_bn_fwd_train(const float* x, const float* res, float* y, int M, int C, float eps, float momentum,
                               const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
                               float* save_mean, float* save_invstd, float* scale, float* shift, float* part, int relu,
                               hipStream_t st) {
  if (C % 4 || M < 1) return (int)hipErrorInvalidValue;
  const int rpb = bnf_rows_per_block(M, C), nblk = cdiv(M, rpb);
  const int tpr = std::min(C / 4, FT);
  hipLaunchKernelGGL(bnf_stats_kernel<false>, dim3(nblk, cdiv(C, tpr * 4)), dim3(FT), 0, st, x, nullptr, nullptr,
                     nullptr, part, M, C, rpb, 0);
  BnF32Fin f{};
  f.M = M; f.C = C; f.nblk = nblk; f.rpb = rpb; f.eps = eps; f.momentum = momentum; f.gamma = gamma; f.beta = beta;
  f.rmean = rmean; f.rvar = rvar; f.nbt = nbt; f.save_mean = save_mean; f.save_invstd = save_invstd;
  f.scale = scale; f.shift = shift;
  hipLaunchKernelGGL(bnf_finalize_kernel<false>, dim3(cdiv(C, 256)), dim3(256), 0, st, part, f);
  if (y) {
    const int64_t nvec = (int64_t)M * C / 4;
    hipLaunchKernelGGL(bnf_apply_kernel, dim3(ew_grid(nvec)), dim3(FT), 0, st, x, res, y, scale, shift, save_mean,
                       nvec, C, relu);
  }
  return (int)hipGetLastError();
}

// y = act(x * scale + shift (+ res)) (eval mode / precomputed coefficients)
MI_API int mi_f32_bn_apply(const float* x, const float* res, float* y, int M, int C, const float* scale,
                           const float* shift, int relu, hipStream_t st) {
  if (C % 4) return (int)hipErrorInvalidValue;
  const int64_t nvec = (int64_t)M * C / 4;
  hipLaunchKernelGGL(bnf_apply_kernel, dim3(ew_grid(nvec)), dim3(FT), 0, st, x, res, y, scale, shift, nullptr, nvec,
                     C, relu);
  return (int)hipGetLastError();
}

// training backward: dz = dy * [y > 0] (relu), statistics -> dgamma / dbeta (+=) and dx (and dres = dz)
MI_API int mi_f32_bn_bwd_train(const float* dy, const float* y, const float* x, float* dx, float* dres, int M, int C,
                               const float* gamma, const float* mean, const float* invstd, float* dgamma,
                               float* dbeta, float* coef, float* part, int relu, hipStream_t st) {
  if (C % 4 || M < 1) return (int)hipErrorInvalidValue;
  const int rpb = bnf_rows_per_block(M, C), nblk = cdiv(M, rpb);
  const int tpr = std::min(C / 4, FT);
  hipLaunchKernelGGL(bnf_stats_kernel<true>, dim3(nblk, cdiv(C, tpr * 4)), dim3(FT), 0, st, x, dy, y, mean, part, M,
                     C, rpb, relu);
  BnF32Fin f{};
  f.M = M; f.C = C; f.nblk = nblk; f.gamma = gamma; f.mean = mean; f.invstd = invstd;
  f.dgamma = dgamma; f.dbeta = dbeta; f.coef = coef;
  hipLaunchKernelGGL(bnf_finalize_kernel<true>, dim3(cdiv(C, 256)), dim3(256), 0, st, part, f);
  const int64_t nvec = (int64_t)M * C / 4;
  hipLaunchKernelGGL(bnf_bwd_apply_kernel, dim3(ew_grid(nvec)), dim3(FT), 0, st, dy, y, x, coef, dx, dres, nvec, C,
                     relu);
  return (int)hipGetLastError();
}

MI_API int mi_f32_maxpool_fwd(const float* x, float* y, uint8_t* tap, int Nb, int H, int W, int C, int P, int Q, int k,
                              int s, int pad, hipStream_t st) {
  if (k * k > 256) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)Nb * P * Q * C;
  hipLaunchKernelGGL(maxpoolf_fwd_kernel, dim3(ew_grid(n)), dim3(FT), 0, st, x, y, tap, Nb, H, W, C, P, Q, k, s, pad);
  return (int)hipGetLastError();
}

MI_API int mi_f32_maxpool_bwd(const float* dy, const uint8_t* tap, float* dx, int Nb, int H, int W, int C, int P,
                              int Q, int k, int s, int pad, hipStream_t st) {
  const int64_t n = (int64_t)Nb * H * W * C;
  hipLaunchKernelGGL(maxpoolf_bwd_kernel, dim3(ew_grid(n)), dim3(FT), 0, st, dy, tap, dx, Nb, H, W, C, P, Q, k, s,
                     pad);
  return (int)hipGetLastError();
}

MI_API int mi_f32_gap_fwd(const float* x, float* y, int Nb, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gapf_fwd_kernel, dim3(cdiv((int64_t)Nb * C, FT)), dim3(FT), 0, st, x, y, Nb, HW, C);
  return (int)hipGetLastError();
}

MI_API int mi_f32_gap_bwd(const float* dy, float* dx, int Nb, int HW, int C, hipStream_t st) {
  const int64_t n = (int64_t)Nb * HW * C;
  hipLaunchKernelGGL(gapf_bwd_kernel, dim3(ew_grid(n)), dim3(FT), 0, st, dy, dx, Nb, HW, C);
  return (int)hipGetLastError();
}

MI_API int mi_f32_colsum(const float* dy, float* g, int rows, int N, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(colsum_f32_kernel, dim3(cdiv(N, FT)), dim3(FT), 0, st, dy, g, rows, N, accumulate);
  return (int)hipGetLastError();
}
