// BatchNorm2d (train + eval) over NHWC bf16 activations with fused ReLU and
// residual add, for gfx950.  Replaces cuDNN BN fwd/bwd + ATen ReLU / add
// kernels on the reference's ResNet hot path.
//
// Forward (train):  stats partials -> finalize (mean/invstd, running stats,
//                   num_batches_tracked, scale/shift) -> apply y = act(x*a+b (+res))
// Backward:         partial sums of dz and dz*xhat (dz = dy * [y>0]) ->
//                   finalize (dgamma/dbeta accumulated into the fp32 grad buffer,
//                   per-channel affine dx = k0*dz + k1*x + k2) -> apply (+ dres = dz)
// The ReLU mask is recovered from the saved output y, so no mask tensor exists.
// All loads/stores are 16-byte vectors (8 bf16 per lane).
#include "common.h"
#include <mutex>
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int NT = 256;
// BN-backward statistics and stem BN+pool passes: cached input loads (non-temporal ones measured
// neutral or slower, round 5: profiles/raw/r5/bnx/)
constexpr bool kBnxNt = false;

struct SlabGeom {
  int tpr;   // threads per row (each covers 8 channels)
  int rp;    // rows processed in parallel per block
  int cw;    // channel slab width
};

__host__ __device__ inline SlabGeom slab_geom(int C) {
  SlabGeom g;
  g.tpr = C / 8 < NT ? C / 8 : NT;
  g.rp = NT / g.tpr;
  g.cw = g.tpr * 8;
  return g;
}

// Reduce the per-thread 8-channel partials over the rp row-groups and write
// two rows (s0, s1) of the partial slab for this block.
__device__ __forceinline__ void block_reduce_store(float* s0, float* s1, float* part, int C, int cbase,
                                                   const SlabGeom& g) {
  __shared__ float red[2][NT * 8];
  const int tid = threadIdx.x;
  const int c8 = tid % g.tpr, r0 = tid / g.tpr;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][r0 * g.cw + c8 * 8 + j] = s0[j];
    red[1][r0 * g.cw + c8 * 8 + j] = s1[j];
  }
  __syncthreads();
  // each of the first cw threads sums one channel over rp rows
  for (int c = tid; c < g.cw; c += NT) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < g.rp; ++r) { a += red[0][r * g.cw + c]; b += red[1][r * g.cw + c]; }
    part[(size_t)(blockIdx.x * 2 + 0) * C + cbase + c] = a;
    part[(size_t)(blockIdx.x * 2 + 1) * C + cbase + c] = b;
  }
}

__global__ __launch_bounds__(NT) void bn_stats_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                      int M, int C, int rows_per_block) {
  const SlabGeom g = slab_geom(C);
  const int tid = threadIdx.x;
  const int c8 = tid % g.tpr, r0 = tid / g.tpr;
  const int cbase = blockIdx.y * g.cw;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  float s[8] = {0}, q[8] = {0};
  const bf16_t* base = x + cbase + c8 * 8;
  for (int r = rb + r0; r < re; r += g.rp) {
    uint4 v = *(const uint4*)(base + (size_t)r * C);
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] += f[j] * f[j]; }
  }
  block_reduce_store(s, q, part, C, cbase, g);
}

// Reduce the [nblk][2][C] partial slab for 64 consecutive channels per block:
// 1024 threads = 64 channel lanes x 16 row groups, coalesced 256-B row reads,
// fp64 accumulation, LDS tree over the 16 groups.  Result in (s, q) of tid<64.
constexpr int FIN_T = 1024, FIN_G = FIN_T / 64;

// a += sum of p[2 i * C + c], b += sum of p[(2 i + 1) * C + c] over rows i = i0, i0 + step, .. < i1,
// in row order (bitwise the plain loop's result), with FIN_U rows' loads in flight at once: the
// one-row-per-iteration loops waited a full memory round trip per row (s_waitcnt vmcnt(0) each
// iteration) -- 8 L2 trips in a split, 3+ memory trips (agent-scope hand-off loads) in the final
// stage, ~9 us of the ~10 us a finalize launch took.  ATOMIC: agent-scope loads (hand-off rows).
constexpr int FIN_U = 8;
template <bool ATOMIC>
__device__ __forceinline__ void sum_rows(const float* __restrict__ p, int i0, int i1, int step, int C, int c,
                                         double& a, double& b) {
  for (int i = i0; i < i1; i += FIN_U * step) {
    float va[FIN_U], vb[FIN_U];
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) {
      const int r = i + u * step;
      va[u] = 0.f;
      vb[u] = 0.f;
      if (r < i1) {
        const float* q = p + (size_t)(2 * r) * C + c;
        if constexpr (ATOMIC) {
          va[u] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          vb[u] = __hip_atomic_load(q + C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          va[u] = q[0];
          vb[u] = q[C];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) {  // + 0.0 past the end: exact, the order is the plain loop's
      a += va[u];
      b += vb[u];
    }
  }
}

__device__ __forceinline__ bool slab_reduce64(const float* __restrict__ part, int nblk, int C, double& s, double& q) {
  __shared__ double red[2][FIN_G][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (c < C) sum_rows<false>(part, rg, nblk, FIN_G, C, c, a, b);
  red[0][rg][cl] = a;
  red[1][rg][cl] = b;
  __syncthreads();
  if (rg != 0) return false;
  for (int g = 1; g < FIN_G; ++g) { a += red[0][g][cl]; b += red[1][g][cl]; }
  s = a; q = b;
  return c < C;
}

// Stage-1 of a tall slab: block (cg, split) reduces rows [split*rows_per, ...) of 64 channels
// into out[split][2][C] (fp32, deterministic; no atomics).  Stage 2 is the finalize kernel.
__global__ __launch_bounds__(FIN_T) void slab_split_kernel(const float* __restrict__ part, int nblk, int C,
                                                           int rows_per, float* __restrict__ out) {
  __shared__ double red[2][FIN_G][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int b0 = blockIdx.y * rows_per, b1 = min(nblk, b0 + rows_per);
  double a = 0.0, b = 0.0;
  if (c < C) sum_rows<false>(part, b0 + rg, b1, FIN_G, C, c, a, b);
  red[0][rg][cl] = a;
  red[1][rg][cl] = b;
  __syncthreads();
  if (rg != 0 || c >= C) return;
  for (int g = 1; g < FIN_G; ++g) { a += red[0][g][cl]; b += red[1][g][cl]; }
  out[(size_t)(2 * blockIdx.y) * C + c] = (float)a;
  out[(size_t)(2 * blockIdx.y + 1) * C + c] = (float)b;
}

// per-channel finalize operands of the training forward (F) and backward (B)
struct FinArgs {
  int M, C;
  float eps, momentum;                                        // F
  const float* gamma; const float* beta;                      // F (gamma also B)
  float* rmean; float* rvar; int64_t* nbt;                    // F
  float* save_mean; float* save_invstd; float* scale; float* shift;  // F
  const float* mean; const float* invstd;                     // B
  float* dgamma; float* dbeta; float* coef;                   // B
};

__device__ __forceinline__ void fin_fwd(int c, double s, double q, const FinArgs& f) {
  const int M = f.M;
  const float eps = f.eps, momentum = f.momentum;
  const float* gamma = f.gamma; const float* beta = f.beta;
  float* rmean = f.rmean; float* rvar = f.rvar;
  float* save_mean = f.save_mean; float* save_invstd = f.save_invstd;
  float* scale = f.scale; float* shift = f.shift;
  const double mean = s / M;
  double var = q / M - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale[c] = gm * invstd;
  shift[c] = bt - (float)mean * gm * invstd;
  if (rmean) {
    const double unbiased = M > 1 ? var * M / (M - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
  }
}

// training-mode finalize
__global__ __launch_bounds__(FIN_T) void bn_finalize_kernel(const float* __restrict__ part, int nblk, FinArgs f) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && f.nbt) f.nbt[0] += 1;
  double s, q;
  if (!slab_reduce64(part, nblk, f.C, s, q)) return;
  fin_fwd(blockIdx.x * 64 + (threadIdx.x & 63), s, q, f);
}

__global__ void bn_eval_coeffs_kernel(int C, float eps, const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar,
                                      float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rvar[c] + eps);
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale[c] = gm * invstd;
  shift[c] = bt - rmean[c] * gm * invstd;
}

// Elementwise passes are HBM-bound: each thread keeps EW_U 16-byte vectors (EW_U x grid stride
// apart, so every wave-instruction stays 1 KB contiguous) in flight before using any, instead of
// one load -> use -> store chain per iteration.  Channel of vector v: (8 v) mod C, advanced
// incrementally by the (uniform) stride's channel step.
constexpr int EW_U = 4;
constexpr int kEwGridCap = 65536;  // default elementwise grid cap (MI355X_DP_EW_GRID_CAP)

// 16-byte store of an elementwise result: non-temporal, streaming past L2 (plain stores measured
// -1.0 % on the BN-backward apply, round 5)
__device__ __forceinline__ void st16(void* base, int64_t v, uint4 val) {
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4, val), (u32x4*)base + v);
}
// the forward apply's output (the next conv's input): the same policy
__device__ __forceinline__ void st16f(void* base, int64_t v, uint4 val) {
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4, val), (u32x4*)base + v);
}

struct EwIter {
  int64_t v0, stride;
  int c0, cstep;
  __device__ EwIter(int64_t nvec, int C) {
    stride = (int64_t)gridDim.x * NT;
    v0 = blockIdx.x * (int64_t)NT + threadIdx.x;
    cstep = (int)((stride * 8) % C);
    c0 = (int)((v0 * 8) % C);
  }
  __device__ __forceinline__ int chan(int c, int C) const { return c + cstep >= C ? c + cstep - C : c + cstep; }
  __device__ __forceinline__ void next(int C) {
    v0 += stride * EW_U;
    c0 = (int)((v0 * 8) % C);
  }
};

// y = act(x*scale + shift (+ res)); grid-stride over 8-element vectors.  RES_BN: the residual is
// itself a raw BN input, normalised on the fly (res*rscale + rshift) -- the downsample branch's
// BatchNorm output is never stored (ResNet projection shortcut).
// FIXC: the grid stride (in elements) is a multiple of C, so every vector a thread touches has the
// same 8 channels -- the coefficients are loaded into registers once instead of four 16-byte L1
// loads per 16 bytes of data (which made the pass TA/L1-issue-bound at ~3 TB/s).  Host picks it
// when (grid * NT * 8) % C == 0 (every ResNet width).
__device__ __forceinline__ void load8f(const float* __restrict__ p, int c, float* o) {
  *(float4*)&o[0] = *(const float4*)(p + c);
  *(float4*)&o[4] = *(const float4*)(p + c + 4);
}

template <bool RES_BN, bool FIXC>
__global__ __launch_bounds__(NT) void bn_apply_kernel_t(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                        bf16_t* __restrict__ y, const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ rscale,
                                                        const float* __restrict__ rshift, int64_t nvec, int C,
                                                        int relu, uint8_t* __restrict__ bits) {
  EwIter it(nvec, C);
  float a[8], b[8], pr[8], qr[8];
  if (FIXC) {
    load8f(scale, it.c0, a);
    load8f(shift, it.c0, b);
    if (RES_BN) {
      load8f(rscale, it.c0, pr);
      load8f(rshift, it.c0, qr);
    }
  }
  for (; it.v0 < nvec; it.next(C)) {
    uint4 xv[EW_U], rv[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = it.v0 + u * it.stride;
      if (v < nvec) {
        xv[u] = ld_nt16(x, v);
        if (res) rv[u] = ld_nt16(res, v);
      }
    }
    int c = it.c0;
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = it.v0 + u * it.stride;
      if (v >= nvec) break;
      float f[8];
      unpack8(xv[u], f);
      if (!FIXC) {
        load8f(scale, c, a);
        load8f(shift, c, b);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * a[j] + b[j];
      if (res) {
        float r[8];
        unpack8(rv[u], r);
        if (RES_BN) {
          if (!FIXC) {
            load8f(rscale, c, pr);
            load8f(rshift, c, qr);
          }
          // round like a stored bf16 shortcut activation: bit-identical to the unfused sequence
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = bf2f(f2bf(r[j] * pr[j] + qr[j]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += r[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      const uint4 o = pack8(f);
      st16f(y, v, o);
      if (bits) bits[v] = (uint8_t)nz_bits8(o);  // the consumer's ReLU mask, 1/16 of y's bytes
      if (!FIXC) c = it.chan(c, C);
    }
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_stats_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                          float* __restrict__ part, int M, int C, int rows_per_block,
                                                          int relu) {
  const SlabGeom g = slab_geom(C);
  const int tid = threadIdx.x;
  const int c8 = tid % g.tpr, r0 = tid / g.tpr;
  const int cbase = blockIdx.y * g.cw;
  const int cc = cbase + c8 * 8;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  float mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) mu[j] = mean[cc + j];
  float s[8] = {0}, q[8] = {0};
  for (int r = rb + r0; r < re; r += g.rp) {
    const size_t off = (size_t)r * C + cc;
    float d[8], xv[8];
    unpack8(epi_ld16<kBnxNt>(dy + off), d);
    unpack8(epi_ld16<kBnxNt>(x + off), xv);
    if (relu) {
      float yv[8];
      unpack8(epi_ld16<kBnxNt>(y + off), yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] += d[j]; q[j] += d[j] * (xv[j] - mu[j]); }
  }
  block_reduce_store(s, q, part, C, cbase, g);
}

// per-channel affine of the BN backward: dx = k0*dz + k1*x + k2 (dz = relu-masked dy)
__device__ __forceinline__ void bwd_coefs(int c, double s, double q, const FinArgs& f, float& k0, float& k1,
                                          float& k2) {
  const float is = f.invstd[c];
  const float sum_dz = (float)s;
  const float sum_dz_xhat = (float)q * is;
  const float gm = f.gamma ? f.gamma[c] : 1.f;
  k0 = gm * is;
  const float mdz = sum_dz / f.M, mdzx = sum_dz_xhat / f.M;
  // dx = k0*(dz - mdz - xhat*mdzx),  xhat = (x-mean)*is
  k1 = -k0 * is * mdzx;
  k2 = -k0 * mdz - k1 * f.mean[c];
}

// -> dgamma/dbeta (+=) and coef[0..2][C] so that dx = coef0*dz + coef1*x + coef2.  SC1: the
// coefficients are stored write-through (sc1) for consumers on other CUs of the SAME launch
// (bn_bwd_fin_apply_kernel), which read them with sc1 loads after an agent-scope signal
template <bool SC1 = false>
__device__ __forceinline__ void fin_bwd(int c, double s, double q, const FinArgs& f) {
  const int C = f.C;
  const float is = f.invstd[c];
  if (f.dgamma) f.dgamma[c] += (float)q * is;
  if (f.dbeta) f.dbeta[c] += (float)s;
  float k0, k1, k2;
  bwd_coefs(c, s, q, f, k0, k1, k2);
  if (SC1) {
    __hip_atomic_store(f.coef + c, k0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f.coef + C + c, k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f.coef + 2 * C + c, k2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    f.coef[c] = k0;
    f.coef[C + c] = k1;
    f.coef[2 * C + c] = k2;
  }
}

__global__ __launch_bounds__(FIN_T) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, FinArgs f) {
  double s, q;
  if (!slab_reduce64(part, nblk, f.C, s, q)) return;
  fin_bwd(blockIdx.x * 64 + (threadIdx.x & 63), s, q, f);
}

// Tall slabs in ONE launch: block (cg, split) reduces its rows of 64 channels into out[split][2][C]
// like slab_split_kernel, then counts its arrival; the last arriving split of channel group cg
// (device-scope release/acquire) reduces the S rows and runs the finalize for those channels.
// Deterministic: fixed split ranges, fixed reduction order.  cnt[cg] is reset by the finalizer.
// Returns true in the block that finalized group cg (its wave 0 wrote the per-channel outputs).
template <bool BWD, bool SC1, int TG = FIN_G>  // TG row groups of 64 channel lanes (blockDim = 64 TG)
__device__ __forceinline__ bool split_fin_body(const float* __restrict__ part, int nblk, int rows_per,
                                               float* __restrict__ out, int* __restrict__ cnt, const FinArgs& f,
                                               int cg, int split, int S, double (*red)[TG][64], int* last) {
  const int C = f.C;
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = cg * 64 + cl;
  const int b0 = split * rows_per, b1 = min(nblk, b0 + rows_per);
  double a = 0.0, b = 0.0;
  if (c < C) sum_rows<false>(part, b0 + rg, b1, TG, C, c, a, b);
  red[0][rg][cl] = a;
  red[1][rg][cl] = b;
  __syncthreads();
  // Hand-off to the last-arriving block without fences (MI355X_MICROARCH.md, inter-workgroup
  // visibility, first table row): wave 0 alone stores this split's row with sc1 (write-through,
  // dropped from the XCD's L2), waits for its stores, and then one lane counts the arrival with an
  // agent-scope atomic; the finalizer reads the rows with sc1 loads.  The acq_rel __threadfence
  // pair this replaces cost ~3.5 us per fence on the compute stream's critical path, 89 times per
  // ResNet-50 step.
  if (rg == 0) {
    if (c < C) {
      for (int g = 1; g < TG; ++g) { a += red[0][g][cl]; b += red[1][g][cl]; }
      __hip_atomic_store(out + (size_t)(2 * split) * C + c, (float)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(out + (size_t)(2 * split + 1) * C + c, (float)b, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) *last = atomicAdd(cnt + cg, 1) == S - 1;
  }
  __syncthreads();
  if (!*last) return false;
  if (threadIdx.x == 0) {
    cnt[cg] = 0;  // ready for the next launch (stream order)
    if (!BWD && cg == 0 && f.nbt) f.nbt[0] += 1;
  }
  // second stage over the S split rows (other blocks' rows: sc1 loads, see above)
  double s2 = 0.0, q2 = 0.0;
  if (c < C) sum_rows<true>(out, rg, S, TG, C, c, s2, q2);
  __syncthreads();
  red[0][rg][cl] = s2;
  red[1][rg][cl] = q2;
  __syncthreads();
  if (rg != 0 || c >= C) return true;
  for (int g = 1; g < TG; ++g) { s2 += red[0][g][cl]; q2 += red[1][g][cl]; }
  if (BWD) fin_bwd<SC1>(c, s2, q2, f);
  else fin_fwd(c, s2, q2, f);
  return true;
}

template <bool BWD>
__global__ __launch_bounds__(FIN_T) void slab_split_fin_kernel(const float* __restrict__ part, int nblk,
                                                               int rows_per, float* __restrict__ out,
                                                               int* __restrict__ cnt, FinArgs f) {
  __shared__ double red[2][FIN_G][64];
  __shared__ int last;
  split_fin_body<BWD, false>(part, nblk, rows_per, out, cnt, f, blockIdx.x, blockIdx.y, gridDim.y, red, &last);
}

template <bool FIXC>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                                          bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                                          int64_t nvec, int C, int relu) {
  EwIter it(nvec, C);
  float k0[8], k1[8], k2[8];
  if (FIXC) {  // see bn_apply_kernel_t: one channel octet per thread for the whole pass
    load8f(coef, it.c0, k0);
    load8f(coef + C, it.c0, k1);
    load8f(coef + 2 * C, it.c0, k2);
  }
  for (; it.v0 < nvec; it.next(C)) {
    uint4 dv[EW_U], xq[EW_U], yq[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = it.v0 + u * it.stride;
      if (v < nvec) {
        dv[u] = ld_nt16(dy, v);
        xq[u] = ld_nt16(x, v);
        if (relu) yq[u] = ld_nt16(y, v);
      }
    }
    int c = it.c0;
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = it.v0 + u * it.stride;
      if (v >= nvec) break;
      float d[8], xv[8];
      unpack8(dv[u], d);
      unpack8(xq[u], xv);
      if (relu) {
        float yv[8];
        unpack8(yq[u], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
      }
      if (dres) st16(dres, v, pack8(d));
      if (!FIXC) {
        load8f(coef, c, k0);
        load8f(coef + C, c, k1);
        load8f(coef + 2 * C, c, k2);
      }
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k0[j] * d[j] + k1[j] * xv[j] + k2[j];
      st16(dx, v, pack8(o));
      if (!FIXC) c = it.chan(c, C);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// BN backward of a tall slab in ONE launch: finalize + apply (the finalize's own
// launch -- ~6-12 us and a dependent kernel boundary, 46 times per ResNet-50 step on the compute
// stream -- folded into its consumer).  Blocks [0, G*S) are the finalizer blocks of
// slab_split_fin_kernel (G channel groups x S splits; the last-arriving split of each group
// finalizes it and writes its coefficients write-through); the group whose arrival completes all G
// raises `ready`.  Blocks [G*S, G*S + A) apply: each issues the loads of its first EW_U vectors,
// then waits for `ready` (one lane polls with sc1 loads and s_sleep), reads its channel octet's
// coefficients with sc1 loads (MI355X_MICROARCH.md hand-off table, first row) and sweeps its vectors.
// The finalizer blocks have the lowest block indices, so they are dispatched first; a bounded wait
// never hangs anyway: an apply block that waited kFinWaitTicks (100 MHz) computes the
// coefficients itself from the slab (no dgamma / dbeta writes) and counts the event in sync[3].
// `ready` is reset for the next launch by whichever of {the A apply blocks after their wait, the
// block that raised it} arrives last (sync[2]); sync[0] counts finalized groups.
constexpr uint64_t kFinWaitTicks = 200000;  // 2 ms
constexpr int FUSED_MAX_C = 2048;
constexpr int FUSED_T = 512, FUSED_G = FUSED_T / 64;  // 2 waves per SIMD: up to 256 VGPRs, no spills
struct FusedBwdArgs {
  const float* part; int nblk, rows_per, S, G;
  float* out; int* cnt; uint32_t* sync;
  FinArgs f;
  const bf16_t* dy; const bf16_t* y; const bf16_t* x; bf16_t* dx; bf16_t* dres;
  int64_t nvec; int A; int relu;
};

__device__ __forceinline__ void ld8_sc1(const float* p, float* o) {
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = __hip_atomic_load(p + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool RELU>
__global__ __launch_bounds__(FUSED_T) void bn_bwd_fin_apply_kernel(FusedBwdArgs p) {
  __shared__ double red[2][FUSED_G][64];
  __shared__ int last, ok;
  const int F = p.G * p.S;
  const int C = p.f.C;
  if ((int)blockIdx.x < F) {
    if (split_fin_body<true, true, FUSED_G>(p.part, p.nblk, p.rows_per, p.out, p.cnt, p.f, blockIdx.x % p.G,
                                   blockIdx.x / p.G, p.S, red, &last)) {
      // wave 0 wrote this group's coefficients (sc1); after its stores, lane 0 counts the group
      if (threadIdx.x < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0 && atomicAdd(p.sync, 1u) == (uint32_t)p.G - 1) {
          p.sync[0] = 0;
          __hip_atomic_store(p.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (atomicAdd(p.sync + 2, 1u) == (uint32_t)p.A) {  // every apply block already gave up waiting
            __hip_atomic_store(p.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            p.sync[2] = 0;
          }
        }
      }
    }
    return;
  }
  // ------------------------------------------------------------------ apply block
  const int64_t stride = (int64_t)p.A * FUSED_T;
  const int64_t v0 = (int64_t)(blockIdx.x - F) * FUSED_T + threadIdx.x;
  const int c0 = (int)((v0 * 8) % C);  // fixed for the whole sweep: (stride * 8) % C == 0 (host)
  uint4 dv[EW_U], xq[EW_U], yq[EW_U];
#pragma unroll
  for (int u = 0; u < EW_U; ++u) {  // the first batch in flight while the coefficients are finalized
    const int64_t v = v0 + u * stride;
    if (v < p.nvec) {
      dv[u] = ld_nt16(p.dy, v);
      xq[u] = ld_nt16(p.x, v);
      if (RELU) yq[u] = ld_nt16(p.y, v);
    }
  }
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int good = 1;
    while (__hip_atomic_load(p.sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kFinWaitTicks) {
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(32);  // ~1 us between polls: many tight pollers of one word slow the chip
    }
    ok = good;
  }
  __syncthreads();
  float k0[8], k1[8], k2[8];
  if (ok) {
    ld8_sc1(p.f.coef + c0, k0);
    ld8_sc1(p.f.coef + C + c0, k1);
    ld8_sc1(p.f.coef + 2 * C + c0, k2);
  } else {
    // fallback: every channel's coefficients from the complete slab (written by the previous
    // kernel) into LDS, 64 channels at a time through the block-wide fixed-order reduction; the
    // prefetched batch is dropped and re-read (keeps it out of this path's registers)
    __shared__ float lc[3][FUSED_MAX_C];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    for (int cg = 0; cg < p.G; ++cg) {
      const int c = cg * 64 + cl;
      double a = 0.0, b = 0.0;
      if (c < C) sum_rows<false>(p.part, rg, p.nblk, FUSED_G, C, c, a, b);
      __syncthreads();
      red[0][rg][cl] = a;
      red[1][rg][cl] = b;
      __syncthreads();
      if (rg == 0 && c < C) {
        for (int g = 1; g < FUSED_G; ++g) { a += red[0][g][cl]; b += red[1][g][cl]; }
        bwd_coefs(c, a, b, p.f, lc[0][c], lc[1][c], lc[2][c]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) { k0[j] = lc[0][c0 + j]; k1[j] = lc[1][c0 + j]; k2[j] = lc[2][c0 + j]; }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = v0 + u * stride;
      if (v < p.nvec) {
        dv[u] = ld_nt16(p.dy, v);
        xq[u] = ld_nt16(p.x, v);
        if (RELU) yq[u] = ld_nt16(p.y, v);
      }
    }
    if (threadIdx.x == 0) atomicAdd(p.sync + 3, 1u);
  }
  if (threadIdx.x == 0 && atomicAdd(p.sync + 2, 1u) == (uint32_t)p.A) {  // last of A readers + raiser
    __hip_atomic_store(p.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.sync[2] = 0;
  }
  for (int64_t base = v0;; base += stride * EW_U) {
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = base + u * stride;
      if (v >= p.nvec) break;
      float d[8], xv[8];
      unpack8(dv[u], d);
      unpack8(xq[u], xv);
      if (RELU) {
        float yv[8];
        unpack8(yq[u], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
      }
      if (p.dres) st16(p.dres, v, pack8(d));
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k0[j] * d[j] + k1[j] * xv[j] + k2[j];
      st16(p.dx, v, pack8(o));
    }
    const int64_t nb = base + stride * EW_U;
    if (nb >= p.nvec) break;
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const int64_t v = nb + u * stride;
      if (v < p.nvec) {
        dv[u] = ld_nt16(p.dy, v);
        xq[u] = ld_nt16(p.x, v);
        if (RELU) yq[u] = ld_nt16(p.y, v);
      }
    }
  }
}

// eval-mode / frozen BN backward: dx = scale * dz
__global__ __launch_bounds__(NT) void bn_bwd_eval_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                         const float* __restrict__ scale, bf16_t* __restrict__ dx,
                                                         bf16_t* __restrict__ dres, int64_t nvec, int C, int relu) {
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    const int c = (int)((v * 8) % C);
    float d[8];
    unpack8(((const uint4*)dy)[v], d);
    if (relu) {
      float yv[8];
      unpack8(((const uint4*)y)[v], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
    }
    if (dres) ((uint4*)dres)[v] = pack8(d);
    float o[8], sc[8];
    *(float4*)&sc[0] = *(const float4*)(scale + c); *(float4*)&sc[4] = *(const float4*)(scale + c + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = sc[j] * d[j];
    ((uint4*)dx)[v] = pack8(o);
  }
}

// ------------------------------------------------ ResNet stem: BN apply + ReLU + MaxPool, fused
// The stem's BN/ReLU output is the largest activation of the network (64 x 112 x 112 per image)
// and its only consumer is the 3x3/2 max pool.  Forward reads the conv output c and pools
// relu(c*scale + shift) directly (values rounded to bf16 before the compare, so the arg-max and
// torch's first-max tie rule match the unfused bn -> relu -> maxpool chain); the full-resolution
// activation is never written.  Backward recomputes the mask from c instead of reading it:
// pass 1 (STATS) gathers dz = [y > 0] * sum(dpool routed by the arg-max) per input pixel and
// reduces (sum dz, sum dz*(c - mean)) into the BN backward slab; pass 2 (APPLY) regathers dz and
// writes dc = k0*dz + k1*c + k2.  Neither pass writes dz.
__global__ __launch_bounds__(NT) void bnpool_fwd_kernel(const bf16_t* __restrict__ c, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                        uint8_t* __restrict__ idx, int Nb, int H, int W, int C, int P,
                                                        int Q, int k, int s, int pad) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)Nb * P * Q * C8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c8 = (int)(t % C8);
    int64_t pix = t / C8;
    const int q = (int)(pix % Q); pix /= Q;
    const int p = (int)(pix % P);
    const int n = (int)(pix / P);
    float a[8], b[8], best[8];
    uint8_t bi[8];
    *(float4*)&a[0] = *(const float4*)(scale + c8 * 8); *(float4*)&a[4] = *(const float4*)(scale + c8 * 8 + 4);
    *(float4*)&b[0] = *(const float4*)(shift + c8 * 8); *(float4*)&b[4] = *(const float4*)(shift + c8 * 8 + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int r = 0; r < k; ++r) {
      const int ih = p * s - pad + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int cc = 0; cc < k; ++cc) {
        const int iw = q * s - pad + cc;
        if ((unsigned)iw >= (unsigned)W) continue;
        float f[8];
        unpack8(*(const uint4*)(c + (((size_t)n * H + ih) * W + iw) * C + c8 * 8), f);
        const uint8_t tap = (uint8_t)(r * k + cc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(f2bf(fmaxf(f[j] * a[j] + b[j], 0.f)));
          if (v > best[j]) { best[j] = v; bi[j] = tap; }
        }
      }
    }
    const size_t o = (size_t)t * 8;
    *(uint4*)(y + o) = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *(uint2*)(idx + o) = packed;
  }
}

// dz (8 channels at input pixel (n,h,w), channel base cc) from the pooled gradient, the arg-max
// taps and the conv output (relu mask recomputed); also returns the 8 conv outputs.
__device__ __forceinline__ void bnpool_dz(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                          const bf16_t* __restrict__ c, const float* a, const float* b, int n,
                                          int h, int w, int cc, int H, int W, int C, int P, int Q, int k, int s,
                                          int pad, float* dz, float* cv) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int p_lo = max(0, (h + pad - k + s) / s), p_hi = min(P - 1, (h + pad) / s);
  const int q_lo = max(0, (w + pad - k + s) / s), q_hi = min(Q - 1, (w + pad) / s);
  for (int p = p_lo; p <= p_hi; ++p) {
    const int r = h + pad - p * s;
    if (r < 0 || r >= k) continue;
    for (int q = q_lo; q <= q_hi; ++q) {
      const int t = w + pad - q * s;
      if (t < 0 || t >= k) continue;
      const size_t o = (((size_t)n * P + p) * Q + q) * C + cc;
      const uint2 ii = *(const uint2*)(idx + o);
      float g[8];
      unpack8(*(const uint4*)(dy + o), g);
      const uint32_t tap = (uint32_t)(r * k + t);
      const uint32_t wds[2] = {ii.x, ii.y};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((wds[j >> 2] >> (8 * (j & 3))) & 0xffu) == tap) acc[j] += g[j];
    }
  }
  unpack8(*(const uint4*)(c + (((size_t)n * H + h) * W + w) * C + cc), cv);
#pragma unroll
  for (int j = 0; j < 8; ++j) dz[j] = bf2f(f2bf(cv[j] * a[j] + b[j])) > 0.f ? acc[j] : 0.f;
}

__global__ __launch_bounds__(NT) void bnpool_bwd_stats_kernel(const bf16_t* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              const bf16_t* __restrict__ c,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ mean,
                                                              float* __restrict__ part, int Nb, int H, int W, int C,
                                                              int P, int Q, int k, int s, int pad,
                                                              int rows_per_block) {
  const SlabGeom g = slab_geom(C);
  const int tid = threadIdx.x;
  const int c8 = tid % g.tpr, r0 = tid / g.tpr;
  const int cbase = blockIdx.y * g.cw;
  const int cc = cbase + c8 * 8;
  const int M = Nb * H * W;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  float a[8], b[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = scale[cc + j]; b[j] = shift[cc + j]; mu[j] = mean[cc + j]; }
  float sd[8] = {0}, sq[8] = {0};
  for (int r = rb + r0; r < re; r += g.rp) {
    const int w = r % W, nh = r / W;
    const int h = nh % H, n = nh / H;
    float dz[8], cv[8];
    bnpool_dz(dy, idx, c, a, b, n, h, w, cc, H, W, C, P, Q, k, s, pad, dz, cv);
#pragma unroll
    for (int j = 0; j < 8; ++j) { sd[j] += dz[j]; sq[j] += dz[j] * (cv[j] - mu[j]); }
  }
  block_reduce_store(sd, sq, part, C, cbase, g);
}

__global__ __launch_bounds__(NT) void bnpool_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              const bf16_t* __restrict__ c,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ coef,
                                                              bf16_t* __restrict__ dc, int Nb, int H, int W, int C,
                                                              int P, int Q, int k, int s, int pad) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)Nb * H * W * C8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c8 = (int)(t % C8);
    int64_t pix = t / C8;
    const int w = (int)(pix % W); pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    const int cc = c8 * 8;
    float a[8], b[8], k0[8], k1[8], k2[8];
    *(float4*)&a[0] = *(const float4*)(scale + cc); *(float4*)&a[4] = *(const float4*)(scale + cc + 4);
    *(float4*)&b[0] = *(const float4*)(shift + cc); *(float4*)&b[4] = *(const float4*)(shift + cc + 4);
    float dz[8], cv[8], o[8];
    bnpool_dz(dy, idx, c, a, b, n, h, w, cc, H, W, C, P, Q, k, s, pad, dz, cv);
    *(float4*)&k0[0] = *(const float4*)(coef + cc); *(float4*)&k0[4] = *(const float4*)(coef + cc + 4);
    *(float4*)&k1[0] = *(const float4*)(coef + C + cc); *(float4*)&k1[4] = *(const float4*)(coef + C + cc + 4);
    *(float4*)&k2[0] = *(const float4*)(coef + 2 * C + cc); *(float4*)&k2[4] = *(const float4*)(coef + 2 * C + cc + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = k0[j] * dz[j] + k1[j] * cv[j] + k2[j];
    *(uint4*)(dc + (size_t)t * 8) = pack8(o);
  }
}

// k=3, s=2, pad=1 (every ResNet stem) specialisations.  Forward: one thread per (output pixel,
// 8 channels), all nine 16-byte taps issued before the first compare (out-of-image taps load the
// always-valid centre and are skipped).  Backward: one thread per output pixel (p,q) owns the 2x2
// input pixels (2p..2p+1, 2q..2q+1), whose gradients come only from windows (p..p+1, q..q+1):
//   (0,0) <- W00 tap 4;  (0,1) <- W00 tap 5, W01 tap 3;  (1,0) <- W00 tap 7, W10 tap 1;
//   (1,1) <- W00 tap 8, W01 tap 6, W10 tap 2, W11 tap 0   (same summation order as the gather).
// 4 window loads + 4 pixel loads per thread, all independent, 32-bit index math.
__global__ __launch_bounds__(NT) void bnpool3_fwd_kernel(const bf16_t* __restrict__ c, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int H, int W, int C, int P, int Q,
                                                         int total) {
  const int C8 = C / 8;
  for (int t = blockIdx.x * NT + threadIdx.x; t < total; t += gridDim.x * NT) {
    const int c8 = t % C8;
    const int pix = t / C8;
    const int q = pix % Q, np = pix / Q;
    const int p = np % P, n = np / P;
    const int cc = c8 * 8;
    const bf16_t* base = c + ((size_t)n * H * W) * C + cc;
    const int h0 = 2 * p, w0 = 2 * q;
    uint4 v[9];
    bool ok[9];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int ih = h0 - 1 + r, iw = w0 - 1 + u;
        const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        ok[r * 3 + u] = in;
        v[r * 3 + u] = epi_ld16<kBnxNt>(base + ((size_t)(in ? ih : h0) * W + (in ? iw : w0)) * C);
      }
    }
    float a[8], b[8], best[8];
    uint32_t bi[8];
    *(float4*)&a[0] = *(const float4*)(scale + cc); *(float4*)&a[4] = *(const float4*)(scale + cc + 4);
    *(float4*)&b[0] = *(const float4*)(shift + cc); *(float4*)&b[4] = *(const float4*)(shift + cc + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      if (!ok[tp]) continue;
      float f[8];
      unpack8(v[tp], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = bf2f(f2bf(fmaxf(f[j] * a[j] + b[j], 0.f)));
        if (val > best[j]) { best[j] = val; bi[j] = tp; }
      }
    }
    const size_t o = (size_t)t * 8;
    *(uint4*)(y + o) = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(idx + o) = packed;
  }
}

__device__ __forceinline__ uint32_t tap_of(const uint2& ii, int j) {
  return ((j < 4 ? ii.x : ii.y) >> (8 * (j & 3))) & 0xffu;
}

// dz and c of the 2x2 input pixels owned by output pixel (n,p,q), channels cc..cc+7.
// valid[i]: pixel i = (dh,dw) = (i>>1, i&1) lies inside the image.
__device__ __forceinline__ void bnpool3_quad(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                             const bf16_t* __restrict__ c, const float* a, const float* b, int n,
                                             int p, int q, int cc, int H, int W, int C, int P, int Q, float dz[4][8],
                                             float cv[4][8], bool valid[4]) {
  const bool pn = p + 1 < P, qn = q + 1 < Q;
  const size_t o00 = (((size_t)n * P + p) * Q + q) * C + cc;
  const size_t o01 = qn ? o00 + C : o00, o10 = pn ? o00 + (size_t)Q * C : o00;
  const size_t o11 = (pn && qn) ? o00 + (size_t)Q * C + C : o00;
  const uint4 g00 = epi_ld16<kBnxNt>(dy + o00), g01 = epi_ld16<kBnxNt>(dy + o01);
  const uint4 g10 = epi_ld16<kBnxNt>(dy + o10), g11 = epi_ld16<kBnxNt>(dy + o11);
  const uint2 i00 = *(const uint2*)(idx + o00), i01 = *(const uint2*)(idx + o01);
  const uint2 i10 = *(const uint2*)(idx + o10), i11 = *(const uint2*)(idx + o11);
  const int h0 = 2 * p, w0 = 2 * q;
  uint4 xv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = h0 + (i >> 1), w = w0 + (i & 1);
    valid[i] = h < H && w < W;
    xv[i] = epi_ld16<kBnxNt>(c + (((size_t)n * H + (valid[i] ? h : h0)) * W + (valid[i] ? w : w0)) * C + cc);
  }
  float f00[8], f01[8], f10[8], f11[8];
  unpack8(g00, f00); unpack8(g01, f01); unpack8(g10, f10); unpack8(g11, f11);
#pragma unroll
  for (int i = 0; i < 4; ++i) unpack8(xv[i], cv[i]);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t t00 = tap_of(i00, j), t01 = qn ? tap_of(i01, j) : 0xffu;
    const uint32_t t10 = pn ? tap_of(i10, j) : 0xffu, t11 = (pn && qn) ? tap_of(i11, j) : 0xffu;
    float acc[4];
    acc[0] = t00 == 4u ? f00[j] : 0.f;
    acc[1] = (t00 == 5u ? f00[j] : 0.f) + (t01 == 3u ? f01[j] : 0.f);
    acc[2] = (t00 == 7u ? f00[j] : 0.f) + (t10 == 1u ? f10[j] : 0.f);
    acc[3] = (t00 == 8u ? f00[j] : 0.f) + (t01 == 6u ? f01[j] : 0.f) + (t10 == 2u ? f10[j] : 0.f) +
             (t11 == 0u ? f11[j] : 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) dz[i][j] = bf2f(f2bf(cv[i][j] * a[j] + b[j])) > 0.f ? acc[i] : 0.f;
  }
}

__global__ __launch_bounds__(NT) void bnpool3_bwd_stats_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               const bf16_t* __restrict__ c,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift,
                                                               const float* __restrict__ mean,
                                                               float* __restrict__ part, int Nb, int H, int W, int C,
                                                               int P, int Q, int rows_per_block) {
  const SlabGeom g = slab_geom(C);
  const int tid = threadIdx.x;
  const int c8 = tid % g.tpr, r0 = tid / g.tpr;
  const int cbase = blockIdx.y * g.cw;
  const int cc = cbase + c8 * 8;
  const int M = Nb * P * Q;
  const int rb = blockIdx.x * rows_per_block, re = min(M, rb + rows_per_block);
  float a[8], b[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = scale[cc + j]; b[j] = shift[cc + j]; mu[j] = mean[cc + j]; }
  float sd[8] = {0}, sq[8] = {0};
  for (int r = rb + r0; r < re; r += g.rp) {
    const int q = r % Q, np = r / Q;
    const int p = np % P, n = np / P;
    float dz[4][8], cv[4][8];
    bool valid[4];
    bnpool3_quad(dy, idx, c, a, b, n, p, q, cc, H, W, C, P, Q, dz, cv, valid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!valid[i]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) { sd[j] += dz[i][j]; sq[j] += dz[i][j] * (cv[i][j] - mu[j]); }
    }
  }
  block_reduce_store(sd, sq, part, C, cbase, g);
}

__global__ __launch_bounds__(NT) void bnpool3_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               const bf16_t* __restrict__ c,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift,
                                                               const float* __restrict__ coef,
                                                               bf16_t* __restrict__ dc, int H, int W, int C, int P,
                                                               int Q, int total) {
  const int C8 = C / 8;
  for (int t = blockIdx.x * NT + threadIdx.x; t < total; t += gridDim.x * NT) {
    const int c8 = t % C8;
    const int pix = t / C8;
    const int q = pix % Q, np = pix / Q;
    const int p = np % P, n = np / P;
    const int cc = c8 * 8;
    float a[8], b[8], k0[8], k1[8], k2[8];
    *(float4*)&a[0] = *(const float4*)(scale + cc); *(float4*)&a[4] = *(const float4*)(scale + cc + 4);
    *(float4*)&b[0] = *(const float4*)(shift + cc); *(float4*)&b[4] = *(const float4*)(shift + cc + 4);
    *(float4*)&k0[0] = *(const float4*)(coef + cc); *(float4*)&k0[4] = *(const float4*)(coef + cc + 4);
    *(float4*)&k1[0] = *(const float4*)(coef + C + cc); *(float4*)&k1[4] = *(const float4*)(coef + C + cc + 4);
    *(float4*)&k2[0] = *(const float4*)(coef + 2 * C + cc); *(float4*)&k2[4] = *(const float4*)(coef + 2 * C + cc + 4);
    float dz[4][8], cv[4][8];
    bool valid[4];
    bnpool3_quad(dy, idx, c, a, b, n, p, q, cc, H, W, C, P, Q, dz, cv, valid);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!valid[i]) continue;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k0[j] * dz[i][j] + k1[j] * cv[i][j] + k2[j];
      *(uint4*)(dc + (((size_t)n * H + 2 * p + (i >> 1)) * W + 2 * q + (i & 1)) * C + cc) = pack8(o);
    }
  }
}

// grid of the elementwise BN passes: one EW_U-vector batch per thread, capped at
// MI355X_DP_EW_GRID_CAP blocks (default kEwGridCap; a cap near the resident block count turns
// the launch into a grid-stride sweep without block turnover)
inline int ew_grid_cap() {
  static int cap = -1;
  if (cap < 0) {
    const char* e = std::getenv("MI355X_DP_EW_GRID_CAP");
    cap = (e && std::atoi(e) > 0) ? std::atoi(e) : kEwGridCap;
  }
  return cap;
}

inline int ew_grid(int64_t nvec) {
  int64_t g = (nvec + NT * EW_U - 1) / (NT * EW_U);
  const int cap = ew_grid_cap();
  return (int)(g < cap ? g : cap);
}

// channel octet fixed per thread for the whole grid-stride pass (bn_apply_kernel_t FIXC)
inline bool ew_fixc(int grid, int C) { return ((int64_t)grid * NT * 8) % C == 0; }

template <bool RES_BN>
inline void launch_bn_apply(const void* x, const void* res, void* y, const float* scale, const float* shift,
                            const float* rscale, const float* rshift, int64_t nvec, int C, int relu, hipStream_t st,
                            void* bits = nullptr) {
  const int grid = ew_grid(nvec);
  if (ew_fixc(grid, C))
    hipLaunchKernelGGL((bn_apply_kernel_t<RES_BN, true>), dim3(grid), dim3(NT), 0, st, (const bf16_t*)x,
                       (const bf16_t*)res, (bf16_t*)y, scale, shift, rscale, rshift, nvec, C, relu, (uint8_t*)bits);
  else
    hipLaunchKernelGGL((bn_apply_kernel_t<RES_BN, false>), dim3(grid), dim3(NT), 0, st, (const bf16_t*)x,
                       (const bf16_t*)res, (bf16_t*)y, scale, shift, rscale, rshift, nvec, C, relu, (uint8_t*)bits);
}

inline void launch_bn_bwd_apply(const void* dy, const void* y, const void* x, const float* coef, void* dx, void* dres,
                                int64_t nvec, int C, int relu, hipStream_t st) {
  const int grid = ew_grid(nvec);
  if (ew_fixc(grid, C))
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(grid), dim3(NT), 0, st, (const bf16_t*)dy, (const bf16_t*)y,
                       (const bf16_t*)x, coef, (bf16_t*)dx, (bf16_t*)dres, nvec, C, relu);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(grid), dim3(NT), 0, st, (const bf16_t*)dy, (const bf16_t*)y,
                       (const bf16_t*)x, coef, (bf16_t*)dx, (bf16_t*)dres, nvec, C, relu);
}

// Small BatchNorm layers (ResNet-18 on 32x32 images at 32 per GPU: 32-2048 rows): the slab
// finalize and the apply in ONE launch.  Block (cg, rb) reduces the slab for channels
// [64 cg, 64 cg + 64) itself -- a few KB, read by every row block of the channel group, in a fixed
// order, so every block computes identical coefficients -- and applies them to its rows; only
// row block 0 writes the statistics outputs (running statistics, saved mean / invstd, scale /
// shift; backward: dgamma / dbeta).  Saves a launch and a dependent kernel boundary per BN per
// direction (~40 per step of the reference's per-GPU shape, where each cost ~5 us).
constexpr int SMALL_T = 256, SMALL_G = SMALL_T / 64;
constexpr int64_t kBnSmallElems = 1 << 20;  // M * C at or below which the fused path runs

__device__ __forceinline__ void small_slab_reduce(const float* __restrict__ part, int nblk, int C, int c, double& s,
                                                  double& q, double (*red)[SMALL_G][64]) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  double a = 0.0, b = 0.0;
  if (c < C)
    for (int i = rg; i < nblk; i += SMALL_G) {
      a += part[(size_t)(2 * i) * C + c];
      b += part[(size_t)(2 * i + 1) * C + c];
    }
  red[0][rg][cl] = a;
  red[1][rg][cl] = b;
  __syncthreads();
  s = red[0][0][cl]; q = red[1][0][cl];
  for (int g = 1; g < SMALL_G; ++g) { s += red[0][g][cl]; q += red[1][g][cl]; }
}

template <bool BWD>
__global__ __launch_bounds__(SMALL_T) void bn_small_fin_apply_kernel(const bf16_t* __restrict__ x,
                                                                     const bf16_t* __restrict__ res_or_dz,
                                                                     bf16_t* __restrict__ out, const float* part,
                                                                     int nblk, FinArgs f, int rows_per, int relu) {
  __shared__ double red[2][SMALL_G][64];
  __shared__ float k[3][64];
  const int C = f.C, M = f.M;
  const int cl = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + cl;
  double s, q;
  small_slab_reduce(part, nblk, C, c, s, q, red);
  if (threadIdx.x < 64 && c < C) {
    // every row block computes the same coefficients; row block 0 also publishes the outputs
    float tmp[3];
    if (BWD) {
      const float is = f.invstd[c];
      const float sum_dz = (float)s, sum_dzx = (float)q * is;
      const float gm = f.gamma ? f.gamma[c] : 1.f;
      const float k0 = gm * is, mdz = sum_dz / M, mdzx = sum_dzx / M;
      const float k1 = -k0 * is * mdzx;
      tmp[0] = k0; tmp[1] = k1; tmp[2] = -k0 * mdz - k1 * f.mean[c];
      if (blockIdx.y == 0) {
        if (f.dgamma) f.dgamma[c] += sum_dzx;
        if (f.dbeta) f.dbeta[c] += sum_dz;
      }
    } else {
      const double mean = s / M;
      double var = q / M - mean * mean;
      if (var < 0) var = 0;
      const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
      const float gm = f.gamma ? f.gamma[c] : 1.f, bt = f.beta ? f.beta[c] : 0.f;
      tmp[0] = gm * invstd;
      tmp[1] = bt - (float)mean * gm * invstd;
      tmp[2] = 0.f;
      if (blockIdx.y == 0) {
        f.save_mean[c] = (float)mean;
        f.save_invstd[c] = invstd;
        f.scale[c] = tmp[0];
        f.shift[c] = tmp[1];
        if (f.rmean) {
          const double unbiased = M > 1 ? var * M / (M - 1) : var;
          f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * (float)mean;
          f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * (float)unbiased;
        }
        if (cl == 0 && blockIdx.x == 0 && f.nbt) f.nbt[0] += 1;
      }
    }
    k[0][cl] = tmp[0]; k[1][cl] = tmp[1]; k[2][cl] = tmp[2];
  }
  __syncthreads();
  // apply: 8 threads per row (8 channels each), 32 rows per pass
  const int ch = (threadIdx.x & 7) * 8, rsub = threadIdx.x >> 3;
  const int cbase = blockIdx.x * 64 + ch;
  if (cbase >= C) return;
  float a0[8], a1[8], a2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a0[j] = k[0][ch + j]; a1[j] = k[1][ch + j]; a2[j] = k[2][ch + j]; }
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  for (int r = r0 + rsub; r < r1; r += SMALL_T / 8) {
    const size_t off = (size_t)r * C + cbase;
    float v[8], o[8];
    unpack8(*(const uint4*)(x + off), v);
    if (BWD) {  // dx = k0 dz + k1 x + k2
      float d[8];
      unpack8(*(const uint4*)(res_or_dz + off), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = a0[j] * d[j] + a1[j] * v[j] + a2[j];
    } else {   // y = act(x scale + shift (+ res))
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[j] * a0[j] + a1[j];
      if (res_or_dz) {
        float rv[8];
        unpack8(*(const uint4*)(res_or_dz + off), rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rv[j];
      }
      if (relu)
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    *(uint4*)(out + off) = pack8(o);
  }
}

static int64_t g_bn_small_elems = -1;  // MI355X_DP_BN_SMALL_ELEMS, or mi_bn_set_small_elems (tests)
inline bool bn_small(int M, int C, int nblk) {
  if (g_bn_small_elems < 0) {
    const char* e = std::getenv("MI355X_DP_BN_SMALL_ELEMS");
    g_bn_small_elems = e ? std::max(0LL, std::atoll(e)) : kBnSmallElems;
  }
  return (int64_t)M * C <= g_bn_small_elems && C % 64 == 0 && nblk <= 256 && M > 0;
}

inline void launch_bn_small(bool bwd, const void* x, const void* res_or_dz, void* out, const float* part, int nblk,
                            const FinArgs& f, int relu, hipStream_t st) {
  const int rows_per = 128;
  const dim3 grid(cdiv(f.C, 64), cdiv(f.M, rows_per));
  if (bwd)
    hipLaunchKernelGGL(bn_small_fin_apply_kernel<true>, grid, dim3(SMALL_T), 0, st, (const bf16_t*)x,
                       (const bf16_t*)res_or_dz, (bf16_t*)out, part, nblk, f, rows_per, relu);
  else
    hipLaunchKernelGGL(bn_small_fin_apply_kernel<false>, grid, dim3(SMALL_T), 0, st, (const bf16_t*)x,
                       (const bf16_t*)res_or_dz, (bf16_t*)out, part, nblk, f, rows_per, relu);
}

inline void slab_launch_dims(int M, int C, int& nblk, int& rows_per_block, dim3& grid) {
  SlabGeom g = slab_geom(C);
  int ncs = C / g.cw;
  // ~2048 blocks in total, each handling >= 4*rp rows
  int target = std::max(1, 1024 / ncs);
  rows_per_block = std::max(g.rp * 4, cdiv(M, target));
  rows_per_block = cdiv(rows_per_block, g.rp) * g.rp;
  nblk = cdiv(M, rows_per_block);
  grid = dim3(nblk, ncs);
}

// Tall slabs (e.g. one row per conv M-tile) are first reduced by a (C/64) x S grid into S rows
// written just past the slab (callers allocate SLAB_EXTRA_ROWS spare rows), then finalized.
// split rows: the split stage is latency-bound (a 6272-row x 256-channel slab is 12.8 MB read by
// S x C/64 blocks), so tall slabs are cut into more, shorter splits (kSlabSplitRows rows each;
// A/B on RN50 bs256: 16 rows 22.38 ms, 32 22.03, 64 21.89, 128 21.87, 256 22.04 ms/step)
constexpr int kSlabSplitRows = 128;
constexpr int SLAB_EXTRA_ROWS = 256;

inline int tall_slab_split(float* part, int nblk, int C, hipStream_t st, const float*& fin) {
  fin = part;
  if (nblk <= 256) return nblk;
  const int S = std::min(SLAB_EXTRA_ROWS, cdiv(nblk, kSlabSplitRows));
  const int rows_per = cdiv(nblk, S);
  float* out = part + (size_t)nblk * 2 * C;
  hipLaunchKernelGGL(slab_split_kernel, dim3(cdiv(C, 64), S), dim3(FIN_T), 0, st, part, nblk, C, rows_per, out);
  fin = out;
  return S;
}

// Arrival counters of slab_split_fin_kernel (one per 64-channel group, reset by the finalizing
// block).  Two finalizes in flight on DIFFERENT streams must not share counters, so every (device,
// stream) gets its own slot of a table allocated up front by mi_bn_init_counters() (called when
// the library is loaded -- never lazily, which would break a HIP graph capture).  A stream beyond
// the table, or a device that was never initialised, takes the two-launch split + finalize path,
// which needs no counters (deterministic either way; the two paths may round differently in the last
// bit, so every rank of a job must use the same streams -- which the engine guarantees).
constexpr int FIN_STREAM_SLOTS = 16, FIN_GROUPS = 128;  // 128 x 64 = 8192 channels
// per stream slot: FIN_GROUPS arrival counters, then 8 words of the fused finalize + apply launch
// (bn_bwd_fin_apply_kernel: [0] groups finalized, [1] ready, [2] readers + raiser, [3] fallbacks)
constexpr int FIN_SLOT = FIN_GROUPS + 8;
struct FinCounters {
  int* cnt = nullptr;  // [FIN_STREAM_SLOTS][FIN_SLOT]
  hipStream_t owner[FIN_STREAM_SLOTS] = {};
  bool used[FIN_STREAM_SLOTS] = {};
};
static FinCounters g_fin_cnt[16];
static std::mutex g_fin_mu;

static int* fin_counters(int groups, hipStream_t st) {
  if (groups > FIN_GROUPS) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_fin_mu);
  FinCounters& w = g_fin_cnt[dev & 15];
  if (!w.cnt) return nullptr;
  for (int i = 0; i < FIN_STREAM_SLOTS; ++i)
    if (w.used[i] && w.owner[i] == st) return w.cnt + i * FIN_SLOT;
  for (int i = 0; i < FIN_STREAM_SLOTS; ++i)
    if (!w.used[i]) {
      w.used[i] = true;
      w.owner[i] = st;
      return w.cnt + i * FIN_SLOT;
    }
  // table full: the counter-free two-launch path (no host synchronisation, safe inside a capture)
  return nullptr;
}

// finalize a [nblk][2][C] partial slab: one launch (finalize, or split + finalize for tall slabs)
template <bool BWD>
inline void slab_finalize(float* part, int nblk, const FinArgs& f, hipStream_t st) {
  const int C = f.C;
  int* cnt = nblk > 256 ? fin_counters(cdiv(C, 64), st) : nullptr;
  if (cnt) {
    const int S = std::min(SLAB_EXTRA_ROWS, cdiv(nblk, kSlabSplitRows));
    const int rows_per = cdiv(nblk, S);
    float* out = part + (size_t)nblk * 2 * C;
    hipLaunchKernelGGL(slab_split_fin_kernel<BWD>, dim3(cdiv(C, 64), S), dim3(FIN_T), 0, st, part, nblk, rows_per,
                       out, cnt, f);
    return;
  }
  const float* fin = part;
  const int n = tall_slab_split(part, nblk, C, st, fin);
  if (BWD) hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 64)), dim3(FIN_T), 0, st, fin, n, f);
  else hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 64)), dim3(FIN_T), 0, st, fin, n, f);
}

// BN backward of a tall slab as ONE launch (bn_bwd_fin_apply_kernel) instead of split-finalize +
// apply; false: the caller takes the two-launch path (MI355X_DP_BN_FUSED_FIN=0, small slabs, wide
// layers, a stream without a counter slot, or a grid on which a thread's channel octet would move)
// MI355X_DP_BN_FUSED_FIN=1 enables it (mi_bn_set_fused_fin: tests).  OFF by default: on ResNet-50
// bs256 it measured 12.49k / 12.48k img/s against 12.74k / 12.69k for the two-launch path on one box
// (512 apply blocks: 12.36k; profiles/bn_fused_finalize_r5.md) -- the apply blocks can do nothing
// useful while the coefficients are finalized, and the persistent sweep at one 512-thread block per
// CU (141-157 VGPRs) moves bytes slower than the 256-thread launch it replaces.
static int g_bn_fused_fin = -1;
inline bool launch_bn_bwd_fused(const float* part, int nblk, const FinArgs& f, const void* dy, const void* y,
                                const void* x, void* dx, void* dres, int relu, hipStream_t st) {
  if (g_bn_fused_fin < 0) {
    const char* e = std::getenv("MI355X_DP_BN_FUSED_FIN");
    g_bn_fused_fin = (e && e[0] == '1') ? 1 : 0;
  }
  const int C = f.C;
  if (!g_bn_fused_fin || nblk <= 256 || C > FUSED_MAX_C || C % 8) return false;
  int* cnt = fin_counters(cdiv(C, 64), st);
  if (!cnt) return false;
  FusedBwdArgs a{};
  // splits of 64 rows: with 8 row groups a thread loads 8 rows -- one round of FIN_U loads
  a.S = std::min(SLAB_EXTRA_ROWS, cdiv(nblk, 64));
  a.rows_per = cdiv(nblk, a.S);
  a.G = cdiv(C, 64);
  a.nvec = (int64_t)f.M * C / 8;
  // a persistent sweep: about one apply block per CU (MI355X_DP_BN_FUSED_BLOCKS), so the blocks that
  // wait for the coefficients -- and count themselves out with one atomic each -- are few
  static int cap = -1;
  if (cap < 0) {
    const char* e = std::getenv("MI355X_DP_BN_FUSED_BLOCKS");
    cap = (e && std::atoi(e) > 0) ? std::atoi(e) : 256;
  }
  a.A = (int)std::max<int64_t>(
      1, std::min<int64_t>(cap, (a.nvec + (int64_t)FUSED_T * EW_U - 1) / ((int64_t)FUSED_T * EW_U)));
  if (((int64_t)a.A * FUSED_T * 8) % C) return false;  // a thread's channel octet must stay fixed
  a.part = part; a.nblk = nblk; a.out = const_cast<float*>(part) + (size_t)nblk * 2 * C; a.cnt = cnt;
  a.sync = (uint32_t*)(cnt + FIN_GROUPS);
  a.f = f;
  a.dy = (const bf16_t*)dy; a.y = (const bf16_t*)y; a.x = (const bf16_t*)x; a.dx = (bf16_t*)dx;
  a.dres = (bf16_t*)dres; a.relu = relu;
  const dim3 grid(a.G * a.S + a.A);
  if (relu) hipLaunchKernelGGL(bn_bwd_fin_apply_kernel<true>, grid, dim3(FUSED_T), 0, st, a);
  else hipLaunchKernelGGL(bn_bwd_fin_apply_kernel<false>, grid, dim3(FUSED_T), 0, st, a);
  return true;
}

inline FinArgs fin_fwd_args(int M, int C, float eps, float momentum, const float* gamma, const float* beta,
                            float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                            float* scale, float* shift) {
  FinArgs f{};
  f.M = M; f.C = C; f.eps = eps; f.momentum = momentum; f.gamma = gamma; f.beta = beta;
  f.rmean = rmean; f.rvar = rvar; f.nbt = nbt; f.save_mean = save_mean; f.save_invstd = save_invstd;
  f.scale = scale; f.shift = shift;
  return f;
}

inline FinArgs fin_bwd_args(int M, int C, const float* gamma, const float* mean, const float* invstd, float* dgamma,
                            float* dbeta, float* coef) {
  FinArgs f{};
  f.M = M; f.C = C; f.gamma = gamma; f.mean = mean; f.invstd = invstd; f.dgamma = dgamma; f.dbeta = dbeta;
  f.coef = coef;
  return f;
}

}  // namespace

MI_API int mi_bn_slab_extra_rows() { return SLAB_EXTRA_ROWS; }

MI_API int mi_bn_set_fused_fin(int on) {
  g_bn_fused_fin = on ? 1 : 0;
  return 0;
}

// fused finalize + apply launches whose apply blocks gave up waiting (diagnostics; tests assert 0)
MI_API int mi_bn_fused_fallbacks() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> lk(g_fin_mu);
  FinCounters& w = g_fin_cnt[dev & 15];
  if (!w.cnt) return 0;
  int host[FIN_STREAM_SLOTS * FIN_SLOT];
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(host, w.cnt, sizeof(host), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  int n = 0;
  for (int i = 0; i < FIN_STREAM_SLOTS; ++i) n += host[i * FIN_SLOT + FIN_GROUPS + 3];
  return n;
}

// threshold (M * C elements) of the fused small-layer finalize + apply path; 0 disables (tests)
MI_API int mi_bn_set_small_elems(long long n) {
  g_bn_small_elems = n < 0 ? 0 : (int64_t)n;
  return 0;
}

// Allocate the current device's finalize-counter table (zeroed, synchronously).  Idempotent; call
// before any graph capture (the Python loader does, at library load).
MI_API int mi_bn_init_counters() {
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return (int)e;
  std::lock_guard<std::mutex> lk(g_fin_mu);
  FinCounters& w = g_fin_cnt[dev & 15];
  if (w.cnt) return 0;
  int* p = nullptr;
  const size_t bytes = sizeof(int) * FIN_STREAM_SLOTS * FIN_SLOT;
  if (hipError_t e = hipMalloc(&p, bytes); e != hipSuccess) return (int)e;
  if (hipError_t e = hipMemset(p, 0, bytes); e != hipSuccess) return (int)e;
  if (hipError_t e = hipDeviceSynchronize(); e != hipSuccess) return (int)e;
  w.cnt = p;
  return 0;
}

MI_API int mi_bn_partial_rows(int M, int C) {
  int nblk, rpb; dim3 grid;
  slab_launch_dims(M, C, nblk, rpb, grid);
  return nblk;
}

// Training-mode forward.  part: fp32 workspace [mi_bn_partial_rows(M,C)][2][C], or -- when
// pre_rows > 0 -- a [pre_rows][2][C] slab of (sum, sumsq) already written by the conv epilogue.
MI_API int mi_bn_fwd_train(const void* x, const void* res, void* y, int M, int C, float eps, float momentum,
                           const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
                           float* save_mean, float* save_invstd, float* scale, float* shift, float* part,
                           int pre_rows, int relu, hipStream_t st) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  int nblk, rpb; dim3 grid;
  slab_launch_dims(M, C, nblk, rpb, grid);
  if (pre_rows > 0) {
    nblk = pre_rows;  // partials already produced by the producing conv's epilogue
  } else {
    hipLaunchKernelGGL(bn_stats_kernel, grid, dim3(NT), 0, st, (const bf16_t*)x, part, M, C, rpb);
  }
  const FinArgs fa = fin_fwd_args(M, C, eps, momentum, gamma, beta, rmean, rvar, nbt, save_mean, save_invstd, scale,
                                  shift);
  if (y && bn_small(M, C, nblk)) {  // finalize + apply in one launch
    launch_bn_small(false, x, res, y, part, nblk, fa, relu, st);
    return (int)hipGetLastError();
  }
  slab_finalize<false>(part, nblk, fa, st);
  if (!y) return (int)hipGetLastError();  // statistics + coefficients only (the consumer applies them)
  int64_t nvec = (int64_t)M * C / 8;
  launch_bn_apply<false>(x, res, y, scale, shift, nullptr, nullptr, nvec, C, relu, st);
  return (int)hipGetLastError();
}

// y = act(x*scale + shift + res*rscale + rshift): a block's last BatchNorm (coefficients from
// mi_bn_fwd_train with y = null) fused with its projection shortcut's BatchNorm applied to the raw
// shortcut conv output -- one pass, the shortcut's normalised activation never written.
MI_API int mi_bn_apply_dual(const void* x, const void* res, void* y, int M, int C, const float* scale,
                            const float* shift, const float* rscale, const float* rshift, int relu, hipStream_t st) {
  if (C % 8 != 0 || !x || !res || !y) return (int)hipErrorInvalidValue;
  int64_t nvec = (int64_t)M * C / 8;
  launch_bn_apply<true>(x, res, y, scale, shift, rscale, rshift, nvec, C, relu, st);
  return (int)hipGetLastError();
}

// y = relu(x*scale + shift + res') with res' = res (rscale null) or res*rscale + rshift, plus the
// ReLU mask of y as one byte per 8 channels (bits [M][C/8], bit j = channel 8i+j of y is > 0): a
// block output whose mask the next block's data-gradient epilogue reads instead of y.
MI_API int mi_bn_apply_bits(const void* x, const void* res, void* y, void* bits, int M, int C, const float* scale,
                            const float* shift, const float* rscale, const float* rshift, hipStream_t st) {
  if (C % 8 != 0 || !x || !y || !bits || (rscale && (!res || !rshift))) return (int)hipErrorInvalidValue;
  int64_t nvec = (int64_t)M * C / 8;
  if (rscale)
    launch_bn_apply<true>(x, res, y, scale, shift, rscale, rshift, nvec, C, 1, st, bits);
  else
    launch_bn_apply<false>(x, res, y, scale, shift, nullptr, nullptr, nvec, C, 1, st, bits);
  return (int)hipGetLastError();
}

MI_API int mi_bn_fwd_eval(const void* x, const void* res, void* y, int M, int C, float eps, const float* gamma,
                          const float* beta, const float* rmean, const float* rvar, float* scale, float* shift,
                          int relu, hipStream_t st) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, C, eps, gamma, beta, rmean, rvar,
                     scale, shift);
  int64_t nvec = (int64_t)M * C / 8;
  launch_bn_apply<false>(x, res, y, scale, shift, nullptr, nullptr, nvec, C, relu, st);
  return (int)hipGetLastError();
}

// Training-mode backward.  coef: fp32 [3][C] workspace; dres may be null.
MI_API int mi_bn_bwd_train(const void* dy, const void* y, const void* x, void* dx, void* dres, int M, int C,
                           const float* gamma, const float* save_mean, const float* save_invstd, float* dgamma,
                           float* dbeta, float* coef, float* part, int relu, hipStream_t st) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  int nblk, rpb; dim3 grid;
  slab_launch_dims(M, C, nblk, rpb, grid);
  hipLaunchKernelGGL(bn_bwd_stats_kernel, grid, dim3(NT), 0, st, (const bf16_t*)dy, (const bf16_t*)y,
                     (const bf16_t*)x, save_mean, part, M, C, rpb, relu);
  const FinArgs fb = fin_bwd_args(M, C, gamma, save_mean, save_invstd, dgamma, dbeta, coef);
  if (dx && launch_bn_bwd_fused(part, nblk, fb, dy, y, x, dx, dres, relu, st)) return (int)hipGetLastError();
  slab_finalize<true>(part, nblk, fb, st);
  if (!dx && !dres) return (int)hipGetLastError();  // statistics + coefficients only (a folded consumer)
  int64_t nvec = (int64_t)M * C / 8;
  launch_bn_bwd_apply(dy, y, x, coef, dx, dres, nvec, C, relu, st);
  return (int)hipGetLastError();
}

// BN training backward from statistics a conv dgrad epilogue already produced (epi 4):
// dz (relu already applied), part[pre_rows][2][C] = per-tile (sum dz, sum dz * (x - mean)).
// Skips the statistics pass; dres (optional) <- dz (the residual branch's gradient).
MI_API int mi_bn_bwd_train_pre(const void* dz, const void* x, void* dx, void* dres, int M, int C, const float* gamma,
                               const float* save_mean, const float* save_invstd, float* dgamma, float* dbeta,
                               float* coef, float* part, int pre_rows, hipStream_t st) {
  if (C % 8 != 0 || pre_rows <= 0) return (int)hipErrorInvalidValue;
  const FinArgs fb = fin_bwd_args(M, C, gamma, save_mean, save_invstd, dgamma, dbeta, coef);
  if (!dres && bn_small(M, C, pre_rows)) {  // finalize + apply in one launch
    launch_bn_small(true, x, dz, dx, part, pre_rows, fb, 0, st);
    return (int)hipGetLastError();
  }
  if (launch_bn_bwd_fused(part, pre_rows, fb, dz, nullptr, x, dx, dres, 0, st)) return (int)hipGetLastError();
  slab_finalize<true>(part, pre_rows, fb, st);
  int64_t nvec = (int64_t)M * C / 8;
  launch_bn_bwd_apply(dz, nullptr, x, coef, dx, dres, nvec, C, 0, st);
  return (int)hipGetLastError();
}

// the finalize of mi_bn_bwd_train_pre alone: dgamma / dbeta (+=) and coef = (k0, k1, k2) [3][C] of
// dx = k0 dz + k1 x + k2, for a consumer that folds the BN backward into its GEMM instead of
// reading a materialised dx (conv_panel.hip mi_panel_dgrad_fbb, gemm_conv.hip mi_conv2d_wgrad_fbb)
MI_API int mi_bn_bwd_coef(int M, int C, const float* gamma, const float* save_mean, const float* save_invstd,
                          float* dgamma, float* dbeta, float* coef, float* part, int pre_rows, hipStream_t st) {
  if (C % 8 != 0 || pre_rows <= 0 || !coef) return (int)hipErrorInvalidValue;
  const FinArgs fb = fin_bwd_args(M, C, gamma, save_mean, save_invstd, dgamma, dbeta, coef);
  slab_finalize<true>(part, pre_rows, fb, st);
  return (int)hipGetLastError();
}

MI_API int mi_bn_bwd_eval(const void* dy, const void* y, const float* scale, void* dx, void* dres, int M, int C,
                          int relu, hipStream_t st) {
  int64_t nvec = (int64_t)M * C / 8;
  hipLaunchKernelGGL(bn_bwd_eval_kernel, dim3(ew_grid(nvec)), dim3(NT), 0, st, (const bf16_t*)dy,
                     (const bf16_t*)y, scale, (bf16_t*)dx, (bf16_t*)dres, nvec, C, relu);
  return (int)hipGetLastError();
}

// The gather-bound statistics pass wants more blocks in flight than the plain slab geometry gives.
inline void bnpool_launch_dims(int M, int C, int& nblk, int& rows_per_block, dim3& grid) {
  SlabGeom g = slab_geom(C);
  const int ncs = C / g.cw;
  const int target = std::max(1, 4096 / ncs);
  rows_per_block = std::max(g.rp * 4, cdiv(M, target));
  rows_per_block = cdiv(rows_per_block, g.rp) * g.rp;
  nblk = cdiv(M, rows_per_block);
  grid = dim3(nblk, ncs);
}

MI_API int mi_bnpool_partial_rows(int M, int C) {
  int nblk, rpb; dim3 grid;
  bnpool_launch_dims(M, C, nblk, rpb, grid);
  return nblk;
}

// Stem forward tail: pooled = maxpool(relu(c*scale + shift)), idx = arg-max tap (uint8).
MI_API int mi_bnpool_fwd(const void* c, const float* scale, const float* shift, void* y, void* idx, int Nb, int H,
                         int W, int C, int P, int Q, int k, int s, int pad, hipStream_t st) {
  if (C % 8 || k * k > 255) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)Nb * P * Q * (C / 8);
  const int64_t g = std::min<int64_t>((total + NT - 1) / NT, 16384);
  if (k == 3 && s == 2 && pad == 1 && total < INT32_MAX && (int64_t)Nb * H * W * C < INT32_MAX * 8ll) {
    hipLaunchKernelGGL(bnpool3_fwd_kernel, dim3((int)g), dim3(NT), 0, st, (const bf16_t*)c, scale, shift,
                       (bf16_t*)y, (uint8_t*)idx, H, W, C, P, Q, (int)total);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bnpool_fwd_kernel, dim3((int)g), dim3(NT), 0, st, (const bf16_t*)c, scale, shift, (bf16_t*)y,
                     (uint8_t*)idx, Nb, H, W, C, P, Q, k, s, pad);
  return (int)hipGetLastError();
}

// Stem backward: dpool -> dc (BN training backward through ReLU and MaxPool), dgamma/dbeta += .
// part: [mi_bnpool_partial_rows(Nb*H*W, C) + mi_bn_slab_extra_rows()][2][C] fp32, coef: [3][C] fp32.
MI_API int mi_bnpool_bwd(const void* dy, const void* idx, const void* c, void* dc, int Nb, int H, int W, int C, int P,
                         int Q, int k, int s, int pad, const float* scale, const float* shift, const float* gamma,
                         const float* save_mean, const float* save_invstd, float* dgamma, float* dbeta, float* coef,
                         float* part, hipStream_t st) {
  if (C % 8 || k * k > 255) return (int)hipErrorInvalidValue;
  const int M = Nb * H * W;
  const bool k3 = k == 3 && s == 2 && pad == 1 && (int64_t)M * C < INT32_MAX;
  int nblk, rpb; dim3 grid;
  bnpool_launch_dims(k3 ? Nb * P * Q : M, C, nblk, rpb, grid);
  if (k3)
    hipLaunchKernelGGL(bnpool3_bwd_stats_kernel, grid, dim3(NT), 0, st, (const bf16_t*)dy, (const uint8_t*)idx,
                       (const bf16_t*)c, scale, shift, save_mean, part, Nb, H, W, C, P, Q, rpb);
  else
    hipLaunchKernelGGL(bnpool_bwd_stats_kernel, grid, dim3(NT), 0, st, (const bf16_t*)dy, (const uint8_t*)idx,
                       (const bf16_t*)c, scale, shift, save_mean, part, Nb, H, W, C, P, Q, k, s, pad, rpb);
  slab_finalize<true>(part, nblk, fin_bwd_args(M, C, gamma, save_mean, save_invstd, dgamma, dbeta, coef), st);
  if (k3) {
    const int total3 = Nb * P * Q * (C / 8);
    hipLaunchKernelGGL(bnpool3_bwd_apply_kernel, dim3(std::min(cdiv(total3, NT), 16384)), dim3(NT), 0, st,
                       (const bf16_t*)dy, (const uint8_t*)idx, (const bf16_t*)c, scale, shift, coef, (bf16_t*)dc, H,
                       W, C, P, Q, total3);
    return (int)hipGetLastError();
  }
  const int64_t total = (int64_t)M * (C / 8);
  const int64_t g = std::min<int64_t>((total + NT - 1) / NT, 16384);
  hipLaunchKernelGGL(bnpool_bwd_apply_kernel, dim3((int)g), dim3(NT), 0, st, (const bf16_t*)dy, (const uint8_t*)idx,
                     (const bf16_t*)c, scale, shift, coef, (bf16_t*)dc, Nb, H, W, C, P, Q, k, s, pad);
  return (int)hipGetLastError();
}
