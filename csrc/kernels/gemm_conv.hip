// MFMA implicit-GEMM convolution / GEMM kernels for gfx950 (MI355X, CDNA4).
//
// Replaces the cuDNN conv fwd / bwd-data / bwd-weight and cuBLAS GEMM calls the
// reference reaches through torchvision's ResNet (SURVEY.md §2.5 K1/K2/K3/K10;
// reference hot loop cifar10-distributed-smddp-gpu.py:160-179).  Activations are
// NHWC bf16, accumulation fp32 on v_mfma_f32_16x16x32_bf16.
//
//  * nt_kernel  : C[m][n] = sum_k A[m][k] * B[n][k]   (both operands K-contiguous)
//      - mode 0  plain GEMM (A row stride lda)                     -> Linear fwd / dgrad
//      - mode 1  conv fwd  : A gathered from NHWC input per (r,s) tap  -> Conv fwd
//      - mode 2  conv dgrad: A gathered from NHWC dY (transposed-conv indexing),
//                B = W^T [Cin][R][S][Cout]                         -> Conv bwd-data
//    Tile BMxBNx64, 256 threads = 2x2 waves, register-staged double-buffered LDS,
//    XOR-swizzled 128-B rows (conflict-free ds_read_b128), XCD-aware tile order.
//
//  * tn_kernel  : C[m][n] += sum_k A[k][m] * B[k][n]  (both operands reduction-major)
//      - mode 0 plain, mode 1 conv wgrad (B gathered from NHWC input)
//    LDS tiles stay in global (row = reduction index) order and the MFMA
//    fragments are read transposed with ds_read_b64_tr_b16; split-K over the
//    (huge) N*P*Q reduction with fp32 atomics into the fp32 gradient buffer.
#include "common.h"
#include <algorithm>

namespace {

// ---------------------------------------------------------------- fast division
struct FastDiv {
  uint32_t d, mul, shift;
};

static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d == 1) { f.mul = 0; f.shift = 0; return f; }
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  f.mul = (uint32_t)m;
  f.shift = s;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  if (f.d == 1) return x;
  uint32_t t = __umulhi(x, f.mul);
  return (t + ((x - t) >> 1)) >> (f.shift - 1);
}

struct ConvGeom {
  int H, W, Cs;      // gathered tensor spatial dims / channels (NHWC)
  int P, Q;          // "row pixel" spatial dims: rows index (n, p, q)
  int R, S, stride, pad;
  FastDiv fPQ, fQ, fS, fCpt;  // divisors: P*Q, Q, S, Cs/64 (channel chunks per tap)
  // mode 3 (strided dgrad, one parity class per blockIdx.y): class row dims
  int Pc[4], Qc[4];
  FastDiv fPQc[4], fQc[4];
};

struct NTArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const float* bias;
  float* stats;      // optional [tiles_m][2][N] per-channel (sum, sumsq) partials of the bf16 output
  int M, N, K;
  int lda, ldb, ldc;
  int mode;
  int out_f32;
  int accumulate;
  int tiles_m;       // m-tiles per class (mode 3) / total (others)
  ConvGeom g;
};

struct TNArgs {
  const bf16_t* A;  // [K][M] (row stride lda)
  const bf16_t* B;  // plain [K][N] (ldb) or gathered NHWC input (mode 1)
  float* C;         // [M][N] fp32 (ldc), accumulated atomically
  int M, N, K;
  int lda, ldb, ldc;
  int mode;
  int k_per_split;
  ConvGeom g;
};

constexpr int BK = 64;

// ----------------------------------------------------------------- NT kernel
// modes: 0 plain GEMM, 1 conv fwd, 2 conv dgrad (stride-1 or masked), 3 conv dgrad
// decomposed by output parity class (stride 2: only the taps that hit real dY pixels).
template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void nt_kernel(NTArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  constexpr int A_CH = BM / 32, B_CH = BN / 32;  // 16-byte chunks per thread per k-step
  constexpr int SMEM_U4 = 2 * (BM + BN) * 8;
  __shared__ __attribute__((aligned(16))) uint4 smem[SMEM_U4];
  uint4* As = smem;                 // [2][BM][8]
  uint4* Bs = smem + 2 * BM * 8;    // [2][BN][8]

  const int nbn = (a.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / nbn;
  const int m0 = tm * BM, n0 = (tile % nbn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int chk = tid & 7;
  const int rbase = tid >> 3;  // + 32*i

  // ---- class geometry (mode 3)
  int cls = 0, ph = 0, pw = 0, r0 = 0, s0 = 0, nr = a.g.R, ns = a.g.S, dh = 0, dw = 0;
  int Mrows = a.M;
  FastDiv fPQ = a.g.fPQ, fQ = a.g.fQ;
  if (a.mode == 3) {
    cls = blockIdx.y;
    ph = cls / a.g.stride; pw = cls - ph * a.g.stride;
    r0 = (ph + a.g.pad) % a.g.stride; s0 = (pw + a.g.pad) % a.g.stride;
    nr = r0 < a.g.R ? (a.g.R - r0 + a.g.stride - 1) / a.g.stride : 0;
    ns = s0 < a.g.S ? (a.g.S - s0 + a.g.stride - 1) / a.g.stride : 0;
    dh = (ph + a.g.pad - r0) / a.g.stride; dw = (pw + a.g.pad - s0) / a.g.stride;
    fPQ = a.g.fPQc[cls]; fQ = a.g.fQc[cls];
    Mrows = (a.M / (a.g.P * a.g.Q)) * a.g.Pc[cls] * a.g.Qc[cls];
  }
  if (m0 >= Mrows) return;

  // ---- per-thread A row geometry (fixed over the K loop)
  int a_m[A_CH], a_img[A_CH], a_hb[A_CH], a_wb[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int m = m0 + rbase + 32 * i;
    a_m[i] = m;
    if (a.mode != 0) {
      uint32_t mm = m < Mrows ? (uint32_t)m : 0u;
      uint32_t img = fdiv(mm, fPQ);
      uint32_t rem = mm - img * fPQ.d;
      uint32_t p = fdiv(rem, fQ);
      uint32_t q = rem - p * fQ.d;
      a_img[i] = (int)img;
      if (a.mode == 1)      { a_hb[i] = (int)p * a.g.stride - a.g.pad; a_wb[i] = (int)q * a.g.stride - a.g.pad; }
      else if (a.mode == 2) { a_hb[i] = (int)p + a.g.pad;             a_wb[i] = (int)q + a.g.pad; }
      else                  { a_hb[i] = (int)p + dh;                  a_wb[i] = (int)q + dw; }
    } else {
      a_img[i] = 0; a_hb[i] = 0; a_wb[i] = 0;
    }
  }

  const int cpt = (int)a.g.fCpt.d;
  const int nk = (a.mode == 3) ? nr * ns * cpt : (a.K + BK - 1) / BK;
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    int c = 0, r = 0, s = 0, kB = kt * BK + chk * 8;
    int tr = 0, ts = 0;
    if (a.mode != 0) {
      const int tap = (int)fdiv((uint32_t)kt, a.g.fCpt);
      c = (kt - tap * cpt) * 64 + chk * 8;
      if (a.mode == 3) {
        tr = tap / ns; ts = tap - tr * ns;
        r = r0 + a.g.stride * tr; s = s0 + a.g.stride * ts;
      } else {
        r = (int)fdiv((uint32_t)tap, a.g.fS);
        s = tap - r * a.g.S;
      }
      kB = (r * a.g.S + s) * a.g.Cs + c;
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const bf16_t* src = nullptr;
      if (a.mode == 0) {
        if (a_m[i] < a.M && kB < a.K) src = a.A + (size_t)a_m[i] * a.lda + kB;
      } else if (a.mode == 1) {
        int ih = a_hb[i] + r, iw = a_wb[i] + s;
        if (a_m[i] < Mrows && (unsigned)ih < (unsigned)a.g.H && (unsigned)iw < (unsigned)a.g.W)
          src = a.A + ((size_t)(a_img[i] * a.g.H + ih) * a.g.W + iw) * a.g.Cs + c;
      } else if (a.mode == 2) {
        int th = a_hb[i] - r, tw = a_wb[i] - s;
        bool ok = a_m[i] < Mrows && th >= 0 && tw >= 0;
        int ih = th, iw = tw;
        if (a.g.stride != 1) {
          ok = ok && (th % a.g.stride) == 0 && (tw % a.g.stride) == 0;
          ih = th / a.g.stride; iw = tw / a.g.stride;
        }
        if (ok && ih < a.g.H && iw < a.g.W)
          src = a.A + ((size_t)(a_img[i] * a.g.H + ih) * a.g.W + iw) * a.g.Cs + c;
      } else {
        int ih = a_hb[i] - tr, iw = a_wb[i] - ts;
        if (a_m[i] < Mrows && (unsigned)ih < (unsigned)a.g.H && (unsigned)iw < (unsigned)a.g.W)
          src = a.A + ((size_t)(a_img[i] * a.g.H + ih) * a.g.W + iw) * a.g.Cs + c;
      }
      ra[i] = src ? *(const uint4*)src : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int n = n0 + rbase + 32 * i;
      rb[i] = (n < a.N && kB < a.K) ? *(const uint4*)(a.B + (size_t)n * a.ldb + kB) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int row = rbase + 32 * i;
      As[(buf * BM + row) * 8 + (chk ^ (row & 7))] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int row = rbase + 32 * i;
      Bs[(buf * BN + row) * 8 + (chk ^ (row & 7))] = rb[i];
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  if (nk > 0) {
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int row = wm * WM + 16 * i + fr;
        uint4 v = As[(cur * BM + row) * 8 + ((kk * 4 + fq) ^ (row & 7))];
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int row = wn * WN + 16 * j + fr;
        uint4 v = Bs[(cur * BN + row) * 8 + ((kk * 4 + fq) ^ (row & 7))];
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // output row offset (elements) of tile row m
  auto row_off = [&](int m) -> size_t {
    if (a.mode != 3) return (size_t)m * a.ldc;
    uint32_t img = fdiv((uint32_t)m, fPQ);
    uint32_t rem = (uint32_t)m - img * fPQ.d;
    uint32_t i = fdiv(rem, fQ);
    uint32_t j = rem - i * fQ.d;
    const int h = (int)i * a.g.stride + ph, w = (int)j * a.g.stride + pw;
    return ((size_t)((int)img * a.g.P + h) * a.g.Q + w) * a.ldc;
  };

  if (a.out_f32) {
    // ---- direct epilogue (fp32 logits etc.): lane holds D[n = 16j + 4fq + r][m = 16i + fr]
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * WM + 16 * i + fr;
      if (m >= Mrows) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WN + 16 * j + 4 * fq;
        if (n >= a.N) continue;
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if (a.bias) { v0 += a.bias[n]; v1 += a.bias[n + 1]; v2 += a.bias[n + 2]; v3 += a.bias[n + 3]; }
        float* dst = (float*)a.C + row_off(m) + n;
        if (a.accumulate) { float4 o = *(float4*)dst; v0 += o.x; v1 += o.y; v2 += o.z; v3 += o.w; }
        *(float4*)dst = make_float4(v0, v1, v2, v3);
      }
    }
    return;
  }

  // ---- bf16 epilogue staged through LDS: full 16-byte row chunks to HBM (+ BN partial stats)
  constexpr int CST = BN + 8;                    // padded row stride (elements): 16-B aligned rows
  bf16_t* Ct = (bf16_t*)smem;                    // [BM][CST]
  float* Sred = (float*)(smem) + (BM * CST) / 2; // [rows_par][2][BN] stats scratch
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int ml = wm * WM + 16 * i + fr;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nl = wn * WN + 16 * j + 4 * fq;
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if (a.bias && n0 + nl < a.N) {
        v0 += a.bias[n0 + nl]; v1 += a.bias[n0 + nl + 1]; v2 += a.bias[n0 + nl + 2]; v3 += a.bias[n0 + nl + 3];
      }
      *(uint2*)&Ct[ml * CST + nl] = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;          // 16-B chunks per row
  constexpr int RPP = 256 / CPR;       // rows per pass
  const int cc = tid % CPR, rr = tid / CPR;
  const int n = n0 + cc * 8;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int ml = rr; ml < BM; ml += RPP) {
    const int m = m0 + ml;
    if (m >= Mrows) break;
    const uint4 v = *(const uint4*)&Ct[ml * CST + cc * 8];
    if (n < a.N) *(uint4*)((bf16_t*)a.C + row_off(m) + n) = v;
    if (a.stats) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int q = 0; q < 8; ++q) { s1[q] += f[q]; s2[q] += f[q] * f[q]; }
    }
  }
  if (a.stats) {
    // reduce the RPP row groups of each column chunk through LDS (Sred is disjoint from Ct)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      Sred[(rr * 2 + 0) * BN + cc * 8 + q] = s1[q];
      Sred[(rr * 2 + 1) * BN + cc * 8 + q] = s2[q];
    }
    __syncthreads();
    const int prow = blockIdx.y * a.tiles_m + tm;
    for (int c = tid; c < 2 * BN; c += 256) {
      const int which = c / BN, col = c - which * BN;
      float t = 0.f;
      for (int g = 0; g < RPP; ++g) t += Sred[(g * 2 + which) * BN + col];
      if (n0 + col < a.N) a.stats[((size_t)prow * 2 + which) * a.N + n0 + col] = t;
    }
  }
}

// ----------------------------------------------------------------- TN kernel
// LDS tile [BK rows][X cols] bf16, 8-byte units swizzled u' = u ^ sw(k) so the
// transposed 4x16 reads of ds_read_b64_tr_b16 are conflict-free.
template <int UNITS>
__device__ __forceinline__ int tr_swz(int k) {
  return (4 * (k & 3) + 16 * ((k >> 3) & 1)) & (UNITS - 1);
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void tn_kernel(TNArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  constexpr int AU = BM / 4, BU = BN / 4;            // 8-byte units per LDS row
  constexpr int ACPR = BM / 8, BCPR = BN / 8;        // 16-byte chunks per row
  constexpr int A_CH = BK * ACPR / 256, B_CH = BK * BCPR / 256;
  constexpr int A_RSTEP = 256 / ACPR, B_RSTEP = 256 / BCPR;
  __shared__ __attribute__((aligned(16))) uint2 smem[2 * BK * (AU + BU)];
  uint2* As = smem;                   // [2][BK][AU]
  uint2* Bs = smem + 2 * BK * AU;     // [2][BK][BU]

  const int nbn = (a.N + BN - 1) / BN;
  const int ntiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
  const int kbeg = blockIdx.y * a.k_per_split;
  const int kend = min(a.K, kbeg + a.k_per_split);
  if (kbeg >= kend) return;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int a_cc = tid % ACPR, a_r = tid / ACPR;
  const int b_cc = tid % BCPR, b_r = tid / BCPR;

  // conv-mode B column geometry: the block's n range sits inside one (r,s) tap
  int tap_r = 0, tap_s = 0, c0 = 0;
  if (a.mode == 1) {
    int tap = n0 / a.g.Cs;
    c0 = n0 - tap * a.g.Cs;
    tap_r = tap / a.g.S;
    tap_s = tap - tap_r * a.g.S;
  }

  uint4 ra[A_CH], rb[B_CH];
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int k = k0 + a_r + A_RSTEP * i;
      int m = m0 + a_cc * 8;
      ra[i] = (k < kend && m < a.M) ? *(const uint4*)(a.A + (size_t)k * a.lda + m) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int k = k0 + b_r + B_RSTEP * i;
      const bf16_t* src = nullptr;
      if (k < kend) {
        if (a.mode == 0) {
          int n = n0 + b_cc * 8;
          if (n < a.N) src = a.B + (size_t)k * a.ldb + n;
        } else {
          uint32_t img = fdiv((uint32_t)k, a.g.fPQ);
          uint32_t rem = (uint32_t)k - img * a.g.fPQ.d;
          uint32_t p = fdiv(rem, a.g.fQ);
          uint32_t q = rem - p * a.g.fQ.d;
          int ih = (int)p * a.g.stride - a.g.pad + tap_r;
          int iw = (int)q * a.g.stride - a.g.pad + tap_s;
          if ((unsigned)ih < (unsigned)a.g.H && (unsigned)iw < (unsigned)a.g.W)
            src = a.B + ((size_t)((int)img * a.g.H + ih) * a.g.W + iw) * a.g.Cs + c0 + b_cc * 8;
        }
      }
      rb[i] = src ? *(const uint4*)src : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int k = a_r + A_RSTEP * i;
      int u = (2 * a_cc) ^ tr_swz<AU>(k);
      *(uint4*)&As[(buf * BK + k) * AU + u] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int k = b_r + B_RSTEP * i;
      int u = (2 * b_cc) ^ tr_swz<BU>(k);
      *(uint4*)&Bs[(buf * BK + k) * BU + u] = rb[i];
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  load_tiles(kbeg);
  store_tiles(0);
  __syncthreads();
  const int nk = (kend - kbeg + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NJ];
      const int k1 = kk * 32 + 8 * g + q4;
      const int k2 = k1 + 4;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        int u = (wm * WM + 16 * i) / 4 + p4;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &As[(cur * BK + k1) * AU + (u ^ tr_swz<AU>(k1))]));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &As[(cur * BK + k2) * AU + (u ^ tr_swz<AU>(k2))]));
        short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int u = (wn * WN + 16 * j) / 4 + p4;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &Bs[(cur * BK + k1) * BU + (u ^ tr_swz<BU>(k1))]));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &Bs[(cur * BK + k2) * BU + (u ^ tr_swz<BU>(k2))]));
        short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v8);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds D[m = 16i + 4g + r][n = 16j + li]; fp32 atomics (split-K)
  const bool single = (gridDim.y == 1);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * WN + 16 * j + li;
      if (n >= a.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + 16 * i + 4 * g + r;
        if (m >= a.M) continue;
        float* dst = a.C + (size_t)m * a.ldc + n;
        if (single) *dst += acc[i][j][r];
        else atomicAdd(dst, acc[i][j][r]);
      }
    }
  }
}

// -------------------------------------------------------- weight transpose
// W[K][RS][C] -> Wt[C][RS][K]  (conv dgrad B operand), bf16.
__global__ void wtrans_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, int K, int RS, int C) {
  __shared__ bf16_t t[64][65];
  const int tap = blockIdx.z;
  const int k0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads -> 4 rows per pass
  for (int r = ty; r < 64; r += 4) {
    int k = k0 + r, c = c0 + tx;
    t[r][tx] = (k < K && c < C) ? w[((size_t)k * RS + tap) * C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    int c = c0 + r, k = k0 + tx;
    if (c < C && k < K) wt[((size_t)c * RS + tap) * K + k] = t[tx][r];
  }
}

ConvGeom make_geom(int H, int W, int Cs, int P, int Q, int S, int stride, int pad, int R = 1) {
  ConvGeom g{};
  g.H = H; g.W = W; g.Cs = Cs; g.P = P; g.Q = Q; g.R = R; g.S = S; g.stride = stride; g.pad = pad;
  g.fPQ = make_fastdiv((uint32_t)(P * Q));
  g.fQ = make_fastdiv((uint32_t)Q);
  g.fS = make_fastdiv((uint32_t)S);
  g.fCpt = make_fastdiv((uint32_t)(Cs >= 64 ? Cs / 64 : 1));
  return g;
}

template <int BM, int BN>
hipError_t launch_nt(NTArgs& a, hipStream_t st) {
  int classes = 1, mrows = a.M;
  if (a.mode == 3) {
    classes = a.g.stride * a.g.stride;
    mrows = 0;
    const int nimg = a.M / (a.g.P * a.g.Q);
    for (int c = 0; c < classes; ++c) mrows = std::max(mrows, nimg * a.g.Pc[c] * a.g.Qc[c]);
  }
  a.tiles_m = cdiv(mrows, BM);
  int grid = a.tiles_m * cdiv(a.N, BN);
  hipLaunchKernelGGL((nt_kernel<BM, BN>), dim3(grid, classes), dim3(256), 0, st, a);
  return hipGetLastError();
}

// tile choice shared with the host-side stats-slab sizing (mi_nt_tile_m)
int nt_choice(int M, int N) {
  if (N <= 64) return 1;                                         // 128x64
  if ((int64_t)cdiv(M, 128) * cdiv(N, 128) < 512) return 2;     // 64x64 (fill 256 CUs)
  return 0;                                                      // 128x128
}

hipError_t dispatch_nt(NTArgs& a, hipStream_t st) {
  switch (nt_choice(a.M, a.N)) {
    case 1: return launch_nt<128, 64>(a, st);
    case 2: return launch_nt<64, 64>(a, st);
    default: return launch_nt<128, 128>(a, st);
  }
}

template <int BM, int BN>
hipError_t launch_tn(TNArgs& a, hipStream_t st, int target_blocks) {
  int tiles = cdiv(a.M, BM) * cdiv(a.N, BN);
  int ksteps = cdiv(a.K, BK);
  int splits = std::max(1, std::min(ksteps, target_blocks / std::max(tiles, 1)));
  int steps_per = cdiv(ksteps, splits);
  a.k_per_split = steps_per * BK;
  splits = cdiv(a.K, a.k_per_split);
  hipLaunchKernelGGL((tn_kernel<BM, BN>), dim3(tiles, splits), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t dispatch_tn(TNArgs& a, hipStream_t st) {
  const int target = 1024;
  bool n64 = (a.N <= 64) || (a.mode == 1 && (a.g.Cs % 128) != 0);
  bool m64 = a.M <= 64;
  if (m64 && n64) return launch_tn<64, 64>(a, st, target);
  if (m64) return launch_tn<64, 128>(a, st, target);
  if (n64) return launch_tn<128, 64>(a, st, target);
  return launch_tn<128, 128>(a, st, target);
}

}  // namespace

// ============================================================== C ABI
// Conv forward: x NHWC [Nb,H,W,C] bf16, w [K][R][S][C] bf16, y NHWC [Nb,P,Q,K].
// Rows of the per-channel statistics slab written by a conv/GEMM forward with M rows, N cols.
MI_API int mi_nt_stat_rows(int M, int N) {
  const int bm = nt_choice(M, N) == 2 ? 64 : 128;
  return cdiv(M, bm);
}

// Conv forward: x NHWC [Nb,H,W,C] bf16, w [K][R][S][C] bf16, y NHWC [Nb,P,Q,K].
// stats (optional, bf16 output only): fp32 [mi_nt_stat_rows(M,K)][2][K] partial (sum, sumsq).
MI_API int mi_conv2d_fwd(const void* x, const void* w, void* y, const float* bias, float* stats,
                         int Nb, int H, int W, int C, int K, int R, int S,
                         int stride, int pad, int P, int Q, int out_f32, hipStream_t st) {
  if (C % 64 != 0 || K % 8 != 0) return (int)hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = y; a.bias = bias; a.stats = stats;
  a.M = Nb * P * Q; a.N = K; a.K = R * S * C;
  a.lda = 0; a.ldb = a.K; a.ldc = K; a.mode = 1; a.out_f32 = out_f32; a.accumulate = 0;
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_nt(a, st);
}

// Conv backward-data: dy NHWC [Nb,P,Q,K], wt [C][R][S][K] (see mi_conv_wtrans), dx NHWC [Nb,H,W,C].
MI_API int mi_conv2d_dgrad(const void* dy, const void* wt, void* dx,
                           int Nb, int H, int W, int C, int K, int R, int S,
                           int stride, int pad, int P, int Q, hipStream_t st) {
  if (K % 64 != 0 || C % 8 != 0) return (int)hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)wt; a.C = dx; a.bias = nullptr;
  a.M = Nb * H * W; a.N = C; a.K = R * S * K;
  a.lda = 0; a.ldb = a.K; a.ldc = C; a.mode = 2; a.out_f32 = 0; a.accumulate = 0;
  // gathered tensor = dy (spatial P,Q, channels K); rows = dx pixels (H, W)
  a.g = make_geom(P, Q, K, H, W, S, stride, pad, R);
  if (stride == 2) {
    // parity-class decomposition: class (ph, pw) rows only visit taps r = ph+pad (mod 2)
    a.mode = 3;
    for (int c = 0; c < 4; ++c) {
      const int ph = c / 2, pw = c % 2;
      a.g.Pc[c] = (H - ph + 1) / 2;
      a.g.Qc[c] = (W - pw + 1) / 2;
      a.g.fPQc[c] = make_fastdiv((uint32_t)std::max(1, a.g.Pc[c] * a.g.Qc[c]));
      a.g.fQc[c] = make_fastdiv((uint32_t)std::max(1, a.g.Qc[c]));
    }
  }
  return (int)dispatch_nt(a, st);
}

// Conv backward-weight: dw[K][R][S][C] (fp32) += sum over pixels dy^T * im2col(x).
MI_API int mi_conv2d_wgrad(const void* x, const void* dy, float* dw,
                           int Nb, int H, int W, int C, int K, int R, int S,
                           int stride, int pad, int P, int Q, hipStream_t st) {
  if (C % 64 != 0 || K % 8 != 0) return (int)hipErrorInvalidValue;
  TNArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)x; a.C = dw;
  a.M = K; a.N = R * S * C; a.K = Nb * P * Q;
  a.lda = K; a.ldb = 0; a.ldc = a.N; a.mode = 1;
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_tn(a, st);
}

MI_API int mi_conv_wtrans(const void* w, void* wt, int K, int RS, int C, hipStream_t st) {
  dim3 grid(cdiv(C, 64), cdiv(K, 64), RS);
  hipLaunchKernelGGL(wtrans_kernel, grid, dim3(256), 0, st, (const bf16_t*)w, (bf16_t*)wt, K, RS, C);
  return (int)hipGetLastError();
}

// Plain GEMM, "NT": C[M][N] = A[M][K] * B[N][K]^T (+bias[N]); A, B bf16; C bf16 or fp32.
MI_API int mi_gemm_nt(const void* A, const void* B, void* C, const float* bias, float* stats,
                      int M, int N, int K, int lda, int ldb, int ldc,
                      int out_f32, int accumulate, hipStream_t st) {
  if (K % 8 != 0 || N % 4 != 0 || (!out_f32 && N % 8 != 0)) return (int)hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = bias; a.stats = out_f32 ? nullptr : stats;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.mode = 0; a.out_f32 = out_f32; a.accumulate = accumulate;
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_nt(a, st);
}

// Plain GEMM, "TN": C[M][N] (fp32) += A[K][M]^T * B[K][N].
MI_API int mi_gemm_tn(const void* A, const void* B, float* C, int M, int N, int K,
                      int lda, int ldb, int ldc, hipStream_t st) {
  if (M % 8 != 0 || N % 8 != 0) return (int)hipErrorInvalidValue;
  TNArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.mode = 0;
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_tn(a, st);
}
