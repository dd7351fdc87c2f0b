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
//    (huge) N*P*Q reduction: every split writes its partial tile to a slab and a
//    reduce kernel sums the splits into the fp32 gradient (deterministic; the
//    fp32-atomic variant cost ~1 ms per ResNet-50 step at ~1.3 TB/s of atomics).
#include "common.h"
#include "epilogue.h"
#include <algorithm>
#include <array>
#include <cstdio>
#include <vector>
#include <mutex>
#include <cstdlib>

// tuned launch occupancies (blocks per CU the kernels are compiled for): 128x128 / 128x64 NT tiles
// (4 single-stage blocks keep more k-steps and epilogues of the short-K 1x1 convs in flight than 3),
// TN weight-gradient tiles (plain GEMM / conv)
constexpr int kNtBlocksPerCu = 4, kNt64BlocksPerCu = 4;
constexpr int kTnBlocksPerCu = 3, kTnConvBlocksPerCu = 3;
// NT epilogue: row steps whose operand loads are issued together
constexpr int kNtEpiEU = 4;

namespace {

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
  int a_bytes, b_bytes;  // buffer-resource ranges (GLDS path): A / B extents in bytes
  bf16_t* aux;       // bf16 epilogue operand, same layout as C (see epi)
  int epi;           // bf16 epilogue op: 0 none, 1 GELU (aux <- pre-activation, C <- gelu),
                     // 2 GELU backward (C <- acc * gelu'(aux)), 3 residual / accumulate (C <- acc + aux),
                     // 4 BatchNorm backward of the layer that produced this conv's input:
                     //   C <- dz = acc * [aux > 0] (relu mask on the BN output aux, if bn_relu),
                     //   stats <- per-channel (sum dz, sum dz * (aux2 - mean)), aux2 = BN input
                     // 5: as 4 on acc + C (the gradient already in C: a block input's residual sum)
  const bf16_t* aux2;
  const float* mean;
  int bn_relu;
  // halo tiles (3x3 / stride 1 / pad 1, modes 1-2): a tile = halo_rp whole output rows of one image;
  // halo_pb = row blocks per image; fPB / fHW2 divide by halo_pb / (Q + 2)
  int halo_rp, halo_pb;
  FastDiv fPB, fHW2;
  // mode 3: blockIdx.y -> parity class (empty classes -- no tap reaches them -- can be skipped when
  // their zero output is not needed); epi 3 / 5 with aux_even: the gradient accumulated into is
  // defined only at even (h, w) of the row grid (a stride-2 1x1 data gradient written by class
  // (0, 0) alone) and reads as 0 elsewhere
  int cls_map[4], ncls;
  int aux_even;
  // split-K (small grids, see launch_nt): SPLIT 1 blocks (blockIdx.z = split) accumulate k-steps
  // [z * ksplit, (z + 1) * ksplit) and store their fp32 tiles to ws; SPLIT 2 blocks sum the
  // splits in order and run the ordinary epilogue
  float* ws;
  int splits, ksplit;
  int* cnt;          // SPLIT 3: per-tile arrival counters (zero between launches)
  // normalize-on-load (NOL kernels): the gathered A operand of a conv forward is the raw output c
  // of the previous conv and the kernel applies that layer's BatchNorm + ReLU as it stages it:
  // a <- relu(c * nol_scale[ch] + nol_shift[ch]) (padding stays 0); the inner BN's output y is never
  // written.  mask_scale / mask_shift: epi 4 takes the ReLU mask from aux2 (= c) as
  // fma(c, scale, shift) > 0 instead of reading y (aux)
  const float* nol_scale;
  const float* nol_shift;
  const float* mask_scale;
  const float* mask_shift;
  // epi 4 / 5 with bn_relu: the ReLU mask as one byte per 8 channels of C's layout (bit j = channel
  // 8i + j positive; norm_act.hip mi_bn_apply_bits) instead of the bf16 BN output aux -- 1/16 of
  // the bytes
  const uint8_t* mbits;
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
  int a_bytes, b_bytes;
  float* colsum;    // optional [M] fp32 += column sums of A (a Linear layer's bias gradient)
  float* ws;        // split-K partial slabs [tiles][splits][BM*BN] (fragment order), or null: atomics
  int* cnt;         // per-tile arrival counters: the last-arriving split sums the slabs (no reduce launch)
  // normalize-on-load of the gathered input (conv mode, NOL kernels): b <- relu(x * scale[c] + shift[c])
  const float* nol_scale;
  const float* nol_shift;
  ConvGeom g;
  // folded BN backward (conv_panel.hip mi_panel_dgrad_fbb's weight-gradient twin): A is [dz | c] along
  // M -- rows m >= msplit read A2 at m - msplit (msplit a multiple of BM: the choice is per block) --
  // and the CSB variant writes the column sums of B over each split's k-range to bsum[split][N]
  const bf16_t* A2;
  int a2_bytes, msplit, lda2;
  float* bsum;
};

constexpr int BK = 64;


// ----------------------------------------------------------------- NT kernel
// modes: 0 plain GEMM, 1 conv fwd, 2 conv dgrad (stride-1 or masked), 3 conv dgrad
// decomposed by output parity class (stride 2: only the taps that hit real dY pixels).
// halo tile capacity (pixels of one 64-channel chunk, 128 B each): (rp + 2) x (Q + 2) <= HALO_PX
constexpr int HALO_PX = 256;


// normalize-on-load: per-channel (scale, shift) table of the gathered tensor, right after the
// staging ring (the epilogue, which never needs it, may overwrite it); channels <= NOL_MAX_C
constexpr int NOL_MAX_C = 256;
constexpr int NOL_TAB_U4 = 2 * NOL_MAX_C * 4 / 16;

template <int BM, int BN, int STAGES, bool HALO = false, bool NOL = false>
constexpr int nt_smem_u4() {  // NOL: the forward (normalize-on-load) variant's table
  // max(staging ring (+ NOL table), epilogue C tile [BM][BN+8] bf16 + stats scratch [4 waves][2][BN] fp32)
  constexpr int stage = (HALO ? HALO_PX * 8 + 2 * BN * 8 : STAGES * (BM + BN) * 8) + (NOL ? NOL_TAB_U4 : 0);
  constexpr int epi = (BM * (BN + 8) * 2 + 4 * 2 * BN * 4) / 16;
  return stage > epi ? stage : epi;
}

// relu(x * s + h) on one staged 16-B chunk of 8 bf16 (channel-consecutive)
__device__ __forceinline__ void nol_chunk(uint4* p, const float* tab, int ch) {
  float sc[8], sh[8], f[8];
  *(float4*)&sc[0] = *(const float4*)&tab[ch];
  *(float4*)&sc[4] = *(const float4*)&tab[ch + 4];
  *(float4*)&sh[0] = *(const float4*)&tab[NOL_MAX_C + ch];
  *(float4*)&sh[4] = *(const float4*)&tab[NOL_MAX_C + ch + 4];
  unpack8(*p, f);
#pragma unroll
  for (int q = 0; q < 8; ++q) f[q] = fmaxf(fmaf(f[q], sc[q], sh[q]), 0.f);
  *p = pack8(f);
}

// blocks per CU the NT kernel is compiled for: 4 single-stage blocks (38 KB of LDS each at 128x128,
// <= 128 VGPRs) keep more k-steps and epilogues of the short-K 1x1 convs in flight than 3 did
template <int BN, int STAGES, bool HALO>
constexpr int nt_occupancy() {
  return HALO ? 2 : (STAGES == 1 ? (BN == 64 ? kNt64BlocksPerCu : kNtBlocksPerCu) : 2);
}

// STAGES = 1: one LDS buffer, load -> barrier -> MFMA -> barrier per k-step, 3 blocks per CU (the other
//             blocks' MFMAs hide each block's load latency);
// STAGES = 2: double buffer, next k-step's loads in flight during this one's MFMAs, 2 blocks per CU.
// Both stage with buffer_load ... lds (16 B per lane, zero-fill by range check) and track the
// (tap, channel-chunk) position incrementally in scalar registers.
//
// HALO (3x3 / stride 1 / pad 1 forward and data gradient, C % 64 == 0): the tile is halo_rp whole
// output rows of one image; per 64-channel chunk the (rp + 2) x (Q + 2) input halo is staged ONCE
// into LDS and all nine taps read their A fragments from it (shifted row addresses), with the
// weight tile of the next tap loading into the other B buffer during each tap's MFMAs.  The
// per-tap gather re-reads every input pixel ~9x through L2; the halo reads it ~(rp+2)/rp x.
// NOL: 0 off, 1 normalize-on-load of the gathered A operand (conv forward), 2 epi-4 ReLU mask from c
// (data gradient) -- separate instantiations, so each carries only its own registers
template <int BM, int BN, int STAGES, bool SMALLC, bool HALO = false, int SPLIT = 0, int NOL = 0>
__global__ __launch_bounds__(256, (nt_occupancy<BN, STAGES, HALO>())) void nt_kernel(NTArgs a) {
  static_assert(SPLIT == 0 || (STAGES == 1 && !SMALLC && !HALO), "split-K: single-stage gather/plain tiles only");
  static_assert(NOL == 0 || (STAGES == 1 && !SMALLC && SPLIT == 0), "normalize-on-load: single-stage gather tiles");
  // SPLIT 3: as SPLIT 1, then the last-arriving split of each tile sums all the partial tiles (in
  // split order) and runs the epilogue -- one launch instead of SPLIT 1 + SPLIT 2
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  constexpr int A_CH = BM / 32, B_CH = BN / 32;  // 16-byte chunks per thread per k-step
  __shared__ __attribute__((aligned(16))) uint4 smem[nt_smem_u4<BM, BN, STAGES, HALO, NOL == 1>()];
  uint4* As = smem;                      // [STAGES][BM][8]
  uint4* Bs = smem + STAGES * BM * 8;    // [STAGES][BN][8]
  // NOL: [scale[NOL_MAX_C], shift[NOL_MAX_C]] of the gathered tensor's channels, staged once
  float* nol_tab = (float*)(smem + (HALO ? HALO_PX * 8 + 2 * BN * 8 : STAGES * (BM + BN) * 8));
  const bool nol_a = NOL == 1 && a.nol_scale != nullptr && a.mode == 1;
  if constexpr (NOL == 1) {
    if (nol_a) {
      for (int c = threadIdx.x; c < a.g.Cs; c += 256) {
        nol_tab[c] = a.nol_scale[c];
        nol_tab[NOL_MAX_C + c] = a.nol_shift[c];
      }
      __syncthreads();
    }
  }

  const int nbn = (a.N + BN - 1) / BN;
  // mode 3: one parity class per grid row (blockIdx.y).  Folding the classes into an XCD-aware
  // 1-D grid with a tile's classes adjacent cut a stride-2 3x3 dgrad's HBM fetch from 107 to
  // 28 MB but made it slower (0.148 vs 0.118 ms): this launch is not fetch-bound
  const int tile = xcd_remap(blockIdx.x, gridDim.x), cy = blockIdx.y;
  const int tm = tile / nbn;
  int m0 = tm * BM;
  const int n0 = (tile % nbn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int chk = tid & 7;
  const int rbase = tid >> 3;  // + 32*i

  // ---- class geometry (mode 3)
  int cls = 0, ph = 0, pw = 0, r0 = 0, s0 = 0, nr = a.g.R, ns = a.g.S, dh = 0, dw = 0;
  int Mrows = a.M;
  FastDiv fPQ = a.g.fPQ, fQ = a.g.fQ;
  if (a.mode == 3) {
    cls = a.cls_map[cy];
    ph = cls / a.g.stride; pw = cls - ph * a.g.stride;
    r0 = (ph + a.g.pad) % a.g.stride; s0 = (pw + a.g.pad) % a.g.stride;
    nr = r0 < a.g.R ? (a.g.R - r0 + a.g.stride - 1) / a.g.stride : 0;
    ns = s0 < a.g.S ? (a.g.S - s0 + a.g.stride - 1) / a.g.stride : 0;
    dh = (ph + a.g.pad - r0) / a.g.stride; dw = (pw + a.g.pad - s0) / a.g.stride;
    fPQ = a.g.fPQc[cls]; fQ = a.g.fQc[cls];
    Mrows = (a.M / (a.g.P * a.g.Q)) * a.g.Pc[cls] * a.g.Qc[cls];
  }
  // halo tile: image hi, output rows hp0 .. hp0 + hrows / Q - 1
  int hi = 0, hp0 = 0, hrows = 0;
  if constexpr (HALO) {
    hi = (int)fdiv((uint32_t)tm, a.fPB);
    hp0 = (tm - hi * a.halo_pb) * a.halo_rp;
    hrows = min(a.halo_rp, a.g.P - hp0) * a.g.Q;
    m0 = (hi * a.g.P + hp0) * a.g.Q;
  }
  const int Mlim = HALO ? m0 + hrows : Mrows;
  if (m0 >= Mrows) {
    // empty tile of a parity class: its statistics rows still have to be defined
    if (SPLIT != 1 && a.stats) {
      const int prow = cy * a.tiles_m + tm;
      for (int c = threadIdx.x; c < 2 * BN; c += 256) {
        const int which = c / BN, col = c - which * BN;
        if (n0 + col < a.N) a.stats[((size_t)prow * 2 + which) * a.N + n0 + col] = 0.f;
      }
    }
    return;
  }

  // glds writes lane-linear pieces (LDS row rbase+32i, physical chunk chk): the XOR swizzle is on
  // the SOURCE, this lane fetches logical chunk lc of its rows (row & 7 == rbase & 7 for all i).
  const int lc = chk ^ (rbase & 7);
  const int W = a.g.W, H = a.g.H, Cs = a.g.Cs;

  // ---- per-thread A rows: gather-space pixel (hb, wb) and its element offset (may be negative)
  int a_hb[A_CH], a_wb[A_CH], a_base[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + rbase + 32 * i;
    a_ok[i] = m < Mrows;
    if (a.mode != 0) {
      const uint32_t mm = a_ok[i] ? (uint32_t)m : 0u;
      const uint32_t img = fdiv(mm, fPQ);
      const uint32_t rem = mm - img * fPQ.d;
      const uint32_t p = fdiv(rem, fQ);
      const uint32_t q = rem - p * fQ.d;
      if (a.mode == 1 || a.mode == 4) { a_hb[i] = (int)p * a.g.stride - a.g.pad; a_wb[i] = (int)q * a.g.stride - a.g.pad; }
      else if (a.mode == 2)           { a_hb[i] = (int)p + a.g.pad;             a_wb[i] = (int)q + a.g.pad; }
      else                            { a_hb[i] = (int)p + dh;                  a_wb[i] = (int)q + dw; }
      // mode 4 (Cs == 8): the lane's 16-B chunk is one whole tap (8 channels), not a channel slice
      a_base[i] = (((int)img * H + a_hb[i]) * W + a_wb[i]) * Cs + (SMALLC ? 0 : lc * 8);
    } else {
      a_hb[i] = 0; a_wb[i] = 0;
      a_base[i] = m * a.lda + lc * 8;
    }
  }
  int b_base[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int n = n0 + rbase + 32 * i;
    b_base[i] = n < a.N ? n * a.ldb + lc * 8 : -1;
  }

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.b_bytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;

  const int nS = (a.mode == 3) ? ns : a.g.S;
  int nk = (a.mode == 3) ? nr * ns * (int)a.g.fCpt.d : (a.K + BK - 1) / BK;
  // wave-uniform k position: gather-space tap (kr, ks) and channel-chunk base kc
  int kr = 0, ks = 0, kc = 0;
  int kt0 = 0;  // first k-step of this block (split-K)
  if constexpr (SPLIT == 1 || SPLIT == 3) {
    kt0 = blockIdx.z * a.ksplit;
    nk = min(nk, kt0 + a.ksplit);
    if (a.mode != 0) {  // (kr, ks, kc) of k-step kt0: channel chunks fastest, then taps of a row
      const int cpt = (int)a.g.fCpt.d;
      const int t = kt0 / cpt;
      kc = (kt0 - t * cpt) * 64;
      ks = t % nS;
      kr = t / nS;
    }
  }
  // mode 4 (SMALLC): per-LANE tap t = 8*kt + lc -> (tr4, ts4), advanced by 8 taps per k-step
  int tr4 = 0, ts4 = 0, dts4 = 0, dtr4 = 0, ntaps = 0;
  if constexpr (SMALLC) {
    tr4 = lc / a.g.S; ts4 = lc - tr4 * a.g.S;
    dts4 = 8 % a.g.S; dtr4 = 8 / a.g.S; ntaps = a.g.R * a.g.S;
  }

  uint32_t a_okm = 0;  // NOL: A chunks of the last issued k-step that hold real pixels
  int a_kc = 0;        // NOL: their channel-chunk base
  auto issue_loads = [&](int kt, int buf) {
    int r, s, koffA, kB;
    a_okm = 0;
    a_kc = kc;
    if (SMALLC || a.mode == 0) {
      r = 0; s = 0;
      koffA = SMALLC ? (tr4 * W + ts4) * Cs : kt * BK;
      kB = kt * BK;
    } else {
      r = (a.mode == 3) ? r0 + a.g.stride * kr : kr;
      s = (a.mode == 3) ? s0 + a.g.stride * ks : ks;
      const int sgn_tap = (a.mode == 1) ? ((kr * W + ks) * Cs) : -((kr * W + ks) * Cs);
      koffA = sgn_tap + kc;
      kB = (r * a.g.S + s) * Cs + kc;
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      bool ok = a_ok[i];
      if constexpr (SMALLC) {
        const int ih = a_hb[i] + tr4, iw = a_wb[i] + ts4;
        ok = ok && (kt * 8 + lc) < ntaps && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      } else if (a.mode == 0) {
        ok = ok && kt * BK + lc * 8 < a.K;
      } else {
        const int ih = (a.mode == 1) ? a_hb[i] + kr : a_hb[i] - kr;
        const int iw = (a.mode == 1) ? a_wb[i] + ks : a_wb[i] - ks;
        ok = ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      }
      const uint32_t vo = ok ? (uint32_t)(a_base[i] + koffA) * 2u : OOB;
      a_okm |= (ok ? 1u : 0u) << i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, &As[(buf * BM + 32 * i + 8 * wid) * 8]), 16, vo,
                                               0, 0, 0);
    }
    const bool kok = (!SMALLC && a.mode != 0) || (kt * BK + lc * 8 < a.K);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const bool ok = b_base[i] >= 0 && kok;
      const uint32_t vo = ok ? (uint32_t)(b_base[i] + kB) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, LDS_PTR(void, &Bs[(buf * BN + 32 * i + 8 * wid) * 8]), 16, vo,
                                               0, 0, 0);
    }
    // advance the k position
    if constexpr (SMALLC) {
      ts4 += dts4; tr4 += dtr4;
      if (ts4 >= a.g.S) { ts4 -= a.g.S; ++tr4; }
    } else if (a.mode != 0) {
      kc += 64;
      if (kc >= Cs) {
        kc = 0;
        if (++ks >= nS) { ks = 0; ++kr; }
      }
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * WM + 16 * i + fr;
        af[i] = __builtin_bit_cast(bf16x8, As[(cur * BM + row) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * WN + 16 * j + fr;
        bfr[j] = __builtin_bit_cast(bf16x8, Bs[(cur * BN + row) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (HALO) {
    uint4* Hs = smem;                   // [HALO_PX][8] input halo of one channel chunk
    uint4* Bh = smem + HALO_PX * 8;     // [2][BN][8] weight tile of a tap
    const int Q = a.g.Q, HW2 = Q + 2;
    const int HP = (hrows / Q + 2) * HW2;
    const int nit = (HP + 31) / 32;     // 32 halo pixels (256 x 16 B) per block-wide pass
    int hb[MI];                         // halo pixel of tap (0,0) for this lane's fragment rows
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ml = wm * WM + 16 * i + fr;
      const uint32_t mc = ml < hrows ? (uint32_t)ml : 0u;
      const uint32_t pr = fdiv(mc, a.g.fQ);
      hb[i] = (int)pr * HW2 + (int)(mc - pr * (uint32_t)Q);
    }
    auto load_halo = [&](int kc) {
      for (int it = 0; it < nit; ++it) {
        const int f = it * 256 + tid;
        const int px = f >> 3, chp = f & 7;
        const uint32_t hr = fdiv((uint32_t)px, a.fHW2);
        const int hc = px - (int)hr * HW2;
        const int ih = hp0 - 1 + (int)hr, iw = hc - 1;
        const bool ok = px < HP && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const uint32_t vo = ok ? (uint32_t)((((hi * H + ih) * W + iw) * Cs + kc + ((chp ^ (px & 7)) * 8)) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, &Hs[it * 256 + wid * 64]), 16, vo, 0, 0,
                                                 0);
      }
    };
    auto load_b = [&](int t, int kc, int buf) {
      const int kB = t * Cs + kc;  // tap t = r*3 + s of [N][3][3][Cs]
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const bool ok = b_base[i] >= 0;
        const uint32_t vo = ok ? (uint32_t)(b_base[i] + kB) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, LDS_PTR(void, &Bh[(buf * BN + 32 * i + 8 * wid) * 8]), 16,
                                                 vo, 0, 0, 0);
      }
    };
    auto compute_halo = [&](int t, int buf) {
      const int r = t / 3, sx = t - 3 * r;
      const int hoff = (a.mode == 1) ? r * HW2 + sx : (2 - r) * HW2 + (2 - sx);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[MI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int hx = hb[i] + hoff;
          af[i] = __builtin_bit_cast(bf16x8, Hs[hx * 8 + ((kk * 4 + fq) ^ (hx & 7))]);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = wn * WN + 16 * j + fr;
          bfr[j] = __builtin_bit_cast(bf16x8, Bh[(buf * BN + row) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    };
    for (int kc = 0; kc < Cs; kc += 64) {
      load_halo(kc);
      load_b(0, kc, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (NOL == 1) {
        if (nol_a) {  // each thread normalizes the halo chunks its own DMA wrote (padding stays 0)
          for (int it = 0; it < nit; ++it) {
            const int f = it * 256 + tid;
            const int px = f >> 3, chp = f & 7;
            const uint32_t hr = fdiv((uint32_t)px, a.fHW2);
            const int hc = px - (int)hr * HW2;
            const int ih = hp0 - 1 + (int)hr, iw = hc - 1;
            if (px < HP && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
              nol_chunk(&Hs[f], nol_tab, kc + (chp ^ (px & 7)) * 8);
          }
        }
      }
      __syncthreads();
      for (int t = 0; t < 9; ++t) {
        if (t + 1 < 9) load_b(t + 1, kc, (t + 1) & 1);
        compute_halo(t, t & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else if constexpr (SPLIT == 2) {
    // sum of the splits' partial tiles, in split order (deterministic)
    const int tl = cy * gridDim.x + tile;
    const f32x4* src = (const f32x4*)a.ws + (size_t)tl * a.splits * (MI * NJ * 256) + tid;
    // ZU splits' fragments in flight per chunk (clamped, selected after the loads): one memory
    // latency per chunk instead of one per split (this launch sat at ~8 us for 24 splits)
    constexpr int ZU = (MI * NJ) <= 4 ? 4 : ((MI * NJ) <= 8 ? 2 : 1);
    for (int z0 = 0; z0 < a.splits; z0 += ZU) {
      f32x4 r[ZU][MI][NJ];
#pragma unroll
      for (int u = 0; u < ZU; ++u) {
        const int z = min(z0 + u, a.splits - 1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) r[u][i][j] = src[(size_t)(z * MI * NJ + i * NJ + j) * 256];
      }
#pragma unroll
      for (int u = 0; u < ZU; ++u)
        if (z0 + u < a.splits)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] += r[u][i][j];
    }
  } else if constexpr (STAGES == 1) {
    for (int kt = kt0; kt < nk; ++kt) {
      issue_loads(kt, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (NOL == 1) {
        if (nol_a) {  // this thread's own A chunks (one row each, logical chunk lc), real pixels only
#pragma unroll
          for (int i = 0; i < A_CH; ++i)
            if ((a_okm >> i) & 1u) nol_chunk(&As[(32 * i + 8 * wid) * 8 + lane], nol_tab, a_kc + lc * 8);
        }
      }
      __syncthreads();
      compute(0);
      __syncthreads();
    }
  } else {
    if (nk > 0) issue_loads(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) issue_loads(kt + 1, cur ^ 1);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  if constexpr (SPLIT == 1) {
    const int tl = cy * gridDim.x + tile;
    f32x4* dst = (f32x4*)a.ws + ((size_t)tl * a.splits + blockIdx.z) * (MI * NJ * 256) + tid;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) dst[(size_t)(i * NJ + j) * 256] = acc[i][j];
    return;
  }
  if constexpr (SPLIT == 3) {
    // fence-free hand-off to the last-arriving split (MI355X_MICROARCH.md, first table row; as
    // gemm256.hip's tail split-K): every wave stores its partial with sc1 and waits for the
    // stores, one lane counts the arrival behind a barrier, the last arriver reads with sc1
    const int tl = cy * gridDim.x + tile;
    constexpr int FR = MI * NJ * 256;  // f32x4 per partial tile
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
        a.ws + (size_t)tl * a.splits * FR * 4, (short)0, a.splits * FR * 16, 0x00020000);
    constexpr int SC1 = 16;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(acc[i][j], rsw,
                                               (uint32_t)(((blockIdx.z * MI * NJ + i * NJ + j) * 256 + tid) * 16), 0, SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last_flag;
    if (tid == 0) last_flag = atomicAdd(a.cnt + tl, 1) == a.splits - 1;
    __syncthreads();
    if (!last_flag) return;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int ZU = (MI * NJ) <= 4 ? 4 : ((MI * NJ) <= 8 ? 2 : 1);
    for (int z0 = 0; z0 < a.splits; z0 += ZU) {
      f32x4 r[ZU][MI][NJ];
#pragma unroll
      for (int u = 0; u < ZU; ++u) {
        const int z = min(z0 + u, a.splits - 1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            r[u][i][j] = __builtin_amdgcn_raw_buffer_load_b128(
                rsw, (uint32_t)(((z * MI * NJ + i * NJ + j) * 256 + tid) * 16), 0, SC1);
      }
#pragma unroll
      for (int u = 0; u < ZU; ++u)
        if (z0 + u < a.splits)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] += r[u][i][j];
    }
    if (tid == 0) a.cnt[tl] = 0;  // ready for the next launch (stream order)
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
      if (m >= Mlim) continue;
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
  float* Sred = (float*)(smem) + (BM * CST) / 2; // [4 waves][2][BN] stats scratch
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
      // 8-B slot XOR-swizzled by row bit 3: the 16 contiguous lanes of a ds_write_b64 group (rows
      // fr = 0..15, row stride 4 banks mod 32) hit 16 distinct bank pairs instead of 2-way
      // conflicting rows fr / fr + 8; the swap stays inside the 16-B chunk the reads fetch
      *(uint2*)&Ct[ml * CST + (nl ^ (((ml >> 3) & 1) << 2))] = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;          // 16-B chunks per row
  constexpr int RPP = 256 / CPR;       // rows per pass
  const int cc = tid % CPR, rr = tid / CPR;
  const int n = n0 + cc * 8;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8];
  if (a.epi >= 4 && a.stats && n < a.N) {
    *(float4*)&mu[0] = *(const float4*)(a.mean + n);
    *(float4*)&mu[4] = *(const float4*)(a.mean + n + 4);
  }
  // NOL kernels, epi 4 with mask coefficients: ReLU mask from c (aux2) -- the BN output y is
  // never read (it was never written: its consumer normalized on load)
  // as a per-channel threshold: fma(c, s, h) > 0  <=>  c > -h/s (s > 0), c < -h/s (s < 0), h > 0 (s == 0)
  // -- 8 thresholds and a sign mask instead of 16 coefficients in registers (the 128x128 variant
  // spilled with the coefficients); differs from the fma only where c * s + h rounds to ~0
  constexpr bool MASKC = NOL == 2;  // every launch of this variant takes its mask from c
  const bool mask_c = MASKC;
  float mthr[MASKC ? 8 : 1];
  uint32_t mgt = 0;  // bit q: keep where c > thr[q] (else where c < thr[q])
  if constexpr (MASKC) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float sc = n < a.N ? a.mask_scale[n + q] : 1.f, sh = n < a.N ? a.mask_shift[n + q] : 0.f;
      mthr[q] = sc != 0.f ? -sh / sc : (sh > 0.f ? -INFINITY : INFINITY);
      mgt |= (sc >= 0.f ? 1u : 0u) << q;
    }
  }
  // row steps in groups of EU: a group's global operand loads (residual C, relu source, BN input,
  // epilogue aux) are all issued before its first store, so their latency overlaps instead of
  // serialising behind each step's store (the compiler cannot move a load across a store to C).
  constexpr int NSTEP = BM / RPP;
  // (the mask-from-c 128x128 variant loads one operand per step instead of two: half the group)
  constexpr int EU0 = (NOL == 2 && BN == 128) ? kNtEpiEU / 2 : kNtEpiEU;
  constexpr int EU = NSTEP < EU0 ? NSTEP : EU0;
  constexpr int NG = NSTEP / EU;
  static_assert(NSTEP % EU == 0, "epilogue groups must tile the row steps");
  constexpr int SLOTS = 1;
  uint4 cv[SLOTS][EU], yq[SLOTS][EU], xq[SLOTS][EU];
  size_t offs[SLOTS][EU];
  bool ok[SLOTS][EU];
  auto load_grp = [&](int g, int sl) {
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int m = m0 + rr + (g * EU + u) * RPP;
      ok[sl][u] = m < Mlim && n < a.N;
      offs[sl][u] = ok[sl][u] ? row_off(m) + n : 0;
      bool acc_ok = true;  // the accumulated-into operand exists at this pixel (aux_even)
      if (ok[sl][u] && a.aux_even && (a.epi == 3 || a.epi == 5)) {
        if (a.mode == 3) {
          acc_ok = cls == 0;  // stride-2 parity class (0, 0) = even h, even w
        } else {
          const uint32_t img = fdiv((uint32_t)m, a.g.fPQ), rem = (uint32_t)m - img * a.g.fPQ.d;
          const uint32_t h = fdiv(rem, a.g.fQ), w = rem - h * a.g.fQ.d;
          acc_ok = ((h | w) & 1u) == 0u;
        }
      }
      if (ok[sl][u] && a.epi >= 4) {
        if (a.epi == 5)
          cv[sl][u] = acc_ok ? epi_ld16<kEpiNtCY>((const bf16_t*)a.C + offs[sl][u]) : make_uint4(0, 0, 0, 0);
        if (!MASKC && a.bn_relu) {
          if (a.mbits)
            yq[sl][u].x = a.mbits[offs[sl][u] >> 3];  // mask byte (offs is a multiple of 8)
          else
            yq[sl][u] = epi_ld16<kEpiNtCY>(a.aux + offs[sl][u]);
        }
        if (a.stats || mask_c) xq[sl][u] = epi_ld16<kEpiNtX>(a.aux2 + offs[sl][u]);
      } else if (ok[sl][u] && (a.epi == 2 || a.epi == 3)) {
        yq[sl][u] = acc_ok ? epi_ld16<kEpiNtCY>(a.aux + offs[sl][u]) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto proc_grp = [&](int g, int sl) {
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      if (!ok[sl][u]) continue;
      const int ml = rr + (g * EU + u) * RPP;
      uint4 v = *(const uint4*)&Ct[ml * CST + cc * 8];
      if ((ml >> 3) & 1) v = make_uint4(v.z, v.w, v.x, v.y);  // undo the write swizzle
      const size_t off = offs[sl][u];
      MI_ASSERT(off + 8 <= (size_t)(a.mode == 3 ? a.M : Mrows) * a.ldc, (long long)off);
      uint4 o = v;
      if (a.epi >= 4) {
        // BN backward: dz = dy * relu mask; stats (sum dz, sum dz * (x - mean)) of the rounded dz
        // (epi 5: dy = this dgrad + the gradient already in C -- a block input's residual sum)
        float f[8];
        unpack8(v, f);
        if (a.epi == 5) {
          float c0[8];
          unpack8(cv[sl][u], c0);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] += c0[q];
        }
        if constexpr (MASKC) {
          float xv[8];
          unpack8(xq[sl][u], xv);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float t = mthr[MASKC ? q : 0];
            const bool keep = ((mgt >> q) & 1u) ? xv[q] > t : xv[q] < t;
            f[q] = keep ? f[q] : 0.f;
          }
        } else if (a.bn_relu && a.mbits) {
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = ((yq[sl][u].x >> q) & 1u) ? f[q] : 0.f;
        } else if (a.bn_relu) {
          float yv[8];
          unpack8(yq[sl][u], yv);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = yv[q] > 0.f ? f[q] : 0.f;
        }
        o = pack8(f);
        if (a.stats) {
          float xv[8];
          unpack8(xq[sl][u], xv);
#pragma unroll
          for (int q = 0; q < 8; ++q) { s1[q] += f[q]; s2[q] += f[q] * (xv[q] - mu[q]); }
        }
      } else {
        if (a.epi) o = epilogue_op_v(a.epi, v, a.aux + off, yq[sl][u]);
        if (a.stats) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) { s1[q] += f[q]; s2[q] += f[q] * f[q]; }
        }
      }
      *(uint4*)((bf16_t*)a.C + off) = o;
    }
  };
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    load_grp(g, 0);
    proc_grp(g, 0);
  }
  if (a.stats) {
    // the lanes of a wave sharing a column chunk (lane mod CPR) are reduced by xor shuffles, then
    // the 4 waves' rows through LDS (Sred is disjoint from Ct), in a fixed order
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s1[q] += __shfl_xor(s1[q], o, 64);
        s2[q] += __shfl_xor(s2[q], o, 64);
      }
    }
    if (lane < CPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        Sred[(wid * 2 + 0) * BN + cc * 8 + q] = s1[q];
        Sred[(wid * 2 + 1) * BN + cc * 8 + q] = s2[q];
      }
    }
    __syncthreads();
    const int prow = cy * a.tiles_m + tm;
    for (int c = tid; c < 2 * BN; c += 256) {
      const int which = c / BN, col = c - which * BN;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += Sred[(w * 2 + which) * BN + col];
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

// MODE: 0 plain [K][N] B operand, 1 conv weight gradient (B gathered from the NHWC input); CS: the
// fused bias-gradient column sums (Linear layers only).  Both are compile-time so that neither the
// gather bookkeeping nor the colsum accumulators occupy registers in the variants that do not use
// them (the conv variant fits 128 VGPRs and runs 4 blocks per CU).
template <int BM, int BN, int STAGES, int MODE = 1, bool CS = false, bool NOL = false, bool CSB = false>
__global__ __launch_bounds__(256, STAGES == 1 ? (MODE == 1 && !CS ? kTnConvBlocksPerCu : kTnBlocksPerCu) : 2)
void tn_kernel(TNArgs a) {
  static_assert(!CSB || (STAGES == 1 && !CS && !NOL), "folded BN backward: the plain one-stage variant");
  static_assert(!NOL || (MODE == 1 && STAGES == 1 && !CS), "normalize-on-load: conv weight gradients");
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MI = WM / 16, NJ = WN / 16;
  constexpr int AU = BM / 4, BU = BN / 4;            // 8-byte units per LDS row
  constexpr int ACPR = BM / 8, BCPR = BN / 8;        // 16-byte chunks per row
  constexpr int A_CH = BK * ACPR / 256, B_CH = BK * BCPR / 256;
  constexpr int A_RSTEP = 256 / ACPR, B_RSTEP = 256 / BCPR;
  constexpr int A_RPI = 64 / ACPR, B_RPI = 64 / BCPR;  // LDS rows per wave-instruction
  __shared__ __attribute__((aligned(16))) uint2 smem[STAGES * BK * (AU + BU)];
  uint2* As = smem;                        // [STAGES][BK][AU]
  uint2* Bs = smem + STAGES * BK * AU;     // [STAGES][BK][BU]

  const int nbn = (a.N + BN - 1) / BN;
  // 1-D grid of tiles x splits, XCD-aware: each XCD owns a contiguous run of (split, tile) work
  // items with the tiles of one split adjacent, so the blocks that read the same reduction rows
  // (one split's k-range of dY and of the gathered input, shared by all its output tiles) run
  // together on one XCD and share its L2 -- with the splits as blockIdx.y and XCD = block id % 8
  // they landed on different XCDs and every tile re-fetched the rows from HBM
  const int tiles = ((a.M + BM - 1) / BM) * nbn;
  const int nsplit = gridDim.x / tiles;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int split = w / tiles, tile = w - split * tiles;
  const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
  const int kbeg = split * a.k_per_split;
  const int kend = min(a.K, kbeg + a.k_per_split);
  if (kbeg >= kend) return;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int a_cc = tid % ACPR, a_r = tid / ACPR;
  const int b_cc = tid % BCPR, b_r = tid / BCPR;
  // lane-linear LDS image, tr-read swizzle u' = u ^ sw(k) applied on the SOURCE side
  const int a_lc = a_cc ^ (tr_swz<AU>(a_r) >> 1);
  const int b_lc = b_cc ^ (tr_swz<BU>(b_r) >> 1);

  // conv-mode B column geometry: this thread's 8 columns n0 + 8*b_lc .. +7 = (tap, channel c0..c0+7)
  int tap_r = 0, tap_s = 0, c0 = 0;
  if constexpr (MODE == 1) {
    const int ncol = n0 + b_lc * 8;
    const int tap = ncol / a.g.Cs;
    c0 = ncol - tap * a.g.Cs;
    tap_r = tap / a.g.S;
    tap_s = tap - tap_r * a.g.S;
  }
  const int H = a.g.H, W = a.g.W, P = a.g.P, Q = a.g.Q, Cs = a.g.Cs;
  const int st = a.g.stride, pad = a.g.pad;
  // NOL: this thread's 8 gathered channels c0..c0+7 are fixed for the whole block
  float nsc[NOL ? 8 : 1], nsh[NOL ? 8 : 1];
  if constexpr (NOL) {
    const bool live = n0 + b_lc * 8 < a.N;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      nsc[q] = live ? a.nol_scale[c0 + q] : 0.f;
      nsh[q] = live ? a.nol_shift[c0 + q] : 0.f;
    }
  }

  // ---- per-thread B rows (mode 1): output pixel (img, p, q) of reduction row k, advanced by BK
  int b_img[B_CH], b_p[B_CH], b_q[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const uint32_t k = (uint32_t)min(kbeg + b_r + B_RSTEP * i, a.K - 1);
    if constexpr (MODE == 1) {
      const uint32_t img = fdiv(k, a.g.fPQ);
      const uint32_t rem = k - img * a.g.fPQ.d;
      const uint32_t p = fdiv(rem, a.g.fQ);
      b_img[i] = (int)img; b_p[i] = (int)p; b_q[i] = (int)(rem - p * a.g.fQ.d);
    } else {
      b_img[i] = b_p[i] = b_q[i] = 0;
    }
  }
  // per-step carry deltas for +BK pixels
  const int dq = BK % Q, dp = (BK / Q) % P, dimg = BK / (P * Q);

  // folded BN backward: a block's rows lie wholly in dz (A) or in c (A2, rows m - msplit)
  const bool a_second = CSB && a.msplit && m0 >= a.msplit;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a_second ? a.A2 : a.A), (short)0, a_second ? a.a2_bytes : a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.b_bytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;
  const int a_m = m0 + a_lc * 8;
  const int a_mo = a_second ? a_m - a.msplit : a_m;  // row within the operand read
  const int b_n = n0 + b_lc * 8;

  uint32_t b_okm = 0;  // NOL: B chunks of the last issued k-step that hold real input pixels
  auto issue_loads = [&](int k0, int buf) {
    b_okm = 0;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int k = k0 + a_r + A_RSTEP * i;
      const bool ok = k < kend && a_m < a.M;
      const uint32_t vo = ok ? (uint32_t)(k * (a_second ? a.lda2 : a.lda) + a_mo) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, LDS_PTR(void, &As[(buf * BK + A_RSTEP * i + wid * A_RPI) * AU]), 16, vo, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int k = k0 + b_r + B_RSTEP * i;
      uint32_t vo = OOB;
      if constexpr (MODE == 0) {
        if (k < kend && b_n < a.N) vo = (uint32_t)(k * a.ldb + b_n) * 2u;
      } else {
        const int ih = b_p[i] * st - pad + tap_r, iw = b_q[i] * st - pad + tap_s;
        if (k < kend && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          vo = (b_n < a.N) ? (uint32_t)((((b_img[i] * H + ih) * W + iw) * Cs) + c0) * 2u : OOB;
        b_okm |= (vo != OOB ? 1u : 0u) << i;
        // advance this row by BK output pixels
        int q = b_q[i] + dq, p = b_p[i] + dp, img = b_img[i] + dimg;
        if (q >= Q) { q -= Q; ++p; }
        if (p >= P) { p -= P; ++img; }
        b_q[i] = q; b_p[i] = p; b_img[i] = img;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, LDS_PTR(void, &Bs[(buf * BK + B_RSTEP * i + wid * B_RPI) * BU]), 16, vo, 0, 0, 0);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  // fused bias gradient: the first column-tile's blocks also reduce their A fragments against a
  // ones operand (one extra MFMA per 16 rows in the wn == 0 waves): D[m][*] = sum_k A[k][m]
  const bool do_cs = CS && (tile % nbn) == 0 && wn == 0;
  f32x4 acc_cs[CS ? MI : 1];
#pragma unroll
  for (int i = 0; i < (CS ? MI : 1); ++i) acc_cs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  short ones_s __attribute__((ext_vector_type(8))) = {0x3F80, 0x3F80, 0x3F80, 0x3F80,
                                                      0x3F80, 0x3F80, 0x3F80, 0x3F80};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, ones_s);
  // folded BN backward: the column sums of B (every row of ones x B holds them), first row-tile only
  const bool do_csb = CSB && tile / nbn == 0 && wm == 0;
  f32x4 acc_sb[CSB ? NJ : 1];
#pragma unroll
  for (int j = 0; j < (CSB ? NJ : 1); ++j) acc_sb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NJ];
      const int k1 = kk * 32 + 8 * g + q4;
      const int k2 = k1 + 4;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int u = (wm * WM + 16 * i) / 4 + p4;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &As[(cur * BK + k1) * AU + (u ^ tr_swz<AU>(k1))]));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &As[(cur * BK + k2) * AU + (u ^ tr_swz<AU>(k2))]));
        short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v8);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int u = (wn * WN + 16 * j) / 4 + p4;
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
      if constexpr (CS) {
        if (do_cs)
#pragma unroll
        for (int i = 0; i < MI; ++i) acc_cs[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, acc_cs[i], 0, 0, 0);
      }
      if constexpr (CSB) {
        if (do_csb)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc_sb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bfr[j], acc_sb[j], 0, 0, 0);
      }
    }
  };

  const int nk = (kend - kbeg + BK - 1) / BK;
  if constexpr (STAGES == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      issue_loads(kbeg + kt * BK, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (NOL) {  // this thread's own B chunks (real pixels only; padding stays 0)
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
          if (!((b_okm >> i) & 1u)) continue;
          uint4* p = (uint4*)&Bs[(B_RSTEP * i + wid * B_RPI) * BU + 2 * lane];
          float f[8];
          unpack8(*p, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = fmaxf(fmaf(f[q], nsc[q], nsh[q]), 0.f);
          *p = pack8(f);
        }
      }
      __syncthreads();
      compute(0);
      __syncthreads();
    }
  } else {
    issue_loads(kbeg, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) issue_loads(kbeg + (kt + 1) * BK, cur ^ 1);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // bias gradient first (the split-K epilogues below may return early): every column of the
  // ones-product holds the column sum; lane li == 0 adds it
  if constexpr (CS) if (do_cs && li == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + 16 * i + 4 * g + r;
        if (m < a.M) atomicAdd(a.colsum + m, acc_cs[i][r]);
      }
  }

  // folded BN backward: this split's column sums of B (lane g == 0 holds row 0 of ones x B)
  if constexpr (CSB) if (do_csb && g == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * WN + 16 * j + li;
      if (n < a.N) a.bsum[(size_t)split * a.N + n] = acc_sb[j][0];
    }
  }

  // epilogue: lane holds D[m = 16i + 4g + r][n = 16j + li]
  const bool single = (nsplit == 1);
  if (!single && a.ws) {
    // split-K: this block's partial tile goes to its own slab in fragment order -- every store is one
    // fully coalesced 1 KB wave-instruction (64 lanes x float4) -- and tn_splitk_reduce_kernel sums
    // the splits into C: deterministic, and no fp32 atomics (~1.3 TB/s chip-wide) on the hot path
    if (STAGES == 1 && a.cnt) {  // GLDS (default) slab variants only
      // one launch: fence-free hand-off to the last-arriving split of the tile (as nt_kernel's
      // SPLIT 3): sc1 partial stores, wait, barrier, one arrival count; the last arriver sums the
      // partials in split order from 0 -- what tn_splitk_reduce_kernel does for fewer than 8
      // splits (one split group), so both paths are bit-identical
      constexpr int FR = BM * BN / 4;  // f32x4 per partial tile
      constexpr int SC1 = 16;
      const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
          a.ws + (size_t)tile * nsplit * FR * 4, (short)0, nsplit * FR * 16, 0x00020000);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(
              acc[i][j], rsw, (uint32_t)((split * FR + ((i * NJ + j) * 4 + wid) * 64 + lane) * 16), 0, SC1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __shared__ int last_flag;
      if (tid == 0) last_flag = atomicAdd(a.cnt + tile, 1) == nsplit - 1;
      __syncthreads();
      if (!last_flag) return;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // half a partial tile's fragments in flight at a time: the whole tile's (64 VGPRs next to
      // the 64 accumulators) spilled the 3-blocks-per-CU conv variant
      constexpr int IU = MI >= 2 ? MI / 2 : 1;
      for (int z = 0; z < nsplit; ++z) {
#pragma unroll
        for (int i0 = 0; i0 < MI; i0 += IU) {
          f32x4 r[IU][NJ];
#pragma unroll
          for (int i = 0; i < IU; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              r[i][j] = __builtin_amdgcn_raw_buffer_load_b128(
                  rsw, (uint32_t)((z * FR + (((i0 + i) * NJ + j) * 4 + wid) * 64 + lane) * 16), 0, SC1);
#pragma unroll
          for (int i = 0; i < IU; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i0 + i][j] += r[i][j];
        }
      }
      if (tid == 0) a.cnt[tile] = 0;  // ready for the next launch (stream order)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = n0 + wn * WN + 16 * j + li;
          if (n >= a.N) continue;
          float c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) c[r] = a.C[(size_t)min(m0 + wm * WM + 16 * i + 4 * g + r, a.M - 1) * a.ldc + n];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WM + 16 * i + 4 * g + r;
            if (m < a.M) a.C[(size_t)m * a.ldc + n] = c[r] + acc[i][j][r];
          }
        }
      }
      return;
    }
    f32x4* slab = (f32x4*)a.ws + ((size_t)tile * nsplit + split) * (BM * BN / 4);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x4* q = slab + ((i * NJ + j) * 4 + wid) * 64 + lane;
        *q = acc[i][j];
      }
  } else {
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
}

// Sum the split-K slabs of tn_kernel<BM, BN> into C (+=).  Slab position p = ((i*NJ + j)*4 +
// wave)*64 + lane holds D[m = 16i + 4g + r][n = 16j + li] (r = 0..3) of wave (wm, wn).  A block
// covers 256/G consecutive positions x G split groups (thread t: position t % (256/G), group
// t / (256/G), summing splits group, group + G, ...), so a tile with hundreds of splits is still
// read by the whole chip; the G partials are combined in LDS in a fixed order (deterministic).
template <int BM, int BN>
__global__ __launch_bounds__(256) void tn_splitk_reduce_kernel(const f32x4* __restrict__ ws, float* __restrict__ C,
                                                               int M, int N, int ldc, int nbn, int splits,
                                                               int log2g) {
  constexpr int WM = BM / 2, WN = BN / 2, NJ = WN / 16;
  constexpr int PER = BM * BN / 4;
  __shared__ f32x4 part[256];
  const int G = 1 << log2g, PB = 256 >> log2g;
  const int tile = blockIdx.y;
  const int pl = threadIdx.x & (PB - 1), grp = threadIdx.x >> (8 - log2g);
  const int p = blockIdx.x * PB + pl;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    // 8 split reads per chunk all in flight (clamped indices, selected after the loads): the
    // unrolled `v += src[...]` loop left a vmcnt(0) behind every other load -- a reduce of 8
    // splits per thread paid ~8 memory latencies
    const f32x4* src = ws + (size_t)tile * splits * PER + min(p, PER - 1);
    for (int s0 = grp; s0 < splits; s0 += 8 * G) {
      f32x4 r[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4* q = src + (size_t)min(s0 + i * G, splits - 1) * PER;
        r[i] = *q;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (s0 + i * G < splits) v += r[i];
    }
  }
  part[threadIdx.x] = v;
  __syncthreads();
  if (grp != 0 || p >= PER) return;
  for (int g2 = 1; g2 < G; ++g2) v += part[g2 * PB + pl];
  const int lane = p & 63, wid = (p >> 6) & 3, ij = p >> 8;
  const int i = ij / NJ, j = ij - i * NJ;
  const int wm = wid >> 1, wn = wid & 1, g = lane >> 4, li = lane & 15;
  const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
  const int n = n0 + wn * WN + 16 * j + li;
  if (n >= N) return;
  // the four gradient rows read together (clamped), then written back
  float c[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = C[(size_t)min(m0 + wm * WM + 16 * i + 4 * g + r, M - 1) * ldc + n];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm * WM + 16 * i + 4 * g + r;
    if (m < M) C[(size_t)m * ldc + n] = c[r] + v[r];
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

// All conv weights of a flat bf16 parameter buffer in ONE launch (after the optimizer step):
// desc[t] = {src element offset, dst element offset, K, RS, C, first block}; every 64x64 (k, c)
// tile of every tap is one block; a block finds its tensor by binary search over first-block.
// Replaces one mi_conv_wtrans launch per conv per backward (52 for ResNet-50).
struct WtDesc {
  int src, dst, K, RS, C, blk0;
};
__global__ void wtrans_multi_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                    const WtDesc* __restrict__ desc, int ntens) {
  __shared__ bf16_t t[64][65];
  const int b = blockIdx.x;
  int lo = 0, hi = ntens - 1;
  while (lo < hi) {  // last tensor with blk0 <= b
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const WtDesc d = desc[lo];
  const int nc = (d.C + 63) >> 6, nkb = (d.K + 63) >> 6;
  int r0 = b - d.blk0;
  const int cx = r0 % nc;
  r0 /= nc;
  const int ky = r0 % nkb;
  const int tap = r0 / nkb;
  const int k0 = ky * 64, c0 = cx * 64;
  const bf16_t* src = w + d.src;
  bf16_t* dst = wt + d.dst;
  if ((d.C & 7) == 0 && (d.K & 7) == 0) {
    // 16-byte accesses both ways (every row of both layouts is a whole number of 8-element
    // chunks): thread -> (row, chunk) pairs; the transposed chunk is gathered from 8 LDS rows
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + 256 * i, r = idx >> 3, ch = idx & 7;
      const int k = k0 + r, c = c0 + 8 * ch;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < d.K && c < d.C) v = *(const uint4*)(src + ((size_t)k * d.RS + tap) * d.C + c);
      const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[r][8 * ch + 2 * j] = (bf16_t)(u[j] & 0xffffu);
        t[r][8 * ch + 2 * j + 1] = (bf16_t)(u[j] >> 16);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + 256 * i, r = idx >> 3, ch = idx & 7;  // r: output row (c), ch: k chunk
      const int c = c0 + r, k = k0 + 8 * ch;
      if (c < d.C && k < d.K) {
        uint32_t u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          u[j] = (uint32_t)t[8 * ch + 2 * j][r] | ((uint32_t)t[8 * ch + 2 * j + 1][r] << 16);
        *(uint4*)(dst + ((size_t)c * d.RS + tap) * d.K + k) = make_uint4(u[0], u[1], u[2], u[3]);
      }
    }
    return;
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    t[r][tx] = (k < d.K && c < d.C) ? src[((size_t)k * d.RS + tap) * d.C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < d.C && k < d.K) dst[((size_t)c * d.RS + tap) * d.K + k] = t[tx][r];
  }
}

// byte extent for a buffer resource; 0 (= use the register-staged path) beyond 2 GiB
static int rsrc_bytes(int64_t elems) {
  const int64_t b = elems * 2;
  return b > 0x7FFFFFF0LL ? 0 : (int)b;
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

static int g_nt_glds = -1;  // TN: 0 = register staging, else direct-to-LDS; NT: number of LDS stages (1|2)
static int g_nt_stages = -1;
static bool glds_on() {
  if (g_nt_glds < 0) {
    const char* e = std::getenv("MI355X_DP_GLDS");
    g_nt_glds = (e && e[0] == '0') ? 0 : 1;
  }
  return g_nt_glds != 0;
}
static int nt_stages() {
  if (g_nt_stages < 0) {
    const char* e = std::getenv("MI355X_DP_NT_STAGES");
    g_nt_stages = (e && e[0] == '2') ? 2 : 1;
  }
  return g_nt_stages;
}

static float* splitk_workspace(size_t floats, hipStream_t st);
static int* splitk_counters(hipStream_t st);

// split-K of the NT kernel for small grids: a layer-4 conv of ResNet-18 on 32x32 images at batch
// 32 is 8 output tiles of 72 k-steps each -- 8 of 256 CUs walking a latency-bound serial chain.
// With fewer than MI355X_DP_NT_SPLIT_BLOCKS (default 128) blocks, the k-steps are split over
// blockIdx.z (>= 2 k-steps per split, about 256 blocks in all), the partial tiles go to the
// stream's slab workspace and a second launch sums them in split order and runs the epilogue.
// MI355X_DP_NT_SPLITK=0 disables.
static int g_nt_split_blocks = -1;
// MI355X_DP_NT_SPLIT_FUSED=0: the two-launch split-K (partials, then a reduce + epilogue launch)
static int g_nt_split_fused = -1;
static bool nt_split_fused() {
  if (g_nt_split_fused < 0) {
    const char* e = std::getenv("MI355X_DP_NT_SPLIT_FUSED");
    g_nt_split_fused = (e && e[0] == '0') ? 0 : 1;
  }
  return g_nt_split_fused != 0;
}
constexpr int SPLITK_COUNTERS = 4096;
// TN (weight-gradient) split-K reduced by the last-arriving split, opt-in (MI355X_DP_TN_SPLIT_FUSED=1).
// Bit-identical to the reduce launch but not faster: ResNet-50 / -152 bs256 neutral (12,617 vs
// 12,627, 5,523 vs 5,521 img/s), ResNet-18 @ 32x32 bs32 graphed -4 % (26.1k vs 27.4k, three
// interleaved pairs, profiles/raw/r3_tnf*.log) -- one block summing up to 7 partial tiles is a
// longer tail than the chip-wide reduce kernel
static int g_tn_split_fused = -1;
static bool tn_split_fused() {
  if (g_tn_split_fused < 0) {
    const char* e = std::getenv("MI355X_DP_TN_SPLIT_FUSED");
    g_tn_split_fused = (e && e[0] == '1') ? 1 : 0;
  }
  return g_tn_split_fused != 0;
}
static int nt_split_blocks() {
  if (g_nt_split_blocks < 0) {
    const char* e = std::getenv("MI355X_DP_NT_SPLITK");
    const char* b = std::getenv("MI355X_DP_NT_SPLIT_BLOCKS");
    g_nt_split_blocks = (e && e[0] == '0') ? 0 : (b ? std::max(0, std::atoi(b)) : 128);
  }
  return g_nt_split_blocks;
}

template <int BM, int BN>
hipError_t launch_nt(NTArgs& a, hipStream_t st) {
  int classes = 1, mrows = a.M;
  if (a.mode == 3) {
    classes = a.ncls;
    mrows = 0;
    const int nimg = a.M / (a.g.P * a.g.Q);
    for (int c = 0; c < classes; ++c)
      mrows = std::max(mrows, nimg * a.g.Pc[a.cls_map[c]] * a.g.Qc[a.cls_map[c]]);
  }
  a.tiles_m = cdiv(mrows, BM);
  if (a.halo_rp > 0) a.tiles_m = (a.M / (a.g.P * a.g.Q)) * a.halo_pb;
  int grid = a.tiles_m * cdiv(a.N, BN);
  if (a.a_bytes <= 0 || a.b_bytes <= 0) return hipErrorInvalidValue;  // operand > 2 GiB: split the batch
  if (a.nol_scale || a.mask_scale) {
    // normalize-on-load (forward) / mask-from-c (data gradient) variants: single-stage, no split-K
    if (a.mode == 4 || (a.nol_scale && (a.mode != 1 || a.g.Cs > NOL_MAX_C)) || (a.mask_scale && a.epi != 4) ||
        (a.nol_scale && a.mask_scale))
      return hipErrorNotSupported;
    if (a.nol_scale) {
      if (a.halo_rp > 0)
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, true, 0, 1>), dim3(grid), dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, false, 0, 1>), dim3(grid, classes), dim3(256), 0, st, a);
    } else {
      if (a.halo_rp > 0)
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, true, 0, 2>), dim3(grid), dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, false, 0, 2>), dim3(grid, classes), dim3(256), 0, st, a);
    }
    return hipGetLastError();
  }
  if (a.halo_rp == 0 && a.mode != 4 && grid * classes < nt_split_blocks()) {
    const int cpt = a.mode == 0 ? 0 : (int)a.g.fCpt.d;
    const int nk = a.mode == 0 ? cdiv(a.K, BK)
                 : a.mode == 3 ? cdiv(a.g.R, a.g.stride) * cdiv(a.g.S, a.g.stride) * cpt : a.g.R * a.g.S * cpt;
    int splits = std::min(nk / 2, 256 / std::max(grid * classes, 1));
    if (splits >= 2) {
      a.ksplit = cdiv(nk, splits);
      a.splits = cdiv(nk, a.ksplit);
      a.ws = splitk_workspace((size_t)grid * classes * a.splits * BM * BN, st);
      a.cnt = nt_split_fused() ? splitk_counters(st) : nullptr;
      if (a.ws && a.cnt && grid * classes <= SPLITK_COUNTERS) {
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, false, 3>), dim3(grid, classes, a.splits), dim3(256), 0, st,
                           a);
        return hipGetLastError();
      }
      if (a.ws) {
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, false, 1>), dim3(grid, classes, a.splits), dim3(256), 0, st,
                           a);
        hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, false, 2>), dim3(grid, classes), dim3(256), 0, st, a);
        return hipGetLastError();
      }
    }
  }
  if (a.halo_rp > 0)
    hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false, true>), dim3(grid), dim3(256), 0, st, a);
  else if (a.mode == 4)
    hipLaunchKernelGGL((nt_kernel<BM, BN, 1, true>), dim3(grid, classes), dim3(256), 0, st, a);
  else if (nt_stages() == 2)
    hipLaunchKernelGGL((nt_kernel<BM, BN, 2, false>), dim3(grid, classes), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((nt_kernel<BM, BN, 1, false>), dim3(grid, classes), dim3(256), 0, st, a);
  return hipGetLastError();
}

// tile choice shared with the host-side stats-slab sizing (mi_nt_tile_m)
int nt_choice(int M, int N) {
  if (N <= 64) return 1;                                         // 128x64
  if ((int64_t)cdiv(M, 128) * cdiv(N, 128) < 512) return 2;     // 64x64 (fill 256 CUs)
  return 0;                                                      // 128x128
}

// Halo tiling (see nt_kernel) for a 3x3 / stride-1 / pad-1 conv whose row grid is P x Q (gathered
// tensor the same size), Cs channels: rows per tile, or 0 when it does not apply (rows of >= 75 %
// of a 128-row tile, halo within HALO_PX; 64x64-tile shapes keep the gather path).
// MI355X_DP_HALO=0 disables.
static int g_halo = -1;
static int halo_rp(int M, int N, int R, int S, int stride, int pad, int Cs, int H, int W, int P, int Q) {
  if (g_halo < 0) {
    const char* e = std::getenv("MI355X_DP_HALO");
    g_halo = (e && e[0] == '0') ? 0 : 1;
  }
  if (!g_halo || R != 3 || S != 3 || stride != 1 || pad != 1 || Cs % 64 != 0 || H != P || W != Q) return 0;
  if (nt_choice(M, N) == 2) return 0;
  const int rp = std::min(128 / Q, P);
  if (rp < 1 || rp * Q * 4 < 128 * 3 || (rp + 2) * (Q + 2) > HALO_PX) return 0;
  return rp;
}

// MI355X_DP_TRACE_GEMM=1: print every distinct GEMM / conv dispatch (kernel, geometry, epilogue) once
// to stderr -- maps rocprof kernel rows (grid sizes) back to the network's layers.
static int g_trace_gemm = -1;
static void trace_gemm(const char* what, int mode, int M, int N, int K, int Cs, int R, int stride, int epi,
                       int stats, int blocks, int splits) {
  if (g_trace_gemm < 0) {
    const char* e = std::getenv("MI355X_DP_TRACE_GEMM");
    g_trace_gemm = (e && e[0] == '1') ? 1 : 0;
  }
  if (!g_trace_gemm) return;
  static std::vector<std::array<int, 12>> seen;
  const std::array<int, 12> key{(int)(intptr_t)what, mode, M, N, K, Cs, R, stride, epi, stats, blocks, splits};
  for (auto& k : seen)
    if (k == key) return;
  seen.push_back(key);
  fprintf(stderr, "[gemm] %s mode=%d M=%d N=%d K=%d Cs=%d R=%d s=%d epi=%d stats=%d blocks=%d splits=%d\n", what,
          mode, M, N, K, Cs, R, stride, epi, stats, blocks, splits);
}

hipError_t dispatch_nt(NTArgs& a, hipStream_t st) {
  if (a.mode == 1 || a.mode == 2) {
    const ConvGeom& g = a.g;
    const int rp = halo_rp(a.M, a.N, g.R, g.S, g.stride, g.pad, g.Cs, g.H, g.W, g.P, g.Q);
    if (rp > 0) {
      a.halo_rp = rp;
      a.halo_pb = cdiv(g.P, rp);
      a.fPB = make_fastdiv((uint32_t)a.halo_pb);
      a.fHW2 = make_fastdiv((uint32_t)(g.Q + 2));
      trace_gemm(nt_choice(a.M, a.N) == 1 ? "nt128x64-halo" : "nt128x128-halo", a.mode, a.M, a.N, a.K, g.Cs, g.R,
                 g.stride, a.epi, a.stats != nullptr, (a.M / (g.P * g.Q)) * a.halo_pb, 1);
      return nt_choice(a.M, a.N) == 1 ? launch_nt<128, 64>(a, st) : launch_nt<128, 128>(a, st);
    }
  }
  {
    static const char* names[3] = {"nt128x128", "nt128x64", "nt64x64"};
    const int c = nt_choice(a.M, a.N);
    const int bm = c == 2 ? 64 : 128, bn = c == 0 ? 128 : 64;
    trace_gemm(names[c], a.mode, a.M, a.N, a.K, a.g.Cs, a.g.R, a.g.stride, a.epi, a.stats != nullptr,
               cdiv(a.M, bm) * cdiv(a.N, bn), a.mode == 3 ? a.ncls : 1);
  }
  switch (nt_choice(a.M, a.N)) {
    case 1: return launch_nt<128, 64>(a, st);
    case 2: return launch_nt<64, 64>(a, st);
    default: return launch_nt<128, 128>(a, st);
  }
}

// Split-K slab workspace of the TN kernels (fp32, grown on demand and reused in stream order).  One
// per device for every stream, plus one for the device's registered weight-gradient side stream
// (mi_register_wgrad_stream): side-stream weight gradients run concurrently with compute-stream
// TN work and must not share slabs with it; likewise the residual blocks' auxiliary (shortcut)
// stream (mi_register_aux_stream), whose shortcut weight gradient can run concurrently with
// compute-stream TN work when the weight-gradient stream is off.  Contract: the first call that needs a given size
// allocates (hipMalloc) -- never inside a HIP graph capture (the launch then takes the workspace-free
// schedule); GraphedStep's eager warm-up step makes every allocation first (capture streams use the
// shared slot, like the warm-up).  A grown workspace retires its old buffer instead of freeing it
// (common.h): graphs captured before the growth keep replaying into live memory.
// MI355X_DP_TN_SLABS=0 selects the fp32-atomic split-K path instead.
struct SplitkWs { float* p = nullptr; size_t n = 0; };
static SplitkWs g_splitk_ws[16][3];  // [device][0: any other stream, 1: wgrad stream, 2: aux stream]
static hipStream_t g_wgrad_stream[16];
static hipStream_t g_aux_stream[16];
static std::mutex g_splitk_mu;
static float* splitk_workspace(size_t floats, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_splitk_mu);
  const int slot = st == nullptr ? 0 : st == g_wgrad_stream[dev & 15] ? 1 : st == g_aux_stream[dev & 15] ? 2 : 0;
  SplitkWs& w = g_splitk_ws[dev & 15][slot];
  if (w.n < floats) {
    if (mi_stream_capturing(st)) {  // common.h: never allocate inside a capture
      mi_ws_capture_warn("split-K slab");
      return nullptr;  // -> unsplit / atomic path
    }
    const size_t n = std::max(floats, (size_t)16 << 20);  // >= 64 MB: every RN50 / RN152 wgrad fits
    float* p = nullptr;
    if (hipMalloc(&p, n * sizeof(float)) != hipSuccess) return nullptr;  // -> atomic path
    mi_ws_retire(w.p);  // graphs captured earlier may still replay into it (common.h)
    w.p = p;
    w.n = n;
  }
  return w.p;
}
// per-tile arrival counters of the fused NT split-K (SPLIT 3), one zeroed table per (device, slot)
// like the slab workspace; allocated on first use (a warm-up step runs before any capture) and
// left zeroed by every launch's last arrivers
static int* g_splitk_cnt[16][3];
static int* splitk_counters(hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_splitk_mu);
  const int slot = st == nullptr ? 0 : st == g_wgrad_stream[dev & 15] ? 1 : st == g_aux_stream[dev & 15] ? 2 : 0;
  int*& p = g_splitk_cnt[dev & 15][slot];
  if (!p) {
    if (hipMalloc(&p, sizeof(int) * SPLITK_COUNTERS) != hipSuccess) { p = nullptr; return nullptr; }
    if (hipMemset(p, 0, sizeof(int) * SPLITK_COUNTERS) != hipSuccess) return nullptr;
  }
  return p;
}
// the same per-stream slab workspace for the other kernels of this library that reduce per-block
// partials deterministically (stem_conv.hip's weight gradient); nullptr -> their atomic path
extern "C" float* mi_partials_workspace(size_t floats, hipStream_t st) { return splitk_workspace(floats, st); }
// test hook (tests/test_graph_workspaces_gpu.py): grow this stream's split-K slab to at least `floats`
MI_API int mi_splitk_ws_reserve(size_t floats, hipStream_t st) { return splitk_workspace(floats, st) ? 0 : 1; }
static int g_tn_slabs = -1;
static bool tn_slabs_on() {
  if (g_tn_slabs < 0) {
    const char* e = std::getenv("MI355X_DP_TN_SLABS");
    g_tn_slabs = (e && e[0] == '0') ? 0 : 1;
  }
  return g_tn_slabs != 0;
}

// TN k-loop depth with direct-to-LDS loads: 1 = load, wait, compute per k-step (default); 2 = the
// next k-step's loads in flight under the current one's MFMAs (MI355X_DP_TN_STAGES=2, A/B)
static int g_tn_stages = -1;
static int tn_stages() {
  if (g_tn_stages < 0) {
    const char* e = std::getenv("MI355X_DP_TN_STAGES");
    g_tn_stages = (e && e[0] == '2') ? 2 : 1;
  }
  return g_tn_stages;
}

template <int BM, int BN>
hipError_t launch_tn(TNArgs& a, hipStream_t st, int target_blocks) {
  int tiles = cdiv(a.M, BM) * cdiv(a.N, BN);
  int ksteps = cdiv(a.K, BK);
  int splits = std::max(1, std::min(ksteps, target_blocks / std::max(tiles, 1)));
  int steps_per = cdiv(ksteps, splits);
  a.k_per_split = steps_per * BK;
  splits = cdiv(a.K, a.k_per_split);
  trace_gemm(BM == 128 ? (BN == 128 ? "tn128x128" : "tn128x64") : (BN == 128 ? "tn64x128" : "tn64x64"), a.mode,
             a.M, a.N, a.K, a.g.Cs, a.g.R, a.g.stride, 0, 0, tiles, splits);
  if (a.a_bytes <= 0 || a.b_bytes <= 0) return hipErrorInvalidValue;  // operand > 2 GiB: split the batch
  a.ws = nullptr;
  a.cnt = nullptr;
  // split-K partials through slabs (deterministic), the Linear weight gradients with their fused
  // bias column sums included: fp32 atomics there cost ~37 us per ViT-B/16 weight gradient, all of
  // it after the last k-step (every split block finishes in the same wave)
  if (splits > 1 && tn_slabs_on())
    a.ws = splitk_workspace((size_t)tiles * splits * BM * BN, st);
  // fewer than 8 splits: the reduce is one split group (in-order sum), which the last-arriving
  // split runs itself -- no reduce launch; more splits keep the chip-wide reduce kernel
  const int st_n = glds_on() ? tn_stages() : 2;
  if (a.ws && splits < 8 && tiles <= SPLITK_COUNTERS && st_n == 1 && tn_split_fused() && !a.nol_scale)
    a.cnt = splitk_counters(st);
  if (a.nol_scale) {
    if (a.mode != 1 || st_n != 1 || a.cnt) return hipErrorNotSupported;
    hipLaunchKernelGGL((tn_kernel<BM, BN, 1, 1, false, true>), dim3(tiles * splits), dim3(256), 0, st, a);
  } else if (a.mode == 1 && a.bsum) {  // folded BN backward (mi_conv2d_wgrad_fbb)
    hipLaunchKernelGGL((tn_kernel<BM, BN, 1, 1, false, false, true>), dim3(tiles * splits), dim3(256), 0, st, a);
  } else if (a.mode == 1) {
    if (st_n == 1) hipLaunchKernelGGL((tn_kernel<BM, BN, 1, 1, false>), dim3(tiles * splits), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tn_kernel<BM, BN, 2, 1, false>), dim3(tiles * splits), dim3(256), 0, st, a);
  } else if (a.colsum) {
    if (st_n == 1) hipLaunchKernelGGL((tn_kernel<BM, BN, 1, 0, true>), dim3(tiles * splits), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tn_kernel<BM, BN, 2, 0, true>), dim3(tiles * splits), dim3(256), 0, st, a);
  } else {
    if (st_n == 1) hipLaunchKernelGGL((tn_kernel<BM, BN, 1, 0, false>), dim3(tiles * splits), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tn_kernel<BM, BN, 2, 0, false>), dim3(tiles * splits), dim3(256), 0, st, a);
  }
  if (a.ws && !a.cnt) {
    // split groups per position: ~8 slab reads per thread, at most 64 groups, and enough blocks
    int log2g = 0;
    while (log2g < 6 && (splits >> (log2g + 3)) > 0) ++log2g;
    const int pb = 256 >> log2g;
    hipLaunchKernelGGL((tn_splitk_reduce_kernel<BM, BN>), dim3(cdiv(BM * BN / 4, pb), tiles), dim3(256), 0, st,
                       (const f32x4*)a.ws, a.C, a.M, a.N, a.ldc, cdiv(a.N, BN), splits, log2g);
  }
  return hipGetLastError();
}

// split-K block target of the TN (weight-gradient) kernels: more splits fill the chip, but every
// split adds a partial tile of slab traffic and a longer reduce (MI355X_DP_TN_BLOCKS, default 768).
// On the weight-gradient side stream the TN kernels share the CUs with the data-gradient chain and
// a smaller grid is better (MI355X_DP_TN_BLOCKS_SIDE, default 384: RN50 bs256 12.56k img/s vs 12.32k
// at 768, 12.21k at 256; RN152 5463 vs 5295 -- profiles/rn50_bs256_wgrad_stream.md).
static int g_tn_blocks = -1, g_tn_blocks_side = -1;
static int tn_target_blocks(hipStream_t st) {
  if (g_tn_blocks < 0) {
    const char* e = std::getenv("MI355X_DP_TN_BLOCKS");
    g_tn_blocks = e ? std::max(64, std::atoi(e)) : 768;
    const char* es = std::getenv("MI355X_DP_TN_BLOCKS_SIDE");
    g_tn_blocks_side = es ? std::max(64, std::atoi(es)) : (e ? g_tn_blocks : 384);
  }
  int dev = 0;
  hipGetDevice(&dev);
  return (st != nullptr && st == g_wgrad_stream[dev & 15]) ? g_tn_blocks_side : g_tn_blocks;
}

hipError_t dispatch_tn(TNArgs& a, hipStream_t st) {
  const int target = tn_target_blocks(st);
  bool n64 = a.N <= 64;
  bool m64 = a.M <= 64;
  if (m64 && n64) return launch_tn<64, 64>(a, st, target);
  if (m64) return launch_tn<64, 128>(a, st, target);
  if (n64) return launch_tn<128, 64>(a, st, target);
  return launch_tn<128, 128>(a, st, target);
}

}  // namespace

// ============================================================== C ABI
// Conv forward: x NHWC [Nb,H,W,C] bf16, w [K][R][S][C] bf16, y NHWC [Nb,P,Q,K].
// Select direct-to-LDS (buffer_load ... lds) staging (1) or register staging (0) for all GEMM kernels.
// Weight-gradient split-K reduction: 1 = slab workspace + reduce kernel (default), 0 = fp32 atomics.
// The current device's weight-gradient side stream (its own split-K slab workspace).
MI_API int mi_register_wgrad_stream(hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_splitk_mu);
  g_wgrad_stream[dev & 15] = st;
  return 0;
}

// The current device's auxiliary (projection-shortcut) stream: its own split-K slab workspace.
MI_API int mi_register_aux_stream(hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_splitk_mu);
  g_aux_stream[dev & 15] = st;
  return 0;
}

// A stream whose kernels may only use `ncu` of the device's CUs (hipExtStreamCreateWithCUMask):
// spread = 1 keeps every (total / ncu)-th CU id, 0 keeps the first ncu ids.  For the A/B of a
// weight-gradient stream confined to part of the chip (the compute stream keeps every CU).
MI_API int mi_create_cu_masked_stream(int ncu, int spread, hipStream_t* out) {
  int dev = 0, total = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || total <= 0)
    return (int)hipErrorInvalidValue;
  ncu = std::max(1, std::min(ncu, total));
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (int k = 0; k < ncu; ++k) {
    const int cu = spread ? (int)((int64_t)k * total / ncu) : k;
    mask[cu / 32] |= 1u << (cu % 32);
  }
  return (int)hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data());
}

MI_API int mi_set_tn_slabs(int on) {
  g_tn_slabs = on ? 1 : 0;
  return 0;
}

MI_API int mi_set_glds(int on) {
  g_nt_glds = on ? 1 : 0;
  return 0;
}

// NT split-K reduction: 1 = fused last-arriver launch (default), 0 = partials + reduce launch (tests).
MI_API int mi_set_tn_split_fused(int on) {
  g_tn_split_fused = on ? 1 : 0;
  return 0;
}
MI_API int mi_set_nt_split_fused(int on) {
  g_nt_split_fused = on ? 1 : 0;
  return 0;
}

// NT split-K threshold: grids below this many blocks split their k-steps (0 disables; tests).
MI_API int mi_set_nt_split_blocks(int blocks) {
  g_nt_split_blocks = std::max(0, blocks);
  return 0;
}

// NT (fwd/dgrad/GEMM) kernels: 1 = single LDS stage at 3 blocks/CU, 2 = double-buffered at 2 blocks/CU.
MI_API int mi_set_nt_stages(int stages) {
  g_nt_stages = stages == 2 ? 2 : 1;
  return 0;
}

// Convolutions with >= 256 output channels and enough 256x256 tiles run on the deep-pipelined
// kernel (gemm256.hip): forward and stride-1 data gradient (MI355X_DP_GEMM256=0 disables;
// MI355X_DP_CONV256_MIN_TILES sets the minimum tile count, default 96).
extern "C" int mi_gemm256_conv2(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                                const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs,
                                int P, int Q, int R, int S, int stride, int pad, int N, int aux_even, hipStream_t st);
extern "C" int mi_gemm256_conv(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                               const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs,
                               int P, int Q, int R, int S, int stride, int pad, int N, hipStream_t st);
static int g_gemm256_env = -1, g_conv256_min_tiles = -1, g_conv256_min_k = 64;
extern "C" int mi_g256_stat_rows(int M, int N, int K);  // gemm256.hip: 2 per 224- or 256-row tile
extern "C" int mi_panel_stat_rows(int M, int N, int K);
static int g_panel_first = -1;
static bool use_gemm256_conv(int M, int N, int Cs, int Kt) {
  if (g_gemm256_env < 0) {
    const char* e = std::getenv("MI355X_DP_GEMM256");
    g_gemm256_env = (e && e[0] == '0') ? 0 : 1;
    const char* t = std::getenv("MI355X_DP_CONV256_MIN_TILES");
    g_conv256_min_tiles = t ? std::atoi(t) : 96;
    // GEMM depth (R*S*Cs) below which a conv stays on the 128-tile kernel: a 1x1 conv over few
    // channels is one or two k-tiles -- nothing for the 256x256 pipeline to overlap, and its 128 KB
    // of LDS holds the CU to one block through a load-latency-bound prologue / epilogue
    const char* c = std::getenv("MI355X_DP_CONV256_MIN_K");
    g_conv256_min_k = c ? std::atoi(c) : 512;
  }
  if (!(g_gemm256_env && Cs % 64 == 0 && Kt >= g_conv256_min_k && N % 8 == 0 && N >= 256 &&
        (int64_t)cdiv(M, 256) * cdiv(N, 256) >= g_conv256_min_tiles))
    return false;
  // MI355X_DP_PANEL_FIRST=1: a 1x1 conv the panel kernel takes (K up to 1024 with 32-column panels)
  // leaves the 256-wide kernel (forward and stride-1 data gradient alike: the panel plan does not
  // depend on the direction)
  if (g_panel_first < 0) {
    const char* e = std::getenv("MI355X_DP_PANEL_FIRST");
    g_panel_first = (e && e[0] == '1') ? 1 : 0;
  }
  if (g_panel_first && Kt == Cs && mi_panel_stat_rows(M, N, Kt) > 0) return false;
  return true;
}

MI_API void mi_set_panel_first(int on) {
  use_gemm256_conv(0, 0, 0, 0);  // env init
  g_panel_first = on ? 1 : 0;
}

MI_API void mi_set_conv256_min_tiles(int t) {
  use_gemm256_conv(0, 0, 0, 0);  // env init
  g_conv256_min_tiles = t;
}

// minimum GEMM depth R*S*Cs for the 256x256 conv path (tests force small shapes onto it with 0)
MI_API void mi_set_conv256_min_k(int k) {
  use_gemm256_conv(0, 0, 0, 0);  // env init
  g_conv256_min_k = k;
}

// conv_panel.hip: persistent resident-weight kernel for the short-K 1x1 convolutions (forward)
extern "C" int mi_panel_stat_rows(int M, int N, int K);
extern "C" int mi_panel_stat_rows2(int M, int N, int K, int dgrad);
extern "C" int mi_panel_dgrad(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                              int epi, const void* aux, const void* aux2, const float* mean, int bn_relu, float* stats,
                              int aux_even, const void* mbits, const void* acc_src, hipStream_t st);
extern "C" int mi_panel_conv(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int C, int K,
                             int R, int stride, int pad, int P, int Q, hipStream_t st);
// a 1x1 or 3x3 (pad 1) stride-1 data gradient runs on the panel kernel (the statistics slab rows it
// writes), else 0
extern "C" int mi_panel_3x3();
static int panel_rows_dgrad(int M, int C, int K, int RS, int stride) {
  if ((RS != 1 && !(RS == 9 && mi_panel_3x3())) || stride != 1 || K % 64 != 0) return 0;
  return mi_panel_stat_rows2(M, C, RS * K, 1);
}
extern "C" int mi_panel_conv1x1(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int C,
                                int K, int stride, int P, int Q, hipStream_t st);
static int panel_rows_fwd(int M, int N, int C, int R, int S, int pad, int H, int W, int P, int Q, int stride) {
  if (C % 64 != 0) return 0;
  if (R == 3 && S == 3 && stride == 1 && pad == 1 && P == H && Q == W)
    return mi_panel_3x3() ? mi_panel_stat_rows(M, N, 9 * C) : 0;
  if (R != 1 || S != 1 || pad != 0 || P != (H - 1) / stride + 1 || Q != (W - 1) / stride + 1) return 0;
  return mi_panel_stat_rows(M, N, C);
}

// stem_conv.hip: persistent LDS-ring kernel for the 7x7/2 stem on 8-channel input
extern "C" int mi_stem_conv_ok(int C, int K, int R, int S, int stride, int pad, int Q);
extern "C" int mi_stem_conv_stat_rows(int Nb, int P);
extern "C" int mi_stem_conv_fwd(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int P,
                                int Q, int pad, hipStream_t st);
extern "C" int mi_stem_wgrad(const void* x, const void* dy, float* dw, int Nb, int H, int W, int P, int Q, int pad,
                             hipStream_t st);
static int g_stem = -1;
static bool use_stem_kernel(int C, int K, int R, int S, int stride, int pad, int Q) {
  if (g_stem < 0) {
    const char* e = std::getenv("MI355X_DP_STEM_KERNEL");
    g_stem = (e && e[0] == '0') ? 0 : 1;
  }
  return g_stem && mi_stem_conv_ok(C, K, R, S, stride, pad, Q);
}

// Statistics-slab rows written by mi_conv2d_fwd with stats (full geometry: the halo tiling of
// 3x3 convs depends on the spatial shape).
MI_API int mi_conv_stat_rows_g(int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad, int P, int Q) {
  const int M = Nb * P * Q;
  if (use_stem_kernel(C, K, R, S, stride, pad, Q)) return mi_stem_conv_stat_rows(Nb, P);
  if (C % 64 == 0 && use_gemm256_conv(M, K, C, R * S * C)) return mi_g256_stat_rows(M, K, R * S * C);
  if (const int pr = panel_rows_fwd(M, K, C, R, S, pad, H, W, P, Q, stride); pr > 0) return pr;
  const int rp = C % 64 == 0 ? halo_rp(M, K, R, S, stride, pad, C, H, W, P, Q) : 0;
  if (rp > 0) return Nb * cdiv(P, rp);
  return cdiv(M, nt_choice(M, K) == 2 ? 64 : 128);
}

// Statistics-slab rows written by a conv forward (M output pixels, N channels, Cs input channels),
// for shapes outside the halo tiling (1x1 / strided convs, GEMMs).
MI_API int mi_conv_stat_rows(int M, int N, int Cs, int RS) {
  if (use_gemm256_conv(M, N, Cs, RS * Cs)) return mi_g256_stat_rows(M, N, RS * Cs);
  if (RS == 1 && Cs % 64 == 0)  // a 1x1 (pad 0) conv forward on the panel kernel
    if (const int pr = mi_panel_stat_rows(M, N, Cs); pr > 0) return pr;
  const int bm = nt_choice(M, N) == 2 ? 64 : 128;
  return cdiv(M, bm);
}

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
  if ((C % 64 != 0 && C != 8) || K % 8 != 0) return (int)hipErrorInvalidValue;
  if (!out_f32 && !bias && use_stem_kernel(C, K, R, S, stride, pad, Q))
    return mi_stem_conv_fwd(x, w, y, stats, Nb, H, W, P, Q, pad, st);
  if (!out_f32 && !bias && use_gemm256_conv(Nb * P * Q, K, C, R * S * C))
    return mi_gemm256_conv(1, x, w, y, stats, 0, nullptr, nullptr, nullptr, 0, Nb, H, W, C, P, Q, R, S, stride, pad,
                           K, st);
  if (!out_f32 && !bias && panel_rows_fwd(Nb * P * Q, K, C, R, S, pad, H, W, P, Q, stride) > 0)
    return mi_panel_conv(x, w, y, stats, Nb, H, W, C, K, R, stride, pad, P, Q, st);
  NTArgs a{};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = y; a.bias = bias; a.stats = stats;
  a.M = Nb * P * Q; a.N = K; a.K = R * S * C;
  a.lda = 0; a.ldb = a.K; a.ldc = K; a.mode = (C == 8) ? 4 : 1; a.out_f32 = out_f32; a.accumulate = 0;
  a.a_bytes = rsrc_bytes((int64_t)Nb * H * W * C);
  a.b_bytes = rsrc_bytes((int64_t)K * a.K);
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_nt(a, st);
}

// Conv backward-data: dy NHWC [Nb,P,Q,K], wt [C][R][S][K] (see mi_conv_wtrans), dx NHWC [Nb,H,W,C].
MI_API int mi_conv2d_dgrad(const void* dy, const void* wt, void* dx,
                           int Nb, int H, int W, int C, int K, int R, int S,
                           int stride, int pad, int P, int Q, hipStream_t st) {
  if (K % 64 != 0 || C % 8 != 0 || stride > 2) return (int)hipErrorInvalidValue;
  if (stride == 1 && use_gemm256_conv(Nb * H * W, C, K, R * S * K))
    return mi_gemm256_conv(2, dy, wt, dx, nullptr, 0, nullptr, nullptr, nullptr, 0, Nb, P, Q, K, H, W, R, S, 1, pad, C,
                           st);
  if (R == S && pad == (R == 3 ? 1 : 0) && panel_rows_dgrad(Nb * H * W, C, K, R * S, stride) > 0)
    return mi_panel_dgrad(dy, wt, dx, Nb, H, W, C, K, R, 0, nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr, st);
  NTArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)wt; a.C = dx; a.bias = nullptr;
  a.M = Nb * H * W; a.N = C; a.K = R * S * K;
  a.lda = 0; a.ldb = a.K; a.ldc = C; a.mode = 2; a.out_f32 = 0; a.accumulate = 0;
  a.a_bytes = rsrc_bytes((int64_t)Nb * P * Q * K);
  a.b_bytes = rsrc_bytes((int64_t)C * a.K);
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
      a.cls_map[c] = c;
    }
    a.ncls = 4;
  }
  return (int)dispatch_nt(a, st);
}

// Statistics-slab rows written by mi_conv2d_dgrad_ex with stats (all parity classes).
MI_API int mi_dgrad_stat_rows(int Nb, int H, int W, int C, int P, int Q, int stride, int K, int RS) {
  const int M = Nb * H * W;
  if (stride == 1 && use_gemm256_conv(M, C, K, RS * K)) return mi_g256_stat_rows(M, C, RS * K);
  if (const int pr = panel_rows_dgrad(M, C, K, RS, stride); pr > 0) return pr;
  const int bm = nt_choice(M, C) == 2 ? 64 : 128;
  if (stride == 1 && RS == 9) {
    const int rp = halo_rp(M, C, 3, 3, 1, 1, K, P, Q, H, W);
    if (rp > 0) return Nb * cdiv(H, rp);
  }
  if (stride == 1) return cdiv(M, bm);
  int mrows = 0;
  for (int c = 0; c < 4; ++c) mrows = std::max(mrows, Nb * ((H - c / 2 + 1) / 2) * ((W - c % 2 + 1) / 2));
  return 4 * cdiv(mrows, bm);
}

// Conv dgrad with a fused epilogue: epi 3 accumulates into aux (dx = dgrad + aux; aux may alias
// dx -- the residual-gradient sum of a block input), epi 4 emits dz of the BatchNorm that produced
// this conv's input (aux = BN output y for the relu mask, aux2 = BN input, mean = its batch
// mean) plus its backward statistics into `stats` ([mi_dgrad_stat_rows][2][C]).
MI_API int mi_conv2d_dgrad_ex2(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, hipStream_t st);

MI_API int mi_conv2d_dgrad_ex(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                              int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                              const float* mean, int bn_relu, float* stats, hipStream_t st) {
  return mi_conv2d_dgrad_ex2(dy, wt, dx, Nb, H, W, C, K, R, S, stride, pad, P, Q, epi, aux, aux2, mean, bn_relu, stats,
                             0, st);
}

// mi_conv2d_dgrad_ex with flags: bit 0 (stride 2, epi 0) leaves the parity classes no tap reaches
// unwritten instead of zero-filling them (a 1x1 / stride-2 data gradient then writes only the even
// pixels); bit 1 (epi 3 / 5) reads the accumulated-into gradient only at even (h, w) -- the
// consumer of such a sparse write.  Together they skip 3/4 of a downsample dgrad's bytes.
MI_API int mi_conv2d_dgrad_ex3(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, const float* mask_scale,
                               const float* mask_shift, hipStream_t st);

MI_API int mi_conv2d_dgrad_ex2(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, hipStream_t st) {
  return mi_conv2d_dgrad_ex3(dy, wt, dx, Nb, H, W, C, K, R, S, stride, pad, P, Q, epi, aux, aux2, mean, bn_relu, stats,
                             flags, nullptr, nullptr, st);
}

MI_API int mi_conv2d_dgrad_ex4(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, const float* mask_scale,
                               const float* mask_shift, const void* mbits, hipStream_t st);

MI_API int mi_conv2d_dgrad_ex3(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, const float* mask_scale,
                               const float* mask_shift, hipStream_t st) {
  return mi_conv2d_dgrad_ex4(dy, wt, dx, Nb, H, W, C, K, R, S, stride, pad, P, Q, epi, aux, aux2, mean, bn_relu, stats,
                             flags, mask_scale, mask_shift, nullptr, st);
}

extern "C" int mi_gemm256_conv3(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                                const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs,
                                int P, int Q, int R, int S, int stride, int pad, int N, int aux_even,
                                const void* mbits, hipStream_t st);

// mi_conv2d_dgrad_ex2 with, for epi 4, the ReLU mask of the producing BN taken from its input c (aux2)
// as fma(c, mask_scale, mask_shift) > 0 -- aux (the BN output) unused: normalize-on-load schedules
// never write it.  Only where mi_conv_nol_ok holds (the 128-tile kernels).
// mbits (epi 4 / 5 with bn_relu): the ReLU mask as bytes of 8 channel bits ([Nb*H*W][C/8], from
// mi_bn_apply_bits) instead of reading the BN output aux (which may then be null).
extern "C" int mi_gemm256_nt_scat2(const void* A, const void* B, void* C, int M, int N, int K, int Q, int W,
                                   hipStream_t st);
// MI355X_DP_DS256=0: the stride-2 1x1 shortcut data gradients stay on the 128-tile class kernel
static int g_ds256 = -1;
static bool use_ds256() {
  if (g_ds256 < 0) {
    const char* e = std::getenv("MI355X_DP_DS256");
    g_ds256 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_ds256 != 0;
}
MI_API void mi_set_ds256(int on) { g_ds256 = on ? 1 : 0; }

MI_API int mi_conv2d_dgrad_ex4(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                               int S, int stride, int pad, int P, int Q, int epi, const void* aux, const void* aux2,
                               const float* mean, int bn_relu, float* stats, int flags, const float* mask_scale,
                               const float* mask_shift, const void* mbits, hipStream_t st) {
  const bool mask_c = mask_scale != nullptr;
  if (mask_c && (epi != 4 || !mask_shift || !aux2 || !bn_relu)) return (int)hipErrorInvalidValue;
  if (mbits && (epi < 4 || !bn_relu || mask_c)) return (int)hipErrorInvalidValue;
  if (K % 64 != 0 || C % 8 != 0 || stride > 2 || !(epi == 0 || epi == 3 || epi == 4 || epi == 5) ||
      (epi && !aux && bn_relu && !mask_c && !mbits) || (epi == 3 && !aux) || (epi >= 4 && stats && (!aux2 || !mean)) ||
      ((flags & 1) && (stride != 2 || epi != 0)) || ((flags & 2) && epi != 3 && epi != 5))
    return (int)hipErrorInvalidValue;
  const int aux_even = (flags >> 1) & 1;
  if (mask_c && stride == 1 && use_gemm256_conv(Nb * H * W, C, K, R * S * K)) return (int)hipErrorNotSupported;
  if (stride == 1 && use_gemm256_conv(Nb * H * W, C, K, R * S * K))
    return mi_gemm256_conv3(2, dy, wt, dx, epi >= 4 ? stats : nullptr, epi, const_cast<void*>(aux), aux2, mean,
                            bn_relu, Nb, P, Q, K, H, W, R, S, 1, pad, C, aux_even, mbits, st);
  // the stride-2 1x1 data gradient of a projection shortcut (only the even pixels, flags bit 0) as a
  // plain GEMM over dy's pixels on the 256-wide kernel, rows scattered to the even pixels of dx
  if (stride == 2 && R == 1 && S == 1 && pad == 0 && epi == 0 && (flags & 1) && !mask_c && !mbits && H == 2 * P &&
      W == 2 * Q && use_ds256() && use_gemm256_conv(Nb * P * Q, C, K, K))
    return mi_gemm256_nt_scat2(dy, wt, dx, Nb * P * Q, C, K, Q, W, st);
  if (R == S && pad == (R == 3 ? 1 : 0) && panel_rows_dgrad(Nb * H * W, C, K, R * S, stride) > 0) {
    if (mask_c) return (int)hipErrorNotSupported;  // mi_conv_nol_ok keeps these shapes materialised
    return mi_panel_dgrad(dy, wt, dx, Nb, H, W, C, K, R, epi, aux, aux2, mean, bn_relu, stats, aux_even, mbits,
                          nullptr, st);
  }
  NTArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)wt; a.C = dx; a.bias = nullptr;
  a.M = Nb * H * W; a.N = C; a.K = R * S * K;
  a.lda = 0; a.ldb = a.K; a.ldc = C; a.mode = 2; a.out_f32 = 0; a.accumulate = 0;
  a.epi = epi; a.aux = (bf16_t*)aux; a.aux2 = (const bf16_t*)aux2; a.mean = mean; a.bn_relu = bn_relu;
  a.stats = (epi >= 4) ? stats : nullptr;
  a.aux_even = aux_even;
  a.mask_scale = mask_scale; a.mask_shift = mask_shift;
  a.mbits = (const uint8_t*)mbits;
  a.a_bytes = rsrc_bytes((int64_t)Nb * P * Q * K);
  a.b_bytes = rsrc_bytes((int64_t)C * a.K);
  a.g = make_geom(P, Q, K, H, W, S, stride, pad, R);
  if (stride == 2) {
    a.mode = 3;
    a.ncls = 0;
    for (int c = 0; c < 4; ++c) {
      const int ph = c / 2, pw = c % 2;
      a.g.Pc[c] = (H - ph + 1) / 2;
      a.g.Qc[c] = (W - pw + 1) / 2;
      a.g.fPQc[c] = make_fastdiv((uint32_t)std::max(1, a.g.Pc[c] * a.g.Qc[c]));
      a.g.fQc[c] = make_fastdiv((uint32_t)std::max(1, a.g.Qc[c]));
      // flags bit 0: drop the classes no tap reaches (first tap row/column of the class >= R/S)
      if ((flags & 1) && ((ph + pad) % 2 >= R || (pw + pad) % 2 >= S)) continue;
      a.cls_map[a.ncls++] = c;
    }
    if (a.ncls == 0) return (int)hipSuccess;
  }
  return (int)dispatch_nt(a, st);
}

// MI355X_DP_WGRAD256=T (T >= 1): a 1x1 stride-1 weight gradient with >= T output tiles of 256 x 256
// (K x C) runs as a plain TN GEMM on the 256x256 pipeline (split-K slabs + one reduce) instead of the
// 128-tile implicit-GEMM kernel; 0 (default): never
extern "C" int mi_gemm256_tn(const void* A, const void* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                             hipStream_t st);
static int g_wgrad256 = -1;
static bool use_wgrad256(int K, int C, int R, int S, int stride, int pad, int H, int W, int P, int Q) {
  if (g_wgrad256 < 0) {
    const char* e = std::getenv("MI355X_DP_WGRAD256");
    g_wgrad256 = e ? std::max(0, std::atoi(e)) : 0;
  }
  return g_wgrad256 > 0 && R == 1 && S == 1 && stride == 1 && pad == 0 && P == H && Q == W && K % 8 == 0 &&
         C % 8 == 0 && cdiv(K, 256) * cdiv(C, 256) >= g_wgrad256;
}
MI_API void mi_set_wgrad256(int min_tiles) {
  use_wgrad256(0, 0, 0, 0, 0, 0, 0, 0, 0, 0);  // env init
  g_wgrad256 = std::max(0, min_tiles);
}

// Conv backward-weight: dw[K][R][S][C] (fp32) += sum over pixels dy^T * im2col(x).
MI_API int mi_conv2d_wgrad(const void* x, const void* dy, float* dw,
                           int Nb, int H, int W, int C, int K, int R, int S,
                           int stride, int pad, int P, int Q, hipStream_t st) {
  if (C % 8 != 0 || K % 8 != 0) return (int)hipErrorInvalidValue;
  if (use_stem_kernel(C, K, R, S, stride, pad, Q)) return mi_stem_wgrad(x, dy, dw, Nb, H, W, P, Q, pad, st);
  if (use_wgrad256(K, C, R, S, stride, pad, H, W, P, Q) &&
      mi_gemm256_tn(dy, x, dw, K, C, Nb * H * W, K, C, C, st) == (int)hipSuccess)
    return (int)hipSuccess;
  TNArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)x; a.C = dw;
  a.M = K; a.N = R * S * C; a.K = Nb * P * Q;
  a.lda = K; a.ldb = 0; a.ldc = a.N; a.mode = 1;
  a.a_bytes = rsrc_bytes((int64_t)Nb * P * Q * K);
  a.b_bytes = rsrc_bytes((int64_t)Nb * H * W * C);
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_tn(a, st);
}

// ---- folded BatchNorm backward, data-gradient routing: the panel kernel when the doubled depth fits
// its LDS (conv_panel.hip), else the 256-wide kernel where the unfolded data gradient runs there
// (gemm256.hip mi_gemm256_dgrad_fbb); 0: not eligible (the caller materialises dX)
extern "C" int mi_panel_fbb_rows(int M, int C, int K);
extern "C" int mi_gemm256_dgrad_fbb(const void* dz, const void* c, const float* coef, const void* wt, void* wq,
                                    float* bias, void* dx, float* stats, int epi, void* aux, const void* aux2,
                                    const float* mean, int bn_relu, int Nb, int H, int W, int C, int K, int aux_even,
                                    const void* mbits, hipStream_t st);
MI_API int mi_conv_fbb_route(int M, int C, int K) {
  if (K % 64 != 0 || C % 64 != 0) return 0;
  if (mi_panel_fbb_rows(M, C, K) > 0) return 1;
  if (use_gemm256_conv(M, C, K, K)) return 2;
  return 0;
}

// statistics slab rows of the folded data gradient (route 1 or 2), 0 if not eligible
MI_API int mi_conv_fbb_rows(int M, int C, int K) {
  const int r = mi_conv_fbb_route(M, C, K);
  return r == 1 ? mi_panel_fbb_rows(M, C, K) : (r == 2 ? mi_g256_stat_rows(M, C, 2 * K) : 0);
}

// ---- folded BatchNorm backward, weight-gradient side (conv_panel.hip mi_panel_dgrad_fbb): the weight
// gradient of a 1x1 / stride-1 conv against its output's BN input gradient dX = k0 dz + k1 c + k2 (per
// output channel k) without dX.  With c = x W^T, c^T x = W (x^T x), so
//   dW[k][n] += k0[k] (dz^T x)[k][n] + k1[k] (W G)[k][n] + k2[k] s[n],   G = x^T x, s = colsum(x):
// ONE TN GEMM of [dz | x] (K + C rows: the conv input x is read a second time instead of the K-wide c)
// against x, the column sums of x per split (bsum), and a small combine in split order
// (deterministic).  ws: fp32 [K + C + FBB_MAX_SPLITS][C], zero on entry -- the combine re-zeroes it.
constexpr int FBB_MAX_SPLITS = 1024;

__global__ __launch_bounds__(256) void fbb_wgrad_combine_kernel(float* __restrict__ T, const float* __restrict__ bsum,
                                                                int nsplit, const float* __restrict__ coef,
                                                                const bf16_t* __restrict__ w, float* __restrict__ dw,
                                                                int K, int C) {
  // one output channel k per block; T rows [0, K): dz^T x, [K, K + C): G.  Thread t: column
  // n = t % C (+ 256 strides for C > 256), reduction part t / C of PT = 256 / C parts (split sums of s
  // and the j terms of (W G)[k][n]), combined through LDS in a fixed order
  __shared__ float red[2][256];
  const int k = blockIdx.x;
  const int PT = C < 256 ? 256 / C : 1;
  const int part = threadIdx.x / (C < 256 ? C : 256), n0 = threadIdx.x % (C < 256 ? C : 256);
  const float k0 = coef[k], k1 = coef[K + k], k2 = coef[2 * K + k];
  const float* G = T + (size_t)K * C;
  for (int nb = 0; nb < C; nb += 256) {
    const int n = nb + n0;
    float sn = 0.f, wg = 0.f;
    if (part < PT && n < C) {
      for (int z = part; z < nsplit; z += PT) sn += bsum[(size_t)z * C + n];
      for (int j = part; j < C; j += PT) wg = fmaf(bf2f(w[(size_t)k * C + j]), G[(size_t)j * C + n], wg);
    }
    red[0][threadIdx.x] = sn;
    red[1][threadIdx.x] = wg;
    __syncthreads();
    if (part == 0 && n < C) {
      for (int q = 1; q < PT; ++q) {
        sn += red[0][q * (C < 256 ? C : 256) + n0];
        wg += red[1][q * (C < 256 ? C : 256) + n0];
      }
      dw[(size_t)k * C + n] += k0 * T[(size_t)k * C + n] + k1 * wg + k2 * sn;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void fbb_ws_zero_kernel(float* __restrict__ T, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) T[i] = 0.f;
}

MI_API int mi_conv2d_wgrad_fbb_ws_floats(int K, int C) { return (K + C + FBB_MAX_SPLITS) * C; }

// x NHWC [Nb,H,W,C] (the 1x1 conv's input), dz NHWC [Nb,H,W,K], w bf16 [K][C] (its forward weights),
// dw fp32 [K][C] (+=), ws: mi_conv2d_wgrad_fbb_ws_floats(K, C) floats, zero.  hipErrorNotSupported:
// not eligible (the caller keeps the materialised path)
MI_API int mi_conv2d_wgrad_fbb(const void* x, const void* dz, const void* w, const float* coef, float* dw, float* ws,
                               int Nb, int H, int W, int C, int K, hipStream_t st) {
  if (C % 64 != 0 || K % 64 != 0 || !coef || !ws || !w) return (int)hipErrorInvalidValue;
  const int M2 = K + C, M = Nb * H * W;
  TNArgs a{};
  a.A = (const bf16_t*)dz; a.A2 = (const bf16_t*)x; a.B = (const bf16_t*)x; a.C = ws;
  a.M = M2; a.N = C; a.K = M;
  a.lda = K; a.lda2 = C; a.ldb = 0; a.ldc = C; a.mode = 1;
  a.msplit = K;
  a.a_bytes = rsrc_bytes((int64_t)M * K);
  a.a2_bytes = a.b_bytes = rsrc_bytes((int64_t)M * C);
  a.bsum = ws + (size_t)M2 * C;
  a.g = make_geom(H, W, C, H, W, 1, 1, 0, 1);
  // the dz / x parts must not share a row tile: BM divides K
  const int target = tn_target_blocks(st);
  const bool m128 = K % 128 == 0, n64 = C <= 64;
  const int BMc = m128 ? 128 : 64, BNc = n64 ? 64 : 128;
  const int tiles = cdiv(M2, BMc) * cdiv(C, BNc), ksteps = cdiv(M, BK);
  const int splits0 = std::max(1, std::min(ksteps, target / std::max(tiles, 1)));
  const int splits = cdiv(M, cdiv(ksteps, splits0) * BK);
  if (splits > FBB_MAX_SPLITS) return (int)hipErrorNotSupported;
  hipError_t e;
  if (m128) e = n64 ? launch_tn<128, 64>(a, st, target) : launch_tn<128, 128>(a, st, target);
  else e = n64 ? launch_tn<64, 64>(a, st, target) : launch_tn<64, 128>(a, st, target);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fbb_wgrad_combine_kernel, dim3(K), dim3(256), 0, st, ws, (const float*)a.bsum, splits, coef,
                     (const bf16_t*)w, dw, K, C);
  const int64_t nz = (int64_t)M2 * C;
  hipLaunchKernelGGL(fbb_ws_zero_kernel, dim3((unsigned)std::min<int64_t>(cdiv(nz, 256), 1024)), dim3(256), 0, st, ws,
                     nz);
  return (int)hipGetLastError();
}

// ---- normalize-on-load (the consumer conv applies the producing BatchNorm + ReLU to its raw input c)
// 1 if a conv of this geometry can consume a raw BN input with normalize-on-load in the forward
// (mi_conv2d_fwd_nol), take its data gradient's ReLU mask from c (mi_conv2d_dgrad_nol) and its
// weight gradient from c (mi_conv2d_wgrad_nol): the 128-tile NT gather / halo kernels and the TN
// kernel; shapes routed to the stem or 256x256 kernels keep the materialised BN output.
MI_API int mi_conv_nol_ok(int Nb, int H, int W, int C, int K, int R, int S, int stride, int pad, int P, int Q) {
  if (C % 64 != 0 || C > NOL_MAX_C || K % 64 != 0 || stride > 2 || !glds_on()) return 0;
  if (use_stem_kernel(C, K, R, S, stride, pad, Q)) return 0;
  if (use_gemm256_conv(Nb * P * Q, K, C, R * S * C)) return 0;                    // forward
  if (panel_rows_fwd(Nb * P * Q, K, C, R, S, pad, H, W, P, Q, stride) > 0) return 0;  // forward (panel)
  if (panel_rows_dgrad(Nb * H * W, C, K, R * S, stride) > 0) return 0;               // data gradient (panel)
  if (stride == 1 && use_gemm256_conv(Nb * H * W, C, K, R * S * K)) return 0;    // data gradient
  // small grids keep the materialised path: there the 128-tile kernels split K (nt_split_blocks),
  // which the normalize-on-load variants do not -- and the bytes saved are negligible
  const int tf = cdiv(Nb * P * Q, nt_choice(Nb * P * Q, K) == 2 ? 64 : 128) * cdiv(K, nt_choice(Nb * P * Q, K) == 0 ? 128 : 64);
  const int td = cdiv(Nb * H * W, nt_choice(Nb * H * W, C) == 2 ? 64 : 128) * cdiv(C, nt_choice(Nb * H * W, C) == 0 ? 128 : 64);
  if (tf < nt_split_blocks() || td < nt_split_blocks()) return 0;
  return 1;
}

MI_API int mi_conv2d_fwd_nol(const void* x, const void* w, void* y, float* stats, const float* nol_scale,
                             const float* nol_shift, int Nb, int H, int W, int C, int K, int R, int S, int stride,
                             int pad, int P, int Q, hipStream_t st) {
  if (!mi_conv_nol_ok(Nb, H, W, C, K, R, S, stride, pad, P, Q) || !nol_scale || !nol_shift)
    return (int)hipErrorNotSupported;
  NTArgs a{};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = y; a.bias = nullptr; a.stats = stats;
  a.M = Nb * P * Q; a.N = K; a.K = R * S * C;
  a.lda = 0; a.ldb = a.K; a.ldc = K; a.mode = 1; a.out_f32 = 0; a.accumulate = 0;
  a.nol_scale = nol_scale; a.nol_shift = nol_shift;
  a.a_bytes = rsrc_bytes((int64_t)Nb * H * W * C);
  a.b_bytes = rsrc_bytes((int64_t)K * a.K);
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_nt(a, st);
}

MI_API int mi_conv2d_wgrad_nol(const void* x, const void* dy, float* dw, const float* nol_scale,
                               const float* nol_shift, int Nb, int H, int W, int C, int K, int R, int S, int stride,
                               int pad, int P, int Q, hipStream_t st) {
  if (C % 8 != 0 || K % 8 != 0 || C > NOL_MAX_C || !nol_scale || !nol_shift ||
      use_stem_kernel(C, K, R, S, stride, pad, Q))
    return (int)hipErrorInvalidValue;
  TNArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)x; a.C = dw;
  a.M = K; a.N = R * S * C; a.K = Nb * P * Q;
  a.lda = K; a.ldb = 0; a.ldc = a.N; a.mode = 1;
  a.nol_scale = nol_scale; a.nol_shift = nol_shift;
  a.a_bytes = rsrc_bytes((int64_t)Nb * P * Q * K);
  a.b_bytes = rsrc_bytes((int64_t)Nb * H * W * C);
  a.g = make_geom(H, W, C, P, Q, S, stride, pad, R);
  return (int)dispatch_tn(a, st);
}

MI_API int mi_conv_wtrans(const void* w, void* wt, int K, int RS, int C, hipStream_t st) {
  dim3 grid(cdiv(C, 64), cdiv(K, 64), RS);
  hipLaunchKernelGGL(wtrans_kernel, grid, dim3(256), 0, st, (const bf16_t*)w, (bf16_t*)wt, K, RS, C);
  return (int)hipGetLastError();
}

// desc: device int32 [ntens][6] (WtDesc); nblocks = sum over tensors of RS * cdiv(K,64) * cdiv(C,64)
MI_API int mi_conv_wtrans_multi(const void* w, void* wt, const void* desc, int ntens, int nblocks, hipStream_t st) {
  if (ntens <= 0 || nblocks <= 0) return 0;
  hipLaunchKernelGGL(wtrans_multi_kernel, dim3(nblocks), dim3(256), 0, st, (const bf16_t*)w, (bf16_t*)wt,
                     (const WtDesc*)desc, ntens);
  return (int)hipGetLastError();
}

// Large plain GEMMs go to the deep-pipelined 256x256 kernel (gemm256.hip) when they fill the
// chip with at least one wave of 256x256 tiles; MI355X_DP_GEMM256=0 disables it (A/B runs).
extern "C" int mi_gemm256_nt(const void* A, const void* B, void* C, const float* bias, void* aux, int epi, int M,
                             int N, int K, int lda, int ldb, int ldc, int out_f32, int accumulate, hipStream_t st);
static int g_gemm256 = -1;
static bool use_gemm256(int M, int N, int K) {
  if (g_gemm256 < 0) {
    const char* e = getenv("MI355X_DP_GEMM256");
    g_gemm256 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_gemm256 && K >= 128 && (int64_t)cdiv(M, 256) * cdiv(N, 256) >= 256;
}

MI_API void mi_set_gemm256(int on) { g_gemm256 = on ? 1 : 0; }

// TN: the 256x256 kernel wins only without heavy split-K (>= 128 output tiles); weight-gradient
// shapes with few output tiles (ViT: 9-36) stay on the 128x128 split-K kernel (L2 locality).
extern "C" int mi_gemm256_tn(const void* A, const void* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                             hipStream_t st);
static int g_tn256_min_tiles = -1;
static bool use_gemm256_tn(int M, int N, int K) {
  use_gemm256(0, 0, 0);  // env init
  if (g_tn256_min_tiles < 0) {
    const char* e = std::getenv("MI355X_DP_TN256_MIN_TILES");
    g_tn256_min_tiles = e ? std::max(1, std::atoi(e)) : 128;
  }
  return g_gemm256 && K >= 1024 && (int64_t)cdiv(M, 256) * cdiv(N, 256) >= g_tn256_min_tiles;
}

// Plain GEMM, "NT": C[M][N] = A[M][K] * B[N][K]^T (+bias[N]); A, B bf16; C bf16 or fp32.
MI_API int mi_gemm_nt(const void* A, const void* B, void* C, const float* bias, float* stats,
                      int M, int N, int K, int lda, int ldb, int ldc,
                      int out_f32, int accumulate, hipStream_t st) {
  if (K % 8 != 0 || N % 4 != 0 || (!out_f32 && N % 8 != 0)) return (int)hipErrorInvalidValue;
  if (!stats && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && use_gemm256(M, N, K))
    return mi_gemm256_nt(A, B, C, bias, nullptr, 0, M, N, K, lda, ldb, ldc, out_f32, accumulate, st);
  NTArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = bias; a.stats = out_f32 ? nullptr : stats;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.mode = 0; a.out_f32 = out_f32; a.accumulate = accumulate;
  a.a_bytes = rsrc_bytes((int64_t)M * lda);
  a.b_bytes = rsrc_bytes((int64_t)N * ldb);
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_nt(a, st);
}


// NT GEMM with a bf16 elementwise epilogue (NTArgs::epi): transformer MLP / residual fusion.
MI_API int mi_gemm_nt_epi(const void* A, const void* B, void* C, const float* bias, void* aux, int epi,
                          int M, int N, int K, int lda, int ldb, int ldc, hipStream_t st) {
  if (K % 8 != 0 || N % 8 != 0 || ldc % 8 != 0 || epi < 0 || epi > 3 || (epi && !aux))
    return (int)hipErrorInvalidValue;
  if (use_gemm256(M, N, K) && lda % 8 == 0 && ldb % 8 == 0)
    return mi_gemm256_nt(A, B, C, bias, aux, epi, M, N, K, lda, ldb, ldc, 0, 0, st);
  NTArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = bias; a.stats = nullptr;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.mode = 0; a.out_f32 = 0; a.accumulate = 0; a.aux = (bf16_t*)aux; a.epi = epi;
  a.a_bytes = rsrc_bytes((int64_t)M * lda);
  a.b_bytes = rsrc_bytes((int64_t)N * ldb);
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_nt(a, st);
}

// Plain GEMM, "TN": C[M][N] (fp32) += A[K][M]^T * B[K][N].
MI_API int mi_gemm_tn(const void* A, const void* B, float* C, int M, int N, int K,
                      int lda, int ldb, int ldc, hipStream_t st) {
  if (M % 8 != 0 || N % 8 != 0) return (int)hipErrorInvalidValue;
  if (lda % 8 == 0 && ldb % 8 == 0 && use_gemm256_tn(M, N, K)) return mi_gemm256_tn(A, B, C, M, N, K, lda, ldb, ldc, st);
  TNArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.mode = 0;
  a.a_bytes = rsrc_bytes((int64_t)K * lda);
  a.b_bytes = rsrc_bytes((int64_t)K * ldb);
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_tn(a, st);
}

// mi_gemm_tn that also adds the column sums of A (sum over K of A[k][m], i.e. a Linear layer's
// bias gradient from its output gradient) into colsum[M] fp32 -- one extra MFMA per A fragment in
// the first column tile instead of a separate pass over A.  Always the 128-tile split-K kernel.
MI_API int mi_gemm_tn_bias(const void* A, const void* B, float* C, float* colsum, int M, int N, int K, int lda,
                           int ldb, int ldc, hipStream_t st) {
  if (M % 8 != 0 || N % 8 != 0 || !colsum) return (int)hipErrorInvalidValue;
  TNArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.colsum = colsum;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.mode = 0;
  a.a_bytes = rsrc_bytes((int64_t)K * lda);
  a.b_bytes = rsrc_bytes((int64_t)K * ldb);
  a.g = make_geom(1, 1, 64, 1, 1, 1, 1, 0);
  return (int)dispatch_tn(a, st);
}
