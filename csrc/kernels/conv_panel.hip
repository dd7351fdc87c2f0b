// Persistent resident-weight "panel" kernel for the short-K 1x1 convolutions of a ResNet
// (SURVEY.md §2.5 K1 -- the conv forward of cifar10-distributed-smddp-gpu.py:165's model at the
// BASELINE.json ResNet-50 / -152 configs): C[m][n] = sum_k A[m][k] * W[n][k], A = NHWC activations
// (a 1x1 / stride-s gather), W = [N][K] weights, bf16 in, fp32 MFMA accumulation, bf16 out, with
// the per-channel (sum, sum of squares) BatchNorm statistics of the rounded output fused in.
//
// Why a separate kernel: the 128-tile nt_kernel runs load -> vmcnt(0) ->
// barrier -> MFMA -> barrier per k-step, and a K <= 256 conv has 1-4 k-steps per tile, so every
// tile pays a full memory latency plus an LDS-staged epilogue with nothing in flight; the layer-1
// convs ran at 3.4-4.5 TB/s and ~18 % MFMA busy.  Here:
//
//  * the block's weight panel W[n0, n0 + BN) x [0, K) is loaded into LDS ONCE and stays resident
//    (K <= 256: at most 64 KB); only the activations stream;
//  * 8 waves per block, 1 block per CU; every wave owns 32-row units of the output and streams its
//    OWN A rows through a private S-slot LDS ring (4 KB per slot, direct-to-LDS buffer_load ... lds,
//    XOR-swizzled on the source) -- no workgroup barrier anywhere in the main loop;
//  * the ring runs over the wave's whole sequence of (unit, k-step) pairs: the loads of the next
//    units' k-steps are in flight (S - 1 k-steps ahead) while the current unit computes and stores
//    its epilogue, and every wait is a COUNTED vmcnt (never 0 in the loop): gfx950 counts stores and
//    loads in one in-order counter, so the count adds the epilogue stores issued since the target
//    load (every epilogue issues a fixed number of stores: rows past M go to an out-of-range
//    buffer offset and are dropped, never skipped);
//  * the epilogue stages the unit's bf16 tile through the ring slot it just consumed (free until
//    the next issue) and stores full 16-byte row chunks; the staging stores are inline asm, because
//    an LDS store hipcc can see while LDS-DMA loads are in flight makes it drain vmcnt(0) first
//    (measured: register-direct permlane16 stores of 16 rows x 64 B per instruction instead were
//    up to 1.35x slower on the 512-wide expansions); every lane accumulates the statistics of its
//    fixed 8-channel chunk over ALL its units in registers, reduced across lanes and waves once
//    per block (one statistics row per block).
#include "common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int PN_SLOT_U4 = 32 * 8;          // 4 KB: 32 rows x 64 k bf16
constexpr int PN_LDS_U4 = 163840 / 16;      // the whole 160 KB of a CU
constexpr uint32_t PN_OOB = 0xFFFFFFF0u;

struct PanelArgs {
  const bf16_t* A;  // activations (gathered rows) [..][Cs]
  const bf16_t* B;  // weights [N][K]
  bf16_t* C;        // output [M][ldc]
  float* stats;     // optional [nb][2][N] partial (sum, sumsq) of the bf16 output, one row per block
  int M, N, K, ldc;
  int nk;           // K / 64
  int npanel;       // N / BN
  int nunits;       // cdiv(M, 32)
  int a_bytes, b_bytes, c_bytes;
  // row m -> element offset of its A row: plain (gather == 0): m * lda; 1x1 stride-s gather:
  // pixel (img, p, q) of the P x Q output grid reads input pixel (img, p * s, q * s) of H x W
  // gather 2: 3x3 / stride-1 / pad-1 taps (k-step kt = tap kt / cpt, channel chunk kt % cpt): row
  //   m = pixel (img, h, w) reads pixel (h + tsg (r - 1), w + tsg (s - 1)) of the same H x W grid, zero
  //   outside (tsg +1: forward, -1: data gradient, whose weights wt = [C][3][3][K] run the flipped taps)
  int gather, lda, H, W, stride;
  int tsg, cpt;
  FastDiv fPQ, fQ;
  // data-gradient epilogues (EPI 1; nt_kernel's epi 0 / 3 / 4 / 5 with the same rounding points):
  //   epi 3: C <- bf16(acc) + aux;  epi 4: dz = bf16(acc) * mask;  epi 5: dz = (bf16(acc) + C) * mask
  //   (C read before it is overwritten: a block input's residual gradient sum), mask = the ReLU of
  //   the BN that produced this conv's input: bit of mbits (one byte per 8 channels) or y = aux > 0;
  //   stats <- (sum dz, sum dz * (aux2 - mean)) with aux2 the BN input
  //   aux_even: the gradient in C exists only at even (h, w) of the P x Q grid (fPQ / fQ), 0 elsewhere
  int epi, bn_relu, aux_even;
  const bf16_t* aux;
  const bf16_t* aux2;
  const float* mean;
  const uint8_t* mbits;
  // folded BatchNorm backward (EPI 1, khalf > 0): the consumer GEMM of a BN's
  // input gradient dX = k0 dz + k1 c + k2 (per channel k) without materialising dX -- the A operand
  // is [dz | c] along K (k-steps [0, khalf) read dz from A, [khalf, 2 khalf) read c from A2, same row
  // geometry), the weight panel [diag(k0) W | diag(k1) W] is scaled in LDS from the bf16 W (row
  // stride ldb, khalf k-steps) with coef = (k0, k1, k2) [3][64 khalf], and every accumulator starts
  // at bias[n] = sum_k k2[k] W[n][k]
  const bf16_t* A2;
  int a2_bytes, khalf, ldb;
  const float* coef;
  const bf16_t* acc_src;  // epi 5: read the accumulated-into gradient from here instead of C (out of place)
};

__device__ __forceinline__ void pn_load8f(const float* __restrict__ p, float* o) {
  *(float4*)&o[0] = *(const float4*)p;
  *(float4*)&o[4] = *(const float4*)(p + 4);
}

#define PN_VMWAIT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int N>
__device__ __forceinline__ void pn_vmwait() {
  static_assert(N >= 0 && N <= 63, "vmcnt holds 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait for the k-step issued S - 1 issues ago: younger ops are (S - 1) k-steps of 4 loads plus cnt
// epilogue events of EV ops each (the stores of a unit, and in EPI 1 the next unit's operand loads)
template <int S, int EV>
__device__ __forceinline__ void pn_wait(int cnt) {
  constexpr int B = 4 * (S - 1);
  if (cnt <= 0) pn_vmwait<B>();
  else if (cnt == 1) pn_vmwait<B + EV>();
  else if (S == 2 || cnt == 2) pn_vmwait<B + 2 * EV < 64 ? B + 2 * EV : 63>();
  else pn_vmwait<B + 3 * EV < 64 ? B + 3 * EV : 63>();
}

// BN: block panel width (columns), WN: wave tile width (64 or 128), S: ring slots per wave,
// EPI: 0 forward (+ (sum, sumsq) statistics), 1 data gradient (PanelArgs::epi, WN 64)
template <int BN, int WN, int S, int EPI>
__global__ __launch_bounds__(512) void panel_kernel(PanelArgs a) {
  constexpr int WNW = BN / WN, WMW = 8 / WNW;  // waves along N / along M
  constexpr int NJ = WN / 16;
  constexpr int NP = NJ / 2;                   // fragment pairs: one 16-byte chunk each per row block
  constexpr int ST = 2 * NP;                   // epilogue stores per lane per unit (32 x WN bf16)
  // EPI 1: the next unit's epilogue operands are loaded right after a unit's stores, one unit ahead:
  // per chunk the accumulated-into gradient (or the residual), the BN input and the ReLU source
  constexpr int EL = EPI == 1 ? 3 * ST : 0;
  constexpr int RING_U4 = 8 * S * PN_SLOT_U4;
  static_assert(WNW * WMW == 8 && (WN == 32 || WN == 64 || WN == 128), "8 waves");
  static_assert(EPI == 0 || WN <= 64, "data-gradient operands held in registers: <= 64-column waves");
  // ONE LDS array (a second __shared__ object can make hipcc drain vmcnt before ds_reads):
  // [8 waves][S slots] A rings, then the weight panel [nk][BN][8 chunks]
  __shared__ __attribute__((aligned(16))) uint4 smem[PN_LDS_U4];
  uint4* bpanel = smem + RING_U4;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid % WNW, wm = wid / WNW;
  const int fr = lane & 15, fq = lane >> 4;
  const int idx = xcd_remap(blockIdx.x, gridDim.x);  // a row group's panels share an XCD's L2
  const int panel = idx % a.npanel, rg = idx / a.npanel;
  const int nb = gridDim.x / a.npanel;
  const int n0 = panel * BN;
  const int nk = a.nk;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.b_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)a.C, (short)0, a.c_bytes, 0x00020000);
  const int khalf = EPI == 1 ? a.khalf : 0;  // folded BN backward: k-steps per operand half
  const __amdgpu_buffer_rsrc_t rsA2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(khalf ? a.A2 : a.A), (short)0, khalf ? a.a2_bytes : 0, 0x00020000);
  // EPI 1 operand resources (same layout as C; mbits: one byte per 8 channels)
  __amdgpu_buffer_rsrc_t rsY = rsC, rsX = rsC, rsK = rsC;
  if constexpr (EPI == 1) {
    rsY = __builtin_amdgcn_make_buffer_rsrc((void*)(a.epi == 3 ? a.aux : (a.acc_src ? a.acc_src : a.C)), (short)0,
                                            (a.epi == 3 || a.epi == 5) ? a.c_bytes : 0, 0x00020000);
    rsX = __builtin_amdgcn_make_buffer_rsrc((void*)a.aux2, (short)0, (a.epi >= 4 && a.stats) ? a.c_bytes : 0,
                                            0x00020000);
    const bool relu = a.epi >= 4 && a.bn_relu;
    rsK = a.mbits ? __builtin_amdgcn_make_buffer_rsrc((void*)a.mbits, (short)0, relu ? a.c_bytes / 16 : 0, 0x00020000)
                  : __builtin_amdgcn_make_buffer_rsrc((void*)a.aux, (short)0, relu ? a.c_bytes : 0, 0x00020000);
  }

  // ---- the weight panel, once: piece p = 8 rows x 128 B of k-step kt (lane-linear image, chunk
  // c of row n holds logical chunk c ^ (n & 7))
  {
    constexpr int PPK = BN / 8;  // pieces per k-step
    const int np = (khalf ? khalf : nk) * PPK;  // folded BN backward: the second half is computed below
    const int pr = lane >> 3, pc = lane & 7;
    for (int p = wid; p < np; p += 8) {
      const int kt = p / PPK, r8 = p - kt * PPK;
      const int n = n0 + r8 * 8 + pr;
      const uint32_t vo = n < a.N ? (uint32_t)(n * a.ldb + kt * 64 + ((pc ^ pr) * 8)) * 2u : PN_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, LDS_PTR(void, bpanel + (kt * BN + r8 * 8) * 8), 16, vo, 0, 0, 0);
    }
    PN_VMWAIT(0);
    __syncthreads();
  }
  // folded BN backward: W -> [diag(k0) W | diag(k1) W] in place (chunk position c of panel row n holds
  // channels 8 (c ^ (n & 7)) of its k-step) and bias[n] = sum_k k2[k] W[n][k], reduced over the TPN
  // threads of a column through the (still unused) ring area; every lane keeps the biases of its
  // accumulator columns n = 16 j + 4 fq + r of the wave tile in registers
  float bias_r[WN / 16][4];
#pragma unroll
  for (int j = 0; j < WN / 16; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias_r[j][r] = 0.f;
  if (khalf) {
    constexpr int TPN = 512 / BN;  // threads per panel column
    const int n = tid % BN, tq = tid / BN;
    const int kh = khalf * 64;
    float bs = 0.f;
    for (int kt = 0; kt < khalf; ++kt) {
      for (int c = tq; c < 8; c += TPN) {
        uint4* pw = bpanel + (kt * BN + n) * 8 + c;
        const int ch = kt * 64 + ((c ^ (n & 7)) * 8);
        float w[8], k0[8], k1[8], k2[8], u0[8], u1[8];
        unpack8(*pw, w);
        pn_load8f(a.coef + ch, k0);
        pn_load8f(a.coef + kh + ch, k1);
        pn_load8f(a.coef + 2 * kh + ch, k2);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          u0[q] = w[q] * k0[q];
          u1[q] = w[q] * k1[q];
          bs = fmaf(w[q], k2[q], bs);
        }
        *pw = pack8(u0);
        bpanel[((kt + khalf) * BN + n) * 8 + c] = pack8(u1);
      }
    }
    float* red = (float*)smem;  // [TPN][BN] partial sums, then [BN] biases
    red[tq * BN + n] = bs;
    __syncthreads();
    if (tq == 0) {
      float t = 0.f;
      for (int q = 0; q < TPN; ++q) t += red[q * BN + n];
      red[TPN * BN + n] = t;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < WN / 16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias_r[j][r] = red[TPN * BN + wn * WN + 16 * j + 4 * fq + r];
    __syncthreads();  // the ring's first loads overwrite the reduction area
  }

  // ---- this wave's 32-row units: a balanced contiguous range over the panel's wave slots
  const int slots = nb * WMW, wslot = rg * WMW + wm;
  const int ubase = a.nunits / slots, urem = a.nunits % slots;
  const int u0 = wslot * ubase + min(wslot, urem);
  const int nu = ubase + (wslot < urem ? 1 : 0);
  const int G = nu * nk;  // this wave's k-steps

  uint4* ring = smem + wid * S * PN_SLOT_U4;
  // issue cursor (runs S - 1 k-steps ahead of the compute cursor)
  const int lr = lane >> 3, lc = (lane & 7) ^ (lane >> 3);  // lane's row in a piece, source chunk
  uint32_t ioff[4];
  bool iok[4];
  int ih[4], iw[4];  // gather 2: the row's pixel (h, w)
  int iu = 0, ikt = 0;
  auto set_rows = [&](int lu) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = (u0 + lu) * 32 + u * 8 + lr;
      iok[u] = lu < nu && m < a.M;
      const uint32_t mm = iok[u] ? (uint32_t)m : 0u;
      uint32_t rowe;
      if (a.gather == 2) {
        const uint32_t img = fdiv(mm, a.fPQ), rem = mm - img * a.fPQ.d;
        const uint32_t p = fdiv(rem, a.fQ), q = rem - p * a.fQ.d;
        ih[u] = (int)p;
        iw[u] = (int)q;
        rowe = mm * (uint32_t)a.lda;  // the tap's shift is added per k-step
      } else if (a.gather) {
        const uint32_t img = fdiv(mm, a.fPQ), rem = mm - img * a.fPQ.d;
        const uint32_t p = fdiv(rem, a.fQ), q = rem - p * a.fQ.d;
        rowe = ((img * (uint32_t)a.H + p * (uint32_t)a.stride) * (uint32_t)a.W + q * (uint32_t)a.stride) *
               (uint32_t)a.lda;
      } else {
        rowe = mm * (uint32_t)a.lda;
      }
      ioff[u] = (rowe + (uint32_t)lc * 8u) * 2u;
    }
  };
  auto issue_next = [&](int slot) {
    uint4* dst = ring + slot * PN_SLOT_U4;
    if (a.gather == 2) {
      const int t = ikt / a.cpt, kc = ikt - t * a.cpt;
      const int r = t / 3, sx = t - 3 * r;
      const int dh = a.tsg * (r - 1), dw = a.tsg * (sx - 1);
      const int dpix = (dh * a.W + dw) * a.lda + kc * 64;  // element shift of the tap
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = iok[u] && (unsigned)(ih[u] + dh) < (unsigned)a.H && (unsigned)(iw[u] + dw) < (unsigned)a.W;
        const uint32_t vo = ok ? ioff[u] + (uint32_t)dpix * 2u : PN_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, dst + u * 64), 16, vo, 0, 0, 0);
      }
    } else {
      // folded BN backward: the second half of the k-steps reads c (A2) at the same rows
      // (readfirstlane: the operand choice must be provably wave-uniform, or the descriptor select
      // becomes a waterfall loop with a vmcnt(0) in it)
      const int iktu = __builtin_amdgcn_readfirstlane(ikt);
      if (khalf && iktu >= khalf) {  // a branch, not a descriptor select (that one went to scratch)
        const uint32_t kb = (uint32_t)(iktu - khalf) * 128u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t vo = iok[u] ? ioff[u] + kb : PN_OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA2, LDS_PTR(void, dst + u * 64), 16, vo, 0, 0, 0);
        }
      } else {
        const uint32_t kb = (uint32_t)iktu * 128u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t vo = iok[u] ? ioff[u] + kb : PN_OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, dst + u * 64), 16, vo, 0, 0, 0);
        }
      }
    }
    if (++ikt == nk) {
      ikt = 0;
      ++iu;
      set_rows(iu);
    }
  };

  f32x4 acc[2][NJ];
  // accumulators start at the folded BN backward's bias (0 otherwise)
  auto acc_reset = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{bias_r[j][0], bias_r[j][1], bias_r[j][2], bias_r[j][3]};
  };
  acc_reset();
  // epilogue layout: the unit's bf16 tile is staged in the ring slot it consumed and read back one
  // 16-byte row chunk per lane: lane chunk ec (8 channels) of rows er + RPI u
  constexpr int CPR = WN / 8;     // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;   // rows per read instruction
  constexpr int NR = WN == 128 ? 16 : 32;  // rows staged per pass (4 KB)
  constexpr int NU = NR / RPI;    // chunks a lane reads per pass
  constexpr int HALVES = 32 / NR;
  const int ec = lane % CPR, er = lane / CPR;
  const int ncol = n0 + wn * WN + ec * 8;  // output column of the lane's chunk
  // per-lane statistics of that chunk, over every unit of the wave
  float s1[8], s2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { s1[q] = 0.f; s2[q] = 0.f; }
  const bool want_stats = a.stats != nullptr;
  // EPI 1: the BN mean of the lane's channels, and the epilogue operands of the next unit
  float mu[8];
  uint4 ey[HALVES * NU], ex[HALVES * NU], ek[HALVES * NU];  // ek: mask byte in .x (mbits) or the BN output
#pragma unroll
  for (int q = 0; q < 8; ++q) mu[q] = (EPI == 1 && a.epi >= 4 && a.stats) ? a.mean[ncol + q] : 0.f;
  auto row_of = [&](int lu, int h, int u) { return (u0 + lu) * 32 + h * NR + er + RPI * u; };
  // EL loads per call, every lane, whatever the epilogue needs (an unused operand's resource has
  // range 0: the load is dropped but still counted, so the waits' counts never depend on it)
  auto epi_issue = [&](int lu) {
    if constexpr (EPI == 1) {
#pragma unroll
      for (int h = 0; h < HALVES; ++h)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int m = row_of(lu, h, u), k = h * NU + u;
          bool even = true;
          if (a.aux_even && m < a.M) {
            const uint32_t img = fdiv((uint32_t)m, a.fPQ), rem = (uint32_t)m - img * a.fPQ.d;
            const uint32_t hh = fdiv(rem, a.fQ), w = rem - hh * a.fQ.d;
            even = ((hh | w) & 1u) == 0u;
          }
          const bool ok = lu < nu && m < a.M;
          const uint32_t off = ok ? (uint32_t)(m * a.ldc + ncol) * 2u : PN_OOB;
          ey[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsY, even ? off : PN_OOB, 0, 2));
          ex[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsX, off, 0, 0));
          if (a.mbits)
            ek[k].x = __builtin_amdgcn_raw_buffer_load_b8(rsK, ok ? off >> 4 : PN_OOB, 0, 0);
          else
            ek[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsK, off, 0, 2));
        }
    }
  };

  auto compute = [&](const uint4* As, int kt) {
    const uint4* Bs = bpanel + (kt * BN + wn * WN) * 8;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = (kk * 4 + fq) ^ (fr & 7);
      bf16x8 af[2], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = __builtin_bit_cast(bf16x8, As[(16 * i + fr) * 8 + ch]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = __builtin_bit_cast(bf16x8, Bs[(16 * j + fr) * 8 + ch]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  // epilogue of unit lu through the slot cur it consumed: lane (fr, fq) holds D[n = 16 j + 4 fq + r]
  // [m = 16 i + fr] of each fragment -> row-major bf16 rows in the slot, the 16-B chunk index XOR-
  // swizzled by the row (the ds_write_b64 groups of 16 rows hit distinct bank pairs); read back as
  // full row chunks, one 16-byte store each.  The staging stores are inline asm: an LDS store the
  // compiler can see, with LDS-DMA loads in flight, makes hipcc drain vmcnt(0) before it, and the
  // ring's prefetch would die at every unit (the slot is this wave's own and free until the next
  // issue; its k-step reads completed before the MFMAs that consumed them)
  auto epilogue = [&](uint4* Cs, int lu) {
    const uint32_t cbase = (uint32_t)(uintptr_t)LDS_PTR(void, Cs);
#pragma unroll
    for (int h = 0; h < HALVES; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2 / HALVES; ++ii) {
        const int i = h + ii;  // fragment row block
        const int row = WN == 128 ? fr : 16 * i + fr;
        // chunk swizzle within the row's CPR chunks (WN 32: 4 chunks)
        const int sw = WN == 128 ? row : ((row >> 1) & (CPR - 1));
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const f32x4 v = acc[i][j];
          const int pc = (2 * j + (fq >> 1)) ^ sw;
          const uint32_t addr = cbase + (uint32_t)(row * (WN * 2) + pc * 16 + (fq & 1) * 8);
          const uint2 d = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
          asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(d) : "memory");
        }
      }
      // the read-back, also opaque to hipcc (a visible ds_read of the slot gets a vmcnt(0) as well):
      // the NU reads and their wait in ONE statement, so no consumer can run ahead of the data
      uint32_t ra[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int rr = er + RPI * u;
        const int sw = WN == 128 ? rr : ((rr >> 1) & (CPR - 1));
        ra[u] = cbase + (uint32_t)(rr * (WN * 2) + ((ec ^ sw) * 16));
      }
      static_assert(NU == 4 || NU == 2, "four (WN 32: two) read-back chunks per pass");
      u32x4 rb[NU];
      if constexpr (NU == 4) {
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %5\n\t"
            "ds_read_b128 %2, %6\n\t"
            "ds_read_b128 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(rb[0]), "=&v"(rb[1]), "=&v"(rb[2]), "=&v"(rb[3])
            : "v"(ra[0]), "v"(ra[1]), "v"(ra[2]), "v"(ra[3])
            : "memory");
      } else {
        asm volatile(
            "ds_read_b128 %0, %2\n\t"
            "ds_read_b128 %1, %3\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(rb[0]), "=&v"(rb[1])
            : "v"(ra[0]), "v"(ra[1])
            : "memory");
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int k = h * NU + u;
        uint4 o = __builtin_bit_cast(uint4, rb[u]);
        const int m = row_of(lu, h, u);
        if constexpr (EPI == 0) {
          if (want_stats) {
            float f[8];
            unpack8(o, f);
#pragma unroll
            for (int q = 0; q < 8; ++q) { s1[q] += f[q]; s2[q] = fmaf(f[q], f[q], s2[q]); }
          }
        } else if (a.epi == 3) {
          float f[8], g[8];
          unpack8(o, f);
          unpack8(ey[k], g);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] += g[q];
          o = pack8(f);
        } else if (a.epi >= 4) {
          float f[8];
          unpack8(o, f);
          if (a.epi == 5) {
            float g[8];
            unpack8(ey[k], g);
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] += g[q];
          }
          if (a.bn_relu) {
            const uint32_t bits = a.mbits ? ek[k].x : nz_bits8(ek[k]);
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = ((bits >> q) & 1u) ? f[q] : 0.f;
          }
          o = pack8(f);
          if (want_stats) {
            float xv[8];
            unpack8(ex[k], xv);
            const bool live = m < a.M;  // rows past M hold the folded bias when unmasked
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const float fz = live ? f[q] : 0.f;
              s1[q] += fz;
              s2[q] = fmaf(fz, xv[q] - mu[q], s2[q]);
            }
          }
        }
        const uint32_t off = (m < a.M && ncol < a.N) ? (uint32_t)(m * a.ldc + ncol) * 2u : PN_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsC, off, 0, 0);
      }
    }
    acc_reset();
  };

  // ---- main loop over the wave's k-steps
  epi_issue(0);  // before every ring load: never younger than a k-step's loads
  set_rows(0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue_next(s);
  uint32_t ehist = 0;  // bit t: an epilogue ran t + 1 iterations ago
  int kt = 0, lu = 0, slot = 0;
  for (int g = 0; g < G; ++g) {
    issue_next(slot == 0 ? S - 1 : slot - 1);  // k-step g + S - 1 into the slot k-step g - 1 used
    pn_wait<S, ST + EL>(__builtin_popcount(ehist & ((1u << (S - 1)) - 1u)));
    uint4* cur = ring + slot * PN_SLOT_U4;
    compute(cur, kt);
    ehist <<= 1;
    if (++kt == nk) {
      epilogue(cur, lu);
      epi_issue(lu + 1);  // past the last unit: dropped loads (the counts hold)
      ehist |= 1u;
      kt = 0;
      ++lu;
    }
    slot = slot + 1 == S ? 0 : slot + 1;
  }

  // ---- statistics: lanes sharing a chunk (xor over the row bits of the lane), then the WMW waves of
  // each column sub-panel through LDS, in a fixed order
  if (want_stats) {
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s1[q] += __shfl_xor(s1[q], o, 64);
        s2[q] += __shfl_xor(s2[q], o, 64);
      }
  }
  PN_VMWAIT(0);  // the ring's trailing dummy loads still write LDS
  __syncthreads();
  if (want_stats) {
    float* red = (float*)smem;  // [8 waves][2][WN]
    if (lane < CPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wid * 2 + 0) * WN + ec * 8 + q] = s1[q];
        red[(wid * 2 + 1) * WN + ec * 8 + q] = s2[q];
      }
    }
    __syncthreads();
    for (int c = tid; c < 2 * BN; c += 512) {
      const int which = c / BN, col = c - which * BN;
      const int cwn = col / WN, cc = col - cwn * WN;
      float t = 0.f;
      for (int w = 0; w < WMW; ++w) t += red[((w * WNW + cwn) * 2 + which) * WN + cc];
      if (n0 + col < a.N) a.stats[((size_t)rg * 2 + which) * a.N + n0 + col] = t;
    }
  }
}

// ------------------------------------------------------------------ host side
// MI355X_DP_PANEL (mi_set_panel): 1 route eligible 1x1 convs with >= PN_MIN_M output rows here
// (default), 0 never, 2 any row count (tests: small shapes stay on the split-K 64-tile kernels
// otherwise); + 4 the 3x3 pad-1 stride-1 convs too (off by default, mi_panel_3x3)
static int g_pn_mode = -1;
constexpr int PN_MIN_M = 16384;
static int g_pn_cus = 0;

struct PanelPlan {
  int bn = 0, wn = 0, s = 0, npanel = 0, nb = 0;
};

// panel width / ring depth for an N x K weight panel; bn == 0: not eligible.  dgrad: the data-gradient
// variant (64-column waves: its next-unit epilogue operands live in registers)
PanelPlan panel_plan(int M, int N, int K, bool dgrad) {
  PanelPlan p;
  if (g_pn_mode < 0) {
    const char* e = std::getenv("MI355X_DP_PANEL");
    g_pn_mode = (e && e[0] >= '0' && e[0] <= '7') ? e[0] - '0' : 1;
  }
  if (!(g_pn_mode & 3) || K % 64 != 0 || K > 1024 || N % 32 != 0 || M < ((g_pn_mode & 2) ? 1 : PN_MIN_M)) return p;
  if (g_pn_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_pn_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_pn_cus <= 0)
      g_pn_cus = 256;
  }
  const int64_t kb = (int64_t)K * 2;  // bytes per panel row
  if (N % 256 == 0 && 256 * kb <= 64 * 1024) {
    p.bn = 256;
  } else if (N % 128 == 0 && 128 * kb <= 64 * 1024) {
    p.bn = 128;
  } else if (N % 64 == 0 && 64 * kb <= 96 * 1024) {
    p.bn = 64;
  } else if (32 * kb <= 64 * 1024) {
    p.bn = 32;  // K up to 1024 (e.g. ResNet layer 3's 1024 -> 256 convs): 32-column panels, 8 per 256 cols
  } else {
    return PanelPlan{};
  }
  p.wn = p.bn == 32 ? 32 : (dgrad ? 64 : std::min(p.bn, 128));
  // ring depth from what the weight panel leaves of the 160 KB: 8 waves x S x 4 KB
  const int64_t bpanel = p.bn * kb;
  p.s = bpanel <= 32 * 1024 ? 4 : (bpanel <= 64 * 1024 ? 3 : 2);
  p.npanel = N / p.bn;
  const int units = cdiv(M, 32);
  const int wm = 8 / (p.bn / p.wn);
  p.nb = std::max(1, std::min(g_pn_cus / std::max(1, std::min(p.npanel, g_pn_cus)), cdiv(units, wm)));
  return p;
}

template <int BN, int WN, int EPI>
void launch_panel(const PanelArgs& a, int s, int grid, hipStream_t st) {
  if (s == 4)
    hipLaunchKernelGGL((panel_kernel<BN, WN, 4, EPI>), dim3(grid), dim3(512), 0, st, a);
  else if (s == 3)
    hipLaunchKernelGGL((panel_kernel<BN, WN, 3, EPI>), dim3(grid), dim3(512), 0, st, a);
  else if constexpr (BN == 64)  // a 64-column panel of a 3x3 conv over 64 channels (72 KB)
    hipLaunchKernelGGL((panel_kernel<BN, WN, 2, EPI>), dim3(grid), dim3(512), 0, st, a);
}

template <int EPI>
int launch_plan(const PanelPlan& p, PanelArgs& a, hipStream_t st, const char* what) {
  a.npanel = p.npanel;
  a.nunits = cdiv(a.M, 32);
  if (!a.ldb) a.ldb = a.K;
  const int grid = p.npanel * p.nb;
  if (const char* t = std::getenv("MI355X_DP_TRACE_GEMM"); t && t[0] == '1')
    fprintf(stderr, "[gemm] panel-%s %d/%d s%d M=%d N=%d K=%d epi=%d stats=%d blocks=%d\n", what, p.bn, p.wn, p.s, a.M,
            a.N, a.K, a.epi, a.stats != nullptr, grid);
  if constexpr (EPI == 0) {
    if (p.bn == 256) launch_panel<256, 128, 0>(a, p.s, grid, st);
    else if (p.bn == 128) launch_panel<128, 128, 0>(a, p.s, grid, st);
    else if (p.bn == 64) launch_panel<64, 64, 0>(a, p.s, grid, st);
    else launch_panel<32, 32, 0>(a, p.s, grid, st);
  } else {
    if (p.bn == 256) launch_panel<256, 64, 1>(a, p.s, grid, st);
    else if (p.bn == 128) launch_panel<128, 64, 1>(a, p.s, grid, st);
    else if (p.bn == 64) launch_panel<64, 64, 1>(a, p.s, grid, st);
    else launch_panel<32, 32, 1>(a, p.s, grid, st);
  }
  return (int)hipGetLastError();
}

}  // namespace

MI_API int mi_set_panel(int mode) {
  g_pn_mode = mode & 7;
  return 0;
}

// the 3x3 (pad 1) convolutions route to the panel kernel only with mode bit 4: measured 0.94x (forward)
// and 0.98x (data gradient) of the halo-tiled 3x3 kernels on the layer-1 shapes (profiles/panel_r6.md)
MI_API int mi_panel_3x3() {
  if (g_pn_mode < 0) (void)panel_plan(0, 0, 0, false);  // env init
  return (g_pn_mode & 4) ? 1 : 0;
}

// statistics rows the panel kernel writes for an M x N x K conv forward (dgrad = 0) or data gradient
// (dgrad = 1); 0: not routed there
MI_API int mi_panel_stat_rows2(int M, int N, int K, int dgrad) {
  const PanelPlan p = panel_plan(M, N, K, dgrad != 0);
  return p.bn ? p.nb : 0;
}
MI_API int mi_panel_stat_rows(int M, int N, int K) { return mi_panel_stat_rows2(M, N, K, 0); }

// conv forward on the panel kernel: 1x1 (pad 0, stride s) or 3x3 (stride 1, pad 1); x NHWC [Nb,H,W,C],
// w [K][R][R][C], y NHWC [Nb,P,Q,K] bf16; stats: [mi_panel_stat_rows][2][K].  hipErrorNotSupported:
// shape not eligible.
MI_API int mi_panel_conv(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int C, int K, int R,
                         int stride, int pad, int P, int Q, hipStream_t st) {
  const int M = Nb * P * Q;
  const bool tap3 = R == 3;
  if (!((R == 1 && pad == 0) || (tap3 && stride == 1 && pad == 1 && P == H && Q == W)) || C % 64 != 0)
    return (int)hipErrorNotSupported;
  const PanelPlan p = panel_plan(M, K, R * R * C, false);
  if (!p.bn) return (int)hipErrorNotSupported;
  const int64_t ab = (int64_t)Nb * H * W * C * 2, cb = (int64_t)M * K * 2, bb = (int64_t)K * R * R * C * 2;
  if (ab > 0x7FFFFFF0LL || cb > 0x7FFFFFF0LL || bb > 0x7FFFFFF0LL) return (int)hipErrorNotSupported;
  PanelArgs a{};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = (bf16_t*)y; a.stats = stats;
  a.M = M; a.N = K; a.K = R * R * C; a.ldc = K;
  a.nk = a.K / 64;
  a.a_bytes = (int)ab; a.b_bytes = (int)bb; a.c_bytes = (int)cb;
  a.gather = tap3 ? 2 : ((stride != 1 || P != H || Q != W) ? 1 : 0);
  a.lda = C; a.H = H; a.W = W; a.stride = stride;
  a.tsg = 1; a.cpt = C / 64;
  a.fPQ = make_fastdiv((uint32_t)(P * Q));
  a.fQ = make_fastdiv((uint32_t)Q);
  return launch_plan<0>(p, a, st, tap3 ? "fwd3x3" : "fwd");
}
MI_API int mi_panel_conv1x1(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int C, int K,
                            int stride, int P, int Q, hipStream_t st) {
  return mi_panel_conv(x, w, y, stats, Nb, H, W, C, K, 1, stride, 0, P, Q, st);
}

// 1x1 or 3x3 (pad 1) / stride-1 conv data gradient on the panel kernel: dy NHWC [Nb,H,W,K], wt [C][R][R][K], dx NHWC
// [Nb,H,W,C] with nt_kernel's epilogues (PanelArgs::epi; mbits or aux = the BN output for the ReLU
// mask; stats [mi_panel_stat_rows2(.., 1)][2][C]; epi 5 with acc_src: accumulate acc_src into dx out of
// place).  hipErrorNotSupported: not eligible.
MI_API int mi_panel_dgrad(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C, int K, int R,
                          int epi, const void* aux, const void* aux2, const float* mean, int bn_relu, float* stats,
                          int aux_even, const void* mbits, const void* acc_src, hipStream_t st) {
  const int M = Nb * H * W;
  if ((R != 1 && R != 3) || K % 64 != 0) return (int)hipErrorNotSupported;
  const PanelPlan p = panel_plan(M, C, R * R * K, true);
  if (!p.bn || !(epi == 0 || epi == 3 || epi == 4 || epi == 5)) return (int)hipErrorNotSupported;
  const int64_t ab = (int64_t)M * K * 2, cb = (int64_t)M * C * 2, bb = (int64_t)C * R * R * K * 2;
  if (ab > 0x7FFFFFF0LL || cb > 0x7FFFFFF0LL || bb > 0x7FFFFFF0LL) return (int)hipErrorNotSupported;
  PanelArgs a{};
  a.A = (const bf16_t*)dy; a.B = (const bf16_t*)wt; a.C = (bf16_t*)dx;
  a.stats = epi >= 4 ? stats : nullptr;
  a.M = M; a.N = C; a.K = R * R * K; a.ldc = C;
  a.nk = a.K / 64;
  a.a_bytes = (int)ab; a.b_bytes = (int)bb; a.c_bytes = (int)cb;
  a.gather = R == 3 ? 2 : 0; a.lda = K; a.H = H; a.W = W; a.stride = 1;
  a.tsg = -1; a.cpt = K / 64;
  a.fPQ = make_fastdiv((uint32_t)(H * W));
  a.fQ = make_fastdiv((uint32_t)W);
  a.epi = epi; a.bn_relu = epi >= 4 ? bn_relu : 0; a.aux_even = (epi == 3 || epi == 5) ? aux_even : 0;
  a.aux = (const bf16_t*)aux; a.aux2 = (const bf16_t*)aux2; a.mean = mean; a.mbits = (const uint8_t*)mbits;
  a.acc_src = epi == 5 ? (const bf16_t*)acc_src : nullptr;
  return launch_plan<1>(p, a, st, R == 3 ? "dgrad3x3" : "dgrad");
}

// Folded BatchNorm backward into a 1x1 / stride-1 data gradient: the gradient
// of the conv's input, dx = dgrad(k0 dz + k1 c + k2) with the BN of THIS conv's output (c, its
// masked output gradient dz, coef = (k0, k1, k2) [3][K] from the BN-backward finalize), computed as
// one GEMM over [dz | c] (2K deep) against [diag(k0) W | diag(k1) W] plus a per-column bias, so the
// BN's input gradient is never written or read.  wt [C][K] (bf16, the dgrad weight layout); the
// epilogues and statistics are mi_panel_dgrad's (epi 5 may accumulate out of place: acc_src, the
// gradient added to, and dx, the result, may differ).  hipErrorNotSupported: not eligible.
MI_API int mi_panel_dgrad_fbb(const void* dz, const void* c, const float* coef, const void* wt, void* dx, int Nb, int H,
                              int W, int C, int K, int epi, const void* aux, const void* aux2, const float* mean,
                              int bn_relu, float* stats, int aux_even, const void* mbits, const void* acc_src,
                              hipStream_t st) {
  const int M = Nb * H * W;
  if (K % 64 != 0 || !coef || !(epi == 0 || epi == 3 || epi == 4 || epi == 5)) return (int)hipErrorNotSupported;
  const PanelPlan p = panel_plan(M, C, 2 * K, true);
  if (!p.bn) return (int)hipErrorNotSupported;
  const int64_t ab = (int64_t)M * K * 2, cb = (int64_t)M * C * 2, bb = (int64_t)C * K * 2;
  if (ab > 0x7FFFFFF0LL || cb > 0x7FFFFFF0LL || bb > 0x7FFFFFF0LL) return (int)hipErrorNotSupported;
  PanelArgs a{};
  a.A = (const bf16_t*)dz; a.A2 = (const bf16_t*)c; a.B = (const bf16_t*)wt; a.C = (bf16_t*)dx;
  a.coef = coef;
  a.stats = epi >= 4 ? stats : nullptr;
  a.M = M; a.N = C; a.K = 2 * K; a.ldc = C; a.ldb = K;
  a.nk = a.K / 64; a.khalf = K / 64;
  a.a_bytes = (int)ab; a.a2_bytes = (int)ab; a.b_bytes = (int)bb; a.c_bytes = (int)cb;
  a.gather = 0; a.lda = K; a.H = H; a.W = W; a.stride = 1;
  a.tsg = -1; a.cpt = K / 64;
  a.fPQ = make_fastdiv((uint32_t)(H * W));
  a.fQ = make_fastdiv((uint32_t)W);
  a.epi = epi; a.bn_relu = epi >= 4 ? bn_relu : 0; a.aux_even = (epi == 3 || epi == 5) ? aux_even : 0;
  a.aux = (const bf16_t*)aux; a.aux2 = (const bf16_t*)aux2; a.mean = mean; a.mbits = (const uint8_t*)mbits;
  a.acc_src = epi == 5 ? (const bf16_t*)acc_src : nullptr;
  return launch_plan<1>(p, a, st, "dgrad-fbb");
}

// statistics rows of mi_panel_dgrad_fbb (M rows, C output channels, K = channels of dz / c); 0: the
// folded path does not take the shape
MI_API int mi_panel_fbb_rows(int M, int C, int K) {
  if (K % 64 != 0) return 0;
  return mi_panel_stat_rows2(M, C, 2 * K, 1);
}
