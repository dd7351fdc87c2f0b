// Deep-pipelined 256x256 NT GEMM for gfx950: C[M][N] = A[M][K] · B[N][K]^T (+bias, fused
// bf16 epilogue ops), bf16 operands, fp32 accumulation.  Used for the large plain GEMMs
// (ViT-B/16 projections / MLP, large-batch linear layers); gemm_conv.hip keeps the small
// shapes and the implicit-GEMM convolutions.
//
// Why a second NT kernel: the 128x128 single-stage loop waits vmcnt(0) + barrier every k-step
// (rocprofv3: SQ_WAIT_ANY ~50 % of wave cycles at M=50432 N=3072 K=768).  Here global loads stay
// in flight across barriers:
//
//  * block 256x256, 8 waves (2 along M x 4 along N), wave tile 128x64 = 8x4 MFMA 16x16 tiles;
//  * one "phase" per output quadrant (mq, nq) of the wave tile, order (0,0) (0,1) (1,1) (1,0):
//    16 MFMAs of 16x16x32 over one BK=64 k-tile, A fragments reused in phases 0->1 and 2->3,
//    B fragments in 1->2;
//  * LDS = 2 k-tile buffers x 4 "parts" of 16 KB: A part mq = the 64-row slices of both wave
//    rows that quadrant row mq reads, B part nq likewise for the columns, so a phase needs just
//    one A part and one B part of its k-tile;
//  * every phase issues one part (2 x 16-B buffer_load ... lds per thread) for a future k-tile,
//    scheduled so each part lands >= 3 phases before it is read:
//        phase 0: B0[t+1]  1: A1[t+1]  2: A0[t+2]  3: B1[t+2];
//  * fragments are read from LDS ahead of their MFMAs (B one phase ahead in a second slot, A
//    right after the MFMAs that last use its registers), so LDS latency overlaps MFMA execution;
//  * waits are counted, never 0 in the loop: phase 1 vmcnt(6) (retires A1[t]), phase 3 vmcnt(4)
//    (retires B0[t+1], A0[t+1]), each followed by the only two raw s_barriers of the k-tile (no
//    __syncthreads, which would drain the queue); loads past the last k-tile are issued as
//    zero-fill dummies so the counts hold in the tail;
//  * LDS images are lane-linear (direct-to-LDS), XOR-swizzled on the source side so the 16-row
//    ds_read_b128 fragment reads spread over the banks;
//  * XCD-aware, M-grouped tile order (GROUP_M 8) for L2 reuse of the B panel.
#include "common.h"
#include "epilogue.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>

// epilogue row steps per group of batched operand loads: plain GEMM / conv (BN) epilogues
constexpr int kG256EpiU0 = 8, kG256EpiUBN = 4;

namespace {

constexpr int G_BM = 256, G_BN = 256, G_BK = 64;
constexpr int PART_U4 = 128 * 8;      // 128 rows x 8 x 16-B chunks = 16 KB
constexpr int GROUP_M = 8;
constexpr uint32_t OOB = 0xFFFFFFF0u;

struct G256Args {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const float* bias;
  bf16_t* aux;
  int epi;              // bf16 epilogue op (epilogue.h), 4 = BN backward (see gemm_conv.hip NTArgs)
  int M, N, K, lda, ldb, ldc;
  int out_f32, accumulate;
  int tiles_m, tiles_n;
  int a_bytes, b_bytes;
  // conv modes (1 = forward, gathers x; 2 = stride-1 data gradient, gathers dy): A rows are the
  // output pixels (img, p, q) of a P x Q grid, k = (tap r, tap s, channel) of a gathered NHWC
  // tensor [.., H, W, Cs] with Cs % 64 == 0 (one k-tile = one tap x 64 channels)
  int H, W, Cs, S, stride, pad;
  FastDiv fPQ, fQ, fS, fCpt;
  float* stats;         // per-channel partial statistics, one slab row per (256-row tile, wave row)
  const bf16_t* aux2;   // epi 4: BN input x
  const float* mean;    // epi 4: BN batch mean
  int bn_relu;
  // tail split-K (wave quantization): blocks [0, full_blocks) own whole tiles; the tiles of the
  // last, partial wave are split `tail_split` ways along K; the last-arriving split of a tile adds
  // the others' fp32 partials (workspace `ws`, per-tile arrival `counters`) and runs the epilogue
  int full_blocks, tail_split;
  float* ws;
  int* counters;
  int aux_even;         // epi 3 / 5: accumulated-into gradient defined only at even (h, w) (gemm_conv.hip)
  const uint8_t* mbits; // epi 4 / 5: ReLU mask bytes (8 channels each) instead of aux (gemm_conv.hip NTArgs)
  // folded BN backward (mode 2, 1x1): k-tiles [khalf_kt, 2 khalf_kt) gather c (A2) where the first
  // half gathers dz (A); B = [diag(k0) W | diag(k1) W], bias = k2 W (mi_gemm256_dgrad_fbb)
  const bf16_t* A2;
  int a2_bytes, khalf_kt;
};

// Wave priority: static s_setprio 1 for the second-dispatched half (waves 4-7) before the main loop
// (MI355X_MICROARCH.md, two waves per SIMD, item 4) -- the guard must be provably wave-uniform
// (readfirstlane): a plain `if (wid >= 4)` lowers to s_and_saveexec + an UNCONDITIONAL s_setprio,
// i.e. every wave at priority 1.  (Per-MFMA-cluster setprio flips measured no better; removed.)
__device__ __forceinline__ void static_prio() {
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
}

__device__ __forceinline__ void vm_wait6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }
__device__ __forceinline__ void vm_wait4() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// raw barrier that is also a compiler memory barrier: LDS reads of a phase must not be hoisted
// above the barrier that publishes their part (the builtin s_barrier is not a memory op)
__device__ __forceinline__ void phase_barrier() { asm volatile("s_barrier" ::: "memory"); }

// WR: rows per wave row -- 128 (256-row tiles) or 112 (224-row tiles: a 196-tile grid on 256 CUs becomes
// 224 tiles of 7/8 the work; g256_bm).  The LDS parts keep their 128-row layout: with WR 112 the
// second quadrant row holds 48 real rows (rows 48..63 of each wave row's slice are zero-filled and
// never multiplied), IQ1 = 3 fragment rows instead of 4.
// SCAT (MODE 0, bf16 out): output row m goes to row 2 (m / Q) W + 2 (m % Q) of C -- the even pixels of a
// 2H' x 2W' grid: the stride-2 1x1 data gradient of a projection shortcut written straight into the
// even pixels of dx (Q = a.fQ.d, W = a.W; mi_gemm256_nt_scat2)
template <int MODE, int WR = 128, bool SCAT = false>
__global__ __launch_bounds__(512, 1) void gemm256_nt_kernel(G256Args a) {
  static_assert(WR == 128 || WR == 112, "256- or 224-row tiles");
  static_assert(!SCAT || MODE == 0, "scattered rows: plain GEMM only");
  constexpr int IQ1 = (WR - 64) / 16;  // fragment rows of quadrant row 1
  constexpr int NI = 4 + IQ1;          // accumulator rows per wave
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * 4 * PART_U4];  // 128 KB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // tile order: XCD remap, then GROUP_M-row groups sweeping N; tail tiles split along K
  const int nk = (a.K + G_BK - 1) / G_BK;
  int bid, kt0 = 0, kt1 = nk, split = 0, tail_tile = -1;
  if ((int)blockIdx.x < a.full_blocks) {
    bid = xcd_remap(blockIdx.x, a.full_blocks);
  } else {
    const int nunits = gridDim.x - a.full_blocks;
    const int u = xcd_remap(blockIdx.x - a.full_blocks, nunits);
    tail_tile = u / a.tail_split;
    split = u - tail_tile * a.tail_split;
    bid = a.full_blocks + tail_tile;
    kt0 = split * nk / a.tail_split;
    kt1 = (split + 1) * nk / a.tail_split;
  }
  const int group = bid / (GROUP_M * a.tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(a.tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % (GROUP_M * a.tiles_n)) % gsz;
  const int tn = (bid % (GROUP_M * a.tiles_n)) / gsz;
  const int m0 = tm * (2 * WR), n0 = tn * G_BN;
  const int nkl = kt1 - kt0;  // this block's k-tiles

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.b_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsA2 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(MODE == 2 && a.khalf_kt ? a.A2 : a.A), (short)0, MODE == 2 && a.khalf_kt ? a.a2_bytes : 0, 0x00020000);

  // per-thread load geometry, fixed across k-tiles: 2 chunks per part, LDS rows p = (i*512+tid)/8.
  // plain: byte offset at k-tile t = base + 128 t while t < klim (chunk inside K), else the
  // out-of-range offset (zero fill).  Rows past M / N need no test: their offsets lie beyond the
  // buffer resource's range (the range is exactly the operand), which zero-fills.
  // conv: A row = output pixel; per k-tile the tap (r, s) and channel block are wave-uniform,
  // the row's gathered pixel (hb + r, wb + s) is range-checked (zero padding = zero fill).
  uint32_t a_vo[2][2], b_vo[2][2];
  int klim[2];
  int a_hw[2][2];  // conv: gathered-pixel origin (hb << 16 | wb & 0xffff), row validity in bit 15 of wb
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = i * 512 + tid, p = idx >> 3, c = idx & 7;
    const int gk = (c ^ (p & 7)) * 8;  // source-side swizzle: LDS chunk c of row p holds global chunk c^(p&7)
    klim[i] = gk < a.K ? (a.K - gk + G_BK - 1) / G_BK : 0;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const bool rin = part * 64 + (p & 63) < WR;  // a row of this tile (WR 112: not the padding)
      const int m = m0 + (p >> 6) * WR + part * 64 + (p & 63);
      b_vo[part][i] = (uint32_t)((n0 + (p >> 5) * 64 + part * 32 + (p & 31)) * a.ldb + gk) * 2u;
      if constexpr (MODE == 0) {
        a_vo[part][i] = rin ? (uint32_t)(m * a.lda + gk) * 2u : 0xF0000000u;  // padding: past the range
        a_hw[part][i] = 0;
      } else {
        const uint32_t mm = (rin && m < a.M) ? (uint32_t)m : 0u;
        const uint32_t img = fdiv(mm, a.fPQ);
        const uint32_t rem = mm - img * a.fPQ.d;
        const uint32_t pp = fdiv(rem, a.fQ);
        const uint32_t qq = rem - pp * a.fQ.d;
        const int hb = MODE == 1 ? (int)pp * a.stride - a.pad : (int)pp + a.pad;
        const int wb = MODE == 1 ? (int)qq * a.stride - a.pad : (int)qq + a.pad;
        // element offset of the gathered pixel (hb, wb) channel gk (may be negative: padding)
        a_vo[part][i] = (uint32_t)((((int)img * a.H + hb) * a.W + wb) * a.Cs + gk);
        a_hw[part][i] = (rin && m < a.M) ? (hb << 16) | (wb & 0xffff) : (int)0x80008000;  // invalid: h = -32768
      }
    }
  }

  // issue part `part` of operand `which` (0 = A, 1 = B) for k-tile t (zero-fill past the end)
  auto issue = [&](int t, int which, int part) {  // t: local k-tile (buffer parity), ta: absolute
    uint4* dst = smem + ((t & 1) * 4 + which * 2 + part) * PART_U4;
    const int ta = kt0 + t;
    const uint32_t kb = (uint32_t)ta * (G_BK * 2);
    if (which == 1 || MODE == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t vo = (ta < kt1 && ta < klim[i]) ? (which == 0 ? a_vo[part][i] : b_vo[part][i]) + kb : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(which == 0 ? rsA : rsB, LDS_PTR(void, dst + i * 512 + wid * 64),
                                                 16, vo, 0, 0, 0);
      }
    } else {
      // wave-uniform tap / channel block of k-tile t (folded BN backward: the second half of the
      // k-tiles gathers c from A2 -- a branch, the operand choice must stay scalar)
      const int tt0 = __builtin_amdgcn_readfirstlane(ta < kt1 ? ta : 0);
      const bool second = MODE == 2 && a.khalf_kt && tt0 >= a.khalf_kt;
      const int tt = second ? tt0 - a.khalf_kt : tt0;
      const int tap = (int)fdiv((uint32_t)tt, a.fCpt);
      const int c0 = (tt - tap * (int)a.fCpt.d) * 64;
      const int r = (int)fdiv((uint32_t)tap, a.fS);
      const int sx = tap - r * a.S;
      const int dh = MODE == 1 ? r : -r, dw = MODE == 1 ? sx : -sx;
      const int toff = (dh * a.W + dw) * a.Cs + c0;
      uint32_t vos[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int hw = a_hw[part][i];
        const int h = (hw >> 16) + dh, w = ((int)(short)(hw & 0xffff)) + dw;
        const bool ok = ta < kt1 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        vos[i] = ok ? (uint32_t)((int)a_vo[part][i] + toff) * 2u : OOB;
        MI_ASSERT(vos[i] == OOB || vos[i] + 16u <= (uint32_t)(second ? a.a2_bytes : a.a_bytes), vos[i]);
      }
      if (second) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA2, LDS_PTR(void, dst + i * 512 + wid * 64), 16, vos[i], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, dst + i * 512 + wid * 64), 16, vos[i], 0, 0, 0);
      }
    }
  };

  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment registers: one A set (re-read right after the MFMAs that last use it, so the LDS
  // latency overlaps their execution) and two B slots that swap roles each k-tile (the loop body
  // is unrolled x2 so every slot is a fixed register set)
  bf16x8 af[4][2], bx[2][2], by[2][2];
  auto read_a = [&](bf16x8 (&f)[4][2], int t, int mq) {
    const uint4* src = smem + ((t & 1) * 4 + mq) * PART_U4;
#pragma unroll
    for (int i = 0; i < (mq == 0 ? 4 : IQ1); ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        f[i][kk] = __builtin_bit_cast(bf16x8, src[(wm * 64 + i * 16 + fr) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
  };
  auto read_b = [&](bf16x8 (&f)[2][2], int t, int nq) {
    const uint4* src = smem + ((t & 1) * 4 + 2 + nq) * PART_U4;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        f[j][kk] = __builtin_bit_cast(bf16x8, src[(wn * 32 + j * 16 + fr) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
  };
  auto mma = [&](const bf16x8 (&af_)[4][2], const bf16x8 (&bf)[2][2], int mq, int nq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < (mq == 0 ? 4 : IQ1); ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af_[i][kk], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
  };

  // One k-tile = 4 quadrant phases:
  //   q0: issue B0[t+1]; read B1[t] -> bn;                        MFMA (A0, B0[t] in bc)
  //   q1: vmcnt(6) (A1[t] landed) + barrier; issue A1[t+1];       MFMA (A0, bn); read A1[t] -> af
  //   q2: issue A0[t+2];                                          MFMA (A1, bn)
  //   q3: vmcnt(4) (B0[t+1], A0[t+1] landed) + barrier; issue B1[t+2]; read B0[t+1] -> bn;
  //                                                               MFMA (A1, bc); read A0[t+1] -> af
  // Only q1 / q3 need a barrier: every restaged region was last read >= 1 barrier earlier by
  // reads whose MFMAs every wave has executed before passing it.
  auto ktile = [&](int t, bf16x8 (&bc)[2][2], bf16x8 (&bn)[2][2]) {
    issue(t + 1, 1, 0);
    read_b(bn, t, 1);
    mma(af, bc, 0, 0);
    vm_wait6();
    phase_barrier();
    issue(t + 1, 0, 1);
    mma(af, bn, 0, 1);
    read_a(af, t, 1);
    issue(t + 2, 0, 0);
    mma(af, bn, 1, 1);
    vm_wait4();
    phase_barrier();
    issue(t + 2, 1, 1);
    const bool more = t + 1 < nkl;
    if (more) read_b(bn, t + 1, 0);
    mma(af, bc, 1, 0);
    if (more) read_a(af, t + 1, 0);
  };

  // prologue: the loads steady state would have issued before k-tile 0, then A0[0] / B0[0]
  issue(0, 0, 0); issue(0, 1, 1); issue(0, 1, 0); issue(0, 0, 1); issue(1, 0, 0); issue(1, 1, 1);
  vm_wait6();
  phase_barrier();
  read_a(af, 0, 0);
  read_b(bx, 0, 0);
  // static priority for the second-dispatched half: the two waves sharing a SIMD stop running in
  // lockstep, so one's MFMAs overlap the other's LDS reads / barrier waits
  static_prio();
  for (int t = 0; t < nkl; t += 2) {
    ktile(t, bx, by);
    if (t + 1 < nkl) ktile(t + 1, by, bx);
  }
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy loads of the tail still target LDS
  __syncthreads();

  // ---- tail split-K: publish this split's partial; the last arriver of the tile reduces
  if (tail_tile >= 0) {
    // partial layout [acc index][thread] (16 B per thread): every store / load wave-instruction
    // covers 1 KB contiguous.  Fence-free hand-off (MI355X_MICROARCH.md, inter-workgroup
    // visibility, first table row): every wave stores its partial with sc1 (write-through, dropped
    // from the XCD's L2) and waits for the stores, then behind a barrier one lane counts the
    // arrival with an agent-scope atomic; the last arriver reads the partials with sc1 loads.  The
    // acq_rel __threadfence pair this replaces cost ~3.5 us per fence.
    const size_t tile_f = (size_t)G_BM * G_BN;
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
        a.ws + (size_t)tail_tile * a.tail_split * tile_f, (short)0, (int)(a.tail_split * tile_f * 4), 0x00020000);
    constexpr int SC1 = 16;  // cache-policy bits of the buffer intrinsics: sc1
    const uint32_t mine = (uint32_t)(split * tile_f * 4) + tid * 16;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) __builtin_amdgcn_raw_buffer_store_b128(acc[i][j], rsw, mine + (i * 4 + j) * 8192, 0, SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;  // LDS is free after the loop (no second __shared__ object)
    if (tid == 0) flag[0] = atomicAdd(a.counters + tail_tile, 1) == a.tail_split - 1;
    __syncthreads();
    if (!flag[0]) return;
    // sum the partials in split order 0, 1, ... -- this block's own one re-read from the workspace
    // -- so the result does not depend on which split arrived last (fp32 adds do not associate)
    for (int q = 0; q < a.tail_split; ++q) {
      const uint32_t part = (uint32_t)(q * tile_f * 4) + tid * 16;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsw, part + (i * 4 + j) * 8192, 0, SC1);
          acc[i][j] = q == 0 ? v : acc[i][j] + v;
        }
    }
    if (tid == 0) a.counters[tail_tile] = 0;  // ready for the next launch (stream order)
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // lane holds D[n = 16j + 4fq + r][m = 16i + fr] of each 16x16 tile (weights-first MFMA)
  if (a.out_f32) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = m0 + wm * WR + i * 16 + fr;
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * fq;
        if (n >= a.N) continue;
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if (a.bias) { v0 += a.bias[n]; v1 += a.bias[n + 1]; v2 += a.bias[n + 2]; v3 += a.bias[n + 3]; }
        float* dst = (float*)a.C + (size_t)m * a.ldc + n;
        if (a.accumulate) { const float4 o = *(float4*)dst; v0 += o.x; v1 += o.y; v2 += o.z; v3 += o.w; }
        *(float4*)dst = make_float4(v0, v1, v2, v3);
      }
    }
    return;
  }
  // bf16: each wave stages 64 rows x 64 cols at a time in its own LDS slice, then 16-B row stores.
  // Optional per-channel statistics: the wave's 128 rows x 64 columns go to slab row tm*2 + wm.
  constexpr int CST = 72;  // padded row stride (elements)
  bf16_t* Ct = (bf16_t*)smem + wid * 64 * CST;
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + 4 * fq;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = (a.bias && n + r < a.N) ? a.bias[n + r] : 0.f;
  }
  const int cc = lane & 7;
  const int n = n0 + wn * 64 + cc * 8;
  // plain GEMMs (MODE 0: transformer layers) never carry BN statistics or the BN-backward
  // epilogues: compiled out, their registers go to a deeper batch of epilogue operand loads
  constexpr bool BN_EPI = MODE != 0;
  const bool has_stats = BN_EPI && a.stats != nullptr;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8];
  if (BN_EPI && a.epi >= 4 && a.stats && n < a.N) {
    *(float4*)&mu[0] = *(const float4*)(a.mean + n);
    *(float4*)&mu[4] = *(const float4*)(a.mean + n + 4);
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq) {
#pragma unroll
    for (int i = 0; i < (mq == 0 ? 4 : IQ1); ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = acc[mq * 4 + i][j];
        // 8-B slot XOR-swizzled by row bit 3 (conflict-free ds_write_b64 groups, see gemm_conv.hip)
        *(uint2*)&Ct[(i * 16 + fr) * CST + ((j * 16 + 4 * fq) ^ (((fr >> 3) & 1) << 2))] =
            make_uint2(pack2bf(v[0] + bv[j][0], v[1] + bv[j][1]), pack2bf(v[2] + bv[j][2], v[3] + bv[j][3]));
      }
    lgkm_wait0();
    // 8 row steps in groups of EPI_U: a group's global operand loads (residual C, relu source,
    // BN input) are all issued before its first store, so their HBM latency overlaps instead of
    // serialising behind each step's store (the compiler cannot move a load across a store to C).
    constexpr int EPI_U = MODE == 0 ? kG256EpiU0 : kG256EpiUBN;
    constexpr int NG = 8 / EPI_U;
    constexpr int SL = 1;
    uint4 cv[SL][EPI_U], yq[SL][EPI_U], xq[SL][EPI_U];
    size_t offs[SL][EPI_U];
    bool ok[SL][EPI_U];
    auto load_grp = [&](int g, int sl) {
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        const int rl = (g * EPI_U + u) * 8 + (lane >> 3);
        const int m = m0 + wm * WR + mq * 64 + rl;
        ok[sl][u] = m < a.M && n < a.N && mq * 64 + rl < WR;
        size_t row = (size_t)m;
        if constexpr (SCAT) {
          const uint32_t pq = fdiv((uint32_t)m, a.fQ);
          row = (size_t)(2u * pq) * (uint32_t)a.W + 2u * ((uint32_t)m - pq * a.fQ.d);
        }
        offs[sl][u] = ok[sl][u] ? row * a.ldc + n : 0;
        bool acc_ok = true;
        if (BN_EPI && ok[sl][u] && a.aux_even && (a.epi == 3 || a.epi == 5)) {
          const uint32_t img = fdiv((uint32_t)m, a.fPQ), rem = (uint32_t)m - img * a.fPQ.d;
          const uint32_t h = fdiv(rem, a.fQ), w = rem - h * a.fQ.d;
          acc_ok = ((h | w) & 1u) == 0u;
        }
        if (BN_EPI && ok[sl][u] && a.epi >= 4) {
          if (a.epi == 5)
            cv[sl][u] = acc_ok ? epi_ld16<kEpiNtCY>((const bf16_t*)a.C + offs[sl][u]) : make_uint4(0, 0, 0, 0);
          if (a.bn_relu) {
            if (a.mbits)
              yq[sl][u].x = a.mbits[offs[sl][u] >> 3];  // mask byte (offs is a multiple of 8)
            else
              yq[sl][u] = epi_ld16<kEpiNtCY>(a.aux + offs[sl][u]);
          }
          if (a.stats) xq[sl][u] = epi_ld16<kEpiNtX>(a.aux2 + offs[sl][u]);
        } else if (ok[sl][u] && (a.epi == 2 || a.epi == 3)) {
          yq[sl][u] = acc_ok ? epi_ld16<kEpiNtCY>(a.aux + offs[sl][u]) : make_uint4(0, 0, 0, 0);
        }
      }
    };
    auto proc_grp = [&](int g, int sl) {
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        const int rl = (g * EPI_U + u) * 8 + (lane >> 3);
        uint4 v = *(const uint4*)&Ct[rl * CST + cc * 8];
        if ((rl >> 3) & 1) v = make_uint4(v.z, v.w, v.x, v.y);  // undo the write swizzle
        if (!ok[sl][u]) continue;
        const size_t off = offs[sl][u];
        MI_ASSERT(n + 8 <= a.N, n);
        uint4 o = v;
        if (BN_EPI && a.epi >= 4) {
          float f[8];
          unpack8(v, f);
          if (a.epi == 5) {  // dy = this dgrad + the gradient already in C (residual sum)
            float c0[8];
            unpack8(cv[sl][u], c0);
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] += c0[q];
          }
          if (a.bn_relu && a.mbits) {
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
          if (has_stats) {
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
    lgkm_wait0();  // this wave's reads of the slice retire before the next quadrant row overwrites it
  }
  if (has_stats) {
    // reduce over the 8 lanes sharing a column chunk (lane >> 3), lanes 0..7 write the slab row
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s1[q] += __shfl_xor(s1[q], o, 64);
        s2[q] += __shfl_xor(s2[q], o, 64);
      }
    }
    if (lane < 8 && n < a.N) {
      float* row = a.stats + (size_t)(tm * 2 + wm) * 2 * a.N;
      *(float4*)(row + n) = make_float4(s1[0], s1[1], s1[2], s1[3]);
      *(float4*)(row + n + 4) = make_float4(s1[4], s1[5], s1[6], s1[7]);
      *(float4*)(row + a.N + n) = make_float4(s2[0], s2[1], s2[2], s2[3]);
      *(float4*)(row + a.N + n + 4) = make_float4(s2[4], s2[5], s2[6], s2[7]);
    }
  }
}

int rsrc_bytes256(int64_t elems) {
  const int64_t b = elems * 2;
  return (b > 0x7fffffffLL) ? 0 : (int)b;
}

// ----------------------------------------------------------------- TN (weight gradients)
// C[M][N] (fp32) += sum_k A[k][M] B[k][N] over this block's k range (split-K: fp32 atomics).
// Same phase / part / wait schedule as the NT kernel; the parts are k-major images
// [64 k][128 cols] (two 64-col slices, one per wave row / column group) and the MFMA fragments
// are gathered with ds_read_b64_tr_b16 (4 k-rows x 16 cols transposed per 16-lane group).  8-byte
// units of row k are XOR-swizzled by tr_swz(k) (applied on the load side, 16-B granular) so the
// 4 rows of a transposed read and the 4 lane groups hit different banks.
struct G256TNArgs {
  const bf16_t* A;  // [K][lda]
  const bf16_t* B;  // [K][ldb]
  float* C;         // [M][ldc]
  int M, N, K, lda, ldb, ldc;
  int tiles_m, tiles_n, splits, kt_per_split;
  int a_bytes, b_bytes;
  float* ws;  // split-K partial slabs [tiles][splits][256][256] fp32 (nullptr: fp32 atomics into C)
};

__device__ __forceinline__ int tr_swz32(int k) { return (4 * (k & 3) + 16 * ((k >> 3) & 1)) & 31; }

__global__ __launch_bounds__(512, 1) void gemm256_tn_kernel(G256TNArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * 4 * PART_U4];  // 128 KB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;

  const int nblk_tile = a.tiles_m * a.tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / nblk_tile, tb = bid - split * nblk_tile;
  const int group = tb / (GROUP_M * a.tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(a.tiles_m - first_m, GROUP_M);
  const int tm = first_m + (tb % (GROUP_M * a.tiles_n)) % gsz;
  const int tn = (tb % (GROUP_M * a.tiles_n)) / gsz;
  const int m0 = tm * G_BM, n0 = tn * G_BN;
  const int kt0 = split * a.kt_per_split;
  const int nk = min(a.kt_per_split, (a.K + G_BK - 1) / G_BK - kt0);
  if (nk <= 0) return;
  const int kbeg = kt0 * G_BK;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.b_bytes, 0x00020000);

  // load geometry: chunk idx = i*512 + tid -> part row k = idx>>4, LDS chunk c = idx&15 holding
  // global chunk c ^ swz(k): cols (c'>>3)*128 + part*64 + (c'&7)*8 of the block's 256 (A: m, B: n)
  uint32_t a_vo[2][2], b_vo[2][2];
  int klim[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = i * 512 + tid, k = idx >> 4, c = idx & 15;
    const int gc = c ^ (tr_swz32(k) >> 1);
    const int kk = kbeg + k;
    klim[i] = kk < a.K ? min(nk, (a.K - kk + G_BK - 1) / G_BK) : 0;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int col = (gc >> 3) * 128 + part * 64 + (gc & 7) * 8;
      const int ma = m0 + col, nb = n0 + col;
      a_vo[part][i] = ma < a.M ? (uint32_t)(kk * a.lda + ma) * 2u : OOB;
      b_vo[part][i] = nb < a.N ? (uint32_t)(kk * a.ldb + nb) * 2u : OOB;
    }
  }
  const uint32_t a_kstep = (uint32_t)(G_BK * a.lda) * 2u, b_kstep = (uint32_t)(G_BK * a.ldb) * 2u;

  auto issue = [&](int t, int which, int part) {
    uint4* dst = smem + ((t & 1) * 4 + which * 2 + part) * PART_U4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t base = which == 0 ? a_vo[part][i] : b_vo[part][i];
      const uint32_t vo = (t < klim[i] && base != OOB) ? base + (uint32_t)t * (which == 0 ? a_kstep : b_kstep) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(which == 0 ? rsA : rsB, LDS_PTR(void, dst + i * 512 + wid * 64), 16, vo,
                                               0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bx[2][2], by[2][2];
  // transposed fragment: cols base..base+15 (lane col li), k rows kk*32 + 8g + {0..7}
  auto tr_frag = [&](const uint4* part_img, int colbase, int kk) {
    const uint2* img = (const uint2*)part_img;  // [64 k][32 units of 8 B]
    const int u = colbase / 4 + p4;
    const int k1 = kk * 32 + 8 * g + q4, k2 = k1 + 4;
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &img[k1 * 32 + (u ^ tr_swz32(k1))]));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, &img[k2 * 32 + (u ^ tr_swz32(k2))]));
    short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v8);
  };
  auto read_a = [&](bf16x8 (&f)[4][2], int t, int mq) {
    const uint4* src = smem + ((t & 1) * 4 + mq) * PART_U4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f[i][kk] = tr_frag(src, wm * 64 + i * 16, kk);
  };
  auto read_b = [&](bf16x8 (&f)[2][2], int t, int nq) {
    const uint4* src = smem + ((t & 1) * 4 + 2 + nq) * PART_U4;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f[j][kk] = tr_frag(src, (wn >> 1) * 64 + (wn & 1) * 32 + j * 16, kk);
  };
  auto mma = [&](const bf16x8 (&af_)[4][2], const bf16x8 (&bf)[2][2], int mq, int nq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af_[i][kk], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
  };
  auto ktile = [&](int t, bf16x8 (&bc)[2][2], bf16x8 (&bn)[2][2]) {
    issue(t + 1, 1, 0);
    read_b(bn, t, 1);
    mma(af, bc, 0, 0);
    vm_wait6();
    phase_barrier();
    issue(t + 1, 0, 1);
    mma(af, bn, 0, 1);
    read_a(af, t, 1);
    issue(t + 2, 0, 0);
    mma(af, bn, 1, 1);
    vm_wait4();
    phase_barrier();
    issue(t + 2, 1, 1);
    const bool more = t + 1 < nk;
    if (more) read_b(bn, t + 1, 0);
    mma(af, bc, 1, 0);
    if (more) read_a(af, t + 1, 0);
  };

  issue(0, 0, 0); issue(0, 1, 1); issue(0, 1, 0); issue(0, 0, 1); issue(1, 0, 0); issue(1, 1, 1);
  vm_wait6();
  phase_barrier();
  read_a(af, 0, 0);
  read_b(bx, 0, 0);
  static_prio();
  for (int t = 0; t < nk; t += 2) {
    ktile(t, bx, by);
    if (t + 1 < nk) ktile(t + 1, by, bx);
  }
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // lane holds D[n = 16j + 4g + r][m = 16i + li]: C[m][n..n+3]
  // B part nq holds, for wave column wn, cols (wn>>1)*128 + nq*64 + (wn&1)*32 + j*16 of the tile
  if (a.splits > 1 && a.ws) {
    // this split's partial tile, row-major inside the tile; g256_tn_reduce_kernel sums the splits
    // into C in split order (deterministic, no fp32 atomics)
    float* slab = a.ws + ((size_t)(tm * a.tiles_n + tn) * a.splits + split) * (G_BM * G_BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = wm * 128 + i * 16 + li;
        const int nl = (wn >> 1) * 128 + (j >> 1) * 64 + (wn & 1) * 32 + (j & 1) * 16 + 4 * g;
        *(f32x4*)(slab + ml * G_BN + nl) = acc[i][j];
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + li;
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nq = j >> 1, jj = j & 1;
      const int n = n0 + (wn >> 1) * 128 + nq * 64 + (wn & 1) * 32 + jj * 16 + 4 * g;
      if (n >= a.N) continue;
      float* dst = a.C + (size_t)m * a.ldc + n;
      const f32x4 v = acc[i][j];
      if (a.splits > 1) {
        atomicAdd(dst, v[0]); atomicAdd(dst + 1, v[1]); atomicAdd(dst + 2, v[2]); atomicAdd(dst + 3, v[3]);
      } else {
        const float4 o = *(float4*)dst;
        *(float4*)dst = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
      }
    }
  }
}


// C[M][N] += sum over splits of the gemm256_tn partial slabs: one thread per 4 columns of a tile
// row, the splits summed in order (4 loads in flight)
__global__ __launch_bounds__(256) void g256_tn_reduce_kernel(const float* __restrict__ ws, float* __restrict__ C,
                                                             int M, int N, int ldc, int tiles_n, int splits) {
  const int tile = blockIdx.y;
  const int pos = blockIdx.x * 256 + threadIdx.x;  // f32x4 index inside the 256 x 256 tile
  const int ml = pos >> 6, nl = (pos & 63) * 4;
  const int m = (tile / tiles_n) * G_BM + ml, n = (tile % tiles_n) * G_BN + nl;
  if (m >= M || n >= N) return;
  const f32x4* src = (const f32x4*)(ws + (size_t)tile * splits * (G_BM * G_BN)) + pos;
  constexpr int TS = G_BM * G_BN / 4;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  int z = 0;
  for (; z + 4 <= splits; z += 4) {
    const f32x4 a0 = src[(size_t)z * TS], a1 = src[(size_t)(z + 1) * TS];
    const f32x4 a2 = src[(size_t)(z + 2) * TS], a3 = src[(size_t)(z + 3) * TS];
    s += a0; s += a1; s += a2; s += a3;
  }
  for (; z < splits; ++z) s += src[(size_t)z * TS];
  float* dst = C + (size_t)m * ldc + n;  // N % 8 == 0: the 4 columns are all in range
  const float4 o = *(const float4*)dst;
  *(float4*)dst = make_float4(o.x + s[0], o.y + s[1], o.z + s[2], o.w + s[3]);
}

}  // namespace

extern "C" float* mi_partials_workspace(size_t floats, hipStream_t st);  // gemm_conv.hip

// Tail split-K planning: with 1 block per CU, a grid of `tiles` runs in ceil(tiles / CUs) waves;
// when the last wave is at most 3/4 full its tiles are split along K so it fills the chip.
// Per (device, stream) -- the forward / data-gradient convs of a projection shortcut run on an
// auxiliary stream concurrently with the main chain (ops/resblock.py), so two streams must not
// share the partials or the arrival counters.  A stream beyond the table takes over a slot
// round-robin after a device synchronisation (never inside a graph capture: the capture's warm-up
// on the same stream claimed its slot), so the split -- and the numerics -- never depend on
// which streams ran before.
struct TailWs {
  hipStream_t st = nullptr;
  bool used = false;
  float* ws = nullptr;
  size_t ws_floats = 0;
  int* cnt = nullptr;
  int cnt_n = 0;
};
constexpr int TAIL_WS_STREAMS = 4;
static TailWs g_tail_ws[16][TAIL_WS_STREAMS];
static std::mutex g_tail_mu;
static int g_num_cus = 0;
static int g_tail_split_env = -1;
static int g_tail_min_kt = 12;


static void plan_defaults() {
  int dev = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
    g_num_cus = 256;
  const char* e = std::getenv("MI355X_DP_TAIL_SPLIT");
  g_tail_split_env = (e && e[0] == '0') ? 0 : 1;
  if (const char* m = std::getenv("MI355X_DP_TAIL_MIN_KT")) g_tail_min_kt = std::max(1, std::atoi(m));
}

MI_API int mi_set_tail_split(int on) {
  if (g_num_cus == 0) plan_defaults();
  g_tail_split_env = on ? 1 : 0;
  return 0;
}

static hipError_t plan_tail(G256Args& a, int nk, hipStream_t st) {
  if (g_num_cus == 0) plan_defaults();
  const int tiles = a.tiles_m * a.tiles_n;
  const int full = (tiles / g_num_cus) * g_num_cus, tail = tiles - full;
  int split = 1;
  if (g_tail_split_env && tail > 0 && tail * 4 <= g_num_cus * 3) {
    split = std::min(4, g_num_cus / tail);
    // a split pays ~2 x 256 KB of fp32 partial traffic per tail tile: only worth it when every
    // split still runs >= g_tail_min_kt k-tiles (ViT K=768 GEMMs measured slower when split)
    while (split > 1 && nk / split < g_tail_min_kt) --split;
  }
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_tail_mu);
  TailWs* wp = nullptr;
  if (split > 1) {
    for (auto& e : g_tail_ws[dev & 15])
      if (e.used && e.st == st) { wp = &e; break; }
    if (!wp)
      for (auto& e : g_tail_ws[dev & 15])
        if (!e.used) { e.used = true; e.st = st; wp = &e; break; }
    // table full: no tail split for this stream (a valid schedule that needs no workspace; never a
    // host-blocking takeover of another stream's slot, which would abort a graph capture)
    if (!wp) split = 1;
  }
  const size_t need = (size_t)tail * split * G_BM * G_BN;
  // growth inside a graph capture: no allocation there -- the unsplit schedule (common.h)
  if (split > 1 && (wp->ws_floats < need || wp->cnt_n < tail) && mi_stream_capturing(st)) {
    mi_ws_capture_warn("gemm256 tail split-K");
    split = 1;
  }
  a.full_blocks = split > 1 ? full : tiles;
  a.tail_split = split;
  if (split <= 1) return hipSuccess;
  TailWs& w = *wp;
  // a grown buffer retires the old one (graphs captured earlier may still replay into it)
  if (w.ws_floats < need) {
    float* p = nullptr;
    hipError_t e = hipMalloc(&p, need * sizeof(float));
    if (e != hipSuccess) return e;
    mi_ws_retire(w.ws);
    w.ws = p;
    w.ws_floats = need;
  }
  if (w.cnt_n < tail) {
    int* p = nullptr;
    hipError_t e = hipMalloc(&p, sizeof(int) * tail);
    if (e != hipSuccess) return e;
    hipMemset(p, 0, sizeof(int) * tail);
    hipDeviceSynchronize();
    mi_ws_retire(w.cnt);
    w.cnt = p;
    w.cnt_n = tail;
  }
  a.ws = w.ws;
  a.counters = w.cnt;
  return hipSuccess;
}

// Row tile of the NT kernel: 224 rows (WR 112) when its wave quantization beats 256 rows by >= 3 %
// -- e.g. M = 50,176 (ResNet layer 3, batch 256): 196 tiles of 256 rows leave 60 of 256 CUs idle,
// 224 tiles of 224 rows finish in 7/8 of the time (ResNet-50 +0.9 %, ResNet-152 +1.5 % same box,
// profiles/g256_bm224_r6.md).  Cost model: rounds of the grid after plan_tail's split decision x the
// tile height.  Auto applies to the conv modes only: on ViT-B/16 (its N = K = 768 GEMMs would take
// 224 rows) it measured -0.5 %.  MI355X_DP_G256_BM224 (mi_set_g256_bm224): 0 never, 1 auto (default),
// 2 always (plain GEMMs included).
static int g_bm224 = -1;

MI_API int mi_set_g256_bm224(int mode) {
  g_bm224 = mode < 0 ? 0 : (mode > 2 ? 2 : mode);
  return 0;
}

static double g256_cost(int M, int N, int nk, int bm) {
  const int tiles = cdiv(M, bm) * cdiv(N, G_BN);
  const int full = (tiles / g_num_cus) * g_num_cus, tail = tiles - full;
  double rounds = (double)(full / g_num_cus);
  if (tail > 0) {
    int split = 1;
    if (g_tail_split_env && tail * 4 <= g_num_cus * 3) {
      split = std::min(4, g_num_cus / tail);
      while (split > 1 && nk / split < g_tail_min_kt) --split;
    }
    rounds += 1.0 / split;
  }
  return rounds * bm;
}

static int g256_wr(int M, int N, int K, bool conv) {
  if (g_num_cus == 0) plan_defaults();
  if (g_bm224 < 0) {
    const char* e = std::getenv("MI355X_DP_G256_BM224");
    g_bm224 = e ? std::max(0, std::min(2, std::atoi(e))) : 1;
  }
  if (g_bm224 == 0 || (g_bm224 == 1 && !conv)) return 128;
  if (g_bm224 == 2) return 112;
  const int nk = cdiv(K, G_BK);
  return g256_cost(M, N, nk, 224) < 0.97 * g256_cost(M, N, nk, 256) ? 112 : 128;
}

// statistics slab rows of the conv kernel (mode 1 / 2) for an M x N x K conv: 2 per row tile
MI_API int mi_g256_stat_rows(int M, int N, int K) { return 2 * cdiv(M, 2 * g256_wr(M, N, K, true)); }

static int grid_of(const G256Args& a) {
  const int tiles = a.tiles_m * a.tiles_n;
  return a.tail_split > 1 ? a.full_blocks + (tiles - a.full_blocks) * a.tail_split : tiles;
}

// test hook (tests/test_graph_workspaces_gpu.py): grow this stream's tail split-K workspace
MI_API int mi_g256_tail_ws_reserve(size_t floats, int tail, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_tail_mu);
  TailWs* wp = nullptr;
  for (auto& e : g_tail_ws[dev & 15])
    if (e.used && e.st == st) { wp = &e; break; }
  if (!wp) return 1;
  if (wp->ws_floats < floats) {
    float* p = nullptr;
    if (hipMalloc(&p, floats * sizeof(float)) != hipSuccess) return 2;
    mi_ws_retire(wp->ws);
    wp->ws = p;
    wp->ws_floats = floats;
  }
  if (wp->cnt_n < tail) {
    int* p = nullptr;
    if (hipMalloc(&p, sizeof(int) * tail) != hipSuccess) return 2;
    hipMemset(p, 0, sizeof(int) * tail);
    hipDeviceSynchronize();
    mi_ws_retire(wp->cnt);
    wp->cnt = p;
    wp->cnt_n = tail;
  }
  return 0;
}

// Returns hipErrorInvalidValue when the shape is outside this kernel's contract (caller falls
// back to the 128x128 kernel).
MI_API int mi_gemm256p_nt(const void* A, const void* B, void* C, const float* bias, void* aux, int epi, int M, int N,
                          int K, int lda, int ldb, int ldc, hipStream_t st);  // gemm256p.hip

MI_API int mi_gemm256_nt(const void* A, const void* B, void* C, const float* bias, void* aux, int epi, int M, int N,
                         int K, int lda, int ldb, int ldc, int out_f32, int accumulate, hipStream_t st) {
  // bf16 out, no accumulation, plain / GELU epilogue: the persistent kernel (epilogue overlapped
  // with the next tile's main loop); it declines shapes outside its contract
  if (!out_f32 && !accumulate && (epi == 0 || epi == 1) &&
      mi_gemm256p_nt(A, B, C, bias, aux, epi, M, N, K, lda, ldb, ldc, st) == (int)hipSuccess)
    return (int)hipSuccess;
  if (K % 8 != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || (epi && (out_f32 || !aux)) || M <= 0 || N <= 0)
    return (int)hipErrorInvalidValue;
  G256Args a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = bias; a.aux = (bf16_t*)aux; a.epi = epi;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.out_f32 = out_f32; a.accumulate = accumulate;
  const int wr = g256_wr(M, N, K, false);
  a.tiles_m = cdiv(M, 2 * wr); a.tiles_n = cdiv(N, G_BN);
  a.a_bytes = rsrc_bytes256((int64_t)M * lda);
  a.b_bytes = rsrc_bytes256((int64_t)N * ldb);
  if (!a.a_bytes || !a.b_bytes) return (int)hipErrorInvalidValue;
  if (hipError_t e = plan_tail(a, cdiv(K, G_BK), st); e != hipSuccess) return (int)e;
  if (wr == 112) hipLaunchKernelGGL((gemm256_nt_kernel<0, 112>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm256_nt_kernel<0, 128>), dim3(grid_of(a)), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// Stride-2 1x1 data gradient into the even pixels: C rows 2 (m / Q) W + 2 (m % Q) (ldc = N) get
// A[m][K] . B[N][K]^T, bf16; the odd pixels are not written (their consumer reads the even ones only,
// gemm_conv.hip aux_even).  A = dy [Nb*P*Q][K], B = the transposed 1x1 weight [N = C][K].
MI_API int mi_gemm256_nt_scat2(const void* A, const void* B, void* C, int M, int N, int K, int Q, int W,
                               hipStream_t st) {
  if (K % 8 != 0 || N % 8 != 0 || M <= 0 || N <= 0 || Q <= 0 || W < 2 * Q) return (int)hipErrorInvalidValue;
  G256Args a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = nullptr; a.aux = nullptr; a.epi = 0;
  a.M = M; a.N = N; a.K = K; a.lda = K; a.ldb = K; a.ldc = N;
  a.W = W; a.fQ = make_fastdiv((uint32_t)Q);
  const int wr = g256_wr(M, N, K, true);
  a.tiles_m = cdiv(M, 2 * wr); a.tiles_n = cdiv(N, G_BN);
  a.a_bytes = rsrc_bytes256((int64_t)M * K);
  a.b_bytes = rsrc_bytes256((int64_t)N * K);
  if (!a.a_bytes || !a.b_bytes) return (int)hipErrorInvalidValue;
  if (hipError_t e = plan_tail(a, cdiv(K, G_BK), st); e != hipSuccess) return (int)e;
  if (wr == 112) hipLaunchKernelGGL((gemm256_nt_kernel<0, 112, true>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm256_nt_kernel<0, 128, true>), dim3(grid_of(a)), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// C[M][N] (fp32) += A[K][M]^T B[K][N]; split-K chosen to fill the chip.
MI_API int mi_gemm256_tn(const void* A, const void* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                         hipStream_t st) {
  if (M % 8 != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || M <= 0 || N <= 0 || K <= 0)
    return (int)hipErrorInvalidValue;
  G256TNArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.tiles_m = cdiv(M, G_BM); a.tiles_n = cdiv(N, G_BN);
  const int tiles = a.tiles_m * a.tiles_n, nkt = cdiv(K, G_BK);
  // at most one wave of blocks (1 block per CU), >= 8 k-tiles per split
  if (g_num_cus == 0) plan_defaults();
  int splits = max(1, min(g_num_cus / tiles, nkt / 8));
  a.kt_per_split = cdiv(nkt, splits);
  a.splits = cdiv(nkt, a.kt_per_split);
  a.a_bytes = rsrc_bytes256((int64_t)K * lda);
  a.b_bytes = rsrc_bytes256((int64_t)K * ldb);
  if (!a.a_bytes || !a.b_bytes) return (int)hipErrorInvalidValue;
  // split-K partials through slabs + one reduce launch (fp32 atomics, the fallback when no workspace
  // can be had -- e.g. growth inside a graph capture -- cost ~37 us per ViT-B/16 weight gradient)
  a.ws = a.splits > 1 ? mi_partials_workspace((size_t)tiles * a.splits * G_BM * G_BN, st) : nullptr;
  hipLaunchKernelGGL(gemm256_tn_kernel, dim3(tiles * a.splits), dim3(512), 0, st, a);
  if (a.ws)
    hipLaunchKernelGGL(g256_tn_reduce_kernel, dim3(G_BM * G_BN / 4 / 256, tiles), dim3(256), 0, st, (const float*)a.ws,
                       C, M, N, ldc, a.tiles_n, a.splits);
  return (int)hipGetLastError();
}

// Implicit-GEMM convolution on the 256x256 pipeline.  mode 1 = forward: gathered = x [Nb,H,W,Cs],
// rows = output pixels [Nb,P,Q], B = w [N][R][S][Cs]; mode 2 = stride-1 data gradient:
// gathered = dy [Nb,H,W,Cs] (H,W = the forward output grid, Cs = forward K), rows = dx pixels
// [Nb,P,Q], B = wt [N][R][S][Cs].  Cs % 64 == 0.  stats: [mi_g256_stat_rows(M, N, K)][2][N] partials
// (forward: sum / sum of squares; epi 4: BN-backward sums).  C bf16 [M][N].
MI_API int mi_gemm256_conv2(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                            const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs, int P,
                            int Q, int R, int S, int stride, int pad, int N, int aux_even, hipStream_t st);

MI_API int mi_gemm256_conv(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                           const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs, int P,
                           int Q, int R, int S, int stride, int pad, int N, hipStream_t st) {
  return mi_gemm256_conv2(mode, A, B, C, stats, epi, aux, aux2, mean, bn_relu, Nb, H, W, Cs, P, Q, R, S, stride, pad,
                          N, 0, st);
}

MI_API int mi_gemm256_conv3(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                            const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs, int P,
                            int Q, int R, int S, int stride, int pad, int N, int aux_even, const void* mbits,
                            hipStream_t st);

// as mi_gemm256_conv; aux_even: see G256Args
MI_API int mi_gemm256_conv2(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                            const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs, int P,
                            int Q, int R, int S, int stride, int pad, int N, int aux_even, hipStream_t st) {
  return mi_gemm256_conv3(mode, A, B, C, stats, epi, aux, aux2, mean, bn_relu, Nb, H, W, Cs, P, Q, R, S, stride, pad,
                          N, aux_even, nullptr, st);
}

// as mi_gemm256_conv2; mbits: the epi 4 / 5 ReLU mask as bytes (see G256Args)
MI_API int mi_gemm256_conv3(int mode, const void* A, const void* B, void* C, float* stats, int epi, void* aux,
                            const void* aux2, const float* mean, int bn_relu, int Nb, int H, int W, int Cs, int P,
                            int Q, int R, int S, int stride, int pad, int N, int aux_even, const void* mbits,
                            hipStream_t st) {
  if ((mode != 1 && mode != 2) || Cs % 64 != 0 || N % 8 != 0 || (mode == 2 && stride != 1) ||
      !(epi == 0 || epi == 3 || epi == 4 || epi == 5) || (epi == 3 && !aux) ||
      (epi >= 4 && bn_relu && !aux && !mbits) || (mbits && (epi < 4 || !bn_relu)) ||
      (epi >= 4 && stats && (!aux2 || !mean)))
    return (int)hipErrorInvalidValue;
  G256Args a{};
  a.mbits = (const uint8_t*)mbits;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.bias = nullptr;
  a.aux = (bf16_t*)aux; a.aux2 = (const bf16_t*)aux2; a.mean = mean; a.bn_relu = bn_relu; a.epi = epi;
  a.stats = stats;
  a.aux_even = aux_even;
  a.M = Nb * P * Q; a.N = N; a.K = R * S * Cs; a.lda = 0; a.ldb = a.K; a.ldc = N;
  a.out_f32 = 0; a.accumulate = 0;
  a.H = H; a.W = W; a.Cs = Cs; a.S = S; a.stride = stride; a.pad = pad;
  a.fPQ = make_fastdiv((uint32_t)(P * Q)); a.fQ = make_fastdiv((uint32_t)Q);
  a.fS = make_fastdiv((uint32_t)S); a.fCpt = make_fastdiv((uint32_t)(Cs / 64));
  const int wr = g256_wr(a.M, N, a.K, true);
  a.tiles_m = cdiv(a.M, 2 * wr); a.tiles_n = cdiv(N, G_BN);
  a.a_bytes = rsrc_bytes256((int64_t)Nb * H * W * Cs);
  a.b_bytes = rsrc_bytes256((int64_t)N * a.K);
  if (!a.a_bytes || !a.b_bytes) return (int)hipErrorInvalidValue;
  if (hipError_t e = plan_tail(a, cdiv(a.K, G_BK), st); e != hipSuccess) return (int)e;
  if (const char* t = std::getenv("MI355X_DP_TRACE_GEMM"); t && t[0] == '1')
    fprintf(stderr, "[gemm] g256conv mode=%d M=%d N=%d K=%d Cs=%d R=%d s=%d epi=%d stats=%d blocks=%d bm=%d\n", mode,
            a.M, a.N, a.K, Cs, R, stride, epi, stats != nullptr, grid_of(a), 2 * wr);
  if (mode == 1 && wr == 112)
    hipLaunchKernelGGL((gemm256_nt_kernel<1, 112>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else if (mode == 1)
    hipLaunchKernelGGL((gemm256_nt_kernel<1, 128>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else if (wr == 112)
    hipLaunchKernelGGL((gemm256_nt_kernel<2, 112>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((gemm256_nt_kernel<2, 128>), dim3(grid_of(a)), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

// ---- folded BatchNorm backward on the 256-wide data-gradient kernel (ops/resblock.py _Fold; the
// conv_panel.hip mi_panel_dgrad_fbb twin for convs too deep for the panel): the 1x1 / stride-1 data
// gradient of a BN input gradient k0 dz + k1 c + k2 as ONE GEMM over [dz | c] (2K deep) against
// wq = [diag(k0) W | diag(k1) W] (bf16 [C][2K], written here) plus the bias k2 W (fp32 [C]).
__global__ __launch_bounds__(256) void fbb_wprep_kernel(const bf16_t* __restrict__ wt, const float* __restrict__ coef,
                                                        bf16_t* __restrict__ wq, float* __restrict__ bias, int K) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float b = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float w = bf2f(wt[(size_t)c * K + k]);
    wq[(size_t)c * 2 * K + k] = f2bf(w * coef[k]);
    wq[(size_t)c * 2 * K + K + k] = f2bf(w * coef[K + k]);
    b = fmaf(w, coef[2 * K + k], b);
  }
  red[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bias[c] = red[0];
}

// dz / c NHWC [Nb,H,W,K], wt bf16 [C][K] (the dgrad weight layout), wq: C * 2K bf16 and bias: C
// floats of workspace; epilogue / statistics as mi_gemm256_conv3 mode 2 (stats rows:
// mi_g256_stat_rows(M, C, 2K)).
MI_API int mi_gemm256_dgrad_fbb(const void* dz, const void* c, const float* coef, const void* wt, void* wq, float* bias,
                                void* dx, float* stats, int epi, void* aux, const void* aux2, const float* mean,
                                int bn_relu, int Nb, int H, int W, int C, int K, int aux_even, const void* mbits,
                                hipStream_t st) {
  if (K % 64 != 0 || C % 8 != 0 || !coef || !wq || !bias || !(epi == 0 || epi == 3 || epi == 4 || epi == 5) ||
      (epi == 3 && !aux) || (epi >= 4 && bn_relu && !aux && !mbits) || (mbits && (epi < 4 || !bn_relu)) ||
      (epi >= 4 && stats && (!aux2 || !mean)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fbb_wprep_kernel, dim3(C), dim3(256), 0, st, (const bf16_t*)wt, coef, (bf16_t*)wq, bias, K);
  G256Args a{};
  a.mbits = (const uint8_t*)mbits;
  a.A = (const bf16_t*)dz; a.A2 = (const bf16_t*)c; a.B = (const bf16_t*)wq; a.C = dx; a.bias = bias;
  a.aux = (bf16_t*)aux; a.aux2 = (const bf16_t*)aux2; a.mean = mean; a.bn_relu = bn_relu; a.epi = epi;
  a.stats = stats;
  a.aux_even = aux_even;
  a.M = Nb * H * W; a.N = C; a.K = 2 * K; a.lda = 0; a.ldb = 2 * K; a.ldc = C;
  a.out_f32 = 0; a.accumulate = 0;
  a.H = H; a.W = W; a.Cs = K; a.S = 1; a.stride = 1; a.pad = 0;
  a.khalf_kt = K / 64;
  a.fPQ = make_fastdiv((uint32_t)(H * W)); a.fQ = make_fastdiv((uint32_t)W);
  a.fS = make_fastdiv(1u); a.fCpt = make_fastdiv((uint32_t)(K / 64));
  const int wr = g256_wr(a.M, C, a.K, true);
  a.tiles_m = cdiv(a.M, 2 * wr); a.tiles_n = cdiv(C, G_BN);
  a.a_bytes = a.a2_bytes = rsrc_bytes256((int64_t)a.M * K);
  a.b_bytes = rsrc_bytes256((int64_t)C * a.K);
  if (!a.a_bytes || !a.b_bytes) return (int)hipErrorInvalidValue;
  if (hipError_t e = plan_tail(a, cdiv(a.K, G_BK), st); e != hipSuccess) return (int)e;
  if (const char* t = std::getenv("MI355X_DP_TRACE_GEMM"); t && t[0] == '1')
    fprintf(stderr, "[gemm] g256dgrad-fbb M=%d N=%d K=%d epi=%d stats=%d blocks=%d bm=%d\n", a.M, C, a.K, epi,
            stats != nullptr, grid_of(a), 2 * wr);
  if (wr == 112) hipLaunchKernelGGL((gemm256_nt_kernel<2, 112>), dim3(grid_of(a)), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm256_nt_kernel<2, 128>), dim3(grid_of(a)), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}
