// Persistent 256x256 NT GEMM for gfx950 with the epilogue overlapped with the next tile's main
// loop: C[M][N] (bf16) = A[M][K] · B[N][K]^T (+bias) (EPI 1: GELU, pre-activation kept in aux).
// The ViT-B/16 projections / MLP (M = 50,432 tokens, K = 768 / 3,072) are the target.
//
// Why: gemm256.hip's non-persistent kernel (one 256x256 tile per block, 1 block per CU for its
// 128 KB of LDS) spends about a third of a K = 768 tile's main-loop time storing the 128 KB bf16
// tile after the loop with nothing to overlap -- every CU's blocks reach that store phase together
// -- and every block pays a prologue bubble before its first MFMA.  Here one block per CU walks its
// tiles and the k-steps of consecutive tiles form ONE continuous pipeline:
//
//  * the loop runs over the block's global k-step sequence g = (tile li, k-tile t); a part load for
//    k-step g+1 / g+2 addresses whichever tile that k-step belongs to (per-tile buffer resources:
//    base = the tile's first row, range = the rows left, so rows past M / N zero-fill), so the next
//    tile's first k-tiles stream in under the current tile's last MFMAs -- no prologue bubble, no
//    pipeline drain between tiles;
//  * the previous tile's accumulators are stored from registers in the first k-step of the next
//    tile, one output quadrant per phase, right before the phase whose MFMAs first reuse that
//    quadrant's registers (phase order (0,0) (0,1) (1,1) (1,0)), so the stores overlap the MFMAs of
//    the other wave on the SIMD; the 16x16 MFMA fragments are widened to 16-byte rows with
//    v_permlane16_swap (lane groups 0/1 and 2/3 exchange their 4-column halves), giving 4 dwordx4
//    stores per quadrant per wave, each 16 rows x 64 contiguous bytes;
//  * gfx950 counts stores and loads in ONE in-order vmcnt, so the counted waits of the first two
//    k-steps of each tile add the stores (and the bias loads) issued after their target part
//    (derivation at `ktile`);
//  * bias: the whole vector staged in LDS at kernel start (before any LDS-DMA load, so plain loads
//    cost no pipeline drain), read by the flush -- no registers held across the tile.
//
// Main loop per k-tile (4 phases, 2 raw barriers, part loads 3-6 phases ahead, XOR-swizzled
// lane-linear LDS images, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 of 16x16x32 MFMAs): as
// gemm256.hip's kernel, see its header.  Requires >= 3 k-tiles (K > 128); shorter K, fp32 output,
// accumulation and the aux-reading epilogues stay on gemm256.hip.
#include "common.h"
#include "epilogue.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int P_BM = 256, P_BN = 256, P_BK = 64;
constexpr int P_PART_U4 = 128 * 8;  // 16 KB
constexpr int P_GROUP_M = 8;
constexpr uint32_t P_OOB = 0xFFFFFFF0u;
constexpr int P_BIAS_MAX = 8192;  // bias columns staged in LDS (32 KB: all the LDS left beside the parts)

struct G256PArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  const float* bias;
  bf16_t* aux;  // EPI 1: the pre-activation
  int M, N, K, lda, ldb, ldc;
  int tiles_m, tiles_n, ntiles, nk;
};

__device__ __forceinline__ void p_barrier() { asm volatile("s_barrier" ::: "memory"); }
#define P_VMWAIT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

__device__ __forceinline__ void tile_coords(const G256PArgs& a, int lin, int& m0, int& n0) {
  const int group = lin / (P_GROUP_M * a.tiles_n);
  const int first_m = group * P_GROUP_M;
  const int gsz = min(a.tiles_m - first_m, P_GROUP_M);
  const int r = lin % (P_GROUP_M * a.tiles_n);
  m0 = (first_m + r % gsz) * P_BM;
  n0 = (r / gsz) * P_BN;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const bf16_t* base, int row0, int rows, int ld) {
  const int64_t left = (int64_t)max(rows - row0, 0) * ld * 2;
  const int bytes = (int)min((int64_t)0x7fffffff, left);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * ld), (short)0, bytes, 0x00020000);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm256p_nt_kernel(G256PArgs a) {
  // ONE LDS array (a second __shared__ object can make hipcc drain vmcnt before every ds_read):
  // 128 KB of operand parts, then the whole bias vector (N <= P_BIAS_MAX floats, 32 KB)
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * 4 * P_PART_U4 + P_BIAS_MAX / 4];
  float* bias_lds = (float*)(smem + 2 * 4 * P_PART_U4);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int idx = xcd_remap(blockIdx.x, G);  // XCD-contiguous runs of tiles per round
  const int ntl = (a.ntiles - idx + G - 1) / G;  // this block's tiles: idx, idx + G, ...
  const int nk = a.nk;
  const int total = ntl * nk;

  // per-thread load geometry (tile-independent): 2 chunks per part, LDS row p = (i*512+tid)/8
  uint32_t a_thr[2][2], b_thr[2][2];
  int klim[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = i * 512 + tid, p = id >> 3, c = id & 7;
    const int gk = (c ^ (p & 7)) * 8;  // source-side swizzle: LDS chunk c of row p holds chunk c^(p&7)
    klim[i] = gk < a.K ? (a.K - gk + P_BK - 1) / P_BK : 0;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      a_thr[part][i] = (uint32_t)(((p >> 6) * 128 + part * 64 + (p & 63)) * a.lda + gk) * 2u;
      b_thr[part][i] = (uint32_t)(((p >> 5) * 64 + part * 32 + (p & 31)) * a.ldb + gk) * 2u;
    }
  }

  // buffer resources of the current and the next tile (wave-uniform)
  int m0c, n0c, m0n = 0, n0n = 0;
  tile_coords(a, idx, m0c, n0c);
  __amdgpu_buffer_rsrc_t rsA_c = rows_rsrc(a.A, m0c, a.M, a.lda), rsB_c = rows_rsrc(a.B, n0c, a.N, a.ldb);
  __amdgpu_buffer_rsrc_t rsA_n = rsA_c, rsB_n = rsB_c;
  if (ntl > 1) {
    tile_coords(a, idx + G, m0n, n0n);
    rsA_n = rows_rsrc(a.A, m0n, a.M, a.lda);
    rsB_n = rows_rsrc(a.B, n0n, a.N, a.ldb);
  }

  // issue part `part` of operand `which` for global k-step gg, which is k-tile tt of the current
  // (nxt = false) or the next tile; past the block's last k-step: zero-fill dummies (counts hold)
  auto issue = [&](int gg, int tt, bool nxt, int which, int part) {
    uint4* dst = smem + ((gg & 1) * 4 + which * 2 + part) * P_PART_U4;
    const bool live = gg < total;
    const uint32_t kb = (uint32_t)tt * (P_BK * 2);
    const __amdgpu_buffer_rsrc_t rs = which == 0 ? (nxt ? rsA_n : rsA_c) : (nxt ? rsB_n : rsB_c);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t vo = (live && tt < klim[i]) ? (which == 0 ? a_thr[part][i] : b_thr[part][i]) + kb : P_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, dst + i * 512 + wid * 64), 16, vo, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias: staged in LDS once, before any LDS-DMA load is in flight (plain loads, then ds_write);
  // the flush reads the lane's columns 16 j + 4 fq + [0, 4) with ds_read_b128
  const bool has_bias = a.bias != nullptr;
  if (has_bias) {
    for (int c = tid * 4; c < a.N; c += 512 * 4) *(float4*)(bias_lds + c) = *(const float4*)(a.bias + c);
    __syncthreads();
  }

  bf16x8 af[4][2], bx[2][2], by[2][2];
  auto read_a = [&](bf16x8 (&f)[4][2], int gg, int mq) {
    const uint4* src = smem + ((gg & 1) * 4 + mq) * P_PART_U4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        f[i][kk] = __builtin_bit_cast(bf16x8, src[(wm * 64 + i * 16 + fr) * 8 + ((kk * 4 + fq) ^ (fr & 7))]);
  };
  auto read_b = [&](bf16x8 (&f)[2][2], int gg, int nq) {
    const uint4* src = smem + ((gg & 1) * 4 + 2 + nq) * P_PART_U4;
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
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af_[i][kk], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
  };

  // Store quadrant (mq, nq) of the tile at (pm0, pn0) from the accumulators (+ bias), then zero
  // it.  Lane (fr, fq) holds D[n = 16 j + 4 fq + r][m = 16 i + fr] of each 16x16 fragment; after
  // the permlane16 swap of fragment pair (2nq, 2nq+1) it holds row 16 i + fr, columns
  // 32 nq + 16 (fq & 1) + 8 (fq >> 1) + [0, 8) of the wave tile: one 16-byte store per fragment row.
  // C through a buffer resource: every lane of every wave issues its stores (rows past M and chunks
  // past N get an out-of-range offset and are dropped), so the per-wave store counts the waits
  // below rely on never depend on the tile's edge
  const int c_bytes = (int)min((int64_t)0x7fffffff, (int64_t)a.M * a.ldc * 2);
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)a.C, (short)0, c_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc((void*)(EPI == 1 ? a.aux : a.C), (short)0, c_bytes, 0x00020000);
  auto flush = [&](int mq, int nq, int pm0, int pn0) __attribute__((always_inline)) {
    const int col = pn0 + wn * 64 + nq * 32 + 16 * (fq & 1) + 8 * (fq >> 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4& v0 = acc[mq * 4 + i][nq * 2];
      f32x4& v1 = acc[mq * 4 + i][nq * 2 + 1];
      f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
      if (has_bias) {
        // the two fragments' 4-column groups; a group past N is never stored (N % 8 == 0), its read
        // is only kept inside the staged vector
        const int nb0 = pn0 + wn * 64 + nq * 32 + 4 * fq, nb1 = nb0 + 16;
        b0 = *(const f32x4*)(bias_lds + (nb0 < a.N ? nb0 : a.N - 4));
        b1 = *(const f32x4*)(bias_lds + (nb1 < a.N ? nb1 : a.N - 4));
      }
      const uint32_t p0 = pack2bf(v0[0] + b0[0], v0[1] + b0[1]), p1 = pack2bf(v0[2] + b0[2], v0[3] + b0[3]);
      const uint32_t q0 = pack2bf(v1[0] + b1[0], v1[1] + b1[1]), q1 = pack2bf(v1[2] + b1[2], v1[3] + b1[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(p0, q0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(p1, q1, false, false);
      const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      const int m = pm0 + wm * 128 + (mq * 4 + i) * 16 + fr;
      // N % 8 == 0: a 16-byte chunk is all in or all out
      const uint32_t off = (m < a.M && col < a.N) ? (uint32_t)(m * a.ldc + col) * 2u : P_OOB;
      if constexpr (EPI == 1) {
        // u = bf16(acc + bias); C = bf16(gelu(u)), aux = bf16(gelu'(u)) -- gemm256.hip's rounding points
        float f[8], d[8];
        unpack8(o, f);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          f[r] = gelu_fg(f[r], d[r]);
          __builtin_amdgcn_sched_barrier(0);  // one erf at a time (register pressure)
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pack8(d)), rsX, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pack8(f)), rsC, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsC, off, 0, 0);
      }
      v0 = f32x4{0.f, 0.f, 0.f, 0.f};
      v1 = f32x4{0.f, 0.f, 0.f, 0.f};
      // one fragment row at a time: keeps the epilogue's temporaries (GELU's above all) from being
      // scheduled beside the next rows' and the phase's MFMAs (register pressure -> spills)
      if constexpr (EPI == 1) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- k-step: 4 quadrant phases (gemm256.hip's schedule) plus, in a tile's first k-step, the
  // previous tile's flush.  S = stores per flushed quadrant per wave (4, or 8 with the aux copy).
  // Waits (each retires every op older than its target part):
  //   phase 1 targets A1[g] (issued at g-1 phase 1); younger: A0[g+1], B1[g+1], B0[g+1] (2 each) +
  //     in a first k-step the phase-0 flush (S)            -> 6 (+S)
  //     in a second k-step the previous k-step's phase 1-3 flushes (3S) -> 6 + 3S
  //   phase 3 targets B0[g+1] (g phase 0); younger: A1[g+1], A0[g+2] (2 each) +
  //     in a first k-step the flushes of phases 0-2 (3S)   -> 4 (+3S)
  //   so the stores of a quadrant get >= 4 phases to leave before a wait covers them.
  constexpr int S = EPI == 1 ? 8 : 4;
  auto ktile = [&](int g, int t, bool first, bool second, int pm0, int pn0, bf16x8 (&bc)[2][2],
                   bf16x8 (&bn)[2][2]) __attribute__((always_inline)) {
    // k-steps g+1, g+2 -> (k-tile, next tile?) within this block's sequence
    const int t1 = t + 1 < nk ? t + 1 : 0, t2 = t + 2 < nk ? t + 2 : t + 2 - nk;
    const bool n1 = t + 1 >= nk, n2 = t + 2 >= nk;
    const bool flush_prev = first && g > 0;       // g = li * nk: tiles after the block's first
    const bool prev_flushed = second && g > 1;     // g = li * nk + 1 > 1  <=>  li >= 1 (nk >= 3)
    issue(g + 1, t1, n1, 1, 0);
    if (flush_prev) flush(0, 0, pm0, pn0);  // before the fragment read: its registers are free here
    read_b(bn, g, 1);
    mma(af, bc, 0, 0);
    // phase-1 wait (see above); an over-count would retire too little, so every case is spelled out
    if (flush_prev) {
      if constexpr (S == 8) P_VMWAIT(14); else P_VMWAIT(10);
    } else if (prev_flushed) {
      if constexpr (S == 8) P_VMWAIT(30); else P_VMWAIT(18);
    } else {
      P_VMWAIT(6);
    }
    p_barrier();
    issue(g + 1, t1, n1, 0, 1);
    if (flush_prev) flush(0, 1, pm0, pn0);
    mma(af, bn, 0, 1);
    read_a(af, g, 1);
    issue(g + 2, t2, n2, 0, 0);
    if (flush_prev) flush(1, 1, pm0, pn0);
    mma(af, bn, 1, 1);
    if (flush_prev) {
      if constexpr (S == 8) P_VMWAIT(28); else P_VMWAIT(16);
    } else {
      P_VMWAIT(4);
    }
    p_barrier();
    issue(g + 2, t2, n2, 1, 1);
    const bool more = g + 1 < total;
    if (flush_prev) flush(1, 0, pm0, pn0);
    if (more) read_b(bn, g + 1, 0);
    mma(af, bc, 1, 0);
    if (more) read_a(af, g + 1, 0);
  };

  // prologue: the loads steady state would have issued before k-step 0, then A0[0] / B0[0]
  issue(0, 0, false, 0, 0); issue(0, 0, false, 1, 1); issue(0, 0, false, 1, 0); issue(0, 0, false, 0, 1);
  issue(1, 1, false, 0, 0); issue(1, 1, false, 1, 1);
  P_VMWAIT(6);
  p_barrier();
  read_a(af, 0, 0);
  read_b(bx, 0, 0);
  if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);  // see gemm256.hip

  int li = 0, t = 0;  // tile / k-tile of global k-step g
  int pm0 = m0c, pn0 = n0c;  // the tile whose accumulators a first k-step flushes
  for (int g = 0; g < total; g += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int gg = g + u;
      if (gg >= total) break;
      if (t == 0 && gg > 0) {
        // entering tile li: the resources slide (current <- next, next <- tile li + 1)
        pm0 = m0c; pn0 = n0c;
        m0c = m0n; n0c = n0n;
        rsA_c = rsA_n; rsB_c = rsB_n;
        if (li + 1 < ntl) {
          tile_coords(a, idx + (li + 1) * G, m0n, n0n);
          rsA_n = rows_rsrc(a.A, m0n, a.M, a.lda);
          rsB_n = rows_rsrc(a.B, n0n, a.N, a.ldb);
        }
      }
      if (u == 0) ktile(gg, t, t == 0, t == 1, pm0, pn0, bx, by);
      else ktile(gg, t, t == 0, t == 1, pm0, pn0, by, bx);
      if (++t == nk) { t = 0; ++li; }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  P_VMWAIT(0);  // dummy part loads still target LDS; the last tile's bias has landed
  // the last tile's epilogue
  flush(0, 0, m0c, n0c);
  flush(0, 1, m0c, n0c);
  flush(1, 1, m0c, n0c);
  flush(1, 0, m0c, n0c);
}

}  // namespace

static int g_p_cus = 0;
static int g_p_mode = -1;  // MI355X_DP_GEMM_PERSIST: 1 use the persistent kernel, 0 (default) never

// Returns hipErrorInvalidValue when the shape / options are outside this kernel's contract (the
// caller then uses gemm256.hip's kernel).
MI_API int mi_gemm256p_nt(const void* A, const void* B, void* C, const float* bias, void* aux, int epi, int M, int N,
                          int K, int lda, int ldb, int ldc, hipStream_t st) {
  if (g_p_mode < 0) {
    const char* e = std::getenv("MI355X_DP_GEMM_PERSIST");
    g_p_mode = (e && e[0] == '1') ? 1 : 0;
  }
  const int nk = cdiv(K, P_BK);
  // EPI 1 (GELU) is written but not dispatched: its flush needs a few more registers than the
  // 256 a 2-wave-per-SIMD kernel has (52 B/lane of scratch), see tests/test_build_cpu.py
  if (!g_p_mode || epi != 0 || (bias && N > P_BIAS_MAX) || (epi == 1 && !aux) || nk < 3 || K % 8 || N % 8 || lda % 8 ||
      ldb % 8 || ldc % 8 || M <= 0 || N < 8 || (int64_t)P_BM * lda * 2 >= 0x7fffffffLL ||
      (int64_t)P_BN * ldb * 2 >= 0x7fffffffLL)
    return (int)hipErrorInvalidValue;
  if (g_p_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_p_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_p_cus <= 0)
      g_p_cus = 256;
  }
  G256PArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C; a.bias = bias; a.aux = (bf16_t*)aux;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.tiles_m = cdiv(M, P_BM); a.tiles_n = cdiv(N, P_BN);
  a.ntiles = a.tiles_m * a.tiles_n;
  a.nk = nk;
  const int grid = std::min(a.ntiles, g_p_cus);
  if (const char* t = std::getenv("MI355X_DP_TRACE_GEMM"); t && t[0] == '1')
    fprintf(stderr, "[gemm] g256p M=%d N=%d K=%d epi=%d tiles=%d blocks=%d\n", M, N, K, epi, a.ntiles, grid);
  hipLaunchKernelGGL(gemm256p_nt_kernel<0>, dim3(grid), dim3(512), 0, st, a);
  return (int)hipGetLastError();
}

MI_API int mi_set_gemm_persist(int on) {
  g_p_mode = on ? 1 : 0;
  return 0;
}
