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
//    the next issue), reads it back as 16-byte row chunks (one fixed 8-channel chunk per lane) and
//    stores full chunks; the lane accumulates that chunk's statistics over ALL its units in
//    registers, reduced across lanes and waves once per block (one statistics row per block).
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
  int gather, lda, H, W, stride;
  FastDiv fPQ, fQ;
};

#define PN_VMWAIT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int S, int ST>
__device__ __forceinline__ void pn_wait(int cnt) {
  // younger ops than the target k-step's loads: (S - 1) k-steps of 4 loads + cnt epilogues of ST
  // stores; vmcnt holds 6 bits (every count here is <= 12 + 3 * 8 = 36)
  static_assert(4 * (S - 1) + ST * (S - 1) <= 63, "vmcnt range");
  if constexpr (S == 2) {
    if (cnt == 0) PN_VMWAIT(4); else if constexpr (ST == 8) PN_VMWAIT(12); else PN_VMWAIT(8);
  } else if constexpr (S == 3) {
    if constexpr (ST == 8) {
      if (cnt == 0) PN_VMWAIT(8); else if (cnt == 1) PN_VMWAIT(16); else PN_VMWAIT(24);
    } else {
      if (cnt == 0) PN_VMWAIT(8); else if (cnt == 1) PN_VMWAIT(12); else PN_VMWAIT(16);
    }
  } else {
    static_assert(S == 4, "ring depth 2-4");
    if constexpr (ST == 8) {
      if (cnt == 0) PN_VMWAIT(12); else if (cnt == 1) PN_VMWAIT(20); else if (cnt == 2) PN_VMWAIT(28); else PN_VMWAIT(36);
    } else {
      if (cnt == 0) PN_VMWAIT(12); else if (cnt == 1) PN_VMWAIT(16); else if (cnt == 2) PN_VMWAIT(20); else PN_VMWAIT(24);
    }
  }
}

// BN: block panel width (columns), WN: wave tile width (64 or 128), S: ring slots per wave
template <int BN, int WN, int S>
__global__ __launch_bounds__(512) void panel_fwd_kernel(PanelArgs a) {
  constexpr int WNW = BN / WN, WMW = 8 / WNW;  // waves along N / along M
  constexpr int NJ = WN / 16;
  constexpr int ST = WN / 16;                  // epilogue stores per lane per unit (32 x WN bf16)
  constexpr int RING_U4 = 8 * S * PN_SLOT_U4;
  static_assert(WNW * WMW == 8 && (WN == 64 || WN == 128), "8 waves");
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

  // ---- the weight panel, once: piece p = 8 rows x 128 B of k-step kt (lane-linear image, chunk
  // c of row n holds logical chunk c ^ (n & 7))
  {
    constexpr int PPK = BN / 8;  // pieces per k-step
    const int np = nk * PPK;
    const int pr = lane >> 3, pc = lane & 7;
    for (int p = wid; p < np; p += 8) {
      const int kt = p / PPK, r8 = p - kt * PPK;
      const int n = n0 + r8 * 8 + pr;
      const uint32_t vo = n < a.N ? (uint32_t)(n * a.K + kt * 64 + ((pc ^ pr) * 8)) * 2u : PN_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, LDS_PTR(void, bpanel + (kt * BN + r8 * 8) * 8), 16, vo, 0, 0, 0);
    }
    PN_VMWAIT(0);
    __syncthreads();
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
  int iu = 0, ikt = 0;
  auto set_rows = [&](int lu) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = (u0 + lu) * 32 + u * 8 + lr;
      iok[u] = lu < nu && m < a.M;
      const uint32_t mm = iok[u] ? (uint32_t)m : 0u;
      uint32_t rowe;
      if (a.gather) {
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
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t vo = iok[u] ? ioff[u] + (uint32_t)ikt * 128u : PN_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, LDS_PTR(void, dst + u * 64), 16, vo, 0, 0, 0);
    }
    if (++ikt == nk) {
      ikt = 0;
      ++iu;
      set_rows(iu);
    }
  };

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[8], s2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { s1[q] = 0.f; s2[q] = 0.f; }
  const bool want_stats = a.stats != nullptr;
  // the lane's fixed epilogue chunk (8 channels) and the rows it reads back
  constexpr int CPR = WN / 8;     // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;   // rows per read instruction
  const int ec = lane % CPR, er = lane / CPR;
  const int ncol = n0 + wn * WN + ec * 8;  // output column of the lane's chunk

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

  // epilogue of unit lu through the 4 KB slot it consumed: lane (fr, fq) holds D[n = 16 j + 4 fq +
  // r][m = 16 i + fr]; rows are staged with the 16-B chunk index XOR-swizzled by the row (ds_write_b64
  // groups of 16 rows hit distinct bank pairs), read back one chunk per lane
  auto epilogue = [&](uint4* Cs, int lu) {
    char* cb = (char*)Cs;
    constexpr int HALVES = WN == 128 ? 2 : 1;  // 16 rows x 256 B or 32 rows x 128 B per pass
#pragma unroll
    for (int h = 0; h < HALVES; ++h) {
#pragma unroll
      for (int ii = 0; ii < 2 / HALVES; ++ii) {
        const int i = h + ii;  // fragment row block
        const int row = WN == 128 ? fr : 16 * i + fr;
        const int sw = WN == 128 ? row : ((row >> 1) & 7);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const f32x4 v = acc[i][j];
          const int pc = (2 * j + (fq >> 1)) ^ sw;
          *(uint2*)(cb + row * (WN * 2) + pc * 16 + (fq & 1) * 8) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
      constexpr int NR = WN == 128 ? 16 : 32;  // rows staged in this pass
#pragma unroll
      for (int u = 0; u < NR / RPI; ++u) {
        const int rr = er + RPI * u;
        const int sw = WN == 128 ? rr : ((rr >> 1) & 7);
        const uint4 v = *(const uint4*)(cb + rr * (WN * 2) + ((ec ^ sw) * 16));
        const int m = (u0 + lu) * 32 + (WN == 128 ? 16 * h : 0) + rr;
        if (want_stats) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) { s1[q] += f[q]; s2[q] = fmaf(f[q], f[q], s2[q]); }
        }
        const uint32_t off = (m < a.M && ncol < a.N) ? (uint32_t)(m * a.ldc + ncol) * 2u : PN_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsC, off, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- main loop over the wave's k-steps
  set_rows(0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue_next(s);
  uint32_t ehist = 0;  // bit t: an epilogue ran t + 1 iterations ago
  int kt = 0, lu = 0, slot = 0;
  for (int g = 0; g < G; ++g) {
    issue_next(slot == 0 ? S - 1 : slot - 1);  // k-step g + S - 1 into the slot k-step g - 1 used
    pn_wait<S, ST>(__builtin_popcount(ehist & ((1u << (S - 1)) - 1u)));
    uint4* cur = ring + slot * PN_SLOT_U4;
    compute(cur, kt);
    ehist <<= 1;
    if (++kt == nk) {
      epilogue(cur, lu);
      ehist |= 1u;
      kt = 0;
      ++lu;
    }
    slot = slot + 1 == S ? 0 : slot + 1;
  }

  // ---- statistics: lanes sharing a chunk, then the WMW waves of each column sub-panel (fixed order)
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
// MI355X_DP_PANEL: 1 route eligible 1x1 convs with >= PN_MIN_M output rows here (default), 0 never,
// 2 any row count (tests: small shapes stay on the split-K 64-tile kernels otherwise)
static int g_pn_mode = -1;
constexpr int PN_MIN_M = 16384;
static int g_pn_cus = 0;

struct PanelPlan {
  int bn = 0, wn = 0, s = 0, npanel = 0, nb = 0;
};

// panel width / ring depth for an N x K weight panel; bn == 0: not eligible
PanelPlan panel_plan(int M, int N, int K) {
  PanelPlan p;
  if (g_pn_mode < 0) {
    const char* e = std::getenv("MI355X_DP_PANEL");
    g_pn_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (!g_pn_mode || K % 64 != 0 || K > 512 || N % 64 != 0 || M < (g_pn_mode == 2 ? 1 : PN_MIN_M)) return p;
  if (g_pn_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_pn_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_pn_cus <= 0)
      g_pn_cus = 256;
  }
  const int64_t kb = (int64_t)K * 2;  // bytes per panel row
  if (N % 256 == 0 && 256 * kb <= 64 * 1024) {
    p.bn = 256; p.wn = 128;
  } else if (N % 128 == 0 && 128 * kb <= 64 * 1024) {
    p.bn = 128; p.wn = 128;
  } else if (64 * kb <= 64 * 1024) {
    p.bn = 64; p.wn = 64;
  } else {
    return PanelPlan{};
  }
  const int64_t bpanel = p.bn * kb;
  p.s = bpanel <= 32 * 1024 ? 4 : 3;
  p.npanel = N / p.bn;
  const int units = cdiv(M, 32);
  const int wm = 8 / (p.bn / p.wn);
  p.nb = std::max(1, std::min(g_pn_cus / std::max(1, std::min(p.npanel, g_pn_cus)), cdiv(units, wm)));
  return p;
}

template <int BN, int WN, int S>
void launch_panel(const PanelArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((panel_fwd_kernel<BN, WN, S>), dim3(grid), dim3(512), 0, st, a);
}

}  // namespace

MI_API int mi_set_panel(int mode) {
  g_pn_mode = mode == 2 ? 2 : (mode ? 1 : 0);
  return 0;
}

// statistics rows the panel kernel writes for an M x N x K conv (0: not routed there)
MI_API int mi_panel_stat_rows(int M, int N, int K) {
  const PanelPlan p = panel_plan(M, N, K);
  return p.bn ? p.nb : 0;
}

// 1x1 conv forward (pad 0, stride s) on the panel kernel: x NHWC [Nb,H,W,C], w [K][C], y NHWC
// [Nb,P,Q,K] bf16; stats: [mi_panel_stat_rows][2][K].  hipErrorNotSupported: shape not eligible.
MI_API int mi_panel_conv1x1(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int C,
                                int K, int stride, int P, int Q, hipStream_t st) {
  const int M = Nb * P * Q;
  const PanelPlan p = panel_plan(M, K, C);
  if (!p.bn) return (int)hipErrorNotSupported;
  const int64_t ab = (int64_t)Nb * H * W * C * 2, cb = (int64_t)M * K * 2, bb = (int64_t)K * C * 2;
  if (ab > 0x7FFFFFF0LL || cb > 0x7FFFFFF0LL || bb > 0x7FFFFFF0LL) return (int)hipErrorNotSupported;
  PanelArgs a{};
  a.A = (const bf16_t*)x; a.B = (const bf16_t*)w; a.C = (bf16_t*)y; a.stats = stats;
  a.M = M; a.N = K; a.K = C; a.ldc = K;
  a.nk = C / 64; a.npanel = p.npanel; a.nunits = cdiv(M, 32);
  a.a_bytes = (int)ab; a.b_bytes = (int)bb; a.c_bytes = (int)cb;
  a.gather = (stride != 1 || P != H || Q != W) ? 1 : 0;
  a.lda = C; a.H = H; a.W = W; a.stride = stride;
  a.fPQ = make_fastdiv((uint32_t)(P * Q));
  a.fQ = make_fastdiv((uint32_t)Q);
  const int grid = p.npanel * p.nb;
  if (const char* t = std::getenv("MI355X_DP_TRACE_GEMM"); t && t[0] == '1')
    fprintf(stderr, "[gemm] panel%d/%d s%d M=%d N=%d K=%d stride=%d stats=%d blocks=%d\n", p.bn, p.wn, p.s, M, K, C,
            stride, stats != nullptr, grid);
  if (p.bn == 256) {
    if (p.s == 4) launch_panel<256, 128, 4>(a, grid, st); else launch_panel<256, 128, 3>(a, grid, st);
  } else if (p.bn == 128) {
    if (p.s == 4) launch_panel<128, 128, 4>(a, grid, st); else launch_panel<128, 128, 3>(a, grid, st);
  } else {
    if (p.s == 4) launch_panel<64, 64, 4>(a, grid, st); else launch_panel<64, 64, 3>(a, grid, st);
  }
  return (int)hipGetLastError();
}
