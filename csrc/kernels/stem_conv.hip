// ResNet stem convolution (7x7 / stride 2 / pad 3, 3 input channels zero-padded to 8, 64 output
// channels) as a persistent MFMA kernel with an LDS-resident input ring, for gfx950.
//
// The generic implicit-GEMM path gathers every tap (16 B = one 8-channel pixel) from global memory,
// so each input pixel crosses L2 -> LDS ~12 times (49 taps / stride^2) and the weight tile is
// re-read by every block.  Here one block per CU owns whole images:
//   * each wave keeps its 32 output channels x 49 taps of weights in registers (13 B fragments,
//     loaded once), so the main loop reads only A fragments from LDS;
//   * a ring of 13 input rows (4 KB each) holds the 9 rows a PAIR of output rows needs plus the 4
//     new rows of the next pair, which are fetched with buffer_load ... lds while the current pair
//     computes (8 waves: waves 0-3 output row 2j, waves 4-7 row 2j+1);
//   * every A fragment (one tap of one output pixel = 16 B) comes from the ring, whose rows are
//     stored column-parity split (even input columns, then odd) so the stride-2 reads of 16
//     consecutive output pixels hit consecutive 16-B slots (no 2-way bank conflict);
//   * the epilogue stores bf16 rows straight from the accumulators and keeps the BatchNorm
//     (sum, sumsq) of the rounded outputs in registers across all rows; one statistics row per
//     block is written at the end (the BN finalize reduces them).
// Reference op: torchvision resnet conv1 (cifar10-distributed-smddp-gpu.py:30-32 via resnet18).
#include "common.h"
#include <algorithm>
#include <cstdlib>

// gemm_conv.hip: per-stream slab workspace (allocated on first use; nullptr on failure)
extern "C" float* mi_partials_workspace(size_t floats, hipStream_t st);

namespace {

constexpr int SR = 7, SS = 7, SSTR = 2;            // kernel 7x7, stride 2
constexpr int NTAP = SR * SS;                       // 49 taps of 8 channels (16 B)
constexpr int KSTEPS = (NTAP + 3) / 4;              // MFMA k = 32 = 4 taps
constexpr int KOUT = 64;
constexpr int ROWPX = 256;                          // ring row capacity (pixels of 16 B)
constexpr int PAIR_ROWS = SSTR + SR;                // input rows of two output rows: 9
constexpr int NEW_ROWS = 2 * SSTR;                  // new input rows per output-row pair: 4
constexpr int NRING = PAIR_ROWS + NEW_ROWS;         // 13
constexpr int MAX_BLOCKS = 256;                     // one per CU
constexpr int STEM_T = 512;

struct StemArgs {
  const bf16_t* x;    // [Nb][H][W][8]
  const bf16_t* w;    // [64][7][7][8]
  bf16_t* y;          // [Nb][P][Q][64]
  float* stats;       // [gridDim.x][2][64] or null
  int Nb, H, W, P, Q, pad;
  int pairs_per_img, total_pairs, pairs_per_block;
  int x_bytes;
};

__global__ __launch_bounds__(STEM_T, 1) void stem_conv_kernel(StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 sm[];
  uint4* ring = sm;                                   // [NRING][ROWPX]: even columns, then odd
  float* sred = (float*)(sm + NRING * ROWPX);         // [8 waves][2][64]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = wid >> 2, wq = wid & 3, wm = wq >> 1, wn = wq & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int g0 = blockIdx.x * a.pairs_per_block;
  const int g1 = min(a.total_pairs, g0 + a.pairs_per_block);
  const int HC = (a.Q - 1) * SSTR + SS;               // ring row width in use (<= ROWPX)

  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;

  // one input row -> ring slot (ih + pad) mod NRING; zero outside the image (padding)
  auto load_rows = [&](int img, int ih0, int nrows) {
    for (int c = wid; c < nrows * 4; c += 8) {         // 4 wave-loads of 64 pixels per row
      const int k = c >> 2, part = c & 3;
      const int ih = ih0 + k;
      const int pos = part * 64 + lane;                // ring position -> input column (parity split)
      const int px = pos < ROWPX / 2 ? 2 * pos : 2 * (pos - ROWPX / 2) + 1;
      const int iw = px - a.pad;
      const bool ok = px < HC && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const uint32_t vo = ok ? (uint32_t)((((img * a.H + ih) * a.W + iw) * 8) * 2) : OOB;
      const int slot = (ih + a.pad) % NRING;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, &ring[slot * ROWPX + part * 64]), 16, vo, 0, 0, 0);
    }
  };

  // this wave's weight fragments (channels wn*32 + 16j + fr, tap 4ks + fq), zero past tap 48
  bf16x8 bw[KSTEPS][2];
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t = 4 * ks + fq, n = wn * 32 + 16 * j + fr;
      const bf16x8 zero = {};
      bw[ks][j] = t < NTAP ? __builtin_bit_cast(bf16x8, ((const uint4*)a.w)[n * NTAP + t]) : zero;
    }
  for (int u = tid; u < 8 * 2 * KOUT; u += STEM_T) sred[u] = 0.f;
  if (g0 < g1) {
    const int img = g0 / a.pairs_per_img, j = g0 - img * a.pairs_per_img;
    load_rows(img, 2 * SSTR * j - a.pad, PAIR_ROWS);
  }

  float s1[2][4], s2[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }

  bool first = true;
  int last_stores = 0;
  for (int g = g0; g < g1; ++g) {
    const int img = g / a.pairs_per_img, jp = g - img * a.pairs_per_img;
    // the ring rows of this pair were issued BEFORE the previous pair's epilogue stores; vector
    // memory counts retire in issue order, so leaving exactly those stores in flight still
    // guarantees the loads landed.  The first pair and pairs after a fresh image load wait for all.
    switch (first ? 0 : last_stores) {                 // wave-uniform: stores issued last pair
      case 8: asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
    }
    first = false;
    __syncthreads();
    const bool next_same = g + 1 < g1 && (g + 1) / a.pairs_per_img == img;
    if (next_same) load_rows(img, 2 * SSTR * jp - a.pad + PAIR_ROWS, NEW_ROWS);  // prefetch next pair

    const int p = 2 * jp + half;                       // this half's output row
    last_stores = 0;
    if (p < a.P) {
#pragma unroll
      for (int i = 0; i < 4; ++i) last_stores += (wm * 64 + 16 * i < a.Q) ? 2 : 0;
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int rbase = (SSTR * p) % NRING;            // slot of input row SSTR*p - pad (+ r)
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int t = 4 * ks + fq;
        const bool tv = t < NTAP;
        const int r = t / SS, s = t - (t / SS) * SS;
        int slot = rbase + r;
        slot = slot >= NRING ? slot - NRING : slot;
        slot = slot >= NRING ? slot - NRING : slot;
        bf16x8 af[4];
        const bf16x8 zero = {};
        // input column 2q + s sits at ring position (s & 1) * ROWPX/2 + q + (s >> 1)
        const int cbase = slot * ROWPX + (s & 1) * (ROWPX / 2) + (s >> 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = wm * 64 + 16 * i + fr;        // output column (rows >= Q are discarded)
          const bf16x8 v = __builtin_bit_cast(bf16x8, ring[cbase + min(q, a.Q - 1)]);
          af[i] = tv ? v : zero;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks][j], af[i], acc[i][j], 0, 0, 0);
      }
      // epilogue: lane holds D[n = wn*32 + 16j + 4fq + r][q = wm*64 + 16i + fr]
      bf16_t* yrow = a.y + ((size_t)(img * a.P + p) * a.Q) * KOUT;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = wm * 64 + 16 * i + fr;
        if (q >= a.Q) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = wn * 32 + 16 * j + 4 * fq;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = bf2f(f2bf(acc[i][j][r]));
            s1[j][r] += v[r];
            s2[j][r] += v[r] * v[r];
          }
          *(uint2*)(yrow + (size_t)q * KOUT + n) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
    }
    if (g + 1 < g1 && !next_same) {                    // next pair starts a new image: fresh ring
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int img2 = (g + 1) / a.pairs_per_img, j2 = (g + 1) - img2 * a.pairs_per_img;
      load_rows(img2, 2 * SSTR * j2 - a.pad, PAIR_ROWS);
      first = true;
    }
  }

  if (!a.stats) return;
  // lanes sharing channels (same fq) differ in fr: reduce over lane bits 0-3, then over waves
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] += __shfl_xor(s1[j][r], o, 64);
        s2[j][r] += __shfl_xor(s2[j][r], o, 64);
      }
  __syncthreads();
  if (fr == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wn * 32 + 16 * j + 4 * fq + r;
        sred[(wid * 2 + 0) * KOUT + n] = s1[j][r];
        sred[(wid * 2 + 1) * KOUT + n] = s2[j][r];
      }
  }
  __syncthreads();
  if (tid < 2 * KOUT) {
    const int which = tid / KOUT, n = tid - which * KOUT;
    float t = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) t += sred[(w8 * 2 + which) * KOUT + n];
    a.stats[((size_t)blockIdx.x * 2 + which) * KOUT + n] = t;
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[k][tap][c] = sum over output pixels of dy[pix][k] * x[window(pix, tap)][c]: an MFMA GEMM
// (M = 64 output channels, N = 49 taps x 8 channels as 25 tiles of 2 taps, reduction = pixels)
// whose operands are both pixel-major, so every fragment is a ds_read_b64_tr_b16 transposed read:
// A (dy^T) from a staged pair of dy rows, B straight from the same parity-split input ring as the
// forward (any 8-byte-aligned address per lane), so no operand is ever restaged.  Each block keeps
// its partial dW in registers across all its rows and adds it into the fp32 gradient once.
constexpr int NUT = (NTAP + 1) / 2;                 // 25 n-tiles of 2 taps x 8 channels
constexpr int DYPX = 128;                           // staged pixels per output row (Q <= 128)
constexpr int STEM_WELEMS = KOUT * NTAP * 8;        // dW elements (64 x 49 taps x 8 channels)

struct StemWArgs {
  const bf16_t* x;    // [Nb][H][W][8]
  const bf16_t* dy;   // [Nb][P][Q][64]
  float* dw;          // [64][7][7][8] fp32, accumulated
  float* ws;          // [blocks][64 * 7 * 7 * 8] per-block partials (deterministic path) or null (atomics)
  int Nb, H, W, P, Q, pad;
  int pairs_per_img, total_pairs, pairs_per_block;
  int x_bytes, dy_bytes;
};

// 16-B chunk swizzle of a staged dy row: the two 4-pixel row groups of a 16-lane transposed read
// and the other group of its 32-lane half land on distinct bank octets
__device__ __forceinline__ int dy_swz(int px) { return (((px >> 1) & 1) << 1) | (((px >> 3) & 1) << 2); }

__global__ __launch_bounds__(STEM_T, 1) void stem_wgrad_kernel(StemWArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 sm[];
  uint4* ring = sm;                                   // [NRING][ROWPX]: even columns, then odd
  uint4* dys = sm + NRING * ROWPX;                    // [2 buffers][2 rows][DYPX][8 chunks]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int g0 = blockIdx.x * a.pairs_per_block;
  const int g1 = min(a.total_pairs, g0 + a.pairs_per_block);
  const int HC = (a.Q - 1) * SSTR + SS;

  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsd = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;

  auto load_rows = [&](int img, int ih0, int nrows) {
    for (int c = wid; c < nrows * 4; c += 8) {
      const int k = c >> 2, part = c & 3;
      const int ih = ih0 + k;
      const int pos = part * 64 + lane;
      const int px = pos < ROWPX / 2 ? 2 * pos : 2 * (pos - ROWPX / 2) + 1;
      const int iw = px - a.pad;
      const bool ok = px < HC && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const uint32_t vo = ok ? (uint32_t)((((img * a.H + ih) * a.W + iw) * 8) * 2) : OOB;
      const int slot = (ih + a.pad) % NRING;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, LDS_PTR(void, &ring[slot * ROWPX + part * 64]), 16, vo, 0, 0, 0);
    }
  };
  // output rows 2j, 2j+1 of dy -> buffer buf; a wave-load covers 8 pixels x 8 chunks
  auto load_dy = [&](int img, int jp, int buf) {
    for (int c = wid; c < 2 * DYPX / 8; c += 8) {
      const int h = c / (DYPX / 8), px = (c % (DYPX / 8)) * 8 + (lane >> 3);
      const int p = 2 * jp + h;
      const int lc = (lane & 7) ^ dy_swz(px);
      const bool ok = px < a.Q && p < a.P;
      const uint32_t vo = ok ? (uint32_t)((((img * a.P + p) * a.Q + px) * KOUT + lc * 8) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsd, LDS_PTR(void, &dys[((buf * 2 + h) * DYPX + (c % (DYPX / 8)) * 8) * 8]),
                                               16, vo, 0, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[m][v] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nv = wid + 24 < NUT ? 4 : 3;              // n-tiles u = wid + 8v of this wave

  if (g0 < g1) {
    const int img = g0 / a.pairs_per_img, j = g0 - img * a.pairs_per_img;
    load_rows(img, 2 * SSTR * j - a.pad, PAIR_ROWS);
    load_dy(img, j, 0);
  }
  int buf = 0;
  const uint2* ring2 = (const uint2*)ring;
  const uint2* dys2 = (const uint2*)dys;
  for (int gp = g0; gp < g1; ++gp) {
    const int img = gp / a.pairs_per_img, jp = gp - img * a.pairs_per_img;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool next_same = gp + 1 < g1 && (gp + 1) / a.pairs_per_img == img;
    if (next_same) {
      load_rows(img, 2 * SSTR * jp - a.pad + PAIR_ROWS, NEW_ROWS);
      load_dy(img, jp + 1, buf ^ 1);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = 2 * jp + h;
      if (p >= a.P) continue;
      const int rbase = (SSTR * p) % NRING;
      for (int c = 0; c < DYPX / 32; ++c) {
        if (32 * c >= a.Q) break;
        const int px1 = 32 * c + 8 * g + q4, px2 = px1 + 4;
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int lc = 2 * m + (p4 >> 1);
          const uint2* r1 = dys2 + ((buf * 2 + h) * DYPX + px1) * 16 + 2 * (lc ^ dy_swz(px1)) + (p4 & 1);
          const uint2* r2 = dys2 + ((buf * 2 + h) * DYPX + px2) * 16 + 2 * (lc ^ dy_swz(px2)) + (p4 & 1);
          short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, r1));
          short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, r2));
          short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[m] = __builtin_bit_cast(bf16x8, v8);
        }
        const int qa = min(px1, a.Q - 1), qb = min(px2, a.Q - 1);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          if (v >= nv) break;
          const int u = wid + 8 * v;
          const int t = min(2 * u + (p4 >> 1), NTAP - 1);
          const int r = t / SS, sx = t - (t / SS) * SS;
          int slot = rbase + r;
          slot = slot >= NRING ? slot - NRING : slot;
          const int cb = slot * ROWPX + (sx & 1) * (ROWPX / 2) + (sx >> 1);
          short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, ring2 + (cb + qa) * 2 + (p4 & 1)));
          short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, ring2 + (cb + qb) * 2 + (p4 & 1)));
          short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[v] = __builtin_bit_cast(bf16x8, v8);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          if (v >= nv) break;
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acc[m][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[v], acc[m][v], 0, 0, 0);
        }
      }
    }
    buf ^= 1;
    if (gp + 1 < g1 && !next_same) {                  // next pair starts a new image: fresh stage
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int img2 = (gp + 1) / a.pairs_per_img, j2 = (gp + 1) - img2 * a.pairs_per_img;
      load_rows(img2, 2 * SSTR * j2 - a.pad, PAIR_ROWS);
      load_dy(img2, j2, buf);
    }
  }
  // D[i = out channel 16m + 4g + r][j = 16u + li]: column j = tap 2u + (li >> 3), channel li & 7.
  // Deterministic path: the block's partial dW goes to its own slab row (plain stores; every element
  // of the row is written, zeros for blocks without work) and stem_wgrad_reduce_kernel sums the
  // rows in a fixed order -- bitwise reproducible gradients.  Fallback: fp32 atomics into dw.
  float* prow = a.ws ? a.ws + (size_t)blockIdx.x * STEM_WELEMS : nullptr;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    if (v >= nv) break;
    const int tap = 2 * (wid + 8 * v) + (li >> 3);
    if (tap >= NTAP) continue;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * m + 4 * g + r;
        const size_t o = ((size_t)k * NTAP + tap) * 8 + (li & 7);
        if (prow) prow[o] = acc[m][v][r];
        else atomicAdd(a.dw + o, acc[m][v][r]);
      }
  }
}

// dw[e] += sum over rows b of ws[b][e], b ascending in G interleaved groups combined in LDS in a
// fixed order.  Block: 32 float4 positions x 8 groups.
constexpr int SWR_POS = 32, SWR_G = 8;
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float4* __restrict__ ws, float4* __restrict__ dw,
                                                                int rows) {
  __shared__ float4 red[SWR_G][SWR_POS];
  const int pl = threadIdx.x % SWR_POS, grp = threadIdx.x / SWR_POS;
  const int pos = blockIdx.x * SWR_POS + pl;
  constexpr int NV = STEM_WELEMS / 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pos < NV)
    for (int b = grp; b < rows; b += 4 * SWR_G) {  // 4 rows' loads in flight, summed in row order
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = b + u * SWR_G < rows ? ws[(size_t)(b + u * SWR_G) * NV + pos] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
  red[grp][pl] = s;
  __syncthreads();
  if (grp != 0 || pos >= NV) return;
  for (int gg = 1; gg < SWR_G; ++gg) {
    const float4 v = red[gg][pl];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float4 d = dw[pos];
  d.x += s.x; d.y += s.y; d.z += s.z; d.w += s.w;
  dw[pos] = d;
}

// The same fixed-order row sum for the parameter's own gradient: g[k][c][r][s] (any strides, the
// flat buffer's kernel layout) += sum over rows of ws[.][k][tap][c] for the real channels c < Cw --
// the padded [K][7][7][8] gradient is never materialised, cropped or permuted by extra launches.
__global__ __launch_bounds__(256) void stem_wgrad_reduce_to_kernel(const float* __restrict__ ws, float* __restrict__ g,
                                                                   int rows, int Cw, int64_t sK, int64_t sC,
                                                                   int64_t sR, int64_t sS) {
  __shared__ float red[SWR_G][SWR_POS];
  const int pl = threadIdx.x % SWR_POS, grp = threadIdx.x / SWR_POS;
  const int pos = blockIdx.x * SWR_POS + pl;
  const int ne = KOUT * NTAP * Cw;
  const int c = pos % Cw, t = pos / Cw, tap = t % NTAP, k = t / NTAP;
  const int o = (k * NTAP + tap) * 8 + c;
  float s = 0.f;
  if (pos < ne)
    for (int b = grp; b < rows; b += 8 * SWR_G) {  // 8 rows' loads in flight, summed in row order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = b + u * SWR_G < rows ? ws[(size_t)(b + u * SWR_G) * STEM_WELEMS + o] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  red[grp][pl] = s;
  __syncthreads();
  if (grp != 0 || pos >= ne) return;
  for (int gg = 1; gg < SWR_G; ++gg) s += red[gg][pl];
  float* d = g + k * sK + c * sC + (tap / SS) * sR + (tap % SS) * sS;
  *d += s;
}

// Conv weight [K][Cw][R][S] bf16 (any strides) -> the stem kernel's [K][7][7][8] operand, channels
// >= Cw zero: one launch per step instead of a zero fill plus a strided copy.
__global__ __launch_bounds__(256) void stem_wpack_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                         int total, int Cw, int R, int S, int64_t sK, int64_t sC,
                                                         int64_t sR, int64_t sS) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int c = e & 7, t = e >> 3, tap = t % (R * S), k = t / (R * S);
  dst[e] = c < Cw ? src[k * sK + c * sC + (tap / S) * sR + (tap % S) * sS] : (bf16_t)0;
}

constexpr size_t stem_wgrad_lds_bytes() { return (size_t)(NRING * ROWPX + 2 * 2 * DYPX * 8) * 16; }

constexpr size_t stem_lds_bytes() {
  return (size_t)(NRING * ROWPX) * 16 + 8 * 2 * KOUT * 4;
}

// Blocks of the persistent stem kernels: MAX_BLOCKS = one per CU by default.  MI355X_DP_STEM_BLOCKS
// raises it (e.g. 512: half-image row ranges, so CUs shared with concurrent RCCL kernels during
// the overlapped gradient all-reduce hold back less of the work).
static int g_stem_blocks = -1;
inline int stem_blocks(int total_pairs) {
  if (g_stem_blocks < 0) {
    const char* e = std::getenv("MI355X_DP_STEM_BLOCKS");
    g_stem_blocks = e ? std::max(1, std::atoi(e)) : MAX_BLOCKS;
  }
  return std::max(1, std::min(total_pairs, g_stem_blocks));
}

}  // namespace

// Does the persistent stem kernel take this conv?  (7x7 / stride 2 on an 8-channel NHWC input,
// 64 output channels, output rows narrow enough for the ring.)
MI_API int mi_stem_conv_ok(int C, int K, int R, int S, int stride, int pad, int Q) {
  return C == 8 && K == KOUT && R == SR && S == SS && stride == SSTR && pad >= 0 && pad < SR &&
         (Q - 1) * SSTR + SS <= ROWPX && Q <= 128;
}

// Statistics rows written by mi_stem_conv_fwd (one per block).
MI_API int mi_stem_conv_stat_rows(int Nb, int P) { return stem_blocks(Nb * ((P + 1) / 2)); }

// x [Nb][H][W][8] bf16, w [64][7][7][8] bf16, y [Nb][P][Q][64] bf16, stats [rows][2][64] fp32 (optional)
MI_API int mi_stem_conv_fwd(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W, int P, int Q,
                            int pad, hipStream_t st) {
  if (!mi_stem_conv_ok(8, KOUT, SR, SS, SSTR, pad, Q)) return (int)hipErrorInvalidValue;
  const int64_t xb = (int64_t)Nb * H * W * 8 * 2;
  if (xb > 0x7FFFFFF0LL) return (int)hipErrorInvalidValue;
  StemArgs a{};
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.y = (bf16_t*)y; a.stats = stats;
  a.Nb = Nb; a.H = H; a.W = W; a.P = P; a.Q = Q; a.pad = pad;
  a.pairs_per_img = (P + 1) / 2;
  a.total_pairs = Nb * a.pairs_per_img;
  const int blocks = stem_blocks(a.total_pairs);
  a.pairs_per_block = cdiv(a.total_pairs, blocks);
  a.x_bytes = (int)xb;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)stem_conv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)stem_lds_bytes());
    attr = true;
  }
  hipLaunchKernelGGL(stem_conv_kernel, dim3(blocks), dim3(STEM_T), stem_lds_bytes(), st, a);
  return (int)hipGetLastError();
}

// Gradient destination of stem_wgrad: dw [64][7][7][8] (to == nullptr) or the parameter's own
// gradient g [64][Cw][7][7] with element strides (deterministic partials path only).
struct StemWTo {
  float* g;
  int Cw;
  int64_t sK, sC, sR, sS;
};

static int stem_wgrad_impl(const void* x, const void* dy, float* dw, const StemWTo* to, int Nb, int H, int W, int P,
                           int Q, int pad, hipStream_t st) {
  if (!mi_stem_conv_ok(8, KOUT, SR, SS, SSTR, pad, Q) || Q > DYPX) return (int)hipErrorInvalidValue;
  const int64_t xb = (int64_t)Nb * H * W * 8 * 2, db = (int64_t)Nb * P * Q * KOUT * 2;
  if (xb > 0x7FFFFFF0LL || db > 0x7FFFFFF0LL) return (int)hipErrorInvalidValue;
  StemWArgs a{};
  a.x = (const bf16_t*)x; a.dy = (const bf16_t*)dy; a.dw = dw;
  a.Nb = Nb; a.H = H; a.W = W; a.P = P; a.Q = Q; a.pad = pad;
  a.pairs_per_img = (P + 1) / 2;
  a.total_pairs = Nb * a.pairs_per_img;
  const int blocks = stem_blocks(a.total_pairs);
  a.pairs_per_block = cdiv(a.total_pairs, blocks);
  a.x_bytes = (int)xb;
  a.dy_bytes = (int)db;
  // deterministic per-block partials (MI355X_DP_STEM_ATOMIC=1: the fp32-atomic path instead)
  static int atomic_mode = -1;
  if (atomic_mode < 0) {
    const char* e = std::getenv("MI355X_DP_STEM_ATOMIC");
    atomic_mode = (e && e[0] == '1') ? 1 : 0;
  }
  a.ws = (!atomic_mode && ((uintptr_t)dw & 15) == 0) ? mi_partials_workspace((size_t)blocks * STEM_WELEMS, st)
                                                     : nullptr;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)stem_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)stem_wgrad_lds_bytes());
    attr = true;
  }
  if (to && !a.ws) return (int)hipErrorNotSupported;  // atomic mode: the caller pads and permutes
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(blocks), dim3(STEM_T), stem_wgrad_lds_bytes(), st, a);
  if (to)
    hipLaunchKernelGGL(stem_wgrad_reduce_to_kernel, dim3(cdiv(KOUT * NTAP * to->Cw, SWR_POS)), dim3(256), 0, st,
                       (const float*)a.ws, to->g, blocks, to->Cw, to->sK, to->sC, to->sR, to->sS);
  else if (a.ws)
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(cdiv(STEM_WELEMS / 4, SWR_POS)), dim3(256), 0, st,
                       (const float4*)a.ws, (float4*)dw, blocks);
  return (int)hipGetLastError();
}

// dw [64][7][7][8] fp32 += stem weight gradient; x [Nb][H][W][8], dy [Nb][P][Q][64] bf16.
MI_API int mi_stem_wgrad(const void* x, const void* dy, float* dw, int Nb, int H, int W, int P, int Q, int pad,
                         hipStream_t st) {
  return stem_wgrad_impl(x, dy, dw, nullptr, Nb, H, W, P, Q, pad, st);
}

// g [64][Cw][7][7] fp32 (element strides sK, sC, sR, sS) += stem weight gradient of the real
// channels.  hipErrorNotSupported when the shape is not the stem kernel's or the atomic fallback is
// selected (the caller then uses mi_conv2d_wgrad into a padded buffer).
// K, R, S, stride: the conv's real geometry -- the persistent kernel only computes the 7x7/2/64
// gradient, so any other stem (3x3/1, 32 output channels, ...) must take the generic path.
MI_API int mi_stem_wgrad_to(const void* x, const void* dy, float* g, int Cw, int64_t sK, int64_t sC, int64_t sR,
                            int64_t sS, int Nb, int H, int W, int K, int R, int S, int stride, int P, int Q, int pad,
                            hipStream_t st) {
  if (Cw < 1 || Cw > 8) return (int)hipErrorInvalidValue;
  const char* e = std::getenv("MI355X_DP_STEM_KERNEL");  // =0: the generic path (gemm_conv.hip)
  if ((e && e[0] == '0') || !mi_stem_conv_ok(8, K, R, S, stride, pad, Q)) return (int)hipErrorNotSupported;
  if (P != (H + 2 * pad - R) / stride + 1 || Q != (W + 2 * pad - S) / stride + 1) return (int)hipErrorInvalidValue;
  const StemWTo to{g, Cw, sK, sC, sR, sS};
  return stem_wgrad_impl(x, dy, nullptr, &to, Nb, H, W, P, Q, pad, st);
}

// src: conv weight [K][Cw][R][S] bf16 with element strides; dst: [K][R][S][8] bf16 (any small-channel
// conv of the fused stem: the persistent 7x7 kernel or the generic 8-channel implicit GEMM).
MI_API int mi_stem_wpack(const void* src, void* dst, int K, int Cw, int R, int S, int64_t sK, int64_t sC, int64_t sR,
                         int64_t sS, hipStream_t st) {
  if (K < 1 || R < 1 || S < 1 || Cw < 1 || Cw > 8 || (int64_t)K * R * S * 8 > 0x7FFFFFFF)
    return (int)hipErrorInvalidValue;
  const int total = K * R * S * 8;
  hipLaunchKernelGGL(stem_wpack_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, (const bf16_t*)src, (bf16_t*)dst,
                     total, Cw, R, S, sK, sC, sR, sS);
  return (int)hipGetLastError();
}
