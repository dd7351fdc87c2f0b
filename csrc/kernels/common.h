// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of mi355x_dp.
// Wave = 64 lanes; every block size used here is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MI_API extern "C" __attribute__((visibility("default")))

#include <cstdio>
#include <mutex>
#include <vector>

// ---- workspaces and captured HIP graphs (host side)
// A HIP graph bakes in the device pointers of every workspace its kernels used at capture time.
// A workspace that grows therefore never frees its old buffer: it is retired (kept allocated for
// the life of the process) so that any graph captured earlier still replays into live memory, and
// growth needs no device synchronisation.  A workspace that would have to grow INSIDE a capture
// does not (no allocation may happen there): the caller falls back to its workspace-free schedule
// and says so once on stderr.
inline void mi_ws_retire(void* p) {
  static std::mutex mu;
  static std::vector<void*> retired;
  if (!p) return;
  std::lock_guard<std::mutex> lk(mu);
  retired.push_back(p);
}
// Captures are taken with capture_error_mode="thread_local" (the smddp / RCCL watchdog threads poll
// events during a capture), so a workspace-growth path running on ANOTHER thread or stream than the
// capturing one would not be rejected by the runtime: its allocation / synchronisation would run
// silently outside the graph.  The capturing code therefore also announces every capture here
// (mi_capture_enter / _exit, parallel/step_graph.py, graphs.py), and while any capture is open no
// workspace grows, on any thread or stream.
#include <atomic>
inline std::atomic<int> g_mi_capture_depth{0};
inline bool mi_stream_capturing(hipStream_t st) {
  if (g_mi_capture_depth.load(std::memory_order_acquire) > 0) return true;
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &s) == hipSuccess && s != hipStreamCaptureStatusNone;
}
inline void mi_ws_capture_warn(const char* what) {
  static bool once = false;
  if (once) return;
  once = true;
  fprintf(stderr, "[mi355x_dp] %s workspace would have to grow inside a HIP graph capture: using the "
          "workspace-free schedule for this launch (run one eager step of the shape before capturing)\n", what);
}

// Device-side invariant checks of the debug build (-DMI_DEBUG, MI355X_DP_DEBUG_KERNELS=1): print
// the failing condition with the block / thread and a value, then trap.  Compiled out otherwise.
#ifdef MI_DEBUG
#include <cstdio>
#define MI_ASSERT(cond, val)                                                                          \
  do {                                                                                                \
    if (!(cond)) {                                                                                    \
      printf("MI_ASSERT %s:%d (%s) block %d thread %d value %lld\n", __FILE__, __LINE__, #cond,       \
             (int)blockIdx.x, (int)threadIdx.x, (long long)(val));                                    \
      __builtin_trap();                                                                               \
    }                                                                                                 \
  } while (0)
#else
#define MI_ASSERT(cond, val) \
  do {                       \
  } while (0)
#endif

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16 (plain cast lowers to v_cvt_pk_bf16_f32, NaN-preserving)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// unpack 8 bf16 held in a uint4
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  return v;
}

// bit j set <=> bf16 element j of the octet is nonzero: the ReLU mask of a stored activation
// (relu outputs are >= 0, so nonzero == positive) as one byte per 8 channels
__device__ __forceinline__ uint32_t nz_bits8(const uint4& v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    b |= ((w[k] & 0x7fffu) ? 1u : 0u) << (2 * k) | ((w[k] & 0x7fff0000u) ? 1u : 0u) << (2 * k + 1);
  return b;
}

// streaming 16-byte load (nontemporal: read once, do not keep in the caches)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const void* base, int64_t v) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)base + v));
}

// GEMM-epilogue operand loads: the accumulated-into C and the aux operand (residual / GELU
// derivative / ReLU source) are read once -- non-temporally (kEpiNtCY: +3.3 % on ResNet-50, round
// 5); the BN input read for the BN-backward statistics stays cached (kEpiNtX)
constexpr bool kEpiNtCY = true;
constexpr bool kEpiNtX = false;
template <bool NTL>
__device__ __forceinline__ uint4 epi_ld16(const void* p) {
  if (NTL) return __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)p));
  return *(const uint4*)p;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a linear block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// fast unsigned division by a runtime constant (host-built magic numbers)
struct FastDiv {
  uint32_t d, mul, shift;
};

static inline FastDiv make_fastdiv(uint32_t d) {
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

