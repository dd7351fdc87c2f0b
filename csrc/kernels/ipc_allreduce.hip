// Collectives over IPC peer pointers for the native smddp backend:
// one-shot and two-shot all-reduce, a generic one-shot (any dtype / op, broadcast, barrier) and the
// balanced-shard mesh reduce-scatter / all-gather.  csrc/comm/smddp_backend.cpp resolves them from
// the kernel library and uses them when MI355X_DP_SMDDP_IPC=1 / _IPC_ONLY=1; RCCL stays the path
// for everything else.
//
// Memory (per rank, exported with hipIpcGetMemHandle, opened by every peer):
//   * a data buffer with two slots (alternating by call parity), plain coarse-grained hipMalloc
//     memory -- the bandwidth path;
//   * a flag array in fine-grained / uncached device memory (hipExtMallocWithFlags, see the
//     backend): every flag store and poll goes to memory, never to a stale cache line of another
//     XCD's L2 or another GPU.
// Protocol of one call (epoch e, this rank r, block b; every rank launches the same grid because
// the grid depends only on the element count):
//   1. copy-in: block b copies exactly the input elements that blocks with index b on every rank
//      will read into slot[e & 1] of r's buffer -- the waves that write the data are the ones that
//      release it (no separate hipMemcpyAsync, no reliance on a kernel boundary for visibility);
//   2. publish: every storing wave waits for its stores (s_waitcnt vmcnt(0)), workgroup barrier,
//      then one lane: system-scope release fence (writes the XCD's dirty L2 lines back, so a peer
//      reading this memory over xGMI sees them), s_waitcnt vmcnt(0) (the fence's own wait can be
//      dropped by the compiler, MI355X_MICROARCH.md "Compiler hazard"), and `e` into
//      flag_in[r][b] of every peer (system-scope atomic store);
//   3. wait: one lane polls flag_in[q][b] >= e for every peer q (relaxed system-scope loads of
//      uncached memory, s_sleep between polls, bounded: on timeout the host-visible error word is
//      raised and the output is left untouched -- never a hang), then a system-scope acquire
//      fence and a workgroup barrier before any peer data is read;
//   4. compute: peer slots are read with non-temporal loads.
// Only blocks with the same index talk to each other: no grid barrier, no co-residency assumption.
// Slot reuse is safe without an end barrier: rank r rewrites slot[e & 1] only in call e + 2, which
// starts after r's call e + 1 completed; that needed peer p's e + 1 flags, which p raises only
// after its call e finished (stream order) -- so no peer still reads r's call-e slot.
#include "common.h"

// Grid cap of every IPC collective kernel.  Their blocks spin on peer flags, and the dispatcher
// spreads a grid one block per CU: a 256-block spinner leaves no CU whose register file can take a
// full-CU compute block (gemm256: 8 waves x 256 VGPRs), so backward on the same GPU stalls behind
// the collective -- and with two ranks sharing a GPU the peer's backward never reaches its
// collective at all (a deadlock until the spin bound).  64 blocks keep 3/4 of the CUs free.
#ifndef MI_IPC_MAX_GRID
#define MI_IPC_MAX_GRID 64
#endif

namespace {

constexpr int IPC_MAX_PEERS = 8;
constexpr int IPC_MAX_BLOCKS = 256;
// flag array layout (uint32 words): input flags [src][block], then the two-shot's phase-2 flags
constexpr int IPC_FLAG_IN_OFF = 0;
constexpr int IPC_FLAG2_OFF = IPC_MAX_PEERS * IPC_MAX_BLOCKS;
constexpr int IPC_FLAG_WORDS = 2 * IPC_MAX_PEERS * IPC_MAX_BLOCKS;

struct IpcRaw {
  const void* data[IPC_MAX_PEERS];  // this call's slot in every rank's buffer
  uint32_t* flags[IPC_MAX_PEERS];   // every rank's flag array
};

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ bool ipc_wait_ge(uint32_t* f, uint32_t epoch, uint32_t spin_limit, uint32_t& spins) {
  while ((int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
    if (++spins > spin_limit) return false;
    __builtin_amdgcn_s_sleep(8);
  }
  return true;
}

// steps 2 + 3 for flag region `off` (input flags or the two-shot's phase-2 flags): publish this
// block's stores to every peer (`skip_self`: not to this rank), wait for the same block of every peer
__device__ __forceinline__ bool ipc_block_sync(const IpcRaw& p, int rank, int world, int off, bool skip_self,
                                               uint32_t epoch, int* err, uint32_t spin_limit) {
  __shared__ int ok;
  const int b = blockIdx.x;
  vm_drain();  // this wave's copy-in stores have left the wave
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    vm_drain();
    for (int q = 0; q < world; ++q)
      if (!(skip_self && q == rank))
        __hip_atomic_store(p.flags[q] + off + rank * IPC_MAX_BLOCKS + b, epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t spins = 0;
    bool good = true;
    for (int q = 0; q < world && good; ++q)
      if (!(skip_self && q == rank))
        good = ipc_wait_ge(p.flags[rank] + off + q * IPC_MAX_BLOCKS + b, epoch, spin_limit, spins);
    if (!good) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale cached peer lines
    vm_drain();
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

int ipc_grid(int64_t work) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(MI_IPC_MAX_GRID, (work + 255) / 256));
}

// ------------------------------------------------------------------ one-shot fp32 all-reduce
template <bool VEC>
__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcRaw p, int rank, int world, const float* in,
                                                            float* out, int64_t n, uint32_t epoch, float scale,
                                                            int* err, uint32_t spin_limit) {
  float* mine = (float*)p.data[rank];
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if constexpr (VEC) {
    for (int64_t i = 4 * t0; i < n; i += 4 * step) *(f32x4*)(mine + i) = *(const f32x4*)(in + i);
  } else {
    for (int64_t i = t0; i < n; i += step) mine[i] = in[i];
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  if constexpr (VEC) {
    for (int64_t i = 4 * t0; i < n; i += 4 * step) {
      f32x4 s = __builtin_nontemporal_load((const f32x4*)((const float*)p.data[0] + i));
#pragma unroll 1
      for (int q = 1; q < world; ++q) s += __builtin_nontemporal_load((const f32x4*)((const float*)p.data[q] + i));
      *(f32x4*)(out + i) = s * scale;
    }
  } else {
    for (int64_t i = t0; i < n; i += step) {
      float s = 0.f;
#pragma unroll 1
      for (int q = 0; q < world; ++q) s += __builtin_nontemporal_load((const float*)p.data[q] + i);
      out[i] = s * scale;
    }
  }
}

// ------------------------------------------------------------------ two-shot fp32 all-reduce
// Reduce-scatter + all-gather inside one launch: every rank reads (world-1)/world of the data from
// peers twice instead of (world-1) x all of it once, so each of the 7 point-to-point xGMI links
// carries 2/world of the bucket.
//   copy-in: block b copies chunk b of EVERY shard (the pieces block b of each rank reduces);
//   phase 1: block b sums chunk b of this rank's shard over all peers' slots into its OWN slot
//            (peers read this rank's slot only at their own shard range in phase 1, never at this
//            one) and into `out`; publish through the phase-2 flags;
//   phase 2: block b copies chunk b of every other shard from that shard owner's slot into `out`.
// shard = ceil(n / world) rounded up to 4 elements; chunk = ceil(shard / gridDim.x) rounded to 4.
template <bool VEC>
__device__ __forceinline__ void copy_span(const float* src, float* dst, int64_t lo, int64_t hi) {
  if constexpr (VEC) {
    for (int64_t i = lo + 4 * (int64_t)threadIdx.x; i < hi; i += 4 * (int64_t)blockDim.x)
      *(f32x4*)(dst + i) = *(const f32x4*)(src + i);
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) dst[i] = src[i];
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void ipc_allreduce2_kernel(IpcRaw p, int rank, int world, const float* in,
                                                             float* out, int64_t n, int64_t shard, int64_t chunk,
                                                             uint32_t epoch, float scale, int* err,
                                                             uint32_t spin_limit) {
  const int b = blockIdx.x;
  float* mine = (float*)p.data[rank];
  for (int q = 0; q < world; ++q) {
    const int64_t lo = min(n, q * shard + b * chunk);
    const int64_t hi = min(min(n, (q + 1) * shard), lo + chunk);
    copy_span<VEC>(in, mine, lo, hi);
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  {
    const int64_t lo = min(n, rank * shard + b * chunk);
    const int64_t hi = min(min(n, (rank + 1) * shard), lo + chunk);
    if constexpr (VEC) {
      for (int64_t i = lo + 4 * (int64_t)threadIdx.x; i < hi; i += 4 * (int64_t)blockDim.x) {
        f32x4 s = __builtin_nontemporal_load((const f32x4*)((const float*)p.data[0] + i));
#pragma unroll 1
        for (int q = 1; q < world; ++q) s += __builtin_nontemporal_load((const f32x4*)((const float*)p.data[q] + i));
        s *= scale;
        *(f32x4*)(mine + i) = s;
        *(f32x4*)(out + i) = s;
      }
    } else {
      for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        float s = 0.f;
#pragma unroll 1
        for (int q = 0; q < world; ++q) s += __builtin_nontemporal_load((const float*)p.data[q] + i);
        mine[i] = s * scale;
        out[i] = s * scale;
      }
    }
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG2_OFF, true, epoch, err, spin_limit)) return;
  for (int q = 0; q < world; ++q) {
    if (q == rank) continue;
    const int64_t lo = min(n, q * shard + b * chunk);
    const int64_t hi = min(min(n, (q + 1) * shard), lo + chunk);
    const float* src = (const float*)p.data[q];
    if constexpr (VEC) {
      for (int64_t i = lo + 4 * (int64_t)threadIdx.x; i < hi; i += 4 * (int64_t)blockDim.x)
        *(f32x4*)(out + i) = __builtin_nontemporal_load((const f32x4*)(src + i));
    } else {
      for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = __builtin_nontemporal_load(src + i);
    }
  }
}

// ------------------------------------------------------------- generic one-shot (IPC-only mode)
// op SUM / MAX / MIN over f32 / f64 / i32 / i64 / bf16, COPY = every rank takes the root's slot
// (broadcast), and a zero-byte call is a barrier (flag round only).
enum { IPC_SUM = 0, IPC_MAX = 1, IPC_MIN = 2, IPC_COPY = 3 };

template <typename T, int OP>
__device__ __forceinline__ T ipc_combine(T a, T b) {
  if (OP == IPC_SUM) return a + b;
  if (OP == IPC_MAX) return a > b ? a : b;
  return a < b ? a : b;
}

// bf16 elements (raw bits): combined in fp32, rounded once per step in rank order -- identical on
// every rank
struct Bf16 {
  uint16_t v;
};
template <>
__device__ __forceinline__ Bf16 ipc_combine<Bf16, IPC_SUM>(Bf16 a, Bf16 b) { return {f2bf(bf2f(a.v) + bf2f(b.v))}; }
template <>
__device__ __forceinline__ Bf16 ipc_combine<Bf16, IPC_MAX>(Bf16 a, Bf16 b) { return bf2f(a.v) >= bf2f(b.v) ? a : b; }
template <>
__device__ __forceinline__ Bf16 ipc_combine<Bf16, IPC_MIN>(Bf16 a, Bf16 b) { return bf2f(a.v) <= bf2f(b.v) ? a : b; }

template <typename T, int OP>
__global__ __launch_bounds__(256) void ipc_oneshot_kernel(IpcRaw p, int rank, int world, const T* in,
                                                          T* __restrict__ out, int64_t n, int root, uint32_t epoch,
                                                          int* err, uint32_t spin_limit) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (OP != IPC_COPY || rank == root) {
    T* mine = (T*)p.data[rank];
    for (int64_t i = t0; i < n; i += step) mine[i] = in[i];
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  if (OP == IPC_COPY && rank == root) return;  // the root's tensor is the source
  for (int64_t i = t0; i < n; i += step) {
    if constexpr (OP == IPC_COPY) {
      out[i] = __builtin_nontemporal_load((const T*)p.data[root] + i);
    } else if constexpr (sizeof(T) == 2) {  // Bf16: plain loads (no 2-byte non-temporal struct load)
      T v = ((const T*)p.data[0])[i];
#pragma unroll 1
      for (int q = 1; q < world; ++q) v = ipc_combine<T, OP>(v, ((const T*)p.data[q])[i]);
      out[i] = v;
    } else {
      T v = __builtin_nontemporal_load((const T*)p.data[0] + i);
#pragma unroll 1
      for (int q = 1; q < world; ++q) v = ipc_combine<T, OP>(v, __builtin_nontemporal_load((const T*)p.data[q] + i));
      out[i] = v;
    }
  }
}

template <typename T, int OP>
void launch_oneshot(const IpcRaw& p, int rank, int world, const void* in, void* out, int64_t n, int root,
                    uint32_t epoch, int* err, uint32_t spin_limit, hipStream_t st) {
  hipLaunchKernelGGL((ipc_oneshot_kernel<T, OP>), dim3(ipc_grid(n)), dim3(256), 0, st, p, rank, world, (const T*)in,
                     (T*)out, n, root, epoch, err, spin_limit);
}

template <typename T>
int dispatch_oneshot(int op, const IpcRaw& p, int rank, int world, const void* in, void* out, int64_t n, int root,
                     uint32_t epoch, int* err, uint32_t spin_limit, hipStream_t st) {
  switch (op) {
    case IPC_SUM: launch_oneshot<T, IPC_SUM>(p, rank, world, in, out, n, root, epoch, err, spin_limit, st); break;
    case IPC_MAX: launch_oneshot<T, IPC_MAX>(p, rank, world, in, out, n, root, epoch, err, spin_limit, st); break;
    case IPC_MIN: launch_oneshot<T, IPC_MIN>(p, rank, world, in, out, n, root, epoch, err, spin_limit, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------- mesh reduce-scatter / all-gather (balanced shards)
// SURVEY.md §2.4 / §5.8, SMDDP's "every GPU owns one shard of the fused gradient buffer".  Each rank
// pulls only ITS 1/world of every peer's data, straight over the link to that peer, so the 7 links
// of an MI355X each carry one shard at the same time -- no ring, no multi-hop forwarding.
//   reduce-scatter: copy-in packs the input's `world` pieces (piece q at in + q * in_stride, c
//       elements each, destined for rank q) into the slot at q * c; rank r sums piece r over all
//       slots (fp32 accumulation, rank order) into out[0, c);
//   all-gather: copy-in puts this rank's piece into its slot; rank r copies every rank q's slot into
//       out[q * stride, q * stride + c).
__device__ __forceinline__ float ld_f(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float ld_f(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void st_f(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_f(bf16_t* p, float v) { *p = f2bf(v); }

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ipc_rs_kernel(IpcRaw p, int rank, int world, const T* in, int64_t in_stride,
                                                     T* __restrict__ out, int64_t c, float scale, uint32_t epoch,
                                                     int* err, uint32_t spin_limit) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  T* mine = (T*)p.data[rank];
  for (int q = 0; q < world; ++q) {
    if constexpr (VEC) {
      for (int64_t i = 4 * t0; i < c; i += 4 * step)
        *(f32x4*)((float*)mine + q * c + i) = *(const f32x4*)((const float*)in + q * in_stride + i);
    } else {
      for (int64_t i = t0; i < c; i += step) mine[q * c + i] = in[q * in_stride + i];
    }
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  const int64_t base = (int64_t)rank * c;
  if constexpr (VEC) {
    for (int64_t i = 4 * t0; i < c; i += 4 * step) {
      f32x4 s = __builtin_nontemporal_load((const f32x4*)((const float*)p.data[0] + base + i));
#pragma unroll 1
      for (int q = 1; q < world; ++q) s += __builtin_nontemporal_load((const f32x4*)((const float*)p.data[q] + base + i));
      *(f32x4*)((float*)out + i) = s * scale;
    }
  } else {
    for (int64_t i = t0; i < c; i += step) {
      float s = 0.f;
#pragma unroll 1
      for (int q = 0; q < world; ++q) s += ld_f((const T*)p.data[q] + base + i);
      st_f(out + i, s * scale);
    }
  }
}

template <typename W>
__global__ __launch_bounds__(256) void ipc_ag_kernel(IpcRaw p, int rank, int world, const W* in, W* __restrict__ out,
                                                     int64_t c, int64_t stride, uint32_t epoch, int* err,
                                                     uint32_t spin_limit) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  W* mine = (W*)p.data[rank];
  for (int64_t i = t0; i < c; i += step) mine[i] = in[i];
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  for (int q = 0; q < world; ++q) {
    const W* src = (const W*)p.data[q];
    W* dst = out + (int64_t)q * stride;
    for (int64_t i = t0; i < c; i += step) dst[i] = __builtin_nontemporal_load(src + i);
  }
}

bool make_peers(IpcRaw& p, const void* const* data, uint32_t* const* flags, int world) {
  bool al16 = true;
  for (int q = 0; q < world; ++q) {
    p.data[q] = data[q];
    p.flags[q] = flags[q];
    al16 = al16 && ((uintptr_t)data[q] & 15) == 0;
  }
  return al16;
}

}  // namespace

MI_API int mi_ipc_max_peers() { return IPC_MAX_PEERS; }

// bytes of every rank's flag array (allocated fine-grained / uncached by the backend, zeroed)
MI_API int64_t mi_ipc_flag_bytes() { return (int64_t)IPC_FLAG_WORDS * 4; }

// data: per-rank pointer to THIS call's slot; flags: per-rank flag arrays; in: this rank's input
// (copied into its slot by the kernel); out may alias in; err: host-mapped int.
MI_API int mi_ipc_allreduce_f32(const float* const* data, uint32_t* const* flags, int rank, int world, const float* in,
                                float* out, int64_t n, uint32_t epoch, float scale, int* err, uint32_t spin_limit,
                                hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || n < 0) return (int)hipErrorInvalidValue;
  IpcRaw p{};
  const bool vec = make_peers(p, (const void* const*)data, flags, world) && n % 4 == 0 &&
                   ((uintptr_t)out & 15) == 0 && ((uintptr_t)in & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(ipc_allreduce_kernel<true>, dim3(ipc_grid(n / 4)), dim3(256), 0, st, p, rank, world, in, out,
                       n, epoch, scale, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_allreduce_kernel<false>, dim3(ipc_grid(n)), dim3(256), 0, st, p, rank, world, in, out, n,
                       epoch, scale, err, spin_limit);
  return (int)hipGetLastError();
}

// Two-shot all-reduce; same arguments and slot / flag protocol as mi_ipc_allreduce_f32 (a call is
// either one-shot or two-shot on every rank, chosen by size).
MI_API int mi_ipc_allreduce2_f32(const float* const* data, uint32_t* const* flags, int rank, int world,
                                 const float* in, float* out, int64_t n, uint32_t epoch, float scale, int* err,
                                 uint32_t spin_limit, hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || n < 0) return (int)hipErrorInvalidValue;
  IpcRaw p{};
  const bool vec = make_peers(p, (const void* const*)data, flags, world) && n % 4 == 0 &&
                   ((uintptr_t)out & 15) == 0 && ((uintptr_t)in & 15) == 0;
  const int64_t shard = ((n + world - 1) / world + 3) & ~(int64_t)3;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(IPC_MAX_BLOCKS, MI_IPC_MAX_GRID),
                                                                  (shard + 2047) / 2048));
  const int64_t chunk = ((shard + blocks - 1) / blocks + 3) & ~(int64_t)3;
  if (vec)
    hipLaunchKernelGGL(ipc_allreduce2_kernel<true>, dim3(blocks), dim3(256), 0, st, p, rank, world, in, out, n, shard,
                       chunk, epoch, scale, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_allreduce2_kernel<false>, dim3(blocks), dim3(256), 0, st, p, rank, world, in, out, n,
                       shard, chunk, epoch, scale, err, spin_limit);
  return (int)hipGetLastError();
}

// dtype: 0 f32, 1 f64, 2 i32, 3 i64, 4 bf16 (ignored for COPY); op: 0 SUM, 1 MAX, 2 MIN, 3 COPY (root's slot);
// nbytes: bytes of this call's payload (0 = barrier); in: this rank's input (the root's for COPY).
MI_API int mi_ipc_oneshot(const void* const* data, uint32_t* const* flags, int rank, int world, const void* in,
                          void* out, int64_t nbytes, int dtype, int op, int root, uint32_t epoch, int* err,
                          uint32_t spin_limit, hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || nbytes < 0 || root < 0 || root >= world ||
      op < 0 || op > IPC_COPY)
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  const bool al16 = make_peers(p, data, flags, world) && ((uintptr_t)out & 15) == 0 && ((uintptr_t)in & 15) == 0;
  if (op == IPC_COPY) {
    if (al16 && nbytes % 16 == 0)
      launch_oneshot<u32x4, IPC_COPY>(p, rank, world, in, out, nbytes / 16, root, epoch, err, spin_limit, st);
    else if (nbytes % 4 == 0)
      launch_oneshot<uint32_t, IPC_COPY>(p, rank, world, in, out, nbytes / 4, root, epoch, err, spin_limit, st);
    else
      launch_oneshot<uint8_t, IPC_COPY>(p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    return (int)hipGetLastError();
  }
  switch (dtype) {
    case 0: return dispatch_oneshot<float>(op, p, rank, world, in, out, nbytes / 4, root, epoch, err, spin_limit, st);
    case 1: return dispatch_oneshot<double>(op, p, rank, world, in, out, nbytes / 8, root, epoch, err, spin_limit, st);
    case 2: return dispatch_oneshot<int32_t>(op, p, rank, world, in, out, nbytes / 4, root, epoch, err, spin_limit, st);
    case 3: return dispatch_oneshot<int64_t>(op, p, rank, world, in, out, nbytes / 8, root, epoch, err, spin_limit, st);
    case 4: return dispatch_oneshot<Bf16>(op, p, rank, world, in, out, nbytes / 2, root, epoch, err, spin_limit, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// c: elements of the output piece; in: this rank's `world` pieces, piece q at in + q * in_stride;
// dtype 0 f32, 4 bf16; scale 1/world for AVG.  Every rank's slot must hold world * c elements.
MI_API int mi_ipc_reduce_scatter(const void* const* data, uint32_t* const* flags, int rank, int world, const void* in,
                                 int64_t in_stride, void* out, int64_t c, int dtype, float scale, uint32_t epoch,
                                 int* err, uint32_t spin_limit, hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || c < 0 || in_stride < c ||
      (dtype != 0 && dtype != 4))
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  const bool vec = make_peers(p, data, flags, world) && dtype == 0 && c % 4 == 0 && in_stride % 4 == 0 &&
                   ((uintptr_t)out & 15) == 0 && ((uintptr_t)in & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((ipc_rs_kernel<float, true>), dim3(ipc_grid(c / 4)), dim3(256), 0, st, p, rank, world,
                       (const float*)in, in_stride, (float*)out, c, scale, epoch, err, spin_limit);
  else if (dtype == 0)
    hipLaunchKernelGGL((ipc_rs_kernel<float, false>), dim3(ipc_grid(c)), dim3(256), 0, st, p, rank, world,
                       (const float*)in, in_stride, (float*)out, c, scale, epoch, err, spin_limit);
  else
    hipLaunchKernelGGL((ipc_rs_kernel<bf16_t, false>), dim3(ipc_grid(c)), dim3(256), 0, st, p, rank, world,
                       (const bf16_t*)in, in_stride, (bf16_t*)out, c, scale, epoch, err, spin_limit);
  return (int)hipGetLastError();
}

// nbytes: bytes of every rank's piece; in: this rank's piece; stride_bytes: distance between
// consecutive ranks' pieces in `out`.  Any dtype (a byte copy); `in` may lie inside `out`.
MI_API int mi_ipc_all_gather(const void* const* data, uint32_t* const* flags, int rank, int world, const void* in,
                             void* out, int64_t nbytes, int64_t stride_bytes, uint32_t epoch, int* err,
                             uint32_t spin_limit, hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || nbytes < 0 || stride_bytes < nbytes)
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  const bool al = make_peers(p, data, flags, world);
  const bool al16 = al && ((uintptr_t)out & 15) == 0 && ((uintptr_t)in & 15) == 0 && nbytes % 16 == 0 &&
                    stride_bytes % 16 == 0;
  const bool al4 = ((uintptr_t)out & 3) == 0 && ((uintptr_t)in & 3) == 0 && nbytes % 4 == 0 && stride_bytes % 4 == 0;
  if (al16)
    hipLaunchKernelGGL(ipc_ag_kernel<u32x4>, dim3(ipc_grid(nbytes / 16)), dim3(256), 0, st, p, rank, world,
                       (const u32x4*)in, (u32x4*)out, nbytes / 16, stride_bytes / 16, epoch, err, spin_limit);
  else if (al4)
    hipLaunchKernelGGL(ipc_ag_kernel<uint32_t>, dim3(ipc_grid(nbytes / 4)), dim3(256), 0, st, p, rank, world,
                       (const uint32_t*)in, (uint32_t*)out, nbytes / 4, stride_bytes / 4, epoch, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_ag_kernel<uint8_t>, dim3(ipc_grid(nbytes)), dim3(256), 0, st, p, rank, world,
                       (const uint8_t*)in, (uint8_t*)out, nbytes, stride_bytes, epoch, err, spin_limit);
  return (int)hipGetLastError();
}
