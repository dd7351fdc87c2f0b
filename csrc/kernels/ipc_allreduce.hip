// One-shot and two-shot all-reduce over IPC peer pointers (SURVEY.md §2.3 N4,
// §5.8: "a one-shot IPC all-reduce kernel (peer-pointer loads) to cut latency").  Used by the
// native smddp backend (csrc/comm/smddp_backend.cpp) for small fp32 all-reduces when
// MI355X_DP_SMDDP_IPC=1; RCCL stays the path for everything else.
//
// Every rank owns one IPC-exported buffer: two data slots (alternating by call parity) and a
// flag word per peer.  Per call:
//   1. (host, same stream) the rank copies its input into slot[epoch & 1] of its own buffer;
//   2. block 0 publishes it: system-scope fence, then writes `epoch` into flag[rank] of every
//      peer's buffer (release, system scope -- over xGMI for other GPUs);
//   3. every block waits until all of its own flags are >= epoch (peers may already be one call
//      ahead), spinning with system-scope acquire loads and s_sleep, bounded: on timeout it
//      raises the host-visible error word and leaves the output untouched -- never a hang;
//   4. every rank sums all peers' slots (system-scope loads: peer lines must not come from a
//      stale local L2 copy of the previous call) into the output, times `scale` (1/world: AVG).
// Slot reuse is safe without an end barrier: a rank rewrites slot[e & 1] only at call e+2, after
// its call e+1 completed, which needed every peer's e+1 flag, which each peer raises only after
// finishing its own call e (stream order).
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

struct IpcPeers {
  const float* data[IPC_MAX_PEERS];  // this call's slot in every rank's buffer
  uint32_t* flags[IPC_MAX_PEERS];    // every rank's flag array (world words)
};

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcPeers p, int rank, int world, float* __restrict__ out,
                                                            int64_t n, uint32_t epoch, float scale, int* err,
                                                            uint32_t spin_limit) {
  __shared__ int ok;
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)world) {
    __threadfence_system();
    __hip_atomic_store(p.flags[threadIdx.x] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    int good = 1;
    uint32_t spins = 0;
    for (int q = 0; q < world && good; ++q) {
      while ((int32_t)(__hip_atomic_load(p.flags[rank] + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) <
             0) {
        if (++spins > spin_limit) { good = 0; break; }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    if (!good) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = good;
  }
  __syncthreads();
  if (!ok) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
#pragma unroll 1
    for (int q = 0; q < world; ++q)
      s += __hip_atomic_load(p.data[q] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    out[i] = s * scale;
  }
}

// ---------------------------------------------------------------------------------------------
// Two-shot (reduce-scatter + all-gather) variant for bandwidth-bound buckets: every rank reads
// (world-1)/world of the data from peers twice instead of (world-1) x all of it once, so over 7
// point-to-point xGMI links each link carries 2/world of the bucket instead of all of it.
//   phase 1: wait for every peer's input flag (as above); block b sums chunk b of this rank's
//            shard over all peers' slots and writes the scaled sum into its OWN slot (peers read
//            this rank's slot only at their own shard range in phase 1, never at this one) and
//            into `out`; then a system-scope release and flag2[rank][b] = epoch on every peer;
//   phase 2: block b waits for flag2[q][b] from every peer and copies chunk b of shard q from
//            peer q's slot into `out`.
// Only blocks with the same index talk to each other (no grid barrier, no co-residency
// assumption).  Reads of peer slots follow a system-scope acquire by thread 0 (L1/L2
// invalidation for the CU / XCD) and use non-temporal loads.
// Flag region per rank: [0, IPC_MAX_PEERS) input flags, then IPC_FLAG2_OFF + src * IPC_MAX_BLOCKS2 + b.
constexpr int IPC_MAX_BLOCKS2 = 256;
constexpr int IPC_FLAG2_OFF = 256;

__device__ __forceinline__ bool ipc_wait_ge(uint32_t* f, uint32_t epoch, uint32_t spin_limit, uint32_t& spins) {
  while ((int32_t)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
    if (++spins > spin_limit) return false;
    __builtin_amdgcn_s_sleep(8);
  }
  return true;
}

template <bool VEC>
__device__ __forceinline__ void ipc_sum_chunk(const IpcPeers& p, int world, float* mine, float* out, int64_t lo,
                                              int64_t hi, float scale) {
  if constexpr (VEC) {
    for (int64_t i = lo + 4 * (int64_t)threadIdx.x; i < hi; i += 4 * (int64_t)blockDim.x) {
      f32x4 s = __builtin_nontemporal_load((const f32x4*)(p.data[0] + i));
#pragma unroll 1
      for (int q = 1; q < world; ++q) s += __builtin_nontemporal_load((const f32x4*)(p.data[q] + i));
      s *= scale;
      *(f32x4*)(mine + i) = s;
      *(f32x4*)(out + i) = s;
    }
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float s = 0.f;
#pragma unroll 1
      for (int q = 0; q < world; ++q) s += __builtin_nontemporal_load(p.data[q] + i);
      mine[i] = s * scale;
      out[i] = s * scale;
    }
  }
}

template <bool VEC>
__device__ __forceinline__ void ipc_copy_chunk(const float* src, float* out, int64_t lo, int64_t hi) {
  if constexpr (VEC) {
    for (int64_t i = lo + 4 * (int64_t)threadIdx.x; i < hi; i += 4 * (int64_t)blockDim.x)
      *(f32x4*)(out + i) = __builtin_nontemporal_load((const f32x4*)(src + i));
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = __builtin_nontemporal_load(src + i);
  }
}

// shard = ceil(n / world) rounded up to 4 elements; chunk = ceil(shard / gridDim.x) rounded to 4
template <bool VEC>
__global__ __launch_bounds__(256) void ipc_allreduce2_kernel(IpcPeers p, int rank, int world, float* __restrict__ out,
                                                             int64_t n, int64_t shard, int64_t chunk, uint32_t epoch,
                                                             float scale, int* err, uint32_t spin_limit) {
  __shared__ int ok;
  const int b = blockIdx.x;
  if (b == 0 && threadIdx.x < (unsigned)world) {
    __threadfence_system();
    __hip_atomic_store(p.flags[threadIdx.x] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    uint32_t spins = 0;
    bool good = true;
    for (int q = 0; q < world && good; ++q) good = ipc_wait_ge(p.flags[rank] + q, epoch, spin_limit, spins);
    if (!good) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = good;
  }
  __syncthreads();
  if (!ok) return;
  // phase 1: reduce chunk b of this rank's shard
  {
    const int64_t lo = min(n, rank * shard + b * chunk);
    const int64_t hi = min(min(n, (rank + 1) * shard), lo + chunk);
    ipc_sum_chunk<VEC>(p, world, (float*)p.data[rank], out, lo, hi, scale);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();  // this block's sums (in this XCD's L2) reach memory before the flags
    for (int q = 0; q < world; ++q)
      if (q != rank)
        __hip_atomic_store(p.flags[q] + IPC_FLAG2_OFF + rank * IPC_MAX_BLOCKS2 + b, epoch, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t spins = 0;
    bool good = true;
    for (int q = 0; q < world && good; ++q)
      if (q != rank) good = ipc_wait_ge(p.flags[rank] + IPC_FLAG2_OFF + q * IPC_MAX_BLOCKS2 + b, epoch, spin_limit, spins);
    if (!good) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = good;
  }
  __syncthreads();
  if (!ok) return;
  // phase 2: gather chunk b of every other shard
  for (int q = 0; q < world; ++q) {
    if (q == rank) continue;
    const int64_t lo = min(n, q * shard + b * chunk);
    const int64_t hi = min(min(n, (q + 1) * shard), lo + chunk);
    ipc_copy_chunk<VEC>(p.data[q], out, lo, hi);
  }
}

}  // namespace

MI_API int mi_ipc_max_peers() { return IPC_MAX_PEERS; }

// bytes of flag words every rank's IPC buffer must provide after its two data slots
MI_API int64_t mi_ipc_flag_bytes() { return (int64_t)(IPC_FLAG2_OFF + IPC_MAX_PEERS * IPC_MAX_BLOCKS2) * 4; }

// Two-shot all-reduce; same arguments and slot / flag protocol as mi_ipc_allreduce_f32 (the
// input flags are shared: a call is either one-shot or two-shot on every rank, by size).
MI_API int mi_ipc_allreduce2_f32(const float* const* data, uint32_t* const* flags, int rank, int world, float* out,
                                 int64_t n, uint32_t epoch, float scale, int* err, uint32_t spin_limit,
                                 hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || n < 0) return (int)hipErrorInvalidValue;
  IpcPeers p{};
  bool vec = n % 4 == 0 && ((uintptr_t)out & 15) == 0;
  for (int q = 0; q < world; ++q) {
    p.data[q] = data[q];
    p.flags[q] = flags[q];
    vec = vec && ((uintptr_t)data[q] & 15) == 0;
  }
  const int64_t shard = ((n + world - 1) / world + 3) & ~(int64_t)3;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(IPC_MAX_BLOCKS2, MI_IPC_MAX_GRID),
                                                                  (shard + 2047) / 2048));
  const int64_t chunk = ((shard + blocks - 1) / blocks + 3) & ~(int64_t)3;
  if (vec)
    hipLaunchKernelGGL(ipc_allreduce2_kernel<true>, dim3(blocks), dim3(256), 0, st, p, rank, world, out, n, shard,
                       chunk, epoch, scale, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_allreduce2_kernel<false>, dim3(blocks), dim3(256), 0, st, p, rank, world, out, n, shard,
                       chunk, epoch, scale, err, spin_limit);
  return (int)hipGetLastError();
}

// data: per-rank pointer to THIS call's slot; flags: per-rank flag arrays; err: host-mapped int.
MI_API int mi_ipc_allreduce_f32(const float* const* data, uint32_t* const* flags, int rank, int world, float* out,
                                int64_t n, uint32_t epoch, float scale, int* err, uint32_t spin_limit,
                                hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || n < 0) return (int)hipErrorInvalidValue;
  IpcPeers p{};
  for (int q = 0; q < world; ++q) { p.data[q] = data[q]; p.flags[q] = flags[q]; }
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(MI_IPC_MAX_GRID, (n + 255) / 256));
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(blocks), dim3(256), 0, st, p, rank, world, out, n, epoch, scale, err,
                     spin_limit);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Generic one-shot collective over the same slots / flags, for the smddp backend's IPC-only mode
// (MI355X_DP_SMDDP_IPC_ONLY=1: no RCCL communicator at all -- single-node xGMI, and several ranks
// may share one GPU for rehearsals): op SUM / MAX / MIN over f32 / f64 / i32 / i64, COPY = every
// rank takes the root's slot (broadcast), and a zero-byte call is a barrier (flag round only).
namespace {

enum { IPC_SUM = 0, IPC_MAX = 1, IPC_MIN = 2, IPC_COPY = 3 };

struct IpcRaw {
  const void* data[IPC_MAX_PEERS];
  uint32_t* flags[IPC_MAX_PEERS];
};

__device__ __forceinline__ bool ipc_handshake(const IpcRaw& p, int rank, int world, uint32_t epoch, int* err,
                                              uint32_t spin_limit) {
  __shared__ int ok;
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)world) {
    __threadfence_system();
    __hip_atomic_store(p.flags[threadIdx.x] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    uint32_t spins = 0;
    bool good = true;
    for (int q = 0; q < world && good; ++q) good = ipc_wait_ge(p.flags[rank] + q, epoch, spin_limit, spins);
    if (!good) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

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
__global__ __launch_bounds__(256) void ipc_oneshot_kernel(IpcRaw p, int rank, int world, T* __restrict__ out,
                                                          int64_t n, int root, uint32_t epoch, int* err,
                                                          uint32_t spin_limit) {
  if (!ipc_handshake(p, rank, world, epoch, err, spin_limit)) return;
  if (OP == IPC_COPY && rank == root) return;  // the root's tensor is the source
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
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
void launch_oneshot(const IpcRaw& p, int rank, int world, void* out, int64_t n, int root, uint32_t epoch, int* err,
                    uint32_t spin_limit, hipStream_t st) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(MI_IPC_MAX_GRID, (n + 255) / 256));
  hipLaunchKernelGGL((ipc_oneshot_kernel<T, OP>), dim3(blocks), dim3(256), 0, st, p, rank, world, (T*)out, n, root,
                     epoch, err, spin_limit);
}

template <typename T>
int dispatch_oneshot(int op, const IpcRaw& p, int rank, int world, void* out, int64_t n, int root, uint32_t epoch,
                     int* err, uint32_t spin_limit, hipStream_t st) {
  switch (op) {
    case IPC_SUM: launch_oneshot<T, IPC_SUM>(p, rank, world, out, n, root, epoch, err, spin_limit, st); break;
    case IPC_MAX: launch_oneshot<T, IPC_MAX>(p, rank, world, out, n, root, epoch, err, spin_limit, st); break;
    case IPC_MIN: launch_oneshot<T, IPC_MIN>(p, rank, world, out, n, root, epoch, err, spin_limit, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

// dtype: 0 f32, 1 f64, 2 i32, 3 i64, 4 bf16 (ignored for COPY); op: 0 SUM, 1 MAX, 2 MIN, 3 COPY (root's slot);
// nbytes: bytes of this call's slot payload (0 = barrier).  Same slot / flag protocol and epochs as
// mi_ipc_allreduce_f32.
MI_API int mi_ipc_oneshot(const void* const* data, uint32_t* const* flags, int rank, int world, void* out,
                          int64_t nbytes, int dtype, int op, int root, uint32_t epoch, int* err, uint32_t spin_limit,
                          hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || nbytes < 0 || root < 0 || root >= world ||
      op < 0 || op > IPC_COPY)
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  bool al16 = ((uintptr_t)out & 15) == 0;
  for (int q = 0; q < world; ++q) {
    p.data[q] = data[q];
    p.flags[q] = flags[q];
    al16 = al16 && ((uintptr_t)data[q] & 15) == 0;
  }
  if (op == IPC_COPY) {
    if (al16 && nbytes % 16 == 0)
      launch_oneshot<u32x4, IPC_COPY>(p, rank, world, out, nbytes / 16, root, epoch, err, spin_limit, st);
    else if (nbytes % 4 == 0)
      launch_oneshot<uint32_t, IPC_COPY>(p, rank, world, out, nbytes / 4, root, epoch, err, spin_limit, st);
    else
      launch_oneshot<uint8_t, IPC_COPY>(p, rank, world, out, nbytes, root, epoch, err, spin_limit, st);
    return (int)hipGetLastError();
  }
  switch (dtype) {
    case 0: return dispatch_oneshot<float>(op, p, rank, world, out, nbytes / 4, root, epoch, err, spin_limit, st);
    case 1: return dispatch_oneshot<double>(op, p, rank, world, out, nbytes / 8, root, epoch, err, spin_limit, st);
    case 2: return dispatch_oneshot<int32_t>(op, p, rank, world, out, nbytes / 4, root, epoch, err, spin_limit, st);
    case 3: return dispatch_oneshot<int64_t>(op, p, rank, world, out, nbytes / 8, root, epoch, err, spin_limit, st);
    case 4: return dispatch_oneshot<Bf16>(op, p, rank, world, out, nbytes / 2, root, epoch, err, spin_limit, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------
// Reduce-scatter and all-gather over the same slots / flags: balanced shards over the xGMI mesh
// (SMDDP's "every GPU owns one shard of the fused gradient buffer").  Each
// rank pulls only ITS 1/world of every peer's data, straight over the link to that peer, so the 7
// links of an MI355X each carry one shard at the same time -- no ring, no multi-hop forwarding.
//   reduce-scatter: a rank's slot holds its input re-packed as `world` pieces of `c` elements
//       (piece q is destined for rank q); rank r sums piece r over all slots (fp32 accumulation,
//       rank order) into out[0, c);
//   all-gather: a rank's slot holds its own piece; rank r copies every rank q's slot into
//       out[q * stride, q * stride + c).
// Slot reuse follows the one-shot argument above (a slot is rewritten two calls later, after
// every peer has raised the intermediate call's input flag).
namespace {

__device__ __forceinline__ float ld_f(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float ld_f(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void st_f(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_f(bf16_t* p, float v) { *p = f2bf(v); }

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ipc_rs_kernel(IpcRaw p, int rank, int world, T* __restrict__ out, int64_t c,
                                                     float scale, uint32_t epoch, int* err, uint32_t spin_limit) {
  if (!ipc_handshake(p, rank, world, epoch, err, spin_limit)) return;
  const int64_t base = (int64_t)rank * c;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  if constexpr (VEC) {
    for (int64_t i = 4 * (blockIdx.x * (int64_t)blockDim.x + threadIdx.x); i < c; i += 4 * step) {
      f32x4 s = __builtin_nontemporal_load((const f32x4*)((const float*)p.data[0] + base + i));
#pragma unroll 1
      for (int q = 1; q < world; ++q) s += __builtin_nontemporal_load((const f32x4*)((const float*)p.data[q] + base + i));
      *(f32x4*)((float*)out + i) = s * scale;
    }
  } else {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c; i += step) {
      float s = 0.f;
#pragma unroll 1
      for (int q = 0; q < world; ++q) s += ld_f((const T*)p.data[q] + base + i);
      st_f(out + i, s * scale);
    }
  }
}

template <typename W>
__global__ __launch_bounds__(256) void ipc_ag_kernel(IpcRaw p, int rank, int world, W* __restrict__ out, int64_t c,
                                                     int64_t stride, uint32_t epoch, int* err, uint32_t spin_limit) {
  if (!ipc_handshake(p, rank, world, epoch, err, spin_limit)) return;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int q = 0; q < world; ++q) {
    const W* src = (const W*)p.data[q];
    W* dst = out + (int64_t)q * stride;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c; i += step)
      dst[i] = __builtin_nontemporal_load(src + i);
  }
}

int ipc_grid(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>(MI_IPC_MAX_GRID, (work + 255) / 256)); }

}  // namespace

// c: elements of the output piece; dtype 0 f32, 4 bf16; scale 1/world for AVG.  Every rank's slot
// must hold world * c elements (piece q at q * c) before the call.
MI_API int mi_ipc_reduce_scatter(const void* const* data, uint32_t* const* flags, int rank, int world, void* out,
                                 int64_t c, int dtype, float scale, uint32_t epoch, int* err, uint32_t spin_limit,
                                 hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || c < 0 || (dtype != 0 && dtype != 4))
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  bool vec = dtype == 0 && c % 4 == 0 && ((uintptr_t)out & 15) == 0;
  for (int q = 0; q < world; ++q) {
    p.data[q] = data[q];
    p.flags[q] = flags[q];
    vec = vec && ((uintptr_t)data[q] & 15) == 0;
  }
  if (vec)
    hipLaunchKernelGGL((ipc_rs_kernel<float, true>), dim3(ipc_grid(c / 4)), dim3(256), 0, st, p, rank, world,
                       (float*)out, c, scale, epoch, err, spin_limit);
  else if (dtype == 0)
    hipLaunchKernelGGL((ipc_rs_kernel<float, false>), dim3(ipc_grid(c)), dim3(256), 0, st, p, rank, world,
                       (float*)out, c, scale, epoch, err, spin_limit);
  else
    hipLaunchKernelGGL((ipc_rs_kernel<bf16_t, false>), dim3(ipc_grid(c)), dim3(256), 0, st, p, rank, world,
                       (bf16_t*)out, c, scale, epoch, err, spin_limit);
  return (int)hipGetLastError();
}

// nbytes: bytes of every rank's piece (its slot payload); stride_bytes: distance between
// consecutive ranks' pieces in `out`.  Any dtype (a byte copy).
MI_API int mi_ipc_all_gather(const void* const* data, uint32_t* const* flags, int rank, int world, void* out,
                             int64_t nbytes, int64_t stride_bytes, uint32_t epoch, int* err, uint32_t spin_limit,
                             hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || nbytes < 0 || stride_bytes < nbytes)
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  bool al16 = ((uintptr_t)out & 15) == 0 && nbytes % 16 == 0 && stride_bytes % 16 == 0;
  bool al4 = ((uintptr_t)out & 3) == 0 && nbytes % 4 == 0 && stride_bytes % 4 == 0;
  for (int q = 0; q < world; ++q) {
    p.data[q] = data[q];
    p.flags[q] = flags[q];
    al16 = al16 && ((uintptr_t)data[q] & 15) == 0;
  }
  if (al16)
    hipLaunchKernelGGL(ipc_ag_kernel<u32x4>, dim3(ipc_grid(nbytes / 16)), dim3(256), 0, st, p, rank, world,
                       (u32x4*)out, nbytes / 16, stride_bytes / 16, epoch, err, spin_limit);
  else if (al4)
    hipLaunchKernelGGL(ipc_ag_kernel<uint32_t>, dim3(ipc_grid(nbytes / 4)), dim3(256), 0, st, p, rank, world,
                       (uint32_t*)out, nbytes / 4, stride_bytes / 4, epoch, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_ag_kernel<uint8_t>, dim3(ipc_grid(nbytes)), dim3(256), 0, st, p, rank, world,
                       (uint8_t*)out, nbytes, stride_bytes, epoch, err, spin_limit);
  return (int)hipGetLastError();
}
