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
// Protocol of one call (epoch e, this rank r, block b; every rank launches the same grid and cuts
// the payload into the same 16-byte units per block, both from the payload size alone):
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
namespace {

constexpr int kIpcMaxGrid = 64;

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
  return (int)std::max<int64_t>(1, std::min<int64_t>(kIpcMaxGrid, (work + 255) / 256));
}

// ------------------------------------------------------------------ partition of a payload
// Every one-shot kernel below cuts its payload into 16-byte units; unit u is moved by thread
// u mod (grid x 256), so the block that copies a unit in, releases it and reads it back on every
// rank is a function of the payload size alone (the grid is too).  Where THIS rank's tensor sits
// only picks how the owning thread moves the bytes (one 16-byte access, dwords, or bytes): ranks
// whose tensors differ in alignment still cut the payload identically (an alignment-
// chosen vector width used to change the grid and the block-to-element map per rank).
__device__ __forceinline__ void unit_copy(char* dst, const char* src, int bytes) {
  if (bytes == 16 && (((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    *(u32x4*)dst = *(const u32x4*)src;
  } else if (((bytes | (int)(uintptr_t)dst | (int)(uintptr_t)src) & 3) == 0) {
    for (int i = 0; i < bytes; i += 4) *(uint32_t*)(dst + i) = *(const uint32_t*)(src + i);
  } else {
    for (int i = 0; i < bytes; ++i) dst[i] = src[i];
  }
}

// a unit held in registers, stored to a local tensor
__device__ __forceinline__ void unit_put(char* dst, u32x4 w, int bytes) {
  if (bytes == 16 && ((uintptr_t)dst & 15) == 0) {
    *(u32x4*)dst = w;
  } else if (((bytes | (int)(uintptr_t)dst) & 3) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * i < bytes) *(uint32_t*)(dst + 4 * i) = w[i];
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < bytes) dst[i] = (char)(w[i >> 2] >> (8 * (i & 3)));
  }
}

// a unit of a peer's slot: slots and unit offsets are 16-byte aligned (slot bytes past the payload
// are read but never stored anywhere)
__device__ __forceinline__ u32x4 slot_unit(const void* slot, int64_t u) {
  return __builtin_nontemporal_load((const u32x4*)slot + u);
}

template <typename T>
__device__ __forceinline__ void unit_store(T* dst, const T (&v)[16 / sizeof(T)], int bytes) {
  constexpr int E = 16 / sizeof(T);
  if (bytes == 16 && ((uintptr_t)dst & 15) == 0) {
    *(u32x4*)dst = __builtin_bit_cast(u32x4, v);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (e * (int)sizeof(T) < bytes) dst[e] = v[e];
  }
}

__host__ __device__ __forceinline__ int64_t ipc_units(int64_t nbytes) { return (nbytes + 15) / 16; }

// ------------------------------------------------------------------ one-shot fp32 all-reduce
__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcRaw p, int rank, int world, const float* in,
                                                            float* out, int64_t n, uint32_t epoch, float scale,
                                                            int* err, uint32_t spin_limit) {
  char* mine = (char*)p.data[rank];
  const int64_t nb = n * 4, U = ipc_units(nb);
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t u = t0; u < U; u += step)
    unit_copy(mine + 16 * u, (const char*)in + 16 * u, (int)min<int64_t>(16, nb - 16 * u));
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  for (int64_t u = t0; u < U; u += step) {
    f32x4 s = __builtin_bit_cast(f32x4, slot_unit(p.data[0], u));
#pragma unroll 1
    for (int q = 1; q < world; ++q) s += __builtin_bit_cast(f32x4, slot_unit(p.data[q], u));
    s *= scale;
    float v[4] = {s[0], s[1], s[2], s[3]};
    unit_store<float>(out + 4 * u, v, (int)min<int64_t>(16, nb - 16 * u));
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
                                                          T* __restrict__ out, int64_t nbytes, int root,
                                                          uint32_t epoch, int* err, uint32_t spin_limit) {
  constexpr int E = 16 / sizeof(T);
  const int64_t U = ipc_units(nbytes);
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (OP != IPC_COPY || rank == root) {
    char* mine = (char*)p.data[rank];
    for (int64_t u = t0; u < U; u += step)
      unit_copy(mine + 16 * u, (const char*)in + 16 * u, (int)min<int64_t>(16, nbytes - 16 * u));
  }
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  if (OP == IPC_COPY && rank == root) return;  // the root's tensor is the source
  for (int64_t u = t0; u < U; u += step) {
    const int bytes = (int)min<int64_t>(16, nbytes - 16 * u);
    if constexpr (OP == IPC_COPY) {
      unit_put((char*)out + 16 * u, slot_unit(p.data[root], u), bytes);
    } else {
      T v[E];
      *(u32x4*)v = slot_unit(p.data[0], u);
#pragma unroll 1
      for (int q = 1; q < world; ++q) {
        T w[E];
        *(u32x4*)w = slot_unit(p.data[q], u);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = ipc_combine<T, OP>(v[e], w[e]);
      }
      unit_store<T>(out + E * u, v, bytes);
    }
  }
}

template <typename T, int OP>
void launch_oneshot(const IpcRaw& p, int rank, int world, const void* in, void* out, int64_t n, int root,
                    uint32_t epoch, int* err, uint32_t spin_limit, hipStream_t st) {
  // n: payload BYTES (the grid and the unit partition depend on them alone)
  hipLaunchKernelGGL((ipc_oneshot_kernel<T, OP>), dim3(ipc_grid(ipc_units(n))), dim3(256), 0, st, p, rank, world,
                     (const T*)in, (T*)out, n, root, epoch, err, spin_limit);
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
// slot layout of the reduce-scatter: piece q at q * piece_bytes(c), 16-byte aligned
__host__ __device__ __forceinline__ int64_t piece_bytes(int64_t c, int esz) { return (c * esz + 15) & ~(int64_t)15; }

template <typename T>
__global__ __launch_bounds__(256) void ipc_rs_kernel(IpcRaw p, int rank, int world, const T* in, int64_t in_stride,
                                                     T* __restrict__ out, int64_t c, float scale, uint32_t epoch,
                                                     int* err, uint32_t spin_limit) {
  constexpr int E = 16 / sizeof(T);
  const int64_t nb = c * (int64_t)sizeof(T), pb = piece_bytes(c, sizeof(T)), U = ipc_units(nb);
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  char* mine = (char*)p.data[rank];
  for (int q = 0; q < world; ++q)
    for (int64_t u = t0; u < U; u += step)
      unit_copy(mine + q * pb + 16 * u, (const char*)(in + q * in_stride) + 16 * u, (int)min<int64_t>(16, nb - 16 * u));
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  const int64_t ub = rank * pb / 16;  // this rank's piece, in units of every slot
  for (int64_t u = t0; u < U; u += step) {
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll 1
    for (int q = 0; q < world; ++q) {  // fp32 accumulation in rank order
      T w[E];
      *(u32x4*)w = slot_unit(p.data[q], ub + u);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if constexpr (sizeof(T) == 4) acc[e] += w[e];
        else acc[e] += bf2f(w[e]);
      }
    }
    T v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if constexpr (sizeof(T) == 4) v[e] = acc[e] * scale;
      else v[e] = f2bf(acc[e] * scale);
    }
    unit_store<T>(out + E * u, v, (int)min<int64_t>(16, nb - 16 * u));
  }
}

__global__ __launch_bounds__(256) void ipc_ag_kernel(IpcRaw p, int rank, int world, const char* in,
                                                     char* __restrict__ out, int64_t nbytes, int64_t stride,
                                                     uint32_t epoch, int* err, uint32_t spin_limit) {
  const int64_t U = ipc_units(nbytes);
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  char* mine = (char*)p.data[rank];
  for (int64_t u = t0; u < U; u += step)
    unit_copy(mine + 16 * u, in + 16 * u, (int)min<int64_t>(16, nbytes - 16 * u));
  if (!ipc_block_sync(p, rank, world, IPC_FLAG_IN_OFF, false, epoch, err, spin_limit)) return;
  for (int q = 0; q < world; ++q) {
    char* dst = out + (int64_t)q * stride;
    for (int64_t u = t0; u < U; u += step) {
      unit_put(dst + 16 * u, slot_unit(p.data[q], u), (int)min<int64_t>(16, nbytes - 16 * u));
    }
  }
}

// slots must be 16-byte aligned (the backend's hipMalloc'd buffers and 256-byte-rounded slot sizes)
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
  if (!make_peers(p, (const void* const*)data, flags, world)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(ipc_grid(ipc_units(n * 4))), dim3(256), 0, st, p, rank, world, in, out,
                     n, epoch, scale, err, spin_limit);
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
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(IPC_MAX_BLOCKS, kIpcMaxGrid),
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
  if (!make_peers(p, data, flags, world)) return (int)hipErrorInvalidValue;
  if (op == IPC_COPY) {  // a byte copy, whatever the dtype
    launch_oneshot<uint32_t, IPC_COPY>(p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    return (int)hipGetLastError();
  }
  switch (dtype) {
    case 0: return dispatch_oneshot<float>(op, p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    case 1: return dispatch_oneshot<double>(op, p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    case 2: return dispatch_oneshot<int32_t>(op, p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    case 3: return dispatch_oneshot<int64_t>(op, p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    case 4: return dispatch_oneshot<Bf16>(op, p, rank, world, in, out, nbytes, root, epoch, err, spin_limit, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// c: elements of the output piece; in: this rank's `world` pieces, piece q at in + q * in_stride;
// dtype 0 f32, 4 bf16; scale 1/world for AVG.  Every rank's slot must hold world * piece_bytes(c) bytes
// (pieces start 16-byte aligned).
MI_API int mi_ipc_reduce_scatter(const void* const* data, uint32_t* const* flags, int rank, int world, const void* in,
                                 int64_t in_stride, void* out, int64_t c, int dtype, float scale, uint32_t epoch,
                                 int* err, uint32_t spin_limit, hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || c < 0 || in_stride < c ||
      (dtype != 0 && dtype != 4))
    return (int)hipErrorInvalidValue;
  IpcRaw p{};
  if (!make_peers(p, data, flags, world)) return (int)hipErrorInvalidValue;
  const int esz = dtype == 0 ? 4 : 2;
  const dim3 grid(ipc_grid(ipc_units(c * esz)));
  if (dtype == 0)
    hipLaunchKernelGGL(ipc_rs_kernel<float>, grid, dim3(256), 0, st, p, rank, world, (const float*)in, in_stride,
                       (float*)out, c, scale, epoch, err, spin_limit);
  else
    hipLaunchKernelGGL(ipc_rs_kernel<bf16_t>, grid, dim3(256), 0, st, p, rank, world, (const bf16_t*)in, in_stride,
                       (bf16_t*)out, c, scale, epoch, err, spin_limit);
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
  if (!make_peers(p, data, flags, world)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ipc_ag_kernel, dim3(ipc_grid(ipc_units(nbytes))), dim3(256), 0, st, p, rank, world,
                     (const char*)in, (char*)out, nbytes, stride_bytes, epoch, err, spin_limit);
  return (int)hipGetLastError();
}
