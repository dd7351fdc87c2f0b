// One-shot all-reduce over IPC peer pointers for latency-bound buckets (SURVEY.md §2.3 N4,
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

}  // namespace

MI_API int mi_ipc_max_peers() { return IPC_MAX_PEERS; }

// data: per-rank pointer to THIS call's slot; flags: per-rank flag arrays; err: host-mapped int.
MI_API int mi_ipc_allreduce_f32(const float* const* data, uint32_t* const* flags, int rank, int world, float* out,
                                int64_t n, uint32_t epoch, float scale, int* err, uint32_t spin_limit,
                                hipStream_t st) {
  if (world < 1 || world > IPC_MAX_PEERS || rank < 0 || rank >= world || n < 0) return (int)hipErrorInvalidValue;
  IpcPeers p{};
  for (int q = 0; q < world; ++q) { p.data[q] = data[q]; p.flags[q] = flags[q]; }
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(256, (n + 255) / 256));
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(blocks), dim3(256), 0, st, p, rank, world, out, n, epoch, scale, err,
                     spin_limit);
  return (int)hipGetLastError();
}
