// Cross-process step barrier of the IPC transport (csrc/comm/ipc.h): each rank owns one 64-bit flag
// at the head of its peer-mapped window and only ever writes its own flag; peers read it through
// their IPC mapping (same device: another process's view of the same HBM; other device: over xGMI).
//
// The reference orders its ring steps with blocking Gloo send/recv on the host
// (/root/reference/src/allreduce.py:69-92); here the ordering is a monotonically increasing token
// published and awaited on the comm stream, so the host never blocks.
#include "dla_common.h"
#include "dla_kernels.h"

namespace dla {

__global__ __launch_bounds__(64) void ipc_barrier_kernel(IpcBarrier b) {
  if (threadIdx.x != 0) return;
  if (b.mine) __hip_atomic_store(b.mine, b.set, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < b.npeers; ++i) {
    uint64_t seen;
    while ((seen = __hip_atomic_load(b.peer[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) < b.wait) {
      if (wall_clock64() - t0 > b.timeout_ticks) {
        // keep the first failure's record: later barriers of a broken run time out too
        if (b.diag && __hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
          __hip_atomic_store(b.diag, b.wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(b.diag + 1, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(b.diag + 2, (uint64_t)b.peer_rank[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __hip_atomic_store(b.err, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
}

void launch_ipc_barrier(const IpcBarrier& b, hipStream_t stream) {
  hipLaunchKernelGGL(ipc_barrier_kernel, dim3(1), dim3(64), 0, stream, b);
}

}  // namespace dla
