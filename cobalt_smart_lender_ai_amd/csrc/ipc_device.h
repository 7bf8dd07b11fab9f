// Device side of the IPC group's epoch protocol (ipccomm.hip), shared by the stand-alone exchange
// kernel and the GBDT split evaluation that performs the exchange while reading the histograms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm.h"

// This rank's send slot of `epoch` is complete (written by earlier kernels of the stream): publish it.
// Call from ONE thread of the grid.
__device__ __forceinline__ void ipc_publish(unsigned* myflag, unsigned epoch) {
  if (threadIdx.x == 0) __hip_atomic_store(myflag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block-wide: wait until every rank has published `epoch`. Wave 0 polls all ranks' flag words at
// once (lane r <- rank r: one round trip per poll) with s_sleep back-off and an s_memrealtime
// deadline; on timeout the sticky word and the pinned host error word are set (the host watchdog
// aborts) and every later wait of this rank fails at once. kAcquire: a system-scope acquire follows,
// so the block's plain loads read the peers' slots fresh -- on a multi-XCD gfx950 that invalidates the
// whole L2 of the XCD; callers that read the slots with system-scope (cache-bypassing) loads instead
// pass false. Returns the same value in every thread; call from all threads.
template <bool kAcquire = true>
__device__ __forceinline__ bool ipc_wait(const unsigned* const* ftab, int n, int me, unsigned* myflag,
                                         unsigned epoch, unsigned* err_host, unsigned long long timeout) {
  __shared__ int ipc_ok;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int good = __hip_atomic_load(myflag + kIpcStickyWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    // this rank's own slot is complete by stream order: its lane does not wait on its own flag store
    const bool peer = lane < n && lane != me;
    const unsigned* f = ftab[peer ? lane : 0];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (good) {
      const unsigned v = peer ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : epoch;
      if (__ballot((int)(v - epoch) < 0) == 0) break;  // every peer has published this epoch
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        good = 0;
        if (lane == 0) {
          __hip_atomic_store(myflag + kIpcStickyWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (kAcquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    if (lane == 0) ipc_ok = good;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return ipc_ok != 0;
}
