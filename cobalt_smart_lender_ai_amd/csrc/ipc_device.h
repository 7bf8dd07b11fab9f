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

// Mark this rank's exchange as failed: sticky (its own later waits fail at once), the pinned host error
// word (the host watchdog aborts) and the failure notice its peers' waits poll (kIpcFailWord). One thread.
__device__ __forceinline__ void ipc_fail(unsigned* myflag, unsigned* err_host) {
  __hip_atomic_store(myflag + kIpcStickyWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(myflag + kIpcFailWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block-wide: wait until every rank has published `epoch`. Wave 0 polls all ranks' flag words at once
// (lane r <- rank r's epoch word, lane 32 + r <- its failure notice: one round trip per poll) with
// s_sleep back-off and an s_memrealtime deadline; on timeout, or when a peer has posted its failure
// notice, this rank fails too (ipc_fail: sticky word, host error word, its own notice) and every later
// wait of this rank fails at once. kAcquire: a system-scope acquire follows, so the block's plain loads
// read the peers' slots fresh -- on a multi-XCD gfx950 that invalidates the whole L2 of the XCD; callers
// that read the slots with system-scope (cache-bypassing) loads instead pass false. Returns the same
// value in every thread; call from all threads. (n <= kMaxIpcRanks <= 32)
template <bool kAcquire = true>
__device__ __forceinline__ bool ipc_wait(const unsigned* const* ftab, int n, int me, unsigned* myflag,
                                         unsigned epoch, unsigned* err_host, unsigned long long timeout) {
  __shared__ int ipc_ok;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int r = lane & 31;
    const bool notice = lane >= 32;
    int good = __hip_atomic_load(myflag + kIpcStickyWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    // this rank's own slot is complete by stream order: its lane does not wait on its own flag store
    const bool peer = r < n && r != me;
    const unsigned* f = ftab[peer ? r : 0] + (notice ? kIpcFailWord : 0);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (good) {
      const unsigned v = peer ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : (notice ? 0u : epoch);
      const bool failed = notice && v != 0u;
      const bool lag = !notice && (int)(v - epoch) < 0;
      if (__ballot(failed) != 0) {  // a peer gave up: so does this rank (the failure reaches every rank)
        good = 0;
        if (lane == 0) ipc_fail(myflag, err_host);
        break;
      }
      if (__ballot(lag) == 0) break;  // every peer has published this epoch
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        good = 0;
        if (lane == 0) ipc_fail(myflag, err_host);
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
