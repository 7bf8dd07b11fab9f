// Microbenchmark: how should a histogram pass's per-block partial histograms reach the level's global
// histogram on gfx950?  (csrc/gbdt.hip k_hist -> slab -> k_hist_reduce today)
//   direct : every block adds its ncell (g, h) int64 pairs straight into the global histogram
//            (2 device-scope atomics per non-zero cell; all blocks hit the same addresses)
//   slab   : every block stores its partial row (plain stores), then a separate reduce kernel sums runs
//            of 16 rows per cell and adds one atomic pair per (run, cell)  [the current design]
//   lastrun: slab store + per-run arrival counter; the LAST block of each 16-block run reduces the run
//            inside the same kernel (last-block-done, no second launch)
// Each variant is timed as a dependent chain of 200 repetitions (one "level" each) with hipEvents.
// Build: hipcc --offload-arch=gfx950 -O3 flush.hip -o flush ; run: ./flush
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kRun = 16;

__device__ __forceinline__ uint64_t part_val(int b, int c) { return ((uint64_t)(b % 7 + 1) << 32) | (uint64_t)(c % 5 + 1); }

__global__ __launch_bounds__(512) void k_direct(int64_t* hist, int ncell) {
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) {
    const uint64_t v = part_val(blockIdx.x, c);
    atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * c), (unsigned long long)(int64_t)(int32_t)(v >> 32));
    atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * c + 1), (unsigned long long)(uint32_t)v);
  }
}

__global__ __launch_bounds__(512) void k_slab(uint64_t* slab, int ncell) {
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) slab[(int64_t)blockIdx.x * ncell + c] = part_val(blockIdx.x, c);
}

__global__ __launch_bounds__(256) void k_reduce(const uint64_t* slab, int64_t* hist, int ncell, int nitems) {
  const int cell = blockIdx.y * blockDim.x + threadIdx.x;
  if (cell >= ncell) return;
  const int i0 = blockIdx.x * kRun;
  int64_t g = 0, h = 0;
#pragma unroll
  for (int k = 0; k < kRun; ++k) {
    const int it = min(i0 + k, nitems - 1);
    const uint64_t v = i0 + k < nitems ? slab[(int64_t)it * ncell + cell] : 0ull;
    g += (int64_t)(int32_t)(v >> 32);
    h += (int64_t)(uint32_t)v;
  }
  atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * cell), (unsigned long long)g);
  atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * cell + 1), (unsigned long long)h);
}

__global__ __launch_bounds__(512) void k_lastrun(uint64_t* slab, int64_t* hist, unsigned* cnt, int ncell, int nitems) {
  __shared__ int last;
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) slab[(int64_t)blockIdx.x * ncell + c] = part_val(blockIdx.x, c);
  const int run = blockIdx.x / kRun;
  const int rsize = min(kRun, nitems - run * kRun);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned old = __hip_atomic_fetch_add(cnt + run, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (unsigned)rsize - 1;
    if (last) cnt[run] = 0;  // reset for the next repetition (no other block of the run is left)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!last) return;
  const int i0 = run * kRun;
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) {
    int64_t g = 0, h = 0;
    uint64_t v[kRun];
#pragma unroll
    for (int k = 0; k < kRun; ++k)  // all loads of the run in flight together (clamped rows, masked after)
      v[k] = slab[(int64_t)(i0 + min(k, rsize - 1)) * ncell + c];
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      if (k >= rsize) v[k] = 0;
      g += (int64_t)(int32_t)(v[k] >> 32);
      h += (int64_t)(uint32_t)v[k];
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * c), (unsigned long long)g);
    atomicAdd(reinterpret_cast<unsigned long long*>(hist + 2 * c + 1), (unsigned long long)h);
  }
}

int main() {
  const int ncell = 1300;
  const int reps = 200;
  int64_t* hist;
  uint64_t* slab;
  unsigned* cnt;
  CHECK(hipMalloc(&hist, 2 * ncell * sizeof(int64_t)));
  CHECK(hipMalloc(&slab, (size_t)4096 * ncell * sizeof(uint64_t)));
  CHECK(hipMalloc(&cnt, 4096 * sizeof(unsigned)));
  CHECK(hipMemset(cnt, 0, 4096 * sizeof(unsigned)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("ncell %d, us per level (mean of %d dependent repetitions)\n", ncell, reps);
  printf("%8s %10s %10s %10s %10s\n", "blocks", "direct", "slab+red", "lastrun", "empty");
  for (int blocks : {16, 64, 256, 512, 1024, 2048}) {
    float t[4];
    for (int v = 0; v < 4; ++v) {
      CHECK(hipMemset(hist, 0, 2 * ncell * sizeof(int64_t)));
      for (int w = 0; w < 2; ++w) {  // warm-up + timed
        CHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < (w ? reps : 5); ++r) {
          if (v == 0) hipLaunchKernelGGL(k_direct, dim3(blocks), dim3(512), 0, 0, hist, ncell);
          if (v == 1) {
            hipLaunchKernelGGL(k_slab, dim3(blocks), dim3(512), 0, 0, slab, ncell);
            hipLaunchKernelGGL(k_reduce, dim3((blocks + kRun - 1) / kRun, (ncell + 255) / 256), dim3(256), 0, 0, slab,
                               hist, ncell, blocks);
          }
          if (v == 2) hipLaunchKernelGGL(k_lastrun, dim3(blocks), dim3(512), 0, 0, slab, hist, cnt, ncell, blocks);
          if (v == 3) hipLaunchKernelGGL(k_slab, dim3(blocks), dim3(512), 0, 0, slab, 0);
        }
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
      }
      CHECK(hipEventElapsedTime(&t[v], e0, e1));
      // correctness of the accumulated sums: every variant adds the same per-level totals
      int64_t h0[2];
      CHECK(hipMemcpy(h0, hist, 16, hipMemcpyDeviceToHost));
      if (v < 3) {
        int64_t g = 0, hh = 0;
        for (int b = 0; b < blocks; ++b) { g += b % 7 + 1; hh += 1; }
        if (h0[0] != g * (reps + 5) || h0[1] != hh * (reps + 5)) printf("  MISMATCH variant %d: %lld %lld\n", v, (long long)h0[0], (long long)h0[1]);
      }
    }
    printf("%8d %10.2f %10.2f %10.2f %10.2f\n", blocks, t[0] * 1e3 / reps, t[1] * 1e3 / reps, t[2] * 1e3 / reps,
           t[3] * 1e3 / reps);
  }
  return 0;
}
