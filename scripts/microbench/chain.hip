// Microbenchmark: what a dependent kernel boundary and an in-kernel grid barrier cost on gfx950,
// for the shapes of the GBDT per-level kernels (a few hundred blocks, 2-3 dependent round trips).
//   k_empty      : 372 x 256 threads, nothing                     -> per-kernel floor
//   k_bigarg     : same with a 512-byte by-value argument (GbdtDev-sized)
//   k_chase3     : 3 dependent global loads per thread
//   k_atom       : 16 loads + int64 atomics into a shared 48 KB table (k_hist_reduce shape)
//   k_lds40      : 500 x 512 threads, zero 40 KB of LDS + one load (k_hist setup shape)
//   k_barrier    : persistent 256 x 1024 (or 512 x 512), N grid barriers (counter, sc1 poll + s_sleep)
// Build: hipcc --offload-arch=gfx950 -O3 chain.hip -o chain
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Big { int64_t v[64]; };

__global__ void k_empty(int* p) { if (p == nullptr) p[0] = 0; }
__global__ void k_bigarg(Big b, int* p) { if (b.v[3] == 12345) p[0] = 1; }
__global__ void k_chase3(const int* __restrict__ a, int* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  int x = a[i & 4095];
  x = a[x];
  x = a[x];
  if (x == -7) out[0] = x;
}
__global__ void k_atom(const uint64_t* slab, unsigned long long* hist, int ncell) {
  const int cell = (blockIdx.y * blockDim.x + threadIdx.x);
  if (cell >= ncell) return;
  const int i0 = blockIdx.x * 16;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += slab[(int64_t)(i0 + k) * ncell + cell];
  atomicAdd(hist + 2 * cell, s);
  atomicAdd(hist + 2 * cell + 1, s >> 3);
}
__global__ void k_lds40(const int* a, int* out) {
  extern __shared__ uint64_t s[];
  for (int i = threadIdx.x; i < 5120; i += blockDim.x) s[i] = 0;
  __syncthreads();
  int x = a[(blockIdx.x * 7 + threadIdx.x) & 4095];
  s[x & 4095] += 1;
  __syncthreads();
  if (s[threadIdx.x] == 77777) out[0] = 1;
}

__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned target, unsigned* tmo) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) { __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__global__ void k_barrier(unsigned* ctr, int nbar, unsigned* tmo) {
  for (int b = 1; b <= nbar; ++b) {
    grid_barrier(ctr, (unsigned)b * gridDim.x, tmo);
    if (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  }
}

template <class F>
float time_chain(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  int* ia; int* out; uint64_t* slab; unsigned long long* hist; unsigned* ctr; unsigned* tmo;
  CHECK(hipMalloc(&ia, 4096 * 4));
  CHECK(hipMalloc(&out, 16));
  const int ncell = 3000, items = 496;
  CHECK(hipMalloc(&slab, (size_t)items * ncell * 8));
  CHECK(hipMalloc(&hist, (size_t)ncell * 16));
  CHECK(hipMalloc(&ctr, 64));
  CHECK(hipMalloc(&tmo, 64));
  CHECK(hipMemset(slab, 0, (size_t)items * ncell * 8));
  int h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (i * 2654435761u) & 4095;
  CHECK(hipMemcpy(ia, h, sizeof(h), hipMemcpyHostToDevice));
  Big big{};
  const int reps = 2000;
  printf("empty 372x256        %7.2f us/kernel\n", time_chain([&] { k_empty<<<372, 256>>>(out); }, reps));
  printf("empty 1x64           %7.2f us/kernel\n", time_chain([&] { k_empty<<<1, 64>>>(out); }, reps));
  printf("bigarg 372x256       %7.2f us/kernel\n", time_chain([&] { k_bigarg<<<372, 256>>>(big, out); }, reps));
  printf("chase3 372x256       %7.2f us/kernel\n", time_chain([&] { k_chase3<<<372, 256>>>(ia, out); }, reps));
  printf("atom 31x12 x256      %7.2f us/kernel\n",
         time_chain([&] { k_atom<<<dim3(31, 12), 256>>>(slab, hist, ncell); }, reps));
  printf("lds40 500x512        %7.2f us/kernel\n", time_chain([&] { k_lds40<<<500, 512, 40960>>>(ia, out); }, reps));
  // hipGraph of 100 chained empty kernels
  {
    hipStream_t s; CHECK(hipStreamCreate(&s));
    hipGraph_t g; hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) k_chase3<<<372, 256, 0, s>>>(ia, out);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float t = time_chain([&] { (void)hipGraphLaunch(ge, s); }, 50);
    printf("graph chase3 x100    %7.2f us/kernel\n", t / 100);
  }
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int grid = cfg == 0 ? 256 : 512, block = cfg == 0 ? 1024 : 512;
    int nb = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_barrier, block, 0));
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    if (nb * ncu < grid) { printf("barrier grid %d not resident (%d x %d)\n", grid, nb, ncu); continue; }
    const int nbar = 1000;
    CHECK(hipMemset(ctr, 0, 64));
    CHECK(hipMemset(tmo, 0, 64));
    float t = time_chain([&] {
      (void)hipMemsetAsync(ctr, 0, 64);
      k_barrier<<<grid, block>>>(ctr, nbar, tmo);
    }, 5);
    unsigned to = 0;
    CHECK(hipMemcpy(&to, tmo, 4, hipMemcpyDeviceToHost));
    printf("barrier %dx%d        %7.2f us/barrier (timeout=%u)\n", grid, block, t / nbar, to);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
