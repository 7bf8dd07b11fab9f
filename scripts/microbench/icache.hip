// Microbenchmark: does instruction fetch bound a cold, large, straight-line kernel on gfx950?
// k_unrolled executes N_OPS FMAs as straight-line code (~8 B/op); k_rolled executes the same FMAs in a
// loop of 64-op bodies. Each is timed in a chain after a kernel that streams 512 MB (evicting L2/MALL),
// and back-to-back (code hot). Build: hipcc --offload-arch=gfx950 -O3 icache.hip -o icache
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int N_OPS = 4096;

__global__ void k_unrolled(float* out, float a) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
#pragma unroll
  for (int i = 0; i < N_OPS / 8; ++i) {
    const float c = a + (float)i;  // distinct literal per op: no CSE, no loop
    x0 = fmaf(x0, c, 0.5f); x1 = fmaf(x1, c, 0.25f); x2 = fmaf(x2, c, 0.125f); x3 = fmaf(x3, c, 0.0625f);
    x4 = fmaf(x4, c, 1.5f); x5 = fmaf(x5, c, 1.25f); x6 = fmaf(x6, c, 1.125f); x7 = fmaf(x7, c, 1.0625f);
  }
  const float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (s == 12345.f) out[0] = s;
}

__global__ void k_rolled(float* out, float a) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
#pragma unroll 1
  for (int j = 0; j < N_OPS / 64; ++j) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float c = a + (float)(i + 8 * j);
      x0 = fmaf(x0, c, 0.5f); x1 = fmaf(x1, c, 0.25f); x2 = fmaf(x2, c, 0.125f); x3 = fmaf(x3, c, 0.0625f);
      x4 = fmaf(x4, c, 1.5f); x5 = fmaf(x5, c, 1.25f); x6 = fmaf(x6, c, 1.125f); x7 = fmaf(x7, c, 1.0625f);
    }
  }
  const float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (s == 12345.f) out[0] = s;
}

__global__ void k_stream(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

int main() {
  float* out; float4 *src, *dst;
  const size_t n = (256u << 20) / 16;
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMalloc(&src, n * 16));
  CHECK(hipMalloc(&dst, n * 16));
  CHECK(hipMemset(src, 0, n * 16));
  hipEvent_t e0, e1, e2;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1)); CHECK(hipEventCreate(&e2));
  for (int cold = 0; cold < 2; ++cold)
    for (int which = 0; which < 2; ++which)
      for (int blocks : {1, 256}) {
        float tot = 0.f;
        const int reps = 50;
        for (int r = 0; r < reps + 3; ++r) {
          if (cold) k_stream<<<2048, 256>>>(src, dst, n);
          CHECK(hipEventRecord(e0));
          if (which == 0) k_unrolled<<<blocks, 64>>>(out, 1.0001f); else k_rolled<<<blocks, 64>>>(out, 1.0001f);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
          if (r >= 3) tot += ms;
        }
        printf("%-9s %-5s blocks=%3d  %7.2f us\n", which == 0 ? "unrolled" : "rolled", cold ? "cold" : "hot", blocks,
               tot * 1000.f / reps);
      }
  return 0;
}
