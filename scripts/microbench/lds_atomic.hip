// Microbenchmark: LDS atomic throughput on gfx950 for the histogram kernel design.
// mode 0: ds_add_u64, 1: ds_add_u32, 2: 2x ds_add_u32 (g,h), 3: ds_add_f32, 4: plain ds_read+ds_write (no atomic)
// pattern 0: lane-private distinct addresses, 1: 2 hot addresses per wave (binary feature), 2: random over 256 cells
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE, int PAT>
__global__ __launch_bounds__(256) void k(int iters, unsigned long long* out) {
  __shared__ unsigned long long s[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) s[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    int a;
    if (PAT == 0) a = (w * 64 + lane + it * 256) & 4095;
    else if (PAT == 1) a = ((x >> 16) & 1) + (it & 15) * 2;
    else a = (x >> 8) & 255;
    if (MODE == 0) atomicAdd(&s[a], 3ull);
    else if (MODE == 1) atomicAdd(reinterpret_cast<unsigned*>(s) + a, 3u);
    else if (MODE == 2) { atomicAdd(reinterpret_cast<unsigned*>(s) + 2 * a, 3u); atomicAdd(reinterpret_cast<unsigned*>(s) + 2 * a + 1, 5u); }
    else if (MODE == 3) atomicAdd(reinterpret_cast<float*>(s) + a, 1.0f);
    else { s[a] += 3ull; }
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, s[blockIdx.x & 4095]);
}

template <int MODE, int PAT>
void run(const char* name) {
  unsigned long long* out;
  (void)hipMalloc(&out, 8);
  const int iters = 4096, blocks = 2048;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  k<MODE, PAT><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(a);
  k<MODE, PAT><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  const double ops = (double)iters * blocks * 256 * (MODE == 2 ? 2 : 1);
  printf("%-28s pat=%d  %8.3f ms  %8.2f G lane-ops/s  %6.2f lane-ops/clk/CU\n", name, PAT, ms, ops / ms / 1e6,
         ops / (ms * 1e-3) / 256 / 2.4e9);
  (void)hipFree(out);
}

int main() {
  run<0, 0>("ds_add_u64"); run<0, 1>("ds_add_u64"); run<0, 2>("ds_add_u64");
  run<1, 0>("ds_add_u32"); run<1, 1>("ds_add_u32"); run<1, 2>("ds_add_u32");
  run<2, 0>("2x ds_add_u32"); run<2, 2>("2x ds_add_u32");
  run<3, 0>("ds_add_f32"); run<3, 2>("ds_add_f32");
  run<4, 0>("plain rmw u64 (racy)"); run<4, 2>("plain rmw u64 (racy)");
  return 0;
}
