// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of cobalt_smart_lender_ai_amd.
//
// Everything here is written for 64-lane wavefronts. Kernels are exported through a plain C ABI
// (extern "C", raw device pointers + hipStream_t) and bound from Python with ctypes, so the
// library has no dependency on the PyTorch C++ ABI: PyTorch-ROCm owns the tensors and streams,
// this library owns the compute.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

#define COBALT_API extern "C" __attribute__((visibility("default")))

#define CK(expr)                                      \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return static_cast<int>(_e); \
  } while (0)

#define CK_LAUNCH() CK(hipGetLastError())

namespace cobalt {

constexpr int kWave = 64;
constexpr uint8_t kMissingBin = 255;   // bin id reserved for NaN
constexpr int kMaxBins = 256;          // row stride of the cut table (255 usable bins + missing)

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / kWave; }

// Inclusive prefix sum over the 64 lanes of a wavefront (generic shuffle form; int / int64 use the
// DPP overloads below).
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T t = __shfl_up(v, o, kWave);
    if (lane >= o) v += t;
  }
  return v;
}

// ---- DPP cross-lane moves (GFX9 / CDNA data-parallel primitives: row_shr within 16-lane rows,
// row_bcast across rows). A lane without a source (shifted in, or in a disabled row / bank) gets
// `old`. They run at VALU latency; __shfl lowers to ds_bpermute, an LDS round trip per step.
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;
constexpr int kDppWaveShr1 = 0x138;  // whole-wave shift by one lane (lane i <- lane i - 1; lane 0 <- old)

template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ int dpp32(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWM, BANKM, false);
}

template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ int64_t dpp64(int64_t v, int64_t old) {
  const int lo = dpp32<CTRL, ROWM, BANKM>((int)(uint32_t)(uint64_t)v, (int)(uint32_t)(uint64_t)old);
  const int hi = dpp32<CTRL, ROWM, BANKM>((int)((uint64_t)v >> 32), (int)((uint64_t)old >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int readlane32(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

__device__ __forceinline__ int64_t readlane64(int64_t v, int lane) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, lane);
  const int hi = __builtin_amdgcn_readlane((int)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Wave64 inclusive prefix sums on DPP (Hillis-Steele within rows, then the row totals via
// row_bcast:15 into rows 1 / 3 and row_bcast:31 into rows 2 / 3). Every lane must be active.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += dpp32<kDppRowShr1>(v, 0);
  v += dpp32<kDppRowShr2>(v, 0);
  v += dpp32<kDppRowShr4>(v, 0);
  v += dpp32<kDppRowShr8>(v, 0);
  v += dpp32<kDppRowBcast15, 0xa>(v, 0);
  v += dpp32<kDppRowBcast31, 0xc>(v, 0);
  return v;
}

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v) {
  v += dpp64<kDppRowShr1>(v, 0);
  v += dpp64<kDppRowShr2>(v, 0);
  v += dpp64<kDppRowShr4>(v, 0);
  v += dpp64<kDppRowShr8>(v, 0);
  v += dpp64<kDppRowBcast15, 0xa>(v, 0);
  v += dpp64<kDppRowBcast31, 0xc>(v, 0);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// int / int64 totals in every lane: the DPP scan's last lane, read back as a scalar (all lanes active).
__device__ __forceinline__ int wave_sum(int v) { return readlane32(wave_incl_scan(v), kWave - 1); }
__device__ __forceinline__ int64_t wave_sum(int64_t v) { return readlane64(wave_incl_scan(v), kWave - 1); }

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    T t = __shfl_xor(v, o, kWave);
    v = t > v ? t : v;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    T t = __shfl_xor(v, o, kWave);
    v = t < v ? t : v;
  }
  return v;
}

// Number of active lanes below this one in a 64-bit ballot mask.
__device__ __forceinline__ int mask_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0));
}

// splitmix64: counter-based hash used for reproducible per-row / per-tree randomness.
// The same function lives in the host oracle (models/gbdt_host.py) so the GPU and CPU paths
// draw identical row samples.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__host__ __device__ __forceinline__ double uniform01(uint64_t h) {
  return static_cast<double>(h >> 11) * (1.0 / 9007199254740992.0);
}

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace cobalt
