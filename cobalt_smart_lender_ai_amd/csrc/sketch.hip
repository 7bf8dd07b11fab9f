// Exact full-data weighted-quantile sketch (K12 in SURVEY.md §2.4) for gfx950: the cut points of
// models/sketch.py compute_cuts over EVERY row, without sorting the rows.
//
// XGBoost's `hist` updater, which the reference drives through XGBClassifier.fit (reference:
// src/model_train_test/model_tree_train_test.py:111-118,159; max_bin = 256), sketches all rows. A
// segmented sort of F x N (value, weight) pairs costs ~85 ms at 10M x 20 on one MI355X; 255 order
// statistics per feature do not need the order of all N values:
//
//  1. boundaries: <= 4095 distinct values of a strided sample, sorted (host side, torch.sort of a
//     few 10k values per feature). They split the value axis into buckets 2k+1 = {u_k} (a value of
//     the sample) and 2k = (u_{k-1}, u_k) (strictly between two of them) -- 2m + 1 buckets.
//  2. k_sk_hist: one pass over the (feature-major) values: the bucket of every value by a branchless
//     binary search over the boundaries in LDS, integer weight sums per bucket in an LDS histogram,
//     written as the block's slab row (no global atomics), plus the block's minimum value.
//  3. (torch) prefix sums over the buckets locate every target rank: a target in an equal bucket IS
//     its value; one in an open bucket needs that bucket's values ("candidates", ~N / 4096 rows each).
//  4. k_sk_gather: a second pass writes the values of the selected open buckets into per-bucket
//     segments (LDS-aggregated range reservations: one global atomic per block and bucket).
//  5. k_sk_select: one block per selected bucket sorts its segment in LDS (bitonic, values with their
//     weights), scans the weights and answers that bucket's targets: the first value whose cumulative
//     weight w satisfies (prefix + w) * maxb > j * W -- the rule of compute_cuts, so the cuts are
//     bit-identical to the sort-based path (tests/test_sketch.py).
// Under data parallelism the bucket histograms are all-reduced and the candidates all-gathered, so
// every rank selects from the global multiset.
#include "common.h"

using namespace cobalt;

namespace {

constexpr int kSkMaxBounds = 4096;               // LDS boundary table (<= 4095 real + +inf padding)
constexpr int kSkBuckets = 2 * kSkMaxBounds + 1;  // 2 m + 1 <= 8191 used
constexpr int kSkThreads = 1024;

__device__ __forceinline__ float canon(float v) { return v + 0.0f; }  // -0 -> +0 (compute_cuts' rule)

// number of boundaries < v (branchless over the padded power-of-two table) and whether u[k] == v
__device__ __forceinline__ int sk_bucket(const float* __restrict__ u, int m, float v) {
  int k = 0;
#pragma unroll
  for (int s = kSkMaxBounds / 2; s > 0; s >>= 1) k += (u[k + s - 1] < v) ? s : 0;
  const bool eq = k < m && u[k] == v;
  return 2 * k + (eq ? 1 : 0);
}

__device__ __forceinline__ void sk_load_bounds(float* s_u, const float* __restrict__ bounds, int f) {
  for (int i = threadIdx.x; i < kSkMaxBounds; i += blockDim.x) s_u[i] = bounds[(int64_t)f * kSkMaxBounds + i];
}

// Pass 1. grid = (blocks per feature, F); X feature-major [F][ldx]; w: int32 quantised weights or
// nullptr (unit). cnt_slab [gridDim.x][F][kSkBuckets] u32 row counts; w_slab (kW) the same shape in
// u64 weight sums; bmm [gridDim.x][F][2] the block's min / max valid value.
template <bool kW>
__global__ __launch_bounds__(kSkThreads) void k_sk_hist(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                       const int32_t* __restrict__ w, const float* __restrict__ bounds,
                                                       const int32_t* __restrict__ nbound, uint32_t* __restrict__ cnt_slab,
                                                       unsigned long long* __restrict__ w_slab, float* __restrict__ bmm) {
  __shared__ float s_u[kSkMaxBounds];
  __shared__ uint32_t s_c[kSkBuckets];
  __shared__ unsigned long long s_w[kW ? kSkBuckets : 1];
  __shared__ float s_mm[2][kSkThreads / kWave];
  const int f = blockIdx.y, F = gridDim.y;
  sk_load_bounds(s_u, bounds, f);
  for (int i = threadIdx.x; i < kSkBuckets; i += blockDim.x) {
    s_c[i] = 0u;
    if (kW) s_w[i] = 0ull;
  }
  const int m = nbound[f];
  __syncthreads();
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(n, r0 + per);
  const float* col = X + (int64_t)f * ldx;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const float v = canon(col[r]);
    if (v != v) continue;  // NaN: the missing bin, no weight
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    const int b = sk_bucket(s_u, m, v);
    atomicAdd(&s_c[b], 1u);
    if (kW) {
      const int32_t wi = w[r];
      if (wi) atomicAdd(&s_w[b], (unsigned long long)wi);
    }
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  if (lane_id() == 0) {
    s_mm[0][wave_id()] = mn;
    s_mm[1][wave_id()] = mx;
  }
  __syncthreads();
  const int64_t row = (int64_t)blockIdx.x * F + f;
  for (int i = threadIdx.x; i < kSkBuckets; i += blockDim.x) {
    cnt_slab[row * kSkBuckets + i] = s_c[i];
    if (kW) w_slab[row * kSkBuckets + i] = s_w[i];
  }
  if (threadIdx.x == 0) {
    float a = INFINITY, b = -INFINITY;
    for (int k = 0; k < kSkThreads / kWave; ++k) {
      a = fminf(a, s_mm[0][k]);
      b = fmaxf(b, s_mm[1][k]);
    }
    bmm[row * 2] = a;
    bmm[row * 2 + 1] = b;
  }
}

// Pass 2. slot [F][kSkBuckets]: the bucket's segment index (-1 = not selected); seg_off [nseg + 1]
// (exclusive), cursor [nseg] (zeroed). Writes candidate values (and int32 weights) into their
// bucket's segment. Per block: count per selected bucket in LDS, reserve one range per bucket with
// a global atomic, then a second walk over the rows writes through LDS cursors.
template <bool kW>
__global__ __launch_bounds__(kSkThreads) void k_sk_gather(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                         const int32_t* __restrict__ w, const float* __restrict__ bounds,
                                                         const int32_t* __restrict__ nbound,
                                                         const int32_t* __restrict__ slot, const int64_t* __restrict__ seg_off,
                                                         unsigned long long* __restrict__ cursor, float* __restrict__ cval,
                                                         int32_t* __restrict__ cw) {
  __shared__ float s_u[kSkMaxBounds];
  __shared__ int32_t s_slot[kSkBuckets];
  __shared__ uint32_t s_cnt[kSkBuckets];  // per bucket: rows of this block, then the write cursor
  const int f = blockIdx.y;
  sk_load_bounds(s_u, bounds, f);
  for (int i = threadIdx.x; i < kSkBuckets; i += blockDim.x) {
    s_slot[i] = slot[(int64_t)f * kSkBuckets + i];
    s_cnt[i] = 0u;
  }
  const int m = nbound[f];
  __syncthreads();
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(n, r0 + per);
  const float* col = X + (int64_t)f * ldx;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const float v = canon(col[r]);
    if (v != v) continue;
    const int b = sk_bucket(s_u, m, v);
    if (s_slot[b] >= 0) atomicAdd(&s_cnt[b], 1u);
  }
  __syncthreads();
  // reserve this block's range in every selected bucket it touches; s_cnt becomes the write cursor
  for (int b = threadIdx.x; b < kSkBuckets; b += blockDim.x) {
    const uint32_t c = s_cnt[b];
    if (c) {
      const int sg = s_slot[b];
      s_cnt[b] = (uint32_t)(seg_off[sg] + (int64_t)atomicAdd(cursor + sg, (unsigned long long)c));
    }
  }
  __syncthreads();
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const float v = canon(col[r]);
    if (v != v) continue;
    const int b = sk_bucket(s_u, m, v);
    if (s_slot[b] < 0) continue;
    const uint32_t pos = atomicAdd(&s_cnt[b], 1u);
    cval[pos] = v;
    if (kW) cw[pos] = w[r];
  }
}

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Pass 3. One block per selected segment of <= kSkSortCap values: bitonic sort in LDS (key = ordered
// float bits, payload = weight), an inclusive weight scan, then the segment's targets. Targets of
// segment s are tgt_off[s] .. tgt_off[s+1]): target t asks for the first value whose cumulative weight
// cw satisfies (prefix[t] + cw) * maxb[t] > thr[t]; its value goes to out[t]. Segments larger than
// the cap are left to the host (torch.sort) -- flagged by the caller.
constexpr int kSkSortCap = 8192;  // keys (32 KB) + int64 weight sums (64 KB) of LDS

template <bool kW>
__global__ __launch_bounds__(kSkThreads) void k_sk_select(const float* __restrict__ cval, const int32_t* __restrict__ cw,
                                                         const int64_t* __restrict__ seg_off,
                                                         const int32_t* __restrict__ tgt_off,
                                                         const int64_t* __restrict__ prefix, const int64_t* __restrict__ thr,
                                                         const int64_t* __restrict__ maxb, float* __restrict__ out) {
  extern __shared__ uint32_t s_dyn[];
  const int s = blockIdx.x;
  const int64_t o0 = seg_off[s], o1 = seg_off[s + 1];
  const int len = (int)(o1 - o0);
  const int t0 = tgt_off[s], t1 = tgt_off[s + 1];
  if (len <= 0 || len > kSkSortCap || t0 >= t1) return;
  int P = 1;
  while (P < len) P <<= 1;
  uint32_t* key = s_dyn;                                   // [P]
  int64_t* cum = reinterpret_cast<int64_t*>(s_dyn + kSkSortCap);  // [P] weights, then inclusive sums
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    key[i] = i < len ? fkey(cval[o0 + i]) : 0xFFFFFFFFu;
    cum[i] = i < len ? (kW ? (int64_t)cw[o0 + i] : 1) : 0;
  }
  __syncthreads();
  // bitonic sort of (key, weight) pairs
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ix = i ^ j;
        if (ix > i) {
          const uint32_t a = key[i], b = key[ix];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[ix] = a;
            if (kW) {
              const int64_t t = cum[i];
              cum[i] = cum[ix];
              cum[ix] = t;
            }
          }
        }
      }
      __syncthreads();
    }
  }
  // inclusive scan of the weights (Hillis-Steele over the block, in place)
  for (int d = 1; d < P; d <<= 1) {
    int64_t add[kSkSortCap / kSkThreads];
    int c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) add[c] = i >= d ? cum[i - d] : 0;
    __syncthreads();
    c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) cum[i] += add[c];
    __syncthreads();
  }
  // targets: first i with (prefix + cum[i]) * maxb > thr (binary search over the non-decreasing sums)
  for (int t = t0 + threadIdx.x; t < t1; t += blockDim.x) {
    const int64_t pre = prefix[t], mb = maxb[t], th = thr[t];
    int lo = 0, hi = len - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((pre + cum[mid]) * mb > th) hi = mid; else lo = mid + 1;
    }
    out[t] = fval(key[lo]);
  }
}

}  // namespace

COBALT_API int cobalt_sk_hist(const float* X, int64_t n, int64_t ldx, int F, const int32_t* w, const float* bounds,
                              const int32_t* nbound, int nblk, uint32_t* cnt_slab, void* w_slab, float* bmm,
                              hipStream_t stream) {
  if (F <= 0 || nblk <= 0) return -3;
  const dim3 grid(nblk, F);
  if (w)
    hipLaunchKernelGGL(k_sk_hist<true>, grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, cnt_slab,
                       static_cast<unsigned long long*>(w_slab), bmm);
  else
    hipLaunchKernelGGL(k_sk_hist<false>, grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, cnt_slab,
                       static_cast<unsigned long long*>(w_slab), bmm);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_gather(const float* X, int64_t n, int64_t ldx, int F, const int32_t* w, const float* bounds,
                                const int32_t* nbound, const int32_t* slot, const int64_t* seg_off, void* cursor,
                                float* cval, int32_t* cw, int nblk, hipStream_t stream) {
  if (F <= 0 || nblk <= 0) return -3;
  const dim3 grid(nblk, F);
  if (w)
    hipLaunchKernelGGL(k_sk_gather<true>, grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, slot,
                       seg_off, static_cast<unsigned long long*>(cursor), cval, cw);
  else
    hipLaunchKernelGGL(k_sk_gather<false>, grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, slot,
                       seg_off, static_cast<unsigned long long*>(cursor), cval, cw);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_select(const float* cval, const int32_t* cw, const int64_t* seg_off, int nseg,
                                const int32_t* tgt_off, const int64_t* prefix, const int64_t* thr, const int64_t* maxb,
                                float* out, hipStream_t stream) {
  if (nseg <= 0) return 0;
  const size_t lds = (size_t)kSkSortCap * (sizeof(uint32_t) + sizeof(int64_t));
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute((const void*)k_sk_select<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_sk_select<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  if (cw)
    hipLaunchKernelGGL(k_sk_select<true>, dim3(nseg), dim3(kSkThreads), lds, stream, cval, cw, seg_off, tgt_off, prefix,
                       thr, maxb, out);
  else
    hipLaunchKernelGGL(k_sk_select<false>, dim3(nseg), dim3(kSkThreads), lds, stream, cval, cw, seg_off, tgt_off,
                       prefix, thr, maxb, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_bounds() { return kSkMaxBounds; }
COBALT_API int cobalt_sk_buckets() { return kSkBuckets; }
COBALT_API int cobalt_sk_sort_cap() { return kSkSortCap; }
