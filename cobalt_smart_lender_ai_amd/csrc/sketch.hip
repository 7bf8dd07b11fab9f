// Exact full-data weighted-quantile sketch (K12 in SURVEY.md §2.4) for gfx950: the cut points of
// models/sketch.py compute_cuts over EVERY row, without sorting the rows.
//
// XGBoost's `hist` updater, which the reference drives through XGBClassifier.fit (reference:
// src/model_train_test/model_tree_train_test.py:111-118,159; max_bin = 256), sketches all rows. A
// segmented sort of F x N (value, weight) pairs costs ~85 ms at 10M x 20 on one MI355X; 255 order
// statistics per feature do not need the order of all N values:
//
//  1. boundaries: <= 4095 distinct values of a strided sample (torch.sort of a few 10k values per
//     feature, then k_sk_bounds). They split the value axis into buckets 2k+1 = {u_k} (a value of
//     the sample) and 2k = (u_{k-1}, u_k) (strictly between two of them) -- 2m + 1 buckets.
//  2. k_sk_hist: one pass over the (feature-major) values: the bucket of every value by a branchless
//     binary search over the boundaries in LDS, integer weight sums per bucket in an LDS histogram,
//     written as the block's slab row (no global atomics), plus the block's minimum value.
//  3. k_sk_plan1-3: prefix sums over the buckets locate every target rank: a target in an equal
//     bucket IS its value; one in an open bucket needs that bucket's values ("candidates", ~N / 4096
//     rows each). The selected buckets become segments with their offsets (one host read: the sizes).
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

// Number of boundaries < v and whether u[k] == v. The search runs over the boundaries in Eytzinger
// (breadth-first) order, e[i] = the BST node i of u[0..4094]: at step l a wave's lanes can only touch
// the 2^l consecutive words [2^l - 1, 2^(l+1) - 1), distinct LDS banks -- over the sorted table the
// candidates of steps 2-7 were 2^l words 4096 / 2^l apart, ALL in one bank (up to 32-way conflicts
// per step: ~10x the search's conflict-free LDS time, most of k_sk_hist).
constexpr int kSkTreeNodes = kSkMaxBounds - 1;  // 4095 = a complete BST of 12 levels
__device__ __forceinline__ int sk_bucket(const float* __restrict__ u, const float* __restrict__ e, int m, float v) {
  int k = 0;
#pragma unroll
  for (int l = 0; l < 12; ++l) k = 2 * k + 1 + (e[k] < v ? 1 : 0);
  k -= kSkTreeNodes;  // the in-order rank: boundaries < v
  const bool eq = k < m && u[k] == v;
  return 2 * k + (eq ? 1 : 0);
}

// The feature's sorted boundaries into s_u and their Eytzinger order into s_e (BFS node i at depth d,
// position p in its level = in-order index (2 p + 1) 2^(11 - d) - 1). Publish with a barrier.
__device__ __forceinline__ void sk_load_bounds(float* s_u, float* s_e, const float* __restrict__ bounds, int f) {
  const float* b = bounds + (int64_t)f * kSkMaxBounds;
  for (int i = threadIdx.x; i < kSkMaxBounds; i += blockDim.x) s_u[i] = b[i];
  for (int i = threadIdx.x; i < kSkTreeNodes; i += blockDim.x) {
    const int d = 31 - __clz(i + 1), p = i + 1 - (1 << d);
    s_e[i] = b[((2 * p + 1) << (11 - d)) - 1];
  }
}

// Pass 1. grid = (blocks per feature, F); X feature-major [F][ldx]; w: int32 quantised weights or
// nullptr (unit). cnt_slab [gridDim.x][F][kSkBuckets] u32 row counts; w_slab (kW) the same shape in
// u64 weight sums; bmm [gridDim.x][F][2] the block's min / max valid value.
// kIds: every value's bucket also goes to bid [F][ldx] (u16, 0xFFFF = missing), so pass 2 (k_sk_gather<..,
// true>) reads 2 bytes per value instead of repeating the 12-step search (the in-core sketch, one chunk).
template <bool kW, bool kIds>
__global__ __launch_bounds__(kSkThreads) void k_sk_hist(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                       const int32_t* __restrict__ w, const float* __restrict__ bounds,
                                                       const int32_t* __restrict__ nbound, uint32_t* __restrict__ cnt_slab,
                                                       unsigned long long* __restrict__ w_slab, float* __restrict__ bmm,
                                                       uint16_t* __restrict__ bid) {
  __shared__ float s_u[kSkMaxBounds], s_e[kSkTreeNodes];
  __shared__ uint32_t s_c[kSkBuckets];
  __shared__ unsigned long long s_w[kW ? kSkBuckets : 1];
  __shared__ float s_mm[2][kSkThreads / kWave];
  const int f = blockIdx.y, F = gridDim.y;
  sk_load_bounds(s_u, s_e, bounds, f);
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
  const int lane = lane_id();
  // every lane runs every iteration (whole-wave ballots / sums below)
  for (int64_t base = r0; base < r1; base += blockDim.x) {
    const int64_t r = base + threadIdx.x;
    const float v = r < r1 ? canon(col[r]) : __int_as_float(0x7fc00000);
    int b = -1;
    int64_t wi = 0;
    if (v == v) {  // NaN: the missing bin, no weight
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
      b = sk_bucket(s_u, s_e, m, v);
      wi = kW ? (int64_t)w[r] : 1;
    }
    if (kIds && r < r1) bid[(int64_t)f * ldx + r] = b >= 0 ? (uint16_t)b : (uint16_t)0xFFFFu;
    // Low-cardinality features put most lanes of a wave on one or two buckets: 64 same-address LDS
    // atomics serialise. Two leader rounds add the wave's most common buckets once (popcount /
    // wave sum), the remaining lanes add their own.
#pragma unroll
    for (int round = 0; round < 2; ++round) {
      const uint64_t act = __ballot(b >= 0);
      if (!act) break;
      const int lead = __builtin_ctzll(act);
      const int bl = __builtin_amdgcn_readlane(b, lead);
      const bool mine = b == bl;
      const uint64_t same = __ballot(mine);
      if (__popcll(same) < 8) break;  // a spread wave: per-lane atomics are cheaper than the sums
      if (kW) {
        const int64_t ws = wave_sum(mine ? wi : (int64_t)0);
        if (lane == lead) {
          atomicAdd(&s_c[bl], (uint32_t)__popcll(same));
          if (ws) atomicAdd(&s_w[bl], (unsigned long long)ws);
        }
      } else if (lane == lead) {
        atomicAdd(&s_c[bl], (uint32_t)__popcll(same));
      }
      if (mine) b = -1;
    }
    if (b >= 0) {
      atomicAdd(&s_c[b], 1u);
      if (kW && wi) atomicAdd(&s_w[b], (unsigned long long)wi);
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

// Pass 2. slot [F][kSkBuckets]: the bucket's segment index (-1 = not selected); blk_off [gridDim.x][nseg]:
// where this block's rows of each segment start (the exclusive prefix over the blocks of pass 1's
// per-block bucket counts, plus the segment's offset -- the same row partition as k_sk_hist, so one
// walk over the rows suffices). Writes candidate values (and int32 weights) into their segments
// through LDS cursors.
// kIds: the buckets come from pass 1's bid table (no boundary search; a value is loaded only when its
// bucket is selected).
template <bool kW, bool kIds>
__global__ __launch_bounds__(kSkThreads) void k_sk_gather(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                         const int32_t* __restrict__ w, const float* __restrict__ bounds,
                                                         const int32_t* __restrict__ nbound,
                                                         const int32_t* __restrict__ slot, const int64_t* __restrict__ blk_off,
                                                         int nseg, float* __restrict__ cval, int32_t* __restrict__ cw,
                                                         const uint16_t* __restrict__ bid) {
  __shared__ float s_u[kIds ? 1 : kSkMaxBounds], s_e[kIds ? 1 : kSkTreeNodes];
  __shared__ int32_t s_slot[kSkBuckets];
  // per selected bucket: this block's rows written so far (relative to the block's int64 segment offset
  // bo[segment]: a streamed sketch accumulates offsets across chunks, past 2^32 candidates at billions of
  // rows, while one block's count always fits 32 bits)
  __shared__ uint32_t s_cur[kSkBuckets];
  const int f = blockIdx.y;
  if (!kIds) sk_load_bounds(s_u, s_e, bounds, f);
  const int64_t* bo = blk_off + (int64_t)blockIdx.x * nseg;
  for (int i = threadIdx.x; i < kSkBuckets; i += blockDim.x) {
    s_slot[i] = slot[(int64_t)f * kSkBuckets + i];
    s_cur[i] = 0u;
  }
  const int m = nbound[f];
  __syncthreads();
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(n, r0 + per);
  const float* col = X + (int64_t)f * ldx;
  // kIds: the bucket ids 4 per 8-byte load over the 4-aligned middle of the range (rows of a feature
  // start 4-aligned when ldx % 4 == 0); the head and tail go through the loop below
  int64_t lo = r0, hi = r1;
  if (kIds && (ldx & 3) == 0) {
    const int64_t a0 = min(r1, (r0 + 3) & ~(int64_t)3), a1 = max(a0, r1 & ~(int64_t)3);
    const uint16_t* bf = bid + (int64_t)f * ldx;
    for (int64_t g = a0 / 4 + threadIdx.x; g < a1 / 4; g += blockDim.x) {
      const uint2 q = *reinterpret_cast<const uint2*>(bf + 4 * g);
      const uint32_t bq[4] = {q.x & 0xFFFFu, q.x >> 16, q.y & 0xFFFFu, q.y >> 16};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t bb = bq[c];
        if (bb == 0xFFFFu) continue;
        const int sg = s_slot[bb];
        if (sg < 0) continue;
        const int64_t r = 4 * g + c;
        const int64_t pos = bo[sg] + (int64_t)atomicAdd(&s_cur[bb], 1u);
        cval[pos] = canon(col[r]);
        if (kW) cw[pos] = w[r];
      }
    }
    // the scalar loop takes [r0, a0) and [a1, r1)
    lo = r0;
    hi = a0;
    for (int64_t r = a1 + threadIdx.x; r < r1; r += blockDim.x) {
      const uint32_t bb = bf[r];
      if (bb == 0xFFFFu) continue;
      const int sg = s_slot[bb];
      if (sg < 0) continue;
      const int64_t pos = bo[sg] + (int64_t)atomicAdd(&s_cur[bb], 1u);
      cval[pos] = canon(col[r]);
      if (kW) cw[pos] = w[r];
    }
  }
  for (int64_t r = lo + threadIdx.x; r < hi; r += blockDim.x) {
    int b;
    float v;
    if (kIds) {
      const uint32_t bb = bid[(int64_t)f * ldx + r];
      if (bb == 0xFFFFu || s_slot[bb] < 0) continue;
      b = (int)bb;
      v = canon(col[r]);
    } else {
      v = canon(col[r]);
      if (v != v) continue;
      b = sk_bucket(s_u, s_e, m, v);
    }
    const int sg = s_slot[b];
    if (sg < 0) continue;
    const int64_t pos = bo[sg] + (int64_t)atomicAdd(&s_cur[b], 1u);
    cval[pos] = v;
    if (kW) cw[pos] = w[r];
  }
}

// Row-major X [n][F] -> feature-major XT [F][n] (F <= 32): a tile of 256 rows is read as one
// contiguous run into LDS (rows padded to F + 1 words), then written as F runs of 256 values. 16-byte
// loads when the tile starts 16-byte aligned, 16-byte stores (4 rows of one feature) for whole tiles
// when n % 4 == 0; scalar otherwise.
constexpr int kTrRows = 256;
__global__ __launch_bounds__(256) void k_sk_transpose(const float* __restrict__ X, int64_t n, int F,
                                                      float* __restrict__ XT) {
  __shared__ float s_t[kTrRows * 33];
  const int64_t r0 = (int64_t)blockIdx.x * kTrRows;
  const int rows = (int)min((int64_t)kTrRows, n - r0);
  const float* src = X + r0 * F;
  const int tot = rows * F, P = F + 1;
  int j0 = 0;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    const int t4 = tot >> 2;
    for (int j = threadIdx.x; j < t4; j += blockDim.x) {
      const float4 v = reinterpret_cast<const float4*>(src)[j];
      int i = (4 * j) / F, f = 4 * j - i * F;
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s_t[i * P + f] = vv[c];
        if (++f == F) { f = 0; ++i; }
      }
    }
    j0 = 4 * t4;
  }
  for (int j = j0 + threadIdx.x; j < tot; j += blockDim.x) {
    const int i = j / F, f = j - i * F;
    s_t[i * P + f] = src[j];
  }
  __syncthreads();
  if ((n & 3) == 0 && rows == kTrRows) {
    constexpr int Q = kTrRows / 4;
    for (int j = threadIdx.x; j < F * Q; j += blockDim.x) {
      const int f = j / Q, q = j - f * Q;
      float4 v;
      v.x = s_t[(4 * q) * P + f];
      v.y = s_t[(4 * q + 1) * P + f];
      v.z = s_t[(4 * q + 2) * P + f];
      v.w = s_t[(4 * q + 3) * P + f];
      reinterpret_cast<float4*>(XT + (int64_t)f * n + r0)[q] = v;
    }
  } else {
    for (int j = threadIdx.x; j < kTrRows * F; j += blockDim.x) {
      const int f = j / kTrRows, i = j - f * kTrRows;
      if (i < rows) XT[(int64_t)f * n + r0 + i] = s_t[i * P + f];
    }
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
                                                         const int64_t* __restrict__ maxb, float* __restrict__ out,
                                                         const uint8_t* __restrict__ want, float* __restrict__ dval,
                                                         int32_t* __restrict__ ndist) {
  extern __shared__ uint32_t s_dyn[];
  const int s = blockIdx.x;
  const int64_t o0 = seg_off[s], o1 = seg_off[s + 1];
  const int len = (int)(o1 - o0);
  const int t0 = tgt_off[s], t1 = tgt_off[s + 1];
  const bool wd = want != nullptr && want[s];
  if (len <= 0 || len > kSkSortCap || (t0 >= t1 && !wd)) return;
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
  if (!wd) return;
  // distinct values of the segment (a feature whose every value may get its own bin): the sorted run's
  // first occurrences, compacted by an inclusive scan of the flags
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += blockDim.x) cum[i] = (i < len && (i == 0 || key[i] != key[i - 1])) ? 1 : 0;
  __syncthreads();
  for (int d = 1; d < P; d <<= 1) {
    int64_t add[kSkSortCap / kSkThreads];
    int c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) add[c] = i >= d ? cum[i - d] : 0;
    __syncthreads();
    c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) cum[i] += add[c];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < len; i += blockDim.x)
    if (i == 0 || key[i] != key[i - 1]) dval[o0 + cum[i] - 1] = fval(key[i]);
  if (threadIdx.x == 0) ndist[s] = (int32_t)cum[len - 1];
}

// Pass 3 with unit weights: the cumulative weight of sorted position i is i + 1, so the weight scan
// goes and target t is the closed form i = clamp(thr / maxb - prefix, 0, len - 1) -- the first i with
// (prefix + i + 1) * maxb > thr (integers, maxb > 0). Keys only in LDS (32 KB, + 32 KB of int32 flags
// for the distinct values): two blocks per CU where the weighted form holds one.
__global__ __launch_bounds__(kSkThreads) void k_sk_select_u(const float* __restrict__ cval, const int64_t* __restrict__ seg_off,
                                                           const int32_t* __restrict__ tgt_off,
                                                           const int64_t* __restrict__ prefix, const int64_t* __restrict__ thr,
                                                           const int64_t* __restrict__ maxb, float* __restrict__ out,
                                                           const uint8_t* __restrict__ want, float* __restrict__ dval,
                                                           int32_t* __restrict__ ndist) {
  extern __shared__ uint32_t s_dyn[];
  const int s = blockIdx.x;
  const int64_t o0 = seg_off[s], o1 = seg_off[s + 1];
  const int len = (int)(o1 - o0);
  const int t0 = tgt_off[s], t1 = tgt_off[s + 1];
  const bool wd = want != nullptr && want[s];
  if (len <= 0 || len > kSkSortCap || (t0 >= t1 && !wd)) return;
  int P = 1;
  while (P < len) P <<= 1;
  uint32_t* key = s_dyn;                 // [P]
  int32_t* cnt = reinterpret_cast<int32_t*>(s_dyn + kSkSortCap);  // [P] distinct flags, then their scan
  for (int i = threadIdx.x; i < P; i += blockDim.x) key[i] = i < len ? fkey(cval[o0 + i]) : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ix = i ^ j;
        if (ix > i) {
          const uint32_t a = key[i], b = key[ix];
          if ((a > b) == ((i & k) == 0)) {
            key[i] = b;
            key[ix] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int t = t0 + threadIdx.x; t < t1; t += blockDim.x) {
    const int64_t i = thr[t] / maxb[t] - prefix[t];
    out[t] = fval(key[min(max(i, (int64_t)0), (int64_t)len - 1)]);
  }
  if (!wd) return;
  for (int i = threadIdx.x; i < P; i += blockDim.x) cnt[i] = (i < len && (i == 0 || key[i] != key[i - 1])) ? 1 : 0;
  __syncthreads();
  for (int d = 1; d < P; d <<= 1) {
    int32_t add[kSkSortCap / kSkThreads];
    int c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) add[c] = i >= d ? cnt[i - d] : 0;
    __syncthreads();
    c = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x, ++c) cnt[i] += add[c];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < len; i += blockDim.x)
    if (i == 0 || key[i] != key[i - 1]) dval[o0 + cnt[i] - 1] = fval(key[i]);
  if (threadIdx.x == 0) ndist[s] = cnt[len - 1];
}

// Exact-bin features (one bin per distinct value when a feature has <= maxb of them), one block per
// feature: the distinct values in bucket order are the sample values whose equal bucket has rows and,
// for a feature with rows in open buckets (every such bucket is a selected segment then), the
// segments' distinct values from k_sk_select. nd[f] = the distinct count (-1: not decidable here, the
// segment was too large for the LDS sort); cut i - 1 = distinct value i (i >= 1) when nd <= maxb.
__global__ __launch_bounds__(1024) void k_sk_exact(const int64_t* __restrict__ cnt, const float* __restrict__ bounds,
                                                   const int32_t* __restrict__ slot, const int64_t* __restrict__ seg_off,
                                                   const int32_t* __restrict__ ndist, const float* __restrict__ dval,
                                                   const int64_t* __restrict__ maxb, float* __restrict__ cuts_ex,
                                                   int64_t* __restrict__ nd) {
  constexpr int kPer = (kSkBuckets + 1023) / 1024;  // buckets per thread (8)
  __shared__ int64_t s_tot[1024 / kWave];
  __shared__ int s_bad;
  const int f = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_bad = 0;
  __syncthreads();
  const int64_t* c = cnt + (int64_t)f * kSkBuckets;
  const int32_t* sl = slot + (int64_t)f * kSkBuckets;
  int k0 = t * kPer;
  int64_t cntd[kPer];
  int64_t mine = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = k0 + q;
    int64_t v = 0;
    if (b < kSkBuckets && c[b] > 0) {
      if (b & 1) {
        v = 1;
      } else {
        const int sg = sl[b];
        if (sg >= 0) {
          v = ndist[sg];
          if (v < 0) atomicOr(&s_bad, 1);
        } else {
          atomicOr(&s_bad, 1);  // rows in an open bucket that is not a segment: not an exact feature
        }
      }
    }
    cntd[q] = v < 0 ? 0 : v;
    mine += cntd[q];
  }
  // exclusive block scan of the per-thread totals
  int64_t incl = mine;
  const int lane = lane_id(), wv = wave_id();
  for (int o = 1; o < kWave; o <<= 1) {
    const int64_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == kWave - 1) s_tot[wv] = incl;
  __syncthreads();
  int64_t base = 0, total = 0;
  for (int i = 0; i < 1024 / kWave; ++i) {
    if (i < wv) base += s_tot[i];
    total += s_tot[i];
  }
  int64_t r = base + incl - mine;
  const bool bad = s_bad != 0;
  const bool fits = !bad && total <= maxb[f];
  if (t == 0) nd[f] = bad ? -1 : total;
  if (!fits) return;
  float* row = cuts_ex + (int64_t)f * 257;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int b = k0 + q;
    if (cntd[q] == 0) continue;
    if (b & 1) {
      if (r >= 1 && r - 1 < 256) row[r - 1] = bounds[(int64_t)f * kSkMaxBounds + (b >> 1)];
    } else {
      const int64_t o = seg_off[sl[b]];
      for (int64_t j = 0; j < cntd[q]; ++j)
        if (r + j >= 1 && r + j - 1 < 256) row[r + j - 1] = dval[o + j];
    }
    r += cntd[q];
  }
}

// ------------------------------------------------------------------------------------------
// The planning between the passes, on the device. The bucket arithmetic between pass 1 and the
// candidate select (boundaries from the sorted sample, slab sums, the target buckets, the selected
// segments and their offsets, the per-target arguments of k_sk_select, the cut tables) was ~150 small
// torch launches and five host synchronisations: ~2 ms per sketch, most of the sketch's wall time
// (1.25M rows: 2.5 ms of which ~0.4 ms kernel time). Here it is six kernels and ONE host read of the
// plan's sizes. Every quantity is the same integer / float arithmetic as the torch form it replaces
// (models/sketch.py keeps the rare host fallbacks), so the cuts stay bit-identical to compute_cuts.
// ------------------------------------------------------------------------------------------
constexpr int kSkT = 255;                                 // targets j = 1..255 per feature
constexpr int kSkPer = (kSkBuckets + 1023) / 1024;        // buckets per thread of a 1024-thread block (9)

// Block-wide exclusive scan of one int64 per thread (1024 threads); `total` = the block's sum in every
// thread. s_w: 16 int64 of LDS. Contains the barriers that publish LDS writes made before the call.
__device__ __forceinline__ int64_t sk_block_excl(int64_t v, int64_t* s_w, int64_t& total) {
  const int lane = lane_id(), wv = wave_id();
  const int64_t incl = wave_incl_scan(v);
  if (lane == kWave - 1) s_w[wv] = incl;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int i = 0; i < (int)(blockDim.x / kWave); ++i) {
    const int64_t x = s_w[i];
    if (i < wv) base += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return base + incl - v;
}

// Boundaries from the sorted strided sample sv [F][S] (NaN last): the values at positions k * cnt / K
// (K = kSkMaxBounds - 1, k = 0..K-1) that differ from their predecessor, compacted; +inf padding.
__global__ __launch_bounds__(1024) void k_sk_bounds(const float* __restrict__ sv, int S, float* __restrict__ bounds,
                                                    int32_t* __restrict__ nbound) {
  constexpr int K = kSkMaxBounds - 1;
  __shared__ int64_t s_w[16];
  __shared__ int s_cnt;
  const int f = blockIdx.x, t = threadIdx.x;
  const float* x = sv + (int64_t)f * S;
  float* bo = bounds + (int64_t)f * kSkMaxBounds;
  if (t == 0) {  // valid values = the index of the first NaN
    int lo = 0, hi = S;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (x[mid] == x[mid]) lo = mid + 1; else hi = mid;
    }
    s_cnt = lo;
  }
  for (int i = t; i < kSkMaxBounds; i += blockDim.x) bo[i] = INFINITY;
  __syncthreads();
  const int64_t cnt = s_cnt;
  float u[4];
  bool nv[4];
  int64_t c = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * t + q;
    nv[q] = false;
    u[q] = 0.0f;
    if (k < K) {
      const int64_t pos = (int64_t)k * cnt / K;
      u[q] = x[min(pos, (int64_t)S - 1)];
      const bool ok = pos < cnt;
      bool diff = true;
      if (k > 0) diff = u[q] != x[min((int64_t)(k - 1) * cnt / K, (int64_t)S - 1)];
      nv[q] = ok && diff;
    }
    c += nv[q] ? 1 : 0;
  }
  int64_t total;
  int64_t r = sk_block_excl(c, s_w, total);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (nv[q]) bo[r++] = u[q];
  if (t == 0) nbound[f] = (int32_t)total;
}

// The boundaries straight from the strided sample (S <= kSkSampleCap values per feature): the sample's
// column is loaded (-0 -> +0; NaN and padding as the largest key, torch.sort's NaN-last order) and
// bitonic-sorted as ordered-float keys, 32 per thread in registers: the stages with partners in the
// same thread (j < 32) are register compare-exchanges, the others go through LDS (element t * 32 + e at
// word e * 1024 + t: conflict-free), then reduced to boundaries as k_sk_bounds does -- one launch
// instead of a segmented torch.sort and k_sk_bounds. value (i, f) = X[i * srow + f * scol].
constexpr int kSkSampleCap = 32768;  // 128 KB of keys in LDS
constexpr int kSkSortE = kSkSampleCap / 1024;  // keys per thread

__global__ __launch_bounds__(1024) void k_sk_sample_bounds(const float* __restrict__ X, int64_t srow, int64_t scol, int S,
                                                           float* __restrict__ bounds, int32_t* __restrict__ nbound) {
  constexpr int K = kSkMaxBounds - 1;
  constexpr int E = kSkSortE;
  extern __shared__ uint32_t s_key[];
  __shared__ int64_t s_w[16];
  const int f = blockIdx.x, t = threadIdx.x;
  uint32_t r[E];
  int64_t valid = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = t * E + e;
    uint32_t k = 0xFFFFFFFFu;
    if (i < S) {
      const float v = X[(int64_t)i * srow + (int64_t)f * scol] + 0.0f;
      if (v == v) {
        k = fkey(v);
        ++valid;
      }
    }
    r[e] = k;
  }
  float* bo = bounds + (int64_t)f * kSkMaxBounds;
  for (int i = t; i < kSkMaxBounds; i += blockDim.x) bo[i] = INFINITY;
  for (int k = 2; k <= kSkSampleCap; k <<= 1) {
    for (int j = k >> 1; j >= E; j >>= 1) {  // partner in thread t ^ (j / E), same register
#pragma unroll
      for (int e = 0; e < E; ++e) s_key[e * 1024 + t] = r[e];
      __syncthreads();
      const int tp = t ^ (j / E);
      const bool lower = t < tp;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint32_t a = r[e], b = s_key[e * 1024 + tp];
        const bool up = ((t * E + e) & k) == 0;
        r[e] = (lower == up) ? min(a, b) : max(a, b);
      }
      __syncthreads();
    }
#pragma unroll
    for (int jj = E / 2; jj >= 1; jj >>= 1) {  // partner in the same thread
      if (jj < k) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int pe = e ^ jj;
          if (pe > e) {
            const uint32_t a = r[e], b = r[pe];
            const bool up = ((t * E + e) & k) == 0;
            const bool sw = (a > b) == up;
            r[e] = sw ? b : a;
            r[pe] = sw ? a : b;
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) s_key[e * 1024 + t] = r[e];
  int64_t cnt;
  sk_block_excl(valid, s_w, cnt);  // (its barriers publish the sorted keys)
  auto key_at = [&](int64_t p) { return s_key[(p % E) * 1024 + p / E]; };
  float u[4];
  bool nv[4];
  int64_t c = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * t + q;
    nv[q] = false;
    u[q] = 0.0f;
    if (k < K) {
      const int64_t pos = (int64_t)k * cnt / K;
      u[q] = fval(key_at(min(pos, (int64_t)S - 1)));
      const bool ok = pos < cnt;
      bool diff = true;
      if (k > 0) diff = u[q] != fval(key_at(min((int64_t)(k - 1) * cnt / K, (int64_t)S - 1)));
      nv[q] = ok && diff;
    }
    c += nv[q] ? 1 : 0;
  }
  int64_t total;
  int64_t rr = sk_block_excl(c, s_w, total);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (nv[q]) bo[rr++] = u[q];
  if (t == 0) nbound[f] = (int32_t)total;
}

// Pass-1 slabs summed into the bucket tables (accumulated: a streamed sketch adds chunk by chunk) and
// the blocks' value ranges into vmin / vmax. grid = (buckets / 256, F).
template <bool kW>
__global__ __launch_bounds__(256) void k_sk_reduce(const uint32_t* __restrict__ cnt_slab,
                                                   const unsigned long long* __restrict__ w_slab,
                                                   const float* __restrict__ bmm, int nblk, int F, int64_t* __restrict__ cnt,
                                                   int64_t* __restrict__ wsum, float* __restrict__ vmin,
                                                   float* __restrict__ vmax) {
  const int f = blockIdx.y;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < kSkBuckets) {
    int64_t s = 0, sw = 0;
    for (int k = 0; k < nblk; ++k) {
      const int64_t row = (int64_t)k * F + f;
      s += cnt_slab[row * kSkBuckets + b];
      if (kW) sw += (int64_t)w_slab[row * kSkBuckets + b];
    }
    cnt[(int64_t)f * kSkBuckets + b] += s;
    if (kW) wsum[(int64_t)f * kSkBuckets + b] += sw;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float a = vmin[f], z = vmax[f];
    for (int k = 0; k < nblk; ++k) {
      a = fminf(a, bmm[((int64_t)k * F + f) * 2]);
      z = fmaxf(z, bmm[((int64_t)k * F + f) * 2 + 1]);
    }
    vmin[f] = a;
    vmax[f] = z;
  }
}

// The plan's device arrays, carved from one int64 workspace (offsets in int64 words: sk_plan_layout).
enum SkArr {
  kSel, kFstat, kFbase, kSummary, kQ0, kThr, kPre, kTb, kNeed, kSlot, kSegFeat, kSegBucket, kLocSizes, kGlobSizes,
  kLocOff, kGlobOff, kTgtOff, kWant, kNdist, kTpos, kTprefix, kTthr, kTmaxb, kSkArrCount
};
// per-feature statistics (kFstat, 5 words): selected buckets, open targets, local / global rows of the
// selected buckets, uncertain flag; bases (kFbase, 4 words): the exclusive prefixes of the first four.
// summary (8 words): nseg, T, local rows, global rows, any uncertain, big segments with targets, big
// segments of uncertain features, 0.
struct SkPlan {
  uint8_t* sel;
  int64_t *fstat, *fbase, *summary;
  float* q0;
  int64_t *thr, *pre;
  int32_t* tb;
  uint8_t* need;
  int32_t *slot, *seg_feat, *seg_bucket;
  int64_t *loc_sizes, *glob_sizes, *loc_off, *glob_off;
  int32_t* tgt_off;
  uint8_t* want;
  int32_t *ndist, *tpos;
  int64_t *tprefix, *tthr, *tmaxb;
};

__host__ inline void sk_plan_layout(int F, int64_t* off) {
  const int64_t SC = (int64_t)F * kSkBuckets, TC = (int64_t)F * kSkT;
  const int64_t words[kSkArrCount] = {
      (SC + 7) / 8, 5LL * F, 4LL * F, 8, (TC + 1) / 2, TC, TC, (TC + 1) / 2, (TC + 7) / 8, (SC + 1) / 2, (SC + 1) / 2,
      (SC + 1) / 2, SC, SC, SC + 1, SC + 1, (SC + 2) / 2, (SC + 7) / 8, (SC + 1) / 2, (TC + 1) / 2, TC, TC, TC};
  int64_t o = 0;
  for (int i = 0; i < kSkArrCount; ++i) {
    off[i] = o;
    o += words[i];
  }
  off[kSkArrCount] = o;
}

__host__ inline SkPlan sk_plan_views(int F, int64_t* ws) {
  int64_t off[kSkArrCount + 1];
  sk_plan_layout(F, off);
  SkPlan p;
  p.sel = reinterpret_cast<uint8_t*>(ws + off[kSel]);
  p.fstat = ws + off[kFstat];
  p.fbase = ws + off[kFbase];
  p.summary = ws + off[kSummary];
  p.q0 = reinterpret_cast<float*>(ws + off[kQ0]);
  p.thr = ws + off[kThr];
  p.pre = ws + off[kPre];
  p.tb = reinterpret_cast<int32_t*>(ws + off[kTb]);
  p.need = reinterpret_cast<uint8_t*>(ws + off[kNeed]);
  p.slot = reinterpret_cast<int32_t*>(ws + off[kSlot]);
  p.seg_feat = reinterpret_cast<int32_t*>(ws + off[kSegFeat]);
  p.seg_bucket = reinterpret_cast<int32_t*>(ws + off[kSegBucket]);
  p.loc_sizes = ws + off[kLocSizes];
  p.glob_sizes = ws + off[kGlobSizes];
  p.loc_off = ws + off[kLocOff];
  p.glob_off = ws + off[kGlobOff];
  p.tgt_off = reinterpret_cast<int32_t*>(ws + off[kTgtOff]);
  p.want = reinterpret_cast<uint8_t*>(ws + off[kWant]);
  p.ndist = reinterpret_cast<int32_t*>(ws + off[kNdist]);
  p.tpos = reinterpret_cast<int32_t*>(ws + off[kTpos]);
  p.tprefix = ws + off[kTprefix];
  p.tthr = ws + off[kTthr];
  p.tmaxb = ws + off[kTmaxb];
  return p;
}

// Plan 1, one block per feature: prefix sums C of the bucket weights, the target bucket b_j of every
// rank j W / maxb (first bucket with C * maxb > j W), its value when b_j is an equal bucket, the
// feature's class (many / exactly known / uncertain distinct values), the open targets and the
// selected buckets (the open targets' buckets; for an uncertain feature also every open bucket with
// rows), and the per-feature totals.
__global__ __launch_bounds__(1024) void k_sk_plan1(const int64_t* __restrict__ cnt_h, const int64_t* __restrict__ w_h,
                                                   const int64_t* __restrict__ cnt_loc, const float* __restrict__ bounds,
                                                   const int64_t* __restrict__ maxb, const float* __restrict__ vmax,
                                                   SkPlan p) {
  __shared__ int64_t s_C[kSkBuckets];
  __shared__ uint8_t s_sel[kSkBuckets];
  __shared__ int64_t s_w[16];
  const int f = blockIdx.x, t = threadIdx.x;
  const int64_t* ch = cnt_h + (int64_t)f * kSkBuckets;
  const int64_t* wh = w_h ? w_h + (int64_t)f * kSkBuckets : ch;
  const int64_t* cl = cnt_loc + (int64_t)f * kSkBuckets;
  const int b0 = t * kSkPer;
  int64_t v[kSkPer];
  int64_t mine = 0, e = 0, o = 0;
#pragma unroll
  for (int q = 0; q < kSkPer; ++q) {
    const int b = b0 + q;
    v[q] = b < kSkBuckets ? wh[b] : 0;
    mine += v[q];
    if (b < kSkBuckets) {
      s_sel[b] = 0;
      if (ch[b] > 0) {
        if (b & 1) ++e; else ++o;
      }
    }
  }
  int64_t W, E, O;
  int64_t run = sk_block_excl(mine, s_w, W);
#pragma unroll
  for (int q = 0; q < kSkPer; ++q) {
    run += v[q];
    if (b0 + q < kSkBuckets) s_C[b0 + q] = run;
  }
  sk_block_excl(e, s_w, E);
  sk_block_excl(o, s_w, O);  // (its barriers publish s_C and the zeroed s_sel)
  const int64_t mb = maxb[f];
  const bool many = E + O > mb, exact_known = O == 0 && E <= mb, uncertain = !many && O > 0;
  int64_t need = 0;
  if (t < kSkT) {
    const int j = t + 1;
    const int64_t th = (int64_t)j * W;
    int lo = 0, hi = kSkBuckets;  // first bucket with C * maxb > j W (searchsorted right), clamped
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_C[mid] * mb > th) hi = mid; else lo = mid + 1;
    }
    const int bt = min(lo, kSkBuckets - 1);
    const bool inb = j < mb, eq = (bt & 1) != 0;
    const int qi = min(max((bt - 1) / 2, 0), kSkMaxBounds - 1);
    const float q = W > 0 ? bounds[(int64_t)f * kSkMaxBounds + qi] : vmax[f];
    need = (inb && !eq && W > 0 && !exact_known) ? 1 : 0;
    const int64_t i = (int64_t)f * kSkT + t;
    p.q0[i] = q;
    p.thr[i] = th;
    p.pre[i] = bt > 0 ? s_C[bt - 1] : 0;
    p.tb[i] = bt;
    p.need[i] = (uint8_t)need;
    if (need) s_sel[bt] = 1;
  }
  __syncthreads();
  if (t == 0) s_sel[kSkBuckets - 1] = 0;  // never a used bucket (m <= kSkMaxBounds - 1)
  __syncthreads();
  if (uncertain)
    for (int b = t; b < kSkBuckets; b += blockDim.x)
      if (!(b & 1) && ch[b] > 0) s_sel[b] = 1;
  __syncthreads();
  int64_t ns = 0, sl = 0, sg = 0;
#pragma unroll
  for (int q = 0; q < kSkPer; ++q) {
    const int b = b0 + q;
    if (b < kSkBuckets) {
      const uint8_t s = s_sel[b];
      p.sel[(int64_t)f * kSkBuckets + b] = s;
      if (s) { ++ns; sl += cl[b]; sg += ch[b]; }
    }
  }
  int64_t NS, NT, SL, SG;
  sk_block_excl(ns, s_w, NS);
  sk_block_excl(need, s_w, NT);
  sk_block_excl(sl, s_w, SL);
  sk_block_excl(sg, s_w, SG);
  if (t == 0) {
    int64_t* fs = p.fstat + 5LL * f;
    fs[0] = NS;
    fs[1] = NT;
    fs[2] = SL;
    fs[3] = SG;
    fs[4] = uncertain ? 1 : 0;
  }
}

// Plan 2 (one thread): the features' bases and the plan summary.
__global__ void k_sk_plan2(int F, SkPlan p) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t a = 0, b = 0, c = 0, d = 0, u = 0;
  for (int f = 0; f < F; ++f) {
    const int64_t* fs = p.fstat + 5LL * f;
    int64_t* fb = p.fbase + 4LL * f;
    fb[0] = a; fb[1] = b; fb[2] = c; fb[3] = d;
    a += fs[0]; b += fs[1]; c += fs[2]; d += fs[3];
    u |= fs[4];
  }
  int64_t* s = p.summary;
  s[0] = a; s[1] = b; s[2] = c; s[3] = d; s[4] = u; s[5] = 0; s[6] = 0; s[7] = 0;
  p.loc_off[a] = c;
  p.glob_off[a] = d;
  p.tgt_off[a] = (int32_t)b;
}

// Plan 3, one block per feature: the global layout -- every bucket's segment (slot), the segments'
// feature / bucket / local and global rows / offsets / first target / distinct-value request, the
// open targets' global index (tpos) and k_sk_select arguments; big segments (beyond the LDS sort) are
// counted in the summary for the host fallbacks.
__global__ __launch_bounds__(1024) void k_sk_plan3(const int64_t* __restrict__ cnt_h, const int64_t* __restrict__ cnt_loc,
                                                   const int64_t* __restrict__ maxb, SkPlan p) {
  __shared__ int64_t s_w[16];
  __shared__ int32_t s_tb[kSkT];
  const int f = blockIdx.x, t = threadIdx.x;
  const int64_t* ch = cnt_h + (int64_t)f * kSkBuckets;
  const int64_t* cl = cnt_loc + (int64_t)f * kSkBuckets;
  const int64_t* fb = p.fbase + 4LL * f;
  const int64_t segbase = fb[0], tgtbase = fb[1], locbase = fb[2], globbase = fb[3];
  const bool unc = p.fstat[5LL * f + 4] != 0;
  const int64_t mb = maxb[f];
  // open targets (ascending j, so ascending bucket)
  const int64_t nd = t < kSkT ? p.need[(int64_t)f * kSkT + t] : 0;
  int64_t nt;
  const int64_t lt = sk_block_excl(nd, s_w, nt);
  if (t < kSkT) {
    const int64_t i = (int64_t)f * kSkT + t;
    const int64_t g = tgtbase + lt;
    p.tpos[i] = nd ? (int32_t)g : -1;
    if (nd) {
      p.tprefix[g] = p.pre[i];
      p.tthr[g] = p.thr[i];
      p.tmaxb[g] = mb;
      s_tb[lt] = p.tb[i];
    }
  }
  // selected buckets: segment index and row offsets
  const int b0 = t * kSkPer;
  int64_t ns = 0, sl = 0, sg = 0;
  uint32_t selm = 0;
#pragma unroll
  for (int q = 0; q < kSkPer; ++q) {
    const int b = b0 + q;
    if (b < kSkBuckets && p.sel[(int64_t)f * kSkBuckets + b]) {
      selm |= 1u << q;
      ++ns;
      sl += cl[b];
      sg += ch[b];
    }
  }
  int64_t tot;
  int64_t es = sk_block_excl(ns, s_w, tot);
  int64_t el = sk_block_excl(sl, s_w, tot);
  int64_t eg = sk_block_excl(sg, s_w, tot);  // (its barriers publish s_tb)
  const int T_f = (int)nt;
#pragma unroll
  for (int q = 0; q < kSkPer; ++q) {
    const int b = b0 + q;
    if (b >= kSkBuckets) break;
    if (!((selm >> q) & 1u)) {
      p.slot[(int64_t)f * kSkBuckets + b] = -1;
      continue;
    }
    const int64_t s = segbase + es;
    p.slot[(int64_t)f * kSkBuckets + b] = (int32_t)s;
    p.seg_feat[s] = f;
    p.seg_bucket[s] = b;
    p.loc_sizes[s] = cl[b];
    p.glob_sizes[s] = ch[b];
    p.loc_off[s] = locbase + el;
    p.glob_off[s] = globbase + eg;
    p.want[s] = unc ? 1 : 0;
    p.ndist[s] = -1;
    int lo = 0, hi = T_f;  // first open target with bucket >= b
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_tb[mid] < b) lo = mid + 1; else hi = mid;
    }
    p.tgt_off[s] = (int32_t)(tgtbase + lo);
    if (ch[b] > kSkSortCap) {  // beyond the LDS sort: the host takes its targets / distinct values
      const bool has_t = lo < T_f && s_tb[lo] == b;
      if (has_t) atomicAdd(reinterpret_cast<unsigned long long*>(p.summary + 5), 1ull);
      if (unc) atomicAdd(reinterpret_cast<unsigned long long*>(p.summary + 6), 1ull);
    }
    ++es;
    el += cl[b];
    eg += ch[b];
  }
}

// Pass-2 block offsets of one chunk: blk_off [nblk][nseg] = cursor + the exclusive prefix over the
// blocks of the chunk's per-block rows of each segment (pass 1's slabs); cursor advances by them.
__global__ __launch_bounds__(256) void k_sk_blkoff(SkPlan p, int nseg, int F, const uint32_t* __restrict__ cnt_slab,
                                                   int nblk, int64_t* __restrict__ cursor, int64_t* __restrict__ blk_off) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const int f = p.seg_feat[s], b = p.seg_bucket[s];
  int64_t run = cursor[s];
  for (int k = 0; k < nblk; ++k) {
    blk_off[(int64_t)k * nseg + s] = run;
    run += cnt_slab[((int64_t)k * F + f) * kSkBuckets + b];
  }
  cursor[s] = run;
}

// The cut tables, one 256-thread block per feature: q_j (the equal bucket's value, or the selected
// candidate of an open target), the quantile path's de-duplicated cuts above the minimum, the exact
// path's distinct values when the feature has <= maxb of them, the sentinel, -0 -> +0.
__global__ __launch_bounds__(256) void k_sk_assemble(SkPlan p, const float* __restrict__ sel_out,
                                                     const float* __restrict__ vmin, const int64_t* __restrict__ maxb,
                                                     const int64_t* __restrict__ nd, const float* __restrict__ cuts_ex,
                                                     float* __restrict__ cuts, int32_t* __restrict__ nbins) {
  __shared__ float s_q[kSkT];
  __shared__ float s_cut[256];
  __shared__ int s_cnt[4];
  const int f = blockIdx.x, t = threadIdx.x;
  const int64_t mb = maxb[f];
  float q = 0.0f;
  if (t < kSkT) {
    const int64_t i = (int64_t)f * kSkT + t;
    const int tp = p.tpos[i];
    q = tp >= 0 ? sel_out[tp] : p.q0[i];
    s_q[t] = q;
  }
  s_cut[t] = FLT_MAX;
  __syncthreads();
  const bool keep = t < kSkT && (t + 1) < mb && q > vmin[f] && (t == 0 || q != s_q[t - 1]);
  const uint64_t bal = __ballot(keep);
  const int wv = wave_id();
  if (lane_id() == 0) s_cnt[wv] = __popcll(bal);
  __syncthreads();
  int base = 0, K = 0;
  for (int w = 0; w < 4; ++w) {
    if (w < wv) base += s_cnt[w];
    K += s_cnt[w];
  }
  if (keep) s_cut[base + mask_rank(bal)] = q;
  __syncthreads();
  const int64_t ndf = nd[f];
  const bool exact = ndf >= 0 && ndf <= mb;
  const int nbv = exact ? (int)(ndf > 0 ? ndf : 1) : K + 1;
  float c = exact ? cuts_ex[(int64_t)f * 257 + t] : s_cut[t];
  if (t == max(nbv - 1, 0)) c = FLT_MAX;
  cuts[(int64_t)f * 256 + t] = c + 0.0f;
  if (t == 0) nbins[f] = nbv;
}

}  // namespace

// bid: nullptr, or [F][ldx] u16 -- every value's bucket for a later cobalt_sk_gather(.., bid) of the same rows
COBALT_API int cobalt_sk_hist(const float* X, int64_t n, int64_t ldx, int F, const int32_t* w, const float* bounds,
                              const int32_t* nbound, int nblk, uint32_t* cnt_slab, void* w_slab, float* bmm,
                              uint16_t* bid, hipStream_t stream) {
  if (F <= 0 || nblk <= 0) return -3;
  const dim3 grid(nblk, F);
  auto* ws = static_cast<unsigned long long*>(w_slab);
#define SK_HIST(KW, KI) \
  hipLaunchKernelGGL((k_sk_hist<KW, KI>), grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, cnt_slab, ws, bmm, bid)
  if (w) {
    if (bid) SK_HIST(true, true); else SK_HIST(true, false);
  } else {
    if (bid) SK_HIST(false, true); else SK_HIST(false, false);
  }
#undef SK_HIST
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_gather(const float* X, int64_t n, int64_t ldx, int F, const int32_t* w, const float* bounds,
                                const int32_t* nbound, const int32_t* slot, const int64_t* blk_off, int nseg,
                                float* cval, int32_t* cw, int nblk, const uint16_t* bid, hipStream_t stream) {
  if (F <= 0 || nblk <= 0 || nseg <= 0) return -3;
  const dim3 grid(nblk, F);
#define SK_GATHER(KW, KI) \
  hipLaunchKernelGGL((k_sk_gather<KW, KI>), grid, dim3(kSkThreads), 0, stream, X, n, ldx, w, bounds, nbound, slot, blk_off, \
                     nseg, cval, cw, bid)
  if (w) {
    if (bid) SK_GATHER(true, true); else SK_GATHER(true, false);
  } else {
    if (bid) SK_GATHER(false, true); else SK_GATHER(false, false);
  }
#undef SK_GATHER
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_transpose(const float* X, int64_t n, int F, float* XT, hipStream_t stream) {
  if (F <= 0 || F > 32 || n <= 0) return -3;
  hipLaunchKernelGGL(k_sk_transpose, dim3((unsigned)((n + kTrRows - 1) / kTrRows)), dim3(256), 0, stream, X, n, F, XT);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_exact(int F, const int64_t* cnt, const float* bounds, const int32_t* slot, const int64_t* seg_off,
                               const int32_t* ndist, const float* dval, const int64_t* maxb, float* cuts_ex, int64_t* nd,
                               hipStream_t stream) {
  if (F <= 0) return -3;
  hipLaunchKernelGGL(k_sk_exact, dim3(F), dim3(1024), 0, stream, cnt, bounds, slot, seg_off, ndist, dval, maxb, cuts_ex,
                     nd);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_select(const float* cval, const int32_t* cw, const int64_t* seg_off, int nseg,
                                const int32_t* tgt_off, const int64_t* prefix, const int64_t* thr, const int64_t* maxb,
                                float* out, const uint8_t* want, float* dval, int32_t* ndist, hipStream_t stream) {
  if (nseg <= 0) return 0;
  const size_t lds = (size_t)kSkSortCap * (sizeof(uint32_t) + sizeof(int64_t));
  const size_t lds_u = (size_t)kSkSortCap * (sizeof(uint32_t) + sizeof(int32_t));
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute((const void*)k_sk_select<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_sk_select_u, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_u));
    attr = true;
  }
  if (cw)
    hipLaunchKernelGGL(k_sk_select<true>, dim3(nseg), dim3(kSkThreads), lds, stream, cval, cw, seg_off, tgt_off, prefix,
                       thr, maxb, out, want, dval, ndist);
  else
    hipLaunchKernelGGL(k_sk_select_u, dim3(nseg), dim3(kSkThreads), lds_u, stream, cval, seg_off, tgt_off, prefix, thr,
                       maxb, out, want, dval, ndist);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_bounds() { return kSkMaxBounds; }
COBALT_API int cobalt_sk_buckets() { return kSkBuckets; }
COBALT_API int cobalt_sk_sort_cap() { return kSkSortCap; }

// ---- the device planning (see k_sk_plan1) ----
COBALT_API int cobalt_sk_bounds_build(const float* sv, int F, int S, float* bounds, int32_t* nbound, hipStream_t stream) {
  if (F <= 0 || S <= 0) return -3;
  hipLaunchKernelGGL(k_sk_bounds, dim3(F), dim3(1024), 0, stream, sv, S, bounds, nbound);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_reduce(const uint32_t* cnt_slab, const void* w_slab, const float* bmm, int nblk, int F,
                                int64_t* cnt, int64_t* wsum, float* vmin, float* vmax, hipStream_t stream) {
  if (F <= 0 || nblk <= 0) return -3;
  const dim3 grid((kSkBuckets + 255) / 256, F);
  if (w_slab)
    hipLaunchKernelGGL(k_sk_reduce<true>, grid, dim3(256), 0, stream, cnt_slab,
                       static_cast<const unsigned long long*>(w_slab), bmm, nblk, F, cnt, wsum, vmin, vmax);
  else
    hipLaunchKernelGGL(k_sk_reduce<false>, grid, dim3(256), 0, stream, cnt_slab, nullptr, bmm, nblk, F, cnt, wsum, vmin,
                       vmax);
  CK_LAUNCH();
  return 0;
}

// int64 word offsets of the plan's arrays inside its workspace (kSkArrCount + 1 entries, the last = the
// workspace size), in SkArr order.
COBALT_API int cobalt_sk_plan_layout(int F, int64_t* off) {
  if (F <= 0) return -3;
  sk_plan_layout(F, off);
  return kSkArrCount;
}

// Plan 1-3 over the (global) bucket tables, then ONE host read of the summary (8 int64 to `summary_host`).
// w_h: nullptr = unit weights (cnt_h); cnt_loc: this rank's counts (== cnt_h on one rank).
COBALT_API int cobalt_sk_plan(int F, const int64_t* cnt_h, const int64_t* w_h, const int64_t* cnt_loc, const float* bounds,
                              const int64_t* maxb, const float* vmax, int64_t* ws, int64_t* summary_host,
                              hipStream_t stream) {
  if (F <= 0) return -3;
  const SkPlan p = sk_plan_views(F, ws);
  hipLaunchKernelGGL(k_sk_plan1, dim3(F), dim3(1024), 0, stream, cnt_h, w_h, cnt_loc, bounds, maxb, vmax, p);
  CK_LAUNCH();
  hipLaunchKernelGGL(k_sk_plan2, dim3(1), dim3(64), 0, stream, F, p);
  CK_LAUNCH();
  hipLaunchKernelGGL(k_sk_plan3, dim3(F), dim3(1024), 0, stream, cnt_h, cnt_loc, maxb, p);
  CK_LAUNCH();
  static int64_t* pinned = nullptr;
  if (!pinned) CK(hipHostMalloc((void**)&pinned, 8 * sizeof(int64_t), hipHostMallocDefault));
  CK(hipMemcpyAsync(pinned, p.summary, 8 * sizeof(int64_t), hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  for (int i = 0; i < 8; ++i) summary_host[i] = pinned[i];
  return 0;
}

COBALT_API int cobalt_sk_blkoff(int F, int64_t* ws, int nseg, const uint32_t* cnt_slab, int nblk, int64_t* cursor,
                                int64_t* blk_off, hipStream_t stream) {
  if (F <= 0 || nblk <= 0) return -3;
  if (nseg <= 0) return 0;
  hipLaunchKernelGGL(k_sk_blkoff, dim3((nseg + 255) / 256), dim3(256), 0, stream, sk_plan_views(F, ws), nseg, F, cnt_slab,
                     nblk, cursor, blk_off);
  CK_LAUNCH();
  return 0;
}

// sel_out: k_sk_select's answers by global target index (nullptr when there are no open targets);
// nd / cuts_ex: k_sk_exact's (after any host fallback). cuts [F][256], nbins [F] int32.
COBALT_API int cobalt_sk_assemble(int F, int64_t* ws, const float* sel_out, const float* vmin, const int64_t* maxb,
                                  const int64_t* nd, const float* cuts_ex, float* cuts, int32_t* nbins, hipStream_t stream) {
  if (F <= 0) return -3;
  hipLaunchKernelGGL(k_sk_assemble, dim3(F), dim3(256), 0, stream, sk_plan_views(F, ws), sel_out, vmin, maxb, nd, cuts_ex,
                     cuts, nbins);
  CK_LAUNCH();
  return 0;
}

// Boundaries from the strided sample without a torch sort (k_sk_sample_bounds); -4: S beyond the LDS sort.
COBALT_API int cobalt_sk_sample_bounds(const float* X, int64_t srow, int64_t scol, int S, int F, float* bounds,
                                       int32_t* nbound, hipStream_t stream) {
  if (F <= 0 || S <= 0) return -3;
  if (S > kSkSampleCap) return -4;
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute((const void*)k_sk_sample_bounds, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)(kSkSampleCap * sizeof(uint32_t))));
    attr = true;
  }
  hipLaunchKernelGGL(k_sk_sample_bounds, dim3(F), dim3(1024), (size_t)kSkSampleCap * sizeof(uint32_t), stream, X, srow,
                     scol, S, bounds, nbound);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_sample_cap() { return kSkSampleCap; }
