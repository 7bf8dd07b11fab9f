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
// kIds: every value's bucket also goes to bid [F][ldx] (u16, 0xFFFF = missing), so pass 2 (k_sk_gather<..,
// true>) reads 2 bytes per value instead of repeating the 12-step search (the in-core sketch, one chunk).
template <bool kW, bool kIds>
__global__ __launch_bounds__(kSkThreads) void k_sk_hist(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                       const int32_t* __restrict__ w, const float* __restrict__ bounds,
                                                       const int32_t* __restrict__ nbound, uint32_t* __restrict__ cnt_slab,
                                                       unsigned long long* __restrict__ w_slab, float* __restrict__ bmm,
                                                       uint16_t* __restrict__ bid) {
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
      b = sk_bucket(s_u, m, v);
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
  __shared__ float s_u[kSkMaxBounds];
  __shared__ int32_t s_slot[kSkBuckets];
  // per selected bucket: this block's rows written so far (relative to the block's int64 segment offset
  // bo[segment]: a streamed sketch accumulates offsets across chunks, past 2^32 candidates at billions of
  // rows, while one block's count always fits 32 bits)
  __shared__ uint32_t s_cur[kSkBuckets];
  const int f = blockIdx.y;
  if (!kIds) sk_load_bounds(s_u, bounds, f);
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
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
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
      b = sk_bucket(s_u, m, v);
    }
    const int sg = s_slot[b];
    if (sg < 0) continue;
    const int64_t pos = bo[sg] + (int64_t)atomicAdd(&s_cur[b], 1u);
    cval[pos] = v;
    if (kW) cw[pos] = w[r];
  }
}

// Row-major X [n][F] -> feature-major XT [F][n] (F <= 32): a tile of 256 rows is read as one
// contiguous run into LDS (rows padded to F + 1 words: conflict-free column reads), then written as
// F runs of 256 values.
constexpr int kTrRows = 256;
__global__ __launch_bounds__(256) void k_sk_transpose(const float* __restrict__ X, int64_t n, int F,
                                                      float* __restrict__ XT) {
  __shared__ float s_t[kTrRows * 33];
  const int64_t r0 = (int64_t)blockIdx.x * kTrRows;
  const int rows = (int)min((int64_t)kTrRows, n - r0);
  const float* src = X + r0 * F;
  for (int j = threadIdx.x; j < rows * F; j += blockDim.x) {
    const int i = j / F, f = j - i * F;
    s_t[i * (F + 1) + f] = src[j];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < kTrRows * F; j += blockDim.x) {
    const int f = j / kTrRows, i = j - f * kTrRows;
    if (i < rows) XT[(int64_t)f * n + r0 + i] = s_t[i * (F + 1) + f];
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
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute((const void*)k_sk_select<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_sk_select<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  if (cw)
    hipLaunchKernelGGL(k_sk_select<true>, dim3(nseg), dim3(kSkThreads), lds, stream, cval, cw, seg_off, tgt_off, prefix,
                       thr, maxb, out, want, dval, ndist);
  else
    hipLaunchKernelGGL(k_sk_select<false>, dim3(nseg), dim3(kSkThreads), lds, stream, cval, cw, seg_off, tgt_off,
                       prefix, thr, maxb, out, want, dval, ndist);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_sk_bounds() { return kSkMaxBounds; }
COBALT_API int cobalt_sk_buckets() { return kSkBuckets; }
COBALT_API int cobalt_sk_sort_cap() { return kSkSortCap; }
