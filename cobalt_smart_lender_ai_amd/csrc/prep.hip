// Tabular preprocessing kernels (K1-K9, K11, K30 in SURVEY.md §2.4) for gfx950.
//
// Replace the pandas/NumPy/sklearn C loops behind the reference's cleaning and feature-engineering
// steps (src/data_preprocessing/clean_data.py:31-158, feature_engineering.py:44-184) and the
// notebook's outlier/scaler utilities (notebooks/01_data_cleaning.ipynb:10742, 04:3739).
//
// Data layout: a numeric frame is column-major fp64 [C][N] (each pandas column contiguous), so every
// per-column pass is fully coalesced; per-row passes read C coalesced streams.
#include "common.h"

using namespace cobalt;

// K1: per-column NaN counts. grid = (blocks_per_col, C); wave ballot + popcount, one atomic per wave.
__global__ __launch_bounds__(256) void k_col_null_counts(const double* __restrict__ X, int64_t n, int C,
                                                         unsigned long long* __restrict__ out) {
  const int c = blockIdx.y;
  const double* col = X + (int64_t)c * n;
  unsigned long long cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = col[i];
    cnt += __popcll(__ballot(v != v)) * (lane_id() == 0);
  }
  // lanes other than 0 carry 0; sum the wave's lane-0 partials
  if (lane_id() == 0 && cnt) atomicAdd(out + c, cnt);
}

// K2: per-row NaN counts over the C columns (optionally a subset given by a column mask).
__global__ __launch_bounds__(256) void k_row_null_counts(const double* __restrict__ X, int64_t n, int C,
                                                         const uint8_t* __restrict__ colmask, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int cnt = 0;
    for (int c = 0; c < C; ++c) {
      if (colmask && !colmask[c]) continue;
      const double v = X[(int64_t)c * n + i];
      cnt += (v != v);
    }
    out[i] = cnt;
  }
}

// K6: masked log1p on the selected columns, in place: x -> log1p(x) where x > 0 (NaN, 0 and
// negatives unchanged), the element-wise rule of feature_engineering.py:133-139 without the
// per-element Python lambda.
__global__ __launch_bounds__(256) void k_masked_log1p(double* __restrict__ X, int64_t n, const int32_t* __restrict__ cols,
                                                      int ncols) {
  const int c = cols[blockIdx.y];
  double* col = X + (int64_t)c * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = col[i];
    if (v > 0.0) col[i] = log1p(v);
  }
}

// K3 + K5 fused: fill NaN of column cols[j] with values[j] and write the missing indicator (int8).
__global__ __launch_bounds__(256) void k_fill_indicator(double* __restrict__ X, int64_t n, const int32_t* __restrict__ cols,
                                                        const double* __restrict__ values, int8_t* __restrict__ ind) {
  const int j = blockIdx.y;
  double* col = X + (int64_t)cols[j] * n;
  const double fill = values[j];
  int8_t* o = ind ? ind + (int64_t)j * n : nullptr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = col[i];
    const bool miss = v != v;
    if (o) o[i] = miss ? 1 : 0;
    if (miss) col[i] = fill;
  }
}

// K9: 64-bit row hash for duplicate detection (NaN canonicalised so NaN == NaN as in pandas).
__global__ __launch_bounds__(256) void k_row_hash(const double* __restrict__ X, int64_t n, int C,
                                                  uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int c = 0; c < C; ++c) {
      double v = X[(int64_t)c * n + i];
      uint64_t bits = (v != v) ? 0x7FF8000000000000ull : (v == 0.0 ? 0ull : __double_as_longlong(v));
      h = splitmix64(h ^ (bits + 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1)));
    }
    out[i] = h;
  }
}

// Row-equality check of candidate duplicates: eq[k] = rows a[k] and b[k] are identical (NaN == NaN).
__global__ __launch_bounds__(256) void k_rows_equal(const double* __restrict__ X, int64_t n, int C,
                                                    const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                    int64_t m, uint8_t* __restrict__ eq) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
    bool same = true;
    for (int c = 0; c < C && same; ++c) {
      const double x = X[(int64_t)c * n + a[k]], y = X[(int64_t)c * n + b[k]];
      same = (x == y) || (x != x && y != y);
    }
    eq[k] = same;
  }
}

// K7: one-hot of dictionary codes with drop_first: out[i][code-1] = 1 for code >= 1; code < 0 (NaN
// category) -> all zeros (pandas get_dummies(dummy_na=False) semantics).
__global__ __launch_bounds__(256) void k_onehot(const int32_t* __restrict__ codes, int64_t n, int levels, int drop_first,
                                                uint8_t* __restrict__ out) {
  const int w = levels - (drop_first ? 1 : 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = codes[i] - (drop_first ? 1 : 0);
    uint8_t* row = out + i * w;
    for (int k = 0; k < w; ++k) row[k] = (uint8_t)(k == c);
  }
}

// K11/K30: per-column sum, sum of squares, min, max over non-NaN values (fp64); grid.y = column.
__global__ __launch_bounds__(256) void k_col_moments(const double* __restrict__ X, int64_t n, double* __restrict__ out) {
  // out[c*5 + {0 count, 1 sum, 2 sumsq, 3 min, 4 max}]; min/max via atomic CAS on ordered bits
  const int c = blockIdx.y;
  const double* col = X + (int64_t)c * n;
  double s = 0, s2 = 0, mn = INFINITY, mx = -INFINITY, k = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = col[i];
    if (v == v) { s += v; s2 += v * v; mn = fmin(mn, v); mx = fmax(mx, v); k += 1; }
  }
  __shared__ double sh[5][4];
  s = wave_sum(s); s2 = wave_sum(s2); k = wave_sum(k); mn = wave_min(mn); mx = wave_max(mx);
  if (lane_id() == 0) { sh[0][wave_id()] = k; sh[1][wave_id()] = s; sh[2][wave_id()] = s2; sh[3][wave_id()] = mn; sh[4][wave_id()] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) { k += sh[0][w]; s += sh[1][w]; s2 += sh[2][w]; mn = fmin(mn, sh[3][w]); mx = fmax(mx, sh[4][w]); }
    double* o = out + c * 5;
    atomicAdd(o + 0, k);
    atomicAdd(o + 1, s);
    atomicAdd(o + 2, s2);
    // ordered-integer trick for fp64 min/max
    unsigned long long* omn = reinterpret_cast<unsigned long long*>(o + 3);
    unsigned long long* omx = reinterpret_cast<unsigned long long*>(o + 4);
    unsigned long long cur = *omn;
    while (mn < __longlong_as_double(cur)) {
      unsigned long long prev = atomicCAS(omn, cur, __double_as_longlong(mn));
      if (prev == cur) break;
      cur = prev;
    }
    cur = *omx;
    while (mx > __longlong_as_double(cur)) {
      unsigned long long prev = atomicCAS(omx, cur, __double_as_longlong(mx));
      if (prev == cur) break;
      cur = prev;
    }
  }
}

// K30 transform: (x - min) / (max - min) per column (zero range -> 0), NaN preserved; float32 out.
__global__ __launch_bounds__(256) void k_minmax_apply(const double* __restrict__ X, int64_t n, const double* __restrict__ mn,
                                                      const double* __restrict__ mx, float* __restrict__ out_rowmajor, int C) {
  const int c = blockIdx.y;
  const double lo = mn[c], rng = mx[c] - mn[c];
  const double sc = rng > 0 ? 1.0 / rng : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = X[(int64_t)c * n + i];
    out_rowmajor[i * C + c] = (float)((v - lo) * sc);
  }
}


// K10 (ingest): 64-bit hash of every string of an Arrow string column, one thread per string, so a
// near-unique text column (url, titles) never needs a host dictionary: the hash stands in for the
// value in null counts and row dedupe (equal strings -> equal hash; candidate duplicates are verified
// exactly on the host). Mirrors prep_ops._string_hash_host: h = len ^ seed, then splitmix64 over the
// little-endian 8-byte words (zero padded); 0 is reserved for missing.
__global__ __launch_bounds__(256) void k_str_hash(const uint8_t* __restrict__ data, const int64_t* __restrict__ off,
                                                  const uint8_t* __restrict__ valid, int64_t n,
                                                  unsigned long long* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) { out[i] = 0ull; continue; }
    const int64_t b = off[i], e = off[i + 1];
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(e - b);
    for (int64_t p = b; p < e; p += 8) {
      uint64_t w = 0;
      const int m = (int)((e - p) < 8 ? (e - p) : 8);
      for (int j = 0; j < m; ++j) w |= (uint64_t)data[p + j] << (8 * j);
      h = splitmix64(h ^ w);
    }
    out[i] = h ? h : 1ull;
  }
}

static dim3 col_grid(int64_t n, int C) {
  return dim3(std::max(1, std::min(ceil_div(n, 256), 512)), C);
}

COBALT_API int cobalt_col_null_counts(const double* X, int64_t n, int C, unsigned long long* out, hipStream_t s) {
  if (n <= 0 || C <= 0) return 0;
  CK(hipMemsetAsync(out, 0, C * sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_col_null_counts, col_grid(n, C), dim3(256), 0, s, X, n, C, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_row_null_counts(const double* X, int64_t n, int C, const uint8_t* colmask, int32_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_row_null_counts, dim3(std::min(ceil_div(n, 256), 4096)), dim3(256), 0, s, X, n, C, colmask, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_masked_log1p(double* X, int64_t n, const int32_t* cols, int ncols, hipStream_t s) {
  if (n <= 0 || ncols <= 0) return 0;
  hipLaunchKernelGGL(k_masked_log1p, col_grid(n, ncols), dim3(256), 0, s, X, n, cols, ncols);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_fill_indicator(double* X, int64_t n, const int32_t* cols, const double* values, int ncols,
                                     int8_t* ind, hipStream_t s) {
  if (n <= 0 || ncols <= 0) return 0;
  hipLaunchKernelGGL(k_fill_indicator, col_grid(n, ncols), dim3(256), 0, s, X, n, cols, values, ind);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_row_hash(const double* X, int64_t n, int C, uint64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_row_hash, dim3(std::min(ceil_div(n, 256), 4096)), dim3(256), 0, s, X, n, C, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_rows_equal(const double* X, int64_t n, int C, const int64_t* a, const int64_t* b, int64_t m,
                                 uint8_t* eq, hipStream_t s) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(k_rows_equal, dim3(std::min(ceil_div(m, 256), 4096)), dim3(256), 0, s, X, n, C, a, b, m, eq);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_onehot(const int32_t* codes, int64_t n, int levels, int drop_first, uint8_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_onehot, dim3(std::min(ceil_div(n, 256), 4096)), dim3(256), 0, s, codes, n, levels, drop_first, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_col_moments(const double* X, int64_t n, int C, double* out, hipStream_t s) {
  if (C <= 0) return 0;
  // init: count/sum/sumsq = 0, min = +inf, max = -inf (host-prepared buffer is simpler)
  hipLaunchKernelGGL(k_col_moments, col_grid(n, C), dim3(256), 0, s, X, n, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_minmax_apply(const double* X, int64_t n, int C, const double* mn, const double* mx, float* out,
                                   hipStream_t s) {
  if (n <= 0 || C <= 0) return 0;
  hipLaunchKernelGGL(k_minmax_apply, col_grid(n, C), dim3(256), 0, s, X, n, mn, mx, out, C);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_str_hash(const uint8_t* data, const int64_t* off, const uint8_t* valid, int64_t n,
                               unsigned long long* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_str_hash, dim3(std::min(ceil_div(n, 256), 8192)), dim3(256), 0, s, data, off, valid, n, out);
  CK_LAUNCH();
  return 0;
}
