// Tree-ensemble inference (K21) and path-dependent TreeSHAP (K22) for gfx950.
//
// Replaces XGBoost's predictor (`predict_proba`, reference src/api/cobalt_fast_api.py:90-91,
// src/model_train_test/model_tree_train_test.py:171-172) and SHAP's C TreeSHAP extension
// (`shap.TreeExplainer(...).shap_values`, src/api/cobalt_fast_api.py:46,100).
//
// Forest layout (built on the host at model load, ops/predict_ops.py): every tree is renumbered in
// BFS order so the right child is always left+1; a node is 8 bytes
//   uint32 meta = left_child(16 bits, 0xFFFF = leaf) | feature(15 bits) << 16 | default_left << 31
//   float  val  = split threshold (x < val goes left) or leaf value
// Trees are grouped into tiles of <= tile_cap nodes that are staged in LDS; each thread walks
// one row (features staged in LDS with an odd stride, conflict-free) through every tree of the
// tile, accumulating the margin in fp32 in tree order (XGBoost CPU predictor semantics).
//
// TreeSHAP follows the path formulation (every root->leaf path with repeated features merged into
// one element: feature, [lo, hi) interval, NaN-follows flag, product of cover ratios): one thread
// per (row, path) runs EXTEND over the path and the UNWOUND sum per element in fp64, contributions
// are reduced per block in LDS and flushed with one fp64 atomic per (row, feature).
#include "common.h"
#include "knobs.h"
#include <algorithm>

using namespace cobalt;

namespace {
// LDS tile capacity (nodes) is chosen per model by the host packer (ops/predict_ops.py
// pack_forest: 2048 unless one tree is larger) and passed to the launch. Small tiles keep the
// per-block LDS footprint low -> more resident blocks per CU, which is what bounds this
// latency-bound walk: 125M-row scoring went 490M (6144-node tiles) -> 810M rows/s (2048).
constexpr int kMaxTileNodes = 8192;
constexpr int kMaxPath = 16;       // max unique elements per path (incl. bias) in the SHAP kernel
}

// ------------------------------------------------------------------------------------ predictor
// A tree walk is a chain of dependent LDS reads (node -> feature value -> next node), so one
// thread walks kWalk trees at once: the kWalk chains' loads are independent and overlap. The leaf
// values are still added to the margin one tree at a time in tree order (same fp32 sum).
// kWalk is the default; COBALT_PRED_WALK=2|8 selects the other instantiations for sweeps.
constexpr int kWalk = 4;

template <int kWalk = ::kWalk, typename Leaf>
__device__ __forceinline__ void walk_trees(const uint2* s_nodes, const int32_t* __restrict__ tree_ptr, int nbase,
                                           int t_begin, int t_end, const float* x, Leaf&& leaf) {
  for (int t = t_begin; t < t_end; t += kWalk) {
    uint32_t base[kWalk];
    uint2 nd[kWalk];
#pragma unroll
    for (int k = 0; k < kWalk; ++k) {  // past the tile's end: walk tree t again, result unused
      base[k] = (uint32_t)(tree_ptr[t + k < t_end ? t + k : t] - nbase);
      nd[k] = s_nodes[base[k]];
    }
    bool more = true;
    while (more) {
      more = false;
#pragma unroll
      for (int k = 0; k < kWalk; ++k) {
        if ((nd[k].x & 0xFFFFu) != 0xFFFFu) {
          const int f = (nd[k].x >> 16) & 0x7FFF;
          const float v = x[f];
          const bool left = (v != v) ? ((nd[k].x >> 31) != 0) : (v < __uint_as_float(nd[k].y));
          nd[k] = s_nodes[base[k] + (nd[k].x & 0xFFFFu) + (left ? 0u : 1u)];
          more = true;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kWalk; ++k)
      if (t + k < t_end) leaf(t + k, __uint_as_float(nd[k].y));
  }
}

template <int W>
__global__ __launch_bounds__(256) void k_predict(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                                 const uint2* __restrict__ nodes, const int32_t* __restrict__ tree_ptr,
                                                 const int32_t* __restrict__ tile_ptr, int n_tiles, float base_margin,
                                                 float* __restrict__ out_margin, float* __restrict__ out_prob,
                                                 int tile_cap) {
  extern __shared__ unsigned char smem[];
  uint2* s_nodes = reinterpret_cast<uint2*>(smem);
  float* s_x = reinterpret_cast<float*>(smem + (size_t)tile_cap * sizeof(uint2));
  const int xs = F | 1;  // odd stride -> conflict-free LDS reads
  const int64_t row0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t row = row0 + threadIdx.x;
  const int nrows = (int)min((int64_t)blockDim.x, n - row0);
  // stage the block's rows (coalesced over the contiguous [nrows][F] slab when ldx == F)
  for (int e = threadIdx.x; e < nrows * F; e += blockDim.x) {
    const int r = e / F, f = e - r * F;
    s_x[r * xs + f] = X[(row0 + r) * ldx + f];
  }
  float acc = base_margin;
  const float* x = s_x + threadIdx.x * xs;
  for (int tile = 0; tile < n_tiles; ++tile) {
    const int t_begin = tile_ptr[tile], t_end = tile_ptr[tile + 1];
    const int nbase = tree_ptr[t_begin];
    const int nn = tree_ptr[t_end] - nbase;
    __syncthreads();
    for (int i = threadIdx.x; i < nn; i += blockDim.x) s_nodes[i] = nodes[nbase + i];
    __syncthreads();
    if (row < n) walk_trees<W>(s_nodes, tree_ptr, nbase, t_begin, t_end, x, [&](int, float v) { acc += v; });
  }
  if (row < n) {
    if (out_margin) out_margin[row] = acc;
    if (out_prob) out_prob[row] = 1.0f / (1.0f + expf(-acc));
  }
}

COBALT_API int cobalt_predict(const float* X, int64_t n, int F, int64_t ldx, const void* nodes, const int32_t* tree_ptr,
                              const int32_t* tile_ptr, int n_tiles, int tile_cap, float base_margin,
                              float* out_margin, float* out_prob, hipStream_t stream) {
  if (n <= 0) return 0;
  if (tile_cap < 1 || tile_cap > kMaxTileNodes) return -2;
  const int block = 256;
  const size_t lds = (size_t)tile_cap * sizeof(uint2) + (size_t)block * (F | 1) * sizeof(float);
  if (lds > 160 * 1024) return -3;
  static const int walk = [] {
    const int w = cobalt::knob_int(cobalt::Knob::PredWalk, kWalk);
    return (w == 2 || w == 8) ? w : kWalk;
  }();
  const void* fn = walk == 2 ? (const void*)k_predict<2> : walk == 8 ? (const void*)k_predict<8>
                                                                       : (const void*)k_predict<kWalk>;
  static size_t attr_set = 64 * 1024;
  if (lds > attr_set) {
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = lds;
  }
  const int grid = ceil_div(n, block);
  const uint2* nd = static_cast<const uint2*>(nodes);
  if (walk == 2)
    hipLaunchKernelGGL(k_predict<2>, dim3(grid), dim3(block), lds, stream, X, n, F, ldx, nd, tree_ptr, tile_ptr,
                       n_tiles, base_margin, out_margin, out_prob, tile_cap);
  else if (walk == 8)
    hipLaunchKernelGGL(k_predict<8>, dim3(grid), dim3(block), lds, stream, X, n, F, ldx, nd, tree_ptr, tile_ptr,
                       n_tiles, base_margin, out_margin, out_prob, tile_cap);
  else
    hipLaunchKernelGGL(k_predict<kWalk>, dim3(grid), dim3(block), lds, stream, X, n, F, ldx, nd, tree_ptr, tile_ptr,
                       n_tiles, base_margin, out_margin, out_prob, tile_cap);
  CK_LAUNCH();
  return 0;
}

// Small/medium batches: the row-block kernel above gives each block ALL trees, so n / 256 blocks
// would leave most CUs idle (a 1-row request streamed the whole 59k-node forest through one CU).
// Here the grid is (row blocks x tree tiles); each block writes its rows' leaf values of its tile's
// trees to leaves[t][row], and k_sum_leaves adds them per row in tree order starting from the base
// margin -- the same fp32 sequence as k_predict, so results are bit-identical across the paths.
__global__ __launch_bounds__(256) void k_predict_leaves(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                                        const uint2* __restrict__ nodes,
                                                        const int32_t* __restrict__ tree_ptr,
                                                        const int32_t* __restrict__ tile_ptr,
                                                        float* __restrict__ leaves, int tile_cap) {
  extern __shared__ unsigned char smem[];
  uint2* s_nodes = reinterpret_cast<uint2*>(smem);
  float* s_x = reinterpret_cast<float*>(smem + (size_t)tile_cap * sizeof(uint2));
  const int xs = F | 1;
  const int64_t row0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t row = row0 + threadIdx.x;
  const int nrows = (int)min((int64_t)blockDim.x, n - row0);
  const int tile = blockIdx.y;
  const int t_begin = tile_ptr[tile], t_end = tile_ptr[tile + 1];
  const int nbase = tree_ptr[t_begin];
  const int nn = tree_ptr[t_end] - nbase;
  for (int e = threadIdx.x; e < nrows * F; e += blockDim.x) {
    const int r = e / F, f = e - r * F;
    s_x[r * xs + f] = X[(row0 + r) * ldx + f];
  }
  for (int i = threadIdx.x; i < nn; i += blockDim.x) s_nodes[i] = nodes[nbase + i];
  __syncthreads();
  if (row >= n) return;
  const float* x = s_x + threadIdx.x * xs;
  walk_trees(s_nodes, tree_ptr, nbase, t_begin, t_end, x,
             [&](int t, float v) { leaves[(int64_t)t * n + row] = v; });
}

__global__ void k_sum_leaves(const float* __restrict__ leaves, int64_t n, int T, float base_margin,
                             float* __restrict__ out_margin, float* __restrict__ out_prob) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  float acc = base_margin;
  for (int t = 0; t < T; ++t) acc += leaves[(int64_t)t * n + row];
  if (out_margin) out_margin[row] = acc;
  if (out_prob) out_prob[row] = 1.0f / (1.0f + expf(-acc));
}

// Rows below which the tile-parallel path is used (fewer than ~2 row blocks per CU otherwise).
COBALT_API int64_t cobalt_predict_small_rows() { return 131072; }

COBALT_API int cobalt_predict_small(const float* X, int64_t n, int F, int64_t ldx, const void* nodes,
                                    const int32_t* tree_ptr, const int32_t* tile_ptr, int n_tiles, int tile_cap,
                                    int n_trees, float base_margin, float* leaves, float* out_margin,
                                    float* out_prob, hipStream_t stream) {
  if (n <= 0) return 0;
  if (tile_cap < 1 || tile_cap > kMaxTileNodes) return -2;
  const int block = 256;
  const size_t lds = (size_t)tile_cap * sizeof(uint2) + (size_t)block * (F | 1) * sizeof(float);
  if (lds > 160 * 1024) return -3;
  static size_t attr_set = 64 * 1024;
  if (lds > attr_set) {
    CK(hipFuncSetAttribute((const void*)k_predict_leaves, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = lds;
  }
  hipLaunchKernelGGL(k_predict_leaves, dim3(ceil_div(n, block), n_tiles), dim3(block), lds, stream, X, n, F, ldx,
                     static_cast<const uint2*>(nodes), tree_ptr, tile_ptr, leaves, tile_cap);
  CK_LAUNCH();
  hipLaunchKernelGGL(k_sum_leaves, dim3(ceil_div(n, 256)), dim3(256), 0, stream, leaves, n, n_trees, base_margin,
                     out_margin, out_prob);
  CK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------ TreeSHAP
struct PathElem {
  float lo, hi;        // row follows the path on this feature iff lo <= x < hi (non-missing)
  int32_t feat;        // feature index
  int32_t nan_ok;      // row with NaN follows the path on this feature
  double zero;         // product of cover(child)/cover(parent) over the merged occurrences
};
static_assert(sizeof(PathElem) == 24, "PathElem");

// EXTEND / UNWIND without per-step divisions: the integer ratios (j + 1) / (l + 1) fold to constants of
// the unrolled loops, 1 / (k - j) comes from kShapInv and 1 / zero is taken once per element; both SHAP
// kernels (and so the pattern tables) use the same operation order, so their values stay bit-identical
// to each other (and within rounding of the division form and of the host oracle).
__constant__ double kShapInv[18] = {0.0,       1.0,        1.0 / 2,  1.0 / 3,  1.0 / 4,  1.0 / 5,
                                    1.0 / 6,   1.0 / 7,    1.0 / 8,  1.0 / 9,  1.0 / 10, 1.0 / 11,
                                    1.0 / 12,  1.0 / 13,   1.0 / 14, 1.0 / 15, 1.0 / 16, 1.0 / 17};

// Canonical summation order (shared by both SHAP kernels, so a row's values do not depend on the
// batch size or on which kernel ran): paths are cut into fixed chunks of kShapChunk; within a chunk
// contributions are added in path order; k_shap_reduce adds the chunk sums in chunk order. No
// floating-point atomics anywhere.
constexpr int kShapChunk = 256;
constexpr int kShapMaxF = 80;  // path-parallel kernel: [kShapChunk][F] doubles of LDS

// Path-parallel kernel (small batches): block = (chunk, row), one path per thread; each thread
// writes its path's contributions to its LDS row, then thread f sums column f in path order.
template <int P>
__global__ __launch_bounds__(kShapChunk) void k_treeshap(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                                        const PathElem* __restrict__ elems,
                                                        const int32_t* __restrict__ path_ptr,
                                                        const double* __restrict__ path_val, int n_paths, int nchunks,
                                                        double* __restrict__ out) {
  extern __shared__ double s_c[];  // [kShapChunk][F]
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.y;
  for (int f = 0; f < F; ++f) s_c[tid * F + f] = 0.0;
  const int p = blockIdx.x * kShapChunk + tid;
  const float* x = X + row * ldx;
  if (p < n_paths) {
    const int e0 = path_ptr[p], k = path_ptr[p + 1] - e0;  // k unique features (bias excluded)
    double z[P], o[P], w[P];
    int feat[P];
    z[0] = 1.0; o[0] = 1.0; w[0] = 1.0; feat[0] = -1;
#pragma unroll
    for (int i = 1; i < P; ++i) { z[i] = 0.0; o[i] = 0.0; w[i] = 0.0; feat[i] = -1; }
    // EXTEND each element
#pragma unroll
    for (int l = 1; l < P; ++l) {
      if (l <= k) {
        const PathElem e = elems[e0 + l - 1];
        const float v = x[e.feat];
        const double one = (v != v) ? (e.nan_ok ? 1.0 : 0.0) : ((v >= e.lo && v < e.hi) ? 1.0 : 0.0);
        z[l] = e.zero; o[l] = one; feat[l] = e.feat;
        w[l] = 0.0;
#pragma unroll
        for (int j = P - 2; j >= 0; --j) {
          if (j <= l - 1) {
            w[j + 1] += one * w[j] * ((double)(j + 1) / (double)(l + 1));
            w[j] = e.zero * w[j] * ((double)(l - j) / (double)(l + 1));
          }
        }
      }
    }
    const double leaf = path_val[p];
    // UNWOUND sum per element
#pragma unroll
    for (int i = 1; i < P; ++i) {
      if (i <= k) {
        const double one = o[i], zero = z[i];
        double total = 0.0;
        if (one != 0.0) {  // (one is 1 here)
          double next = w[k];
#pragma unroll
          for (int j = P - 2; j >= 0; --j) {
            if (j <= k - 1) {
              const double tmp = next * (1.0 / (double)(j + 1));
              total += tmp;
              next = w[j] - tmp * zero * (double)(k - j);
            }
          }
        } else {
          const double iz = 1.0 / zero;
#pragma unroll
          for (int j = P - 2; j >= 0; --j) {
            if (j <= k - 1) total += w[j] * (iz * kShapInv[k - j]);
          }
        }
        total *= (double)(k + 1);
        s_c[tid * F + feat[i]] = total * (one - zero) * leaf;
      }
    }
  }
  __syncthreads();
  const int np = min(kShapChunk, n_paths - (int)blockIdx.x * kShapChunk);
  for (int f = tid; f < F; f += blockDim.x) {
    double acc = 0.0;
    for (int q = 0; q < np; ++q) acc += s_c[q * F + f];
    out[(row * nchunks + blockIdx.x) * F + f] = acc;
  }
}

// ---------------------------------------------------------------- TreeSHAP with pattern tables
// Fast TreeSHAP "v2" (Yang 2021): the EXTEND/UNWOUND result of a path depends on the row only
// through which of the path's k elements the row satisfies (a k-bit pattern), so all 2^k outcomes
// are tabulated once per model (k_shap_table: the same fp64 arithmetic as k_treeshap, pattern bits
// in place of the row's one-fractions). Scoring a (row, path) is then k interval tests plus k
// table reads. Values and accumulation order equal k_treeshap's, so results are bit-identical.
template <int P>
__global__ void k_shap_table(const PathElem* __restrict__ elems, const int32_t* __restrict__ path_ptr,
                             const double* __restrict__ path_val, int n_paths, const int64_t* __restrict__ tab_ptr,
                             double* __restrict__ table) {
  const int p = blockIdx.x;
  if (p >= n_paths) return;
  const int e0 = path_ptr[p], k = path_ptr[p + 1] - e0;
  const double leaf = path_val[p];
  for (int pat = threadIdx.x; pat < (1 << k); pat += blockDim.x) {
    double z[P], o[P], w[P];
    z[0] = 1.0; o[0] = 1.0; w[0] = 1.0;
#pragma unroll
    for (int i = 1; i < P; ++i) { z[i] = 0.0; o[i] = 0.0; w[i] = 0.0; }
#pragma unroll
    for (int l = 1; l < P; ++l) {
      if (l <= k) {
        const PathElem e = elems[e0 + l - 1];
        const double one = ((pat >> (l - 1)) & 1) ? 1.0 : 0.0;
        z[l] = e.zero; o[l] = one;
        w[l] = 0.0;
#pragma unroll
        for (int j = P - 2; j >= 0; --j) {
          if (j <= l - 1) {
            w[j + 1] += one * w[j] * ((double)(j + 1) / (double)(l + 1));
            w[j] = e.zero * w[j] * ((double)(l - j) / (double)(l + 1));
          }
        }
      }
    }
    double* out = table + tab_ptr[p] + (int64_t)pat * k;
#pragma unroll
    for (int i = 1; i < P; ++i) {
      if (i <= k) {
        const double one = o[i], zero = z[i];
        double total = 0.0;
        if (one != 0.0) {  // (one is 1 here)
          double next = w[k];
#pragma unroll
          for (int j = P - 2; j >= 0; --j) {
            if (j <= k - 1) {
              const double tmp = next * (1.0 / (double)(j + 1));
              total += tmp;
              next = w[j] - tmp * zero * (double)(k - j);
            }
          }
        } else {
          const double iz = 1.0 / zero;
#pragma unroll
          for (int j = P - 2; j >= 0; --j) {
            if (j <= k - 1) total += w[j] * (iz * kShapInv[k - j]);
          }
        }
        total *= (double)(k + 1);
        out[i - 1] = total * (one - zero) * leaf;
      }
    }
  }
}

// Row-parallel kernel (batches): block = (kShapRowsB rows, chunk of paths); every thread walks the
// chunk's paths in order for ITS row: k interval tests -> pattern -> k table values added to its
// private LDS column. A path's elements are the same for every lane, so they come by scalar loads
// (SGPRs) -- no LDS staging of the chunk's elements (which held a block to one per CU: 90 KB of LDS
// for 256 rows, one wave per SIMD) -- and the block is 128 rows: 30 KB of LDS, several blocks per CU.
// Two paths per step: the second path's tests and table loads are issued before the first's adds.
constexpr int kShapRowsF = 48;  // row-parallel kernel: [F][kShapRowsB] doubles of per-row accumulators
constexpr int kShapRowsB = 128;
constexpr int kMaxTabK = 10;

__device__ __forceinline__ int shap_pattern(const PathElem* __restrict__ el, int k, const float* x, int* fe) {
  int pat = 0;
#pragma unroll
  for (int l = 0; l < kMaxTabK; ++l) {
    if (l < k) {
      const PathElem e = el[l];
      const float v = x[e.feat];
      const bool one = (v != v) ? (e.nan_ok != 0) : (v >= e.lo && v < e.hi);
      pat |= (int)one << l;
      fe[l] = e.feat;
    }
  }
  return pat;
}

__global__ __launch_bounds__(kShapRowsB) void k_treeshap_rows(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                                              const PathElem* __restrict__ elems,
                                                              const int32_t* __restrict__ path_ptr, int n_paths,
                                                              const int64_t* __restrict__ tab_ptr,
                                                              const double* __restrict__ table, int nchunks,
                                                              double* __restrict__ out) {
  extern __shared__ double s_dyn[];
  constexpr int B = kShapRowsB;
  const int tid = threadIdx.x;
  double* s_phi = s_dyn;                                              // [F][B]
  float* s_x = reinterpret_cast<float*>(s_phi + (size_t)F * B);        // [B][F|1]
  const int xs = F | 1;
  const int c = blockIdx.y;
  const int p0 = c * kShapChunk, p1 = min(n_paths, p0 + kShapChunk);
  const int64_t row0 = (int64_t)blockIdx.x * B;
  const int nrows = (int)min((int64_t)B, n - row0);
  for (int e = tid; e < B * F; e += B) {  // (rows past the batch: zeros, computed and not stored)
    const int r = e / F, f = e - r * F;
    s_x[r * xs + f] = r < nrows ? X[(row0 + r) * ldx + f] : 0.0f;
  }
  for (int f = 0; f < F; ++f) s_phi[f * B + tid] = 0.0;
  __syncthreads();
  const float* x = s_x + tid * xs;
  int p = p0;
  for (; p + 1 < p1; p += 2) {
    const int e0 = path_ptr[p], e1 = path_ptr[p + 1], e2 = path_ptr[p + 2];
    const int ka = e1 - e0, kb = e2 - e1;
    int fa[kMaxTabK], fb[kMaxTabK];
    const int pa = shap_pattern(elems + e0, ka, x, fa);
    const int pb = shap_pattern(elems + e1, kb, x, fb);
    const double* ta = table + tab_ptr[p] + (int64_t)pa * ka;
    const double* tb = table + tab_ptr[p + 1] + (int64_t)pb * kb;
    double va[kMaxTabK], vb[kMaxTabK];
#pragma unroll
    for (int l = 0; l < kMaxTabK; ++l) {
      if (l < ka) va[l] = ta[l];
      if (l < kb) vb[l] = tb[l];
    }
#pragma unroll
    for (int l = 0; l < kMaxTabK; ++l)
      if (l < ka) s_phi[fa[l] * B + tid] += va[l];
#pragma unroll
    for (int l = 0; l < kMaxTabK; ++l)
      if (l < kb) s_phi[fb[l] * B + tid] += vb[l];
  }
  if (p < p1) {
    const int e0 = path_ptr[p], k = path_ptr[p + 1] - e0;
    int fa[kMaxTabK];
    const int pa = shap_pattern(elems + e0, k, x, fa);
    const double* ta = table + tab_ptr[p] + (int64_t)pa * k;
#pragma unroll
    for (int l = 0; l < kMaxTabK; ++l)
      if (l < k) s_phi[fa[l] * B + tid] += ta[l];
  }
  if (tid < nrows) {
    const int64_t row = row0 + tid;
    for (int f = 0; f < F; ++f) out[(row * nchunks + c) * F + f] = s_phi[f * B + tid];
  }
}

__global__ void k_shap_reduce(const double* __restrict__ slab, int64_t n, int F, int nchunks,
                              double* __restrict__ phi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * F) return;
  const int64_t row = i / F;
  const int f = (int)(i - row * F);
  const double* src = slab + row * nchunks * F + f;
  double acc = 0.0;
  for (int c = 0; c < nchunks; ++c) acc += src[(int64_t)c * F];
  phi[i] = acc;
}

// Number of path chunks (and so slab slots per row): fixed by the forest, never by the batch.
COBALT_API int cobalt_treeshap_chunks(int64_t n, int F, int n_paths) {
  (void)n;
  (void)F;
  return n_paths <= 0 ? 1 : (int)ceil_div((int64_t)n_paths, (int64_t)kShapChunk);
}

static int shap_reduce_launch(const double* work, int64_t n, int F, int nchunks, double* phi, hipStream_t stream) {
  const int64_t tot = n * F;
  hipLaunchKernelGGL(k_shap_reduce, dim3((unsigned)ceil_div(tot, (int64_t)256)), dim3(256), 0, stream, work, n, F,
                     nchunks, phi);
  CK_LAUNCH();
  return 0;
}

// Pattern tables exist for paths of <= kMaxTabK unique features (longer: the direct kernel).

COBALT_API int cobalt_shap_table_build(const void* elems, const int32_t* path_ptr, const double* path_val, int n_paths,
                                       int max_len, const int64_t* tab_ptr, double* table, hipStream_t stream) {
  if (n_paths <= 0) return 0;
  if (max_len > kMaxTabK) return -3;
  const PathElem* pe = static_cast<const PathElem*>(elems);
  if (max_len + 1 <= 8)
    hipLaunchKernelGGL(k_shap_table<8>, dim3(n_paths), dim3(128), 0, stream, pe, path_ptr, path_val, n_paths, tab_ptr,
                       table);
  else
    hipLaunchKernelGGL(k_shap_table<kMaxPath>, dim3(n_paths), dim3(256), 0, stream, pe, path_ptr, path_val, n_paths,
                       tab_ptr, table);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_treeshap_tab(const float* X, int64_t n, int F, int64_t ldx, const void* elems,
                                   const int32_t* path_ptr, int n_paths, int max_len, const int64_t* tab_ptr,
                                   const double* table, double* phi, double* work, int nchunks, hipStream_t stream) {
  if (n <= 0 || n_paths <= 0) return 0;
  if (F > kShapRowsF || max_len > kMaxTabK) return -5;
  if (nchunks != cobalt_treeshap_chunks(n, F, n_paths)) return -8;
  if (nchunks > 1 && work == nullptr) return -7;
  const int B = kShapRowsB;
  const size_t lds = (size_t)F * B * sizeof(double) + (size_t)B * (F | 1) * sizeof(float);
  if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)k_treeshap_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_treeshap_rows, dim3((unsigned)ceil_div(n, (int64_t)B), (unsigned)nchunks), dim3(B), lds, stream,
                     X, n, F, ldx, static_cast<const PathElem*>(elems), path_ptr, n_paths, tab_ptr, table, nchunks,
                     nchunks > 1 ? work : phi);
  CK_LAUNCH();
  return nchunks > 1 ? shap_reduce_launch(work, n, F, nchunks, phi, stream) : 0;
}

COBALT_API int cobalt_treeshap(const float* X, int64_t n, int F, int64_t ldx, const void* elems, const int32_t* path_ptr,
                               const double* path_val, int n_paths, int max_len, double* phi, double* work,
                               int nchunks, hipStream_t stream) {
  if (n <= 0 || n_paths <= 0) return 0;
  if (max_len + 1 > kMaxPath) return -3;
  if (n > 65535) return -4;  // grid.y limit; the caller batches rows
  if (F > kShapMaxF) return -5;
  if (nchunks != cobalt_treeshap_chunks(n, F, n_paths)) return -8;
  if (nchunks > 1 && work == nullptr) return -7;
  const size_t lds = (size_t)F * kShapChunk * sizeof(double);
  dim3 grid((unsigned)nchunks, (unsigned)n);
  const PathElem* pe = static_cast<const PathElem*>(elems);
  double* dst = nchunks > 1 ? work : phi;
  if (max_len + 1 <= 8) {
    if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)k_treeshap<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_treeshap<8>, grid, dim3(kShapChunk), lds, stream, X, n, F, ldx, pe, path_ptr, path_val,
                       n_paths, nchunks, dst);
  } else {
    if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)k_treeshap<kMaxPath>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_treeshap<kMaxPath>, grid, dim3(kShapChunk), lds, stream, X, n, F, ldx, pe, path_ptr, path_val,
                       n_paths, nchunks, dst);
  }
  CK_LAUNCH();
  return nchunks > 1 ? shap_reduce_launch(work, n, F, nchunks, phi, stream) : 0;
}
