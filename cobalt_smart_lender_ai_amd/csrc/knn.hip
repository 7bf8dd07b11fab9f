// Exact k-nearest-neighbour search for SMOTE (K29; reference imblearn SMOTE(k_neighbors=5) at
// notebooks/04_model_training.ipynb cell 38).
//
// Squared distances ||r||^2 + ||q||^2 - 2 r.q: the dot products of a 32-reference x 32-query tile
// come from fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products, F/2 instructions per tile),
// the reference tile is staged through LDS once per workgroup and shared by its 4 waves (128
// queries per workgroup). Accumulator layout: lane l owns query column l & 31 and 16 reference
// rows (reg&3) + 8 (reg>>2) + 4 (l>>5); each lane keeps a sorted top-K (distance, index) list in
// registers for its half of the rows and the two halves merge at the end. Ordering is the
// lexicographic (distance, reference index) -- deterministic, independent of the grid.
#include "common.h"

using namespace cobalt;

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kRefTile = 256;  // references staged per LDS pass
constexpr int kMaxFk = 32;

template <int K>
__device__ __forceinline__ void topk_insert(float (&bd)[K], int (&bi)[K], float d, int idx) {
  if (d < bd[K - 1] || (d == bd[K - 1] && idx < bi[K - 1])) {
    bd[K - 1] = d;
    bi[K - 1] = idx;
#pragma unroll
    for (int j = K - 1; j > 0; --j) {
      const bool sw = bd[j] < bd[j - 1] || (bd[j] == bd[j - 1] && bi[j] < bi[j - 1]);
      if (sw) {
        const float td = bd[j]; bd[j] = bd[j - 1]; bd[j - 1] = td;
        const int ti = bi[j]; bi[j] = bi[j - 1]; bi[j - 1] = ti;
      }
    }
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_knn(const float* __restrict__ Q, int64_t nq, const float* __restrict__ R,
                                             int64_t nr, int F, int32_t* __restrict__ out_idx,
                                             float* __restrict__ out_dist) {
  const int Fp = (F + 1) & ~1;       // k pairs
  const int ld = Fp + 1;              // odd LDS row stride: conflict-free A-operand reads
  __shared__ float s_r[kRefTile * (kMaxFk + 1)];
  __shared__ float s_rn[kRefTile];
  __shared__ float s_md[4][32][K];
  __shared__ int s_mi[4][32][K];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 31, half = lane >> 5;
  const int64_t q = (int64_t)blockIdx.x * 128 + wave * 32 + col;
  const bool qok = q < nq;
  // B operand registers: Q[q][k = 2 s + half]
  float qb[kMaxFk / 2];
  float qn = 0.0f;
#pragma unroll
  for (int s = 0; s < kMaxFk / 2; ++s) {
    const int k = 2 * s + half;
    qb[s] = (qok && k < F) ? Q[q * F + k] : 0.0f;
  }
  if (qok)
    for (int k = 0; k < F; ++k) { const float v = Q[q * F + k]; qn = fmaf(v, v, qn); }
  float bd[K];
  int bi[K];
#pragma unroll
  for (int j = 0; j < K; ++j) { bd[j] = INFINITY; bi[j] = 0x7fffffff; }

  for (int64_t t0 = 0; t0 < nr; t0 += kRefTile) {
    const int nt = (int)min((int64_t)kRefTile, nr - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < kRefTile * Fp; i += blockDim.x) {
      const int r = i / Fp, k = i - r * Fp;
      s_r[r * ld + k] = (r < nt && k < F) ? R[(t0 + r) * F + k] : 0.0f;
    }
    __syncthreads();
    for (int r = threadIdx.x; r < kRefTile; r += blockDim.x) {
      float s = 0.0f;
      for (int k = 0; k < F; ++k) { const float v = s_r[r * ld + k]; s = fmaf(v, v, s); }
      s_rn[r] = s;
    }
    __syncthreads();
    for (int sub = 0; sub < nt; sub += 32) {
      f32x16 acc;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
      const float* ra = s_r + (sub + col) * ld + half;
#pragma unroll
      for (int s = 0; s < kMaxFk / 2; ++s) {
        if (2 * s < Fp) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[2 * s], qb[s], acc, 0, 0, 0);
      }
      if (qok) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int m = (j & 3) + 8 * (j >> 2) + 4 * half;
          if (sub + m < nt) {
            const float d = s_rn[sub + m] + qn - 2.0f * acc[j];
            topk_insert<K>(bd, bi, d, (int)(t0 + sub + m));
          }
        }
      }
    }
  }
  // merge the two halves of each query column
  if (half == 1) {
#pragma unroll
    for (int j = 0; j < K; ++j) { s_md[wave][col][j] = bd[j]; s_mi[wave][col][j] = bi[j]; }
  }
  __syncthreads();
  if (half == 0 && qok) {
#pragma unroll
    for (int j = 0; j < K; ++j) topk_insert<K>(bd, bi, s_md[wave][col][j], s_mi[wave][col][j]);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      out_idx[q * K + j] = bi[j];
      if (out_dist) out_dist[q * K + j] = fmaxf(bd[j], 0.0f);
    }
  }
}

// SMOTE interpolation in fp64 (imblearn works in the frame's float64):
// new[i] = X[rows[i]] + steps[i] * (X[nn[rows[i]][cols[i]]] - X[rows[i]]).
__global__ void k_smote_interp(const double* __restrict__ X, int F, const int32_t* __restrict__ nn, int knn,
                               const int64_t* __restrict__ rows, const int64_t* __restrict__ cols,
                               const double* __restrict__ steps, int64_t n_new, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_new * F) return;
  const int64_t s = i / F;
  const int k = (int)(i - s * F);
  const int64_t r = rows[s];
  const int64_t o = nn[r * knn + cols[s]];
  const double a = X[r * F + k], b = X[o * F + k];
  out[i] = a + steps[s] * (b - a);
}
}  // namespace

COBALT_API int cobalt_knn(const float* Q, int64_t nq, const float* R, int64_t nr, int F, int k, int32_t* out_idx,
                          float* out_dist, hipStream_t stream) {
  if (F < 1 || F > kMaxFk) return -1;
  if (nq <= 0) return 0;
  if (nr <= 0) return -2;
  const dim3 grid((unsigned)ceil_div(nq, (int64_t)128));
  switch (k) {
#define KNN_CASE(KK) \
  case KK: hipLaunchKernelGGL(k_knn<KK>, grid, dim3(256), 0, stream, Q, nq, R, nr, F, out_idx, out_dist); break;
    KNN_CASE(1) KNN_CASE(2) KNN_CASE(3) KNN_CASE(4) KNN_CASE(5) KNN_CASE(6) KNN_CASE(7) KNN_CASE(8)
    KNN_CASE(11) KNN_CASE(16)
#undef KNN_CASE
    default: return -3;
  }
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_smote_interp(const double* X, int F, const int32_t* nn, int knn, const int64_t* rows,
                                   const int64_t* cols, const double* steps, int64_t n_new, double* out,
                                   hipStream_t stream) {
  if (n_new <= 0) return 0;
  const int64_t tot = n_new * F;
  hipLaunchKernelGGL(k_smote_interp, dim3((unsigned)ceil_div(tot, (int64_t)256)), dim3(256), 0, stream, X, F, nn, knn,
                     rows, cols, steps, n_new, out);
  CK_LAUNCH();
  return 0;
}
