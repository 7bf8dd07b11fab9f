// Fused MLP challenger (K31): the notebook's Dense 128-32-16-1 ReLU/sigmoid network
// (notebooks/04_model_training.ipynb cell 39 `build_and_train_nn`).
//
// Training (k_mlp_train): sequential mini-batch SGD is a chain of tiny dependent steps (batch 32,
// 7,361 parameters), so instead of ~20 library launches per step the WHOLE epoch runs inside one
// workgroup: weights, AdamW moments and the batch activations live in LDS (~140 KB at F = 20) and
// every step is forward -> backward -> AdamW with workgroup barriers only. One workgroup trains one
// model; a launch with G workgroups trains G independent models (seeds / hyper-parameters) on G
// CUs at the cost of one.
//
// Semantics follow the Keras model the reference builds:
//   * loss = mean BCE computed from the logit (Keras uses the sigmoid's logit when present),
//     gradient (p - y) / batch_rows; last partial batch = its own mean;
//   * L2 kernel regulariser lambda * sum(W^2) on the three hidden Dense layers (not the output
//     layer, not biases) -> + 2 * lambda * W;
//   * AdamW (Keras 3): p -= lr * wd * p, then m += (g - m)(1 - b1), v += (g^2 - v)(1 - b2),
//     p -= lr * sqrt(1 - b2^t) / (1 - b1^t) * m / (sqrt(v) + eps), t = step + 1;
//   * ExponentialDecay(staircase): lr = lr0 * rate^floor(step / decay_steps).
// Parameter layout per model (floats): W1[F][128] b1[128] W2[128][32] b2[32] W3[32][16] b3[16]
// W4[16] b4[1]  (P = 128 F + 4801).
//
// Inference (k_mlp_forward): 32-row tiles per workgroup iteration with the same LDS-resident
// forward code; writes sigmoid probabilities (and optionally logits).
//
// MFMA versions (default from Python): k_mlp_forward_mfma (bulk inference, 7.8G rows/s) and
// k_mlp_train_mfma (the same epoch on 4 waves, every contraction on v_mfma_f32_32x32x2_f32,
// 9.4 us per batch-32 step vs 29.6 us here) -- see their comments below.
#include "common.h"

namespace {
constexpr int H1 = 128, H2 = 32, H3 = 16, MB = 32, NT = 1024;  // 16 waves: 4 per SIMD hide LDS latency
constexpr int kMaxF = 32;

struct MlpHyper {
  float lr0, decay_rate;
  int32_t decay_steps, staircase;
  float weight_decay, beta1, beta2, eps;
  float l2;
  int32_t batch;
  int32_t pad[2];
};
static_assert(sizeof(MlpHyper) == 48, "MlpHyper layout mirrored in nn/mlp.py");
static_assert(NT == 1024, "forward_tile thread maps assume 1024 threads");
static_assert(MB * kMaxF <= NT, "one batch element per thread");

__host__ __device__ constexpr int mlp_params(int F) { return F * H1 + H1 + H1 * H2 + H2 + H2 * H3 + H3 + H3 + 1; }
__host__ __device__ constexpr int act_floats(int F) {
  (void)F;
  return MB * kMaxF + MB + 2 * MB * H1 + 2 * MB * H2 + 2 * MB * H3 + MB + 64;
}

struct Views {
  float *W1, *b1, *W2, *b2, *W3, *b3, *W4, *b4;
};
__device__ __forceinline__ Views views(float* base, int F) {
  Views v;
  v.W1 = base;
  v.b1 = v.W1 + F * H1;
  v.W2 = v.b1 + H1;
  v.b2 = v.W2 + H1 * H2;
  v.W3 = v.b2 + H2;
  v.b3 = v.W3 + H2 * H3;
  v.W4 = v.b3 + H3;
  v.b4 = v.W4 + H3;
  return v;
}

struct Acts {
  float *xb, *yb, *h1, *d1, *h2, *d2, *h3, *d3, *d4, *red;
};
__device__ __forceinline__ Acts acts(float* base) {
  Acts a;
  a.xb = base;
  a.yb = a.xb + MB * kMaxF;
  a.h1 = a.yb + MB;
  a.d1 = a.h1 + MB * H1;
  a.h2 = a.d1 + MB * H1;
  a.d2 = a.h2 + MB * H2;
  a.h3 = a.d2 + MB * H2;
  a.d3 = a.h3 + MB * H3;
  a.d4 = a.d3 + MB * H3;
  a.red = a.d4 + MB;
  return a;
}

// Forward of one 32-row tile held in a.xb (rows >= bs are zero). Leaves ReLU outputs in h1/h2/h3
// and the logits in d4 (overwritten by the backward pass in training).
__device__ __forceinline__ void forward_tile(const Views& w, const Acts& a, int F) {
  const int t = threadIdx.x;
  {  // layer 1: thread -> hidden j, 4 rows
    const int j = t & (H1 - 1), r0 = (t >> 7) * 4;
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = w.b1[j];
    for (int k = 0; k < F; ++k) {
      const float wk = w.W1[k * H1 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(a.xb[(r0 + i) * kMaxF + k], wk, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) a.h1[(r0 + i) * H1 + j] = fmaxf(acc[i], 0.0f);
  }
  __syncthreads();
  {  // layer 2: thread -> (row, j)
    const int j = t & (H2 - 1), r = t >> 5;
    float acc = w.b2[j];
    for (int k = 0; k < H1; ++k) acc = fmaf(a.h1[r * H1 + k], w.W2[k * H2 + j], acc);
    a.h2[r * H2 + j] = fmaxf(acc, 0.0f);
  }
  __syncthreads();
  if (t < MB * H3) {  // layer 3: thread -> (row, j)
    const int j = t & (H3 - 1), r = t >> 4;
    float acc = w.b3[j];
    for (int k = 0; k < H2; ++k) acc = fmaf(a.h2[r * H2 + k], w.W3[k * H3 + j], acc);
    a.h3[r * H3 + j] = fmaxf(acc, 0.0f);
  }
  __syncthreads();
  if (t < MB) {  // output logit
    float z = w.b4[0];
    for (int k = 0; k < H3; ++k) z = fmaf(a.h3[t * H3 + k], w.W4[k], z);
    a.d4[t] = z;
  }
  __syncthreads();
}

struct AdamStep {
  float lr, lr_t, wd, b1, b2, eps, l2;
};

__device__ __forceinline__ void adam(float* p, float* m, float* v, float g, bool reg, const AdamStep& s) {
  float w = *p;
  if (reg) g = fmaf(2.0f * s.l2, w, g);
  w -= s.lr * s.wd * w;
  float mm = *m, vv = *v;
  mm += (g - mm) * (1.0f - s.b1);
  vv += (g * g - vv) * (1.0f - s.b2);
  w -= s.lr_t * mm / (sqrtf(vv) + s.eps);
  *p = w;
  *m = mm;
  *v = vv;
}

__global__ __launch_bounds__(NT) void k_mlp_train(const float* __restrict__ X, int64_t ldx, const float* __restrict__ y,
                                                  int64_t n, int F, const int32_t* __restrict__ perm,
                                                  float* __restrict__ params, float* __restrict__ mom1,
                                                  float* __restrict__ mom2, int64_t* __restrict__ steps,
                                                  MlpHyper hp, float* __restrict__ loss_out,
                                                  uint64_t* __restrict__ prof) {
  extern __shared__ float sm[];
  const int P = mlp_params(F);
  const int model = blockIdx.x;
  // optional phase timer (thread 0 of model 0, s_memrealtime ticks): prof[0..6]
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t ph_last = 0;
  const bool timing = prof != nullptr && model == 0 && threadIdx.x == 0;
#define MLP_PHASE(i)                      \
  if (timing) {                           \
    const uint64_t now = wall_clock64();  \
    ph[i] += now - ph_last;               \
    ph_last = now;                        \
  }
  const int t = threadIdx.x;
  float* Wb = sm;
  float* Mb = Wb + P;
  float* Vb = Mb + P;
  const Acts a = acts(Vb + P);
  const Views w = views(Wb, F), m = views(Mb, F), v = views(Vb, F);
  float* gp = params + (int64_t)model * P;
  float* gm = mom1 + (int64_t)model * P;
  float* gv = mom2 + (int64_t)model * P;
  for (int i = t; i < P; i += NT) {
    Wb[i] = gp[i];
    Mb[i] = gm[i];
    Vb[i] = gv[i];
  }
  for (int i = t; i < MB * kMaxF; i += NT) a.xb[i] = 0.0f;
  int64_t step = steps[model];
  const int32_t* pm = perm + (int64_t)model * n;
  const int B = hp.batch;
  const int64_t nb = (n + B - 1) / B;
  float loss_acc = 0.0f;  // thread 0 only
  __syncthreads();
  // Batch b + 1 is fetched into registers while step b computes (MB * F <= NT: one element per
  // thread), hiding the dependent perm -> X global-load latency behind the step.
  const int xr = t / F, xk = t - (t / F) * F;
  auto fetch = [&](int64_t bb, float& xv, float& yv) {
    const int bsz = (int)min((int64_t)B, n - bb * B);
    xv = (t < MB * F && xr < bsz) ? X[(int64_t)pm[bb * B + xr] * ldx + xk] : 0.0f;
    yv = (t < bsz) ? y[pm[bb * B + t]] : 0.0f;
  };
  float nx = 0.0f, ny = 0.0f;
  if (nb > 0) fetch(0, nx, ny);
  for (int64_t b = 0; b < nb; ++b) {
    const int bs = (int)min((int64_t)B, n - b * B);
    if (t < MB * F) a.xb[xr * kMaxF + xk] = nx;
    if (t < MB) a.yb[t] = ny;
    if (timing) ph_last = wall_clock64();
    __syncthreads();
    MLP_PHASE(0)
    if (b + 1 < nb) fetch(b + 1, nx, ny);
    forward_tile(w, a, F);
    MLP_PHASE(1)
    // schedule + bias correction for this step
    AdamStep s;
    {
      const float e = hp.staircase ? floorf((float)step / (float)hp.decay_steps) : (float)step / (float)hp.decay_steps;
      s.lr = hp.lr0 * powf(hp.decay_rate, e);
      const float tt = (float)(step + 1);
      s.lr_t = s.lr * sqrtf(1.0f - powf(hp.beta2, tt)) / (1.0f - powf(hp.beta1, tt));
      s.wd = hp.weight_decay;
      s.b1 = hp.beta1;
      s.b2 = hp.beta2;
      s.eps = hp.eps;
      s.l2 = hp.l2;
    }
    if (t < MB) {  // BCE from the logit; gradient (p - y) / bs
      const float z = a.d4[t];
      const float yy = a.yb[t];
      const float p = 1.0f / (1.0f + expf(-z));
      const float l = fmaxf(z, 0.0f) - z * yy + log1pf(expf(-fabsf(z)));
      a.red[t] = t < bs ? l : 0.0f;
      a.d4[t] = t < bs ? (p - yy) / (float)bs : 0.0f;
    }
    __syncthreads();
    if (t == 0) {
      float sl = 0.0f;
      for (int r = 0; r < bs; ++r) sl += a.red[r];
      loss_acc += sl / (float)bs;
    }
    MLP_PHASE(2)
    // phase A: delta3 = d4 * W4 * relu'(h3)
    for (int e = t; e < MB * H3; e += NT) {
      const int r = e / H3, k = e - r * H3;
      a.d3[e] = a.h3[e] > 0.0f ? a.d4[r] * w.W4[k] : 0.0f;
    }
    __syncthreads();
    MLP_PHASE(3)
    // phase B: update W4/b4; delta2 = (d3 W3^T) * relu'(h2)
    if (t < H3) {
      float g = 0.0f;
      for (int r = 0; r < MB; ++r) g = fmaf(a.h3[r * H3 + t], a.d4[r], g);
      adam(&w.W4[t], &m.W4[t], &v.W4[t], g, false, s);
    } else if (t == H3) {
      float g = 0.0f;
      for (int r = 0; r < MB; ++r) g += a.d4[r];
      adam(&w.b4[0], &m.b4[0], &v.b4[0], g, false, s);
    }
    for (int e = t; e < MB * H2; e += NT) {
      const int r = e / H2, k = e - r * H2;
      float acc = 0.0f;
      if (a.h2[e] > 0.0f)  // rotated j: lanes (consecutive k) hit different banks of the W3 rows
        for (int jj = 0; jj < H3; ++jj) {
          const int j = (jj + k) & (H3 - 1);
          acc = fmaf(a.d3[r * H3 + j], w.W3[k * H3 + j], acc);
        }
      a.d2[e] = acc;
    }
    __syncthreads();
    MLP_PHASE(4)
    // phase C: update W3/b3; delta1 = (d2 W2^T) * relu'(h1)
    for (int e = t; e < H2 * H3 + H3; e += NT) {
      if (e < H2 * H3) {
        const int k = e / H3, j = e - k * H3;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g = fmaf(a.h2[r * H2 + k], a.d3[r * H3 + j], g);
        adam(&w.W3[e], &m.W3[e], &v.W3[e], g, true, s);
      } else {
        const int j = e - H2 * H3;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g += a.d3[r * H3 + j];
        adam(&w.b3[j], &m.b3[j], &v.b3[j], g, false, s);
      }
    }
    for (int e = t; e < MB * H1; e += NT) {
      const int r = e / H1, k = e - r * H1;
      float acc = 0.0f;
      if (a.h1[e] > 0.0f)  // rotated j (see above): W2 rows are 32 floats apart
        for (int jj = 0; jj < H2; ++jj) {
          const int j = (jj + k) & (H2 - 1);
          acc = fmaf(a.d2[r * H2 + j], w.W2[k * H2 + j], acc);
        }
      a.d1[e] = acc;
    }
    __syncthreads();
    MLP_PHASE(5)
    // phase D: update W2/b2 and W1/b1
    for (int e = t; e < H1 * H2 + H2; e += NT) {
      if (e < H1 * H2) {
        const int k = e / H2, j = e - k * H2;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g = fmaf(a.h1[r * H1 + k], a.d2[r * H2 + j], g);
        adam(&w.W2[e], &m.W2[e], &v.W2[e], g, true, s);
      } else {
        const int j = e - H1 * H2;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g += a.d2[r * H2 + j];
        adam(&w.b2[j], &m.b2[j], &v.b2[j], g, false, s);
      }
    }
    for (int e = t; e < F * H1 + H1; e += NT) {
      if (e < F * H1) {
        const int k = e / H1, j = e - k * H1;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g = fmaf(a.xb[r * kMaxF + k], a.d1[r * H1 + j], g);
        adam(&w.W1[e], &m.W1[e], &v.W1[e], g, true, s);
      } else {
        const int j = e - F * H1;
        float g = 0.0f;
        for (int r = 0; r < MB; ++r) g += a.d1[r * H1 + j];
        adam(&w.b1[j], &m.b1[j], &v.b1[j], g, false, s);
      }
    }
    ++step;
    __syncthreads();
    MLP_PHASE(6)
  }
#undef MLP_PHASE
  if (timing)
    for (int i = 0; i < 7; ++i) prof[i] += ph[i];
  for (int i = t; i < P; i += NT) {
    gp[i] = Wb[i];
    gm[i] = Mb[i];
    gv[i] = Vb[i];
  }
  if (t == 0) {
    steps[model] = step;
    loss_out[model] = loss_acc;
  }
}

__global__ __launch_bounds__(NT) void k_mlp_forward(const float* __restrict__ X, int64_t ldx, int64_t n, int F,
                                                    const float* __restrict__ params, float* __restrict__ prob,
                                                    float* __restrict__ logit) {
  extern __shared__ float sm[];
  const int P = mlp_params(F);
  const int t = threadIdx.x;
  float* Wb = sm;
  const Acts a = acts(Wb + P);
  const Views w = views(Wb, F);
  for (int i = t; i < P; i += NT) Wb[i] = params[i];
  for (int i = t; i < MB * kMaxF; i += NT) a.xb[i] = 0.0f;
  __syncthreads();
  const int64_t tiles = (n + MB - 1) / MB;
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t r0 = tile * MB;
    const int bs = (int)min((int64_t)MB, n - r0);
    for (int i = t; i < MB * F; i += NT) {
      const int r = i / F, k = i - r * F;
      a.xb[r * kMaxF + k] = r < bs ? X[(r0 + r) * ldx + k] : 0.0f;
    }
    __syncthreads();
    forward_tile(w, a, F);
    if (t < bs) {
      const float z = a.d4[t];
      prob[r0 + t] = 1.0f / (1.0f + expf(-z));
      if (logit) logit[r0 + t] = z;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- MFMA bulk inference
// k_mlp_forward_mfma: every wave owns 32-row tiles and runs the whole network on fp32 MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation) with activations never leaving
// registers. Each layer is computed transposed, hT = W^T . xT, so the batch rows are the MFMA's N
// dimension: the accumulator of layer L (lane l holds column n = l & 31, output rows
// (v & 3) + 8 (v >> 2) + 4 (l >> 5), v < 16) is directly the B operand of layer L + 1 when the K
// steps of layer L + 1 walk the hidden units in that same order, m(s, hi) = 32 (s >> 4) +
// 8 ((s & 15) >> 2) + 4 hi + (s & 3). The matching A operands (weights, permuted once per workgroup)
// sit in LDS as [s / 4][lane][s % 4], one conflict-free ds_read_b128 per 4 MFMAs. Layer 1 splits
// the features between the two lane halves (k = hi * S1 + s, S1 = ceil(F / 2)), so each lane reads
// a contiguous run of its row. Layer 3 (16 outputs) pads M to 32 with zero weights; the 16 -> 1
// output is a VALU dot plus one cross-half exchange. MFMAs per 32 rows: 4 S1 + 64 + 16 (120 at
// F = 20) at 64 cycles each per SIMD.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kFwdThreads = 256;  // 4 waves, one 32-row tile each per iteration
constexpr int kS1Max = kMaxF / 2;

__host__ __device__ constexpr int fwd_lds_floats(int S1) {
  return S1 * 256 + 16 * 256 + 4 * 256 + H1 + H2 + 32 + 32 + 4;
}

__device__ __forceinline__ int hid_of(int s, int hi) {  // hidden index of K step s, lane half hi
  return 32 * (s >> 4) + 8 * ((s & 15) >> 2) + 4 * hi + (s & 3);
}

__global__ __launch_bounds__(kFwdThreads) void k_mlp_forward_mfma(const float* __restrict__ X, int64_t ldx, int64_t n,
                                                                  int F, const float* __restrict__ params,
                                                                  float* __restrict__ prob, float* __restrict__ logit) {
  extern __shared__ float4 smv[];
  float* sm = reinterpret_cast<float*>(smv);
  const int S1 = (F + 1) >> 1;
  float* A1 = sm;
  float* A2 = A1 + S1 * 256;
  float* A3 = A2 + 16 * 256;
  float* b1 = A3 + 4 * 256;
  float* b2 = b1 + H1;
  float* b3 = b2 + H2;  // padded to 32 (zeros)
  float* w4 = b3 + 32;  // padded to 32 (zeros)
  float* b4 = w4 + 32;
  {
    float* base = const_cast<float*>(params);
    const Views w = views(base, F);
    for (int e = threadIdx.x; e < S1 * 256; e += kFwdThreads) {
      const int s = e >> 8, l = (e >> 2) & 63, t = e & 3;
      const int k = (l >> 5) * S1 + s;
      A1[e] = k < F ? w.W1[k * H1 + 32 * t + (l & 31)] : 0.0f;
    }
    for (int e = threadIdx.x; e < 16 * 256; e += kFwdThreads) {
      const int l = (e >> 2) & 63, s = ((e >> 8) << 2) | (e & 3);
      A2[e] = w.W2[hid_of(s, l >> 5) * H2 + (l & 31)];
    }
    for (int e = threadIdx.x; e < 4 * 256; e += kFwdThreads) {
      const int l = (e >> 2) & 63, s = ((e >> 8) << 2) | (e & 3);
      A3[e] = (l & 31) < H3 ? w.W3[hid_of(s, l >> 5) * H3 + (l & 31)] : 0.0f;
    }
    for (int e = threadIdx.x; e < H1; e += kFwdThreads) b1[e] = w.b1[e];
    if (threadIdx.x < 32) {
      b2[threadIdx.x] = w.b2[threadIdx.x];
      b3[threadIdx.x] = threadIdx.x < H3 ? w.b3[threadIdx.x] : 0.0f;
      w4[threadIdx.x] = threadIdx.x < H3 ? w.W4[threadIdx.x] : 0.0f;
    }
    if (threadIdx.x == 0) b4[0] = w.b4[0];
  }
  __syncthreads();
  const float4* A1v = reinterpret_cast<const float4*>(A1);
  const float4* A2v = reinterpret_cast<const float4*>(A2);
  const float4* A3v = reinterpret_cast<const float4*>(A3);
  const int lane = threadIdx.x & 63, hi = lane >> 5;
  const int kbase = hi * S1;
  const int nk = max(0, min(S1, F - kbase));  // features this lane half contributes
  const float bias4 = b4[0];
  const int64_t tiles = (n + 31) >> 5;
  const int64_t stride = (int64_t)gridDim.x * (kFwdThreads / 64);
  for (int64_t tile = (int64_t)blockIdx.x * (kFwdThreads / 64) + (threadIdx.x >> 6); tile < tiles; tile += stride) {
    const int64_t row = (tile << 5) + (lane & 31);
    const bool ok = row < n;
    float xv[kS1Max];
#pragma unroll
    for (int s = 0; s < kS1Max; ++s) xv[s] = (ok && s < nk) ? X[row * ldx + kbase + s] : 0.0f;
    // layer 1: h1T[128 x 32] = W1T . xT  (+ b1 as the accumulator's initial value)
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(b1 + 32 * t + 8 * q + 4 * hi);
        acc[t][4 * q + 0] = b.x;
        acc[t][4 * q + 1] = b.y;
        acc[t][4 * q + 2] = b.z;
        acc[t][4 * q + 3] = b.w;
      }
#pragma unroll
    for (int s = 0; s < kS1Max; ++s) {
      if (s < S1) {
        const float4 a = A1v[s * 64 + lane];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, xv[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, xv[s], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, xv[s], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, xv[s], acc[3], 0, 0, 0);
      }
    }
    // layer 2: h2T[32 x 32] = W2T . relu(h1T), K walked in accumulator order
    f32x16 acc2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(b2 + 8 * q + 4 * hi);
      acc2[4 * q + 0] = b.x;
      acc2[4 * q + 1] = b.y;
      acc2[4 * q + 2] = b.z;
      acc2[4 * q + 3] = b.w;
    }
#pragma unroll
    for (int sg = 0; sg < 16; ++sg) {
      const float4 a = A2v[sg * 64 + lane];
      const int t = sg >> 2, v = (sg & 3) * 4;
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, fmaxf(acc[t][v + 0], 0.0f), acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, fmaxf(acc[t][v + 1], 0.0f), acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, fmaxf(acc[t][v + 2], 0.0f), acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, fmaxf(acc[t][v + 3], 0.0f), acc2, 0, 0, 0);
    }
    // layer 3: h3T[16 (padded 32) x 32] = W3T . relu(h2T)
    f32x16 acc3;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(b3 + 8 * q + 4 * hi);
      acc3[4 * q + 0] = b.x;
      acc3[4 * q + 1] = b.y;
      acc3[4 * q + 2] = b.z;
      acc3[4 * q + 3] = b.w;
    }
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      const float4 a = A3v[sg * 64 + lane];
      acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, fmaxf(acc2[4 * sg + 0], 0.0f), acc3, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, fmaxf(acc2[4 * sg + 1], 0.0f), acc3, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, fmaxf(acc2[4 * sg + 2], 0.0f), acc3, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, fmaxf(acc2[4 * sg + 3], 0.0f), acc3, 0, 0, 0);
    }
    // output: rows 0..15 of acc3 are v < 8; each half holds 8 of the 16 units
    float z = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; ++v) z = fmaf(w4[(v & 3) + 8 * (v >> 2) + 4 * hi], fmaxf(acc3[v], 0.0f), z);
    z += __shfl_xor(z, 32);
    z += bias4;
    if (hi == 0 && ok) {
      prob[row] = 1.0f / (1.0f + expf(-z));
      if (logit) logit[row] = z;
    }
  }
}
// ------------------------------------------------------------------------------ MFMA training
// k_mlp_train_mfma: the same epoch semantics as k_mlp_train (bit-for-bit the same algorithm, sums in
// a different order) with every contraction on fp32 MFMA. One workgroup = 4 waves = one model;
// wave w owns hidden tile w (units 32w..32w+31) of layer 1 and the matching K slice of layer 2.
//   * Forward and deltas are computed transposed (batch rows = MFMA N, lane n & 31), each layer's
//     accumulator feeding the next MFMA directly as its B operand (K walked in accumulator-register
//     order, rowD(s, hi)), as in k_mlp_forward_mfma.
//   * Weight gradients contract over the batch rows (K = 32 rows), reading activations and deltas
//     that the forward / backward phases stored row-major in LDS; their accumulators come out in the
//     layout of the weights' registers: W1 (with b1 folded in as row F, the input carrying a
//     constant-1 column) and W2 -- values and AdamW moments -- live in registers for the whole
//     epoch as exactly the A operands their forward MFMAs consume. W2 is mirrored in LDS for the
//     transposed read of the layer-1 delta; W3 / b2 / b3 / W4 / b4 and their moments live in LDS.
//   * 3 workgroup barriers per step: layer-2 partial sums, activations/deltas stored, parameters
//     updated (the next batch is staged into the other x buffer in between).
constexpr int kTrThreads = 256;
constexpr int kTrMaxF = 31;  // column F of the input is the constant 1 of the folded bias
constexpr int XP = 33, H1P = 129, W2P = 33, W3P = 17, H2P = 33, H3P = 17;

struct TrLayout {
  int MV1, MV2, W2s, W3s, sm, sched, xb, ys, h1s, d1s, h2s, d2s, h3s, d3s, d4s, red, total;
};
__host__ __device__ constexpr TrLayout tr_layout() {
  TrLayout L{};
  int o = 0;
  L.MV1 = o;  o += 2 * 32 * H1;  // AdamW (m, v) of W1 rows 0..F-1, b1 at row F, zero rows above
  L.MV2 = o;  o += 2 * H1 * H2;  // AdamW (m, v) of W2
  L.W2s = o;  o += H1 * W2P;
  L.W3s = o;  o += H2 * W3P;
  L.sm = o;   o += 3 * 96;       // small params b2[32] b3[32] W4[32] (padded) + b4: value / m / v
  L.sched = o;  o += 2 * kTrThreads;  // (lr, lr_t) of the next 256 steps
  L.xb = o;   o += 2 * MB * XP;  // double-buffered batch, column F = 1, columns > F = 0
  L.ys = o;   o += 2 * MB;
  L.h1s = o;  o += MB * H1P;
  L.d1s = o;  o += MB * H1P;
  L.h2s = o;  o += MB * H2P;
  L.d2s = o;  o += MB * H2P;
  L.h3s = o;  o += MB * H3P;
  L.d3s = o;  o += MB * H3P;
  L.d4s = o;  o += MB;
  o = (o + 3) & ~3;
  L.red = o;  o += 4 * 16 * 64;
  L.total = o;
  return L;
}
// small-parameter slots inside L.sm (value at +0, first moment at +96, second at +192)
constexpr int kSmB2 = 0, kSmB3 = 32, kSmW4 = 64, kSmB4 = 95;

__device__ __forceinline__ int rowD(int v, int hi) { return (v & 3) + 8 * (v >> 2) + 4 * hi; }

// AdamW step with the hardware square root / reciprocal (1 ulp each; no IEEE division sequence):
// the update differs from k_mlp_train's by rounding only.
__device__ __forceinline__ void adam_f(float& w, float& mm, float& vv, float g, float regk, const AdamStep& s) {
  g = fmaf(regk, w, g);  // regk = 2 * lambda on regularised kernels, 0 elsewhere
  w -= s.lr * s.wd * w;
  mm += (g - mm) * (1.0f - s.b1);
  vv += (g * g - vv) * (1.0f - s.b2);
  w -= s.lr_t * mm * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv) + s.eps);
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// NQ = F / 8 + 1: layer 1 runs 4 NQ K steps (rows 0..F, the bias row F included), a compile-time
// count so the accumulator chain has no data-dependent control flow.
template <int NQ>
__global__ __launch_bounds__(kTrThreads) void k_mlp_train_mfma(const float* __restrict__ X, int64_t ldx,
                                                               const float* __restrict__ y, int64_t n, int F,
                                                               const int32_t* __restrict__ perm,
                                                               float* __restrict__ params, float* __restrict__ mom1,
                                                               float* __restrict__ mom2, int64_t* __restrict__ steps,
                                                               MlpHyper hp, float* __restrict__ loss_out,
                                                               uint64_t* __restrict__ prof) {
  extern __shared__ float4 smv[];
  float* sm = reinterpret_cast<float*>(smv);
  constexpr TrLayout L = tr_layout();
  // optional phase timer (lane 0 of waves 0 and 3 of model 0, s_memrealtime): prof[8 * (w == 3) + i]
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t ph_last = 0;
  const bool timing = prof != nullptr && blockIdx.x == 0 && (threadIdx.x == 0 || threadIdx.x == 192);
#define TR_PHASE(i)                       \
  if (timing) {                           \
    const uint64_t now = wall_clock64();  \
    ph[i] += now - ph_last;               \
    ph_last = now;                        \
  }
  float2* MV1 = reinterpret_cast<float2*>(sm + L.MV1);
  float2* MV2 = reinterpret_cast<float2*>(sm + L.MV2);
  float* W2s = sm + L.W2s;
  float* W3s = sm + L.W3s;
  float* SP = sm + L.sm;
  float2* sched = reinterpret_cast<float2*>(sm + L.sched);
  float* xbuf = sm + L.xb;
  float* ybuf = sm + L.ys;
  float* h1s = sm + L.h1s;
  float* d1s = sm + L.d1s;
  float* h2s = sm + L.h2s;
  float* d2s = sm + L.d2s;
  float* h3s = sm + L.h3s;
  float* d3s = sm + L.d3s;
  float* d4s = sm + L.d4s;
  float* red = sm + L.red;

  const int model = blockIdx.x;
  const int P = mlp_params(F);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hi = lane >> 5, li = lane & 31;
  const Views gp = views(params + (int64_t)model * P, F);
  const Views gm = views(mom1 + (int64_t)model * P, F);
  const Views gv = views(mom2 + (int64_t)model * P, F);

  // ---- prologue: W1 (+ b1 as row F) and W2 tile w into registers, the rest into LDS
  float w1r[16], w2r[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int f = rowD(v, hi), c = 32 * w + li;
    w1r[v] = f < F ? gp.W1[f * H1 + c] : (f == F ? gp.b1[c] : 0.0f);
    MV1[f * H1 + c] = f < F ? make_float2(gm.W1[f * H1 + c], gv.W1[f * H1 + c])
                            : (f == F ? make_float2(gm.b1[c], gv.b1[c]) : make_float2(0.0f, 0.0f));
    const int k = 32 * w + rowD(v, hi);
    w2r[v] = gp.W2[k * H2 + li];
    MV2[k * H2 + li] = make_float2(gm.W2[k * H2 + li], gv.W2[k * H2 + li]);
  }
  for (int e = t; e < H1 * H2; e += kTrThreads) W2s[(e / H2) * W2P + (e % H2)] = gp.W2[e];
  for (int e = t; e < H2 * H3; e += kTrThreads) W3s[(e / H3) * W3P + (e % H3)] = gp.W3[e];
  // W3's AdamW state: waves 1 and 3 own rows rowD(v, hi), v in [0, 8) / [8, 16), of columns li < 16
  float w3r[8], m3r[8], v3r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = rowD(q + (w == 3 ? 8 : 0), hi) * H3 + li;
    const bool own = (w & 1) && li < H3;
    w3r[q] = own ? gp.W3[e] : 0.0f;
    m3r[q] = own ? gm.W3[e] : 0.0f;
    v3r[q] = own ? gv.W3[e] : 0.0f;
  }
  if (t < 96) {
    float pv = 0.0f, pm = 0.0f, pw = 0.0f;
    if (t < 32) {
      pw = gp.b2[t]; pm = gm.b2[t]; pv = gv.b2[t];
    } else if (t < 32 + H3) {
      pw = gp.b3[t - 32]; pm = gm.b3[t - 32]; pv = gv.b3[t - 32];
    } else if (t >= 64 && t < 64 + H3) {
      pw = gp.W4[t - 64]; pm = gm.W4[t - 64]; pv = gv.W4[t - 64];
    } else if (t == kSmB4) {
      pw = gp.b4[0]; pm = gm.b4[0]; pv = gv.b4[0];
    }
    SP[t] = pw;
    SP[96 + t] = pm;
    SP[192 + t] = pv;
  }
  for (int e = t; e < 2 * MB * XP; e += kTrThreads) xbuf[e] = ((e % XP) == F) ? 1.0f : 0.0f;

  int64_t step = steps[model];
  const int32_t* pm = perm + (int64_t)model * n;
  const int B = hp.batch;
  const int64_t nb = (n + B - 1) / B;
  float loss_acc = 0.0f;  // lane 0 of wave 0
  // batch prefetch, two-stage: the row ids of batch b + 2 are loaded while batch b computes and
  // batch b + 1's features (whose ids arrived during step b - 1) are in flight, so no step waits on
  // the dependent perm -> X round trip. Element e = t + 256 q of the B x F block (<= 4 * 256).
  float nx[4], ny = 0.0f;
  int32_t nid[4], nyid = 0;
  auto fetch_ids = [&](int64_t bb) {
    const int bsz = bb < nb ? (int)min((int64_t)B, n - bb * B) : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (t + kTrThreads * q) / F;
      nid[q] = r < bsz ? pm[bb * B + r] : -1;
    }
    nyid = t < bsz ? pm[bb * B + t] : -1;
  };
  auto fetch = [&]() {  // features of the batch whose ids are in nid
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = t + kTrThreads * q, f = e - (e / F) * F;
      nx[q] = nid[q] >= 0 ? X[(int64_t)nid[q] * ldx + f] : 0.0f;
    }
    ny = nyid >= 0 ? y[nyid] : 0.0f;
  };
  auto stage = [&](int buf) {
    float* xb = xbuf + buf * MB * XP;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = t + kTrThreads * q, r = e / F, f = e - r * F;
      if (r < MB) xb[r * XP + f] = nx[q];
    }
    if (t < MB) ybuf[buf * MB + t] = ny;
  };
  __syncthreads();  // x buffer constants before the first stage
  if (nb > 0) {
    fetch_ids(0);
    fetch();
    stage(0);
    fetch_ids(1);
  }
  __syncthreads();

  if (timing) ph_last = wall_clock64();
  for (int64_t b = 0; b < nb; ++b) {
    // The lane index is laundered once per step: every LDS address below is loop-invariant, and
    // hoisted out of the step loop they would pin ~300 VGPRs for the whole epoch (spilling).
    int lane_ = lane;
    asm volatile("" : "+v"(lane_));
    const int li = lane_ & 31, hi = lane_ >> 5;
    int w = __builtin_amdgcn_readfirstlane(t >> 6);
    asm volatile("" : "+s"(w));
    const int buf = (int)(b & 1);
    const int bs = (int)min((int64_t)B, n - b * B);
    const float* xb = xbuf + buf * MB * XP;
    if (b + 1 < nb) {
      fetch();           // batch b + 1 (ids loaded during the previous step)
      fetch_ids(b + 2);  // ids of batch b + 2
    }
    if ((b & (kTrThreads - 1)) == 0) {
      // learning-rate schedule and bias correction of the next 256 steps, one step per thread (the
      // three powf per step would otherwise cost every wave ~450 instructions per step)
      const float st = (float)(step + t);
      const float e = hp.staircase ? floorf(st / (float)hp.decay_steps) : st / (float)hp.decay_steps;
      const float lr = hp.lr0 * powf(hp.decay_rate, e);
      const float tt = st + 1.0f;
      sched[t] = make_float2(lr, lr * sqrtf(1.0f - powf(hp.beta2, tt)) / (1.0f - powf(hp.beta1, tt)));
      __syncthreads();
    }
    TR_PHASE(0)
    AdamStep s;
    {
      const float2 sc = sched[b & (kTrThreads - 1)];
      s.lr = sc.x;
      s.lr_t = sc.y;
      s.wd = hp.weight_decay;
      s.b1 = hp.beta1;
      s.b2 = hp.beta2;
      s.eps = hp.eps;
      s.l2 = hp.l2;
    }
    // ---- F1: layer 1 tile w, layer-2 partial over this tile
    f32x16 a1 = {};
#pragma unroll
    for (int s_ = 0; s_ < 4 * NQ; ++s_) a1 = MFMA32(w1r[s_], xb[li * XP + rowD(s_, hi)], a1);
    f32x16 a2 = {};
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const float h = fmaxf(a1[v], 0.0f);
      h1s[li * H1P + 32 * w + rowD(v, hi)] = h;
      a2 = MFMA32(w2r[v], h, a2);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      reinterpret_cast<float4*>(red)[(w * 4 + q) * 64 + lane] = make_float4(a2[4 * q], a2[4 * q + 1], a2[4 * q + 2], a2[4 * q + 3]);
    TR_PHASE(1)
    __syncthreads();
    TR_PHASE(2)
    // ---- F2 (every wave, redundantly): layer 2 sum, layer 3, output, deltas 3 / 2, delta 1 tile w
    float h2[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const float4 r = reinterpret_cast<const float4*>(red)[(ww * 4 + q) * 64 + lane];
        acc.x += r.x;
        acc.y += r.y;
        acc.z += r.z;
        acc.w += r.w;
      }
      h2[4 * q + 0] = fmaxf(acc.x + SP[kSmB2 + rowD(4 * q + 0, hi)], 0.0f);
      h2[4 * q + 1] = fmaxf(acc.y + SP[kSmB2 + rowD(4 * q + 1, hi)], 0.0f);
      h2[4 * q + 2] = fmaxf(acc.z + SP[kSmB2 + rowD(4 * q + 2, hi)], 0.0f);
      h2[4 * q + 3] = fmaxf(acc.w + SP[kSmB2 + rowD(4 * q + 3, hi)], 0.0f);
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x16 a3;
#pragma unroll
    for (int v = 0; v < 16; ++v) a3[v] = SP[kSmB3 + rowD(v, hi)];  // zero above unit 15
#pragma unroll
    for (int s_ = 0; s_ < 16; ++s_) a3 = MFMA32(li < H3 ? W3s[rowD(s_, hi) * W3P + li] : 0.0f, h2[s_], a3);
    float h3[8];
    float z = 0.0f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      h3[v] = fmaxf(a3[v], 0.0f);
      z = fmaf(SP[kSmW4 + rowD(v, hi)], h3[v], z);
    }
    z += __shfl_xor(z, 32);
    z += SP[kSmB4];
    const float yy = ybuf[buf * MB + li];
    const float pr = __builtin_amdgcn_rcpf(1.0f + __expf(-z));
    const float d4 = li < bs ? (pr - yy) / (float)bs : 0.0f;
    float d3[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) d3[v] = h3[v] > 0.0f ? SP[kSmW4 + rowD(v, hi)] * d4 : 0.0f;
    __builtin_amdgcn_sched_barrier(0);
    f32x16 a2d = {};
#pragma unroll
    for (int s_ = 0; s_ < 8; ++s_) a2d = MFMA32(W3s[li * W3P + rowD(s_, hi)], d3[s_], a2d);
    float d2[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) d2[v] = h2[v] > 0.0f ? a2d[v] : 0.0f;
    __builtin_amdgcn_sched_barrier(0);
    f32x16 a1d = {};
#pragma unroll
    for (int s_ = 0; s_ < 16; ++s_) a1d = MFMA32(W2s[(32 * w + li) * W2P + rowD(s_, hi)], d2[s_], a1d);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int o = li * H1P + 32 * w + rowD(v, hi);
      d1s[o] = h1s[o] > 0.0f ? a1d[v] : 0.0f;
    }
    __builtin_amdgcn_sched_barrier(0);
    if (w == 0) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        h2s[li * H2P + rowD(v, hi)] = h2[v];
        d2s[li * H2P + rowD(v, hi)] = d2[v];
      }
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        h3s[li * H3P + rowD(v, hi)] = h3[v];
        d3s[li * H3P + rowD(v, hi)] = d3[v];
      }
      if (hi == 0) d4s[li] = d4;
    }
    TR_PHASE(3)
    __syncthreads();
    TR_PHASE(4)
    // ---- G: weight gradients over the batch rows + AdamW. VALU updates are interleaved with the
    // next gradient chain so they issue between its MFMAs: W1 with dW2, W2 with dW3 (waves 1, 3).
    const float l2x2 = 2.0f * s.l2;
    f32x16 g1 = {};
#pragma unroll
    for (int s_ = 0; s_ < 16; ++s_) {
      const int r = 2 * s_ + hi;
      g1 = MFMA32(xb[r * XP + li], d1s[r * H1P + 32 * w + li], g1);
    }
    f32x16 g2 = {};
#pragma unroll
    for (int s_ = 0; s_ < 16; ++s_) {
      const int r = 2 * s_ + hi;
      g2 = MFMA32(h1s[r * H1P + 32 * w + li], d2s[r * H2P + li], g2);
      if (s_ < 4 * NQ) {  // registers above 4 NQ hold rows > F only (zero weight, gradient, moments)
        const int f = rowD(s_, hi);  // rows F+1 .. 4 NQ stay zero the same way
        float2 mv = MV1[f * H1 + 32 * w + li];
        adam_f(w1r[s_], mv.x, mv.y, g1[s_], f < F ? l2x2 : 0.0f, s);
        MV1[f * H1 + 32 * w + li] = mv;
      }
    }
    auto adam_w2 = [&](int v) {
      const int k = 32 * w + rowD(v, hi);
      float2 mv = MV2[k * H2 + li];
      adam_f(w2r[v], mv.x, mv.y, g2[v], l2x2, s);
      MV2[k * H2 + li] = mv;
      W2s[k * W2P + li] = w2r[v];
    };
    if (w & 1) {  // W3 (columns j = li < 16): waves 1 and 3 both form the gradient, each updates half
      f32x16 g3 = {};
#pragma unroll
      for (int s_ = 0; s_ < 16; ++s_) {
        const int r = 2 * s_ + hi;
        g3 = MFMA32(h2s[r * H2P + li], li < H3 ? d3s[r * H3P + li] : 0.0f, g3);
        adam_w2(s_);
      }
      if (li < H3) {
        if (w == 1) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            adam_f(w3r[q], m3r[q], v3r[q], g3[q], l2x2, s);
            W3s[rowD(q, hi) * W3P + li] = w3r[q];
          }
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            adam_f(w3r[q], m3r[q], v3r[q], g3[8 + q], l2x2, s);
            W3s[rowD(8 + q, hi) * W3P + li] = w3r[q];
          }
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < 16; ++v) adam_w2(v);
      if (w == 0) {  // batch loss (reported only): mean BCE from the logit over the bs real rows
        float l = (hi == 0 && li < bs) ? fmaxf(z, 0.0f) - z * yy + __logf(1.0f + __expf(-fabsf(z))) : 0.0f;
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) l += __shfl_xor(l, o);
        if (lane == 0) loss_acc += l / (float)bs;
      } else {  // wave 2: b2 (lanes 0..31), b3 (32..47), W4 (48..63), b4 (lane 48 too)
        float gg = 0.0f;
        int slot;
        if (lane < 32) {
          slot = kSmB2 + lane;
#pragma unroll
          for (int r = 0; r < MB; ++r) gg += d2s[r * H2P + lane];
        } else if (lane < 48) {
          slot = kSmB3 + lane - 32;
#pragma unroll
          for (int r = 0; r < MB; ++r) gg += d3s[r * H3P + lane - 32];
        } else {
          slot = kSmW4 + lane - 48;
          float g4 = 0.0f;
#pragma unroll
          for (int r = 0; r < MB; ++r) {
            const float d = d4s[r];
            gg = fmaf(h3s[r * H3P + lane - 48], d, gg);
            g4 += d;
          }
          if (lane == 48) adam_f(SP[kSmB4], SP[96 + kSmB4], SP[192 + kSmB4], g4, 0.0f, s);
        }
        adam_f(SP[slot], SP[96 + slot], SP[192 + slot], gg, 0.0f, s);
      }
    }
    if (b + 1 < nb) stage(buf ^ 1);
    ++step;
    TR_PHASE(5)
    __syncthreads();
    TR_PHASE(6)
  }
#undef TR_PHASE
  if (timing)
    for (int i = 0; i < 7; ++i) prof[8 * (threadIdx.x == 192) + i] += ph[i];
  // ---- epilogue: parameters and moments back to the flat layout
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int f = rowD(v, hi), c = 32 * w + li;
    const float2 mv1 = MV1[f * H1 + c];
    if (f < F) {
      gp.W1[f * H1 + c] = w1r[v];
      gm.W1[f * H1 + c] = mv1.x;
      gv.W1[f * H1 + c] = mv1.y;
    } else if (f == F) {
      gp.b1[c] = w1r[v];
      gm.b1[c] = mv1.x;
      gv.b1[c] = mv1.y;
    }
    const int k = 32 * w + rowD(v, hi);
    const float2 mv2 = MV2[k * H2 + li];
    gp.W2[k * H2 + li] = w2r[v];
    gm.W2[k * H2 + li] = mv2.x;
    gv.W2[k * H2 + li] = mv2.y;
  }
  if ((w & 1) && li < H3) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = rowD(q + (w == 3 ? 8 : 0), hi) * H3 + li;
      gp.W3[e] = w3r[q];
      gm.W3[e] = m3r[q];
      gv.W3[e] = v3r[q];
    }
  }
  if (t < 96) {
    float* dst[3] = {nullptr, nullptr, nullptr};
    if (t < 32) {
      dst[0] = gp.b2 + t; dst[1] = gm.b2 + t; dst[2] = gv.b2 + t;
    } else if (t < 32 + H3) {
      dst[0] = gp.b3 + t - 32; dst[1] = gm.b3 + t - 32; dst[2] = gv.b3 + t - 32;
    } else if (t >= 64 && t < 64 + H3) {
      dst[0] = gp.W4 + t - 64; dst[1] = gm.W4 + t - 64; dst[2] = gv.W4 + t - 64;
    } else if (t == kSmB4) {
      dst[0] = gp.b4; dst[1] = gm.b4; dst[2] = gv.b4;
    }
    if (dst[0]) {
      *dst[0] = SP[t];
      *dst[1] = SP[96 + t];
      *dst[2] = SP[192 + t];
    }
  }
  if (t == 0) {
    steps[model] = step;
    loss_out[model] = loss_acc;
  }
}
#undef MFMA32
}  // namespace

COBALT_API int cobalt_mlp_num_params(int F) { return mlp_params(F); }

COBALT_API int cobalt_mlp_train_epoch(const float* X, int64_t ldx, const float* y, int64_t n, int F,
                                      const int32_t* perm, float* params, float* m, float* v, int64_t* steps,
                                      const void* hyper, int n_models, float* loss_out, uint64_t* prof,
                                      hipStream_t stream) {
  if (F < 1 || F > kMaxF) return -1;
  if (n < 1 || n_models < 1) return 0;
  MlpHyper hp = *static_cast<const MlpHyper*>(hyper);
  if (hp.batch < 1 || hp.batch > MB || hp.decay_steps < 1) return -2;
  const size_t lds = ((size_t)3 * mlp_params(F) + act_floats(F)) * sizeof(float);
  if (lds > 160 * 1024) return -3;
  CK(hipFuncSetAttribute((const void*)k_mlp_train, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_mlp_train, dim3(n_models), dim3(NT), lds, stream, X, ldx, y, n, F, perm, params, m, v, steps,
                     hp, loss_out, prof);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_mlp_train_epoch_mfma(const float* X, int64_t ldx, const float* y, int64_t n, int F,
                                           const int32_t* perm, float* params, float* m, float* v, int64_t* steps,
                                           const void* hyper, int n_models, float* loss_out, uint64_t* prof,
                                           hipStream_t stream) {
  if (F < 1 || F > kTrMaxF) return -1;
  if (n < 1 || n_models < 1) return 0;
  MlpHyper hp = *static_cast<const MlpHyper*>(hyper);
  if (hp.batch < 1 || hp.batch > MB || hp.decay_steps < 1) return -2;
  const size_t lds = (size_t)tr_layout().total * sizeof(float);  // 157 KB
  static_assert(tr_layout().total * sizeof(float) <= 160 * 1024, "trainer LDS image exceeds 160 KB");
  const void* fn = nullptr;
  switch (F / 8 + 1) {
    case 1: fn = (const void*)k_mlp_train_mfma<1>; break;
    case 2: fn = (const void*)k_mlp_train_mfma<2>; break;
    case 3: fn = (const void*)k_mlp_train_mfma<3>; break;
    default: fn = (const void*)k_mlp_train_mfma<4>; break;
  }
  CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {(void*)&X, (void*)&ldx, (void*)&y, (void*)&n, (void*)&F, (void*)&perm, (void*)&params, (void*)&m,
                  (void*)&v, (void*)&steps, (void*)&hp, (void*)&loss_out, (void*)&prof};
  CK(hipLaunchKernel(fn, dim3(n_models), dim3(kTrThreads), args, lds, stream));
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_mlp_forward(const float* X, int64_t ldx, int64_t n, int F, const float* params, float* prob,
                                  float* logit, hipStream_t stream) {
  if (F < 1 || F > kMaxF) return -1;
  if (n < 1) return 0;
  const size_t lds = ((size_t)mlp_params(F) + act_floats(F)) * sizeof(float);
  if (lds > 64 * 1024)
    CK(hipFuncSetAttribute((const void*)k_mlp_forward, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t tiles = (n + MB - 1) / MB;
  const int grid = (int)std::min<int64_t>(tiles, 2048);
  hipLaunchKernelGGL(k_mlp_forward, dim3(grid), dim3(NT), lds, stream, X, ldx, n, F, params, prob, logit);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_mlp_forward_mfma(const float* X, int64_t ldx, int64_t n, int F, const float* params, float* prob,
                                       float* logit, hipStream_t stream) {
  if (F < 1 || F > kMaxF) return -1;
  if (n < 1) return 0;
  const size_t lds = (size_t)fwd_lds_floats((F + 1) / 2) * sizeof(float);  // 37.4 KB at F = 20
  if (lds > 64 * 1024)
    CK(hipFuncSetAttribute((const void*)k_mlp_forward_mfma, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t tiles = (n + 31) / 32;
  const int64_t waves = kFwdThreads / 64;
  const int grid = (int)std::min<int64_t>((tiles + waves - 1) / waves, 1024);  // 4 workgroups per CU
  hipLaunchKernelGGL(k_mlp_forward_mfma, dim3(grid), dim3(kFwdThreads), lds, stream, X, ldx, n, F, params, prob,
                     logit);
  CK_LAUNCH();
  return 0;
}
