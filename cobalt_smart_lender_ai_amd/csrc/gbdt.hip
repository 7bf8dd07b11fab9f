// Histogram gradient-boosted-tree trainer for gfx950 (MI355X).
//
// Replaces the XGBoost 3.0 `hist` updater the reference drives through
// `XGBClassifier.fit` (reference: src/model_train_test/model_tree_train_test.py:111-164,
// notebooks/04_model_training.ipynb:1877-2016).
//
// Design (MI355X-first, not a translation of XGBoost's CPU/CUDA code):
//  * Features are pre-quantised to uint8 bins (255 real bins + 255 = missing), stored twice:
//    row-major [N][stride] for histogram gathers (one row = a few dwords) and feature-major
//    [F][N] for the partition step (one byte per row, coalesced within a node).
//  * Gradients are quantised to fixed point and packed into one u64 per row
//    (hi 32 = signed g_q, lo 32 = unsigned h_q). A single LDS `ds_add_u64` then accumulates
//    both statistics of a (feature, bin) cell; the h half never carries into the g half
//    because per-block sums stay below 2^32. Integer sums make every histogram exact and
//    independent of atomic order, so 1-GPU and N-GPU training give bit-identical trees.
//  * Rows of each node are contiguous in a ping-pong row-index buffer (stable-ish two-ended
//    partition). Only the child with the smaller global hessian is histogrammed; its sibling
//    comes from parent - child (subtraction trick).
//  * All sizes that depend on data live in device memory: every kernel is launched with a
//    host-side upper-bound grid and early-exits, so the host never synchronises inside a tree
//    and a whole tree (or fit) can be enqueued back to back / captured in a hipGraph.
//  * Data parallel: the only cross-rank traffic is one int64 SUM all-reduce of the built
//    histogram slots per level, issued on the same stream through a native RCCL communicator.
#include "common.h"
#include <math.h>
#include <string.h>
#include <vector>
#include <algorithm>

using namespace cobalt;

namespace {

enum NodeStatus : int32_t { kNone = 0, kActive = 1, kSplit = 2, kLeaf = 3 };

// 64-byte node record; mirrored by NODE_DTYPE in ops/gbdt_ops.py.
struct Node {
  int64_t G, H;            // quantised gradient / hessian sums (global across ranks)
  int32_t start, count;    // local row range in the ridx buffer of this node's level parity
  int32_t status, build;   // NodeStatus; build=1 -> histogram built directly, 0 -> by subtraction
  int32_t feat, bin;       // split feature, split bin j (left <=> bin <= j)
  int32_t default_left;
  float split_cond;        // threshold (x < cond goes left) or leaf value for leaves
  float loss_chg, leaf_value;
  float sum_hess, base_weight;
};
static_assert(sizeof(Node) == 64, "Node layout");

struct WorkItem {
  int32_t node, slot, begin, end;
};

struct Cand {
  double gain;
  int32_t key;
  int64_t gl, hl;
};

__device__ __forceinline__ bool cand_better(const Cand& a, const Cand& b) {
  return a.gain > b.gain || (a.gain == b.gain && a.key < b.key);
}

__device__ __forceinline__ Cand cand_shfl_xor(const Cand& c, int o) {
  Cand r;
  r.gain = __shfl_xor(c.gain, o, kWave);
  r.key = __shfl_xor(c.key, o, kWave);
  r.gl = __shfl_xor(c.gl, o, kWave);
  r.hl = __shfl_xor(c.hl, o, kWave);
  return r;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Public configuration (mirrored by the ctypes Structure GbdtConfig in ops/gbdt_ops.py)
// ------------------------------------------------------------------------------------------
struct GbdtConfig {
  int64_t n_rows;        // local rows on this rank
  int64_t row_offset;    // global index of local row 0 (keys the row-sampling hash)
  int32_t n_feat;
  int32_t row_stride;    // bytes per row of the row-major bin matrix (multiple of 4)
  int32_t max_depth;
  int32_t max_trees;
  int32_t chunk;         // rows per histogram / partition work item (<= 16384)
  int32_t feat_tile;     // features per histogram block (multiple of 4)
  double eta, lambda_, alpha, gamma, min_child_weight, subsample;
  double gscale, hscale; // g_q = rint(g * gscale), h_q = rint(h * hscale)
  float base_margin;
  int32_t world_size;
  uint64_t seed;
  void* comm;            // native RCCL communicator (cobalt_comm_*) or nullptr
};

struct GbdtDev {
  // inputs
  const uint8_t* bins;    // [N][stride]
  const uint8_t* binsT;   // [F][N]
  const float* cuts;      // [F][256]
  const int32_t* nbins;   // [F]
  const float* label;     // [N]
  const float* weight;    // [N] sample weight incl. scale_pos_weight for positives
  float* margin;          // [N]
  const uint8_t* fmask;   // [max_trees][F] colsample_bytree masks
  // workspace
  uint64_t* gpair;        // [N]
  int32_t* ridx[2];       // [N] x2
  int64_t* hist_b[2];     // [pairs][F+1][256][2]
  int64_t* hist_s[2];
  Node* nodes;            // [max_nodes]
  Node* trees;            // [max_trees][max_nodes]
  WorkItem* items_h;      // histogram work list
  WorkItem* items_p;      // partition work list
  int32_t* counters;      // [0] = #hist items, [1] = #partition items
  int32_t* cursors;       // [max_nodes][2]
  int64_t n;
  int64_t row_offset;
  int32_t F, stride, max_depth, max_nodes, chunk, feat_tile;
  int64_t slot_elems;     // (F+1)*256*2
  double eta, lambda_, alpha, gamma, mcw, subsample, gscale, hscale, ginv, hinv;
  uint64_t seed;
};

// ------------------------------------------------------------------------------------------
// Binning: X fp32 [N][F] (row-major, NaN = missing) -> uint8 bins (row-major + feature-major)
// bin(x) = #cuts <= x (upper_bound), clamped to nbins-1; NaN -> 255.
// ------------------------------------------------------------------------------------------
template <bool CUTS_IN_LDS>
__global__ __launch_bounds__(256) void k_bin(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                             const float* __restrict__ cuts, const int32_t* __restrict__ nbins,
                                             uint8_t* __restrict__ bins, int stride,
                                             uint8_t* __restrict__ binsT) {
  extern __shared__ float s_cuts[];
  if (CUTS_IN_LDS) {
    for (int i = threadIdx.x; i < F * kMaxBins; i += blockDim.x) s_cuts[i] = cuts[i];
    __syncthreads();
  }
  const float* C = CUTS_IN_LDS ? s_cuts : cuts;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n;
       row += (int64_t)gridDim.x * blockDim.x) {
    const float* x = X + row * ldx;
    uint32_t word = 0;
    for (int f = 0; f < stride; ++f) {
      uint32_t b = 0;
      if (f < F) {
        float v = x[f];
        const int nb = nbins[f];
        if (v != v) {
          b = kMissingBin;
        } else {
          // upper_bound over cuts[f][0..nb)
          const float* c = C + f * kMaxBins;
          int lo = 0, hi = nb;
          while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (c[mid] <= v) lo = mid + 1; else hi = mid;
          }
          b = lo >= nb ? (uint32_t)(nb - 1) : (uint32_t)lo;
        }
        binsT[(int64_t)f * n + row] = (uint8_t)b;
      }
      word |= b << (8 * (f & 3));
      if ((f & 3) == 3) {
        *reinterpret_cast<uint32_t*>(bins + row * stride + (f & ~3)) = word;
        word = 0;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Per-tree initialisation + binary:logistic gradients (K14)
// ------------------------------------------------------------------------------------------
__global__ void k_init_tree(GbdtDev d) {
  for (int i = threadIdx.x; i < d.max_nodes; i += blockDim.x) {
    Node nd = {};
    if (i == 0) {
      nd.status = kActive;
      nd.build = 1;
      nd.start = 0;
      nd.count = (int32_t)d.n;
    }
    nd.feat = -1;
    nd.bin = -1;
    d.nodes[i] = nd;
    d.cursors[2 * i] = 0;
    d.cursors[2 * i + 1] = 0;
  }
}

__global__ __launch_bounds__(256) void k_grad(GbdtDev d, int tree) {
  const uint64_t tree_key = splitmix64(d.seed ^ (0xA5A5A5A5ull + (uint64_t)tree * 0x632BE59BD9B4E019ull));
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    d.ridx[0][i] = (int32_t)i;
    const double m = (double)d.margin[i];
    const double p = 1.0 / (1.0 + exp(-m));
    const double y = (double)d.label[i];
    const double w = (double)d.weight[i];
    double g = (p - y) * w;
    double h = fmax(p * (1.0 - p), 1e-16) * w;
    if (d.subsample < 1.0) {
      const uint64_t hsh = splitmix64(tree_key ^ (uint64_t)(d.row_offset + i));
      if (!(uniform01(hsh) < d.subsample)) { g = 0.0; h = 0.0; }
    }
    int64_t gq = (int64_t)rint(g * d.gscale);
    int64_t hq = (int64_t)rint(h * d.hscale);
    gq = gq > 65536 ? 65536 : (gq < -65536 ? -65536 : gq);
    hq = hq > 65536 ? 65536 : (hq < 0 ? 0 : hq);
    d.gpair[i] = ((uint64_t)(uint32_t)(int32_t)gq << 32) | (uint64_t)(uint32_t)hq;
  }
}

// ------------------------------------------------------------------------------------------
// Level planning: child row ranges from partition cursors, choose which child to build,
// emit histogram work items. One block.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_plan_hist(GbdtDev d, int level) {
  __shared__ int32_t s_chunks[1024];
  __shared__ int32_t s_node[1024];
  __shared__ int32_t s_off[1025];
  const int npairs = level == 0 ? 1 : (1 << (level - 1));
  for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
    int built = -1;
    if (level == 0) {
      built = 0;
    } else {
      const int q = (1 << (level - 1)) - 1 + p;  // parent
      Node& par = d.nodes[q];
      if (par.status == kSplit) {
        const int L = 2 * q + 1, R = 2 * q + 2;
        const int lc = d.cursors[2 * q];
        d.nodes[L].start = par.start;
        d.nodes[L].count = lc;
        d.nodes[R].start = par.start + lc;
        d.nodes[R].count = par.count - lc;
        const bool left_small = d.nodes[L].H <= d.nodes[R].H;
        d.nodes[L].build = left_small ? 1 : 0;
        d.nodes[R].build = left_small ? 0 : 1;
        built = left_small ? L : R;
      }
    }
    s_node[p] = built;
    s_chunks[p] = built >= 0 ? (d.nodes[built].count + d.chunk - 1) / d.chunk : 0;
  }
  // reset partition cursors of this level's nodes
  const int first = (1 << level) - 1, nlev = 1 << level;
  for (int i = threadIdx.x; i < nlev; i += blockDim.x) {
    d.cursors[2 * (first + i)] = 0;
    d.cursors[2 * (first + i) + 1] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int p = 0; p < npairs; ++p) { s_off[p] = acc; acc += s_chunks[p]; }
    s_off[npairs] = acc;
    d.counters[0] = acc;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
    const int nd = s_node[p];
    if (nd < 0) continue;
    const int st = d.nodes[nd].start, cnt = d.nodes[nd].count;
    for (int c = 0; c < s_chunks[p]; ++c) {
      WorkItem w;
      w.node = nd;
      w.slot = p;
      w.begin = st + c * d.chunk;
      w.end = min(st + cnt, w.begin + d.chunk);
      d.items_h[s_off[p] + c] = w;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Histogram build (K15): LDS-privatised packed-u64 histograms, one work item per block,
// blockIdx.y = feature tile. Flush = one int64 global atomic per non-zero cell per block.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hist(GbdtDev d, int parity, int tree) {
  extern __shared__ uint64_t s_hist[];  // [feat_tile][256]
  __shared__ int64_t s_tot[2][4];
  const int item = blockIdx.x;
  if (item >= d.counters[0]) return;
  const WorkItem w = d.items_h[item];
  const int f0 = blockIdx.y * d.feat_tile;
  if (f0 >= d.F) return;
  const int ft = min(d.feat_tile, d.F - f0);
  const uint8_t* fm = d.fmask + (int64_t)tree * d.F + f0;
  uint64_t fbits = 0;
  for (int k = 0; k < ft; ++k) fbits |= (uint64_t)(fm[k] != 0) << k;

  for (int i = threadIdx.x; i < ft * kMaxBins; i += blockDim.x) s_hist[i] = 0ull;
  __syncthreads();

  const int32_t* rix = d.ridx[parity];
  int64_t tg = 0, th = 0;
  const int nwords = (ft + 3) >> 2;
  for (int i = w.begin + threadIdx.x; i < w.end; i += blockDim.x) {
    const int r = rix[i];
    const uint64_t gp = d.gpair[r];
    tg += (int64_t)(int32_t)(uint32_t)(gp >> 32);
    th += (int64_t)(uint32_t)gp;
    if (gp == 0ull) continue;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(d.bins + (int64_t)r * d.stride + f0);
    for (int q = 0; q < nwords; ++q) {
      const uint32_t word = row[q];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int fl = q * 4 + k;
        const uint32_t b = (word >> (8 * k)) & 0xffu;
        if (fl < ft && b != kMissingBin && ((fbits >> fl) & 1ull)) atomicAdd(reinterpret_cast<unsigned long long*>(&s_hist[fl * kMaxBins + b]),
                                                               (unsigned long long)gp);
      }
    }
  }
  __syncthreads();
  int64_t* gh = d.hist_b[parity] + (int64_t)w.slot * d.slot_elems;
  for (int e = threadIdx.x; e < ft * kMaxBins; e += blockDim.x) {
    const uint64_t v = s_hist[e];
    if (v) {
      const int64_t g = (int64_t)(int32_t)(uint32_t)(v >> 32);
      const int64_t h = (int64_t)(uint32_t)v;
      int64_t* cell = gh + ((int64_t)(f0 * kMaxBins + e)) * 2;
      atomicAdd(reinterpret_cast<unsigned long long*>(cell), (unsigned long long)g);
      atomicAdd(reinterpret_cast<unsigned long long*>(cell + 1), (unsigned long long)h);
    }
  }
  if (blockIdx.y == 0) {
    tg = wave_sum(tg);
    th = wave_sum(th);
    if (lane_id() == 0) { s_tot[0][wave_id()] = tg; s_tot[1][wave_id()] = th; }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t G = 0, H = 0;
      for (int k = 0; k < (int)(blockDim.x / kWave); ++k) { G += s_tot[0][k]; H += s_tot[1][k]; }
      int64_t* cell = gh + (int64_t)d.F * kMaxBins * 2;
      atomicAdd(reinterpret_cast<unsigned long long*>(cell), (unsigned long long)G);
      atomicAdd(reinterpret_cast<unsigned long long*>(cell + 1), (unsigned long long)H);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Split evaluation (K16 + K17): one block per node of the level, one wavefront per feature,
// 4 bins per lane, 64-lane int64 prefix scan, both default directions.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double thresh_l1(double g, double alpha) {
  if (g > alpha) return g - alpha;
  if (g < -alpha) return g + alpha;
  return 0.0;
}

__device__ __forceinline__ double calc_gain(double g, double h, double lambda_, double alpha, double mcw) {
  if (h < mcw) return 0.0;
  const double t = alpha == 0.0 ? g : thresh_l1(g, alpha);
  return (t * t) / (h + lambda_);
}

__device__ __forceinline__ double calc_weight(double g, double h, double lambda_, double alpha, double mcw) {
  if (h < mcw || h <= 0.0) return 0.0;
  const double t = alpha == 0.0 ? g : thresh_l1(g, alpha);
  return -t / (h + lambda_);
}

__global__ __launch_bounds__(256) void k_eval(GbdtDev d, int level, int parity, int tree) {
  const int pos = blockIdx.x;
  const int n = (1 << level) - 1 + pos;
  Node* nodes = d.nodes;
  if (nodes[n].status != kActive) return;
  __shared__ Cand s_best[4];
  __shared__ int64_t s_GH[2];

  const int pair = level == 0 ? 0 : (pos >> 1);
  const int64_t SE = d.slot_elems;
  const int64_t* hb = d.hist_b[parity] + pair * SE;
  int64_t* hs = d.hist_s[parity] + pair * SE;
  const bool built = nodes[n].build != 0;

  if (threadIdx.x == 0) {
    if (level == 0) {
      nodes[n].G = hb[(int64_t)d.F * kMaxBins * 2];
      nodes[n].H = hb[(int64_t)d.F * kMaxBins * 2 + 1];
    }
    s_GH[0] = nodes[n].G;
    s_GH[1] = nodes[n].H;
  }
  __syncthreads();
  const int64_t G = s_GH[0], H = s_GH[1];
  const double Gd = (double)G * d.ginv, Hd = (double)H * d.hinv;

  if (level < d.max_depth) {
    const int64_t* parent = nullptr;
    if (!built) {
      const int ppos = pos >> 1;
      const int q = (1 << (level - 1)) - 1 + ppos;
      const int ppair = level == 1 ? 0 : (ppos >> 1);
      parent = (nodes[q].build ? d.hist_b[parity ^ 1] : d.hist_s[parity ^ 1]) + ppair * SE;
    }
    const double parent_gain = calc_gain(Gd, Hd, d.lambda_, d.alpha, d.mcw);
    Cand best;
    best.gain = -INFINITY;
    best.key = 0x7fffffff;
    best.gl = 0;
    best.hl = 0;
    const int lane = lane_id();
    const uint8_t* fm = d.fmask + (int64_t)tree * d.F;
    for (int f = wave_id(); f < d.F; f += (int)(blockDim.x / kWave)) {
      if (!fm[f]) continue;
      const int nb = d.nbins[f];
      int64_t g[4], h[4];
      const int64_t base = ((int64_t)f * kMaxBins + lane * 4) * 2;
      if (built) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { g[k] = hb[base + 2 * k]; h[k] = hb[base + 2 * k + 1]; }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          g[k] = parent[base + 2 * k] - hb[base + 2 * k];
          h[k] = parent[base + 2 * k + 1] - hb[base + 2 * k + 1];
          hs[base + 2 * k] = g[k];
          hs[base + 2 * k + 1] = h[k];
        }
      }
      int64_t cg[4], ch[4];
      cg[0] = g[0]; ch[0] = h[0];
#pragma unroll
      for (int k = 1; k < 4; ++k) { cg[k] = cg[k - 1] + g[k]; ch[k] = ch[k - 1] + h[k]; }
      const int64_t ig = wave_incl_scan(cg[3]), ih = wave_incl_scan(ch[3]);
      const int64_t eg = ig - cg[3], eh = ih - ch[3];
      const int64_t sg = __shfl(ig, kWave - 1, kWave), sh = __shfl(ih, kWave - 1, kWave);
      const int64_t mg = G - sg, mh = H - sh;  // missing-value statistics
      const bool has_missing = (mg != 0) || (mh != 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int b = lane * 4 + k;
        if (b >= nb) continue;
        // direction 0: missing -> right, left = bins <= b
        {
          const int64_t GL = eg + cg[k], HL = eh + ch[k];
          const double gl = (double)GL * d.ginv, hl = (double)HL * d.hinv;
          const double gr = (double)(G - GL) * d.ginv, hr = (double)(H - HL) * d.hinv;
          if (hl >= d.mcw && hr >= d.mcw) {
            Cand c;
            c.gain = calc_gain(gl, hl, d.lambda_, d.alpha, d.mcw) + calc_gain(gr, hr, d.lambda_, d.alpha, d.mcw) - parent_gain;
            c.key = f * 1024 + b;
            c.gl = GL;
            c.hl = HL;
            if (cand_better(c, best)) best = c;
          }
        }
        // direction 1: missing -> left, left = bins <= b-1 (+ missing)
        if (has_missing && b <= nb - 1) {
          const int64_t GL = eg + cg[k] - g[k] + mg, HL = eh + ch[k] - h[k] + mh;
          const double gl = (double)GL * d.ginv, hl = (double)HL * d.hinv;
          const double gr = (double)(G - GL) * d.ginv, hr = (double)(H - HL) * d.hinv;
          if (hl >= d.mcw && hr >= d.mcw) {
            Cand c;
            c.gain = calc_gain(gl, hl, d.lambda_, d.alpha, d.mcw) + calc_gain(gr, hr, d.lambda_, d.alpha, d.mcw) - parent_gain;
            c.key = f * 1024 + 512 + (nb - 1 - b);
            c.gl = GL;
            c.hl = HL;
            if (cand_better(c, best)) best = c;
          }
        }
      }
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      Cand other = cand_shfl_xor(best, o);
      if (cand_better(other, best)) best = other;
    }
    if (lane == 0) s_best[wave_id()] = best;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int k = 1; k < (int)(blockDim.x / kWave); ++k)
      if (cand_better(s_best[k], best)) best = s_best[k];
    const float loss = (float)best.gain;
    const bool ok = best.key != 0x7fffffff && loss > 1e-6f && loss >= (float)d.gamma;
    const double wgt = calc_weight(Gd, Hd, d.lambda_, d.alpha, d.mcw);
    Node& nd = nodes[n];
    nd.sum_hess = (float)Hd;
    nd.base_weight = (float)(wgt * d.eta);
    if (ok) {
      const int f = best.key >> 10;
      const int r = best.key & 1023;
      const int nb = d.nbins[f];
      int j, dl;
      if (r < 512) { j = r; dl = 0; } else { j = (nb - 1 - (r - 512)) - 1; dl = 1; }
      nd.status = kSplit;
      nd.feat = f;
      nd.bin = j;
      nd.default_left = dl;
      nd.split_cond = j >= 0 ? d.cuts[f * kMaxBins + j] : -FLT_MAX;
      nd.loss_chg = loss;
      Node& L = nodes[2 * n + 1];
      Node& R = nodes[2 * n + 2];
      L.status = kActive; L.G = best.gl; L.H = best.hl;
      R.status = kActive; R.G = G - best.gl; R.H = H - best.hl;
    } else {
      nd.status = kLeaf;
      nd.leaf_value = (float)(wgt * d.eta);
      nd.split_cond = nd.leaf_value;
    }
  } else if (threadIdx.x == 0) {
    const double wgt = calc_weight(Gd, Hd, d.lambda_, d.alpha, d.mcw);
    Node& nd = nodes[n];
    nd.sum_hess = (float)Hd;
    nd.base_weight = (float)(wgt * d.eta);
    nd.status = kLeaf;
    nd.leaf_value = (float)(wgt * d.eta);
    nd.split_cond = nd.leaf_value;
  }
}

// ------------------------------------------------------------------------------------------
// Partition planning + row partition (K18) + leaf margin update (K19)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_plan_part(GbdtDev d, int level) {
  __shared__ int32_t s_chunks[1024];
  __shared__ int32_t s_off[1025];
  const int first = (1 << level) - 1, nlev = 1 << level;
  for (int i = threadIdx.x; i < nlev; i += blockDim.x) {
    const Node& nd = d.nodes[first + i];
    const bool live = (nd.status == kSplit || nd.status == kLeaf) && nd.count > 0;
    s_chunks[i] = live ? (nd.count + d.chunk - 1) / d.chunk : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < nlev; ++i) { s_off[i] = acc; acc += s_chunks[i]; }
    d.counters[1] = acc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nlev; i += blockDim.x) {
    const Node& nd = d.nodes[first + i];
    for (int c = 0; c < s_chunks[i]; ++c) {
      WorkItem w;
      w.node = first + i;
      w.slot = 0;
      w.begin = nd.start + c * d.chunk;
      w.end = min(nd.start + nd.count, w.begin + d.chunk);
      d.items_p[s_off[i] + c] = w;
    }
  }
}

__global__ __launch_bounds__(256) void k_partition(GbdtDev d, int parity) {
  __shared__ int32_t s_cnt[2][4];
  __shared__ int32_t s_base[2];
  const int item = blockIdx.x;
  if (item >= d.counters[1]) return;
  const WorkItem w = d.items_p[item];
  const Node nd = d.nodes[w.node];
  const int32_t* cur = d.ridx[parity];
  if (nd.status == kLeaf) {
    const float v = nd.leaf_value;
    for (int i = w.begin + threadIdx.x; i < w.end; i += blockDim.x) d.margin[cur[i]] += v;
    return;
  }
  int32_t* nxt = d.ridx[parity ^ 1];
  const uint8_t* col = d.binsT + (int64_t)nd.feat * d.n;
  const int j = nd.bin;
  const bool dl = nd.default_left != 0;
  const int wv = wave_id(), nw = blockDim.x / kWave;
  int32_t* cursor = d.cursors + 2 * w.node;
  for (int base = w.begin; base < w.end; base += blockDim.x) {
    const int i = base + threadIdx.x;
    const bool valid = i < w.end;
    int r = 0;
    bool left = false;
    if (valid) {
      r = cur[i];
      const int b = col[r];
      left = (b == kMissingBin) ? dl : (b <= j);
    }
    const bool right = valid && !left;
    const uint64_t lm = __ballot(left), rm = __ballot(right);
    const int lo = mask_rank(lm), ro = mask_rank(rm);
    if (lane_id() == 0) { s_cnt[0][wv] = __popcll(lm); s_cnt[1][wv] = __popcll(rm); }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tl = 0, tr = 0;
      for (int k = 0; k < nw; ++k) { tl += s_cnt[0][k]; tr += s_cnt[1][k]; }
      s_base[0] = tl ? atomicAdd(cursor, tl) : 0;
      s_base[1] = tr ? atomicAdd(cursor + 1, tr) : 0;
    }
    __syncthreads();
    int wl = 0, wr = 0;
    for (int k = 0; k < wv; ++k) { wl += s_cnt[0][k]; wr += s_cnt[1][k]; }
    if (left) nxt[nd.start + s_base[0] + wl + lo] = r;
    if (right) nxt[nd.start + nd.count - 1 - (s_base[1] + wr + ro)] = r;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// Host-side trainer context
// ------------------------------------------------------------------------------------------
// RCCL all-reduce hook implemented in comm.cpp
extern "C" int cobalt_comm_allreduce_sum_i64(void* comm, int64_t* buf, int64_t count, hipStream_t stream);

struct GbdtCtx {
  GbdtConfig cfg;
  GbdtDev d;
  int max_nodes, pairs_max, items_cap;
  size_t lds_hist;
  void* alloc_list[16];
  int n_alloc;
};

static int dev_alloc(GbdtCtx* c, void** p, size_t bytes) {
  CK(hipMalloc(p, bytes < 16 ? 16 : bytes));
  c->alloc_list[c->n_alloc++] = *p;
  return 0;
}

COBALT_API int cobalt_gbdt_create(const GbdtConfig* cfg, void** out) {
  if (cfg->max_depth < 1 || cfg->max_depth > 10) return -1;
  if (cfg->chunk < 64 || cfg->chunk > 16384) return -2;
  if (cfg->row_stride % 4 != 0 || cfg->row_stride < cfg->n_feat) return -3;
  if (cfg->feat_tile % 4 != 0 || cfg->feat_tile <= 0 || cfg->feat_tile > 64) return -4;
  if (cfg->n_rows >= (int64_t)INT32_MAX) return -5;
  GbdtCtx* c = new GbdtCtx();
  memset(c, 0, sizeof(GbdtCtx));
  c->cfg = *cfg;
  const int F = cfg->n_feat;
  const int64_t N = cfg->n_rows;
  c->max_nodes = (1 << (cfg->max_depth + 1)) - 1;
  c->pairs_max = 1 << (cfg->max_depth - 1);
  c->items_cap = ceil_div(N, cfg->chunk) + (1 << cfg->max_depth) + 8;
  GbdtDev& d = c->d;
  d.n = N;
  d.row_offset = cfg->row_offset;
  d.F = F;
  d.stride = cfg->row_stride;
  d.max_depth = cfg->max_depth;
  d.max_nodes = c->max_nodes;
  d.chunk = cfg->chunk;
  d.feat_tile = cfg->feat_tile;
  d.slot_elems = (int64_t)(F + 1) * kMaxBins * 2;
  d.eta = cfg->eta;
  d.lambda_ = cfg->lambda_;
  d.alpha = cfg->alpha;
  d.gamma = cfg->gamma;
  d.mcw = cfg->min_child_weight;
  d.subsample = cfg->subsample;
  d.gscale = cfg->gscale;
  d.hscale = cfg->hscale;
  d.ginv = 1.0 / cfg->gscale;
  d.hinv = 1.0 / cfg->hscale;
  d.seed = cfg->seed;
  c->lds_hist = (size_t)cfg->feat_tile * kMaxBins * sizeof(uint64_t);
  int rc = 0;
  const size_t hist_bytes = (size_t)c->pairs_max * d.slot_elems * sizeof(int64_t);
  if ((rc = dev_alloc(c, (void**)&d.gpair, N * sizeof(uint64_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.ridx[0], N * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.ridx[1], N * sizeof(int32_t)))) return rc;
  for (int k = 0; k < 2; ++k) {
    if ((rc = dev_alloc(c, (void**)&d.hist_b[k], hist_bytes))) return rc;
    if ((rc = dev_alloc(c, (void**)&d.hist_s[k], hist_bytes))) return rc;
  }
  if ((rc = dev_alloc(c, (void**)&d.nodes, c->max_nodes * sizeof(Node)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.trees, (size_t)cfg->max_trees * c->max_nodes * sizeof(Node)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.items_h, c->items_cap * sizeof(WorkItem)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.items_p, c->items_cap * sizeof(WorkItem)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.counters, 16 * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.cursors, 2 * c->max_nodes * sizeof(int32_t)))) return rc;
  if (c->lds_hist > 64 * 1024) {
    CK(hipFuncSetAttribute((const void*)k_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_hist));
  }
  *out = c;
  return 0;
}

COBALT_API int cobalt_gbdt_set_data(void* h, const uint8_t* bins, const uint8_t* binsT, const float* cuts,
                                    const int32_t* nbins, const float* label, const float* weight,
                                    float* margin, const uint8_t* fmask) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  c->d.bins = bins;
  c->d.binsT = binsT;
  c->d.cuts = cuts;
  c->d.nbins = nbins;
  c->d.label = label;
  c->d.weight = weight;
  c->d.margin = margin;
  c->d.fmask = fmask;
  return 0;
}

// Enqueue `n_trees` boosting rounds starting at tree index `t0`. No host synchronisation.
COBALT_API int cobalt_gbdt_grow(void* h, int t0, int n_trees, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  GbdtDev& d = c->d;
  const int D = d.max_depth;
  const int grad_grid = std::min(ceil_div(d.n, 256), 256 * 16);
  const int ftiles = ceil_div(d.F, d.feat_tile);
  for (int t = t0; t < t0 + n_trees; ++t) {
    if (t >= c->cfg.max_trees) return -10;
    hipLaunchKernelGGL(k_init_tree, dim3(1), dim3(256), 0, stream, d);
    hipLaunchKernelGGL(k_grad, dim3(std::max(grad_grid, 1)), dim3(256), 0, stream, d, t);
    CK_LAUNCH();
    for (int level = 0; level <= D; ++level) {
      const int parity = level & 1;
      hipLaunchKernelGGL(k_plan_hist, dim3(1), dim3(256), 0, stream, d, level);
      if (level < D) {
        const int slots = level == 0 ? 1 : (1 << (level - 1));
        const size_t hbytes = (size_t)slots * d.slot_elems * sizeof(int64_t);
        CK(hipMemsetAsync(d.hist_b[parity], 0, hbytes, stream));
        const int ub = ceil_div(d.n, d.chunk) + (1 << level);
        hipLaunchKernelGGL(k_hist, dim3(ub, ftiles), dim3(256), c->lds_hist, stream, d, parity, t);
        CK_LAUNCH();
        if (c->cfg.comm && c->cfg.world_size > 1) {
          int rc = cobalt_comm_allreduce_sum_i64(c->cfg.comm, d.hist_b[parity], (int64_t)slots * d.slot_elems, stream);
          if (rc) return rc;
        }
      }
      hipLaunchKernelGGL(k_eval, dim3(1 << level), dim3(256), 0, stream, d, level, parity, t);
      hipLaunchKernelGGL(k_plan_part, dim3(1), dim3(256), 0, stream, d, level);
      const int ubp = ceil_div(d.n, d.chunk) + (1 << level);
      hipLaunchKernelGGL(k_partition, dim3(ubp), dim3(256), 0, stream, d, parity);
      CK_LAUNCH();
    }
    CK(hipMemcpyAsync(d.trees + (size_t)t * c->max_nodes, d.nodes, c->max_nodes * sizeof(Node),
                      hipMemcpyDeviceToDevice, stream));
  }
  return 0;
}

// Copy node records of trees [t0, t0+n) to host memory (blocking on `stream`).
COBALT_API int cobalt_gbdt_fetch_trees(void* h, int t0, int n, void* host_out, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  CK(hipMemcpyAsync(host_out, c->d.trees + (size_t)t0 * c->max_nodes, (size_t)n * c->max_nodes * sizeof(Node),
                    hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  return 0;
}

COBALT_API int cobalt_gbdt_max_nodes(void* h) { return static_cast<GbdtCtx*>(h)->max_nodes; }

COBALT_API int cobalt_gbdt_destroy(void* h) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (!c) return 0;
  for (int i = 0; i < c->n_alloc; ++i) (void)hipFree(c->alloc_list[i]);
  delete c;
  return 0;
}

COBALT_API int cobalt_bin_matrix(const float* X, int64_t n, int F, int64_t ldx, const float* cuts,
                                 const int32_t* nbins, uint8_t* bins, int stride, uint8_t* binsT,
                                 hipStream_t stream) {
  if (stride % 4 != 0 || stride < F) return -3;
  const int grid = std::max(1, std::min(ceil_div(n, 256), 256 * 8));
  const size_t lds = (size_t)F * kMaxBins * sizeof(float);
  if (lds <= 64 * 1024) {
    hipLaunchKernelGGL(k_bin<true>, dim3(grid), dim3(256), lds, stream, X, n, F, ldx, cuts, nbins, bins, stride, binsT);
  } else {
    hipLaunchKernelGGL(k_bin<false>, dim3(grid), dim3(256), 0, stream, X, n, F, ldx, cuts, nbins, bins, stride, binsT);
  }
  CK_LAUNCH();
  return 0;
}
