// Histogram gradient-boosted-tree trainer for gfx950 (MI355X).
//
// Replaces the XGBoost 3.0 `hist` updater the reference drives through
// `XGBClassifier.fit` (reference: src/model_train_test/model_tree_train_test.py:111-164,
// notebooks/04_model_training.ipynb:1877-2016).
//
// Design (MI355X-first, not a translation of XGBoost's CPU/CUDA code):
//  * Features are pre-quantised to uint8 bins (<= 255 real bins + code 255 = missing; 256 real bins
//    for a feature without missing values, see hist_add_rec32), stored twice:
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
#include "comm.h"
#include "ipc_device.h"
#include "knobs.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
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

struct CandRec {  // a group's best split candidate (k_eval<true> -> k_eval_finish)
  double gain;
  int32_t key;
  float cut;
  int64_t gl, hl;
};

__device__ __forceinline__ bool cand_better(const Cand& a, const Cand& b) {
  return a.gain > b.gain || (a.gain == b.gain && a.key < b.key);
}

template <int CTRL, int ROWM>
__device__ __forceinline__ void best_step(double& g, int& k) {
  const double og = __longlong_as_double(dpp64<CTRL, ROWM>(__double_as_longlong(g), __double_as_longlong(-INFINITY)));
  const int ok = dpp32<CTRL, ROWM>(k, 0x7fffffff);
  if (og > g || (og == g && ok < k)) { g = og; k = ok; }
}

// The wave's best candidate (max under cand_better), returned in every lane: a DPP max-scan of
// (gain, key) leaves the winner in lane 63, a ballot finds the lane it came from (keys are unique
// per lane), and that lane's gl / hl / cut are read back -- the same result as a shuffle butterfly
// over the whole Cand, at VALU instead of LDS latency per step.
__device__ __forceinline__ void wave_best(Cand& best, float& cut) {
  double g = best.gain;
  int k = best.key;
  best_step<kDppRowShr1, 0xf>(g, k);
  best_step<kDppRowShr2, 0xf>(g, k);
  best_step<kDppRowShr4, 0xf>(g, k);
  best_step<kDppRowShr8, 0xf>(g, k);
  best_step<kDppRowBcast15, 0xa>(g, k);
  best_step<kDppRowBcast31, 0xc>(g, k);
  const double wg = __longlong_as_double(readlane64(__double_as_longlong(g), kWave - 1));
  const int wk = readlane32(k, kWave - 1);
  const uint64_t m = __ballot(best.key == wk && best.gain == wg);
  const int src = m ? __ffsll((unsigned long long)m) - 1 : 0;
  best.gain = wg;
  best.key = wk;
  best.gl = readlane64(best.gl, src);
  best.hl = readlane64(best.hl, src);
  cut = __int_as_float(readlane32(__float_as_int(cut), src));
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
  double gscale, hscale; // g_q = floor(g * gscale + u), h_q = floor(h * hscale + u) (quantize_gh)
  float base_margin;
  int32_t world_size;
  uint64_t seed;
  void* comm;            // native RCCL communicator (cobalt_comm_*) or nullptr
  int32_t grad_bits;     // quantised (g, h) magnitude bits: 17 (packed u64 LDS cells) or 25 (wide cells)
  int32_t reserved0;
};

struct GbdtDev {
  // inputs
  uint8_t* bins;          // [N][stride] row records: bins[0..F) | pad | packed (g,h) u64 at goff
  const uint8_t* binsT;   // [F][N]
  const float* cuts;      // [F][256]
  const int32_t* nbins;   // [F]
  const float* label;     // [N]
  const float* weight;    // [N] sample weight incl. scale_pos_weight for positives
  float* margin;          // [N]
  const uint8_t* fmask;   // [max_trees][F] colsample_bytree masks
  // workspace
  int32_t goff;           // byte offset of the packed gradient pair inside a row record
  int32_t* ridx[2];       // [N] x2
  int64_t* hist_b[2];     // [pairs][F+1][256][2]
  int64_t* hist_s[2];     // [nodes of the level][F+1][256][2]: every node's full histogram (k_eval), by position
  Node* nodes;            // [max_nodes] the tree being grown (one of nodes_buf, alternating per tree)
  Node* prev_nodes;       // [max_nodes] the previous tree (the other buffer), applied + archived by k_grad
  Node* nodes_buf[2];
  Node* trees;            // [max_trees][max_nodes]
  WorkItem* items_h;      // histogram work list (written by the histogram blocks for the reduce pass)
  int32_t* counters;      // [0] = #hist items of the current level
  int32_t* cursors;       // [max_nodes][2]
  int2* layout;           // [F] histogram LDS layout: x = cell offset within tile, y = log2(copies)
  int32_t* tile_entries;  // [n_tiles] LDS cells per feature tile
  uint64_t* slab;         // [items][F][256] packed per-item partial histograms
  int64_t* slab_tot;      // [items][2] per-item (G, H) totals
  int32_t ablate;         // timing-only ablation (COBALT_HIST_ABLATE): 1 no LDS atomics, 2 no flush, 3 no rows,
                          // 4 plan only (k_hist); 12 partition without the cursor claims; root pass: 20 no exp,
                          // 21 no LDS atomics, 22 no previous-tree walk
  int32_t dp;             // data parallel (a native communicator is attached)
  int32_t by_hess;        // build k_eval's (global) hessian choice: under data parallelism (every rank builds the
                          // same child, so the collective sums it as is); one GPU builds the locally smaller one
  int32_t hist_pair;      // k_hist gathers each record with a lane pair (hist_rows_pair); COBALT_HIST_PAIR
  CandRec* cand;          // [2^(max_depth-1)][64] per-group split candidates (grouped evaluation)
  int64_t n;
  int64_t ldt;            // row pitch of binsT (= the rows the context was created for; n <= ldt)
  int64_t row_offset;
  int32_t F, stride, max_depth, max_nodes, chunk, feat_tile;
  int64_t slot_elems;     // (ncells + 1) * 2: compact histogram slot (int64 g, h per cell + node total)
  int32_t* hoff;          // [F+1] compact cell offset of feature f (cells = its nbins); hoff[F] = ncells
  int32_t ncells;         // sum of nbins: real bins only, so low-cardinality features cost 2-3 cells
  double eta, lambda_, alpha, gamma, mcw, subsample, gscale, hscale, ginv, hinv;
  uint64_t seed;
  uint64_t* stamps;       // COBALT_STAMPS diagnostics: [launch][kStampBlocks][2] block {start, end} in 10 ns
                          // ticks; nullptr in normal runs and in unsampled trees
  int32_t seq;            // launch index into `stamps` (set by the host before every launch)
  // data-parallel IPC exchange (appended: the single-GPU kernels' argument layout is unchanged)
  int64_t* hist_red;      // k_hist_reduce destination: nullptr = hist_b[parity]; the IPC group's send slot
                          // under IPC data parallelism (the exchange then writes the global sums to hist_b)
  int64_t* zero_red;      // the next reduce destination, zeroed by k_grad* (root) / k_partition (next level):
                          // nullptr = hist_b; the IPC group's next send slot under the fused exchange
  const IpcFusedView* ipcv;  // fused IPC exchange: the group's device views (per slot parity) ...
  unsigned ipc_epoch;        // ... and this level's epoch (k_eval only; 0 = hist_b already holds global sums)
  // write-through (sc1) stores of data the NEXT launch reads from other XCDs (COBALT_WT, bit 0: the
  // per-item histogram slabs, bit 1: the partition's row ids, bit 2: the root pass's (g, h) record
  // halves): the lines leave L2 as they are written
  // instead of at the kernel-end write-back that the dependent launch waits for
  int32_t wt;
  // binary labels held in the row records (cobalt_gbdt_set_binary_labels): byte 23 of a 32-byte record
  // (F <= 23) is the 0/1 label and the weight is `spw` for positives, 1 otherwise (no sample weights),
  // so the gradient pass reads neither the label nor the weight array
  int32_t ylab;
  float spw;
  // label bit (F <= 20 with ylab): the 0/1 label is bit 31 of the record's h word (word 6, bytes 24-27; h_q <
  // 2^26 never reaches it -- the histogram passes mask it off) instead of byte 23, which frees record word 5
  // (bytes 20-23) for the row's margin: mrec = the fused root pass keeps every row's fp32 margin THERE
  // (copied in at the start of a grow call, out at its end), so it reads and writes the record it streams
  // anyway instead of a separate margin array -- 64 instead of 72 bytes per row per tree
  int32_t lab31;
  int32_t mrec;
  // In-flight replica check (data parallel only; dig == nullptr on one GPU). Every node decision a
  // tree finalises adds a 32-bit hash to dig[tree & 1] (eval_finalize). At level 0 of the next tree
  // the reduce writes the previous tree's sum into an extra int64 cell right after the root slot
  // (element slot_elems), the level's collective sums it over the ranks with the histograms, and the
  // evaluation checks sum == world x own: a rank that grew a different tree (a stale peer read, a
  // corrupted exchange) makes the check fail on EVERY rank within one tree. The failure goes to the
  // mapped host word err_host (2 = replica divergence), which the host polls while a segment runs.
  int64_t* dig;
  int32_t dig_slot;   // tree & 1 of the tree being grown
  int32_t dig_check;  // the previous tree was grown by this context (its digest is comparable)
  int32_t world;
  int32_t corrupt;    // fault injection (COBALT_FAULT_CORRUPT_RANK): perturb this tree's root totals
  unsigned* err_host;
  // fused evaluation + partition pass (k_eval_part): ep_chunk = the level's item size (0: the level has
  // no fused pass), ep_zero = active nodes without local rows get an empty item (DP)
  int32_t ep_chunk, ep_zero;
  // node ownership (fused IPC exchange): from level own_level on, a node is evaluated only by the rank
  // owning its level-own_level ancestor; the others copy its decision (-1: every rank evaluates all)
  int32_t own_level;
  // k_eval_part<.., 2>: per-node decision granules {launch tag, decision} (decision_word)
  uint64_t* dec;
  // wide gradients (grad_bits 25): |g_q| < 2^25, h_q <= 2^25, and the LDS histograms hold a cell as two
  // int64 words (g, h) -- ds_add_u64 each -- instead of one packed u64; slabs likewise (see kWide)
  int32_t wide;
};


// 32-bit hash of one finalised node decision (position, status, split feature / bin / default
// direction, threshold or leaf value): summed over a tree's nodes into GbdtDev::dig.
// (G, H: the node's global sums -- under node ownership the other ranks copy a node's record, so a
// rank whose sums went wrong at a level every rank evaluates must still show in the digest)
__device__ __forceinline__ uint32_t node_hash(int n, int status, int feat, int bin, int dl, float cond, int64_t G,
                                              int64_t H) {
  uint64_t x = ((uint64_t)(uint32_t)n << 32) ^ ((uint64_t)(uint32_t)status << 40) ^ ((uint64_t)(uint32_t)feat << 44) ^
               ((uint64_t)(uint32_t)(bin & 0x3FF) << 52) ^ ((uint64_t)(uint32_t)dl << 62) ^ __float_as_uint(cond);
  x ^= (uint64_t)G * 0x9E3779B97F4A7C15ull;
  x ^= ((uint64_t)H << 29) | ((uint64_t)H >> 35);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// Level 0 of a tree, after the collective: `sum` is the digest cell summed over the ranks.
__device__ __forceinline__ void digest_check(const GbdtDev& d, int64_t sum) {
  const int64_t own = d.dig_check ? d.dig[d.dig_slot ^ 1] : 0;
  if (sum != (int64_t)d.world * own) __hip_atomic_store(d.err_host, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Final replica check of a grow call (data parallel): the in-flight check compares tree t's digest at
// tree t + 1's root exchange, which never comes for the LAST tree of a call -- so that tree's digest gets
// an all-reduce of its own (k_dig_stage -> the communicator's int64 sum of dig[2] -> k_dig_cmp) before the
// host fetches or checkpoints the trees. dig[2] is the staging cell.
__global__ void k_dig_stage(int64_t* dig, int slot) {
  if (threadIdx.x == 0) dig[2] = dig[slot];
}
__global__ void k_dig_cmp(const int64_t* dig, int slot, int world, unsigned* err_host) {
  if (threadIdx.x == 0 && dig[2] != (int64_t)world * dig[slot])
    __hip_atomic_store(err_host, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Store of a value the next launch reads: plain, or write-through (agent-scope relaxed atomic store =
// global_store ... sc1) when `wt`.
template <typename T>
__device__ __forceinline__ void store_wt(T* p, T v, bool wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// In-kernel timing (diagnostic switch COBALT_STAMPS, off by default): the block's first thread
// stores when the block started and each wave's lane 0 raises the block's end time, into a slot of
// the block's own ([launch][kStampBlocks][2] ticks of the 100 MHz clock), so the diagnostic adds no
// contended atomics. Only a few sampled trees are stamped (the host clears d.stamps otherwise).
constexpr int kStampBlocks = 4096;
constexpr int kStampSlot = 8;  // per block: start, end, probes 1..6 (thread 0)
struct BlockStamp {
  unsigned long long* p;
  __device__ __forceinline__ explicit BlockStamp(const GbdtDev& d) : p(nullptr) {
    const int b = blockIdx.x + blockIdx.y * gridDim.x;
    if (d.stamps && b < kStampBlocks) {
      p = reinterpret_cast<unsigned long long*>(d.stamps) + ((int64_t)d.seq * kStampBlocks + b) * kStampSlot;
      if (threadIdx.x == 0) p[0] = __builtin_amdgcn_s_memrealtime();
    }
  }
  // thread 0's time at probe point k (1..6) of the kernel body
  __device__ __forceinline__ void probe(int k) {
    if (p && threadIdx.x == 0) p[1 + k] = __builtin_amdgcn_s_memrealtime();
  }
  // the LAST wave's time at probe point k (every wave's lane 0 contributes)
  __device__ __forceinline__ void probe_max(int k) {
    if (p && (threadIdx.x & (kWave - 1)) == 0) atomicMax(p + 1 + k, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
  __device__ __forceinline__ ~BlockStamp() {
    if (p && (threadIdx.x & (kWave - 1)) == 0) atomicMax(p + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
};

// ------------------------------------------------------------------------------------------
// Binning: X fp32 [N][F] (row-major, NaN = missing) -> uint8 bins (row-major + feature-major)
// bin(x) = #cuts <= x (upper_bound), clamped to nbins-1; NaN -> 255.
// ------------------------------------------------------------------------------------------
template <bool CUTS_IN_LDS>
__global__ __launch_bounds__(256) void k_bin(const float* __restrict__ X, int64_t n, int F, int64_t ldx,
                                             const float* __restrict__ cuts, const int32_t* __restrict__ nbins,
                                             uint8_t* __restrict__ bins, int stride,
                                             uint8_t* __restrict__ binsT, int64_t ldt) {
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
    const int fw = (F + 3) & ~3;  // bytes written per row (the record tail holds the gradient pair)
    for (int f = 0; f < fw; ++f) {
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
        binsT[(int64_t)f * ldt + row] = (uint8_t)b;
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
// Gradient fixed point (models/gbdt_host.py gradients_host is the oracle): |g| <= w_max and
// h <= w_max / 4 are scaled to 17 bits and rounded UNBIASED, q = floor(x * scale + u) with u ~ U[0,1)
// drawn from a per-(tree, global row) hash -- E[q] = x * scale, so small hessians are not flushed
// to 0 and rounding errors of histogram sums average out instead of accumulating a bias. The draw is
// deterministic (same trees on every device and rank count). Bounds: a <= 16384-row histogram block
// sums to |sum g| < 2^31 and sum h <= 2^31, so the packed u64 (signed g high, h low) never carries.
// Wide gradients (GbdtConfig::grad_bits 25): 25-bit magnitudes, summed in int64 cells (a 16384-row block
// < 2^39; 10M rows < 2^49, exact in the host oracle's float64 sums too).
constexpr int64_t kGClip = (1 << 17) - 1, kHClip = 1 << 17;
constexpr int64_t kGClipW = (1 << 25) - 1, kHClipW = 1 << 25;
constexpr uint64_t kDitherSalt = 0xD1B54A32D192ED03ull;

__device__ __forceinline__ uint64_t tree_key_of(uint64_t seed, int tree) {
  return splitmix64(seed ^ (0xA5A5A5A5ull + (uint64_t)tree * 0x632BE59BD9B4E019ull));
}

__device__ __forceinline__ void quantize_gh(double g, double h, double gscale, double hscale, uint64_t dkey,
                                            int64_t grow, int64_t& gq, int64_t& hq, bool wide = false) {
  const uint64_t r = splitmix64(dkey ^ (uint64_t)grow);
  const double ug = (double)(uint32_t)(r >> 32) * (1.0 / 4294967296.0);
  const double uh = (double)(uint32_t)r * (1.0 / 4294967296.0);
  gq = (int64_t)floor(g * gscale + ug);
  hq = (int64_t)floor(h * hscale + uh);
  const int64_t gc = wide ? kGClipW : kGClip, hc = wide ? kHClipW : kHClip;
  gq = gq > gc ? gc : (gq < -gc ? -gc : gq);
  hq = hq > hc ? hc : (hq < 0 ? 0 : hq);
}
// Reset the node table of a new tree (root active with all local rows) and the per-node counters.
__device__ void init_tree_block(const GbdtDev& d) {
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

// Staged split word: feat | (bin + 1) << 16 (9 bits: the split bin j may be -1, a missing-only split
// that sends every non-missing row right) | default_left << 25 | is_split << 26.
constexpr uint32_t kMetaSplit = 1u << 26;
__device__ __forceinline__ uint32_t node_meta(const Node& nd) {
  return (uint32_t)(nd.feat & 0xFFFF) | ((uint32_t)((nd.bin + 1) & 0x1FF) << 16) |
         ((uint32_t)(nd.default_left & 1) << 25) | (nd.status == kSplit ? kMetaSplit : 0u);
}
__device__ __forceinline__ bool meta_left(uint32_t m, uint32_t b) {
  return (b == kMissingBin) ? ((m >> 25) & 1u) : (b < ((m >> 16) & 0x1FFu));
}

// Stage tree `t` (heap-ordered node records) into LDS as {meta, leaf value}.
__device__ __forceinline__ void stage_tree(const GbdtDev& d, const Node* tr, uint32_t* s_meta, float* s_leaf) {
  for (int i = threadIdx.x; i < d.max_nodes; i += blockDim.x) {
    const Node nd = tr[i];
    s_meta[i] = node_meta(nd);
    s_leaf[i] = nd.leaf_value;
  }
}

// Branch-free walk of a staged tree over a 32-byte record held in registers (the fused root pass's
// prediction-cache update). A node is two 16-byte LDS words:
//   {s0, s1, s2, leaf}: v_perm_b32 selectors that pull the split feature's byte out of record words
//     (0, 1), (2, 3) or (4, 5) -- the two pairs that do not hold it select zero bytes (0x0c) -- so
//     b = perm(w1, w0, s0) | perm(w3, w2, s1) | perm(w5, w4, s2) is the bin with no per-lane word select;
//   {K, V, cb, cbr}: the row goes to cb (left) iff K - b >= V (unsigned), else to cbr. With K = 255 - dl
//     and V = 255 - j - dl this is "bin <= j, the missing code 255 -> default_left" in one compare
//     (dl = 1: b = 255 wraps K - b past every V). A leaf has zero selectors, K = V = 0 and cb = cbr = itself,
//     so the walk runs a uniform max_depth steps and a row that reached its leaf stays there.
// 8 VALU ops + two ds_read_b128 per level, no exec-mask branches: the `while (split)` walk over a
// `q == 0 ? .x : q == 1 ? ...` word chain compiled to ~60 instructions of nested s_and_saveexec branches
// per level, the root pass's largest VALU cost after the fp64 gradients.
constexpr uint32_t kPermZero = 0x0c0c0c0cu;
constexpr int kWalkNodeBytes = 32;

__device__ __forceinline__ void stage_walk(const GbdtDev& d, const Node* tr, uint4* s_walk) {
  for (int i = threadIdx.x; i < d.max_nodes; i += blockDim.x) {
    const Node nd = tr[i];
    uint4 a = make_uint4(kPermZero, kPermZero, kPermZero, __float_as_uint(nd.leaf_value));
    uint4 c = make_uint4(0u, 0u, (uint32_t)i, (uint32_t)i);
    if (nd.status == kSplit) {
      const uint32_t f = (uint32_t)nd.feat, dl = (uint32_t)(nd.default_left & 1);
      const uint32_t sel = 0x0c0c0c00u | (f & 7u);
      a.x = (f >> 3) == 0 ? sel : kPermZero;
      a.y = (f >> 3) == 1 ? sel : kPermZero;
      a.z = (f >> 3) == 2 ? sel : kPermZero;
      c = make_uint4(255u - dl, (uint32_t)(255 - nd.bin) - dl, (uint32_t)(2 * i + 1), (uint32_t)(2 * i + 2));
    }
    s_walk[2 * i] = a;
    s_walk[2 * i + 1] = c;
  }
}

// Leaf values of U rows' records (ra = record words 0-3, rb = words 4-7), walked together so the rows'
// dependent LDS reads overlap.
template <int U>
__device__ __forceinline__ void walk_leaves(const uint4* s_walk, int depth, const uint4 (&ra)[U], const uint4 (&rb)[U],
                                            float (&leaf)[U]) {
  uint32_t n[U];
#pragma unroll
  for (int u = 0; u < U; ++u) n[u] = 0;
  for (int s = 0; s < depth; ++s) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 w = s_walk[2 * n[u]];
      const uint4 c = s_walk[2 * n[u] + 1];
      const uint32_t b = __builtin_amdgcn_perm(ra[u].y, ra[u].x, w.x) | __builtin_amdgcn_perm(ra[u].w, ra[u].z, w.y) |
                         __builtin_amdgcn_perm(rb[u].y, rb[u].x, w.z);
      n[u] = (c.x - b >= c.y) ? c.z : c.w;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) leaf[u] = __uint_as_float(s_walk[2 * n[u]].w);
}

// Leaf of row i in a staged tree (the partition step's routing), walked over the FEATURE-MAJOR bins:
// row i's bin of feature f is binsT[f][i], so the lanes of a wave (consecutive rows) read consecutive
// bytes of each column they visit -- a coalesced load per level
// while the lanes share a node, instead of one record line per lane (wide records are 48-128 bytes).
__device__ __forceinline__ float tree_leaf_T(const GbdtDev& d, int64_t i, const uint32_t* s_meta,
                                             const float* s_leaf) {
  int n = 0;
  uint32_t m = s_meta[0];
  while (m & kMetaSplit) {
    const int f = m & 0xFFFF;
    const uint32_t b = d.binsT[(int64_t)f * d.ldt + i];
    const bool left = meta_left(m, b);
    n = 2 * n + (left ? 1 : 2);
    m = s_meta[n];
  }
  return s_leaf[n];
}

// Gradient kernel. When `apply_tree >= 0` it first adds that tree's leaf value to every row's margin
// (the prediction-cache update, done as a coalesced traversal over row-major bins instead of a
// scatter over the leaves' row lists), then computes binary:logistic g/h in fp64, applies row
// subsampling, quantises and packs them into the row record (the root level reads rows in
// identity order, so ridx needs no reset).
__global__ __launch_bounds__(256) void k_grad(GbdtDev d, int tree, int apply_tree) {
  BlockStamp stamp_(d);
  extern __shared__ uint32_t s_tree[];
  {  // zero the root histogram slot
    int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[0]);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < d.slot_elems / 2;
         e += (int64_t)gridDim.x * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
  }
  uint32_t* s_meta = s_tree;
  float* s_leaf = reinterpret_cast<float*>(s_tree + d.max_nodes);
  if (apply_tree >= 0) {
    stage_tree(d, d.prev_nodes, s_meta, s_leaf);
    // archive the previous tree (its node table is the other buffer, untouched by this tree)
    const int4* src = reinterpret_cast<const int4*>(d.prev_nodes);
    int4* dst = reinterpret_cast<int4*>(d.trees + (int64_t)apply_tree * d.max_nodes);
    const int nv = d.max_nodes * (int)(sizeof(Node) / sizeof(int4));
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nv; e += gridDim.x * blockDim.x) dst[e] = src[e];
    __syncthreads();
  }
  if (blockIdx.x == 0) init_tree_block(d);  // the new tree's node table (no other block reads it)
  const uint64_t tree_key = tree_key_of(d.seed, tree);
  const uint64_t dkey = splitmix64(tree_key ^ kDitherSalt);
  const bool rec32 = d.stride == 32 && d.F <= 24;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float mf = d.margin[i];
    uint4 ra = make_uint4(0, 0, 0, 0), rb = make_uint4(0, 0, 0, 0);
    uint4* rec = reinterpret_cast<uint4*>(d.bins + i * 32);
    if (rec32) {
      ra = rec[0];
      rb = rec[1];
    }
    if (apply_tree >= 0) {
      if (rec32) {
        // walk the previous tree with the record held in registers
        int n = 0;
        uint32_t m = s_meta[0];
        while (m & kMetaSplit) {
          const int f = m & 0xFFFF, q = f >> 2;
          const uint32_t word = q == 0 ? ra.x : q == 1 ? ra.y : q == 2 ? ra.z : q == 3 ? ra.w : q == 4 ? rb.x : rb.y;
          const uint32_t b = (word >> (8 * (f & 3))) & 0xffu;
          const bool left = meta_left(m, b);
          n = 2 * n + (left ? 1 : 2);
          m = s_meta[n];
        }
        mf += s_leaf[n];
      } else {
        mf += tree_leaf_T(d, i, s_meta, s_leaf);
      }
      d.margin[i] = mf;
    }
    const double mm = (double)mf;
    const double p = 1.0 / (1.0 + exp(-mm));
    const uint32_t lbit = rb.z & 0x80000000u;
    const float yf = d.ylab ? (d.lab31 ? (lbit ? 1.0f : 0.0f) : (float)(rb.y >> 24)) : d.label[i];
    const double y = (double)yf;
    const double w = d.ylab ? (double)(yf != 0.0f ? d.spw : 1.0f) : (double)d.weight[i];
    double g = (p - y) * w;
    double h = fmax(p * (1.0 - p), 1e-16) * w;
    if (d.subsample < 1.0) {
      const uint64_t hsh = splitmix64(tree_key ^ (uint64_t)(d.row_offset + i));
      if (!(uniform01(hsh) < d.subsample)) { g = 0.0; h = 0.0; }
    }
    int64_t gq, hq;
    quantize_gh(g, h, d.gscale, d.hscale, dkey, d.row_offset + i, gq, hq, d.wide != 0);
    if (rec32) {
      rb.z = (uint32_t)hq | (d.lab31 ? lbit : 0u);
      rb.w = (uint32_t)(int32_t)gq;
      rec[1] = rb;
    } else {
      *reinterpret_cast<uint64_t*>(d.bins + i * d.stride + d.goff) =
          ((uint64_t)(uint32_t)(int32_t)gq << 32) | (uint64_t)(uint32_t)hq;
    }
  }
}

// F <= 20 (GbdtDev::lab31): the label as bit 31 of the h word (word 6; the root pass rewrites h under it)
__global__ __launch_bounds__(256) void k_put_label31(uint8_t* bins, const float* label, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint32_t*>(bins + i * 32)[6] = label[i] != 0.0f ? 0x80000000u : 0u;
}
// GbdtDev::mrec: the margins into record word 5 at the start of a grow call, and back at its end
__global__ __launch_bounds__(256) void k_margin_in(uint8_t* bins, const float* margin, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<float*>(bins + i * 32)[5] = margin[i];
}
// ... together with the label bit at a fit's first grow call (words 5 and 6 of a record, one pass instead of
// two over the records; the root pass rewrites h under the bit)
__global__ __launch_bounds__(256) void k_margin_label_in(uint8_t* bins, const float* margin, const float* label,
                                                         int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t* w = reinterpret_cast<uint32_t*>(bins + i * 32);
    w[5] = (uint32_t)__float_as_int(margin[i]);
    w[6] = label[i] != 0.0f ? 0x80000000u : 0u;
  }
}
__global__ __launch_bounds__(256) void k_margin_out(const uint8_t* bins, float* margin, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    margin[i] = reinterpret_cast<const float*>(bins + i * 32)[5];
}

// Add tree `t`'s leaf values to the margins (used after the last boosting round).
__global__ __launch_bounds__(256) void k_apply_tree(GbdtDev d, int t) {
  BlockStamp stamp_(d);
  extern __shared__ uint32_t s_tree[];
  uint32_t* s_meta = s_tree;
  float* s_leaf = reinterpret_cast<float*>(s_tree + d.max_nodes);
  stage_tree(d, d.trees + (int64_t)t * d.max_nodes, s_meta, s_leaf);
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.n;
       i += (int64_t)gridDim.x * blockDim.x)
    d.margin[i] += tree_leaf_T(d, i, s_meta, s_leaf);
}

// Start of a tree grown from precomputed gradients (external-memory path): node-table reset and the
// root histogram slot zeroed (k_hist_reduce accumulates into it; k_grad does this on the normal path).
__global__ __launch_bounds__(256) void k_tree_begin(GbdtDev d) {
  BlockStamp stamp_(d);
  int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[0]);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < d.slot_elems / 2;
       e += (int64_t)gridDim.x * blockDim.x)
    zp[e] = make_int4(0, 0, 0, 0);
  if (blockIdx.x == 0) init_tree_block(d);
}

// ------------------------------------------------------------------------------------------
// External-memory training (BASELINE.json config "100M-row out-of-core GBDT with
// host-DRAM spill"). The quantised row records live in host memory as pages; per tree every page
// streams through k_ooc_page, which
//   * applies the previous tree to the rows' margins (margins / labels / weights stay on the device),
//   * computes binary:logistic g, h (fp64, as k_grad) and ghat = sqrt(g^2 + h^2),
//   * keeps a minimal-variance sample (MVS -- the sampler of XGBoost's gradient_based external
//     memory mode): row i with probability p_i = min(1, ghat_i / mu), its pair reweighted by 1/p_i
//     (unbiased histograms; |g/p|, h/p <= mu, so the fixed-point scales hold when mu <= w_max),
//   * compacts kept rows into the trainer's row records + feature-major bins (one wave-aggregated
//     claim per wave; the order is irrelevant because every histogram sum is an exact integer),
//   * counts ghat in kOocBins log-spaced bins (binary exponent x 16 mantissa steps, exact integer
//     counts -> the host derives the next mu deterministically, models/external.py).
// The in-core trainer then grows the tree on the sample (cobalt_gbdt_grow_sampled).
// ------------------------------------------------------------------------------------------
constexpr int kOocBins = 2048;

__device__ __forceinline__ int ooc_bin(double v) {
  if (!(v > 0.0)) return 0;
  int e;
  const double f = frexp(v, &e);  // v = f * 2^e, f in [0.5, 1)
  const int b = (e + 64) * 16 + (int)floor((f - 0.5) * 32.0);
  return b < 1 ? 1 : (b >= kOocBins ? kOocBins - 1 : b);
}

// `ps` = page row stride in bytes: 32 (full row records) or the compact spill format, the F bins
// rounded up to 4 bytes (20 B for the 20 deployed features: 37% less PCIe traffic per tree -- the
// per-tree page stream is bound by the H2D copy).
__global__ __launch_bounds__(256) void k_ooc_page(const uint8_t* __restrict__ page, int ps, int64_t n, int64_t r0, int F,
                                                  const Node* __restrict__ prev, int max_nodes,
                                                  float* __restrict__ margin, const float* __restrict__ label,
                                                  const float* __restrict__ weight, uint64_t key, int64_t row_offset,
                                                  double mu, double gscale, double hscale, uint8_t* __restrict__ srec,
                                                  uint8_t* __restrict__ sbinsT, int64_t cap,
                                                  unsigned long long* __restrict__ counter,
                                                  unsigned int* __restrict__ hist) {
  __shared__ uint32_t s_meta[2047];
  __shared__ float s_leaf[2047];
  __shared__ unsigned int s_h[kOocBins];
  for (int i = threadIdx.x; i < kOocBins; i += blockDim.x) s_h[i] = 0u;
  if (prev != nullptr)
    for (int i = threadIdx.x; i < max_nodes; i += blockDim.x) {
      const Node nd = prev[i];
      s_meta[i] = node_meta(nd);
      s_leaf[i] = nd.leaf_value;
    }
  __syncthreads();
  const int lane = lane_id();
  // wave-uniform loop (ballots below): every lane of a wave iterates the same bases
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const bool in = i < n;
    bool keep = false;
    uint4 ra = make_uint4(0, 0, 0, 0), rb = make_uint4(0, 0, 0, 0);
    if (in) {
      if (ps == 32) {
        const uint4* rec = reinterpret_cast<const uint4*>(page + i * 32);
        ra = rec[0];
        rb = rec[1];
        rb.z = rb.w = 0u;  // (g, h) slot: rewritten below for kept rows
      } else {  // compact page: ps / 4 bin words, the rest of the record is zero padding
        const uint32_t* rw = reinterpret_cast<const uint32_t*>(page + i * ps);
        const int nw = ps >> 2;
        ra.x = rw[0];
        if (nw > 1) ra.y = rw[1];
        if (nw > 2) ra.z = rw[2];
        if (nw > 3) ra.w = rw[3];
        if (nw > 4) rb.x = rw[4];
        if (nw > 5) rb.y = rw[5];
      }
      float mf = margin[r0 + i];
      if (prev != nullptr) {
        int nx = 0;
        uint32_t m = s_meta[0];
        while (m & kMetaSplit) {
          const int f = m & 0xFFFF, q = f >> 2;
          const uint32_t word = q == 0 ? ra.x : q == 1 ? ra.y : q == 2 ? ra.z : q == 3 ? ra.w : q == 4 ? rb.x : rb.y;
          const uint32_t b = (word >> (8 * (f & 3))) & 0xffu;
          const bool left = meta_left(m, b);
          nx = 2 * nx + (left ? 1 : 2);
          m = s_meta[nx];
        }
        mf += s_leaf[nx];
        margin[r0 + i] = mf;
      }
      const double p = 1.0 / (1.0 + exp(-(double)mf));
      const double y = (double)label[r0 + i], w = (double)weight[r0 + i];
      const double g = (p - y) * w;
      const double h = fmax(p * (1.0 - p), 1e-16) * w;
      const double gh = sqrt(g * g + h * h);
      atomicAdd(&s_h[ooc_bin(gh)], 1u);
      if (mu > 0.0) {
        const double pk = gh >= mu ? 1.0 : gh / mu;
        keep = uniform01(splitmix64(key ^ (uint64_t)(row_offset + r0 + i))) < pk;
        if (keep) {
          int64_t gq = (int64_t)rint(g / pk * gscale), hq = (int64_t)rint(h / pk * hscale);
          gq = gq > 65536 ? 65536 : (gq < -65536 ? -65536 : gq);
          hq = hq > 65536 ? 65536 : (hq < 0 ? 0 : hq);
          rb.z = (uint32_t)hq;
          rb.w = (uint32_t)(int32_t)gq;
        }
      }
    }
    const uint64_t km = __ballot(keep);
    if (km) {
      const int leader = __ffsll((unsigned long long)km) - 1;
      unsigned long long b0 = 0;
      if (lane == leader) b0 = atomicAdd(counter, (unsigned long long)__popcll(km));
      b0 = (unsigned long long)readlane64((int64_t)b0, leader);
      if (keep) {
        const int64_t slot = (int64_t)b0 + mask_rank(km);
        if (slot < cap) {
          uint4* dst = reinterpret_cast<uint4*>(srec + slot * 32);
          dst[0] = ra;
          dst[1] = rb;
          for (int f = 0; f < F; ++f) {
            const int q = f >> 2;
            const uint32_t word = q == 0 ? ra.x : q == 1 ? ra.y : q == 2 ? ra.z : q == 3 ? ra.w : q == 4 ? rb.x : rb.y;
            sbinsT[(int64_t)f * cap + slot] = (uint8_t)((word >> (8 * (f & 3))) & 0xffu);
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kOocBins; i += blockDim.x)
    if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

COBALT_API int cobalt_ooc_page(const uint8_t* page, int page_stride, int64_t n, int64_t r0, int F, const void* prev,
                               int max_nodes,
                               float* margin, const float* label, const float* weight, uint64_t key,
                               int64_t row_offset, double mu, double gscale, double hscale, uint8_t* srec,
                               uint8_t* sbinsT, int64_t cap, unsigned long long* counter, unsigned int* hist,
                               hipStream_t stream) {
  if (F < 1 || F > 24 || max_nodes > 2047 || n < 0) return -3;  // 32-byte records only
  if (page_stride != 32 && (page_stride % 4 != 0 || page_stride < F || page_stride > 24)) return -3;
  if (n == 0) return 0;
  const int grid = std::max(1, std::min(ceil_div(n, 256), 256 * 8));
  hipLaunchKernelGGL(k_ooc_page, dim3(grid), dim3(256), 0, stream, page, page_stride, n, r0, F,
                     static_cast<const Node*>(prev),
                     max_nodes, margin, label, weight, key, row_offset, mu, gscale, hscale, srec, sbinsT, cap, counter,
                     hist);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_ooc_bins() { return kOocBins; }

// ------------------------------------------------------------------------------------------
// Self-planning work lists. A pass over the rows of several nodes is cut into items of at most
// `chunk` rows; item i of the pass belongs to the entry (node) e with off[e] <= i < off[e+1], where
// off is the exclusive scan of ceil(rows(e) / chunk). Every block of the pass computes this plan for
// itself with wave 0 (a 64-wide scan over the <= 2^level entries, looping for deeper trees) from the
// node table written by the previous kernels -- no separate planning kernel and no kernel boundary.
struct PlanEntry {
  int node, slot, start, count;
};
struct PlanOut {
  int node, slot, begin, end, total;
};

// kZeroItem: an entry with no rows still gets one (empty) item -- the data-parallel evaluation +
// partition pass must finalise every active node on every rank, also where this rank holds none of
// its rows.
template <bool kZeroItem = false, class EntryFn>
__device__ PlanOut block_plan(int n_ent, int chunk, int item, EntryFn entry, int* s_out) {
  if (wave_id() == 0) {
    const int lane = lane_id();
    if (lane == 0) s_out[0] = -1;
    int carry = 0;
    for (int base = 0; base < n_ent; base += kWave) {
      const int e = base + lane;
      PlanEntry en{-1, 0, 0, 0};
      if (e < n_ent) en = entry(e);
      const int nch = en.node < 0 ? 0
                      : (en.count > 0 ? (en.count + chunk - 1) / chunk : (kZeroItem ? 1 : 0));
      const int incl = wave_incl_scan(nch) + carry;
      const int excl = incl - nch;
      if (nch > 0 && item >= excl && item < incl) {
        const int b = en.start + (item - excl) * chunk;
        s_out[0] = en.node;
        s_out[1] = en.slot;
        s_out[2] = b;
        s_out[3] = min(en.start + en.count, b + chunk);
      }
      carry = readlane32(incl, kWave - 1);
    }
    if (lane == 0) s_out[4] = carry;
  }
  __syncthreads();
  return PlanOut{s_out[0], s_out[1], s_out[2], s_out[3], s_out[4]};
}

// Histogram pass of `level`: entries are the node pairs; the child histogrammed from rows is the one
// with fewer LOCAL rows (the partition cursors) on one GPU, the one with the smaller GLOBAL hessian
// (k_eval's choice, the same on every rank) under data parallelism; the sibling comes by exact
// subtraction.
__device__ __forceinline__ PlanEntry hist_entry(const GbdtDev& d, int level, int p) {
  if (level == 0) return PlanEntry{0, 0, 0, (int)d.n};
  const int q = (1 << (level - 1)) - 1 + p;
  const Node& par = d.nodes[q];
  // every load first, selected after: one round trip (a load behind the status test would wait)
  const int st = par.status, pstart = par.start, pcount = par.count;
  const int2 cc = *reinterpret_cast<const int2*>(d.cursors + 2 * q);  // one 8-byte load: both counts
  const int lc = cc.x, rc = cc.y;
  const int lbuild = d.nodes[2 * q + 1].build;
  // selects, not an early return: hipcc sinks loads into the branch that uses them
  const bool ok = st == kSplit;
  const bool left_small = d.by_hess ? lbuild != 0 : lc <= rc;
  PlanEntry en;
  en.node = ok ? (left_small ? 2 * q + 1 : 2 * q + 2) : -1;
  en.slot = p;
  en.start = ok ? (left_small ? pstart : pstart + lc) : 0;
  en.count = ok ? (left_small ? lc : pcount - lc) : 0;
  return en;
}

// Block (0, 0) of the histogram pass publishes the level's node ranges / build flags for the
// evaluation and partition kernels, resets the level's partition counters and the item count.
// `build` is the child whose GLOBAL histogram sits in hist_b after the reduce (+ all-reduce): the
// locally smaller one on one GPU; under data parallelism k_eval's hessian choice stays.
__device__ void publish_level(const GbdtDev& d, int level, int total) {
  if (threadIdx.x == 0) d.counters[0] = total;
  if (level == 0) return;
  const int npairs = 1 << (level - 1);
  for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
    const int q = npairs - 1 + p;
    const Node& par = d.nodes[q];
    if (par.status != kSplit) continue;
    const int L = 2 * q + 1, R = 2 * q + 2;
    const int lc = d.cursors[2 * q];
    const bool left_small = lc <= d.cursors[2 * q + 1];
    d.nodes[L].start = par.start;
    d.nodes[L].count = lc;
    d.nodes[R].start = par.start + lc;
    d.nodes[R].count = par.count - lc;
    if (!d.by_hess) {
      d.nodes[L].build = left_small ? 1 : 0;
      d.nodes[R].build = left_small ? 0 : 1;
    }
  }
  const int first = (1 << level) - 1, nlev = 1 << level;
  for (int i = threadIdx.x; i < nlev; i += blockDim.x) {
    d.cursors[2 * (first + i)] = 0;
    d.cursors[2 * (first + i) + 1] = 0;
  }
}

// LDS histogram helpers shared by k_hist and k_grad_hist (32-byte record fast path).
struct HistLanes {
  uint64_t fbits;                 // colsample mask of the tile's features
  uint32_t trash;                 // per-lane trash cell (masked / padding features of the 32-byte path)
  uint32_t lane;
  // 32-byte record path (hist_add_rec32): per feature fl of the tile, fm = nbins | (copy shift + 3) << 16
  // (uniform -> SGPRs) and lb8 = this lane's byte offset of its copy of the feature's bin 0 (VGPRs)
  uint32_t fm[24];
  uint32_t lb8[24];
};

// Per-tile feature state for the LDS histogram lanes. Lane k loads feature f0 + k's colsample bit, copy
// shift and bin count (one round trip, instead of 2 x ft dependent scalar loads per thread -- ~10 us per
// block for a 32-feature tile); one wave stages them in LDS (hist_meta_store) and every lane reads them
// back as uniform values (hist_lanes_finish). Called by every thread of a block.
// The loads are split from the ballots (hist_lanes_load / hist_lanes_finish) so a kernel can issue
// them together with its other independent loads (work plan, flush offsets): one round trip for all.
struct HistLaneRaw {
  bool on;
  int sh, nb;
};

__device__ __forceinline__ HistLaneRaw hist_lanes_load(const GbdtDev& d, int tree, int f0, int ft) {
  const int lane = lane_id();
  const bool in = lane < ft;
  const int f = f0 + (in ? lane : 0);
  HistLaneRaw r;
  // unconditional loads (f is clamped), masked after: both in one round trip
  const uint8_t fmv = d.fmask[(int64_t)tree * d.F + f];
  const int ly0 = d.layout[f].y;
  const int nb0 = d.nbins[f];
  r.on = in && fmv != 0;
  const int ly = in ? ly0 : 0;
  r.sh = ly & 7;
  r.nb = in ? min(max(nb0, 1), kMaxBins) : 1;
  return r;
}

// Per-feature histogram metadata of lane fl's feature: nbins | (copy shift + cs) << 16 (cs = log2 of the
// LDS cell bytes: 3, or 4 for wide cells); a feature past the tile or masked out by colsample gets
// nbins 0 (it adds into a trash cell).
__device__ __forceinline__ uint32_t hist_meta(const HistLaneRaw& raw, uint32_t cs = 3) {
  return raw.on ? ((uint32_t)raw.nb | ((uint32_t)raw.sh + cs) << 16) : (cs << 16);
}

// Stage the metadata of the tile's features in LDS (s_fm[64], lane fl = feature fl) from ONE wave: the
// row loops read it back with a uniform LDS load + readfirstlane, which is correct under any exec
// mask (a readlane of a lane that is inactive where the compiler places it would read a stale VGPR).
// A caller's later barrier publishes it. Using the block's last wave keeps wave 0 -- the work planner
// -- from waiting on the metadata loads before it issues the plan's.
__device__ __forceinline__ void hist_meta_store(const HistLaneRaw& raw, uint32_t* s_fm, uint32_t cs = 3) {
  if (wave_id() == (int)(blockDim.x / kWave) - 1) s_fm[lane_id()] = hist_meta(raw, cs);
}

__device__ __forceinline__ uint32_t hist_meta_of(const uint32_t* s_fm, int fl) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)s_fm[fl]);
}

__device__ __forceinline__ HistLanes hist_lanes_finish(const HistLaneRaw& raw, int ft, const uint32_t* s_fm,
                                                       uint32_t cs = 3) {
  HistLanes hl;
  hl.lane = lane_id();
  hl.fbits = __ballot(raw.on);
  hl.trash = (uint32_t)(ft * kMaxBins) + hl.lane;
#pragma unroll
  for (int fl = 0; fl < 24; ++fl) {
    const uint32_t m = hist_meta_of(s_fm, fl);
    hl.fm[fl] = m;
    hl.lb8[fl] = (m & 0xffffu) ? ((uint32_t)(fl * kMaxBins) + (hl.lane & ((1u << (((m >> 16) & 15u) - cs)) - 1u))) << cs
                               : hl.trash << cs;
  }
  return hl;
}


// Add one 32-byte record (bins in a.xyzw / b.xy, packed (g, h) in b.wz) to the LDS histogram.
// Per feature: byte extract, clamp, shift-add, ds_add_u64 (3 VALU ops per atomic). The missing code
// 255 clamps to cell nbins, which the layout keeps inside the feature's 256 cells and the flush never
// reads (a 256-bin feature has no missing values: its code 255 is a real bin); features masked out by
// colsample, and the tile's padding up to FT4 (= features rounded up to 4), add into a trash cell.
// kWide: 16-byte cells {int64 g, int64 h}, two ds_add_u64 per (row, feature).
template <int FT4, bool kWide = false>
__device__ __forceinline__ void hist_add_rec32(uint64_t* s_hist, const HistLanes& hl, const uint4& a,
                                               const uint4& b) {
  static_assert(FT4 % 4 == 0 && FT4 > 0 && FT4 <= 24, "32-byte records hold <= 24 bins");
  const uint32_t hz = b.z & 0x7FFFFFFFu;  // (bit 31: the label, lab31 records)
  const uint64_t gp = ((uint64_t)b.w << 32) | hz;
  const uint64_t gw = (uint64_t)(int64_t)(int32_t)b.w, hw = (uint64_t)hz;
  char* base = reinterpret_cast<char*>(s_hist);
#pragma unroll
  for (int fl = 0; fl < FT4; ++fl) {
    {
      const uint32_t m = hl.fm[fl];
      const int q = fl >> 2;
      const uint32_t word = q == 0 ? a.x : q == 1 ? a.y : q == 2 ? a.z : q == 3 ? a.w : q == 4 ? b.x : b.y;
      const uint32_t bb = (word >> (8 * (fl & 3))) & 0xffu;
      const uint32_t off = hl.lb8[fl] + (min(bb, m & 0xffffu) << ((m >> 16) & 15u));
      if constexpr (kWide) {
        atomicAdd(reinterpret_cast<unsigned long long*>(base + off), (unsigned long long)gw);
        atomicAdd(reinterpret_cast<unsigned long long*>(base + off + 8), (unsigned long long)hw);
      } else {
        atomicAdd(reinterpret_cast<unsigned long long*>(base + off), (unsigned long long)gp);
      }
    }
  }
}

// Per-item partial histogram -> compact slab (+ the item's (G, H) totals when tot_block). The tile's
// compact cell offsets and copy shifts are staged in LDS once, and each cell finds its feature by a
// binary search there (a linear scan over global hoff per cell cost ~60 us per launch on the
// 106-feature RFE fits, where every block flushes 4 x 8k cells).
constexpr int kMaxFeatTile = 64;

// Flush metadata of a tile, staged into LDS by the kernel prologue (its loads share the round trip of
// the work plan; the prologue's barrier publishes it): s_fo = compact cell offset of each tile feature
// (+ the end), s_fs = its log2(copies), or -1 when masked out for this tree.
struct FlushMeta {
  int fo, fs;
};

__device__ __forceinline__ FlushMeta flush_meta_load(const GbdtDev& d, int tree, int f0, int ft) {
  FlushMeta m{0, -1};
  const int t = threadIdx.x;
  // unconditional loads at clamped indices, selected after (one round trip, no chained waits)
  const int tc = min(t, ft), tf = min(t, ft - 1);
  const int fo = d.hoff[f0 + tc];
  const uint8_t fmv = d.fmask[(int64_t)tree * d.F + f0 + tf];
  const int ly = d.layout[f0 + tf].y;
  if (t <= ft) m.fo = fo;
  if (t < ft) m.fs = fmv != 0 ? (ly & 7) : -1;
  return m;
}

__device__ __forceinline__ void flush_meta_store(const FlushMeta& m, int ft, int* s_fo, int* s_fs) {
  const int t = threadIdx.x;
  if (t <= ft) s_fo[t] = m.fo;
  if (t < ft) s_fs[t] = m.fs;
}

template <bool kWide = false>
__device__ void hist_flush(const GbdtDev& d, const uint64_t* s_hist, const HistLanes& hl, int item, int f0, int ft,
                           int64_t tg, int64_t th, bool tot_block, int64_t (*s_tot)[16], const int* s_fo,
                           const int* s_fs) {
  // Each cell finds its feature by a binary search over the LDS-staged offsets and sums its copies.
  // (A wave-segmented form -- every thread reads one LDS entry and xor-shuffles the copies together --
  // measured slower at 1M rows: 20.3 vs 18.7 us per k_hist, the 64-bit shuffles of the 64-copy binary
  // features go through ds_bpermute and cost more LDS cycles than the reads they replace.)
  const int c0 = s_fo[0], c1 = s_fo[ft];
  constexpr int kW = kWide ? 2 : 1;  // u64 words per cell
  uint64_t* slab = d.slab + (int64_t)item * d.ncells * kW;
  for (int e = c0 + threadIdx.x; e < c1; e += blockDim.x) {
    int lo = 0, hi = ft - 1;  // largest fl with s_fo[fl] <= e
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_fo[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int sh = s_fs[lo];
    uint64_t v = 0, v2 = 0;
    if (sh >= 0) {
      const uint64_t* cell = s_hist + (lo * kMaxBins + ((e - s_fo[lo]) << sh)) * kW;
      for (int c = 0; c < (1 << sh); ++c) {
        v += cell[c * kW];
        if (kWide) v2 += cell[c * kW + 1];
      }
    }
    store_wt(slab + (int64_t)e * kW, v, (d.wt & 1) != 0);
    if (kWide) store_wt(slab + (int64_t)e * kW + 1, v2, (d.wt & 1) != 0);
  }
  if (tot_block) {
    tg = wave_sum(tg);
    th = wave_sum(th);
    if (hl.lane == 0) { s_tot[0][wave_id()] = tg; s_tot[1][wave_id()] = th; }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t G = 0, H = 0;
      for (int k = 0; k < (int)(blockDim.x / kWave); ++k) { G += s_tot[0][k]; H += s_tot[1][k]; }
      store_wt(d.slab_tot + 2 * item, G, (d.wt & 1) != 0);
      store_wt(d.slab_tot + 2 * item + 1, H, (d.wt & 1) != 0);
    }
  }
}

// Gradients fused with the ROOT histogram (32-byte records, one feature tile): the gradient pass
// already streams every record, so the level-0 LDS histogram is accumulated from the registers
// holding the freshly quantised (g, h) and the bins -- the separate root histogram pass (a full
// 32 B/row re-read) disappears. Block b = root work item b: rows [b*chunk, (b+1)*chunk).
// Also: previous-tree margin update + archive and node-table init, as k_grad.
// kWide: wide gradients (16-byte LDS cells {g, h}, 25-bit quantisation).
template <int U, int FT4, bool kWide>
__device__ __forceinline__ void grad_hist_body(const GbdtDev& d, int tree, int apply_tree, int chunk) {
  constexpr int kW = kWide ? 2 : 1;            // u64 words per LDS cell
  constexpr uint32_t kCs = kWide ? 4u : 3u;    // log2 of the cell bytes
  BlockStamp stamp_(d);
  extern __shared__ uint64_t s_dyn[];
  __shared__ int64_t s_tot[2][16];
  __shared__ int s_fo[kMaxFeatTile + 1], s_fs[kMaxFeatTile];
  __shared__ uint32_t s_fm[kWave];
  const int ft = d.F;
  const int entries = ft * kMaxBins + kWave;  // one tile: tile_entries[0] == F * 256
  // independent metadata loads first (they share the round trip of the previous tree's node table)
  const HistLaneRaw lraw = hist_lanes_load(d, tree, 0, ft);
  const FlushMeta fmeta = flush_meta_load(d, tree, 0, ft);
  uint64_t* s_hist = s_dyn;
  uint4* s_walk = reinterpret_cast<uint4*>(s_dyn + entries * kW);  // the previous tree (stage_walk)
  {  // zero the root histogram slot (k_hist_reduce accumulates into it)
    int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[0]);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < d.slot_elems / 2;
         e += (int64_t)gridDim.x * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
  }
  if (apply_tree >= 0) {
    stage_walk(d, d.prev_nodes, s_walk);
    const int4* src = reinterpret_cast<const int4*>(d.prev_nodes);
    int4* dst = reinterpret_cast<int4*>(d.trees + (int64_t)apply_tree * d.max_nodes);
    const int nv = d.max_nodes * (int)(sizeof(Node) / sizeof(int4));
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nv; e += gridDim.x * blockDim.x) dst[e] = src[e];
  }
  if (blockIdx.x == 0) {
    init_tree_block(d);
    if (threadIdx.x == 0) d.counters[0] = gridDim.x;
  }
  for (int i = threadIdx.x; i < entries * kW; i += blockDim.x) s_hist[i] = 0ull;
  flush_meta_store(fmeta, ft, s_fo, s_fs);
  hist_meta_store(lraw, s_fm, kCs);
  __syncthreads();
  stamp_.probe(1);
  const int item = blockIdx.x;
  const int64_t begin = (int64_t)item * chunk, end = min(d.n, begin + chunk);
  if (threadIdx.x == 0) {
    WorkItem w;
    w.node = 0; w.slot = 0; w.begin = (int32_t)begin; w.end = (int32_t)end;
    d.items_h[item] = w;
  }
  const HistLanes hl = hist_lanes_finish(lraw, ft, s_fm, kCs);
  const uint64_t tree_key = tree_key_of(d.seed, tree);
  const uint64_t dkey = splitmix64(tree_key ^ kDitherSalt);
  int64_t tg = 0, th = 0;
  const int B = blockDim.x;
  for (int64_t i0 = begin + threadIdx.x; i0 < end; i0 += U * B) {
    uint4 ra[U], rb[U];
    float mf[U], yl[U], wt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * B;
      const int64_t ii = i < end ? i : begin;
      const uint4* rec = reinterpret_cast<const uint4*>(d.bins + ii * 32);
      ra[u] = rec[0];
      rb[u] = rec[1];
      mf[u] = d.mrec ? 0.0f : d.margin[ii];
      yl[u] = 0.0f;
      wt[u] = 0.0f;
      if (!d.ylab) {
        yl[u] = d.label[ii];
        wt[u] = d.weight[ii];
      }
    }
    // walk the previous tree with the U records held in registers (branch-free, all rows together; rows
    // past the item walk their clamped copy and are dropped below)
    float lf[U];
    const bool walk = apply_tree >= 0 && d.ablate != 22;
    if (walk) walk_leaves<U>(s_walk, d.max_depth, ra, rb, lf);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * B;
      if (i >= end) continue;
      if (d.mrec) mf[u] = __int_as_float((int)rb[u].y);  // the margin in record word 5
      if (walk) {
        mf[u] += lf[u];
        if (!d.mrec) d.margin[i] = mf[u];
      }
      const double mm = (double)mf[u];
      const double p = d.ablate == 20 ? 0.5 + 0.01 * mm : 1.0 / (1.0 + exp(-mm));  // (20: timing-only, no exp)
      const uint32_t lbit = rb[u].z & 0x80000000u;  // (lab31: the label bit rides in the h word)
      if (d.ylab) {
        yl[u] = d.lab31 ? (lbit ? 1.0f : 0.0f) : (float)(rb[u].y >> 24);
        wt[u] = yl[u] != 0.0f ? d.spw : 1.0f;
      }
      const double y = (double)yl[u];
      const double w = (double)wt[u];
      double g = (p - y) * w;
      double h = fmax(p * (1.0 - p), 1e-16) * w;
      if (d.subsample < 1.0) {
        const uint64_t hsh = splitmix64(tree_key ^ (uint64_t)(d.row_offset + i));
        if (!(uniform01(hsh) < d.subsample)) { g = 0.0; h = 0.0; }
      }
      int64_t gq, hq;
      quantize_gh(g, h, d.gscale, d.hscale, dkey, d.row_offset + i, gq, hq, kWide);
      tg += gq;
      th += hq;
      rb[u].y = d.mrec ? (uint32_t)__float_as_int(mf[u]) : rb[u].y;
      rb[u].z = (uint32_t)hq | (d.lab31 ? lbit : 0u);
      rb[u].w = (uint32_t)(int32_t)gq;
      // (g, h) [+ the margin]: one plain 16-byte store when the margin rides along (write-through of the 16
      // bytes measured slower: 10M 247.5 vs 237.8 ms); else write-through of the 8-byte (g, h) (COBALT_WT bit
      // 2): no dirty record lines left for the kernel-end write-back
      if (!d.mrec && (d.wt & 4))
        store_wt(reinterpret_cast<uint64_t*>(d.bins + i * 32) + 3, ((uint64_t)rb[u].w << 32) | rb[u].z, true);
      else
        reinterpret_cast<uint4*>(d.bins + i * 32)[1] = rb[u];
      if (d.ablate != 21) hist_add_rec32<FT4, kWide>(s_hist, hl, ra[u], rb[u]);  // (21: timing-only, no LDS atomics)
    }
  }
  __syncthreads();
  stamp_.probe(2);
  hist_flush<kWide>(d, s_hist, hl, item, 0, ft, tg, th, true, s_tot, s_fo, s_fs);
}

// U rows in flight per thread; 2 per CU of 512 threads at 95 VGPRs (no waves-per-EU bound: capping U = 2
// at 80 VGPRs spills, 276.5 vs 269.7 ms per 10M fit)
// (wide cells: 1024-thread blocks -- the 16-byte-cell tile holds a CU to one block, so twice the waves)
template <int U, int FT4, bool kWide = false>
__global__ __launch_bounds__(kWide ? 1024 : 512) void k_grad_hist(GbdtDev d, int tree, int apply_tree, int chunk) {
  grad_hist_body<U, FT4, kWide>(d, tree, apply_tree, chunk);
}


// Lane-pair record gathers for the deep histogram levels (16 < F <= 24 features): lanes 2p and 2p+1
// take the SAME row and load its two 16-byte halves in ONE instruction, so a wave-instruction fetches
// 32 whole 32-byte records (32 line requests) instead of 64 half records (64 requests, each record's
// line requested twice). The pair then splits the record's features: lane 0 of the pair histograms
// features [0, FH), lane 1 features [FH, FT4) (FH = FT4 / 2). Lane 0 holds record words 0-3, lane 1
// words 4-7; each lane reads the partner's words z, w by one DPP quad swap -- lane 0 gets (g, h)
// (words 6, 7), lane 1 gets words 2, 3 -- which covers both feature ranges for FH in {8, 10, 12}.
constexpr int kDppQuadSwap = 0xB1;  // quad_perm [1, 0, 3, 2]: lane i <- lane i ^ 1

template <int FT4>
__device__ __forceinline__ void hist_rows_pair(const GbdtDev& d, uint64_t* s_hist, const HistLanes& hl,
                                               const int32_t* rix, bool identity, int begin, int end,
                                               int64_t& tg, int64_t& th) {
  static_assert(FT4 >= 16 && FT4 <= 24, "pair split covers 16 < F <= 24");
  constexpr int FH = FT4 / 2, Q = FH / 4, S = FH % 4;  // lane 1's first byte: word Q, byte S
  constexpr int NW = (FH + 3) / 4;                     // words of bins per lane
  constexpr int U = 4;  // rows in flight per pair (6: 257.3 ms per 10M fit, 4: 252.0; 8 spills at 80 VGPRs;
                        // round 4, same box: 5 at 78 VGPRs 241.0 vs 235.7)
  const int h = (int)(hl.lane & 1u);
  const int P = (int)(blockDim.x >> 1), pslot = (int)(threadIdx.x >> 1);
  // this lane's features: metadata and copy bases (VGPRs, selected once)
  uint32_t fmv[FH], lbv[FH];
#pragma unroll
  for (int k = 0; k < FH; ++k) {
    const uint32_t m = h ? hl.fm[FH + k] : hl.fm[k];
    const uint32_t fl = (uint32_t)(k + h * FH);
    fmv[k] = m;
    lbv[k] = (m & 0xffffu) ? (fl * kMaxBins + (hl.lane & ((1u << (((m >> 16) & 15u) - 3)) - 1u))) * 8u : hl.trash * 8u;
  }
  char* base = reinterpret_cast<char*>(s_hist);
  const int ilast = max(end - 1, begin);
  int rn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = begin + pslot + u * P;
    const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
    rn[u] = i < end ? rv : -1;
  }
  for (int i0 = begin + pslot; i0 < end; i0 += U * P) {
    int r[U];
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = rn[u];
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = reinterpret_cast<const uint4*>(d.bins + (int64_t)(r[u] >= 0 ? r[u] : r[0]) * 32)[h];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + U * P + u * P;
      const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
      rn[u] = i < end ? rv : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t pz = (uint32_t)dpp32<kDppQuadSwap>((int)x[u].z, 0);
      const uint32_t pw = (uint32_t)dpp32<kDppQuadSwap>((int)x[u].w, 0);
      // record words as this lane sees them: lane 0 owns 0-3, lane 1 owns 4-7 and has the partner's 2, 3
      auto w1 = [&](int wi) -> uint32_t {  // lane 1's view, words 2..5
        return wi == 2 ? pz : wi == 3 ? pw : wi == 4 ? x[u].x : x[u].y;
      };
      uint32_t v[NW];
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const uint32_t own = j == 0 ? x[u].x : j == 1 ? x[u].y : x[u].z;  // lane 0: words 0..2
        const uint32_t l1 = S ? __builtin_amdgcn_alignbyte(w1(Q + j + 1), w1(Q + j), S) : w1(Q + j);
        v[j] = h ? l1 : own;
      }
      const bool ok = r[u] >= 0;
      const uint32_t hq = ok ? ((h ? x[u].z : pz) & 0x7FFFFFFFu) : 0u, gq = ok ? (h ? x[u].w : pw) : 0u;
      const uint64_t gp = ((uint64_t)gq << 32) | hq;
      if (h == 0) {
        tg += (int64_t)(int32_t)gq;
        th += (int64_t)hq;
      }
#pragma unroll
      for (int k = 0; k < FH; ++k) {
        const uint32_t bb = (v[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint32_t off = lbv[k] + (min(bb, fmv[k] & 0xffffu) << ((fmv[k] >> 16) & 15u));
        atomicAdd(reinterpret_cast<unsigned long long*>(base + off), (unsigned long long)gp);
      }
    }
  }
}

constexpr int kHistThreads = 512;  // (1024-thread blocks measured 3-8% slower)
constexpr int kHistThreadsWide = 1024;  // wide cells: one block per CU by LDS, so the larger block

// FT4 > 0: 32-byte records with one tile of <= FT4 features (FT4 = F rounded up to 4); 0: generic rows.
// (6 waves per SIMD = the 3 blocks per CU that the LDS tile allows: keeps the kernel within 80 VGPRs)
// PAIR: the lane-pair record gathers of hist_rows_pair (FT4 >= 16).
// kWide: wide gradients (16-byte LDS cells; the one-lane-per-row 32-byte path only).
// (wide cells: one block per CU by LDS -- a 1024-thread block, 4 waves per SIMD)
template <int FT4, bool PAIR, bool kWide = false>
__global__ __launch_bounds__(kWide ? kHistThreadsWide : kHistThreads) __attribute__((amdgpu_waves_per_eu(kWide ? 4 : 6))) void k_hist(
    GbdtDev d, int parity, int tree, int level, int chunk) {
  static_assert(!kWide || (FT4 > 0 && !PAIR), "wide cells: 32-byte records, one lane per row");
  constexpr int kW = kWide ? 2 : 1;
  constexpr uint32_t kCs = kWide ? 4u : 3u;
  BlockStamp stamp_(d);
  extern __shared__ uint64_t s_hist[];
  __shared__ int64_t s_tot[2][16];
  __shared__ int s_plan[5];
  __shared__ int s_fo[kMaxFeatTile + 1], s_fs[kMaxFeatTile];
  const int item = blockIdx.x;
  const int n_ent = level == 0 ? 1 : (1 << (level - 1));
  const int f0 = blockIdx.y * d.feat_tile;  // < F: gridDim.y = ceil(F / feat_tile)
  const int ft = min(d.feat_tile, d.F - f0);
  // Prologue: the tile's lane setup and flush offsets do not depend on the node table, so their loads
  // go out with the plan's (one round trip instead of three), and the LDS histogram is zeroed while
  // they are in flight (block_plan's barrier publishes both).
  const HistLaneRaw lraw = hist_lanes_load(d, tree, f0, ft);
  const FlushMeta fmeta = flush_meta_load(d, tree, f0, ft);
  const int entries = ft * kMaxBins + kWave;  // tile_entries[y] == ft * 256, + per-lane trash cells
  for (int i = threadIdx.x; i < entries * kW; i += blockDim.x) s_hist[i] = 0ull;
  __shared__ uint32_t s_fm[kWave];
  hist_meta_store(lraw, s_fm, kCs);  // (last wave; block_plan's barrier publishes it)
  const PlanOut pl = block_plan(n_ent, chunk, item, [&](int p) { return hist_entry(d, level, p); },
                                s_plan);
  // after the plan (storing first would wait for the metadata before the plan's loads go out); the
  // barrier after the row loop publishes it to the flush
  flush_meta_store(fmeta, ft, s_fo, s_fs);
  stamp_.probe(1);
  if (item == 0 && blockIdx.y == 0) publish_level(d, level, pl.total);
  if (pl.node < 0) return;
  WorkItem w;
  w.node = pl.node;
  w.slot = pl.slot;
  w.begin = pl.begin;
  w.end = pl.end;
  if (blockIdx.y == 0 && threadIdx.x == 0) d.items_h[item] = w;
  if (d.ablate == 4) return;  // timing-only: plan + publish only
  const HistLanes hl = hist_lanes_finish(lraw, ft, s_fm, kCs);
  const uint64_t fbits = hl.fbits;
  stamp_.probe(2);

  const int32_t* rix = d.ridx[parity];
  const bool identity = parity == 0 && w.node == 0;  // root level: ridx is the identity
  if (d.ablate == 3) w.end = w.begin;  // timing-only: no rows
  const int lane = lane_id();
  int64_t tg = 0, th = 0;
  const int B = blockDim.x;
  constexpr int U = 4;  // rows in flight per thread
  if constexpr (PAIR) {
    hist_rows_pair<FT4>(d, s_hist, hl, rix, identity, w.begin, w.end, tg, th);
  } else if constexpr (FT4 > 0) {
    // 32-byte records (bins | pad | (g,h)): one pair of 16-byte loads per row
    // software pipeline: the row ids of iteration k+1 are loaded while iteration k's records are in
    // flight, so each iteration waits on one memory round trip instead of two (ridx -> record)
    // row-id loads are unconditional at a clamped index and masked after (a load guarded per row
    // sits in its own exec branch, and the waits around it cover every load in flight)
    const int ilast = max(w.end - 1, w.begin);
    int rn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = w.begin + threadIdx.x + u * B;
      const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
      rn[u] = i < w.end ? rv : -1;
    }
    for (int i0 = w.begin + threadIdx.x; i0 < w.end; i0 += U * B) {
      int r[U];
      uint4 a[U], b2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = rn[u];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint4* rec = reinterpret_cast<const uint4*>(d.bins + (int64_t)(r[u] >= 0 ? r[u] : r[0]) * 32);
        a[u] = rec[0];
        b2[u] = rec[1];
        asm volatile("" : "+v"(b2[u].y));  // keep two 16-byte loads per row when bins 20-23 are unused
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + U * B + u * B;
        const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
        rn[u] = i < w.end ? rv : -1;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r[u] < 0) { b2[u].z = 0u; b2[u].w = 0u; }
        tg += (int64_t)(int32_t)b2[u].w;
        th += (int64_t)(b2[u].z & 0x7FFFFFFFu);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) hist_add_rec32<FT4, kWide>(s_hist, hl, a[u], b2[u]);
    }
  } else {
    // Generic records (F > 24: the RFE stage's wide fits, or F <= 8): the tile's <= 32 bins are bytes
    // [f0, f0 + 32) of the record (f0 % 16 == 0, pitch a multiple of 16) -> two 16-byte loads, plus the
    // packed (g, h) pair at goff, issued together for U rows, with the next rows' ids prefetched one
    // iteration ahead (the 32-byte path's pipeline): one memory round trip per iteration instead of a
    // dependent ridx -> (g, h) -> chunk-by-chunk chain. Tile metadata is uniform (SGPRs); a masked or
    // padding feature is skipped by a scalar branch (no trash-cell atomics).
    constexpr int UW = 2;  // rows in flight per thread (4 needs more VGPRs than 6 waves / SIMD allow)
    const bool lo_ok = f0 + 16 <= d.stride, hi_ok = f0 + 32 <= d.stride;  // block-uniform
    uint32_t fmv[32];
#pragma unroll
    for (int fl = 0; fl < 32; ++fl) fmv[fl] = fl < ft ? hist_meta_of(s_fm, fl) : (3u << 16);
    const int ilast = max(w.end - 1, w.begin);
    int rn[UW];
#pragma unroll
    for (int u = 0; u < UW; ++u) {
      const int i = w.begin + threadIdx.x + u * B;
      const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
      rn[u] = i < w.end ? rv : -1;
    }
    char* base = reinterpret_cast<char*>(s_hist);
    for (int i0 = w.begin + threadIdx.x; i0 < w.end; i0 += UW * B) {
      int r[UW];
      uint4 a[UW], b[UW];
      uint64_t gp[UW];
#pragma unroll
      for (int u = 0; u < UW; ++u) r[u] = rn[u];
#pragma unroll
      for (int u = 0; u < UW; ++u) {
        const uint8_t* rec = d.bins + (int64_t)(r[u] >= 0 ? r[u] : r[0]) * d.stride;
        const uint4* t = reinterpret_cast<const uint4*>(rec + f0);
        a[u] = lo_ok ? t[0] : make_uint4(0, 0, 0, 0);
        b[u] = hi_ok ? t[1] : make_uint4(0, 0, 0, 0);
        gp[u] = *reinterpret_cast<const uint64_t*>(rec + d.goff) & ~0x80000000ull;  // (bit 31 of h: lab31)
      }
#pragma unroll
      for (int u = 0; u < UW; ++u) {
        const int i = i0 + UW * B + u * B;
        const int rv = identity ? min(i, ilast) : rix[min(i, ilast)];
        rn[u] = i < w.end ? rv : -1;
      }
#pragma unroll
      for (int u = 0; u < UW; ++u) {
        if (r[u] < 0) gp[u] = 0ull;
        tg += (int64_t)(int32_t)(uint32_t)(gp[u] >> 32);
        th += (int64_t)(uint32_t)gp[u];
      }
#pragma unroll
      for (int fl = 0; fl < 32; ++fl) {
        const uint32_t m = fmv[fl];
        const uint32_t nb = m & 0xffffu, sh3 = (m >> 16) & 15u;
        if (nb == 0) continue;  // uniform: masked by colsample, or past the tile
        // as hist_add_rec32: the missing code clamps to the feature's unread cell nbins
        const uint32_t lb8 = ((uint32_t)(fl * kMaxBins) + (lane & ((1u << (sh3 - 3)) - 1u))) * 8u;
        const int q = fl >> 2;
#pragma unroll
        for (int u = 0; u < UW; ++u) {
          const uint32_t word = q == 0 ? a[u].x : q == 1 ? a[u].y : q == 2 ? a[u].z : q == 3 ? a[u].w
                              : q == 4 ? b[u].x : q == 5 ? b[u].y : q == 6 ? b[u].z : b[u].w;
          const uint32_t bb = (word >> (8 * (fl & 3))) & 0xffu;
          atomicAdd(reinterpret_cast<unsigned long long*>(base + lb8 + (min(bb, nb) << sh3)),
                    (unsigned long long)gp[u]);
        }
      }
    }
  }
  __syncthreads();
  stamp_.probe(3);
  // Per-item partial histogram -> slab (plain coalesced stores; the packed u64 of the K copies can
  // be summed directly because the per-item sums obey the same < 2^31 / < 2^32 bounds).
  if (d.ablate == 2) return;  // timing-only: no flush
  hist_flush<kWide>(d, s_hist, hl, item, f0, ft, tg, th, blockIdx.y == 0, s_tot, s_fo, s_fs);
}

// Reduce the per-item slabs into the level's histogram slots: thread = one compact (feature, bin)
// cell (cell == ncells is the node-total cell), block.x = a run of kRedItems consecutive items; one int64
// global atomic per non-zero cell per (run, slot) -- coalesced, 30-100x fewer than per-block flushes.
constexpr int kRedItems = 16;

// kDP: data parallel (the replica-digest cell of level 0); the single-GPU instantiation has none of it.
template <bool kDP>
// `likely`: items below it exist in all but rare levels (the row-count bound); a block starting past it
// (the hessian build rule's all-rows grid under data parallelism) reads the item count first and
// leaves without its loads when it has no items -- usually the upper half of that grid.
__global__ __launch_bounds__(256) void k_hist_reduce(GbdtDev d, int parity, int n_grid, int level, int likely) {
  BlockStamp stamp_(d);
  const int i0 = blockIdx.x * kRedItems;
  const int ncell = d.ncells;
  const int cell = blockIdx.y * blockDim.x + threadIdx.x;
  if (cell > ncell) return;
  if (i0 >= likely && i0 >= __builtin_amdgcn_readfirstlane(d.counters[0])) return;
  const bool tot = cell == ncell;
  // Issue every load of the run before the first add, in ONE round trip together with the item
  // count: the item indices are clamped to the launched work-item range (n_grid <= items_cap), not
  // to the count, so no load waits on it (items past the count are stale and masked below), and the
  // node-total cell's branch sits outside the unrolled loads (a per-element branch made hipcc wait
  // for every load in turn: 16 x 3 dependent round trips, ~7 us of the kernel's ~12). The count is
  // loaded after them in program order: its uniform use (readfirstlane + wait) must not come first.
  int slot[kRedItems];
  int64_t g[kRedItems], h[kRedItems];
  if (tot) {
#pragma unroll
    for (int k = 0; k < kRedItems; ++k) {
      const int it = min(i0 + k, n_grid - 1);
      slot[k] = d.items_h[it].slot;
      g[k] = d.slab_tot[2 * it];
      h[k] = d.slab_tot[2 * it + 1];
    }
  } else if (d.wide) {  // 16-byte slab cells {g, h}
#pragma unroll
    for (int k = 0; k < kRedItems; ++k) {
      const int it = min(i0 + k, n_grid - 1);
      slot[k] = d.items_h[it].slot;
      const longlong2 v = reinterpret_cast<const longlong2*>(d.slab)[(int64_t)it * ncell + cell];
      g[k] = v.x;
      h[k] = v.y;
    }
  } else {
    uint64_t v[kRedItems];
#pragma unroll
    for (int k = 0; k < kRedItems; ++k) {
      const int it = min(i0 + k, n_grid - 1);
      slot[k] = d.items_h[it].slot;
      v[k] = d.slab[(int64_t)it * ncell + cell];
    }
#pragma unroll
    for (int k = 0; k < kRedItems; ++k) {
      g[k] = (int64_t)(int32_t)(uint32_t)(v[k] >> 32);
      h[k] = (int64_t)(uint32_t)v[k];
    }
  }
  const int n_items = d.counters[0];
  stamp_.probe(1);
  // replica check (data parallel): the previous tree's digest goes into the cell after the root slot
  // (all-reduced with it); this tree's accumulator restarts (no eval of this tree has run yet). After
  // the loads above are issued: at the kernel's head its branch delayed them (+0.4 us per launch).
  if (kDP && level == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    int64_t* const red = d.hist_red ? d.hist_red : d.hist_b[parity];
    red[d.slot_elems] = d.dig_check ? d.dig[d.dig_slot ^ 1] : 0;
    red[d.slot_elems + 1] = 0;
    d.dig[d.dig_slot] = 0;
  }
  if (i0 >= n_items) return;
  const int cnt = min(n_items - i0, kRedItems);
#pragma unroll
  for (int k = 0; k < kRedItems; ++k)  // stale tail items: no slot (flushes nothing)
    if (k >= cnt) { g[k] = 0; h[k] = 0; slot[k] = -2; }
  // items of one slot are consecutive: flush one atomic pair per (run, slot)
  stamp_.probe(2);
  int64_t* const red = d.hist_red ? d.hist_red : d.hist_b[parity];
  int cur = slot[0];
  int64_t sg = 0, sh = 0;
#pragma unroll
  for (int k = 0; k < kRedItems; ++k) {
    if (slot[k] != cur) {
      if (cur >= 0 && (sg | sh)) {
        int64_t* dst = red + (int64_t)cur * d.slot_elems + (int64_t)cell * 2;
        atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)sg);
        atomicAdd(reinterpret_cast<unsigned long long*>(dst + 1), (unsigned long long)sh);
      }
      cur = slot[k];
      sg = sh = 0;
    }
    sg += g[k];
    sh += h[k];
  }
  if (cur >= 0 && (sg | sh)) {
    int64_t* dst = red + (int64_t)cur * d.slot_elems + (int64_t)cell * 2;
    atomicAdd(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)sg);
    atomicAdd(reinterpret_cast<unsigned long long*>(dst + 1), (unsigned long long)sh);
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

// Both children's gains of a candidate split with ONE fp64 division: (tl^2 (hr + lambda) + tr^2 (hl +
// lambda)) / ((hl + lambda)(hr + lambda)). Candidates are only scored when both children reach
// min_child_weight. Same operation order as the host oracle (models/gbdt_host.py, _calc_gain_pair).
__device__ __forceinline__ double calc_gain_pair(double gl, double hl, double gr, double hr, double lambda_,
                                                 double alpha) {
  const double tl = alpha == 0.0 ? gl : thresh_l1(gl, alpha);
  const double tr = alpha == 0.0 ? gr : thresh_l1(gr, alpha);
  const double dl = hl + lambda_, dr = hr + lambda_;
  return (tl * tl * dr + tr * tr * dl) / (dl * dr);
}

__device__ __forceinline__ double calc_weight(double g, double h, double lambda_, double alpha, double mcw) {
  if (h < mcw || h <= 0.0) return 0.0;
  const double t = alpha == 0.0 ? g : thresh_l1(g, alpha);
  return -t / (h + lambda_);
}

// Latency structure: one round of scalar loads for the node (and its parent's build flag / the root
// total), then every wave issues ALL loads of its <= 2 features (histogram bins, parent bins for the
// subtraction, masks, bin counts, cut values) before computing, so a level costs ~2 dependent memory
// round trips; the winning candidate carries its cut value (no load after the reduction).
struct EvalFeat {
  int f, nb, off;  // feature, bin count, compact cell offset
  bool on;
  int64_t g[4], h[4];   // bin 64 c + lane of chunk c
  float cut[4];  // cut of bin 64 c + lane (the bin before it, for missing-left splits, comes by DPP)
};

// Node decision from its best candidate (split or leaf; children of the last split level become leaves).
// `nb_known` >= 0: the winning feature's bin count (the compact evaluator has it in LDS), else loaded.
template <bool kDP>
__device__ void eval_finalize(const GbdtDev& d, int level, int n, int64_t G, int64_t H, Cand best, float best_cut,
                              int nb_known = -1) {
  Node* nodes = d.nodes;
  const double Gd = (double)G * d.ginv, Hd = (double)H * d.hinv;
  const float loss = (float)best.gain;
  const bool ok = best.key != 0x7fffffff && loss > 1e-6f && loss >= (float)d.gamma;
  const double wgt = calc_weight(Gd, Hd, d.lambda_, d.alpha, d.mcw);
  Node& nd = nodes[n];
  if (level == 0) { nd.G = G; nd.H = H; }
  nd.sum_hess = (float)Hd;
  nd.base_weight = (float)(wgt * d.eta);
  if (ok) {
    const int f = best.key >> 10;
    const int r = best.key & 1023;
    const int nb = nb_known >= 0 ? nb_known : d.nbins[f];
    int j, dl;
    if (r < 512) { j = r; dl = 0; } else { j = (nb - 1 - (r - 512)) - 1; dl = 1; }
    nd.status = kSplit;
    nd.feat = f;
    nd.bin = j;
    nd.default_left = dl;
    nd.split_cond = j >= 0 ? best_cut : -FLT_MAX;
    nd.loss_chg = loss;
    Node& L = nodes[2 * n + 1];
    Node& R = nodes[2 * n + 2];
    L.status = kActive; L.G = best.gl; L.H = best.hl;
    R.status = kActive; R.G = G - best.gl; R.H = H - best.hl;
    // Child histogrammed from rows by the fused partition pass (k_part_hist): the one with the
    // smaller GLOBAL hessian (known here, before the partition; identical on every rank, and the
    // host oracle's choice). The unfused path overrides this with row counts in publish_level.
    const int lb = best.hl <= H - best.hl ? 1 : 0;
    L.build = lb;
    R.build = 1 - lb;
    if (level + 1 == d.max_depth) {  // children are at max depth: finalise them as leaves here
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        Node& ch = c == 0 ? L : R;
        const double cg = (double)ch.G * d.ginv, chh = (double)ch.H * d.hinv;
        const double cw = calc_weight(cg, chh, d.lambda_, d.alpha, d.mcw);
        ch.sum_hess = (float)chh;
        ch.base_weight = (float)(cw * d.eta);
        ch.status = kLeaf;
        ch.leaf_value = (float)(cw * d.eta);
        ch.split_cond = ch.leaf_value;
      }
    }
  } else {
    nd.status = kLeaf;
    nd.leaf_value = (float)(wgt * d.eta);
    nd.split_cond = nd.leaf_value;
  }
  if (kDP) {  // replica digest (data parallel): this node's decision (+ its max-depth leaf children)
    uint32_t hsum = node_hash(n, nd.status, ok ? nd.feat : -1, ok ? nd.bin : -1, ok ? nd.default_left : 0, nd.split_cond,
                              nd.G, nd.H);
    if (ok && level + 1 == d.max_depth) {
      hsum += node_hash(2 * n + 1, kLeaf, -1, -1, 0, nodes[2 * n + 1].split_cond, nodes[2 * n + 1].G, nodes[2 * n + 1].H);
      hsum += node_hash(2 * n + 2, kLeaf, -1, -1, 0, nodes[2 * n + 2].split_cond, nodes[2 * n + 2].G, nodes[2 * n + 2].H);
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(d.dig + d.dig_slot), (unsigned long long)hsum);
  }
}

// Node ownership over the fused IPC exchange (levels >= d.own_level; 2^own_level >= ranks). A node's
// histogram sums and split evaluation run on ONE rank -- the owner of its level-own_level ancestor, so
// the owner also holds the parent histogram its subtree subtracts from -- instead of on every rank:
// each rank reads 1/world of the level's cells over xGMI instead of all of them (and the sibling
// duplication of the per-node blocks goes with it). The owner publishes the node's record and its
// children's (everything but the rank-local row ranges) with an epoch tag into its exported decision
// table (system-scope stores, the tag last); the other ranks poll the tag and copy the records.
__device__ __forceinline__ int node_owner(const GbdtDev& d, int level, int n, int world) {
  const int pos = n - ((1 << level) - 1);
  return (pos >> (level - d.own_level)) % world;
}

__device__ __forceinline__ void own_publish(const GbdtDev& d, const IpcFusedView* iv, int n) {
  // thread 0, after eval_finalize wrote the three records into this rank's node table
  char* rec = iv->mydtab + (int64_t)n * kIpcDecStride;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(d.nodes + (k == 0 ? n : 2 * n + k));
#pragma unroll
    for (int w = 0; w < 8; ++w)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(rec + k * 64 + w * 8), src[w], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_s_waitcnt(0);  // the records are written through before the tag
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(rec + 192), (unsigned long long)d.ipc_epoch,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A non-owner's block for node n (active at this level): wait for the owner's record of this epoch,
// copy it into the local node table (the rank-local start / count words stay) and add the node's
// replica-digest terms as the owner's eval_finalize did. Call from all threads.
__device__ __forceinline__ void own_copy(const GbdtDev& d, const IpcFusedView* iv, int n, int level, int owner) {
  __shared__ int s_ok;
  const char* rec = iv->dtab[owner] + (int64_t)n * kIpcDecStride;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int ok = __hip_atomic_load(iv->myflag + kIpcStickyWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    const unsigned* notice = iv->ftab[owner] + kIpcFailWord;  // the owner gave up: no record will come
    while (ok) {
      const unsigned long long t = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(rec + 192),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (t == (unsigned long long)d.ipc_epoch) break;
      if (__hip_atomic_load(notice, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
          __builtin_amdgcn_s_memrealtime() - t0 > iv->timeout) {
        ok = 0;
        ipc_fail(iv->myflag, iv->err_host);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok) return;
  if (threadIdx.x < 24) {
    const int k = threadIdx.x >> 3, w = threadIdx.x & 7;
    if (w != 2) {  // word 2 = (start, count): this rank's own row range
      const unsigned long long v = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(rec + k * 64 + w * 8),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      reinterpret_cast<unsigned long long*>(d.nodes + (k == 0 ? n : 2 * n + k))[w] = v;
    }
  }
  __syncthreads();
  // (a record whose node was not active on its owner means the trees diverged at a level every rank
  // evaluates: the copy re-synchronises the node table so the tree completes on every rank, and the
  // digest of those levels, compared at the next tree's root exchange, reports it on every rank alike)
  if (threadIdx.x == 0) {  // (own_copy runs under data parallelism only: d.dig is set)
    const Node nd = d.nodes[n];
    const bool ok = nd.status == kSplit;
    uint32_t hsum = node_hash(n, nd.status, ok ? nd.feat : -1, ok ? nd.bin : -1, ok ? nd.default_left : 0, nd.split_cond,
                              nd.G, nd.H);
    if (ok && level + 1 == d.max_depth) {
      const Node& cl = d.nodes[2 * n + 1];
      const Node& cr = d.nodes[2 * n + 2];
      hsum += node_hash(2 * n + 1, kLeaf, -1, -1, 0, cl.split_cond, cl.G, cl.H);
      hsum += node_hash(2 * n + 2, kLeaf, -1, -1, 0, cr.split_cond, cr.G, cr.H);
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(d.dig + d.dig_slot), (unsigned long long)hsum);
  }
}

// Fused exchange, phase A: the block's histogram cells [cb, cb + mt) and, after them, the totals cell
// (LDS slot mt) and at level 0 the replica-digest cell (slot mt + 1), m cells in all, summed over the
// NR ranks' send slots into LDS. Every cell's NR loads are in flight together
// (one remote round trip per block instead of one per rank); `store`: the sums also go to hist_b
// (the built child's global histogram, for the next level's subtraction), `store_tot`: the totals too.
// The peers' cells are read with system-scope loads (they bypass this XCD's L2, so the wait needs no
// L2-invalidating acquire; kIpcAcquireFence = true restores the fence + plain loads for A/B).
#ifndef COBALT_IPC_ACQUIRE_FENCE
#define COBALT_IPC_ACQUIRE_FENCE 0
#endif
constexpr bool kIpcAcquireFence = COBALT_IPC_ACQUIRE_FENCE != 0;
__device__ __forceinline__ longlong2 ipc_load_cell(const char* p) {
  if (kIpcAcquireFence) return *reinterpret_cast<const longlong2*>(p);
  longlong2 v;
  v.x = __hip_atomic_load(reinterpret_cast<const long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  v.y = __hip_atomic_load(reinterpret_cast<const long long*>(p) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return v;
}

// A peer's cell as ONE 16-byte load with the system-scope cache policy (sc0 sc1: a miss in this XCD's L2,
// as the two 8-byte system-scope atomic loads of ipc_load_cell) through a buffer resource over the
// peer's slot: half the load instructions and fabric requests per cell. (A volatile 16-byte load gets the
// same policy but a wait after every load.)
constexpr int kCpolSystem = 1 | 16;  // buffer aux bits on gfx950: sc0 = bit 0, sc1 = bit 4
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ipc_rsrc(const char* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ longlong2 ipc_load_cell_rs(__amdgpu_buffer_rsrc_t rs, const char* base, uint32_t off) {
  if (kIpcAcquireFence) return *reinterpret_cast<const longlong2*>(base + off);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, kCpolSystem);
  return make_longlong2((long long)(((uint64_t)v[1] << 32) | v[0]), (long long)(((uint64_t)v[3] << 32) | v[2]));
}

template <int NR>
__device__ __forceinline__ void ipc_sum_cells(const IpcFusedView* iv, int64_t pair_bytes, int cb, int mt, int m, int ncells,
                                              longlong2* s_cells, longlong2* hbw, bool store, bool store_tot, bool sub) {
  // U cells per thread per round trip: all U x NR loads (clamped, unconditional) are issued before the
  // first sum -- over xGMI every round trip is a remote latency, and a 1024-thread block sums ~5k cells
  constexpr int U = NR <= 4 ? 4 : 2;
  const char* sp[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) sp[r] = iv->slot[r] + pair_bytes;
  const int B = (int)blockDim.x;
  for (int i0 = threadIdx.x; i0 < m; i0 += U * B) {
    longlong2 t[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ic = min(i0 + u * B, m - 1);
      const int cell = ic < mt ? cb + ic : ncells + (ic - mt);
      // (every slot, this rank's own included, with the system-scope policy: a plain load for the own
      // slot kept a second load form and a select per cell live -- 21 VGPRs more with the buffer loads)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const uint32_t off = (uint32_t)cell * (uint32_t)sizeof(longlong2);
        t[u][r] = ipc_load_cell_rs(ipc_rsrc(sp[r]), sp[r], off);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * B;
      if (i >= m) break;
      const int cell = i < mt ? cb + i : ncells + (i - mt);
      longlong2 acc = t[u][0];
#pragma unroll
      for (int r = 1; r < NR; ++r) {
        acc.x += t[u][r].x;
        acc.y += t[u][r].y;
      }
      s_cells[i] = sub && i < mt ? make_longlong2(s_cells[i].x - acc.x, s_cells[i].y - acc.y) : acc;
      if (i < mt ? store : store_tot) hbw[cell] = acc;
    }
  }
}

// 9-16 ranks (more than one 8-GPU node's worth of processes): two groups of 8 loads per cell, so no
// instantiation holds more than 8 ranks' values in registers (the fused k_eval keeps the parent's
// histogram loads in flight across the exchange and spilled with 16)
__device__ __forceinline__ void ipc_sum_cells_wide(int nr, const IpcFusedView* iv, int64_t pair_bytes, int cb, int mt, int m,
                                                   int ncells, longlong2* s_cells, longlong2* hbw, bool store,
                                                   bool store_tot, bool sub) {
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    const int cell = i < mt ? cb + i : ncells + (i - mt);
    const int64_t off = pair_bytes + (int64_t)cell * (int64_t)sizeof(longlong2);
    longlong2 acc = make_longlong2(0, 0);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      longlong2 t[8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
        t[r] = 8 * g + r < nr ? ipc_load_cell(iv->slot[8 * g + r] + off) : make_longlong2(0, 0);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        acc.x += t[r].x;
        acc.y += t[r].y;
      }
    }
    s_cells[i] = sub && i < mt ? make_longlong2(s_cells[i].x - acc.x, s_cells[i].y - acc.y) : acc;
    if (i < mt ? store : store_tot) hbw[cell] = acc;
  }
}

__device__ __forceinline__ void ipc_sum_cells_n(int nr, const IpcFusedView* iv, int64_t pair_bytes, int cb, int mt, int m,
                                                int ncells, longlong2* s_cells, longlong2* hbw, bool store,
                                                bool store_tot, bool sub) {
  switch (nr) {
#define IPC_SUM_CASE(K) \
    case K: ipc_sum_cells<K>(iv, pair_bytes, cb, mt, m, ncells, s_cells, hbw, store, store_tot, sub); break;
    IPC_SUM_CASE(1) IPC_SUM_CASE(2) IPC_SUM_CASE(3) IPC_SUM_CASE(4) IPC_SUM_CASE(5) IPC_SUM_CASE(6)
    IPC_SUM_CASE(7) IPC_SUM_CASE(8)
#undef IPC_SUM_CASE
    default: ipc_sum_cells_wide(nr, iv, pair_bytes, cb, mt, m, ncells, s_cells, hbw, store, store_tot, sub); break;
  }
}

// kGroups: the node's features are split over gridDim.y blocks of `fg` features each (one CU per
// group instead of one per node: the fp64 gain scan of a wide node -- 106 features in the RFE stage --
// is issue-bound on a single CU); each group writes its best candidate and k_eval_finish reduces them.
//
// Wave w takes features w and w + nw per pass. A feature's bins are laid out LANE-major in chunks of
// 64 (bin = 64 c + lane): a feature costs ceil(nb / 64) chunk steps of fp64 gain work -- one for a
// binary feature, four for a 256-bin one (the former bin-major layout, 4 consecutive bins per lane,
// cost every feature four) -- and each chunk is one coalesced 16-byte (g, h) load per lane. A chunk's
// left sums are a DPP int64 wave scan plus the carry of the chunks before it. Candidates, keys and
// tie-breaks are unchanged, so the trees are bit-identical.
//
// Without groups (one 1024-thread block per node) the feature -> wave assignment is the host's
// eval_assignment table (asg*: slot 2 w + s = wave w's s-th feature, 8 bits each, 0xFF = none): the
// fp64 candidate work is ceil(nb / 64) chunk steps per feature and the 16 waves share 4 SIMDs (wave w
// on SIMD w mod 4), so the table balances chunk steps per SIMD, not per wave.
//
// kFused (data parallel over the one-shot IPC group): this level's histograms are the SUM of every
// rank's send slot, read here -- no separate all-reduce launch. Block (0, 0) publishes this rank's slot
// (complete: the reduce kernel before this one wrote it), every block waits for all ranks after issuing
// its node-record loads (they do not depend on the exchange), sums its cells over the ranks into LDS
// (ipc_sum_cells: dynamic LDS of (cells + 1) x 16 bytes) and reads them from there; the built child's
// global histogram is stored to hist_b for the next level's subtraction. The single-GPU instantiation
// (kFused = false) has none of it.
// Per-slot feature metadata of k_eval<false> (the host's eval_assignment table with each feature's bin
// count and compact offset): slot 2 w + s = wave w's s-th feature, word = f | nb << 8 | off << 17
// (f = 0xFF: no feature). Kernel arguments, read by scalar loads from the kernarg segment, so the
// histogram loads need no global metadata load first.
struct EvalSlots {
  uint32_t w[32];
};

// A node's best split candidate, reduced over the block (eval_core's result, in LDS).
struct EvalOut {
  Cand best;
  float cut;
  int nb;           // the winner's bin count (0 without a candidate)
  int64_t G, H;     // node totals
};

// Split evaluation of node `pos` of the level by the whole (1024-thread) block. Returns false (in every
// thread) for an inactive node or a failed exchange; otherwise thread 0 holds the result in *s_out (the
// other threads see it after a barrier). Shared by k_eval and the fused evaluation + partition pass.
// `kMerged` (k_eval_part): the node counts as active whatever its status (another block of the same
// node may already have finalised it), and only `store_hist` blocks store its histogram.
// kDP: data parallel (kFused implies it): the level-0 replica-digest check and the fault-injection hook;
// the single-GPU instantiation carries neither.
template <bool kGroups, bool kFused, bool kDP, bool kMerged = false>
__device__ __forceinline__ bool eval_core(const GbdtDev& d, int level, int parity, int tree, int fg, const EvalSlots& es,
                                          int pos, BlockStamp& stamp_, EvalOut* s_out, bool store_hist = true) {
  const int fbeg = kGroups ? blockIdx.y * fg : 0;
  const int fend = kGroups ? min(d.F, fbeg + fg) : d.F;
  const int n = (1 << level) - 1 + pos;
  Node* nodes = d.nodes;
  const int pair = level == 0 ? 0 : (pos >> 1);
  const int64_t SE = d.slot_elems;
  const int64_t* hb = d.hist_b[parity] + pair * SE;
  int64_t* hs = d.hist_s[parity] + (int64_t)pos * SE;  // this node's full histogram, for its children
  const int lane = lane_id();
  const int nw = (int)(blockDim.x / kWave);
  const uint8_t* fm = d.fmask + (int64_t)tree * d.F;
  extern __shared__ longlong2 s_cells[];  // kFused: the block's cells summed over the ranks
  // Per-feature metadata (mask, bin count, compact offset, cut values) does not depend on the node:
  // it is loaded in the same round trip as the node record (unconditional, in-bounds loads).
  EvalFeat ef[2];
  auto load_meta = [&](int fbase) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      EvalFeat& e = ef[s];
      int nbv, offv;
      if (kGroups) {
        e.f = fbase + s * nw;
        const int fc = min(e.f, d.F - 1);
        nbv = d.nbins[fc];
        offv = d.hoff[fc];
      } else {  // from the kernel arguments: no global load in front of the histogram loads
        const int slot = __builtin_amdgcn_readfirstlane(wave_id() * 2 + s);
        const uint32_t sw = es.w[slot];
        const int fi = (int)(sw & 0xFFu);
        e.f = fi == 0xFF ? fend : fi;
        nbv = (int)((sw >> 8) & 0x1FFu);
        offv = (int)(sw >> 17);
      }
      const int fc = min(e.f, d.F - 1);
      const bool valid = e.f < fend;
      const uint8_t fmv = fm[fc];  // unconditional loads, masked after (no per-load branch)
      e.on = valid && fmv != 0;
      e.nb = valid ? nbv : 0;
      e.off = offv;
#pragma unroll
      for (int c = 0; c < 4; ++c) e.cut[c] = d.cuts[fc * kMaxBins + c * kWave + lane];
    }
  };
  load_meta(fbeg + wave_id());
  // per-lane byte offsets of this wave's cells (from the kernel-argument metadata) and the load masks:
  // only lanes holding a real bin of an evaluated feature load (exec-masked): the CU's address path
  // costs per active lane, and unmasked, the 16 waves' 2 x 4 chunks (+ the parent's) were 256 full
  // 1 KB load instructions per block for ~26 chunks of real bins -- ~2 us per level at 1M rows.
  // (the colsample bit is applied after the loads: it is a global load of round trip 1 itself)
  // (32-bit byte offsets from the uniform bases: the loads take the SGPR-base + VGPR-offset form
  // instead of a 64-bit VGPR address pair each -- 32 VGPRs the kernel otherwise spilled)
  uint32_t cofs[2][4];
  bool ld[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      cofs[s][c] = (uint32_t)(ef[s].off + min(c * kWave + lane, max(ef[s].nb - 1, 0))) * (uint32_t)sizeof(longlong2);
      ld[s][c] = c * kWave + lane < ef[s].nb;
    }
  // the parent's full histogram (the previous level's k_eval stored every node's by position): its
  // address depends on the block index only
  const int64_t* parent = level > 0 ? d.hist_s[parity ^ 1] + (int64_t)(pos >> 1) * SE : hb;
  const longlong2* pa2 = reinterpret_cast<const longlong2*>(readlane64((int64_t)parent, 0));  // uniform base
  longlong2 pv[2][4];
  auto load_parent = [&]() {
    if (level > 0) {  // kernel argument: uniform, no wait on the node record (whose build flag selects)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          pv[s][c] = ld[s][c] ? *reinterpret_cast<const longlong2*>(reinterpret_cast<const char*>(pa2) + cofs[s][c])
                              : make_longlong2(0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < 4; ++c) pv[s][c] = make_longlong2(0, 0);
    }
  };
  // (fused exchange, per-node blocks: the subtracted sibling's parent histogram goes to LDS while wave 0
  // waits for the peers, and the ranks' sums are subtracted from it there -- no global load after the
  // exchange, and no parent registers held across it; grouped blocks load it after the exchange)
  constexpr bool kParLds = kFused && !kGroups;
  // Without the exchange, the node's histogram bins and its parent's are issued HERE, with the node record's
  // (scalar) loads: their addresses come from the kernel arguments and the block index, and the vector
  // loads do not wait on the scalar ones -- one round trip for both instead of record -> bins
  longlong2 v[2][4];
  auto load_bins = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[s][c] = ld[s][c] ? *reinterpret_cast<const longlong2*>(reinterpret_cast<const char*>(hb) + cofs[s][c])
                           : make_longlong2(0, 0);
  };
  if (!kFused) {
    load_bins();
    load_parent();
  }
  // round trip 1 (uniform scalar loads); unconditional (in-bounds) loads selected after
  const int status = nodes[n].status;
  const bool built = nodes[n].build != 0;
  int64_t rg = 0, rh = 0;
  if (!kFused) {
    rg = hb[(int64_t)d.ncells * 2];
    rh = hb[(int64_t)d.ncells * 2 + 1];
  }
  const int64_t ng = nodes[n].G, nh = nodes[n].H;
  int cb = 0;  // kFused: the block's first cell (LDS slot 0)
  if (kFused) {
    const IpcFusedView* iv = d.ipcv + (d.ipc_epoch & 1u);
    cb = kGroups ? d.hoff[fbeg] : 0;
    const int ce = kGroups ? d.hoff[fend] : d.ncells;
    // (k_eval_part publishes before its plan: its block 0 is not always an evaluating block)
    if (!kMerged && blockIdx.x == 0 && blockIdx.y == 0) ipc_publish(iv->myflag, d.ipc_epoch);
    if (!kGroups && !kMerged && d.own_level >= 0 && level >= d.own_level) {
      const int owner = node_owner(d, level, n, iv->n);
      if (owner != iv->me) {  // another rank evaluates this node: take its decision
        if (status == kActive) own_copy(d, iv, n, level, owner);
        return false;
      }
    }
    const bool sub = kParLds && level > 0 && !built;  // block-uniform
    if (sub && threadIdx.x >= kWave) {  // waves 1.. (wave 0 polls the peers' flags)
      const longlong2* par = reinterpret_cast<const longlong2*>(parent) + cb;
      for (int i = (int)threadIdx.x - kWave; i < ce - cb; i += (int)blockDim.x - kWave) s_cells[i] = par[i];
    }
    if (!ipc_wait<kIpcAcquireFence>(iv->ftab, iv->n, iv->me, iv->myflag, d.ipc_epoch, iv->err_host, iv->timeout))
      return false;
    // the global root totals are stored at level 0 (k_eval_finish reads them)
    // (+ the replica-digest cell at level 0)
    ipc_sum_cells_n(__builtin_amdgcn_readfirstlane(iv->n), iv, (int64_t)pair * SE * (int64_t)sizeof(int64_t), cb,
                    ce - cb, ce - cb + 1 + (level == 0 ? 1 : 0), d.ncells, s_cells,
                    reinterpret_cast<longlong2*>(d.hist_b[parity] + pair * SE), built && status == kActive,
                    level == 0 && blockIdx.y == 0, sub);
    __syncthreads();
    const longlong2 tot = s_cells[ce - cb];
    rg = tot.x;
    rh = tot.y;
  }
  // node totals: wave-uniform, pinned to SGPRs (vector-loaded, they held VGPRs across the scan)
  int64_t G = readlane64(level == 0 ? rg : ng, 0);
  const int64_t H = readlane64(level == 0 ? rh : nh, 0);
  if (kDP && level == 0 && d.corrupt) G += (int64_t)1 << 24;  // fault injection: this rank grows a different tree
  // No early return for an inactive node: a branch here let hipcc sink the feature metadata loads
  // below it (a third dependent round trip). Its block computes on valid buffers and stores nothing.
  const bool active = kMerged ? status != kNone : status == kActive;
  stamp_.probe(1);
  __shared__ Cand s_best[16];
  __shared__ float s_cut[16];
  __shared__ int s_nb[32];  // !kGroups: bin count per feature, for the winner's bin (no global load after the reduction)
  if (!kGroups && lane == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (ef[s].f < 32) s_nb[ef[s].f] = ef[s].nb;
  }
  const double Gd = (double)G * d.ginv, Hd = (double)H * d.hinv;
  // wave-uniform: kept in SGPRs (as a VALU result it held a VGPR pair the candidate loop spilled)
  const double parent_gain = __longlong_as_double(
      readlane64(__double_as_longlong(calc_gain(Gd, Hd, d.lambda_, d.alpha, d.mcw)), 0));
  Cand best;
  best.gain = -INFINITY;
  best.key = 0x7fffffff;
  best.gl = 0;
  best.hl = 0;
  float best_cut = -FLT_MAX;
  const longlong2* hb2 = reinterpret_cast<const longlong2*>(hb);
  // one pass: a block covers at most 2 features per wave (the host keeps F <= 32 per block)
  {
  // the histogram bins (and the parent's, for the subtraction) of both features: loaded above without the
  // exchange; with it, the ranks' sums from LDS (clamped cells: the loads need no per-load guard)
  if (kFused) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[s][c] = ld[s][c] ? s_cells[cofs[s][c] / (uint32_t)sizeof(longlong2) - (uint32_t)cb] : make_longlong2(0, 0);
    if (!kParLds) load_parent();
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    EvalFeat& e = ef[s];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = e.on && c * kWave + lane < e.nb;
      // (kParLds: the LDS cells already hold this node's own histogram)
      const int64_t g = (kParLds || built) ? v[s][c].x : pv[s][c].x - v[s][c].x;
      const int64_t h = (kParLds || built) ? v[s][c].y : pv[s][c].y - v[s][c].y;
      e.g[c] = in ? g : 0;
      e.h[c] = in ? h : 0;
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const EvalFeat& e = ef[s];
    if (!e.on) continue;
    const int f = e.f, nb = e.nb;
    const int nch = (nb + kWave - 1) / kWave;  // wave-uniform
    if (active && store_hist && level + 1 < d.max_depth) {  // this node's histogram, for its children's subtraction
      longlong2* hs2 = reinterpret_cast<longlong2*>(hs);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nch && c * kWave + lane < nb) hs2[e.off + c * kWave + lane] = make_longlong2(e.g[c], e.h[c]);
    }
    // inclusive left sums of every bin: per-chunk wave scans + the carry of the previous chunks
    int64_t ig[4], ih[4];
    int64_t cg = 0, ch = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < nch) {
        const int64_t sg = wave_incl_scan(e.g[c]), sh = wave_incl_scan(e.h[c]);
        ig[c] = sg + cg;
        ih[c] = sh + ch;
        cg += readlane64(sg, kWave - 1);
        ch += readlane64(sh, kWave - 1);
      } else {
        ig[c] = 0;
        ih[c] = 0;
      }
    }
    const int64_t mg = G - cg, mh = H - ch;  // missing-value statistics
    const bool has_missing = (mg != 0) || (mh != 0);
    const double GD = (double)G, HD = (double)H, MGd = (double)mg, MHd = (double)mh;  // exact (< 2^53)
    // Candidates, one chunk per iteration of a rolled loop: the chunk's values are rotated down the
    // register arrays (constant indices), so only one chunk's fp64 temporaries are live at a time
    // (the unrolled form spilled at the 128-VGPR limit of a 1024-thread block).
    int64_t rg[4], rh[4], rig[4], rih[4];
    float rcut[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) { rg[c] = e.g[c]; rh[c] = e.h[c]; rig[c] = ig[c]; rih[c] = ih[c]; rcut[c] = e.cut[c]; }
    float carry_cut = -FLT_MAX;  // cut of the previous chunk's last bin
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      // cut of bin b - 1: the previous lane's (DPP wave shift), lane 0 takes lane 63 of chunk c - 1
      const float cutp = __int_as_float(dpp32<kDppWaveShr1>(__float_as_int(rcut[0]), __float_as_int(carry_cut)));
      carry_cut = __int_as_float(readlane32(__float_as_int(rcut[0]), kWave - 1));
      const int b = c * kWave + lane;
      if (b < nb) {
        // direction 0: missing -> right, left = bins <= b
        // the int64 sums are < 2^53 in magnitude, so integer differences taken in fp64 are exact: the
        // right side is GD - GLd instead of converting G - GL (bit-identical, two int64 -> fp64
        // conversions fewer per direction)
        const double GLd = (double)rig[0], HLd = (double)rih[0];
        {
          const int64_t GL = rig[0], HL = rih[0];
          const double gl = GLd * d.ginv, hl = HLd * d.hinv;
          const double gr = (GD - GLd) * d.ginv, hr = (HD - HLd) * d.hinv;
          if (hl >= d.mcw && hr >= d.mcw) {
            Cand cd;
            cd.gain = calc_gain_pair(gl, hl, gr, hr, d.lambda_, d.alpha) - parent_gain;
            cd.key = f * 1024 + b;
            cd.gl = GL;
            cd.hl = HL;
            if (cand_better(cd, best)) { best = cd; best_cut = rcut[0]; }
          }
        }
        // direction 1: missing -> left, left = bins <= b-1 (+ missing)
        if (has_missing) {
          const int64_t GL = rig[0] - rg[0] + mg, HL = rih[0] - rh[0] + mh;
          const double GL1 = (GLd - (double)rg[0]) + MGd, HL1 = (HLd - (double)rh[0]) + MHd;  // exact
          const double gl = GL1 * d.ginv, hl = HL1 * d.hinv;
          const double gr = (GD - GL1) * d.ginv, hr = (HD - HL1) * d.hinv;
          if (hl >= d.mcw && hr >= d.mcw) {
            Cand cd;
            cd.gain = calc_gain_pair(gl, hl, gr, hr, d.lambda_, d.alpha) - parent_gain;
            cd.key = f * 1024 + 512 + (nb - 1 - b);
            cd.gl = GL;
            cd.hl = HL;
            if (cand_better(cd, best)) { best = cd; best_cut = b == 0 ? -FLT_MAX : cutp; }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        rg[k] = rg[k + 1]; rh[k] = rh[k + 1]; rig[k] = rig[k + 1]; rih[k] = rih[k + 1]; rcut[k] = rcut[k + 1];
      }
    }
  }
  }
  stamp_.probe(2);
  if (!active) return false;  // block-uniform
  wave_best(best, best_cut);
  if (lane == 0) { s_best[wave_id()] = best; s_cut[wave_id()] = best_cut; }
  __syncthreads();
  stamp_.probe(3);
  if (wave_id() == 0) {
    // the waves' winners, one per lane of wave 0, reduced by the same DPP arg-max
    if (lane < nw) { best = s_best[lane]; best_cut = s_cut[lane]; }
    else { best.gain = -INFINITY; best.key = 0x7fffffff; best.gl = 0; best.hl = 0; best_cut = -FLT_MAX; }
    wave_best(best, best_cut);
    if (lane == 0) {
      s_out->best = best;
      s_out->cut = best_cut;
      s_out->nb = (!kGroups && best.key != 0x7fffffff) ? s_nb[(best.key >> 10) & 31] : 0;
      s_out->G = G;
      s_out->H = H;
      // replica check of the previous tree (data parallel; off the evaluation's critical path)
      if (kDP && level == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
        int64_t dsum;
        if (kFused) {
          const int nc = kGroups ? d.hoff[fend] - d.hoff[fbeg] : d.ncells;
          dsum = s_cells[nc + 1].x;
        } else {
          dsum = hb[SE];
        }
        digest_check(d, dsum);
      }
    }
  }
  return true;
}

template <bool kGroups, bool kFused, bool kDP>
__global__ __launch_bounds__(1024) void k_eval(GbdtDev d, int level, int parity, int tree, int fg, EvalSlots es) {
  static_assert(kDP || !kFused, "the fused exchange is data parallel");
  BlockStamp stamp_(d);
  const int pos = blockIdx.x;
  __shared__ EvalOut s_out;
  if (!eval_core<kGroups, kFused, kDP>(d, level, parity, tree, fg, es, pos, stamp_, &s_out)) {
    // an owned node that is not active on its owner still publishes its record: a rank whose tree went
    // another way (replica divergence) and waits for it then learns so instead of timing out
    if (kFused && !kGroups && threadIdx.x == 0 && d.own_level >= 0 && level >= d.own_level) {
      const int n = (1 << level) - 1 + pos;
      const IpcFusedView* iv = d.ipcv + (d.ipc_epoch & 1u);
      if (node_owner(d, level, n, iv->n) == iv->me && d.nodes[n].status != kActive) own_publish(d, iv, n);
    }
    return;
  }
  if (threadIdx.x != 0) return;  // thread 0 wrote s_out
  const Cand best = s_out.best;
  const float best_cut = s_out.cut;
  if (kGroups) {
    CandRec& o = d.cand[(int64_t)pos * gridDim.y + blockIdx.y];
    o.gain = best.gain;
    o.key = best.key;
    o.cut = best_cut;
    o.gl = best.gl;
    o.hl = best.hl;
    return;
  }
  eval_finalize<kDP>(d, level, (1 << level) - 1 + pos, s_out.G, s_out.H, best, best_cut, s_out.nb);
  if (kFused && d.own_level >= 0 && level >= d.own_level)  // the other ranks copy this node's decision
    own_publish(d, d.ipcv + (d.ipc_epoch & 1u), (1 << level) - 1 + pos);
  stamp_.probe(4);
}

// Reduce the per-group candidates of each node of the level (one wave per node, lane = group).
template <bool kDP>
__global__ __launch_bounds__(64) void k_eval_finish(GbdtDev d, int level, int parity, int ngroups) {
  BlockStamp stamp_(d);
  const int pos = blockIdx.x;
  const int n = (1 << level) - 1 + pos;
  const Node& nd = d.nodes[n];
  if (nd.status != kActive) return;
  int64_t G = nd.G, H = nd.H;
  if (level == 0) {
    G = d.hist_b[parity][(int64_t)d.ncells * 2];
    H = d.hist_b[parity][(int64_t)d.ncells * 2 + 1];
  }
  const int lane = lane_id();
  Cand best;
  best.gain = -INFINITY;
  best.key = 0x7fffffff;
  best.gl = 0;
  best.hl = 0;
  float best_cut = -FLT_MAX;
  if (lane < ngroups) {
    const CandRec& c = d.cand[(int64_t)pos * ngroups + lane];
    best.gain = c.gain;
    best.key = c.key;
    best.gl = c.gl;
    best.hl = c.hl;
    best_cut = c.cut;
  }
  wave_best(best, best_cut);
  if (lane == 0) eval_finalize<kDP>(d, level, n, G, H, best, best_cut);
}

// ------------------------------------------------------------------------------------------
// Partition planning + row partition (K18) + leaf margin update (K19)
// ------------------------------------------------------------------------------------------
// Row partition of the split nodes of a level (K18), one launch. A block takes one work item
// (<= 8192 rows of one node); each wavefront owns a contiguous quarter and keeps its <= 32 rows per
// lane in registers: pass 1 loads row ids + split-feature bins and counts, the block claims its
// left range (from the node start, ascending) and right range (from the node end, descending)
// with one atomic pair per item, pass 2 scatters with ballot ranks -- rows are read once.
// Left rows keep their relative order inside an item; only whole items interleave, so a node's
// row list stays sorted in 8192-row runs (the root level reads rows in identity order).
// The per-item cursor claim is a pair of same-address device-scope atomics, whose latency /
// serialisation across the 8 XCDs dominates a level when items are many and small (measured: removing
// the claims took a 10M-row level from 58 to 24 us); hence 1024-thread blocks (16 waves x 8 steps per
// 8192-row item, 4096-row items while they fit one per CU; see chunk_part).
// kSteps: 64-row steps per wave, sized by the host to the item (chunk <= kPartWaves * kSteps * 64):
// steps past the item would still issue their (unconditional) bin loads and ballots.
template <int kPartWaves, int kSteps>
__global__ __launch_bounds__(kPartWaves * 64) void k_partition(GbdtDev d, int parity, int64_t zero_next, int level,
                                                               int chunk) {
  constexpr int kPartSteps = kSteps;
  BlockStamp stamp_(d);
  __shared__ int32_t s_cnt[2][kPartWaves];
  __shared__ int32_t s_base[2];
  __shared__ int s_plan[5];
  {  // zero the next level's histogram slots (hist_b of the other parity is free at this point)
    int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[parity ^ 1]);
    const int64_t nz = zero_next / 2;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nz; e += (int64_t)gridDim.x * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
  }
  const int item = blockIdx.x;
  const int first = (1 << level) - 1;
  const PlanOut pl = block_plan(1 << level, chunk, item, [&](int e) {
    const Node& n = d.nodes[first + e];
    const int st = n.status, cnt = n.count, start = n.start;  // loaded together (no per-load branch)
    return (st == kSplit && cnt > 0) ? PlanEntry{first + e, 0, start, cnt} : PlanEntry{-1, 0, 0, 0};
  }, s_plan);
  stamp_.probe(1);
  if (pl.node < 0) return;
  WorkItem w;
  w.node = pl.node;
  w.slot = 0;
  w.begin = pl.begin;
  w.end = pl.end;
  const Node nd = d.nodes[w.node];
  const bool identity = parity == 0 && w.node == 0;
  const int32_t* cur = d.ridx[parity];
  int32_t* nxt = d.ridx[parity ^ 1];
  const uint8_t* col = d.binsT + (int64_t)nd.feat * d.ldt;
  const int j = nd.bin;
  const bool dl = nd.default_left != 0;
  // wave index as a uniform (SGPR) value: the per-step row counts and prefix masks stay scalar
  const int wv = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int len = w.end - w.begin;
  const int per = ((len + kPartWaves - 1) / kPartWaves + kWave - 1) / kWave * kWave;
  const int wb = min(w.end, w.begin + wv * per), we = min(w.end, wb + per);
  int r[kPartSteps];
  static_assert(kPartSteps <= 32, "step bit masks are 32-bit");
  uint32_t lbits = 0;
  int nl = 0, nv = 0;
  // row ids: unconditional loads at a clamped index (w.end - 1 is a row of this item), masked after
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const int i = wb + k * kWave + lane;
    const int ic = min(i, w.end - 1);
    const int rv = identity ? ic : cur[ic];
    r[k] = i < we ? rv : -1;
  }
  // the split feature's bins: unconditional loads (padding rows read row 0), so all kPartSteps are in
  // flight at once -- a load guarded per step made hipcc wait for each in turn (32 round trips)
  uint8_t bv[kPartSteps];
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) bv[k] = col[max(r[k], 0)];
  // Pass 1 in integer arithmetic (boolean forms compiled to per-step branches and spilled masks): the
  // direction bit of each row (bin <= j, or the default direction for the missing code) goes to bit k of
  // lbits (0 for the padding lanes, r = -1). The valid rows of step k are a prefix of the lanes (rows
  // wb + 64 k + lane < we), so the wave's valid count is we - wb.
  const int jm1 = j + 1;  // left <=> bin - (j + 1) < 0
  const uint32_t dlv = dl ? 1u : 0u;
  nv = max(0, we - wb);
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const uint32_t b = bv[k];
    const uint32_t lt = (uint32_t)((int)b - jm1) >> 31;  // bin <= j
    const uint32_t ms = (b + 1u) >> 8;                    // bin == 255 (missing)
    const uint32_t ok = ~(uint32_t)r[k] >> 31;            // a row, not padding
    const uint32_t left = (lt | (ms & dlv)) & ok;
    lbits |= left << k;
    nl += __popcll(__ballot(left != 0u));
  }
  asm volatile("" : "+v"(lbits));  // pass 2 reads the packed bits (not 32 live per-step values)
  if (lane == 0) { s_cnt[0][wv] = nl; s_cnt[1][wv] = nv - nl; }
  __syncthreads();
  stamp_.probe(2);
  if (threadIdx.x == 0) {
    int tl = 0, tr = 0;
    for (int k = 0; k < kPartWaves; ++k) { tl += s_cnt[0][k]; tr += s_cnt[1][k]; }
    if (d.ablate == 12) {  // timing-only: no cursor atomics
      s_base[0] = 0; s_base[1] = 0;
    } else {  // both cursors in one 64-bit claim (left = low word, right = high word)
      const unsigned long long c = atomicAdd(reinterpret_cast<unsigned long long*>(d.cursors + 2 * w.node),
                                             ((unsigned long long)(uint32_t)tr << 32) | (uint32_t)tl);
      s_base[0] = (int32_t)(uint32_t)c;
      s_base[1] = (int32_t)(c >> 32);
    }
  }
  __syncthreads();
  stamp_.probe(3);
  int bl = s_base[0], br = s_base[1];
  for (int k = 0; k < wv; ++k) { bl += s_cnt[0][k]; br += s_cnt[1][k]; }
  // Pass 2: one destination per lane (left rows ascending from the node start, right rows descending
  // from its end), one store per step under the valid-lane mask.
  uint32_t pl_ = (uint32_t)(nd.start + bl);                 // next left slot
  uint32_t pr_ = (uint32_t)(nd.start + nd.count - 1 - br);  // next right slot (descending)
#pragma unroll
  for (int k = 0; k < kPartSteps; ++k) {
    const bool valid = r[k] >= 0;
    const uint32_t left = (lbits >> k) & 1u;
    const uint64_t lm = __ballot(left != 0u), vm = __ballot(valid);
    const uint32_t rk_l = mask_rank(lm);
    // valid lanes are a prefix: a right row's rank among the right rows is lane - rk_l
    const uint32_t dst = rk_l + (left ? pl_ : pr_ - (uint32_t)lane);
    if (valid) store_wt(nxt + dst, r[k], (d.wt & 2) != 0);
    const uint32_t cl = (uint32_t)__popcll(lm);
    pl_ += cl;
    pr_ -= (uint32_t)__popcll(vm) - cl;
  }
}

// Row partition by POSITION (levels with <= 64 nodes): block b takes the row-id positions [b C, (b + 1) C)
// of the level's ridx buffer (C = 16 waves x kSteps x 64), whatever nodes they belong to. A level's nodes
// own disjoint, position-ordered ranges of that buffer (every child range lies inside its parent's), so the
// block's row-id loads depend on nothing but the block index: they are issued at kernel entry, in the same
// round trip as the level's node records -- where the node-ordered k_partition first plans its item from
// the node table and only then loads its row ids (~1.1-1.4 us per block at 10M rows, one of ~4 dependent
// round trips). A wave's 512 positions cover a few ranges: a uniform walk over the split ranges that start
// before each 64-row step gives every lane its node; positions of leaves (and gaps) route nowhere. Counts
// are kept per (wave, range) in LDS, one cursor claim per range per block (all in one round trip), and the
// scatter advances per-(wave, range) pointers as k_partition's per-wave ones (left rows ascending from the
// node start, right rows descending from its end).
constexpr int kPartPosNodes = 64;

template <int kSteps>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void k_part_pos(GbdtDev d, int parity, int64_t zero_next, int level) {
  constexpr int kPW = 16;
  constexpr int kN = kPartPosNodes;
  BlockStamp stamp_(d);
  __shared__ int s_rs[kN], s_re[kN];  // split ranges (position order): start, end
  __shared__ uint32_t s_rm[kN];        // feature | (j + 1) << 16 | dl << 25
  __shared__ int s_rn[kN];             // node index
  __shared__ int s_nr;
  __shared__ int32_t s_cnt[kPW][kN][2];  // per (wave, range): left / right rows, then the wave's scatter bases
  __shared__ int s_one, s_one_node, s_one_start, s_one_end;  // the block's one range (s_one < 0: several)
  __shared__ uint32_t s_one_meta;
  __shared__ int32_t s_wc[2][kPW];
  __shared__ int32_t s_wbase[2];
  {  // zero the next level's histogram slots (hist_b of the other parity is free at this point)
    int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[parity ^ 1]);
    const int64_t nz = zero_next / 2;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nz; e += (int64_t)gridDim.x * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
  }
  const int n = (int)d.n;
  const int wv = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int wb = blockIdx.x * (kPW * kSteps * kWave) + wv * (kSteps * kWave);
  const bool identity = parity == 0 && level == 0;  // the root's rows in identity order (never written)
  const int32_t* cur = d.ridx[parity];
  int32_t* nxt = d.ridx[parity ^ 1];
  // row ids first: unconditional loads at clamped positions (no dependence on the node table)
  int r[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; ++k) {
    const int p = min(wb + k * kWave + lane, n - 1);
    r[k] = identity ? p : cur[p];
  }
  // the level's split nodes with rows -> LDS, in position order (wave 0, one lane per node)
  const int first = (1 << level) - 1, nlev = 1 << level;
  if (wv == 0) {
    const int e = lane;
    const Node& nd = d.nodes[first + min(e, nlev - 1)];
    const int st = nd.status, start = nd.start, cnt = nd.count, f = nd.feat, j = nd.bin, dl = nd.default_left;
    const bool on = e < nlev && st == kSplit && cnt > 0;
    const uint64_t m = __ballot(on);
    if (on) {
      const int k = mask_rank(m);
      s_rs[k] = start;
      s_re[k] = start + cnt;
      s_rm[k] = (uint32_t)f | ((uint32_t)(j + 1) & 0x1FFu) << 16 | (uint32_t)(dl & 1) << 25;
      s_rn[k] = first + e;
    }
    if (e == 0) s_nr = __popcll(m);
    // the block's positions inside ONE split range (nearly every block: a node's range spans ~10^5 rows)?
    const int b0 = blockIdx.x * (kPW * kSteps * kWave), b1 = min(n, b0 + kPW * kSteps * kWave);
    const uint64_t hit = __ballot(on && start <= b0 && start + cnt >= b1);
    if (e == 0) s_one = hit ? __ffsll((unsigned long long)hit) - 1 : -1;
    if (hit && e == __ffsll((unsigned long long)hit) - 1) {
      s_one_node = first + e;
      s_one_start = start;
      s_one_end = start + cnt;
      s_one_meta = (uint32_t)f | ((uint32_t)(j + 1) & 0x1FFu) << 16 | (uint32_t)(dl & 1) << 25;
    }
  }
  for (int i = threadIdx.x; i < kPW * kN * 2; i += blockDim.x) (&s_cnt[0][0][0])[i] = 0;
  __syncthreads();
  stamp_.probe(1);
  const int nr = s_nr;
  if (nr == 0) return;
  if (s_one >= 0) {
    // One range: k_partition's per-wave passes (counts by ballot, one claim, running per-wave pointers)
    const int node = s_one_node, nstart = s_one_start, nend = s_one_end;
    const uint32_t m = s_one_meta;
    const uint8_t* col = d.binsT + (int64_t)(m & 0xFFFFu) * d.ldt;
    uint8_t bv1[kSteps];
#pragma unroll
    for (int k = 0; k < kSteps; ++k) bv1[k] = col[r[k]];
    const int jm1 = (int)((m >> 16) & 0x1FFu);
    const uint32_t dlv = (m >> 25) & 1u;
    const int nv = max(0, min(n, wb + kSteps * kWave) - wb);  // valid positions of this wave (a prefix)
    uint32_t lb = 0;
    int nl = 0;
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      const uint32_t b = bv1[k];
      const uint32_t lt = (uint32_t)((int)b - jm1) >> 31;
      const uint32_t ms = (b + 1u) >> 8;
      const uint32_t ok = (uint32_t)(k * kWave + lane < nv);
      const uint32_t left = (lt | (ms & dlv)) & ok;
      lb |= left << k;
      nl += __popcll(__ballot(left != 0u));
    }
    asm volatile("" : "+v"(lb));
    if (lane == 0) { s_wc[0][wv] = nl; s_wc[1][wv] = nv - nl; }
    __syncthreads();
    stamp_.probe(2);
    if (threadIdx.x == 0) {
      int tl = 0, tr = 0;
      for (int k = 0; k < kPW; ++k) { tl += s_wc[0][k]; tr += s_wc[1][k]; }
      const unsigned long long c =
          d.ablate == 12 ? 0ull
                         : atomicAdd(reinterpret_cast<unsigned long long*>(d.cursors + 2 * node),
                                     ((unsigned long long)(uint32_t)tr << 32) | (uint32_t)tl);
      s_wbase[0] = (int32_t)(uint32_t)c;
      s_wbase[1] = (int32_t)(c >> 32);
    }
    __syncthreads();
    stamp_.probe(3);
    int bl = s_wbase[0], br = s_wbase[1];
    for (int k = 0; k < wv; ++k) { bl += s_wc[0][k]; br += s_wc[1][k]; }
    uint32_t pl_ = (uint32_t)(nstart + bl);
    uint32_t pr_ = (uint32_t)(nend - 1 - br);
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      const bool valid = k * kWave + lane < nv;
      const uint32_t left = (lb >> k) & 1u;
      const uint64_t lm = __ballot(left != 0u), vm = __ballot(valid);
      const uint32_t rk_l = mask_rank(lm);
      const uint32_t dst = rk_l + (left ? pl_ : pr_ - (uint32_t)lane);
      if (valid) store_wt(nxt + dst, r[k], (d.wt & 2) != 0);
      const uint32_t cl = (uint32_t)__popcll(lm);
      pl_ += cl;
      pr_ -= (uint32_t)__popcll(vm) - cl;
    }
    return;
  }
  // first range that ends past the wave's first position (uniform binary search over the LDS ends)
  int k0 = 0;
  {
    int lo = 0, hi = nr;  // first k with re[k] > wb
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (__builtin_amdgcn_readfirstlane(s_re[mid]) > wb) hi = mid; else lo = mid + 1;
    }
    k0 = lo;
  }
  // pass 1: each lane's range (uniform walk over the ranges that start inside or before the step), the
  // split feature's bin, the direction; per (wave, range) counts
  // each row's range, packed 8 bits per step (0xFF: routes nowhere) -- 2 VGPRs instead of kSteps (the kernel
  // must stay within 64 VGPRs for two 1024-thread blocks per CU)
  uint32_t klp[(kSteps + 3) / 4];
#pragma unroll
  for (int i = 0; i < (kSteps + 3) / 4; ++i) klp[i] = 0xFFFFFFFFu;
  auto kl_of = [&](int k) -> int {
    const uint32_t v = (klp[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    return v == 0xFFu ? -1 : (int)v;
  };
  uint32_t lbits = 0, inbits = 0;
  uint8_t bv[kSteps];
  // Fast path (nearly every wave: a node's range spans ~10^5 positions): the wave's positions lie inside one
  // range -- every lane's node is k0, no per-lane search. Otherwise each lane binary-searches the ranges
  // from k0 on (the last one starting at or before its position) and checks the range's end.
  const bool one = k0 < nr && __builtin_amdgcn_readfirstlane(s_rs[k0]) <= wb &&
                   __builtin_amdgcn_readfirstlane(s_re[k0]) >= wb + kSteps * kWave;
  if (one) {
    const uint32_t m = __builtin_amdgcn_readfirstlane(s_rm[k0]);
    const uint8_t* col = d.binsT + (int64_t)(m & 0xFFFFu) * d.ldt;
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      klp[k >> 2] &= ~((uint32_t)(0xFFu ^ (uint32_t)k0) << (8 * (k & 3)));
      bv[k] = col[max(r[k], 0)];
    }
    inbits = (1u << kSteps) - 1u;
  } else {
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      const int p = wb + k * kWave + lane;
      int lo = k0, hi = nr - 1, kk = -1;  // last t in [k0, nr) with rs[t] <= p
      while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (s_rs[mid] <= p) { kk = mid; lo = mid + 1; } else hi = mid - 1;
      }
      const bool in = kk >= 0 && p < n && p < s_re[max(kk, 0)];
      if (in) klp[k >> 2] &= ~((uint32_t)(0xFFu ^ (uint32_t)kk) << (8 * (k & 3)));
      inbits |= (in ? 1u : 0u) << k;
      // the split feature's bin: an unconditional load (lanes outside a range read their nearest one's column)
      const uint32_t m = s_rm[max(kk, 0)];
      bv[k] = d.binsT[(int64_t)(m & 0xFFFFu) * d.ldt + max(r[k], 0)];
    }
  }
#pragma unroll
  for (int k = 0; k < kSteps; ++k) {
    const int klk = kl_of(k);
    const uint32_t m = s_rm[max(klk, 0)];
    const uint32_t b = bv[k];
    const int jm1 = (int)((m >> 16) & 0x1FFu);  // j + 1
    const uint32_t lt = (uint32_t)((int)b - jm1) >> 31;
    const uint32_t ms = (b + 1u) >> 8;
    const uint32_t left = (lt | (ms & ((m >> 25) & 1u))) & ((inbits >> k) & 1u);
    lbits |= left << k;
    // per-range counts of this step (uniform loop over the ranges present in it; usually one)
    uint64_t rem = __ballot((inbits >> k) & 1u);
    const uint64_t lm = __ballot(left != 0u);
    while (rem) {
      const int src = __ffsll((unsigned long long)rem) - 1;
      const int kk = __builtin_amdgcn_readlane(klk, src);
      const uint64_t mk = __ballot(klk == kk) & rem;
      if (lane == 0) {
        s_cnt[wv][kk][0] += __popcll(mk & lm);
        s_cnt[wv][kk][1] += __popcll(mk & ~lm);
      }
      rem &= ~mk;
    }
  }
  __syncthreads();
  stamp_.probe(2);
  // one claim per range for the whole block (thread t: range t), then each wave's bases
  if ((int)threadIdx.x < nr) {
    const int t = threadIdx.x;
    int tl = 0, tr = 0;
    for (int w = 0; w < kPW; ++w) { tl += s_cnt[w][t][0]; tr += s_cnt[w][t][1]; }
    if (tl + tr > 0) {
      const unsigned long long c =
          d.ablate == 12 ? 0ull
                         : atomicAdd(reinterpret_cast<unsigned long long*>(d.cursors + 2 * s_rn[t]),
                                     ((unsigned long long)(uint32_t)tr << 32) | (uint32_t)tl);
      int bl = s_rs[t] + (int)(uint32_t)c;                // next left slot
      int br = s_re[t] - 1 - (int)(uint32_t)(c >> 32);    // next right slot (descending)
      for (int w = 0; w < kPW; ++w) {
        const int cl = s_cnt[w][t][0], cr = s_cnt[w][t][1];
        s_cnt[w][t][0] = bl;
        s_cnt[w][t][1] = br;
        bl += cl;
        br -= cr;
      }
    }
  }
  __syncthreads();
  stamp_.probe(3);
  // pass 2: scatter with ballot ranks inside each (step, range)
#pragma unroll
  for (int k = 0; k < kSteps; ++k) {
    const bool in = (inbits >> k) & 1u;
    const uint32_t left = (lbits >> k) & 1u;
    const int klk = kl_of(k);
    uint64_t rem = __ballot(in);
    const uint64_t lm = __ballot(left != 0u);
    while (rem) {
      const int src = __ffsll((unsigned long long)rem) - 1;
      const int kk = __builtin_amdgcn_readlane(klk, src);
      const uint64_t mk = __ballot(klk == kk) & rem;
      const int pl = __builtin_amdgcn_readfirstlane(s_cnt[wv][kk][0]);
      const int pr = __builtin_amdgcn_readfirstlane(s_cnt[wv][kk][1]);
      const uint64_t ml = mk & lm, mr = mk & ~lm;
      if (klk == kk) {
        const int dst = left ? pl + mask_rank(ml) : pr - mask_rank(mr);
        store_wt(nxt + dst, r[k], (d.wt & 2) != 0);
      }
      if (lane == 0) {
        s_cnt[wv][kk][0] = pl + __popcll(ml);
        s_cnt[wv][kk][1] = pr - __popcll(mr);
      }
      rem &= ~mk;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Split evaluation fused with the row partition (one GPU, a level's items <= CUs, levels 0 .. max_depth - 2).
// At small row counts a level is a chain of short launches whose fixed costs dominate (1M rows:
// k_eval ~6.6 us + a ~1.5 us boundary per level), so every block of the partition pass evaluates its
// OWN node (the same eval_core, redundantly: ~2 us of fp64 work per block on its own CU, with the
// node's ~42 KB of histograms hot in L2) and partitions its rows by the result -- one launch per level
// fewer. The item's row ids are loaded before the evaluation (they do not depend on the split), so
// their latency hides behind it. The block holding the node's first item finalises the node record
// and stores its histogram for the children (eval_finalize / eval_core's store, as k_eval does).
// The plan covers every node of the level with rows (a block that finalised its node changes the
// status from active to split / leaf; the other blocks accept any status but kNone). A leaf's blocks
// stop after the evaluation.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool split_decision(const GbdtDev& d, const Cand& best, int nb, int& f, int& j, bool& dl) {
  const float loss = (float)best.gain;
  const bool ok = best.key != 0x7fffffff && loss > 1e-6f && loss >= (float)d.gamma;
  f = best.key >> 10;
  const int r = best.key & 1023;
  if (r < 512) { j = r; dl = false; } else { j = (nb - 1 - (r - 512)) - 1; dl = true; }
  return ok;
}

// A node's split decision as ONE 8-byte granule {tag, decision} (evaluator-block modes): written by the
// node's evaluator block with a write-through store, polled by the node's partition blocks.
__device__ __forceinline__ uint64_t decision_word(uint32_t tag, bool ok, bool fail, int f, int j, bool dl) {
  const uint32_t v = (ok ? 1u : 0u) | (fail ? 2u : 0u) | (dl ? 4u : 0u) | ((uint32_t)(j + 1) & 0x3FFu) << 3 |
                     (uint32_t)f << 13;
  return ((uint64_t)tag << 32) | v;
}

// Every block evaluates its node (the items fit one block per CU):
//   kMode 0: one GPU. 1: data parallel with the level's global histograms already in hist_b (RCCL / the
//   separate IPC exchange kernel); every active node gets an item (possibly empty), so each rank
//   finalises every node of the level, also those it holds no rows of.
// kMode 2, EVALUATOR blocks (data parallel over the fused IPC exchange): blocks 0 .. 2^level - 1
// evaluate one node position each, exactly as k_eval<false, true, true> does (block 0 publishes the
// epoch, every evaluator sums its node's cells over the ranks; node ownership on the deep levels; the
// replica digest), publish its decision granule and finalise it; the blocks after them are the
// partition items, which plan and load their row ids while the evaluation runs and then poll their
// node's granule (one lane, bounded by the group's deadline). One evaluation per node -- no xGMI
// traffic multiplied by the items -- and no k_eval -> k_partition boundary, at any item count: blocks
// are dispatched in index order on every XCD, so the evaluators hold CUs before any item does, and no
// evaluator waits on an item. (The same form for one GPU beyond one block per CU measured slower than
// k_eval + k_partition -- 10M rows 238.6 vs 231.9 ms: the fused kernel's 110 VGPRs hold the partition
// to one block per CU; profiles/round5/eval_blocks_10M.txt.)
template <int kSteps, int kMode>
__global__ __launch_bounds__(1024) void k_eval_part(GbdtDev d, int parity, int64_t zero_next, int level, int chunk,
                                                    int tree, EvalSlots es, uint32_t tag) {
  constexpr bool kDP = kMode != 0;
  constexpr bool kEvalBlocks = kMode == 2;
  constexpr bool kIpc = kMode == 2;
  constexpr int kPW = 16;  // waves
  BlockStamp stamp_(d);
  __shared__ int32_t s_cnt[2][kPW];
  __shared__ int32_t s_base[2];
  __shared__ EvalOut s_out;
  // zero the next level's reduce destination (hist_b of the other parity, or the next IPC send slot;
  // kMode 2: the evaluators do, see below)
  int4* zp = reinterpret_cast<int4*>(d.zero_red ? d.zero_red : d.hist_b[parity ^ 1]);
  const int64_t nz = zero_next / 2;
  if (!kIpc)
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nz; e += (int64_t)gridDim.x * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
  const int nlev = 1 << level;
  const int first = nlev - 1;
  if (kIpc && (int)blockIdx.x < nlev) {  // the evaluator of node first + blockIdx.x
    const int pos = blockIdx.x, n = first + pos;
    const IpcFusedView* iv = d.ipcv + (d.ipc_epoch & 1u);
    const bool owned = d.own_level >= 0 && level >= d.own_level;
    const bool mine = !owned || node_owner(d, level, n, iv->n) == iv->me;
    const bool good = eval_core<false, true, true>(d, level, parity, tree, d.F, es, pos, stamp_, &s_out);
    if (threadIdx.x == 0) {
      if (good) {  // the decision first (the items wait on it; they need nothing else of the finalisation)
        int f = 0, j = -1;
        bool dl = false;
        const bool ok = split_decision(d, s_out.best, s_out.nb, f, j, dl);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(d.dec) + n,
                           (unsigned long long)decision_word(tag, ok, false, f, j, dl), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        eval_finalize<true>(d, level, n, s_out.G, s_out.H, s_out.best, s_out.cut, s_out.nb);
        if (owned) own_publish(d, iv, n);
      } else {
        const Node nd = d.nodes[n];  // a non-owner's copy of the owner's record (own_copy), or inactive
        if (owned && mine && nd.status != kActive) own_publish(d, iv, n);  // (as k_eval: a diverged peer learns)
        const bool failed =
            __hip_atomic_load(iv->myflag + kIpcStickyWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        // Always published: a node that is inactive here has no items, but one this rank planned items
        // for can come back inactive from its owner's record (a diverged replica) -- its items then
        // route no rows (and the replica digest reports the divergence at the next tree) instead of
        // waiting for a decision that never comes.
        const uint64_t w = decision_word(tag, nd.status == kSplit, failed || nd.status == kActive, nd.feat, nd.bin,
                                         nd.default_left != 0);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(d.dec) + n, (unsigned long long)w, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // The next send slot (this epoch - 1's) is zeroed once every peer has published this epoch: a peer
    // then has finished reading its previous contents. The evaluators that exchanged waited for that in
    // eval_core; a non-owner (it waited only for its node's owner) polls the flags once more, after its
    // decision is out. A failed exchange zeroes nothing (the fit is aborted).
    const bool synced =
        mine ? __hip_atomic_load(iv->myflag + kIpcStickyWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u
             : ipc_wait<false>(iv->ftab, iv->n, iv->me, iv->myflag, d.ipc_epoch, iv->err_host, iv->timeout);
    if (!synced) return;
    for (int64_t e = (int64_t)pos * blockDim.x + threadIdx.x; e < nz; e += (int64_t)nlev * blockDim.x)
      zp[e] = make_int4(0, 0, 0, 0);
    return;
  }
  const int item = kEvalBlocks ? (int)blockIdx.x - nlev : (int)blockIdx.x;
  // this block's item: the root's rows are fixed slices; deeper levels' items are planned by every
  // block (block_plan over the level's node table)
  PlanOut pl;
  __shared__ int s_plan[5];
  if (level == 0) {
    const int n = (int)d.n, b = item * chunk;
    const int items = max((n + chunk - 1) / chunk, kDP ? 1 : 0);
    pl = PlanOut{item < items ? 0 : -1, 0, min(b, n), min(n, b + chunk), items};
  } else {
    pl = block_plan<kDP>(1 << level, chunk, item, [&](int e) {
      const Node& n = d.nodes[first + e];
      const int st = n.status, cnt = n.count, start = n.start;  // loaded together (no per-load branch)
      return (st != kNone && (kDP || cnt > 0)) ? PlanEntry{first + e, 0, start, cnt} : PlanEntry{-1, 0, 0, 0};
    }, s_plan);
  }
  if (pl.node < 0) return;
  const int node = pl.node;
  // the item's row ids and the node's range: independent of the split, in flight during the evaluation
  const bool identity = parity == 0 && node == 0;
  const int32_t* cur = d.ridx[parity];
  int32_t* nxt = d.ridx[parity ^ 1];
  const int wv = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int len = pl.end - pl.begin;
  const int per = ((len + kPW - 1) / kPW + kWave - 1) / kWave * kWave;
  const int wb = min(pl.end, pl.begin + wv * per), we = min(pl.end, wb + per);
  int r[kSteps];
  auto load_rows = [&]() {
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      const int i = wb + k * kWave + lane;
      const int ic = max(min(i, pl.end - 1), 0);
      const int rv = identity ? ic : cur[ic];
      r[k] = i < we ? rv : -1;
    }
  };
  const int nstart = d.nodes[node].start, ncount = d.nodes[node].count;
  const bool lead = pl.begin == nstart;  // the node's first item
  int f, j;
  bool dlb, ok;
  load_rows();
  if constexpr (kEvalBlocks) {  // the node's evaluator decides; the row ids are in flight meanwhile
    if (len == 0) return;
    __shared__ uint32_t s_dec;
    if (threadIdx.x == 0) {
      // (bounded: the exchange's deadline; without an exchange 20 s, which no evaluator approaches)
      const IpcFusedView* iv = kIpc ? d.ipcv + (d.ipc_epoch & 1u) : nullptr;
      const uint64_t limit = kIpc ? iv->timeout : 2000000000ull;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t v = 2u;  // failed unless the evaluator's granule arrives
      for (;;) {
        const uint64_t w = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(d.dec) + node,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(w >> 32) == tag) { v = (uint32_t)w; break; }
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
          if (kIpc) ipc_fail(iv->myflag, iv->err_host);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_dec = v;
    }
    __syncthreads();
    const uint32_t v = s_dec;
    if (v & 2u) return;  // the exchange failed (the host watchdog reports it)
    ok = (v & 1u) != 0;
    dlb = (v & 4u) != 0;
    j = (int)((v >> 3) & 0x3FFu) - 1;
    f = (int)(v >> 13);
  } else {
    // every block evaluates its node itself (the histograms are L2-hot; the row ids are in flight)
    eval_core<false, false, kDP, true>(d, level, parity, tree, d.F, es, node - first, stamp_, &s_out, lead);
    __syncthreads();
    const Cand best = s_out.best;
    ok = split_decision(d, best, s_out.nb, f, j, dlb);
    if (lead && threadIdx.x == 0) eval_finalize<kDP>(d, level, node, s_out.G, s_out.H, best, s_out.cut, s_out.nb);
  }
  stamp_.probe(4);
  if (!ok || len == 0) return;  // a leaf (its rows are not routed) or an empty item (block-uniform)
  const uint8_t* col = d.binsT + (int64_t)f * d.ldt;
  uint8_t bv[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; ++k) bv[k] = col[max(r[k], 0)];
  // pass 1 / claim / pass 2: k_partition's integer-arithmetic form
  const int jm1 = j + 1;
  const uint32_t dlv = dlb ? 1u : 0u;
  const int nv = max(0, we - wb);
  uint32_t lbits = 0;
  int nl = 0;
#pragma unroll
  for (int k = 0; k < kSteps; ++k) {
    const uint32_t b = bv[k];
    const uint32_t lt = (uint32_t)((int)b - jm1) >> 31;
    const uint32_t ms = (b + 1u) >> 8;
    const uint32_t okr = ~(uint32_t)r[k] >> 31;
    const uint32_t left = (lt | (ms & dlv)) & okr;
    lbits |= left << k;
    nl += __popcll(__ballot(left != 0u));
  }
  if (lane == 0) { s_cnt[0][wv] = nl; s_cnt[1][wv] = nv - nl; }
  __syncthreads();
  stamp_.probe(5);  // the split bins are in: pass 1 done
  if (threadIdx.x == 0) {
    int tl = 0, tr = 0;
    for (int k = 0; k < kPW; ++k) { tl += s_cnt[0][k]; tr += s_cnt[1][k]; }
    const unsigned long long c = atomicAdd(reinterpret_cast<unsigned long long*>(d.cursors + 2 * node),
                                           ((unsigned long long)(uint32_t)tr << 32) | (uint32_t)tl);
    s_base[0] = (int32_t)(uint32_t)c;
    s_base[1] = (int32_t)(c >> 32);
  }
  __syncthreads();
  stamp_.probe(6);  // the item's ranges are claimed
  int bl = s_base[0], br = s_base[1];
  for (int k = 0; k < wv; ++k) { bl += s_cnt[0][k]; br += s_cnt[1][k]; }
  uint32_t pl_ = (uint32_t)(nstart + bl);
  uint32_t pr_ = (uint32_t)(nstart + ncount - 1 - br);
#pragma unroll
  for (int k = 0; k < kSteps; ++k) {
    const bool valid = r[k] >= 0;
    const uint32_t left = (lbits >> k) & 1u;
    const uint64_t lm = __ballot(left != 0u), vm = __ballot(valid);
    const uint32_t rk_l = mask_rank(lm);
    const uint32_t dst = rk_l + (left ? pl_ : pr_ - (uint32_t)lane);
    if (valid) store_wt(nxt + dst, r[k], (d.wt & 2) != 0);
    const uint32_t cl = (uint32_t)__popcll(lm);
    pl_ += cl;
    pr_ -= (uint32_t)__popcll(vm) - cl;
  }
}

// ------------------------------------------------------------------------------------------
// Host-side trainer context
// ------------------------------------------------------------------------------------------
// RCCL all-reduce hook implemented in comm.cpp
extern "C" int cobalt_comm_allreduce_sum_i64(void* comm, int64_t* buf, int64_t count, hipStream_t stream);
extern "C" int cobalt_comm_allreduce(void* comm, void* buf, int64_t count, int dtype, int op, hipStream_t stream);

struct GbdtCtx {
  GbdtConfig cfg{};
  GbdtDev d{};
  int max_nodes = 0, pairs_max = 0, items_cap = 0;
  size_t lds_hist = 0;
  int applied = 0;         // number of leading trees whose leaves are already in the margins
  int grown = 0;            // number of trees grown so far
  std::vector<void*> allocs;
  // k_eval<false> feature -> (wave, slot) table: 32 slots of 8 bits (0xFF = empty), see eval_assignment
  uint64_t eval_asg[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  EvalSlots eval_slots{};  // the table with each slot's bin count and compact offset (k_eval<false> arguments)
  std::vector<int32_t> hoff_h;  // host copy of d.hoff (sizes k_eval's fused-exchange LDS)
  int fit_first = 0;            // first tree this context grows in the current fit (no replica check)
  int fault_tree = -1;          // fault injection: tree whose root totals are perturbed on this rank
  uint32_t dec_tag = 0;         // k_eval_part<.., 2>: the launch tag of the decision granules (d.dec)
  bool label_pending = false;   // lab31 labels set, to be written into the records by the next grow call
  // the last grow call's plan (cobalt_gbdt_plan): fused IPC exchange, ownership level, wide gradients,
  // resident blocks of the fused k_eval, levels run by the fused evaluation + partition pass (and of them
  // the evaluator-block levels, and those whose grid exceeds one block per CU)
  int32_t plan[7] = {0, -1, 0, 0, 0, 0, 0};
  unsigned* err_pinned = nullptr;  // mapped host word behind d.err_host
  // COBALT_STAMPS=<file>: per-launch in-kernel timing of every grow call, appended to <file>
  const char* stamp_path = nullptr;
  int stamp_cap = 0;
  uint64_t* stamp_buf = nullptr;
  std::vector<const char*> stamp_names;
  // exact external-memory mode (cobalt_gbdt_ox_*): per-row state of the streamed data set
  int64_t ox_n = 0;
  uint16_t* ox_pos = nullptr;   // [ox_n] the row's node (heap index) in the tree being grown
  uint64_t* ox_gh = nullptr;    // [ox_n] packed quantised (g, h) of the tree being grown
  int64_t* ox_slab = nullptr;   // [kOxSlab][pairs_max][slot_elems] per-block partial histograms
  float* ox_margin = nullptr;
  const float* ox_label = nullptr;
  const float* ox_weight = nullptr;
};

// Next launch's stamp slot (0 when stamping is off or the tree is not sampled: d.stamps == nullptr).
static int stamp_next(GbdtCtx* c, const char* name) {
  if (!c->stamp_path || !c->d.stamps) return 0;
  if ((int)c->stamp_names.size() >= c->stamp_cap) { c->d.stamps = nullptr; return 0; }
  c->stamp_names.push_back(name);
  return (int)c->stamp_names.size() - 1;
}
// Launch with a stamp slot (COBALT_STAMPS); arguments as hipLaunchKernelGGL.
#define GLAUNCH(tag, ...)               \
  do {                                  \
    c->d.seq = stamp_next(c, tag);      \
    hipLaunchKernelGGL(__VA_ARGS__);    \
  } while (0)

// Trees whose launches are stamped: every 64th from tree 5 (and tree 0 of short fits).
static bool stamp_tree(GbdtCtx* c, int t) { return c->stamp_path && (t % 64 == 5 || (c->grown < 5 && t == 0)); }

static int stamp_begin(GbdtCtx* c, hipStream_t stream) {
  if (!c->stamp_path) return 0;
  c->stamp_names.clear();
  CK(hipMemsetAsync(c->stamp_buf, 0, (size_t)c->stamp_cap * kStampBlocks * kStampSlot * sizeof(uint64_t), stream));
  return 0;
}

static int stamp_dump(GbdtCtx* c, hipStream_t stream) {
  if (!c->stamp_path || c->stamp_names.empty()) return 0;
  const int n = (int)c->stamp_names.size();
  std::vector<uint64_t> v((size_t)n * kStampBlocks * kStampSlot);
  CK(hipStreamSynchronize(stream));
  CK(hipMemcpy(v.data(), c->stamp_buf, v.size() * 8, hipMemcpyDeviceToHost));
  FILE* f = fopen(c->stamp_path, "a");
  if (!f) return 0;
  fprintf(f, "# launch name first_start last_end last_start blocks probe1..6 (mean ticks after block start)\n");
  for (int i = 0; i < n; ++i) {
    uint64_t st = ~0ull, en = 0, ls = 0, nb = 0;
    double pr[6] = {0, 0, 0, 0, 0, 0};
    int pn[6] = {0, 0, 0, 0, 0, 0};
    for (int b = 0; b < kStampBlocks; ++b) {
      const uint64_t* q = &v[((size_t)i * kStampBlocks + b) * kStampSlot];
      if (!q[0]) continue;
      ++nb;
      st = std::min(st, q[0]);
      ls = std::max(ls, q[0]);
      en = std::max(en, q[1]);
      for (int k = 0; k < 6; ++k)
        if (q[2 + k]) { pr[k] += (double)(q[2 + k] - q[0]); ++pn[k]; }
    }
    fprintf(f, "%d %s %llu %llu %llu %llu", i, c->stamp_names[i], (unsigned long long)(nb ? st : 0),
            (unsigned long long)en, (unsigned long long)ls, (unsigned long long)nb);
    for (int k = 0; k < 6; ++k) fprintf(f, " %.1f", pn[k] ? pr[k] / pn[k] : -1.0);
    fprintf(f, "\n");
  }
  fclose(f);
  return 0;
}

static int pow2_clamp(int64_t v, int lo, int hi) {
  int c = lo;
  while (c < v && c < hi) c *= 2;
  return c;
}
// Work-item sizes: the root level uses the configured chunk (~768 items of 512 threads); deeper
// levels histogram at most ~N/2 rows -> aim for ~1536 items; partition items cover all split rows.
static int chunk_hist(const GbdtDev& d, int level) {
  // COBALT_HIST_CHUNK0 / COBALT_HIST_CHUNK override the root / deeper item sizes (tuning experiments)
  static const int env0 = knob_int(Knob::HistChunk0, 0);
  static const int env1 = knob_int(Knob::HistChunk, 0);
  if (level == 0) return env0 > 0 ? std::min(16384, std::max(512, env0)) : d.chunk;
  if (env1 > 0) return std::min(16384, std::max(512, env1));
  // <= 4096 rows: with the reduce at ~3 us per level, more, smaller items balance the CUs better
  // (10M rows: 295.7 vs 304.8 ms per fit with 8192; 2048 is slower again: 311.8); ~768 items of a
  // level's half of the rows: 1024 up to ~1.57M rows (1M: k_hist 68.5 -> 62.7 us per tree, fit 74.6 ->
  // 72.6 ms), 2048 up to ~3.1M (2.5M: 102.8 -> 100.4 ms vs 4096), 4096 above (5M: 1024 / 2048 slower)
  return pow2_clamp((d.n / 2 + 767) / 768, 1024, 4096);
}
// Partition item size (16-wave blocks, see k_partition); COBALT_PART_CHUNK overrides it (<= 8192).
// (16-wave blocks at every size: 10M rows 234.7 -> 230.6 ms, 5M 150.2 -> 147.3 against the 4-wave
// blocks of rounds 1-2, profiles/round3/ab/ab_part_wide.txt; the 4-wave form is gone since round 5)
static int device_cu_count();
static int chunk_part(const GbdtDev& d) {
  static const int env = knob_int(Knob::PartChunk, 0);
  if (env > 0) return std::min(16 * 8 * kWave, std::max(1024, env / 1024 * 1024));
  // 4096-row items while a level's items fit one block per CU (1M rows: 104.7 vs 106.8 ms per fit with
  // 8192 in round 1), else 8192 (1.25M: 4096-row items ran 306 blocks on 256 CUs; 8192: 82.1 -> 79.5 ms,
  // 2.5M 105.5 -> 104.1; 16384 slower at both; at 10M 4096 / 6144 / 12288 / 16384 243.0 / 234.8 / 256.0
  // / 250.6 vs 231.4 ms)
  return (d.n + 4095) / 4096 <= device_cu_count() ? 4096 : 8192;
}

// Histogram kernels by record shape: FT4 = F rounded up to 4 for 32-byte records with one feature tile
// (<= 24 features), 0 otherwise (generic rows / several tiles; the fused root pass is not used then).
typedef void (*HistKernel)(GbdtDev, int, int, int, int);
typedef void (*GradHistKernel)(GbdtDev, int, int, int);
static int hist_ft4(const GbdtDev& d) {
  return (d.stride == 32 && d.F <= 24 && d.feat_tile >= d.F) ? (d.F + 3) / 4 * 4 : 0;
}
static HistKernel hist_kernel(int ft4, bool pair, bool wide = false) {
  if (wide) switch (ft4) {
    case 4: return k_hist<4, false, true>;
    case 8: return k_hist<8, false, true>;
    case 12: return k_hist<12, false, true>;
    case 16: return k_hist<16, false, true>;
    case 20: return k_hist<20, false, true>;
    case 24: return k_hist<24, false, true>;
    default: return nullptr;
  }
  switch (ft4) {
    case 4: return k_hist<4, false>;
    case 8: return k_hist<8, false>;
    case 12: return k_hist<12, false>;
    case 16: return pair ? k_hist<16, true> : k_hist<16, false>;
    case 20: return pair ? k_hist<20, true> : k_hist<20, false>;
    case 24: return pair ? k_hist<24, true> : k_hist<24, false>;
    default: return k_hist<0, false>;
  }
}
static GradHistKernel grad_hist_kernel(int ft4, bool wide = false) {
  if (wide) switch (ft4) {
    case 4: return k_grad_hist<2, 4, true>;
    case 8: return k_grad_hist<2, 8, true>;
    case 12: return k_grad_hist<2, 12, true>;
    case 16: return k_grad_hist<2, 16, true>;
    case 20: return k_grad_hist<2, 20, true>;
    case 24: return k_grad_hist<2, 24, true>;
    default: return nullptr;
  }
  switch (ft4) {
    case 4: return k_grad_hist<2, 4, false>;
    case 8: return k_grad_hist<2, 8, false>;
    case 12: return k_grad_hist<2, 12, false>;
    case 16: return k_grad_hist<2, 16, false>;
    case 20: return k_grad_hist<2, 20, false>;
    case 24: return k_grad_hist<2, 24, false>;
    default: return nullptr;
  }
}

// Compute units of the current device (256 on MI355X), cached per process. COBALT_CU_BUDGET caps it
// for a rank whose stream owns a CU-masked share of a device shared with other ranks
// (parallel/cumask.py): the launch heuristics then size grids for the CUs the rank really has.
static int device_cu_count() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      n = v;
    if (n <= 0) n = 256;
    const int b = knob_int(Knob::CuBudget, 0);
    if (b > 0) n = std::min(n, b);
  }
  return n;
}

static int dev_alloc(GbdtCtx* c, void** p, size_t bytes) {
  CK(hipMalloc(p, bytes < 16 ? 16 : bytes));
  c->allocs.push_back(*p);
  return 0;
}

COBALT_API int cobalt_gbdt_create(const GbdtConfig* cfg, void** out) {
  if (cfg->max_depth < 1 || cfg->max_depth > 10) return -1;
  if (cfg->chunk < 64 || cfg->chunk > 16384) return -2;
  if (cfg->row_stride % 16 != 0 || cfg->row_stride < ((cfg->n_feat + 7) / 8) * 8 + 8) return -3;
  if (cfg->feat_tile % 4 != 0 || cfg->feat_tile <= 0 || cfg->feat_tile > 64) return -4;
  if (cfg->n_rows >= (int64_t)INT32_MAX) return -5;
  // wide gradients: 32-byte records with one feature tile (the fast histogram path) only
  const int gbits = cfg->grad_bits > 0 ? cfg->grad_bits : 17;
  if (gbits != 17 && gbits != 25) return -6;
  const bool wide = gbits == 25;
  if (wide && (cfg->row_stride != 32 || cfg->n_feat > 24 || cfg->feat_tile < cfg->n_feat)) return -6;
  GbdtCtx* c = new GbdtCtx();
  c->cfg = *cfg;
  const int F = cfg->n_feat;
  const int64_t N = cfg->n_rows;
  c->max_nodes = (1 << (cfg->max_depth + 1)) - 1;
  c->pairs_max = 1 << (cfg->max_depth - 1);
  {
    GbdtDev tmp{};
    tmp.n = N;
    tmp.chunk = cfg->chunk;
    const int ch = std::min(chunk_hist(tmp, 0), chunk_hist(tmp, 1));
    c->items_cap = std::max(ceil_div(N, ch), ceil_div(N, chunk_part(tmp))) + (1 << cfg->max_depth) + 8;
  }
  GbdtDev& d = c->d;
  d.n = N;
  d.ldt = N;
  d.row_offset = cfg->row_offset;
  d.F = F;
  d.stride = cfg->row_stride;
  d.goff = ((F + 7) / 8) * 8;
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
  d.ablate = knob_int(Knob::HistAblate, 0);
  // write-through slabs always (10M rows: reduce gaps 14.2 -> 12.0 us per tree, fit 243.7 -> 243.2 ms); write-through
  // row ids below 4M rows only (1M: 240.2 -> 237.4 us per tree with both; at 10M the partition itself
  // slows 210 -> 228 us per tree for 10 us of shorter histogram gaps). COBALT_WT overrides.
  // (bit 2, the root pass's (g, h): 1.25M rows 77.1 / 77.3 -> 76.4 / 76.6 ms per fit, 10M 233.9 / 233.5 ->
  // 233.6 / 233.1, same box, profiles/round6/ab_wt_root.txt -- the kernel-end write-back of the dirty record
  // lines was the 3-4.5 us gap after the root pass)
  d.wt = knob_int(Knob::WriteThrough, N < 4000000 ? 7 : 5);
  // Data parallel: every rank histograms the child with the smaller GLOBAL hessian (k_eval's choice,
  // identical on all ranks), so the level's all-reduce sums the same child everywhere. On one GPU the
  // locally smaller row count (+2% histogram time with the hessian rule).
  d.by_hess = cfg->comm ? 1 : 0;
  // lane-pair record gathers in the histogram levels (16 < F <= 24): default on (10M rows: 260.4 ->
  // 252.0 ms per fit, 1M: 90.9 -> 87.9 ms); COBALT_HIST_PAIR=0 selects the one-lane-per-row kernel
  d.hist_pair = wide ? 0 : knob_int(Knob::HistPair, 1);
  d.wide = wide ? 1 : 0;
  c->lds_hist = (size_t)cfg->feat_tile * kMaxBins * sizeof(uint64_t) * (wide ? 2 : 1);
  int rc = 0;
  const size_t hist_bytes = (size_t)c->pairs_max * d.slot_elems * sizeof(int64_t);
  if ((rc = dev_alloc(c, (void**)&d.ridx[0], N * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.ridx[1], N * sizeof(int32_t)))) return rc;
  for (int k = 0; k < 2; ++k) {
    // + one int64 pair: the level-0 replica-digest cell after the root slot (data parallel)
    if ((rc = dev_alloc(c, (void**)&d.hist_b[k], hist_bytes + 2 * sizeof(int64_t)))) return rc;
    if ((rc = dev_alloc(c, (void**)&d.hist_s[k], 2 * hist_bytes))) return rc;  // node-indexed
  }
  if ((rc = dev_alloc(c, (void**)&d.nodes_buf[0], c->max_nodes * sizeof(Node)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.nodes_buf[1], c->max_nodes * sizeof(Node)))) return rc;
  d.nodes = d.nodes_buf[0];
  d.prev_nodes = d.nodes_buf[1];
  if ((rc = dev_alloc(c, (void**)&d.trees, (size_t)cfg->max_trees * c->max_nodes * sizeof(Node)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.items_h, c->items_cap * sizeof(WorkItem)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.counters, 16 * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.cursors, 2 * c->max_nodes * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.cand, (size_t)c->pairs_max * 64 * sizeof(CandRec)))) return rc;
  if (cfg->comm) {
    // replica check: per-tree-parity digest accumulators and the mapped host error word
    if ((rc = dev_alloc(c, (void**)&d.dig, 4 * sizeof(int64_t)))) return rc;
    CK(hipMemset(d.dig, 0, 4 * sizeof(int64_t)));
    CK(hipHostMalloc((void**)&c->err_pinned, 64, hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->err_pinned, 0, 64);
    CK(hipHostGetDevicePointer((void**)&d.err_host, c->err_pinned, 0));
    d.world = cfg->world_size;
  }
  if ((rc = dev_alloc(c, (void**)&d.dec, c->max_nodes * sizeof(uint64_t)))) return rc;
  CK(hipMemset(d.dec, 0, c->max_nodes * sizeof(uint64_t)));  // (tags start at 1)
  if ((rc = dev_alloc(c, (void**)&d.slab, (size_t)c->items_cap * F * kMaxBins * sizeof(uint64_t) * (wide ? 2 : 1))))
    return rc;
  if ((rc = dev_alloc(c, (void**)&d.slab_tot, (size_t)c->items_cap * 2 * sizeof(int64_t)))) return rc;
  const int ntiles = ceil_div(F, cfg->feat_tile);
  if ((rc = dev_alloc(c, (void**)&d.layout, F * sizeof(int2)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.hoff, (F + 1) * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&d.tile_entries, ntiles * sizeof(int32_t)))) return rc;
  d.stamps = nullptr;
  d.seq = 0;
  if (knob_str(Knob::Stamps)) {
    c->stamp_path = knob_str(Knob::Stamps);
    c->stamp_cap = 512;
    if ((rc = dev_alloc(c, (void**)&c->stamp_buf, (size_t)c->stamp_cap * kStampBlocks * kStampSlot * sizeof(uint64_t))))
      return rc;
  }
  *out = c;
  return 0;
}

// Feature -> (wave, slot) table of k_eval<false> (F <= 32; 16 waves x 2 slots). Longest-processing-
// time first over chunk steps (ceil(nb / 64), 1..4): each feature goes to the least-loaded SIMD that
// still has a free slot (wave w runs on SIMD w mod 4), on its least-loaded wave. The 20 deployed
// features by index order put 11 chunk steps on one SIMD (mean 6.5); the table evens that out. The
// candidate keys, not the wave, order ties: the trees do not depend on the table.
// (index order -- feature f on wave f mod 16 -- measured 57.2 vs 51.7 us of k_eval per tree at 1M.)
static void eval_assignment(const std::vector<int32_t>& nb, uint64_t out[4]) {
  const int F = (int)nb.size();
  uint8_t slot[32];
  memset(slot, 0xFF, sizeof(slot));
  if (F <= 32) {
    std::vector<int> order(F), steps(F);
    for (int f = 0; f < F; ++f) {
      order[f] = f;
      steps[f] = std::max(1, ceil_div(std::max(1, std::min(256, nb[f])), kWave));
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return steps[a] > steps[b]; });
    int simd_load[4] = {0, 0, 0, 0}, wave_load[16] = {0}, wave_cnt[16] = {0};
    for (int f : order) {
      int bs = -1;
      for (int s = 0; s < 4; ++s) {
        const bool free = wave_cnt[s] < 2 || wave_cnt[s + 4] < 2 || wave_cnt[s + 8] < 2 || wave_cnt[s + 12] < 2;
        if (free && (bs < 0 || simd_load[s] < simd_load[bs])) bs = s;
      }
      int bw = -1;
      for (int w = bs; w < 16; w += 4)
        if (wave_cnt[w] < 2 && (bw < 0 || wave_load[w] < wave_load[bw] ||
                                (wave_load[w] == wave_load[bw] && wave_cnt[w] < wave_cnt[bw])))
          bw = w;
      slot[bw * 2 + wave_cnt[bw]++] = (uint8_t)f;
      simd_load[bs] += steps[f];
      wave_load[bw] += steps[f];
    }
  }
  for (int k = 0; k < 4; ++k) {
    uint64_t w = 0;
    for (int j = 0; j < 8; ++j) w |= (uint64_t)slot[k * 8 + j] << (8 * j);
    out[k] = w;
  }
}

COBALT_API int cobalt_gbdt_set_data(void* h, uint8_t* bins, const uint8_t* binsT, const float* cuts,
                                    const int32_t* nbins, const float* label, const float* weight,
                                    float* margin, const uint8_t* fmask) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  c->d.bins = bins;
  c->d.binsT = binsT;
  c->d.cuts = cuts;
  c->d.nbins = nbins;
  c->d.label = label;
  c->d.weight = weight;
  c->d.ylab = 0;
  c->d.lab31 = 0;
  c->label_pending = false;
  c->d.margin = margin;
  c->d.fmask = fmask;
  // Histogram LDS layout from the per-feature bin counts (one small synchronous copy per fit).
  const int F = c->d.F, ft = c->d.feat_tile, ntiles = ceil_div(F, ft);
  std::vector<int32_t> nb(F);
  CK(hipMemcpy(nb.data(), nbins, F * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int2> lay(F);
  std::vector<int32_t> ent(ntiles, 0);
  // Per-lane copies of a low-cardinality feature, capped: with 32, lanes l and l + 32 share a copy but
  // sit in different LDS lane groups of a wave64 access, so the atomics stay conflict-free while the
  // flush sums half as many copies as 64 (10M: 253.4 -> 250.3 ms per fit, 1M: 87.1 -> 85.7). At most
  // 16 since round 3 -- same-address collisions of 4 lanes traded for a quarter of the flush work (two same-box rounds at 1 / 1.25 / 2.5 / 10M rows: 0.3-0.8 ms per fit faster each,
  // profiles/round3/ab/ab_copy_shift4.txt). COBALT_MAX_COPY_SHIFT overrides the log2 (0..6).
  const int max_sh = std::min(6, std::max(0, knob_int(Knob::MaxCopyShift, 4)));
  int max_ent = 0;
  for (int t = 0; t < ntiles; ++t) {
    int off = 0;
    for (int f = t * ft; f < std::min(F, (t + 1) * ft); ++f) {
      const int b = std::max(1, std::min(256, nb[f]));
      // copies = 2^sh with (nb + 1) * copies <= 256: the clamped missing code (cell nb, see
      // hist_add_rec32) stays inside the feature's cells; a 256-bin feature has one copy
      int sh = 0;
      while (sh < max_sh && ((b + 1) << (sh + 1)) <= kMaxBins) ++sh;
      // bit 3: a 256-bin feature (no missing values; code 255 is its real bin 255)
      lay[f] = make_int2((f - t * ft) * kMaxBins, sh | (b >= 256 ? 8 : 0));
      off += kMaxBins;
    }
    ent[t] = off;
    max_ent = std::max(max_ent, off);
  }
  CK(hipMemcpy(c->d.layout, lay.data(), F * sizeof(int2), hipMemcpyHostToDevice));
  std::vector<int32_t> hoff(F + 1, 0);
  for (int f = 0; f < F; ++f) hoff[f + 1] = hoff[f] + std::max(1, std::min(256, nb[f]));
  CK(hipMemcpy(c->d.hoff, hoff.data(), (F + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
  c->hoff_h = hoff;
  eval_assignment(nb, c->eval_asg);
  for (int k = 0; k < 32; ++k) {
    const uint32_t f = (uint32_t)((c->eval_asg[k / 8] >> (8 * (k % 8))) & 0xFFu);
    c->eval_slots.w[k] = (f == 0xFFu || (int)f >= F)
                             ? 0xFFu
                             : f | ((uint32_t)std::min(std::max(nb[f], 0), 511) << 8) | ((uint32_t)hoff[f] << 17);
  }
  c->d.ncells = hoff[F];
  c->d.slot_elems = (int64_t)(hoff[F] + 1) * 2;
  CK(hipMemcpy(c->d.tile_entries, ent.data(), ntiles * sizeof(int32_t), hipMemcpyHostToDevice));
  const bool wide = c->d.wide != 0;
  c->lds_hist = (size_t)(max_ent + kWave) * sizeof(uint64_t) * (wide ? 2 : 1);
  if (c->lds_hist > 64 * 1024) {
    for (int v = 0; v < 3; ++v)
      if (HistKernel k = hist_kernel(hist_ft4(c->d), v == 1, v == 2))
        CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_hist));
  }
  const size_t grad_hist_lds = c->lds_hist + (size_t)c->max_nodes * kWalkNodeBytes;
  if (grad_hist_lds > 64 * 1024 && grad_hist_kernel(hist_ft4(c->d), wide))
    CK(hipFuncSetAttribute((const void*)grad_hist_kernel(hist_ft4(c->d), wide),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)grad_hist_lds));
  return 0;
}

static void launch_eval_part(int steps, int mode, dim3 grid, size_t lds, hipStream_t stream, const GbdtDev& d,
                             int parity, int64_t zero_next, int level, int chunk, int tree, const EvalSlots& es,
                             uint32_t tag) {
#define EP_LAUNCH(S, M) \
  hipLaunchKernelGGL((k_eval_part<S, M>), grid, dim3(1024), lds, stream, d, parity, zero_next, level, chunk, tree, es, tag)
  if (steps <= 4) {
    switch (mode) {
      case 0: EP_LAUNCH(4, 0); break;
      case 1: EP_LAUNCH(4, 1); break;
      default: EP_LAUNCH(4, 2); break;
    }
  } else if (steps <= 6 && mode <= 1) {  // (1.25M rows: 6144-row items; the 8-step form spills 2 VGPRs)
    if (mode == 0) EP_LAUNCH(6, 0); else EP_LAUNCH(6, 1);
  } else {
    switch (mode) {
      case 0: EP_LAUNCH(8, 0); break;
      case 1: EP_LAUNCH(8, 1); break;
      default: EP_LAUNCH(8, 2); break;
    }
  }
#undef EP_LAUNCH
}

// Enqueue `n_trees` boosting rounds starting at tree index `t0`. No host synchronisation.
// `sampled`: the row records already hold the (reweighted) gradient pairs of this tree's rows --
// the external-memory path, where k_ooc_page wrote a fresh sample -- so the tree starts with a
// node-table reset + a plain root histogram instead of the gradient pass, and no margins are kept.
static int grow_impl(GbdtCtx* c, int t0, int n_trees, hipStream_t stream, bool sampled) {
  GbdtDev& d = c->d;
  const int D = d.max_depth;
  const int grad_grid = std::min(ceil_div(d.n, 256), 256 * 16);
  const int ftiles = ceil_div(d.F, d.feat_tile);
  const size_t tree_lds = (size_t)c->max_nodes * 8;
  const size_t walk_lds = (size_t)c->max_nodes * kWalkNodeBytes;  // k_grad_hist's staged tree (stage_walk)
  if (t0 != c->grown) return -11;  // trees must be grown in order
  if (int rc = stamp_begin(c, stream)) return rc;
  // any native communicator turns on the data-parallel protocol (a 1-rank one exercises it on 1 GPU)
  const bool dp = c->cfg.comm != nullptr;
  d.dp = dp ? 1 : 0;
  // IPC one-shot group (ipccomm.hip): the reduce accumulates into this rank's exported send slot and
  // one exchange kernel per level writes the all-reduced histograms into hist_b (no RCCL call)
  CobaltComm* const cc = static_cast<CobaltComm*>(c->cfg.comm);
  const bool ipc = dp && cc->kind == 2;
  d.hist_red = nullptr;
  if (ipc) {
    if (ipc_capacity(cc) < ((int64_t)c->pairs_max * d.slot_elems + 2) * (int64_t)sizeof(int64_t)) {
      comm_set_error("ipc: slot capacity below one level of histograms (raise COBALT_IPC_SLOT_MB)");
      return -14;
    }
    if (int rc = ipc_zero_send(cc, d.slot_elems * (int64_t)sizeof(int64_t), stream)) return rc;
  }
  // gradients + root histogram in one pass (32-byte records, one feature tile)
  const int ft4 = hist_ft4(d);
  const bool fuse_root = !sampled && ft4 > 0 && ftiles == 1 && (d.ablate == 0 || d.ablate >= 10);
  if (d.wide && sampled) return -15;  // (the sampled pages carry 17-bit pairs)
  // margins in the row records for this call (GbdtDev::mrec) from 4M rows: 10M 231.9 / 234.2 vs 235.9 / 235.9
  // ms per fit; at 1.25M the copy-in / copy-out launches and the lost write-through of (g, h) cost more
  // (78.2 / 78.9 vs 77.2 / 77.0; profiles/round6/ab_margin_in_record.txt). COBALT_MARGIN_IN_RECORD: 0 off,
  // 2 at any size
  static const int env_mrec = knob_int(Knob::MarginInRecord, 1);
  d.mrec = (env_mrec != 0 && d.lab31 && fuse_root && d.n > 0 && (env_mrec == 2 || d.n >= 4000000)) ? 1 : 0;
  {
    const dim3 g1(std::max(1, std::min(ceil_div(d.n, 256), 4096)));
    if (c->label_pending && d.mrec)
      hipLaunchKernelGGL(k_margin_label_in, g1, dim3(256), 0, stream, d.bins, d.margin, d.label, d.n);
    else if (c->label_pending)
      hipLaunchKernelGGL(k_put_label31, g1, dim3(256), 0, stream, d.bins, d.label, d.n);
    else if (d.mrec)
      hipLaunchKernelGGL(k_margin_in, g1, dim3(256), 0, stream, d.bins, d.margin, d.n);
    if (c->label_pending || d.mrec) CK_LAUNCH();
    c->label_pending = false;
  }
  // grouped split evaluation: features per block (0 = one 1024-thread block per node); at most 64
  // groups per node, at most 32 features per group (16 waves x 2). COBALT_EVAL_FG overrides.
  static const int env_fg = knob_int(Knob::EvalFg, -1);
  int eval_fg = env_fg >= 0 ? env_fg : (d.F > 32 ? 8 : 0);
  if (eval_fg == 0 && d.F > 32) eval_fg = 8;  // one k_eval block evaluates at most 32 features
  if (eval_fg > 0) eval_fg = std::min(32, std::max(eval_fg, ceil_div(d.F, 64)));
  // IPC exchange fused into the split evaluation (k_eval publishes, waits and sums the ranks' slots
  // itself: one launch per level fewer); COBALT_IPC_FUSED=0 keeps the separate exchange kernel
  const int env_ipc_fused = knob_int(Knob::IpcFused, 1);
  // LDS of the fused k_eval: the block's cells (+ the totals cell) summed over the ranks
  int fused_cells = c->d.ncells;
  if (eval_fg > 0) {
    fused_cells = 0;
    for (int f0 = 0; f0 < d.F; f0 += eval_fg)
      fused_cells = std::max(fused_cells, c->hoff_h[std::min(d.F, f0 + eval_fg)] - c->hoff_h[f0]);
  }
  const size_t fused_lds = (size_t)(fused_cells + 2) * 16;  // + the totals and the level-0 digest cells
  // Co-residency guard. The fused exchange waits inside k_eval: every block polls the peers' epoch flags
  // (each published by block 0 of that rank's launch) and, under node ownership, the owner's record of
  // the SAME block index -- waits on lower-or-equal block indices of the peers' launches, which in-order
  // dispatch starts first, so progress does not need a whole grid resident. The launch is still kept to
  // what this rank's CUs hold at once (occupancy x the CUs of its stream, COBALT_CU_BUDGET on a CU-masked
  // share of a shared device): a deeper level's grid than that runs the separate exchange kernel instead.
  int resident = 0;
  if (ipc) {
    int per_cu = 0;
    const void* kf = eval_fg > 0 ? (const void*)k_eval<true, true, true> : (const void*)k_eval<false, true, true>;
    const int threads = eval_fg > 0 ? ceil_div(eval_fg, 2) * kWave : 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, threads, fused_lds) == hipSuccess)
      resident = per_cu * device_cu_count();
  }
  const int deepest_grid = (1 << (D - 1)) * (eval_fg > 0 ? ceil_div(d.F, eval_fg) : 1);
  const bool ipc_fused = ipc && env_ipc_fused != 0 && fused_lds <= 65536 && resident >= deepest_grid;
  d.ipc_epoch = 0;
  d.ipcv = ipc_fused ? ipc_device_views(cc) : nullptr;
  // Split evaluation fused into the partition pass (k_eval_part): one launch per level fewer.
  //  * While a level's items fit one 1024-thread block per CU, every partition block evaluates its node
  //    itself (modes 0 / 1; 1M rows: 248.0 -> 239.3 us per tree in the stamps). Under data parallelism
  //    that needs the level's global histograms in hist_b first (RCCL, or the separate IPC exchange).
  //  * Beyond that k_eval + k_partition (a second evaluation per CU cost more than it saved: 1.25M
  //    87.0 -> 96.3 ms per fit in round 3; the evaluator-block form below, 10M 238.6 vs 231.9 ms).
  //  * Over the fused IPC exchange, at every level: the evaluator-block form (mode 2): one evaluating
  //    block per node, the items wait for their node's decision granule (1.25M through a 1-rank IPC
  //    group: 86.3 vs 89.0 ms with k_eval + k_partition).
  // COBALT_EVAL_PART=0 disables both (k_eval + k_partition), 2 forces the every-block form on one GPU;
  // COBALT_EVAL_BLOCKS=0 disables the evaluator-block form.
  static const int env_ep = knob_int(Knob::EvalPart, 1);
  static const int env_eb = knob_int(Knob::EvalBlocks, 1);
  const int ep_steps = ceil_div(chunk_part(d), 16 * kWave);
  bool eb_ok = env_eb != 0;  // (over the fused exchange: a CU holds the kernel with the exchange's LDS)
  if (ipc_fused && eb_ok) {
    int per_cu = 0;
    eb_ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_eval_part<8, 2>, 1024, fused_lds) ==
                hipSuccess && per_cu >= 1;
  }
  // node ownership (see node_owner): over the fused exchange (k_eval, or k_eval_part's evaluator blocks),
  // on the three deepest split levels (where the exchange volume is: 56 of a depth-7 tree's 64 pairs;
  // the copy costs the other ranks one more remote round trip, not worth it for a level's few nodes),
  // and never before a level with a node per rank. COBALT_DP_OWNER=0: every rank evaluates every node
  static const int env_owner = knob_int(Knob::DpOwner, 1);
  d.own_level = -1;
  if (ipc_fused && env_owner && d.world > 1 && eval_fg == 0 && c->max_nodes <= kIpcDecNodes) {
    int l0 = 0;
    while ((1 << l0) < d.world) ++l0;
    l0 = std::max(l0, D - 3);
    d.own_level = l0 < D ? l0 : -1;
  }
  const bool eval_part = env_ep != 0 && (!ipc_fused || eb_ok) && eval_fg == 0 && ep_steps <= 8 && d.F <= 32;
  // A level's fused pass: {item rows (0: separate k_eval + k_partition), mode}. Every-block form: the
  // smallest item (1024-row steps from 4096) whose grid -- items + one partial item per node -- is one
  // block per CU (a second round of blocks doubles the level; 1.25M rows: 6144 at every level).
  // Evaluator-block form: the same rule with one more block per node while it fits, else chunk_part.
  auto ep_plan = [&](int level, int& mode) -> int {
    mode = 0;
    if (!eval_part || level + 1 >= D) return 0;
    const int cus = device_cu_count();
    const int extra = (ipc_fused ? 2 : 1) << level;
    for (int ch = std::min(4096, chunk_part(d)); ch <= 8192; ch += 1024)
      if (ceil_div(d.n, ch) + extra <= cus) {
        mode = ipc_fused ? 2 : (dp ? 1 : 0);
        return ch;
      }
    if (ipc_fused) { mode = 2; return chunk_part(d); }
    return (env_ep == 2 && !dp) ? 8192 : 0;
  };
  c->plan[0] = ipc_fused ? 1 : 0;
  c->plan[1] = d.own_level;
  c->plan[2] = d.wide;
  c->plan[3] = resident;
  c->plan[4] = 0;  // levels run by the fused evaluation + partition pass (bit mask)
  c->plan[5] = 0;  // ... of them in the evaluator-block form
  c->plan[6] = 0;  // ... of those, levels whose grid (evaluators + items) exceeds one block per CU: the items
                   // past the resident ones start as earlier blocks retire (in-order dispatch, evaluators first)
  for (int level = 0; level + 1 < D; ++level) {
    int m = 0;
    const int ch = ep_plan(level, m);
    if (ch > 0) {
      c->plan[4] |= 1 << level;
      if (m >= 2) c->plan[5] |= 1 << level;
      if (m >= 2 && ceil_div(d.n, ch) + (2 << level) > device_cu_count()) c->plan[6] |= 1 << level;
    }
  }
  d.zero_red = nullptr;
  // root items of the fused pass: <= 8192 rows (more blocks in flight than the 16384-row k_hist items);
  // COBALT_ROOT_CHUNK overrides (tuning experiments; multiple of 64 in [1024, 16384])
  static const int env_root = knob_int(Knob::RootChunk, 0);
  // (never more root items than the work-item buffers hold)
  const int root_min = (int)((ceil_div(d.n, (int64_t)c->items_cap - 8) + 63) / 64 * 64);
  // Fused root pass: whole rounds of resident blocks (2 per CU at 95 VGPRs x 512 threads) of ~8k rows;
  // a partial last round idles CUs (10M rows: 8192-row items = 2.4 rounds, 9792-row items = 2 rounds:
  // 167.5 -> 158.3 us per tree in the stamps)
  int root_rule = std::min(chunk_hist(d, 0), 8192);
  if (fuse_root) {
    const int64_t res = 2LL * device_cu_count();
    const int64_t rounds = std::max<int64_t>(1, (d.n + res * 4096) / (res * 8192));  // nearest to n / (res * 8192)
    root_rule = (int)std::min<int64_t>(16384, std::max<int64_t>(1024, (ceil_div(d.n, rounds * res) + 63) / 64 * 64));
  }
  const int root_chunk = std::max(root_min, env_root > 0 ? std::min(16384, std::max(1024, env_root / 64 * 64))
                                                         : root_rule);
  // COBALT_PART_POS=0: node-ordered partition items (k_partition) instead of position-ordered blocks
  const bool part_pos = knob_int(Knob::PartPos, 1) != 0;
  // Per tree: grad (+ root histogram, node-table init, archive/apply of the previous tree), then per
  // level: hist -> reduce -> [data parallel: the histogram collective] -> eval [-> partition], or
  // hist -> reduce [-> collective] -> the fused evaluation + partition pass; the last split level's
  // children are finalised by its evaluation.
  for (int t = t0; t < t0 + n_trees; ++t) {
    if (t >= c->cfg.max_trees) return -10;
    d.nodes = d.nodes_buf[t & 1];
    d.prev_nodes = d.nodes_buf[(t + 1) & 1];
    d.dig_slot = t & 1;
    d.dig_check = t > c->fit_first ? 1 : 0;
    d.corrupt = t == c->fault_tree ? 1 : 0;
    d.stamps = stamp_tree(c, t) ? c->stamp_buf : nullptr;
    const int apply = (t >= 1 && c->applied == t - 1) ? t - 1 : -1;  // prediction-cache update
    // the root pass zeroes the root's reduce destination (under the fused exchange: the next send slot)
    d.zero_red = ipc_fused ? static_cast<int64_t*>(ipc_send_buffer(cc)) : nullptr;
    if (sampled)
      GLAUNCH("k_tree_begin", k_tree_begin, dim3(std::max(1, std::min(64, ceil_div(d.slot_elems / 2, 256)))), dim3(256), 0,
              stream, d);
    else if (fuse_root)
      GLAUNCH("k_grad_hist", grad_hist_kernel(ft4, d.wide != 0), dim3(ceil_div(d.n, root_chunk)), dim3(d.wide ? 1024 : 512), c->lds_hist + walk_lds,
              stream, d, t, apply, root_chunk);
    else
      GLAUNCH("k_grad", k_grad, dim3(std::max(grad_grid, 1)), dim3(256), tree_lds, stream, d, t, apply);
    if (apply >= 0 && !sampled) c->applied = t;
    CK_LAUNCH();
    for (int level = 0; level < D; ++level) {
      const int parity = level & 1;
      // this level's evaluation runs in the partition pass (k_eval_part) with items of ep_ch rows
      int ep_mode = 0;
      const int ep_ch = ep_plan(level, ep_mode);
      const bool ep_level = ep_ch > 0;
      d.ep_chunk = ep_ch;
      d.ep_zero = dp ? 1 : 0;
      const int slots = level == 0 ? 1 : (1 << (level - 1));
      const int chh = (level == 0 && fuse_root) ? root_chunk : chunk_hist(d, level);
      // with the row-count rule every pair builds its smaller child (<= half the parent's rows), so the
      // level's items number at most ceil(n / 2 / chunk) + one partial item per pair: half the grid
      // (and half the reduce grid) of the all-rows bound, fewer blocks that only plan and exit. The
      // hessian rule (data parallel) may build the larger child: all-rows bound.
      const int ub = (level > 0 && !d.by_hess) ? ceil_div((d.n + 1) / 2, chh) + (1 << (level - 1)) + 1
                                               : ceil_div(d.n, chh) + (1 << level);
      if (!(level == 0 && fuse_root))  // the fused gradient kernel already built the root histogram
        GLAUNCH("k_hist", hist_kernel(ft4, d.hist_pair != 0, d.wide != 0), dim3(ub, ftiles), dim3(d.wide ? kHistThreadsWide : kHistThreads), c->lds_hist,
                stream, d, parity, t, level, chh);
      d.hist_red = ipc ? static_cast<int64_t*>(ipc_send_buffer(cc)) : nullptr;
      const dim3 rgrid(ceil_div(ub, kRedItems), ceil_div((int64_t)d.ncells + 1, 256));
      const int rn = std::min(ub, c->items_cap);
      // (the row-count bound of the items, for the reduce blocks past it under the hessian rule)
      const int likely = (level > 0 && d.by_hess) ? ceil_div((d.n + 1) / 2, chh) + (1 << (level - 1)) + 1 : rn;
      if (dp)
        GLAUNCH("k_hist_reduce", k_hist_reduce<true>, rgrid, dim3(256), 0, stream, d, parity, rn, level, likely);
      else
        GLAUNCH("k_hist_reduce", k_hist_reduce<false>, rgrid, dim3(256), 0, stream, d, parity, rn, level, likely);
      CK_LAUNCH();
      if (dp) {  // every rank built the globally chosen child (hessian rule): all-reduced as is
        int rc;
        // level 0 carries the replica-digest cell after the root slot (see GbdtDev::dig)
        const int64_t count = (int64_t)slots * d.slot_elems + (level == 0 ? 2 : 0);
        if (ipc_fused) {  // k_eval exchanges this epoch itself
          d.ipc_epoch = ipc_next_epoch(cc);
          rc = 0;
        } else if (ipc) {  // the exchange also zeroes the next level's send slot (next tree's root after the last)
          const int64_t next_slots = level + 1 < D ? (1 << level) : 1;
          rc = ipc_exchange(cc, d.hist_b[parity], count, 0, 0, next_slots * d.slot_elems * (int64_t)sizeof(int64_t),
                            stream);
        } else {
          rc = cobalt_comm_allreduce_sum_i64(c->cfg.comm, d.hist_b[parity], count, stream);
        }
        if (rc) return rc;
      }
      if (ep_level) {
      } else if (eval_fg > 0) {  // features in groups of eval_fg over several CUs, then a per-node reduction
        const int ng = ceil_div(d.F, eval_fg);
        const dim3 eg(1 << level, ng), eb(ceil_div(eval_fg, 2) * kWave);
        if (d.ipc_epoch)
          GLAUNCH("k_eval", (k_eval<true, true, true>), eg, eb, fused_lds, stream, d, level, parity, t, eval_fg, EvalSlots{});
        else if (dp)
          GLAUNCH("k_eval", (k_eval<true, false, true>), eg, eb, 0, stream, d, level, parity, t, eval_fg, EvalSlots{});
        else
          GLAUNCH("k_eval", (k_eval<true, false, false>), eg, eb, 0, stream, d, level, parity, t, eval_fg, EvalSlots{});
        if (dp)
          GLAUNCH("k_eval_finish", k_eval_finish<true>, dim3(1 << level), dim3(kWave), 0, stream, d, level, parity, ng);
        else
          GLAUNCH("k_eval_finish", k_eval_finish<false>, dim3(1 << level), dim3(kWave), 0, stream, d, level, parity, ng);
      } else {
        if (d.ipc_epoch)
          GLAUNCH("k_eval", (k_eval<false, true, true>), dim3(1 << level), dim3(1024), fused_lds, stream, d, level, parity,
                  t, d.F, c->eval_slots);
        else if (dp)
          GLAUNCH("k_eval", (k_eval<false, false, true>), dim3(1 << level), dim3(1024), 0, stream, d, level, parity, t,
                  d.F, c->eval_slots);
        else
          GLAUNCH("k_eval", (k_eval<false, false, false>), dim3(1 << level), dim3(1024), 0, stream, d, level, parity, t,
                  d.F, c->eval_slots);
      }
      if (level + 1 < D) {  // the last split level's children are leaves: no row lists needed
        const int chp = ep_level ? ep_ch : chunk_part(d);
        const int ubp = ceil_div(d.n, chp) + (1 << level);
        // (under the separate IPC exchange it overwrites the next level's hist_b slots whole: nothing to
        // zero; under the fused one the next level's send slot is the reduce destination to zero)
        const int64_t zero_next = (ipc && !ipc_fused) ? 0 : (int64_t)(1 << level) * d.slot_elems;
        d.zero_red = ipc_fused ? static_cast<int64_t*>(ipc_send_buffer(cc)) : nullptr;
        const int steps = ceil_div(chp, 16 * kWave);  // <= 8 (chunk_part's cap)
        if (ep_level) {
          c->d.seq = stamp_next(c, "k_eval_part");
          const int evals = ep_mode >= 2 ? (1 << level) : 0;  // the evaluator blocks come first
          launch_eval_part(steps, ep_mode, dim3(ubp + evals), ep_mode == 2 ? fused_lds : 0, stream, d, parity, zero_next,
                           level, chp, t, c->eval_slots, ++c->dec_tag);
        } else if (part_pos && (1 << level) <= kPartPosNodes) {  // position-ordered blocks (k_part_pos)
          // (the grid from the instantiation's rows per block: COBALT_PART_CHUNK may give 1-3 or 5-7 steps)
          const int ps = steps <= 4 ? 4 : 8;
          const dim3 pg(std::max(1, (int)ceil_div(d.n, (int64_t)16 * kWave * ps)));
          if (ps == 4)
            GLAUNCH("k_partition", (k_part_pos<4>), pg, dim3(16 * kWave), 0, stream, d, parity, zero_next, level);
          else
            GLAUNCH("k_partition", (k_part_pos<8>), pg, dim3(16 * kWave), 0, stream, d, parity, zero_next, level);
        } else if (steps <= 4)
          GLAUNCH("k_partition", (k_partition<16, 4>), dim3(ubp), dim3(16 * kWave), 0, stream, d, parity, zero_next,
                  level, chp);
        else
          GLAUNCH("k_partition", (k_partition<16, 8>), dim3(ubp), dim3(16 * kWave), 0, stream, d, parity, zero_next,
                  level, chp);
      }
      d.ipc_epoch = 0;
      CK_LAUNCH();
    }
    c->grown = t + 1;
    if (sampled) c->applied = t + 1;  // no training margins on a per-tree sample
    d.zero_red = nullptr;
  }
  // archive the last tree of this call (later trees are archived by the next tree's k_grad)
  if (c->grown > t0) {
    const int last = c->grown - 1;
    CK(hipMemcpyAsync(d.trees + (size_t)last * c->max_nodes, d.nodes_buf[last & 1], c->max_nodes * sizeof(Node),
                      hipMemcpyDeviceToDevice, stream));
  }
  if (d.mrec) {  // the margins back into the array (the last tree's leaves follow, below)
    hipLaunchKernelGGL(k_margin_out, dim3(std::min(ceil_div(d.n, 256), 4096)), dim3(256), 0, stream, d.bins, d.margin,
                       d.n);
    CK_LAUNCH();
    d.mrec = 0;
  }
  // bring the margins up to date with the last grown tree
  if (c->applied < c->grown) {
    GLAUNCH("k_apply_tree", k_apply_tree, dim3(std::max(grad_grid, 1)), dim3(256), tree_lds, stream, d, c->grown - 1);
    CK_LAUNCH();
    c->applied = c->grown;
  }
  // the last tree of the call: its replica digest checked by a collective of its own (see k_dig_stage)
  if (dp && c->grown > t0) {
    const int ls = (c->grown - 1) & 1;
    hipLaunchKernelGGL(k_dig_stage, dim3(1), dim3(64), 0, stream, d.dig, ls);
    CK_LAUNCH();
    if (int rc = cobalt_comm_allreduce_sum_i64(c->cfg.comm, d.dig + 2, 1, stream)) return rc;
    hipLaunchKernelGGL(k_dig_cmp, dim3(1), dim3(64), 0, stream, d.dig, ls, d.world, d.err_host);
    CK_LAUNCH();
  }
  d.stamps = nullptr;
  return stamp_dump(c, stream);
}

COBALT_API int cobalt_gbdt_grow(void* h, int t0, int n_trees, hipStream_t stream) {
  return grow_impl(static_cast<GbdtCtx*>(h), t0, n_trees, stream, false);
}

// ------------------------------------------------------------------------------------------
// Exact external-memory training (histograms over page-resident chunks, the analog of
// XGBoost's external-memory `hist` without sampling). The quantised pages stay in host DRAM (or HBM
// under a budget); on the device every row keeps only its margin, label, weight, packed (g, h) and its
// current node (2 B): ~22 B per row instead of the in-core ~72 B. A tree is grown level by level, and
// every level streams every page once:
//   * level -1 (k_ox_page, mode grad): the previous tree's leaf (found through the row's node) is added
//     to its margin, g / h are computed and quantised exactly as the in-core root pass does (same
//     dither key: per tree and GLOBAL row), every row moves to the root, the root histogram is built;
//   * level L >= 0: a row of a node split at level L moves to its child (the split feature's bin from
//     the page), and a row entering the child the evaluation chose to build (smaller hessian) adds its
//     (g, h) to that child pair's histogram;
//   * after each pass: the per-block partial histograms are reduced into the in-core trainer's level
//     slots (k_ox_reduce) and the in-core split evaluation (k_eval) runs on them unchanged -- same
//     node table, same subtraction trick, same finalisation.
// Every histogram is an exact integer sum, so the trees are byte-identical to the in-core fit of the
// same rows (tests/test_external.py). Histograms: each block privatises the pair slots of its group
// (gridDim.y groups) in LDS as packed u64 cells -- flushed to its own int64 slab rows every 16384 rows
// (the packed halves cannot carry within that) -- so the page data is read once per slot group.
// ------------------------------------------------------------------------------------------
constexpr int kOxSlab = 128;           // blocks per page pass (= slab rows per pair slot)
constexpr int kOxFlushRows = 16384;    // rows per LDS flush (packed u64 bound, as the in-core blocks)
constexpr size_t kOxLdsBudget = 150 * 1024;

static int ox_group_slots(const GbdtDev& d) {
  return std::max<int>(1, (int)(kOxLdsBudget / ((size_t)(d.ncells + 1) * sizeof(uint64_t))));
}

// mode: -1 = gradient pass (+ root histogram), L >= 0 = route level L + histogram of level L + 1.
__global__ __launch_bounds__(1024) void k_ox_page(GbdtDev d, const uint8_t* __restrict__ page, int ps, int64_t n,
                                                  int64_t r0, int mode, int tree, int apply, uint16_t* __restrict__ pos,
                                                  uint64_t* __restrict__ gh, int64_t* __restrict__ slab,
                                                  float* __restrict__ margin, const float* __restrict__ label,
                                                  const float* __restrict__ weight, int gslots) {
  extern __shared__ uint64_t s_h[];  // [gslots][ncells + 1] packed (g, h); cell ncells = the slot's totals
  __shared__ uint32_t s_meta[256];
  __shared__ float s_leaf[256];
  __shared__ uint8_t s_build[256];
  __shared__ int s_hoff[kMaxFeatTile + 1];
  __shared__ int s_nb[kMaxFeatTile];  // bin count, 0 for a feature colsample masked out of this tree
  const int F = d.F, nc = d.ncells, cells = nc + 1;
  const int g0 = blockIdx.y * gslots;                                  // first slot of this block's group
  const int nslots = mode < 0 ? 1 : (1 << mode);                       // pairs of level mode + 1
  const int gs = min(gslots, nslots - g0);
  if (gs <= 0) return;
  const Node* tab = (mode < 0) ? d.prev_nodes : d.nodes;              // tree staged for this pass
  for (int i = threadIdx.x; i < d.max_nodes && i < 256; i += blockDim.x) {
    const Node nd = tab[i];
    s_meta[i] = node_meta(nd);
    s_leaf[i] = nd.leaf_value;
    s_build[i] = (uint8_t)(nd.build != 0);
  }
  for (int f = threadIdx.x; f <= F; f += blockDim.x) {
    s_hoff[f] = d.hoff[f];
    if (f < F) s_nb[f] = d.fmask[(int64_t)tree * F + f] ? d.nbins[f] : 0;
  }
  const uint64_t tree_key = tree_key_of(d.seed, tree);
  const uint64_t dkey = splitmix64(tree_key ^ kDitherSalt);
  const int first = mode < 0 ? 0 : (1 << mode) - 1;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = min(n, (int64_t)blockIdx.x * per), b1 = min(n, b0 + per);
  int64_t* my = slab + (int64_t)blockIdx.x * d.slot_elems * (int64_t)(1 << (d.max_depth - 1));
  for (int64_t c0 = b0; c0 < b1; c0 += kOxFlushRows) {
    const int64_t c1 = min(b1, c0 + kOxFlushRows);
    __syncthreads();  // (previous flush done with s_h; staged tables visible)
    for (int i = threadIdx.x; i < gs * cells; i += blockDim.x) s_h[i] = 0ull;
    __syncthreads();
    for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
      const int64_t r = r0 + i;
      const uint8_t* row = page + i * ps;
      int slot = -1;
      uint64_t v = 0;
      if (mode < 0) {  // gradients (+ the previous tree's leaf), every row builds the root
        float mf = margin[r];
        if (apply) {  // the previous tree's leaf: from the row's last routed node down (its last level
                      // was evaluated but not routed), with the page's bins
          int nd = pos[r];
          uint32_t m = s_meta[nd];
          while (m & kMetaSplit) {
            const uint32_t b = row[m & 0xFFFFu];
            const bool left = meta_left(m, b);
            nd = 2 * nd + (left ? 1 : 2);
            m = s_meta[nd];
          }
          mf += s_leaf[nd];
          margin[r] = mf;
        }
        const double p = 1.0 / (1.0 + exp(-(double)mf));
        const double y = (double)label[r], w = (double)weight[r];
        double g = (p - y) * w;
        double h = fmax(p * (1.0 - p), 1e-16) * w;
        if (d.subsample < 1.0) {
          const uint64_t hsh = splitmix64(tree_key ^ (uint64_t)(d.row_offset + r));
          if (!(uniform01(hsh) < d.subsample)) { g = 0.0; h = 0.0; }
        }
        int64_t gq, hq;
        quantize_gh(g, h, d.gscale, d.hscale, dkey, d.row_offset + r, gq, hq);
        v = ((uint64_t)(uint32_t)(int32_t)gq << 32) | (uint64_t)(uint32_t)hq;
        gh[r] = v;
        pos[r] = 0;
        slot = 0;
      } else {  // route a row of a split node of this level; it may build its child's pair histogram
        // (with several slot groups the y = 0 blocks store the routed position; another group's block
        // can read the row before or after that store, so a position already on level mode + 1 counts
        // as routed from its parent)
        int nd = pos[r];
        int ch = -1;
        if (nd >= 2 * first + 1) {
          ch = nd;
          nd = (nd - 1) >> 1;
        } else if (nd >= first) {
          const uint32_t m = s_meta[nd];
          if (m & kMetaSplit) {
            const uint32_t b = row[m & 0xFFFFu];
            const bool left = meta_left(m, b);
            ch = 2 * nd + (left ? 1 : 2);
            if (blockIdx.y == 0) pos[r] = (uint16_t)ch;
          }
        }
        if (ch >= 0 && s_build[ch]) {
          slot = nd - first;
          v = gh[r];
        }
      }
      const int ls = slot - g0;
      if (slot >= 0 && ls >= 0 && ls < gs) {
        unsigned long long* hs = reinterpret_cast<unsigned long long*>(s_h + (int64_t)ls * cells);
        atomicAdd(hs + nc, (unsigned long long)v);  // the slot's (G, H)
        for (int f = 0; f < F; ++f) {
          const int b = row[f];
          if (b < s_nb[f]) atomicAdd(hs + s_hoff[f] + b, (unsigned long long)v);
        }
      }
    }
    __syncthreads();
    // flush: this block owns its slab rows (no atomics); only non-zero cells are written
    for (int i = threadIdx.x; i < gs * cells; i += blockDim.x) {
      const uint64_t pv = s_h[i];
      if (!pv) continue;
      const int ls = i / cells, c = i - ls * cells;
      int64_t* dst = my + (int64_t)(g0 + ls) * d.slot_elems + 2 * c;
      dst[0] += (int64_t)(int32_t)(uint32_t)(pv >> 32);
      dst[1] += (int64_t)(uint32_t)pv;
    }
  }
}

// Level histograms: the kOxSlab per-block slab rows of each pair slot summed into hist_b[parity] (the
// in-core evaluation's input, totals cell included), the slab zeroed behind the read.
__global__ __launch_bounds__(256) void k_ox_reduce(GbdtDev d, int64_t* __restrict__ slab, int parity, int slots) {
  const int s = blockIdx.x;
  const int64_t e = ((int64_t)blockIdx.y * blockDim.x + threadIdx.x) * 2;
  if (e >= d.slot_elems || s >= slots) return;
  const int64_t rowstride = d.slot_elems * (int64_t)(1 << (d.max_depth - 1));
  int64_t g = 0, h = 0;
  for (int b = 0; b < kOxSlab; ++b) {
    int64_t* p = slab + b * rowstride + (int64_t)s * d.slot_elems + e;
    g += p[0];
    h += p[1];
    p[0] = 0;
    p[1] = 0;
  }
  int64_t* o = d.hist_b[parity] + (int64_t)s * d.slot_elems + e;
  o[0] = g;
  o[1] = h;
}

COBALT_API int cobalt_gbdt_ox_init(void* h, int64_t n, float* margin, const float* label, const float* weight) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (c->d.F > kMaxFeatTile || c->max_nodes > 256 || c->d.F > 32) return -15;  // depth <= 7, <= 32 features
  if (c->d.wide) return -15;  // (the out-of-core passes accumulate 17-bit packed pairs)
  if (c->ox_pos) return -16;
  c->ox_n = n;
  int rc;
  if ((rc = dev_alloc(c, (void**)&c->ox_pos, (size_t)std::max<int64_t>(n, 1) * sizeof(uint16_t)))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->ox_gh, (size_t)std::max<int64_t>(n, 1) * sizeof(uint64_t)))) return rc;
  const size_t sb = (size_t)kOxSlab * c->pairs_max * c->d.slot_elems * sizeof(int64_t);
  if ((rc = dev_alloc(c, (void**)&c->ox_slab, sb))) return rc;
  CK(hipMemset(c->ox_slab, 0, sb));
  c->ox_margin = margin;
  c->ox_label = label;
  c->ox_weight = weight;
  const size_t lds = (size_t)ox_group_slots(c->d) * (c->d.ncells + 1) * sizeof(uint64_t);
  CK(hipFuncSetAttribute((const void*)k_ox_page, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return 0;
}

// Start tree t: node tables (the new one reset, the previous one kept for the margin update).
COBALT_API int cobalt_gbdt_ox_begin(void* h, int t, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (t != c->grown || t >= c->cfg.max_trees) return -11;
  GbdtDev& d = c->d;
  d.nodes = d.nodes_buf[t & 1];
  d.prev_nodes = d.nodes_buf[(t + 1) & 1];
  d.zero_red = nullptr;
  d.stamps = nullptr;
  hipLaunchKernelGGL(k_tree_begin, dim3(std::max(1, std::min(64, ceil_div(d.slot_elems / 2, 256)))), dim3(256), 0,
                     stream, d);
  CK_LAUNCH();
  return 0;
}

// One page of the current pass (mode -1 = gradients, L = route level L). Rows r0 .. r0 + n of the data
// set, `ps` bytes per row (the F bins first).
COBALT_API int cobalt_gbdt_ox_page(void* h, const uint8_t* page, int ps, int64_t n, int64_t r0, int mode, int t,
                                   hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  const GbdtDev& d = c->d;
  if (!c->ox_pos || r0 < 0 || r0 + n > c->ox_n || ps < d.F || mode >= d.max_depth - 1) return -3;
  if (n <= 0) return 0;
  const int gsl = ox_group_slots(d);
  const int nslots = mode < 0 ? 1 : (1 << mode);
  const dim3 grid(kOxSlab, ceil_div(nslots, gsl));
  const int gs = std::min(gsl, nslots);
  const size_t lds = (size_t)gs * (d.ncells + 1) * sizeof(uint64_t);
  const int apply = (mode < 0 && t > c->fit_first) ? 1 : 0;
  hipLaunchKernelGGL(k_ox_page, grid, dim3(1024), lds, stream, d, page, ps, n, r0, mode, t, apply, c->ox_pos, c->ox_gh,
                     c->ox_slab, c->ox_margin, c->ox_label, c->ox_weight, gsl);
  CK_LAUNCH();
  return 0;
}

// After the pass that built level `level`'s histograms: reduce them and evaluate the level.
COBALT_API int cobalt_gbdt_ox_level(void* h, int level, int t, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  GbdtDev& d = c->d;
  if (level < 0 || level >= d.max_depth) return -3;
  const int parity = level & 1;
  const int slots = level == 0 ? 1 : (1 << (level - 1));
  hipLaunchKernelGGL(k_ox_reduce, dim3(slots, ceil_div(d.slot_elems / 2, 256)), dim3(256), 0, stream, d, c->ox_slab,
                     parity, slots);
  CK_LAUNCH();
  hipLaunchKernelGGL((k_eval<false, false, false>), dim3(1 << level), dim3(1024), 0, stream, d, level, parity, t, d.F,
                     c->eval_slots);
  CK_LAUNCH();
  return 0;
}

// Finish tree t: archive its node table.
COBALT_API int cobalt_gbdt_ox_end(void* h, int t, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  GbdtDev& d = c->d;
  CK(hipMemcpyAsync(d.trees + (size_t)t * c->max_nodes, d.nodes_buf[t & 1], c->max_nodes * sizeof(Node),
                    hipMemcpyDeviceToDevice, stream));
  c->grown = t + 1;
  c->applied = t;
  return 0;
}

// External memory: grow tree t from the sample the last k_ooc_page passes wrote into the trainer's
// row records / feature-major bins (n_rows set by cobalt_gbdt_set_rows).
COBALT_API int cobalt_gbdt_grow_sampled(void* h, int t, hipStream_t stream) {
  return grow_impl(static_cast<GbdtCtx*>(h), t, 1, stream, true);
}

// Rows of the current sample (<= the capacity the context was created with).
COBALT_API int cobalt_gbdt_set_rows(void* h, int64_t n) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (n < 0 || n > c->cfg.n_rows) return -13;
  c->d.n = n;
  return 0;
}

// Device pointer to the heap-ordered node records of tree t (read by k_ooc_page to apply it).
COBALT_API void* cobalt_gbdt_tree_ptr(void* h, int t) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  return c->d.trees + (size_t)t * c->max_nodes;
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

// Resume: the margins passed to set_data already contain trees [0, t0) (re-predicted from a
// checkpoint); boosting continues at global tree index t0, so row sampling and column masks -- both
// keyed by the global tree index -- follow the uninterrupted run exactly.
// Binary labels into the row records (see GbdtDev::ylab): after set_data, for a fit whose labels are
// all 0 or 1 and whose weights are 1 (negatives) or `spw` (positives) -- the caller checks both. Writes
// byte 23 of every record (padding: bins occupy bytes 0..F-1, F <= 23 -- for F > 20 the histogram reads
// byte 23 as a padding feature's bin, which goes to the trash cell -- and the gradient pass rewrites
// bytes 16..31 from the record it read). Saves 8 of the ~80 bytes per row the gradient pass moves.
__global__ __launch_bounds__(256) void k_put_label(uint8_t* bins, const float* label, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bins[i * 32 + 23] = label[i] != 0.0f ? 1 : 0;
}

COBALT_API int cobalt_gbdt_set_binary_labels(void* h, float spw, hipStream_t stream) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  GbdtDev& d = c->d;
  if (!d.bins || !d.label || d.stride != 32 || d.F > 23) return -13;
  // F <= 20: the label bit in the h word, which frees bytes 20-23 for the margin (GbdtDev::lab31 / mrec)
  const bool l31 = d.F <= 20;
  // (F <= 20: written by the next grow call, together with the margins when they go to the records)
  c->label_pending = l31 && d.n > 0;
  if (d.n > 0 && !l31) {
    const int grid = std::min(ceil_div(d.n, 256), 4096);
    hipLaunchKernelGGL(k_put_label, dim3(grid), dim3(256), 0, stream, d.bins, d.label, d.n);
    CK(hipGetLastError());
  }
  d.lab31 = l31 ? 1 : 0;
  d.ylab = 1;
  d.spw = spw;
  return 0;
}

COBALT_API int cobalt_gbdt_set_start(void* h, int t0) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (t0 < 0 || t0 > c->cfg.max_trees || c->grown != 0) return -12;
  c->grown = t0;
  c->applied = t0;
  c->fit_first = t0;
  return 0;
}

// The last grow call's launch plan (GbdtCtx::plan): out[0] fused IPC exchange, [1] node-ownership level
// (-1 off), [2] wide gradients, [3] blocks of the fused k_eval this rank's CUs hold at once, [4] bit mask of
// the levels run by the fused evaluation + partition pass, [5] of them in the evaluator-block form, [6] of
// those the levels whose grid exceeds one block per CU.
COBALT_API int cobalt_gbdt_plan(void* h, int32_t* out) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  for (int k = 0; k < 7; ++k) out[k] = c->plan[k];
  return 0;
}

// Data-parallel replica check: 0 = healthy, 2 = this rank's trees diverged from its peers' (see
// GbdtDev::dig). Read by the host after / while a segment of trees runs.
COBALT_API int cobalt_gbdt_error(void* h) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  return c && c->err_pinned ? (int)__atomic_load_n(c->err_pinned, __ATOMIC_ACQUIRE) : 0;
}

// Fault injection (tests): perturb tree `t`'s root totals on this rank, so its replica diverges.
COBALT_API int cobalt_gbdt_set_fault(void* h, int t) {
  static_cast<GbdtCtx*>(h)->fault_tree = t;
  return 0;
}

// Re-arm a trainer context for a new fit with the same shapes (rows, features, record pitch, depth,
// tree capacity, item size, tile, communicator): the per-fit scalars come from `cfg`, the tree count
// restarts at 0, and the device buffers -- hundreds of MB at 10M rows -- are kept instead of freed and
// reallocated (models/gbdt.py fits back to back: ~2.5 ms of hipFree + hipMalloc per fit). Returns 1 when
// the shapes differ (the caller creates a new context).
COBALT_API int cobalt_gbdt_reuse(void* h, const GbdtConfig* cfg) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (!c || !cfg) return -3;
  const GbdtConfig& o = c->cfg;
  if (o.n_rows != cfg->n_rows || o.n_feat != cfg->n_feat || o.row_stride != cfg->row_stride ||
      o.max_depth != cfg->max_depth || o.max_trees != cfg->max_trees || o.chunk != cfg->chunk ||
      o.feat_tile != cfg->feat_tile || o.world_size != cfg->world_size || o.comm != cfg->comm ||
      (o.grad_bits > 17) != (cfg->grad_bits > 17))
    return 1;
  c->cfg = *cfg;
  GbdtDev& d = c->d;
  d.n = cfg->n_rows;  // (the external-memory mode's set_rows may have lowered it)
  d.row_offset = cfg->row_offset;
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
  c->grown = 0;
  c->applied = 0;
  c->fit_first = 0;
  c->fault_tree = -1;
  if (c->err_pinned) memset(c->err_pinned, 0, 64);
  return 0;
}

COBALT_API int cobalt_gbdt_destroy(void* h) {
  GbdtCtx* c = static_cast<GbdtCtx*>(h);
  if (!c) return 0;
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->err_pinned) (void)hipHostFree(c->err_pinned);
  delete c;
  return 0;
}

// Quantise n rows into row records (pitch `stride`) and feature-major bins with row pitch `ldt`
// (ldt = n for a whole matrix; the full row count when a streamed chunk is binned in place).
// 32-byte records of <= 24 features with 16-byte aligned fp32 rows (F % 4 == 0, ldx == F): lane = row,
// the row read as F / 4 float4 loads (one 64-lane instruction spans 64 consecutive rows, so the F / 4
// loads of a wave use every byte of the lines they touch), the bins of all features searched in LDS,
// the WHOLE record written as two 16-byte stores (bins | zero pad and (g, h): no separate memset of the
// record array) and the feature-major bytes as one coalesced byte store per feature.
template <int F4>
__global__ __launch_bounds__(256) void k_bin_rec32(const float* __restrict__ X, int64_t n,
                                                   const float* __restrict__ cuts, const int32_t* __restrict__ nbins,
                                                   uint8_t* __restrict__ bins, uint8_t* __restrict__ binsT,
                                                   int64_t ldt) {
  constexpr int F = 4 * F4;
  __shared__ float s_cuts[F * kMaxBins];
  __shared__ int s_nb[F];
  for (int i = threadIdx.x; i < F * kMaxBins; i += blockDim.x) s_cuts[i] = cuts[i];
  if (threadIdx.x < F) s_nb[threadIdx.x] = nbins[threadIdx.x];
  __syncthreads();
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n;
       row += (int64_t)gridDim.x * blockDim.x) {
    const float4* x4 = reinterpret_cast<const float4*>(X + row * F);
    float v[F];
#pragma unroll
    for (int q = 0; q < F4; ++q) {
      const float4 t = x4[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
    uint32_t w[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const int nb = s_nb[f];
      uint32_t b;
      if (v[f] != v[f]) {
        b = kMissingBin;
      } else {  // upper_bound over cuts[f][0..nb), clamped to nb - 1
        const float* c = s_cuts + f * kMaxBins;
        int lo = 0, hi = nb;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (c[mid] <= v[f]) lo = mid + 1; else hi = mid;
        }
        b = lo >= nb ? (uint32_t)(nb - 1) : (uint32_t)lo;
      }
      binsT[(int64_t)f * ldt + row] = (uint8_t)b;
      w[f >> 2] |= b << (8 * (f & 3));
    }
    uint4* rec = reinterpret_cast<uint4*>(bins + row * 32);
    rec[0] = make_uint4(w[0], w[1], w[2], w[3]);
    rec[1] = make_uint4(w[4], w[5], 0u, 0u);
  }
}

COBALT_API int cobalt_bin_matrix_ld(const float* X, int64_t n, int F, int64_t ldx, const float* cuts,
                                    const int32_t* nbins, uint8_t* bins, int stride, uint8_t* binsT, int64_t ldt,
                                    hipStream_t stream) {
  if (stride % 4 != 0 || stride < F || ldt < n) return -3;
  const int grid = std::max(1, std::min(ceil_div(n, 256), 256 * 8));
  // 32-byte records of 16-byte aligned rows: the vectorised kernel (10M x 20: 1.37 ms with k_bin)
  if (stride == 32 && ldx == F && F % 4 == 0 && F >= 4 && F <= 24 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(bins) & 15) == 0 && knob_str(Knob::BinScalar) == nullptr) {
    switch (F / 4) {
#define BIN_CASE(K) \
      case K: hipLaunchKernelGGL(k_bin_rec32<K>, dim3(grid), dim3(256), 0, stream, X, n, cuts, nbins, bins, binsT, ldt); break;
      BIN_CASE(1) BIN_CASE(2) BIN_CASE(3) BIN_CASE(4) BIN_CASE(5) BIN_CASE(6)
#undef BIN_CASE
    }
    CK_LAUNCH();
    return 0;
  }
  const size_t lds = (size_t)F * kMaxBins * sizeof(float);
  if (lds <= 64 * 1024) {
    hipLaunchKernelGGL(k_bin<true>, dim3(grid), dim3(256), lds, stream, X, n, F, ldx, cuts, nbins, bins, stride, binsT,
                       ldt);
  } else {
    hipLaunchKernelGGL(k_bin<false>, dim3(grid), dim3(256), 0, stream, X, n, F, ldx, cuts, nbins, bins, stride, binsT,
                       ldt);
  }
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_bin_matrix(const float* X, int64_t n, int F, int64_t ldx, const float* cuts,
                                 const int32_t* nbins, uint8_t* bins, int stride, uint8_t* binsT,
                                 hipStream_t stream) {
  return cobalt_bin_matrix_ld(X, n, F, ldx, cuts, nbins, bins, stride, binsT, n, stream);
}

// Self-test of the DPP wave primitives (tests/test_gpu_gbdt.py): one wave, inclusive scans of the
// int64 inputs (and of their low 32 bits), and the wave_best arg-max of (gain = in, key = lane).
namespace {
__global__ __launch_bounds__(64) void k_dpp_selftest(const int64_t* __restrict__ in, int64_t* __restrict__ o64,
                                                     int* __restrict__ o32, int64_t* __restrict__ obest) {
  const int lane = threadIdx.x;
  const int64_t v = in[lane];
  o64[lane] = wave_incl_scan(v);
  o32[lane] = wave_incl_scan((int)v);
  Cand c;
  c.gain = (double)(v % 1000);
  c.key = lane;
  c.gl = v;
  c.hl = -v;
  float cut = (float)lane;
  wave_best(c, cut);
  obest[4 * lane + 0] = c.key;
  obest[4 * lane + 1] = c.gl;
  obest[4 * lane + 2] = c.hl;
  obest[4 * lane + 3] = (int64_t)cut;
}
}  // namespace

COBALT_API int cobalt_dpp_selftest(const int64_t* in, int64_t* o64, int* o32, int64_t* obest, hipStream_t s) {
  hipLaunchKernelGGL(k_dpp_selftest, dim3(1), dim3(64), 0, s, in, o64, o32, obest);
  CK_LAUNCH();
  return 0;
}
