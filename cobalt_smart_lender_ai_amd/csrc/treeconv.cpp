// Host-side conversion of the trainer's heap-ordered node records into XGBoost tree arrays (the
// Booster's Tree columns), in one pass per tree. This runs inside every fit (models/gbdt.py,
// booster.trees_from_heap_nodes): the NumPy form -- masks, fancy indexing and per-tree splits over
// 300 x 255 records -- cost ~6 ms per 300-tree fit on the GPU host, 2.5% of a 10M-row fit and 7% of a
// 1.25M-row data-parallel shard's.
//
// XGBoost numbers a tree's nodes in depthwise creation order with children allocated in pairs; the
// heap indices of one level are contiguous and children are allocated in parent order, so that order
// is ascending heap index over the live (split or leaf) nodes.
#include <stdint.h>
#include <string.h>

#include "common.h"

namespace {

struct HeapNode {  // csrc/gbdt.hip Node (64 bytes)
  int64_t G, H;
  int32_t start, count;
  int32_t status, build;
  int32_t feat, bin;
  int32_t default_left;
  float split_cond;
  float loss_chg, leaf_value;
  float sum_hess, base_weight;
};
static_assert(sizeof(HeapNode) == 64, "Node layout");

constexpr int32_t kSplit = 2, kLeaf = 3;
constexpr int32_t kRootParent = 2147483647;

}  // namespace

// nodes: [T][M] records; outputs packed tree after tree (capacity T * M each); counts[t] = live nodes of
// tree t. Returns the total number of live nodes, or -1 on bad arguments.
COBALT_API int64_t cobalt_heap_to_trees(const void* nodes, int T, int M, int32_t* counts, int32_t* left,
                                        int32_t* right, int32_t* parent, int32_t* split_index, float* split_cond,
                                        uint8_t* default_left, float* base_weight, float* loss_chg,
                                        float* sum_hess) {
  if (!nodes || T < 0 || M <= 0) return -1;
  const HeapNode* all = static_cast<const HeapNode*>(nodes);
  int32_t* new_id = new int32_t[M];
  int64_t o = 0;
  for (int t = 0; t < T; ++t) {
    const HeapNode* nd = all + (int64_t)t * M;
    int32_t n = 0;
    for (int i = 0; i < M; ++i) {
      const bool live = nd[i].status == kSplit || nd[i].status == kLeaf;
      new_id[i] = live ? n : -1;
      n += live ? 1 : 0;
    }
    counts[t] = n;
    for (int i = 0; i < M; ++i) {
      const int32_t k = new_id[i];
      if (k < 0) continue;
      const HeapNode& r = nd[i];
      const bool split = r.status == kSplit;
      const int64_t j = o + k;
      const int c = 2 * i + 1;
      left[j] = split && c < M ? new_id[c] : -1;
      right[j] = split && c + 1 < M ? new_id[c + 1] : -1;
      parent[j] = i > 0 ? new_id[(i - 1) / 2] : kRootParent;
      split_index[j] = split ? r.feat : 0;
      split_cond[j] = split ? r.split_cond : r.leaf_value;
      default_left[j] = split ? (uint8_t)r.default_left : (uint8_t)0;
      base_weight[j] = r.base_weight;
      loss_chg[j] = split ? r.loss_chg : 0.0f;
      sum_hess[j] = r.sum_hess;
    }
    o += n;
  }
  delete[] new_id;
  return o;
}
