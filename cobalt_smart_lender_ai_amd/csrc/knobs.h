// The native library's environment knobs, in ONE registry. Every COBALT_* variable the C++/HIP code
// reads is a Knob here and is read through knob_int / knob_str (the only getenv calls of csrc/). The
// documented list, with defaults and meaning, is config.KNOBS (Python); tests/test_knobs.py checks that
// both sides name the same set.
#pragma once
#include <stdint.h>

namespace cobalt {

enum class Knob : int {
  Stamps,        // COBALT_STAMPS: in-kernel launch / probe timestamps of sampled trees, appended to this file
  HistAblate,    // COBALT_HIST_ABLATE: timing-only ablations (wrong models; diagnosis only)
  HistChunk,     // COBALT_HIST_CHUNK: rows per histogram work item, levels >= 1
  HistChunk0,    // COBALT_HIST_CHUNK0: rows per root histogram item (unfused root pass)
  RootChunk,     // COBALT_ROOT_CHUNK: rows per item of the fused gradient + root-histogram pass
  PartChunk,     // COBALT_PART_CHUNK: rows per partition item
  EvalFg,        // COBALT_EVAL_FG: features per split-evaluation group (0 = one block per node)
  EvalPart,      // COBALT_EVAL_PART: the fused evaluation + partition pass (0 off, 1 auto, 2 forced)
  HistPair,      // COBALT_HIST_PAIR: lane-pair record gathers in k_hist (16 < F <= 24)
  MaxCopyShift,  // COBALT_MAX_COPY_SHIFT: log2 of the per-lane histogram copies of a low-cardinality feature
  WriteThrough,  // COBALT_WT: write-through stores (bit 0 slabs, bit 1 row ids, bit 2 root (g, h))
  IpcFused,      // COBALT_IPC_FUSED: the IPC exchange fused into the split evaluation (0: separate kernel)
  DpOwner,       // COBALT_DP_OWNER: node ownership on the deep levels over the fused IPC exchange
  CuBudget,      // COBALT_CU_BUDGET: CUs of this rank's CU-masked stream (parallel/cumask.py sets it)
  BinScalar,     // COBALT_BIN_SCALAR: the generic binning kernel for 32-byte records too (tests)
  PredWalk,      // COBALT_PRED_WALK: trees walked at once per predictor thread (2 / 4 / 8)
  EvalBlocks,    // COBALT_EVAL_BLOCKS: the evaluator-block fused pass over the fused IPC exchange
  MarginInRecord,  // COBALT_MARGIN_IN_RECORD: the root pass keeps the margins in the row records (F <= 20)
  PartPos,       // COBALT_PART_POS: position-ordered partition blocks (k_part_pos; 0: node-ordered items)
  Count
};

// The variable's value as an int (`def` when unset or empty); read at every call (callers that want a
// per-process value cache it in a function-local static).
int knob_int(Knob k, int def);
// The raw value, nullptr when unset.
const char* knob_str(Knob k);
const char* knob_name(Knob k);

}  // namespace cobalt
