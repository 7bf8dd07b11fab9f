// Registry of the native library's environment knobs (see knobs.h): the only getenv call site of csrc/.
#include "knobs.h"

#include <stdlib.h>

#include "common.h"

namespace cobalt {

static const char* const kKnobNames[(int)Knob::Count] = {
    "COBALT_STAMPS",       "COBALT_HIST_ABLATE", "COBALT_HIST_CHUNK",     "COBALT_HIST_CHUNK0",
    "COBALT_ROOT_CHUNK",   "COBALT_PART_CHUNK",  "COBALT_EVAL_FG",        "COBALT_EVAL_PART",
    "COBALT_HIST_PAIR",    "COBALT_MAX_COPY_SHIFT", "COBALT_WT",          "COBALT_IPC_FUSED",
    "COBALT_DP_OWNER",     "COBALT_CU_BUDGET",   "COBALT_BIN_SCALAR",     "COBALT_PRED_WALK",
    "COBALT_EVAL_BLOCKS",  "COBALT_MARGIN_IN_RECORD", "COBALT_PART_POS",
};

const char* knob_name(Knob k) { return kKnobNames[(int)k]; }

const char* knob_str(Knob k) { return getenv(kKnobNames[(int)k]); }

int knob_int(Knob k, int def) {
  const char* v = knob_str(k);
  return (v && *v) ? atoi(v) : def;
}

}  // namespace cobalt

// The registry, for tests/test_knobs.py (every native knob is documented in config.KNOBS).
COBALT_API int cobalt_knob_count() { return (int)cobalt::Knob::Count; }
COBALT_API const char* cobalt_knob_name(int i) {
  return (i >= 0 && i < (int)cobalt::Knob::Count) ? cobalt::kKnobNames[i] : nullptr;
}
