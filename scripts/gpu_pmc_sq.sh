#!/bin/bash
# Wave-level counters per trainer kernel (10M rows x 20 trees): waves, wave-cycles, cycles waiting on
# anything / issuing anything, LDS instructions and LDS bank conflicts. One pass (6 SQ counters).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d /tmp/pmcsq -o run -- python3 $R/bench.py --trees 20 --steps 1 --warmup 0 \
  --test-rows 10000 > $R/gpurun_out/pmcsq.log 2>&1 || exit $?
f=$(find /tmp/pmcsq -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > $R/gpurun_out/pmc_sq_summary.txt
import sys, pandas as pd
pd.set_option("display.width", 250)
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.replace("void ", "").str.split("(").str[0].str.slice(0, 26)
t = t[t["name"].str.startswith("k_")]
g = t.groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack()
g["wait_frac"] = g["SQ_WAIT_ANY"] / g["SQ_WAVE_CYCLES"]
g["issue_frac"] = g["SQ_ACTIVE_INST_ANY"] / g["SQ_WAVE_CYCLES"]
g["lds_conflict_per_lds_inst"] = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_INSTS_LDS"].clip(lower=1)
print(g.to_string(float_format=lambda v: f"{v:.4g}"))
PY
cat $R/gpurun_out/pmc_sq_summary.txt
