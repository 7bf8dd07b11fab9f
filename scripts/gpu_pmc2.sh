#!/bin/bash
# Wave-state PMC counters per trainer kernel for a short fit (kernel-trace + pmc only, one pass per
# counter set, each under its own time limit). usage: gpu_pmc2.sh [bench args...]
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
: > $R/gpurun_out/pmc2_summary.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o run -- python3 $R/bench.py --trees 20 --steps 1 --warmup 0 --test-rows 10000 "$@" > $R/gpurun_out/pmc2_$i.log 2>&1 || exit $?
  f=$(find /tmp/pmc$i -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY' >> $R/gpurun_out/pmc2_summary.txt
import sys, pandas as pd
pd.set_option("display.width", 250)
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.replace("void ", "").str.split("(").str[0].str.slice(0, 26)
g = t[t["name"].str.startswith("k_")].groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack()
print(g.to_string(float_format=lambda v: f"{v:.4g}"))
PY
done
cat $R/gpurun_out/pmc2_summary.txt
