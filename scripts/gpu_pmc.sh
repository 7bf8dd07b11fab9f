#!/bin/bash
# PMC counters per kernel for a short 10M-row fit (kernel-trace + pmc only; no sys/hip traces).
# (FETCH_SIZE/WRITE_SIZE aborted rocprofv3 on this pool: not collected.)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o run -- python3 $R/bench.py --trees 20 --steps 1 --warmup 0 --test-rows 10000 "$@" > $R/gpurun_out/pmc$i.log 2>&1 || exit $?
  f=$(find /tmp/pmc$i -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY' >> $R/gpurun_out/pmc_summary.txt
import sys, pandas as pd
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.split("(").str[0].str.slice(0, 30)
g = t[t["name"].str.startswith(("k_", "void k_"))].groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack()
print(g.to_string())
PY
done
cat $R/gpurun_out/pmc_summary.txt
