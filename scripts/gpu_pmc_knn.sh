#!/bin/bash
# MFMA evidence for the SMOTE kNN distance kernel: available MFMA counters, then one PMC pass.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1
grep -io "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*" $R/gpurun_out/rocprof_counters.txt | sort -u > $R/gpurun_out/mfma_counters.txt
cat $R/gpurun_out/mfma_counters.txt
timeout -k 10 120 python3 $R/scripts/knn_probe.py 295000 > $R/gpurun_out/knn_probe.log 2>&1 || exit $?
cat $R/gpurun_out/knn_probe.log
set=$(grep -E "^SQ_(INSTS_VALU_MFMA_MOPS_F32|INSTS_VALU_MFMA_F32|VALU_MFMA_BUSY_CYCLES)$" $R/gpurun_out/mfma_counters.txt | head -3 | tr '\n' ' ')
echo "PMC set: $set SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $set SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d /tmp/pmc_knn -o run -- python3 $R/scripts/knn_probe.py 100000 > $R/gpurun_out/pmc_knn.log 2>&1 || exit $?
f=$(find /tmp/pmc_knn -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > $R/gpurun_out/pmc_knn_summary.txt
import sys, pandas as pd
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.split("(").str[0].str.slice(0, 40)
print(t.groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack().to_string())
PY
cat $R/gpurun_out/pmc_knn_summary.txt
