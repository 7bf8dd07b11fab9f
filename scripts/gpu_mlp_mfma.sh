#!/bin/bash
# MLP inference on fp32 MFMA: numerics tests, throughput vs the scalar-FMA kernel, kernel stats and
# one PMC pass (MFMA instruction / busy counters).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nn.py -k forward > $R/gpurun_out/mlp_tests.log 2>&1 || { tail -40 $R/gpurun_out/mlp_tests.log; exit 1; }
tail -3 $R/gpurun_out/mlp_tests.log
timeout -k 10 120 python3 scripts/mlp_infer_probe.py 10000000 10 > $R/gpurun_out/mlp_probe.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/mlp_infer_probe.py 100000000 5 >> $R/gpurun_out/mlp_probe.log 2>&1 || exit $?
cat $R/gpurun_out/mlp_probe.log
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_mlp -o run -- python3 $R/scripts/mlp_infer_probe.py 10000000 5 > $R/gpurun_out/mlp_prof.log 2>&1 || exit $?
f=$(find /tmp/prof_mlp -name '*kernel_stats.csv' | head -1)
cp "$f" $R/gpurun_out/mlp_kernel_stats.csv
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d /tmp/pmc_mlp -o run -- python3 $R/scripts/mlp_infer_probe.py 1000000 2 > $R/gpurun_out/pmc_mlp.log 2>&1 || exit $?
f=$(find /tmp/pmc_mlp -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > $R/gpurun_out/pmc_mlp_summary.txt
import sys, pandas as pd
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.extract(r"(k_\w+)", expand=False).fillna(t["Kernel_Name"].str.slice(0, 40))
print(t.groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack().to_string())
PY
cat $R/gpurun_out/pmc_mlp_summary.txt
