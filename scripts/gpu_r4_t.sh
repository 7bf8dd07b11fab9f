#!/bin/bash
# per-level LDS bank conflicts of k_hist at 10M rows (30 trees)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d /tmp/r4t -o p -- python3 bench.py --steps 1 --warmup 0 --trees 30 > gpurun_out/r4t/run.log 2>&1 || exit $?
cc=$(find /tmp/r4t -name "*counter_collection.csv" | head -1); kt=$(find /tmp/r4t -name "*kernel_trace.csv" | head -1)
echo "$cc $kt"
python scripts/pmc_hist_levels.py "$cc" "$kt" > gpurun_out/r4t/hist_levels.txt 2>&1 || exit $?
cat gpurun_out/r4t/hist_levels.txt
