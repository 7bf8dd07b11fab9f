#!/bin/bash
# Kernel-level profile of the GPU CSV reader + writer (1M x 143 synthetic raw export).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/csv_probe.py 1000000 --no-arrow > $R/gpurun_out/csv_probe.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_csv -o run -- python3 $R/scripts/csv_probe.py 1000000 --no-arrow > $R/gpurun_out/csv_prof.log 2>&1 || exit $?
mkdir -p $R/gpurun_out/prof_csv && cp $(find /tmp/prof_csv -name '*kernel_stats.csv') $R/gpurun_out/prof_csv/
cat $R/gpurun_out/csv_probe.log
