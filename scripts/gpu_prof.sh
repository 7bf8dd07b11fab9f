#!/bin/bash
# Kernel-trace one bench run and keep only the summary (the raw trace CSV is large).
# usage: gpu_prof.sh NAME SECONDS TREES bench-args...
name=$1; secs=$2; trees=$3; shift 3
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_$name.log 2>&1
rc=$?
echo "[gpu_prof] $name exit=$rc"
[ $rc -ne 0 ] && exit $rc
f=$(find /tmp/prof_$name -name '*kernel_trace.csv' | head -1)
s=$(find /tmp/prof_$name -name '*kernel_stats.csv' | head -1)
python3 $R/scripts/prof_summary.py "$f" "$trees" > $R/gpurun_out/prof_$name.summary.txt 2>&1
cp "$s" $R/gpurun_out/prof_$name.kernel_stats.csv
python3 $R/scripts/prof_prelude.py "$f" > $R/gpurun_out/prof_$name.prelude.txt 2>&1
tail -n 60 $R/gpurun_out/prof_$name.summary.txt
