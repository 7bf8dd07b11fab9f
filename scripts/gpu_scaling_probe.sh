#!/bin/bash
# Per-GPU work sweep (what each rank does under strong scaling) + kernel traces at 10M and 1.25M rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
for rows in 1250000 2500000 5000000; do
  bash scripts/gpu_step.sh bench_$rows 300 python bench.py --rows $rows --steps 3 --warmup 1 --profile-fit || exit $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof10m -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof10m.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1m -o run -- python3 $R/bench.py --rows 1250000 --steps 1 --warmup 1 > $R/gpurun_out/prof1m.log 2>&1 || exit $?
echo done
