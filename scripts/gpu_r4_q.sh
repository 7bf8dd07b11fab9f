#!/bin/bash
# Round 4 evidence: row-scaling fits, stamps (1M, 10M), rocprofv3 kernel stats of 2 fits at 10M
set -o pipefail
S=scripts/gpu_step.sh
export TMPDIR=/tmp
for rows in 1000000 1250000 2500000 5000000 10000000; do
  bash $S r4q_fin_$rows 200 python bench.py --rows $rows --steps 3 --warmup 1 --profile-fit || exit $?
done
for rows in 1000000 10000000; do
  rm -f gpurun_out/st_r4q_$rows.txt
  COBALT_TRAINER_CACHE=0 COBALT_STAMPS=gpurun_out/st_r4q_$rows.txt bash $S r4q_st_$rows 200 python -u scripts/stamps_single.py $rows || exit $?
  python scripts/stamp_summary.py gpurun_out/st_r4q_$rows.txt > gpurun_out/stamps_r4q_$rows.summary.txt || exit $?
  rm -f gpurun_out/st_r4q_$rows.txt
done
mkdir -p gpurun_out/r4q_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4q_prof -o p -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/r4q_prof/run.log 2>&1 || exit $?
find /tmp/r4q_prof -name "*stats.csv" -exec cp {} gpurun_out/r4q_prof/ \;
find /tmp/r4q_prof -name "*kernel_trace.csv" -exec cp {} /tmp/r4q_trace.csv \;
python scripts/prof_summary.py /tmp/r4q_trace.csv 600 > gpurun_out/r4q_prof/kernel_trace_summary.txt 2>&1 || true
ls -la gpurun_out/r4q_prof
