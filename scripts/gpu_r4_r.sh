#!/bin/bash
# DP protocol variants at the 8-GPU shard size after the planner default change: fit times (+ stamps)
set -o pipefail
timeout -k 10 400 python -u scripts/dp_overhead_probe.py --rows 1250000 > gpurun_out/r4r_dpo.log 2>&1 || exit $?
COBALT_DP_EVAL_PART=1 timeout -k 10 400 python -u scripts/dp_overhead_probe.py --rows 1250000 > gpurun_out/r4r_dpo_ep.log 2>&1 || exit $?
bash scripts/gpu_dp_stamps.sh > gpurun_out/r4r_stamps.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r4r_dpo.log gpurun_out/r4r_dpo_ep.log
grep -h "per tree" gpurun_out/dpst_*.summary.txt
