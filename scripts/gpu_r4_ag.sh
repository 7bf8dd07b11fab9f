#!/bin/bash
# 8 DP processes on one GPU (unmasked, time-sliced) with node ownership: 1 tree, depth 7
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4ag_dp8 400 python -u scripts/dp8_diag.py eight1 1 || exit $?
grep -h '^{' gpurun_out/r4ag_dp8.log | cut -c1-700
