#!/bin/bash
# 8 processes sharing one GPU without CU masks (time-sliced): the 8-rank exchange's correctness
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4n_dp8 700 python -u scripts/dp8_diag.py eight 1 || exit $?
grep -h '^{' gpurun_out/r4n_dp8.log | cut -c1-900
