#!/bin/bash
# 5 / 6 processes sharing one GPU, 1 tree, long exchange deadline: starvation or protocol bug?
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4m_dp56 560 python -u scripts/dp8_diag.py width 1 || exit $?
grep -h '^{' gpurun_out/r4m_dp56.log | cut -c1-900
