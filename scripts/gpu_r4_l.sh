#!/bin/bash
# reference-UI exchanges on the GPU engine; 8 processes on one GPU with fewer HW queues per process
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4l_ui 300 python -u -m pytest tests/test_reference_ui.py -v -m gpu --timeout 250 --timeout-method thread || exit $?
bash $S r4l_dp8 600 python -u scripts/dp8_diag.py 3 || exit $?
grep -E "passed|failed" gpurun_out/r4l_ui.log | tail -2
grep -h '^{' gpurun_out/r4l_dp8.log | cut -c1-700
