#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4af_dp 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -v -m gpu --timeout 800 --timeout-method thread || exit $?
grep -hE "PASSED|FAILED|passed|failed" gpurun_out/r4af_dp.log | tail -8
