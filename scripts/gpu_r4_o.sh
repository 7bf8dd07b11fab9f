#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4o_dp 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -v -m gpu --timeout 700 --timeout-method thread || exit $?
bash $S r4o_ui 300 python -u -m pytest tests/test_reference_ui.py -v -m gpu --timeout 250 --timeout-method thread || exit $?
grep -hE "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/r4o_dp.log gpurun_out/r4o_ui.log
