#!/bin/bash
# node-owner evaluation over the fused IPC exchange: DP process tests (2-5 ranks), 1-rank probe
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4ac_dp 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -v -m gpu --timeout 800 --timeout-method thread || exit $?
grep -hE "PASSED|FAILED|passed|failed" gpurun_out/r4ac_dp.log | tail -8
grep -q "FAILED\| failed" gpurun_out/r4ac_dp.log && exit 1
bash $S r4ac_gbdt 600 python -u -m pytest tests/test_gpu_gbdt.py -x -q -m gpu --timeout 500 --timeout-method thread || exit $?
grep -hE "passed|failed" gpurun_out/r4ac_gbdt.log | tail -2
