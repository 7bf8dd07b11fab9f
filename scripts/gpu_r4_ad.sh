#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4ad_dp 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -v -m gpu --timeout 800 --timeout-method thread || exit $?
grep -hE "passed|failed" gpurun_out/r4ad_dp.log | tail -2
grep -q "FAILED\| failed" gpurun_out/r4ad_dp.log && exit 1
bash $S r4ad_gbdt 600 python -u -m pytest tests/test_gpu_gbdt.py -x -q -m gpu --timeout 500 --timeout-method thread || exit $?
bash $S r4ad_ab 600 python -u scripts/dp_owner_ab.py 2000000 || exit $?
grep -hE "passed|failed" gpurun_out/r4ad_gbdt.log | tail -1
grep -h '^{' gpurun_out/r4ad_ab.log
