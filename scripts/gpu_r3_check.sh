#!/bin/bash
# Round-3 trainer iteration: GBDT oracle / DP / external-memory GPU tests, then in-kernel stamps at 1M
# and 10M rows and the 10M / 1.25M bench fits. Stops at the first failing or faulting step.
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 420 python -u -m pytest tests/test_gpu_gbdt.py tests/test_00gpu_dp_ipc.py tests/test_external.py \
  tests/test_stream.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q -E " failed|[0-9]+ error" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
STAMP_ROWS="1000000 10000000" bash scripts/gpu_stamps.sh > gpurun_out/stamps_all.log 2>&1 || exit $?
grep -A6 "per tree" gpurun_out/stamps_all.log
bash $S bench10m 200 python bench.py --steps 3 --warmup 1 || exit $?
bash $S bench1p25m 200 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
grep -h '^{' gpurun_out/bench10m.log gpurun_out/bench1p25m.log | cut -c1-330
