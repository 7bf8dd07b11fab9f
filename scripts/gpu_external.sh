#!/bin/bash
# External-memory GBDT: GPU test, a small run, then the 100M-row config (with the in-core comparison).
set -o pipefail
S=scripts/gpu_step.sh
bash $S ext_test 300 python -u -m pytest tests/test_external.py tests/test_gpu_gbdt.py -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/ext_test.log && { echo "tests failed"; exit 1; }
bash $S ext_10m 300 python scripts/bench_external.py --rows 10000000 --chunk 2097152 --compare-in-core || exit $?
bash $S ext_100m 900 python -u scripts/bench_external.py --rows 100000000 --compare-in-core || exit $?
grep -h '"metric"' gpurun_out/ext_10m.log gpurun_out/ext_100m.log
