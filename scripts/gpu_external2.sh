#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S ext_test 300 python -u -m pytest tests/test_external.py -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/ext_test.log && { echo "tests failed"; exit 1; }
bash $S ext_100m_half 600 python -u scripts/bench_external.py --rows 100000000 --device-page-gb 1.5 || exit $?
grep -h '"metric"' gpurun_out/ext_100m_half.log
