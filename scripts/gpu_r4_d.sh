#!/bin/bash
# Round 4 call D: exact out-of-core streaming (test + 100M measurement), 8-rank diagnostics.
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4d_ext_tests 600 python -u -m pytest tests/test_external.py -x -v -m gpu --timeout 500 --timeout-method thread || exit $?
grep -q " failed" gpurun_out/r4d_ext_tests.log && { echo "external tests failed"; exit 1; }
bash $S r4d_ooc_exact_10m 400 python -u scripts/bench_external.py --rows 10000000 --sample-rate 1.0 --compare-in-core || exit $?
bash $S r4d_ooc_exact_100m 900 python -u scripts/bench_external.py --rows 100000000 --sample-rate 1.0 --compare-in-core || exit $?
