#!/bin/bash
# chunked exact sketch (in-core refactor + streams): tests, timing, bench
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4z_tests 900 python -u -m pytest tests/test_00gpu_dp_ipc.py tests/test_sketch.py tests/test_stream.py tests/test_external.py tests/test_gpu_gbdt.py -v -m gpu --timeout 700 --timeout-method thread || exit $?
grep -q "FAILED\| failed" gpurun_out/r4z_tests.log && { echo "tests failed"; grep -E "FAILED" gpurun_out/r4z_tests.log; exit 1; }
bash $S r4z_probe 200 python -u scripts/sketch_exact_probe.py --reps 5 || exit $?
bash $S r4z_bench 300 python bench.py || exit $?
grep -hE "passed|failed" gpurun_out/r4z_tests.log | tail -2
grep -h '^{' gpurun_out/r4z_probe.log
grep -ho '"ms_per_step": [0-9.]*\|"fit_breakdown_ms": {[^}]*}' gpurun_out/r4z_bench.log
