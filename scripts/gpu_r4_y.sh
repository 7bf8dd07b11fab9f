#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4y_gbdt 800 python -u -m pytest tests/test_gpu_gbdt.py tests/test_sketch.py tests/test_stream.py tests/test_external.py -v -m gpu --timeout 700 --timeout-method thread || exit $?
grep -hE "passed|failed|FAILED" gpurun_out/r4y_gbdt.log | tail -8
