#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4ab_tests 900 python -u -m pytest tests/test_00gpu_dp_ipc.py tests/test_sketch.py tests/test_stream.py tests/test_external.py tests/test_gpu_gbdt.py tests/test_gpu_pipeline.py -v -m gpu --timeout 700 --timeout-method thread || exit $?
grep -q "FAILED\| failed" gpurun_out/r4ab_tests.log && { grep FAILED gpurun_out/r4ab_tests.log; exit 1; }
bash $S r4ab_pipe 600 python -u scripts/bench_configs.py pipeline-100k || exit $?
grep -hE "passed|failed" gpurun_out/r4ab_tests.log | tail -1
grep -ho '"stages_s": {[^}]*}\|"test_auc": [0-9.]*' gpurun_out/r4ab_pipe.log
