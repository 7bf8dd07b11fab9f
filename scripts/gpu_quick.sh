#!/bin/bash
# GBDT GPU tests + RFE-fit probe + 10M bench (quick regression check after a kernel change)
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 400 python -u -m pytest tests/test_gpu_gbdt.py tests/test_external.py tests/test_stream.py -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
bash $S rfe_probe 200 python -u scripts/rfe_probe.py || exit $?
bash $S bench 300 python bench.py --steps 3 --warmup 1 || exit $?
grep -h "width\|^{" gpurun_out/rfe_probe.log gpurun_out/bench.log | cut -c1-200
for fg in $EVAL_FG_SWEEP; do
  COBALT_EVAL_FG=$fg bash $S bench_fg$fg 300 python bench.py --steps 3 --warmup 1 || exit $?
  COBALT_EVAL_FG=$fg bash $S rfe_fg$fg 200 python -u scripts/rfe_probe.py || exit $?
  grep -h "width\|^{" gpurun_out/rfe_fg$fg.log gpurun_out/bench_fg$fg.log | cut -c1-160
done
