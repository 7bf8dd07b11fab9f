#!/bin/bash
# 8 processes on one GPU with fewer HW queues per process; then the full GPU suite + smoke + bench
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4k_dp8 600 python -u scripts/dp8_diag.py 3 || exit $?
bash $S r4k_gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread || exit $?
bash $S r4k_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r4k_bench 300 python bench.py || exit $?
grep -E "passed|failed" gpurun_out/r4k_gpu_tests.log | tail -2
grep -h '^{' gpurun_out/r4k_dp8.log gpurun_out/r4k_bench.log | cut -c1-900
