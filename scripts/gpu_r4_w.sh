#!/bin/bash
# round-4 rehearsal: the driver's GPU tiers (pytest -m gpu, smoke, bench)
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4w_gpu_tests 1100 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread || exit $?
bash $S r4w_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r4w_bench 300 python bench.py || exit $?
grep -E "passed|failed" gpurun_out/r4w_gpu_tests.log | tail -2
grep -h '^{' gpurun_out/r4w_bench.log | cut -c1-400
