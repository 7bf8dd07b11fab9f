#!/bin/bash
# Round-end rehearsal: the whole GPU test tier, smoke() and the default bench, each under its own limit.
set -o pipefail
S=scripts/gpu_step.sh
bash $S full_gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S full_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S full_bench 300 python bench.py || exit $?
tail -3 gpurun_out/full_gpu_tests.log
grep -h "smoke ok" gpurun_out/full_smoke.log
grep -h "^{" gpurun_out/full_bench.log | cut -c1-260
