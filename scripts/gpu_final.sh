#!/bin/bash
# Round-end rehearsal + evidence: the whole GPU test tier, smoke(), the default bench, the 1M / 1.25M fits
# and the in-kernel stamps of the current trainer.
set -o pipefail
S=scripts/gpu_step.sh
bash $S full_gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
grep -q " failed" gpurun_out/full_gpu_tests.log && { echo "tests failed"; exit 1; }
bash $S full_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S full_bench 300 python bench.py || exit $?
bash $S fin1p25m 200 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
bash $S fin1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash scripts/gpu_stamps.sh || exit $?
tail -3 gpurun_out/full_gpu_tests.log
grep -h "smoke ok" gpurun_out/full_smoke.log
for f in full_bench fin1p25m fin1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
