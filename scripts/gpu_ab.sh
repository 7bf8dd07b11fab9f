#!/bin/bash
# Trainer kernel change check: GBDT oracle tests, then the 10M / 1.25M / 1M fits (3 timed steps each).
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
bash $S ab10m 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S ab1p25m 200 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
bash $S ab1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
for f in ab10m ab1p25m ab1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
