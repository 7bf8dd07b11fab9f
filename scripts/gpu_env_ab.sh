#!/bin/bash
# A/B of a trainer switch in one build: GBDT oracle tests with the switch on, then the 10M / 1M fits
# with it off and on. usage: gpu_env_ab.sh VAR VALUE
set -o pipefail
V=$1; X=$2
S=scripts/gpu_step.sh
env $V=$X bash $S envtests 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/envtests.log && { echo "tests failed"; exit 1; }
bash $S off10m 300 python bench.py --steps 3 --warmup 1 || exit $?
env $V=$X bash $S on10m 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S off1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
env $V=$X bash $S on1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
for f in off10m on10m off1m on1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
