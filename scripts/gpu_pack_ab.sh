#!/bin/bash
# Packed small-feature chunks in split evaluation: GBDT + DP GPU tests (trees equal the oracle's), then
# stamps / 10M fits with packs on (default) and off (COBALT_EVAL_PACK=0), and 1M / 1.25M fits.
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 420 python -u -m pytest tests/test_gpu_gbdt.py tests/test_00gpu_dp_ipc.py tests/test_external.py \
  tests/test_stream.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q -E " failed|[0-9]+ error" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
bash scripts/gpu_env_multi.sh COBALT_EVAL_PACK 1 0 || exit $?
for rows in 1000000 1250000; do
  for x in 1 0 1 0; do
    line=$(COBALT_EVAL_PACK=$x timeout -k 10 200 python bench.py --rows $rows --steps 3 --warmup 1 2>/dev/null | grep '^{') || exit 1
    echo "COBALT_EVAL_PACK=$x rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")"
  done
done
