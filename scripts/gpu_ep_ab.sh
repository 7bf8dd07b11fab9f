#!/bin/bash
# A/B of the fused evaluation + partition pass (COBALT_EVAL_PART=1, default) against the separate
# k_eval + k_partition launches (=0): GBDT GPU tests (trees equal the oracle's), in-kernel stamps at
# 1M rows, and fits at 1M / 1.25M / 2.5M / 3.9M rows.
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 420 python -u -m pytest tests/test_gpu_gbdt.py tests/test_external.py tests/test_stream.py \
  -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q -E " failed|[0-9]+ error" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
for ep in 1 0; do
  COBALT_EVAL_PART=$ep STAMP_ROWS=1000000 bash scripts/gpu_stamps.sh > /dev/null || exit $?
  mv gpurun_out/stamps_1000000.summary.txt gpurun_out/ep${ep}_stamps_1M.txt
  tail -7 gpurun_out/ep${ep}_stamps_1M.txt
done
for rows in 1000000 1250000 2500000 3900000; do
  for ep in 1 0 1 0; do
    line=$(COBALT_EVAL_PART=$ep timeout -k 10 200 python bench.py --rows $rows --steps 3 --warmup 1 2>/dev/null | grep '^{') || exit 1
    echo "ep=$ep rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")"
  done
done
