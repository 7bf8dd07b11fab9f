#!/bin/bash
# Round 4 combined call: oracle tests (precomputed eval_part items), exact full-data sketch, small
# shards, the new GPU tests, DP test matrix, DP stamps, part_rec A/B, headline bench.
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4c_oracle 600 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 300 --timeout-method thread || exit $?
grep -q " failed" gpurun_out/r4c_oracle.log && { echo "oracle tests failed"; exit 1; }
bash $S r4b_sketch_tests 300 python -u -m pytest tests/test_sketch.py -x -v -m gpu --timeout 200 --timeout-method thread || exit $?
bash $S r4b_sketch_probe 200 python -u scripts/sketch_exact_probe.py || exit $?
for rows in 1000000 1250000 2500000; do
  bash $S r4c_fit_$rows 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
done
bash $S r4b_new_tests 700 python -u -m pytest tests/test_gpu_auc_parity.py tests/test_reference_ui.py tests/test_gpu_serve.py -x -v -s -m gpu --timeout 600 --timeout-method thread || exit $?
bash $S r4b_dp_tests 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -x -v --timeout 600 --timeout-method thread || exit $?
bash $S r4b_dp_stamps 600 bash scripts/gpu_dp_stamps.sh || exit $?
for rows in 10000000 1000000; do
  COBALT_PART_REC=1 bash $S r4b_prec1_$rows 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
done
bash $S r4c_bench 300 python bench.py || exit $?
