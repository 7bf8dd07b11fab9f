#!/bin/bash
# Round 4 call C: precomputed eval_part items (ep_plan) -- oracle tests, small-shard fits, 1M stamps.
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4c_oracle 600 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 300 --timeout-method thread || exit $?
for rows in 1000000 1250000 2500000; do
  bash $S r4c_fit_$rows 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
done
STAMP_ROWS=1000000 bash $S r4c_stamps 300 bash scripts/gpu_stamps.sh || exit $?
bash $S r4c_bench 300 python bench.py || exit $?
bash $S r4c_ooc_exact 700 python -u scripts/bench_external.py --rows 100000000 --sample-rate 1.0 --compare-in-core || exit $?
