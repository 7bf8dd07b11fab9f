#!/bin/bash
# eval_part items in 1024-row steps: oracle tests, same-box A/B at the small-shard sizes
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4u_gbdt 600 python -u -m pytest tests/test_gpu_gbdt.py -x -v -m gpu --timeout 500 --timeout-method thread || exit $?
grep -q "FAILED\| failed" gpurun_out/r4u_gbdt.log && { echo "tests failed"; exit 1; }
for rep in 1 2; do
  for rows in 1000000 1250000 2000000; do
    bash $S r4u_fine_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
    COBALT_EP_FINE=0 bash $S r4u_dbl_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
  done
done
for f in gpurun_out/r4u_*_*_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
