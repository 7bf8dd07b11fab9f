#!/bin/bash
# eval_part items up to 32768 rows in partition rounds: oracle + DP tests, same-box A/B vs cap 8192
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4v_gbdt 800 python -u -m pytest tests/test_gpu_gbdt.py tests/test_00gpu_dp_ipc.py -x -v -m gpu --timeout 700 --timeout-method thread || exit $?
grep -q "FAILED\| failed" gpurun_out/r4v_gbdt.log && { echo "tests failed"; exit 1; }
for rep in 1 2; do
  for rows in 1250000 2500000 5000000; do
    bash $S r4v_big_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
    COBALT_EP_MAX=8192 bash $S r4v_cap_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
  done
done
for f in gpurun_out/r4v_*_*_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
