#!/bin/bash
# Root-pass (k_grad_hist) item size sweep at 10M rows (COBALT_ROOT_CHUNK), 3 timed fits each.
set -o pipefail
S=scripts/gpu_step.sh
: > gpurun_out/root_sweep.txt
for c in 0 9792 6528 13056; do
  if [ $c = 0 ]; then E=""; else E="COBALT_ROOT_CHUNK=$c"; fi
  env $E bash $S root_$c 300 python bench.py --steps 3 --warmup 1 --test-rows 100000 || exit $?
  echo "rows=10000000 COBALT_ROOT_CHUNK=$c $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/root_$c.log)" >> gpurun_out/root_sweep.txt
done
cat gpurun_out/root_sweep.txt
