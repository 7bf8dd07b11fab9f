#!/bin/bash
# Deep-level histogram item size sweep (COBALT_HIST_CHUNK) at 10M and 1M rows, 3 timed fits each.
set -o pipefail
S=scripts/gpu_step.sh
: > gpurun_out/chunk_sweep.txt
for c in 2048 4096 8192; do
  COBALT_HIST_CHUNK=$c bash $S sw10m_$c 300 python bench.py --steps 3 --warmup 1 --test-rows 100000 || exit $?
  echo "rows=10000000 COBALT_HIST_CHUNK=$c $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/sw10m_$c.log)" >> gpurun_out/chunk_sweep.txt
done
for c in 1024 2048 4096; do
  COBALT_HIST_CHUNK=$c bash $S sw1m_$c 200 python bench.py --rows 1000000 --steps 3 --warmup 1 --test-rows 100000 || exit $?
  echo "rows=1000000 COBALT_HIST_CHUNK=$c $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/sw1m_$c.log)" >> gpurun_out/chunk_sweep.txt
done
cat gpurun_out/chunk_sweep.txt
