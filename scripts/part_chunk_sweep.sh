#!/bin/bash
# Partition item-size sweep at a given row count: prints ms/fit per COBALT_PART_CHUNK value.
rows=${1:-10000000}
for c in 0 4096 8192 16384 32768; do
  COBALT_PART_CHUNK=$c timeout -k 10 240 python bench.py --rows $rows --steps 2 --warmup 1 --test-rows 10000 > gpurun_out/sweep_$c.log 2>&1 || exit $?
  echo "chunk=$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$c.log)"
done
