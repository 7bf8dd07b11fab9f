#!/bin/bash
# In-kernel timing of the trainer's launches (COBALT_STAMPS) at a few row counts.
set -o pipefail
mkdir -p gpurun_out
for rows in ${STAMP_ROWS:-1000000 10000000}; do
  rm -f gpurun_out/stamps_$rows.txt
  COBALT_STAMPS=gpurun_out/stamps_$rows.txt timeout -k 10 200 python bench.py --rows $rows --steps 1 --warmup 0 \
    --test-rows 1000 > gpurun_out/stamps_bench_$rows.log 2>&1 || exit $?
  python scripts/stamp_summary.py gpurun_out/stamps_$rows.txt > gpurun_out/stamps_$rows.summary.txt || exit $?
  rm -f gpurun_out/stamps_$rows.txt
  cat gpurun_out/stamps_$rows.summary.txt
done
