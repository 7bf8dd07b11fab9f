#!/bin/bash
# Round-3 ablation stamps: per-kernel spans at 1M and 10M rows with timing-only switches
# (COBALT_HIST_ABLATE: 12 partition without cursor claims; 20 root pass without exp; 21 root pass
# without LDS atomics; 22 root pass without the previous-tree walk). Trees of ablated runs are wrong.
set -o pipefail
mkdir -p gpurun_out/abl
for a in ${ABL_LIST:-0 12 20 21 22}; do
  for rows in ${STAMP_ROWS:-1000000 10000000}; do
    COBALT_HIST_ABLATE=$a COBALT_STAMPS=gpurun_out/abl/s.txt timeout -k 10 200 python bench.py --rows $rows \
      --steps 1 --warmup 0 --test-rows 1000 > gpurun_out/abl/bench_${a}_$rows.log 2>&1 || exit $?
    python scripts/stamp_summary.py gpurun_out/abl/s.txt > gpurun_out/abl/abl_${a}_$rows.txt || exit $?
    rm -f gpurun_out/abl/s.txt
    echo "== ablate $a rows $rows"; tail -6 gpurun_out/abl/abl_${a}_$rows.txt
  done
done
