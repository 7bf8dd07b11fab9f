#!/bin/bash
while read rows c0 c1; do
  COBALT_HIST_CHUNK0=$c0 COBALT_HIST_CHUNK=$c1 timeout -k 10 240 python bench.py --rows $rows --steps 2 --warmup 1 --test-rows 10000 > gpurun_out/hs.log 2>&1 || exit $?
  echo "rows=$rows c0=$c0 c1=$c1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hs.log)"
done <<LIST
10000000 0 0
10000000 0 16384
10000000 32768 16384
1250000 0 0
1250000 0 4096
1250000 4096 4096
LIST
