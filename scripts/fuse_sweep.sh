#!/bin/bash
while read rows c0 nofuse; do
  if [ "$nofuse" = "1" ]; then export COBALT_NO_FUSED_ROOT=1; else unset COBALT_NO_FUSED_ROOT; fi
  COBALT_HIST_CHUNK0=$c0 timeout -k 10 240 python bench.py --rows $rows --steps 2 --warmup 1 --test-rows 10000 > gpurun_out/fs.log 2>&1 || exit $?
  echo "rows=$rows c0=$c0 nofuse=$nofuse $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fs.log)"
done <<LIST
10000000 0 1
10000000 0 0
10000000 8192 0
10000000 4096 0
10000000 2048 0
1250000 0 1
1250000 1024 0
1250000 2048 0
LIST
