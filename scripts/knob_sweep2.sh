#!/bin/bash
# Item-size sweep after the load-batching fixes: "rows ENV=VALUE..." lines -> ms/fit + AUC.
# usage: knob_sweep2.sh < list   (one run per line; "-" = defaults)
mkdir -p gpurun_out
while read rows envs; do
  [ -z "$rows" ] && continue
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 240 python bench.py --rows $rows --steps 2 --warmup 1 --test-rows 100000 > gpurun_out/ks.log 2>&1 || exit $?
  echo "rows=$rows $envs $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ks.log) $(grep -o '"auc": [0-9.]*' gpurun_out/ks.log)" | tee -a gpurun_out/knob_sweep2.txt
done
