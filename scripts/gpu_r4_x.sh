#!/bin/bash
# knob sweep on the round-4 code (all-row sketch): 10M and 1.25M, each knob vs the default on one box
set -o pipefail
S=scripts/gpu_step.sh
run() {  # name rows env...
  local name=$1 rows=$2; shift 2
  env "$@" bash $S r4x_${name}_${rows} 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
}
for rows in 10000000 1250000; do
  run base $rows COBALT_X=0
  run w6 $rows COBALT_GRAD_W6=1
  run wt0 $rows COBALT_WT=0
  run wt2 $rows COBALT_WT=2
  run wt3 $rows COBALT_WT=3
  run cs3 $rows COBALT_MAX_COPY_SHIFT=3
  run cs5 $rows COBALT_MAX_COPY_SHIFT=5
  run hc2 $rows COBALT_HIST_CHUNK=2048
  run hc8 $rows COBALT_HIST_CHUNK=8192
  run base2 $rows COBALT_X=1
done
for f in gpurun_out/r4x_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
