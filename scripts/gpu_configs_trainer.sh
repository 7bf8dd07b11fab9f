#!/bin/bash
# Refresh the trainer-dependent BASELINE configuration results (gpurun_out/configs/ -> profiles/configs/).
set -o pipefail
S=scripts/gpu_step.sh
for c in gbdt-10m gbdt-1m pipeline-100k ooc-100m; do
  bash $S cfg_$c 400 python -u scripts/bench_configs.py $c --save || exit $?
done
ls gpurun_out/configs
