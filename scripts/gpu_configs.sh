#!/bin/bash
# Refresh the BASELINE configuration results (profiles/configs/*.json via gpurun_out/configs/).
set -o pipefail
S=scripts/gpu_step.sh
for c in gbdt-10m gbdt-1m score-1b pipeline-100k ooc-100m; do
  bash $S cfg_$c 900 python -u scripts/bench_configs.py $c --save || exit $?
done
ls gpurun_out/configs
