#!/bin/bash
# refresh the BASELINE configs' records with the round-4 code (one step per config)
set -o pipefail
S=scripts/gpu_step.sh
for c in gbdt-1m gbdt-10m ooc-100m score-1b pipeline-100k pipeline-full prep-full; do
  bash $S r4ae_$c 900 python -u scripts/bench_configs.py $c --save || exit $?
done
ls -la profiles/configs/
