#!/bin/bash
# Per-GPU work at the strong-scaling shard sizes (10M / 5M / 2.5M / 1.25M rows per GPU) and the DP
# protocol overhead on one GPU (1-rank RCCL communicator, scripts/dp_overhead_probe.py).
set -o pipefail
S=scripts/gpu_step.sh
: > gpurun_out/shards.txt
for r in 5000000 2500000; do
  bash $S shard_$r 300 python bench.py --rows $r --steps 3 --warmup 1 --test-rows 100000 || exit $?
  echo "rows=$r $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/shard_$r.log)" >> gpurun_out/shards.txt
done
bash $S dp_probe 300 python -u scripts/dp_overhead_probe.py || exit $?
cat gpurun_out/shards.txt
tail -3 gpurun_out/dp_probe.log
