#!/bin/bash
# Strong-scaling shard sizes (1.25M / 2.5M rows = the 8- / 4-GPU shards of the 10M config): A/B of the
# trainer switches that trade launches for work, one bench line per variant.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/small_n_ab.txt
: > $out
for rows in ${AB_ROWS:-1250000 2500000}; do
  for v in "base:" "fused_part:COBALT_FUSED_PART=1" "eval_compact:COBALT_EVAL_COMPACT=1" "eval_fg4:COBALT_EVAL_FG=4"; do
    name=${v%%:*}; envs=${v#*:}
    line=$(env $envs timeout -k 10 200 python bench.py --rows $rows --steps 5 --warmup 1 --test-rows 100000 2>/dev/null | grep '^{') || exit 1
    ms=$(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")
    echo "$rows $name $ms" | tee -a $out
  done
done
