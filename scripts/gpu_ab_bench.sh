#!/bin/bash
# Same-box interleaved A/B of bench.py fits: gpu_ab_bench.sh NAME=ENVSPEC ... (ENVSPEC as gpu_ab_variants.sh:
# comma-joined VAR=value list, or "-"). ROUNDS (default 2) rounds x BENCH_ROWS (default "10000000 1250000");
# each fit set under its own time limit; stops at the first failure.
set -o pipefail
envof() { [ "$1" = "-" ] && echo "" || echo "$1" | tr ',' ' '; }
for k in $(seq 1 ${ROUNDS:-2}); do
  for rows in ${BENCH_ROWS:-10000000 1250000}; do
    for spec in "$@"; do
      name=${spec%%=*}; e=$(envof "${spec#*=}")
      line=$(env $e timeout -k 10 200 python bench.py --rows $rows --steps ${STEPS:-5} --warmup 2 --test-rows 100000 \
             2>/dev/null | grep '^{') || exit 1
      echo "$name rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'], d['fit_breakdown_ms']['boost'])" "$line")"
    done
  done
done
