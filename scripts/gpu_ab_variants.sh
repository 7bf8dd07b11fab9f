#!/bin/bash
# Same-box A/B of trainer variants given as NAME=ENVSPEC arguments (ENVSPEC: space-free VAR=value list joined
# by commas, or "-" for none; "ref" variants usually set COBALT_NATIVE_LIB=$PWD/abref/libcobalt_hip_ref.so).
# Stamps at STAMP_ROWS (default 1M and 10M) per variant, then 2 interleaved rounds of fits at BENCH_ROWS.
set -o pipefail
envof() { [ "$1" = "-" ] && echo "" || echo "$1" | tr ',' ' '; }
for spec in "$@"; do
  name=${spec%%=*}; e=$(envof "${spec#*=}")
  for rows in ${STAMP_ROWS:-1000000 10000000}; do
    env $e STAMP_ROWS=$rows bash scripts/gpu_stamps.sh > /dev/null || exit $?
    mv gpurun_out/stamps_$rows.summary.txt gpurun_out/var_${name}_$rows.txt
    echo "== $name rows=$rows"; tail -6 gpurun_out/var_${name}_$rows.txt
  done
done
for k in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; e=$(envof "${spec#*=}")
    for rows in ${BENCH_ROWS:-10000000}; do
      line=$(env $e timeout -k 10 200 python bench.py --rows $rows --steps 3 --warmup 1 2>/dev/null | grep '^{') || exit 1
      echo "$name rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")"
    done
  done
done
