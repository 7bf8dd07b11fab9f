#!/bin/bash
# Same-box A/B of several values of one trainer switch: in-kernel stamps (STAMP_ROWS, default 1M and
# 10M) per value, then interleaved 10M fits (value order repeated twice). usage: gpu_env_multi.sh VAR v1 v2 ...
set -o pipefail
V=$1; shift
for x in "$@"; do
  for rows in ${STAMP_ROWS:-1000000 10000000}; do
    env $V=$x STAMP_ROWS=$rows bash scripts/gpu_stamps.sh > /dev/null || exit $?
    mv gpurun_out/stamps_$rows.summary.txt gpurun_out/env_${V}_${x}_$rows.txt
    echo "== $V=$x rows=$rows"; tail -6 gpurun_out/env_${V}_${x}_$rows.txt
  done
done
for k in 1 2; do
  for x in "$@"; do
    line=$(env $V=$x timeout -k 10 200 python bench.py --rows ${BENCH_ROWS:-10000000} --steps 3 --warmup 1 2>/dev/null | grep '^{') || exit 1
    echo "$V=$x $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")"
  done
done
