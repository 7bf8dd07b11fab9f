#!/bin/bash
# persistent pipelined partition (COBALT_PART_PP=1): same models, then same-box timings at 10M / 5M
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/pp_d0.log 2>&1 &&
COBALT_PART_PP=1 $T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/pp_d1.log 2>&1 &&
COBALT_PART_PP=1 $T 200 python scripts/model_digest.py --rows 3000000 > gpurun_out/pp_d1s.log 2>&1 &&
$T 200 python scripts/model_digest.py --rows 3000000 > gpurun_out/pp_d0s.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pp_off10m.log 2>&1 &&
COBALT_PART_PP=1 $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pp_on10m.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pp_off10m_b.log 2>&1 &&
COBALT_PART_PP=1 $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/pp_on10m_b.log 2>&1 &&
$T 300 python bench.py --rows 5000000 --steps 3 --warmup 1 > gpurun_out/pp_off5m.log 2>&1 &&
COBALT_PART_PP=1 $T 300 python bench.py --rows 5000000 --steps 3 --warmup 1 > gpurun_out/pp_on5m.log 2>&1
for f in pp_d0 pp_d1 pp_d0s pp_d1s; do echo "$f $(tail -1 gpurun_out/$f.log)"; done
for f in pp_off10m pp_on10m pp_off10m_b pp_on10m_b pp_off5m pp_on5m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
