#!/bin/bash
# root pass with the U previous-tree walks interleaved vs the previous library (scratch_ab/): same
# models, same-box timings
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
OLD="env COBALT_NATIVE_LIB=$PWD/scratch_ab/libcobalt_hip_old.so"
$T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/wk_d1.log 2>&1 &&
$OLD $T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/wk_d0.log 2>&1 &&
$T 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/wk_tests.log 2>&1 &&
$OLD $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/wk_off10m.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/wk_on10m.log 2>&1 &&
$OLD $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/wk_off10m_b.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/wk_on10m_b.log 2>&1 &&
$OLD $T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/wk_off1m.log 2>&1 &&
$T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/wk_on1m.log 2>&1
rc=$?
for f in wk_d1 wk_d0; do echo "$f $(tail -1 gpurun_out/$f.log)"; done
tail -1 gpurun_out/wk_tests.log
for f in wk_off10m wk_on10m wk_off10m_b wk_on10m_b wk_off1m wk_on1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
exit $rc
