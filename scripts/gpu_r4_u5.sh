#!/bin/bash
# k_hist lane-pair gathers with 5 rows in flight per pair (F <= 20) vs the previous library (scratch_ab/):
# same models, same-box timings
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
OLD="env COBALT_NATIVE_LIB=$PWD/scratch_ab/libcobalt_hip_old.so"
$T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/u5_d1.log 2>&1 &&
$OLD $T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/u5_d0.log 2>&1 &&
$T 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/u5_tests.log 2>&1 &&
$OLD $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/u5_off10m.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/u5_on10m.log 2>&1 &&
$OLD $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/u5_off10m_b.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/u5_on10m_b.log 2>&1 &&
$OLD $T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/u5_off1m.log 2>&1 &&
$T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/u5_on1m.log 2>&1
rc=$?
for f in u5_d1 u5_d0; do echo "$f $(tail -1 gpurun_out/$f.log)"; done
tail -1 gpurun_out/u5_tests.log
for f in u5_off10m u5_on10m u5_off10m_b u5_on10m_b u5_off1m u5_on1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
exit $rc
