#!/bin/bash
# root-pass record prefetch (COBALT_GRAD_PREFETCH): same models, then same-box timings (0 = off)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/gpf_d1.log 2>&1 &&
COBALT_GRAD_PREFETCH=0 $T 200 python scripts/model_digest.py --rows 10000000 > gpurun_out/gpf_d0.log 2>&1 &&
$T 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpf_tests.log 2>&1 &&
COBALT_GRAD_PREFETCH=0 $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/gpf_off10m.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/gpf_on10m.log 2>&1 &&
COBALT_GRAD_PREFETCH=0 $T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/gpf_off10m_b.log 2>&1 &&
$T 300 python bench.py --steps 3 --warmup 1 > gpurun_out/gpf_on10m_b.log 2>&1 &&
COBALT_GRAD_PREFETCH=0 $T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/gpf_off1m.log 2>&1 &&
$T 300 python bench.py --rows 1000000 --steps 3 --warmup 1 > gpurun_out/gpf_on1m.log 2>&1
rc=$?
for f in gpf_d1 gpf_d0; do echo "$f $(tail -1 gpurun_out/$f.log)"; done
tail -2 gpurun_out/gpf_tests.log
for f in gpf_off10m gpf_on10m gpf_off10m_b gpf_on10m_b gpf_off1m gpf_on1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
exit $rc
