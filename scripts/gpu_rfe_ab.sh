#!/bin/bash
# A/B of two trainer builds: GBDT oracle tests on the current one, then the RFE-stage fit probe and
# the 10M / 1M fits with the reference library (abref/) and the current one.
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
REF=$PWD/abref/libcobalt_hip_ref.so
COBALT_NATIVE_LIB=$REF bash $S rfe_ref 200 python -u scripts/rfe_probe.py || exit $?
bash $S rfe_new 200 python -u scripts/rfe_probe.py || exit $?
COBALT_NATIVE_LIB=$REF bash $S ref10m 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S new10m 300 python bench.py --steps 3 --warmup 1 || exit $?
COBALT_NATIVE_LIB=$REF bash $S ref1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash $S new1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
grep -h "width" gpurun_out/rfe_ref.log gpurun_out/rfe_new.log
for f in ref10m new10m ref1m new1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
