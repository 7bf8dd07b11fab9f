#!/bin/bash
# A/B of two trainer builds (abref/ = reference, in-tree = new): GBDT oracle tests on the new one, the
# 10M in-kernel stamps and the 10M / 1M fits of both.
set -o pipefail
S=scripts/gpu_step.sh
REF=$PWD/abref/libcobalt_hip_ref.so
bash $S libtests 400 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed" gpurun_out/libtests.log && { echo "tests failed"; exit 1; }
COBALT_NATIVE_LIB=$REF STAMP_ROWS=10000000 bash scripts/gpu_stamps.sh > /dev/null || exit $?
mv gpurun_out/stamps_10000000.summary.txt gpurun_out/stamps_ref.txt
STAMP_ROWS=10000000 bash scripts/gpu_stamps.sh > /dev/null || exit $?
mv gpurun_out/stamps_10000000.summary.txt gpurun_out/stamps_new.txt
COBALT_NATIVE_LIB=$REF bash $S ref10m 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S new10m 300 python bench.py --steps 3 --warmup 1 || exit $?
COBALT_NATIVE_LIB=$REF bash $S ref1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash $S new1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
tail -6 gpurun_out/stamps_ref.txt; tail -6 gpurun_out/stamps_new.txt
for f in ref10m new10m ref1m new1m; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
