#!/bin/bash
# OOC exact debug after the staging-buffer fix; same-box stamps of round-3 vs HEAD single-GPU fits
set -o pipefail
S=scripts/gpu_step.sh
REF=$PWD/abref/libcobalt_hip_ref.so
bash $S r4g_oxdbg 300 python -u scripts/ox_debug.py || exit $?
bash $S r4g_ext_tests 600 python -u -m pytest tests/test_external.py -v -m gpu --timeout 500 --timeout-method thread || exit $?
for v in ref new; do
  lib=""; [ $v = ref ] && lib=$REF
  rm -f gpurun_out/st_$v.txt
  COBALT_NATIVE_LIB=$lib COBALT_TRAINER_CACHE=0 COBALT_STAMPS=gpurun_out/st_$v.txt bash $S r4g_st_$v 200 python -u scripts/stamps_single.py 1000000 || exit $?
  python scripts/stamp_summary.py gpurun_out/st_$v.txt > gpurun_out/st_$v.summary.txt || exit $?
  rm -f gpurun_out/st_$v.txt
done
for rep in 1 2; do
  COBALT_NATIVE_LIB=$REF bash $S r4g_ref_1000000_$rep 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
  bash $S r4g_new_1000000_$rep 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
done
for f in gpurun_out/r4g_*_*_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
