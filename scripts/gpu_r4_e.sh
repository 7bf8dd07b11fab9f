#!/bin/bash
# Round 4 call E: same-box A/B of the round-3 library (abref) vs HEAD (ep_plan on / off) at the
# strong-scaling shard sizes + 10M; exact-sketch stage timings; exact OOC streaming tests.
set -o pipefail
S=scripts/gpu_step.sh
REF=$PWD/abref/libcobalt_hip_ref.so
bash $S r4e_oxdbg 300 python -u scripts/ox_debug.py || exit $?
bash $S r4e_ext_tests 600 python -u -m pytest tests/test_external.py -v -m gpu --timeout 500 --timeout-method thread || exit $?
COBALT_SK_TIMING=1 bash $S r4e_sketch 200 python -u scripts/sketch_exact_probe.py --reps 3 || exit $?
for rep in 1 2; do
  for rows in 1000000 1250000 10000000; do
    COBALT_NATIVE_LIB=$REF bash $S r4e_ref_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
    bash $S r4e_new_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
    COBALT_EP_PLAN=0 bash $S r4e_nop_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
  done
done
for f in gpurun_out/r4e_*_*_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
