#!/bin/bash
# sketch v2 (single-pass gather, transpose kernel, device exact rows): tests + timings
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4i_sketch_tests 300 python -u -m pytest tests/test_sketch.py -v -m gpu --timeout 250 --timeout-method thread || exit $?
COBALT_SK_TIMING=1 bash $S r4i_sketch_timing 200 python -u scripts/sketch_exact_probe.py --reps 3 || exit $?
bash $S r4i_sketch_probe 200 python -u scripts/sketch_exact_probe.py --reps 5 || exit $?
bash $S r4i_bench_all 300 python bench.py --sketch-rows 0 --steps 3 --warmup 1 || exit $?
grep -h '^{' gpurun_out/r4i_sketch_probe.log gpurun_out/r4i_bench_all.log
