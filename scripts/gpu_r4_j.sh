#!/bin/bash
# sketch v2 + wave-aggregated hist atomics: tests, stage timings, bench default (all rows) vs 2^18 sample
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4j_sketch_tests 300 python -u -m pytest tests/test_sketch.py -v -m gpu --timeout 250 --timeout-method thread || exit $?
COBALT_SK_TIMING=1 bash $S r4j_sketch_timing 200 python -u scripts/sketch_exact_probe.py --reps 3 || exit $?
bash $S r4j_sketch_probe 200 python -u scripts/sketch_exact_probe.py --reps 5 || exit $?
for rep in 1 2; do
bash $S r4j_bench_all_$rep 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S r4j_bench_samp_$rep 300 python bench.py --sketch-rows 262144 --steps 3 --warmup 1 || exit $?
done
grep -h '^{' gpurun_out/r4j_sketch_probe.log
for f in gpurun_out/r4j_bench_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*\|"fit_breakdown_ms": {[^}]*}\|"auc": [0-9.]*' $f | tr '\n' ' ')"; done
