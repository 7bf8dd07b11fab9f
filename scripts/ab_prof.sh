#!/bin/bash
# Kernel traces of the unfused / fused / hessian-choice variants + timing of the hessian-choice variant.
set -o pipefail
bash scripts/gpu_step.sh fused_test 300 python -u -m pytest tests/test_gpu_gbdt.py -k fused -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
bash scripts/gpu_prof.sh unfused 300 300 --steps 1 --warmup 0 > /dev/null || exit $?
COBALT_FUSED_PART=1 bash scripts/gpu_prof.sh fused 300 300 --steps 1 --warmup 0 > /dev/null || exit $?
COBALT_BUILD_BY_HESS=1 bash scripts/gpu_prof.sh byhess 300 300 --steps 1 --warmup 0 > /dev/null || exit $?
COBALT_BUILD_BY_HESS=1 bash scripts/gpu_step.sh bench_byhess 300 python bench.py --steps 3 --warmup 1 || exit $?
for v in unfused fused byhess; do echo "== $v"; head -12 gpurun_out/prof_$v.summary.txt; done
