#!/bin/bash
# One trainer iteration on the GPU box: GBDT GPU tests, 1M / 10M benches, in-kernel stamps.
# usage: [AB_ENV="VAR=value"] gpu_iter.sh [pytest-selection...]
# AB_ENV: also run both benches with that environment setting (A/B of a tuning switch).
set -o pipefail
S=scripts/gpu_step.sh
sel=${@:-tests/test_gpu_gbdt.py}
bash $S iter_tests 500 python -u -m pytest $sel -x -q --timeout 600 --timeout-method thread || exit $?
bash $S iter_bench1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash $S iter_bench10m 300 python bench.py --steps 3 --warmup 1 || exit $?
if [ -n "$AB_ENV" ]; then
  env $AB_ENV bash $S iter_bench1m_ab 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
  env $AB_ENV bash $S iter_bench10m_ab 300 python bench.py --steps 3 --warmup 1 || exit $?
fi
bash scripts/gpu_stamps.sh || exit $?
for f in gpurun_out/iter_bench*.log; do echo "$f: $(grep -h '^{' $f | cut -c1-220)"; done
