#!/bin/bash
# exact out-of-core with the all-row (streamed) sketch: 10M host / HBM, 100M HBM (+ in-core compare)
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4d3_ooc_exact_10m_host 400 python -u scripts/bench_external.py --rows 10000000 --sample-rate 1.0 --compare-in-core || exit $?
bash $S r4d3_ooc_exact_100m_dev 700 python -u scripts/bench_external.py --rows 100000000 --sample-rate 1.0 --device-page-gb 8 --compare-in-core || exit $?
grep -h '^{' gpurun_out/r4d3_*.log | cut -c1-600
