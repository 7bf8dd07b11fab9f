#!/bin/bash
# Round 4 call D: exact out-of-core streaming measurements (host-streamed and HBM-resident pages).
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4d_ooc_exact_10m_host 400 python -u scripts/bench_external.py --rows 10000000 --sample-rate 1.0 --compare-in-core || exit $?
bash $S r4d_ooc_exact_10m_dev 400 python -u scripts/bench_external.py --rows 10000000 --sample-rate 1.0 --device-page-gb 8 || exit $?
bash $S r4d_ooc_sampled_10m_host 400 python -u scripts/bench_external.py --rows 10000000 || exit $?
grep -h '^{' gpurun_out/r4d_*.log
