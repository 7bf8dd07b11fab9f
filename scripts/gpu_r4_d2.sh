#!/bin/bash
# Round 4 call D2: exact out-of-core streaming at 100M rows (HBM-resident pages vs host-streamed pages).
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4d_ooc_exact_100m_dev 600 python -u scripts/bench_external.py --rows 100000000 --sample-rate 1.0 --device-page-gb 8 --compare-in-core || exit $?
bash $S r4d_ooc_exact_100m_host 600 python -u scripts/bench_external.py --rows 100000000 --sample-rate 1.0 || exit $?
grep -h '^{' gpurun_out/r4d_*100m*.log
