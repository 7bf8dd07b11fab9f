#!/bin/bash
# Round-2 baseline: headline bench (10M), 1M / 1.25M fits, and a kernel trace of the 1M fit.
set -o pipefail
S=scripts/gpu_step.sh
bash $S bench10m 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S bench1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash $S bench1p25m 200 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
COBALT_FUSED_PART=1 bash $S bench1m_fused 200 python bench.py --rows 1000000 --steps 3 --warmup 1 || exit $?
bash scripts/gpu_prof.sh r1m 300 300 --rows 1000000 --steps 1 --warmup 1 || exit $?
grep -h "^{" gpurun_out/bench*.log | cut -c1-260
