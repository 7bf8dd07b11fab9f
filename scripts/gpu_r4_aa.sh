#!/bin/bash
# the reference's training job on the GPU with the all-row default sketch vs the 2^18 sample
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4aa_pipe_auto 600 python -u scripts/bench_configs.py pipeline-100k || exit $?
grep -h '^{' gpurun_out/r4aa_pipe_auto.log | cut -c1-600
