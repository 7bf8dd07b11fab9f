#!/bin/bash
# In-kernel stamps at 10M rows without and with an environment switch. usage: gpu_env_stamps.sh VAR VALUE
set -o pipefail
STAMP_ROWS=10000000 bash scripts/gpu_stamps.sh > /dev/null || exit $?
mv gpurun_out/stamps_10000000.summary.txt gpurun_out/stamps_off.txt
env $1=$2 STAMP_ROWS=10000000 bash scripts/gpu_stamps.sh > /dev/null || exit $?
mv gpurun_out/stamps_10000000.summary.txt gpurun_out/stamps_on.txt
head -4 gpurun_out/stamps_off.txt; tail -6 gpurun_out/stamps_off.txt
head -4 gpurun_out/stamps_on.txt; tail -6 gpurun_out/stamps_on.txt
