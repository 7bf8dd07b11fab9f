#!/bin/bash
# the driver's N=2 and N=4 bench commands rehearsed on one GPU (ranks share cuda:0, IPC exchange with
# node ownership), 10M rows, each checked against the 1-rank bench (same AUC = same trees)
set -o pipefail
export PYTHONUNBUFFERED=1
ROWS=10000000 bash scripts/gpu_bench_multirank.sh 2 > gpurun_out/mr2.txt 2>&1 &&
ROWS=10000000 bash scripts/gpu_bench_multirank.sh 4 > gpurun_out/mr4.txt 2>&1
rc=$?
tail -3 gpurun_out/mr2.txt gpurun_out/mr4.txt
exit $rc
