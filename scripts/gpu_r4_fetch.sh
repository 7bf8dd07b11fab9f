#!/bin/bash
# HBM bytes fetched per dispatch (FETCH_SIZE, one counter pass) of the 10M-row fit's main kernels
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && cd $R
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_hist|k_partition|k_grad_hist' --output-format csv -d /tmp/fetch -o run -- python3 bench.py --rows 10000000 --trees 10 --steps 1 --warmup 0 --test-rows 100000 > gpurun_out/fetch.log 2>&1 &&
find /tmp/fetch -name '*counter_collection.csv' -exec cp {} gpurun_out/fetch_10M.csv \; &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_hist|k_partition|k_grad_hist' --output-format csv -d /tmp/wsz -o run -- python3 bench.py --rows 10000000 --trees 10 --steps 1 --warmup 0 --test-rows 100000 > gpurun_out/wsz.log 2>&1 &&
find /tmp/wsz -name '*counter_collection.csv' -exec cp {} gpurun_out/write_10M.csv \;
