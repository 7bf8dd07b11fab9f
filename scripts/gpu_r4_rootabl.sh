#!/bin/bash
# timing-only ablations of the fused root pass at 10M rows (results are wrong by design):
# 0 = none, 20 = no exp, 21 = no LDS histogram atomics, 22 = no previous-tree walk
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && cd $R
for m in 0 20 21 22; do
  COBALT_HIST_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/rabl$m -o run -- python3 bench.py --rows 10000000 --trees 20 --steps 1 --warmup 0 --test-rows 100000 > gpurun_out/rabl$m.log 2>&1 || exit $?
  echo "ablate=$m"; python3 scripts/prof_summary.py /tmp/rabl$m/run_kernel_trace.csv 20 | grep -E "k_grad_hist" | head -3
done
