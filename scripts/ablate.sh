#!/bin/bash
# timing-only ablations of the histogram kernel (results are wrong by design)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 0 1 2; do
  COBALT_HIST_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abl$m -o run -- python bench.py --rows 10000000 --trees 5 --steps 1 --warmup 0 --test-rows 100000 > gpurun_out/abl$m.log 2>&1 || exit $?
  python scripts/prof_summary.py gpurun_out/abl$m/run_kernel_trace.csv 5 | grep -E "k_hist" | head -12
done
