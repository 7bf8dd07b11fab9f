#!/bin/bash
# Timing-only ablations of k_partition (results are wrong by construction): 11 no bin gathers,
# 12 no cursor atomics, 13 no scatter stores. Kernel-trace summaries land in gpurun_out/.
R=$GRAFT_REPO_ROOT
for ab in 0 11 12 13; do
  COBALT_HIST_ABLATE=$ab bash $R/scripts/gpu_prof.sh abl$ab 300 30 --trees 30 --steps 1 --warmup 1 --test-rows 10000 > /dev/null || exit $?
  echo "== ablate $ab"; grep -E "k_partition|k_hist " $R/gpurun_out/prof_abl$ab.summary.txt | head -3
done
