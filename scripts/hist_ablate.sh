#!/bin/bash
# k_hist time split on the small, wide RFE fits (timing-only ablations; results are wrong by design)
for a in 0 1 2 3 4; do
  COBALT_HIST_ABLATE=$a timeout -k 10 120 python -u scripts/rfe_probe.py > gpurun_out/abl_$a.log 2>&1 || exit $?
  echo "ablate $a: $(grep 'width 106' gpurun_out/abl_$a.log | tail -1)"
done
