#!/bin/bash
# Final-state profiles: rocprofv3 kernel trace of one 300-tree 10M fit, TA busy and HBM bytes per kernel.
set -o pipefail
bash scripts/gpu_prof.sh final10m 300 300 --steps 1 --warmup 0 --test-rows 10000 || exit $?
bash scripts/gpu_pmc_ta.sh || exit $?
bash scripts/gpu_pmc_bytes.sh || exit $?
