#!/bin/bash
# Profile evidence of the current trainer: in-kernel stamps (1M, 10M), rocprofv3 kernel traces of one
# 300-tree fit (10M, 1M) and the wave-state PMC passes (10M, 20 trees). Each step has its own limit.
set -o pipefail
bash scripts/gpu_stamps.sh || exit $?
bash scripts/gpu_prof.sh r10m 300 300 --steps 1 --warmup 0 --test-rows 10000 || exit $?
bash scripts/gpu_prof.sh r1m 200 300 --rows 1000000 --steps 1 --warmup 0 --test-rows 10000 || exit $?
bash scripts/gpu_pmc2.sh || exit $?
