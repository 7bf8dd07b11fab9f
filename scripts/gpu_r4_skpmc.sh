#!/bin/bash
# SQ counters of the exact-sketch kernels at 10M x 20 (one pass, counters only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT --kernel-include-regex 'k_sk_' --output-format csv -d /tmp/skpmc -o run -- python3 $R/scripts/sketch_exact_probe.py --rows 10000000 --reps 1 --only-exact > $R/gpurun_out/skpmc.log 2>&1 &&
find /tmp/skpmc -name '*counter_collection.csv' -exec cp {} $R/gpurun_out/skpmc.csv \;
