#!/bin/bash
# stamps of the DP protocol variants at the 8-GPU shard size (1-rank groups on one GPU)
set -o pipefail
for v in single ipc ipc_ep rccl; do
  ep=0; [ "$v" = ipc_ep ] && ep=1
  rm -f gpurun_out/dpst_$v.txt
  COBALT_DP_EVAL_PART=$ep COBALT_TRAINER_CACHE=0 COBALT_STAMPS=gpurun_out/dpst_$v.txt timeout -k 10 200 \
    python -u scripts/dp_stamps_probe.py 1250000 $v > gpurun_out/dpst_$v.log 2>&1 || exit $?
  python scripts/stamp_summary.py gpurun_out/dpst_$v.txt > gpurun_out/dpst_$v.summary.txt || exit $?
  rm -f gpurun_out/dpst_$v.txt
  tail -8 gpurun_out/dpst_$v.summary.txt
done
