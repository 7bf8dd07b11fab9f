#!/bin/bash
# tail-fused reduce: correctness (oracle bit-identity, DP), stamps, same-box A/B vs COBALT_FUSE_RED=0
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4p_gbdt 600 python -u -m pytest tests/test_gpu_gbdt.py tests/test_00gpu_dp_ipc.py -x -v -m gpu --timeout 500 --timeout-method thread || exit $?
grep -q " failed\|FAILED\| error" gpurun_out/r4p_gbdt.log && { echo "tests failed"; exit 1; }
rm -f gpurun_out/st_fused.txt
COBALT_TRAINER_CACHE=0 COBALT_STAMPS=gpurun_out/st_fused.txt bash $S r4p_st 200 python -u scripts/stamps_single.py 1000000 || exit $?
python scripts/stamp_summary.py gpurun_out/st_fused.txt > gpurun_out/st_fused.summary.txt || exit $?
rm -f gpurun_out/st_fused.txt
for rep in 1 2; do
  for rows in 1000000 1250000 10000000; do
    bash $S r4p_on_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
    COBALT_FUSE_RED=0 bash $S r4p_off_${rows}_$rep 200 python bench.py --rows $rows --steps 3 --warmup 1 || exit $?
  done
done
for f in gpurun_out/r4p_o*_*.log; do echo "$(basename $f) $(grep -ho '"ms_per_step": [0-9.]*' $f)"; done
