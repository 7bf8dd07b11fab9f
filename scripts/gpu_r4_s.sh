#!/bin/bash
# IPC peer reads with system-scope loads (no L2-invalidating acquire): DP correctness + 1-rank A/B
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4s_dp 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -v -m gpu --timeout 700 --timeout-method thread || exit $?
grep -q "FAILED\| failed" gpurun_out/r4s_dp.log && { echo "dp tests failed"; exit 1; }
for rep in 1 2; do
  bash $S r4s_new_$rep 400 python -u scripts/dp_overhead_probe.py --rows 1250000 || exit $?
  COBALT_NATIVE_LIB=$PWD/abref/libcobalt_hip_fence.so bash $S r4s_fence_$rep 400 python -u scripts/dp_overhead_probe.py --rows 1250000 || exit $?
done
grep -h "passed\|failed" gpurun_out/r4s_dp.log | tail -1
for f in gpurun_out/r4s_new_*.log gpurun_out/r4s_fence_*.log; do echo "$(basename $f) $(grep -h '^{' $f)"; done
