#!/bin/bash
# Round 4: data-parallel correctness (2/3/4/8 processes on one GPU with CU-masked streams, replica
# divergence fault injection), oracle tests, then the DP-protocol cost at the 8-GPU shard size.
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4dp_tests 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -x -v --timeout 600 --timeout-method thread || exit $?
bash $S r4dp_oracle 600 python -u -m pytest tests/test_gpu_gbdt.py -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r4dp_1m 200 python bench.py --rows 1000000 --steps 3 --warmup 1 --profile-fit || exit $?
bash $S r4dp_1p25m 200 python bench.py --rows 1250000 --steps 3 --warmup 1 --profile-fit || exit $?
bash $S r4dp_probe 300 python -u scripts/dp_overhead_probe.py --rows 1250000 || exit $?
bash $S r4dp_bench 300 python bench.py || exit $?
