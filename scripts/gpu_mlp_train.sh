#!/bin/bash
# MFMA MLP trainer: numerics vs the PyTorch oracle, epoch timing vs the scalar-FMA trainer.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_nn.py > $R/gpurun_out/mlp_train_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|\[nn\]|Error|assert" $R/gpurun_out/mlp_train_tests.log | head -60
exit $rc
