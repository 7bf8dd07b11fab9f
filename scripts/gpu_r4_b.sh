#!/bin/bash
# Round 4 call B: exact full-data sketch (tests + 10M timing), DP test matrix, 8-rank diagnostics,
# the new GPU tests (AUC parity at 2M, reference UI on the GPU engine, concurrent serving).
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4b_sketch_tests 300 python -u -m pytest tests/test_sketch.py -x -v -m gpu --timeout 200 --timeout-method thread || exit $?
bash $S r4b_sketch_probe 200 python -u scripts/sketch_exact_probe.py || exit $?
bash $S r4b_new_tests 700 python -u -m pytest tests/test_gpu_auc_parity.py tests/test_reference_ui.py tests/test_gpu_serve.py -x -v -s -m gpu --timeout 600 --timeout-method thread || exit $?
bash $S r4b_dp_tests 900 python -u -m pytest tests/test_00gpu_dp_ipc.py -x -v --timeout 600 --timeout-method thread || exit $?
bash $S r4b_dp8 900 python -u scripts/dp8_diag.py || exit $?
