#!/bin/bash
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4f_oxdbg 300 python -u scripts/ox_debug.py || exit $?
