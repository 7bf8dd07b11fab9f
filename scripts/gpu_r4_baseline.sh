#!/bin/bash
# Round-4 opening call: the GPU test tier, the driver's bench, and the 4- / 8-process IPC data-parallel
# rehearsal on one GPU (ipc_sum_cells<4> / <8>, the instantiations an 8-GPU node runs).
set -o pipefail
S=scripts/gpu_step.sh
bash $S r4_gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r4_bench 300 python bench.py || exit $?
bash $S r4_dp48 600 python -u -c "
from cobalt_smart_lender_ai_amd.parallel import dp_check
import json
ref = dp_check.run(1, 300000)[0]
print('ref', ref.get('ok'), ref.get('model_sha256'), ref.get('fit_s'), flush=True)
for n in (4, 8):
    got = dp_check.run(n, 300000, timeout_s=250)
    print(n, json.dumps([{k: g.get(k) for k in ('rank','ok','transport','error','message','fit_s','ipc_epochs')} for g in got]), flush=True)
    print(n, 'identical', all(g.get('model_sha256') == ref['model_sha256'] for g in got), flush=True)
" || exit $?
