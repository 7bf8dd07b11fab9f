#!/bin/bash
# 10M-row bench under tuning knobs (one line per variant: name ms auc)
set -o pipefail
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/knob_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/knob_$name.log; exit 1; }
  python -c "import json,sys; l=[x for x in open('gpurun_out/knob_$name.log') if x.startswith('{')][-1]; d=json.loads(l); print('$name', d['ms_per_step'], d['auc'])" | tee -a gpurun_out/knob_summary.txt
}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  run $name $envs || exit 1
done
