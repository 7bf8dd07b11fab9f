#!/bin/bash
# 1-GPU rehearsal of the driver's multi-rank bench: N torchrun ranks share cuda:0 over a gloo bootstrap
# and the native IPC communicator (the 8-GPU run bootstraps over RCCL and runs the same IPC exchange
# across GPUs), then the 1-rank bench of the same rows; the two AUCs must be equal (same trees).
set -o pipefail
N=${1:-2}
ROWS=${ROWS:-2000000}
mkdir -p gpurun_out
COBALT_DIST_BACKEND=gloo COBALT_DIST_NATIVE=1 COBALT_BENCH_SHARED_DEVICE=1 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus "$N" --rows "$ROWS" --steps 2 --warmup 1 > gpurun_out/bench_multirank_$N.json \
  2> gpurun_out/bench_multirank_$N.err || exit $?
timeout -k 10 300 python bench.py --rows "$ROWS" --steps 2 --warmup 1 > gpurun_out/bench_multirank_1.json \
  2> gpurun_out/bench_multirank_1.err || exit $?
cat gpurun_out/bench_multirank_$N.json gpurun_out/bench_multirank_1.json
python - "$N" <<'PY'
import json, sys
n = sys.argv[1]
a = json.loads(open(f"gpurun_out/bench_multirank_{n}.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/bench_multirank_1.json").read().strip().splitlines()[-1])
assert a["n_gpus"] == int(n) and a["dp_transport"] == "ipc", a
assert a["auc"] == b["auc"], (a["auc"], b["auc"])
assert a["replicas_agree"] is True, a  # every rank holds the same model
print(f"ranks {n}: {a['ms_per_step']} ms/fit (all ranks on one GPU), 1 rank {b['ms_per_step']} ms; AUC {a['auc']} equal")
PY
