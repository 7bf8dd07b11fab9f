#!/usr/bin/env python
"""In-kernel stamps (COBALT_STAMPS) of one 1.25M-row fit per data-parallel protocol variant on ONE GPU,
1-rank groups: single GPU / IPC fused exchange (k_eval_part's evaluator blocks; with COBALT_EVAL_BLOCKS=0
k_eval + k_partition) / RCCL (k_eval_part mode 1). The caller sets COBALT_STAMPS (raw stamps, summarised
by scripts/stamp_summary.py). usage: dp_stamps_probe.py ROWS single|ipc|rccl"""
import ctypes
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd import _native  # noqa: E402
from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402
from cobalt_smart_lender_ai_amd.parallel.dist import DistContext, create_ipc_comm  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(rows, seed=0, device=dev)
spw = float((y == 0).sum() / (y == 1).sum())
p = gbdt.GBDTParams(n_estimators=70, max_depth=7, learning_rate=0.05, gamma=5.0, scale_pos_weight=spw, random_state=78)
lib = _native.lib()
assert lib.cobalt_comm_load(_native.rccl_path().encode()) == 0
uid = (ctypes.c_uint8 * 128)()
assert lib.cobalt_comm_unique_id(uid) == 0
h = ctypes.c_void_p()
assert lib.cobalt_comm_init(uid, 1, 0, ctypes.byref(h)) == 0
rccl = DistContext(rank=0, world=1, local_rank=0, backend="none", native_comm=h.value, transport="rccl")
ipc = DistContext(rank=0, world=1, local_rank=0, backend="none", transport="ipc")
ipc.native_comm = create_ipc_comm(ipc)
# COBALT_STAMPS / COBALT_EVAL_BLOCKS are read when a trainer context is created / per process: one
# variant per process invocation (argv[2])
name = sys.argv[2]
kw = {"single": {}, "ipc": {"dist": ipc}, "rccl": {"dist": rccl}}[name]
gbdt.train(X, y, p, device=dev, **kw)
torch.cuda.synchronize()
print(f"{name} done", flush=True)
