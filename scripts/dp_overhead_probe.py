#!/usr/bin/env python
"""Data-parallel protocol overhead on ONE GPU: a fit with 1-rank communicators (the trainer then runs
the DP code path: global-hessian child choice + one histogram collective per level) against the plain
single-GPU fit, for each transport:
  rccl      : in-stream RCCL int64 all-reduce per level (csrc/comm.cpp)
  ipc       : IPC one-shot group, exchange fused into the split evaluation (csrc/ipccomm.hip, default)
  ipc-sep   : IPC one-shot group, separate exchange kernel per level (COBALT_IPC_FUSED=0)
Same trees (asserted). ``--rows`` (default 10M; 1.25M = the 8-GPU strong-scaling shard)."""
import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd import _native  # noqa: E402
from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402
from cobalt_smart_lender_ai_amd.parallel.dist import DistContext, create_ipc_comm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(a.rows, seed=0, device=dev)
spw = float((y == 0).sum() / (y == 1).sum())
p = gbdt.GBDTParams(n_estimators=300, max_depth=7, learning_rate=0.05, gamma=5.0, scale_pos_weight=spw,
                    random_state=78)
lib = _native.lib()
assert lib.cobalt_comm_load(_native.rccl_path().encode()) == 0
uid = (ctypes.c_uint8 * 128)()
assert lib.cobalt_comm_unique_id(uid) == 0
h = ctypes.c_void_p()
assert lib.cobalt_comm_init(uid, 1, 0, ctypes.byref(h)) == 0
rccl = DistContext(rank=0, world=1, local_rank=0, backend="none", native_comm=h.value, transport="rccl")
ipc = DistContext(rank=0, world=1, local_rank=0, backend="none", transport="ipc")
ipc.native_comm = create_ipc_comm(ipc)


def timed(**kw):
    gbdt.train(X, y, p, device=dev, **kw)  # warm-up
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        b = gbdt.train(X, y, p, device=dev, **kw)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return b, min(ts)


b0, t0 = timed()
res = {"rows": a.rows, "single_gpu_ms": round(t0, 2)}
for name, ctx, env in (("rccl", rccl, "1"), ("ipc", ipc, "1"), ("ipc-sep", ipc, "0")):
    os.environ["COBALT_IPC_FUSED"] = env
    b, t = timed(dist=ctx)
    assert b.save_raw("ubj") == b0.save_raw("ubj"), name
    res[f"{name}_ms"] = round(t, 2)
    res[f"{name}_overhead_us_per_level"] = round((t - t0) / (300 * 7) * 1e3, 2)
print(json.dumps(res), flush=True)
lib.cobalt_comm_destroy(h, 0)
lib.cobalt_comm_destroy(ctypes.c_void_p(ipc.native_comm), 0)
