#!/usr/bin/env python
"""Data-parallel protocol overhead on ONE GPU: the 10M-row fit with a 1-rank RCCL communicator (the
trainer then runs the DP code path: global-hessian child choice + an in-stream RCCL int64
all-reduce per level) against the plain single-GPU fit. Same trees (asserted); prints both times."""
import ctypes
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd import _native  # noqa: E402
from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402
from cobalt_smart_lender_ai_amd.parallel.dist import DistContext  # noqa: E402

dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(10_000_000, seed=0, device=dev)
spw = float((y == 0).sum() / (y == 1).sum())
p = gbdt.GBDTParams(n_estimators=300, max_depth=7, learning_rate=0.05, gamma=5.0, scale_pos_weight=spw,
                    random_state=78)
lib = _native.lib()
assert lib.cobalt_comm_load(_native.rccl_path().encode()) == 0
uid = (ctypes.c_uint8 * 128)()
assert lib.cobalt_comm_unique_id(uid) == 0
h = ctypes.c_void_p()
assert lib.cobalt_comm_init(uid, 1, 0, ctypes.byref(h)) == 0
ctx = DistContext(rank=0, world=1, local_rank=0, backend="none", native_comm=h.value)


def timed(**kw):
    gbdt.train(X, y, p, device=dev, **kw)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b = gbdt.train(X, y, p, device=dev, **kw)
    torch.cuda.synchronize()
    return b, (time.perf_counter() - t0) * 1e3


b1, t1 = timed()
b2, t2 = timed(dist=ctx)
assert b1.save_raw("ubj") == b2.save_raw("ubj")
print(f"single-GPU path {t1:.1f} ms   DP path with 1-rank RCCL {t2:.1f} ms   overhead {t2 - t1:+.1f} ms "
      f"({(t2 - t1) / 300 * 1e3:.0f} us per tree, 7 all-reduces)", flush=True)
lib.cobalt_comm_destroy(h, 0)
