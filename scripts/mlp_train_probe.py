#!/usr/bin/env python
"""Epoch time of the MLP trainers (78k rows x 20 features, batch 32 = 2439 steps, one model; and
G models in one launch) and the per-phase split of the MFMA trainer (s_memrealtime, waves 0 and 3)."""
import ctypes
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd import _native  # noqa: E402
from cobalt_smart_lender_ai_amd.nn import mlp  # noqa: E402

rng = np.random.default_rng(0)
N, F = 78034, 20
X = torch.as_tensor(rng.random((N, F)).astype(np.float32), device="cuda")
y = torch.as_tensor((rng.random(N) < 0.13).astype(np.float32), device="cuda")
cfg = mlp.MLPConfig()
rate, ds = cfg.decay(N)
hp = mlp._Hyper(cfg.initial_lr, rate, ds, 1, cfg.weight_decay, cfg.beta1, cfg.beta2, cfg.eps, cfg.lambda_l2, 32)
lib = _native.lib()
nsteps = -(-N // 32)


def run(kernel, G, prof=None):
    p = torch.as_tensor(np.stack([mlp.init_params(F, s) for s in range(G)]), device="cuda").contiguous()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    steps = torch.zeros(G, dtype=torch.int64, device="cuda")
    loss = torch.zeros(G, device="cuda")
    perm = torch.as_tensor(np.stack([rng.permutation(N) for _ in range(G)]).astype(np.int32), device="cuda")
    pp = prof.data_ptr() if prof is not None else None
    ts = []
    for _ in range(3):
        if prof is not None:
            prof.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        if kernel == "mfma":
            rc = lib.cobalt_mlp_train_epoch_mfma(X.data_ptr(), F, y.data_ptr(), N, F, perm.data_ptr(), p.data_ptr(),
                                                 m.data_ptr(), v.data_ptr(), steps.data_ptr(), ctypes.byref(hp), G,
                                                 loss.data_ptr(), pp, _native.stream_handle())
        else:
            rc = lib.cobalt_mlp_train_epoch(X.data_ptr(), F, y.data_ptr(), N, F, perm.data_ptr(), p.data_ptr(),
                                            m.data_ptr(), v.data_ptr(), steps.data_ptr(), ctypes.byref(hp), G,
                                            loss.data_ptr(), pp, _native.stream_handle())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
        assert rc == 0
    dt = min(ts)
    print(f"{kernel:5s} G={G:4d}: {dt * 1e3:7.2f} ms/epoch  {dt / nsteps * 1e6:6.2f} us/step  "
          f"{G * N / dt / 1e6:8.2f}M rows/s  loss={float(loss[0]) / nsteps:.5f}", flush=True)


prof = torch.zeros(16, dtype=torch.int64, device="cuda")
run("mfma", 1, prof)
us = prof.cpu().numpy() / 100.0 / nsteps
names = ["fetch", "F1 (L1, L2 partial)", "barrier 1", "F2 (L2..out, deltas)", "barrier 2", "G (grads, AdamW)",
         "barrier 3"]
for i, nm in enumerate(names):
    print(f"  {nm:22s} wave0 {us[i]:6.2f} us/step   wave3 {us[8 + i]:6.2f}")
prof7 = torch.zeros(7, dtype=torch.int64, device="cuda")
run("fma", 1, prof7)
us = prof7.cpu().numpy() / 100.0 / nsteps
print("  fma phases (us/step): " + " ".join(f"{u:.2f}" for u in us))
for G in (64, 256, 1024):
    run("mfma", G)
    run("fma", G)
