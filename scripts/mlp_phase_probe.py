"""Per-phase timing of the fused MLP trainer (s_memrealtime, 100 MHz) for one full-size epoch."""
import ctypes

import numpy as np
import torch

from cobalt_smart_lender_ai_amd import _native
from cobalt_smart_lender_ai_amd.nn import mlp

rng = np.random.default_rng(0)
N, F = 78034, 20
X = torch.as_tensor(rng.random((N, F)).astype(np.float32), device="cuda")
y = torch.as_tensor((rng.random(N) < 0.13).astype(np.float32), device="cuda")
cfg = mlp.MLPConfig()
rate, ds = cfg.decay(N)
hp = mlp._Hyper(cfg.initial_lr, rate, ds, 1, cfg.weight_decay, cfg.beta1, cfg.beta2, cfg.eps, cfg.lambda_l2, 32)
p = torch.as_tensor(mlp.init_params(F)[None], device="cuda").contiguous()
m, v = torch.zeros_like(p), torch.zeros_like(p)
steps = torch.zeros(1, dtype=torch.int64, device="cuda")
loss = torch.zeros(1, device="cuda")
perm = torch.as_tensor(rng.permutation(N).astype(np.int32)[None], device="cuda").contiguous()
prof = torch.zeros(7, dtype=torch.int64, device="cuda")
lib = _native.lib()
for it in range(2):
    prof.zero_()
    torch.cuda.synchronize()
    import time
    t = time.perf_counter()
    rc = lib.cobalt_mlp_train_epoch(X.data_ptr(), F, y.data_ptr(), N, F, perm.data_ptr(), p.data_ptr(), m.data_ptr(),
                                    v.data_ptr(), steps.data_ptr(), ctypes.byref(hp), 1, loss.data_ptr(),
                                    prof.data_ptr(), _native.stream_handle())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    assert rc == 0
names = ["load+sync", "forward", "loss", "phaseA", "phaseB", "phaseC", "phaseD"]
us = prof.cpu().numpy() / 100.0 / (N // 32 + 1)
print(f"epoch {dt*1e3:.1f} ms, {dt/(N//32+1)*1e6:.2f} us/step")
for n_, u in zip(names, us):
    print(f"{n_:10s} {u:7.2f} us/step")
