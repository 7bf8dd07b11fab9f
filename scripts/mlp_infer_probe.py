#!/usr/bin/env python
"""MLP challenger bulk inference (20 features, Dense 128-32-16-1), device-resident rows: the fp32
MFMA kernel vs the scalar-FMA kernel (csrc/mlp.hip). Prints rows/s and effective fp32 TFLOP/s
(2 * 7184 flops per row at F = 20). ``python scripts/mlp_infer_probe.py [N] [reps] [kernels]``."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.nn import mlp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
kernels = sys.argv[3].split(",") if len(sys.argv) > 3 else ["mfma", "fma"]
F = 20
macs = F * 128 + 128 * 32 + 32 * 16 + 16
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.rand((n, F), device="cuda", generator=g)
p = torch.as_tensor(mlp.init_params(F, seed=1), device="cuda")
out = torch.empty(n, device="cuda")
for k in kernels:
    mlp.mlp_forward_gpu(X, p, out, kernel=k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        mlp.mlp_forward_gpu(X, p, out, kernel=k)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    dt = sorted(ts)[len(ts) // 2]
    print(f"mlp forward kernel={k} n={n}: {dt * 1e3:.3f} ms  {n / dt / 1e9:.3f}G rows/s  "
          f"{2 * macs * n / dt / 1e12:.1f} TFLOP/s  mean_prob={float(out.mean()):.6f}", flush=True)
