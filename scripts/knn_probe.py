#!/usr/bin/env python
"""SMOTE kNN at the full-data minority size (~295k rows x 20 features, k=5 + self) on the MFMA distance
kernel (csrc/knn.hip)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.nn.smote import kneighbors  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 295_000
X = np.random.default_rng(0).random((n, 20), dtype=np.float32)
kneighbors(X[:4096], X[:4096], 6, device="cuda")
torch.cuda.synchronize()
t = time.perf_counter()
kneighbors(X, X, 6, device="cuda")
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(f"knn n={n} k=6: {dt * 1e3:.1f} ms, {n * n * 20 * 2 / dt / 1e12:.1f} TFLOP/s of distance GEMM", flush=True)
