#!/usr/bin/env python
"""Per-fit cost of the reference's RFE fits at production scale (XGBoost defaults: 100 trees, depth 6,
eta 0.3) on ``--rows`` training rows: 106 features (the first RFE step) vs the 21 survivors of the
last step (repacked bins, models/gbdt.subset_features). One line per fit; run under rocprofv3
--kernel-trace --stats for the per-kernel split."""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_320_000)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
n, F = a.rows, 106
X = torch.randn((n, F), generator=g, device=dev)
X[:, ::3] = torch.round(X[:, ::3] * 2)
X[:, 1::7] = (X[:, 1::7] > 0).float()
X[torch.rand((n, F), generator=g, device=dev) < 0.05] = float("nan")
z = torch.nan_to_num(X[:, 0]) - torch.nan_to_num(X[:, 5]) + 0.5 * torch.nan_to_num(X[:, 50])
y = (torch.rand(n, generator=g, device=dev) < torch.sigmoid(z - 1.5)).float()
bd = gbdt.bin_dataset(X, device=dev)
p = gbdt.GBDTParams.from_kwargs(**dict(gbdt.XGB_DEFAULTS, scale_pos_weight=6.0))
for width in (106, 21):
    sub = bd if width == F else gbdt.subset_features(bd, np.arange(width) * (F // width))
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = gbdt.FitReport()
        gbdt.train_binned(sub, y, p, report=r)
        torch.cuda.synchronize()
        print(f"width {width} fit {(time.perf_counter() - t0) * 1e3:.1f} ms  boost {r.t_boost * 1e3:.1f} ms", flush=True)
