#!/usr/bin/env python
"""Gradient-precision ablation (docs/PERF.md "Gradient precision"): test AUC and logloss of the
17-bit fixed-point trainer (default), the 25-bit one (grad_bits=25, int64 histogram cells) and the
unquantised fp64 trainer (exact_fp64, CPU only) on the headline configuration (300 trees, depth 7,
eta 0.05, gamma 5, lambda 1, max_bin 256, spw = neg/pos; every row sketched).

The GPU trainer grows the NumPy oracle's trees byte for byte at both precisions
(tests/test_gpu_gbdt.py), so the CPU fits here are the GPU fits' models; --device cuda runs the
quantised fits on the GPU instead (timings). One JSON line per trainer.

usage: precision_probe.py [--rows 2000000] [--test-rows 500000] [--trees 300] [--device cpu]"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--test-rows", type=int, default=500_000)
    ap.add_argument("--trees", type=int, default=300)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--only", default="17,25,fp64")
    a = ap.parse_args()
    X, y = synth.make_lendingclub(a.rows, seed=11)
    Xte, yte = synth.make_lendingclub(a.test_rows, seed=11, row_offset=a.rows)
    yte_np = yte.numpy().astype(np.float64)
    spw = float((y == 0).sum() / (y == 1).sum())
    base = dict(n_estimators=a.trees, max_depth=7, learning_rate=0.05, gamma=5.0, reg_lambda=1.0, min_child_weight=1.0,
                max_bin=256, scale_pos_weight=spw, random_state=78, sketch_rows=None)
    for which in a.only.split(","):
        fp64 = which == "fp64"
        dev = "cpu" if fp64 else a.device
        p = gbdt.GBDTParams(**base, grad_bits=17 if fp64 else int(which))
        Xd, yd = (X.to(dev), y.to(dev)) if dev != "cpu" else (X, y)
        t0 = time.perf_counter()
        b = gbdt.train(Xd, yd, p, device=dev, exact_fp64=fp64)
        if dev != "cpu":
            torch.cuda.synchronize()
        fit_s = time.perf_counter() - t0
        pr = np.clip(np.asarray(b.predict_proba(Xte, device="cpu"), np.float64), 1e-15, 1 - 1e-15)
        ll = float(-(yte_np * np.log(pr) + (1 - yte_np) * np.log(1 - pr)).mean())
        print(json.dumps({"trainer": "exact_fp64" if fp64 else f"{which}-bit", "device": dev, "rows": a.rows,
                          "trees": a.trees, "test_auc": round(float(roc_auc(yte_np, pr)), 6), "test_logloss": round(ll, 6),
                          "fit_s": round(fit_s, 2)}), flush=True)


if __name__ == "__main__":
    main()
