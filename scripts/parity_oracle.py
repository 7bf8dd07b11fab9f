#!/usr/bin/env python
"""Same-configuration AUC reference of the headline bench (bench.py ``auc_parity_ref``).

Trains the host trainer (models/gbdt_host.py, NumPy -- the executable specification the GPU trainer
matches byte for byte on identical inputs, tests/test_gpu_gbdt.py) with EXACTLY the bench protocol:
synthetic rows [0, rows) of seed ``seed`` for training, the next ``test_rows`` rows for the test AUC,
300 trees, depth 7, eta 0.05, gamma 5, lambda 1, min_child_weight 1, max_bin 256, every row sketched,
random_state 78 and scale_pos_weight computed as bench.py does ((n - pos) / pos in float64).

``--trainer 17`` is the GPU trainer's default 17-bit fixed-point gradients; ``fp64`` the unquantised
float64 trainer (CPU only). One JSON line per run; the recorded results live in
profiles/configs/parity-oracle-*.json and bench.py PARITY_AUC.

usage: parity_oracle.py [--rows 10000000] [--test-rows 1000000] [--trainer 17|fp64] [--seed 0]"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--test-rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=300)
    ap.add_argument("--depth", type=int, default=7)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--trainer", default="17", choices=["17", "25", "fp64"])
    a = ap.parse_args()
    X, y = synth.make_lendingclub(a.rows, seed=a.seed)
    pos = float(y.sum())
    spw = (a.rows - pos) / pos  # bench.py: (n_global - pos) / pos
    fp64 = a.trainer == "fp64"
    p = gbdt.GBDTParams(n_estimators=a.trees, max_depth=a.depth, learning_rate=0.05, gamma=5.0, reg_lambda=1.0,
                        min_child_weight=1.0, max_bin=256, scale_pos_weight=spw, random_state=78, sketch_rows=None,
                        grad_bits=17 if fp64 else int(a.trainer))
    t0 = time.perf_counter()
    b = gbdt.train(X, y, p, device="cpu", exact_fp64=fp64)
    fit_s = time.perf_counter() - t0
    del X, y
    Xt, yt = synth.make_lendingclub(a.test_rows, seed=a.seed, row_offset=a.rows)
    pr = np.clip(np.asarray(b.predict_proba(Xt, device="cpu"), np.float64), 1e-15, 1 - 1e-15)
    yv = yt.numpy().astype(np.float64)
    ll = float(-(yv * np.log(pr) + (1 - yv) * np.log(1 - pr)).mean())
    print(json.dumps({"config": f"parity-oracle-{a.rows}", "trainer": "exact_fp64" if fp64 else f"{a.trainer}-bit",
                      "engine": "cobalt host trainer (models/gbdt_host.py, NumPy)", "rows": a.rows,
                      "test_rows": a.test_rows, "trees": a.trees, "max_depth": a.depth, "seed": a.seed,
                      "scale_pos_weight": spw, "auc": round(float(roc_auc(yv, pr)), 6), "test_logloss": round(ll, 6),
                      "fit_s": round(fit_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
