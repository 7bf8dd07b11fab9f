#!/usr/bin/env python
"""Every configuration BASELINE.json lists, one command each; prints one JSON line per config and
(with ``--save``) writes it to ``profiles/configs/<name>.json``.

  plumbing-10k   "LendingClub 10k-row sample, sklearn LogisticRegression on CPU (plumbing, no GPU)":
                 synthetic raw LendingClub rows -> the reference's cleaning + feature engineering
                 (prep/) -> leakage drop -> 80/20 split -> sklearn LogisticRegression on CPU (the
                 plumbing check the config names), with this framework's GBDT on the same rows for
                 comparison.
  gbdt-1m        "1M-row synthetic LendingClub-shaped GBDT on 1 MI355X"       (bench.py --rows 1000000)
  gbdt-10m       "10M-row GBDT data-parallel ..." (1 GPU here; the driver runs N = 1..8 with torchrun)
  ooc-100m       "100M-row out-of-core GBDT with host-DRAM spill"             (scripts/bench_external.py)
  score-1b       "Batch inference: 1B-row scoring via hipGraph on 8xMI355X" -- one 125M-row shard per
                 GPU (serve/batch_score.py; ranks are independent, so 8 GPUs = 8 x the shard rate)
  cpu-hist-gbdt-10m  CPU reference point for the headline metric (scikit-learn's OpenMP histogram
                 GBDT on the same 10M rows; the reference publishes no throughput)
  prep-full      the reference's full-data preprocessing (clean_data.py full + feature_engineering.py) on a
                 2.9M-row x 143-column synthetic raw export: pandas path vs the device-resident path
                 (scripts/bench_prep.py)
  pipeline-100k  the reference's training job (RFE 106 -> 20 + 20 x 3-fold search + refit) end to end
                 on a 100k-row synthetic sample (scripts/bench_pipeline.py), device-resident hand-off
  pipeline-full  the same job at the reference's production scale: 2.9M raw rows -> ~2.3M training
                 rows, device-resident from the GPU CSV reader to the artifacts (+ the pandas hand-off)
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def plumbing_10k(rows: int = 10_000, trees: int = 300) -> dict:
    import numpy as np
    from sklearn.linear_model import LogisticRegression
    from sklearn.preprocessing import StandardScaler

    from cobalt_smart_lender_ai_amd.config import LEAKAGE_COLUMNS
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc
    from cobalt_smart_lender_ai_amd.models import gbdt
    from cobalt_smart_lender_ai_amd.prep.clean import clean_data_flow
    from cobalt_smart_lender_ai_amd.prep.features import clean_lending_data, feature_engineer_lending_data
    from cobalt_smart_lender_ai_amd.select.split import train_test_split_indices

    t0 = time.perf_counter()
    raw = make_raw_lendingclub(rows, seed=0)
    df = clean_data_flow(raw, device="cpu")
    df = clean_lending_data(df, reference_date="2025-07-04", device="cpu")
    tree, _ = feature_engineer_lending_data(df, device="cpu")
    tree = tree.dropna(subset=["loan_default"])
    tree = tree.drop(columns=[c for c in LEAKAGE_COLUMNS if c in tree.columns])
    y = tree["loan_default"].to_numpy(np.float32)
    X = tree.drop(columns=["loan_default"]).apply(lambda s: s.astype(np.float32)).to_numpy(np.float32)
    t_prep = time.perf_counter() - t0
    tr, te = train_test_split_indices(len(X), test_size=0.2, random_state=22)
    med = np.nanmedian(X[tr], axis=0)
    Xf = np.where(np.isnan(X), med, X)
    sc = StandardScaler().fit(Xf[tr])
    t0 = time.perf_counter()
    lr = LogisticRegression(max_iter=2000).fit(sc.transform(Xf[tr]), y[tr])
    t_lr = time.perf_counter() - t0
    auc_lr = roc_auc(y[te], lr.predict_proba(sc.transform(Xf[te]))[:, 1])
    spw = float((y[tr] == 0).sum() / max((y[tr] == 1).sum(), 1))
    t0 = time.perf_counter()
    b = gbdt.train(X[tr], y[tr], dict(n_estimators=trees, max_depth=7, learning_rate=0.05, gamma=5.0,
                                      scale_pos_weight=spw), device="cpu")
    t_gb = time.perf_counter() - t0
    auc_gb = roc_auc(y[te], b.predict_proba(X[te], device="cpu"))
    return {"config": "plumbing-10k", "metric": "AUC + wall time, CPU plumbing", "raw_rows": rows,
            "rows_after_prep": int(len(X)), "features": int(X.shape[1]), "prep_s": round(t_prep, 3),
            "logreg_fit_s": round(t_lr, 3), "logreg_auc": round(float(auc_lr), 5),
            "gbdt_cpu_fit_s": round(t_gb, 3), "gbdt_cpu_auc": round(float(auc_gb), 5),
            "data": "synthetic raw LendingClub-shaped rows (dataio/synth_raw.py), reference-date 2025-07-04"}


def cpu_hist_gbdt(rows: int = 10_000_000) -> dict:
    """CPU reference point for the headline metric: scikit-learn's HistGradientBoostingClassifier
    (OpenMP C++ histogram GBDT, the closest installed stand-in for the reference's XGBoost CPU
    `hist` fit; xgboost itself is not installed) on the same synthetic 10M x 20 rows and the deployed
    hyper-parameters (300 trees, depth 7, eta 0.05, lambda 1, 255 bins, class weight = spw)."""
    import os

    from sklearn.ensemble import HistGradientBoostingClassifier

    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc

    X, y = synth.make_lendingclub(rows, seed=0)
    Xte, yte = synth.make_lendingclub(1_000_000, seed=0, row_offset=rows)
    X, y, Xte, yte = X.numpy(), y.numpy(), Xte.numpy(), yte.numpy()
    spw = float((y == 0).sum() / (y == 1).sum())
    clf = HistGradientBoostingClassifier(max_iter=300, max_depth=7, learning_rate=0.05, l2_regularization=1.0,
                                         max_bins=255, min_samples_leaf=1, max_leaf_nodes=None,
                                         early_stopping=False, class_weight={0: 1.0, 1: spw}, random_state=78,
                                         verbose=1)
    t0 = time.perf_counter()
    clf.fit(X, y)
    dt = time.perf_counter() - t0
    auc = roc_auc(yte, clf.predict_proba(Xte)[:, 1])
    return {"config": "cpu-hist-gbdt-10m", "metric": "rows/sec GBDT train, CPU reference point",
            "value": round(rows / dt, 1), "unit": "rows/s", "fit_s": round(dt, 3), "auc": round(float(auc), 5),
            "engine": "sklearn HistGradientBoostingClassifier", "threads": os.environ.get("OMP_NUM_THREADS"),
            "cpus_visible": os.cpu_count(), "rows": rows}


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if not lines:
        raise RuntimeError(out[-2000:])
    return json.loads(lines[-1])


def _named(name: str, res: dict) -> dict:
    """bench.py's own "config" object moves to "bench_config"; "config" names the BASELINE entry."""
    return {"config": name, **{k: v for k, v in res.items() if k != "config"}, "bench_config": res.get("config")}


def _run(cmd: list[str], timeout: int) -> dict:
    p = subprocess.run([sys.executable, *cmd], cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"{cmd} failed ({p.returncode}):\n{p.stderr[-3000:]}")
    return _json_line(p.stdout)


CONFIGS = {
    "plumbing-10k": lambda: plumbing_10k(),
    "cpu-hist-gbdt-10m": lambda: cpu_hist_gbdt(),
    "pipeline-100k": lambda: {"config": "pipeline-100k", **_run(["scripts/bench_pipeline.py"], 1100)},
    "pipeline-full": lambda: _run(["scripts/bench_pipeline.py", "--full", "--also-pandas"], 1100),
    "gbdt-1m": lambda: _named("gbdt-1m", _run(["bench.py", "--rows", "1000000", "--steps", "3"], 600)),
    "gbdt-10m": lambda: _named("gbdt-10m", _run(["bench.py", "--steps", "3"], 600)),
    "ooc-100m": lambda: {"config": "ooc-100m",
                         **_run(["scripts/bench_external.py", "--rows", "100000000", "--compare-in-core"], 1100)},
    "prep-full": lambda: {"config": "prep-full", **_run(["scripts/bench_prep.py"], 1100)},
    "score-1b": lambda: {"config": "score-1b", "note": "one 125M-row shard of the 1B-row job (8 ranks x 125M)",
                         **_run(["-m", "cobalt_smart_lender_ai_amd.serve.batch_score", "--rows-per-gpu",
                                 "125000000"], 600)},
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+", choices=sorted(CONFIGS) + ["all"])
    ap.add_argument("--save", action="store_true", help="write profiles/configs/<name>.json")
    a = ap.parse_args()
    names = sorted(CONFIGS) if "all" in a.configs else a.configs
    for name in names:
        res = CONFIGS[name]()
        line = json.dumps(res)
        print(line, flush=True)
        if a.save:  # gpurun_out/ too: that is the directory a GPU-box run copies back
            for d in (ROOT / "profiles" / "configs", ROOT / "gpurun_out" / "configs"):
                d.mkdir(parents=True, exist_ok=True)
                (d / f"{name}.json").write_text(line + "\n")


if __name__ == "__main__":
    main()
