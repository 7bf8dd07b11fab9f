#!/usr/bin/env python
"""The reference's training job end to end (src/model_train_test/model_tree_train_test.py main():
leakage drop -> 80/20 split -> RFE to 20 features with step 1 -> RandomizedSearchCV 20 x 3-fold ->
refit -> evaluation -> artifacts) on a synthetic LendingClub-shaped tree dataset of the notebook's
shape: ~97.5k rows x 106 features entering RFE (the synthetic raw schema yields fewer columns, so it
is padded with generated stand-in columns to 106), i.e. the reference's 87 sequential RFE fits plus
61 search fits. Prints one JSON line with the stage timings."""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--raw-rows", type=int, default=100_000)
    ap.add_argument("--rfe-features", type=int, default=106)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--n-iter", type=int, default=20)
    a = ap.parse_args()

    from cobalt_smart_lender_ai_amd.config import LEAKAGE_COLUMNS, TrainConfig
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.pipeline.train_tree import run_training
    from cobalt_smart_lender_ai_amd.prep.clean import clean_data_flow
    from cobalt_smart_lender_ai_amd.prep.features import clean_lending_data, feature_engineer_lending_data

    raw = make_raw_lendingclub(a.raw_rows, seed=0)
    if a.device.startswith("cuda"):  # the CLI's default: raw CSV -> GPU reader -> device-resident stages
        from cobalt_smart_lender_ai_amd.prep.device_prep import run_device_prep

        data = raw.to_csv(index=False).encode()
        t0 = time.perf_counter()
        tree = run_device_prep(data, device=a.device, reference_date="2025-07-04")["tree"].to_pandas()
    else:
        t0 = time.perf_counter()
        df = clean_data_flow(raw, device=a.device)
        df = clean_lending_data(df, reference_date="2025-07-04", device=a.device)
        tree, _ = feature_engineer_lending_data(df, device=a.device)
    t_prep = time.perf_counter() - t0
    n_feat = len([c for c in tree.columns if c != "loan_default" and c not in LEAKAGE_COLUMNS])
    rng = np.random.default_rng(7)
    pad = max(0, a.rfe_features - n_feat)
    for k in range(pad):  # stand-ins for LendingClub columns the synthetic raw schema does not model
        v = rng.lognormal(0, 1, len(tree)).astype(np.float32)
        v[rng.random(len(tree)) < 0.1] = np.nan
        tree[f"synthetic_extra_{k}"] = v
    cfg = TrainConfig(device=a.device)
    cfg.search_n_iter = a.n_iter
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        m = run_training(tree, cfg, local_dir=d, device=a.device)
        t_train = time.perf_counter() - t0
    print(json.dumps({"metric": "reference training job wall time (RFE + RandomizedSearchCV + refit + eval)",
                      "rows": int(len(tree)), "features_into_rfe": n_feat + pad, "padded_features": pad,
                      "rfe_fits": n_feat + pad - 20 + 1, "search_fits": a.n_iter * 3 + 1,
                      "prep_s": round(t_prep, 2), "rfe_s": round(m["timing_s"]["rfe"], 2),
                      "search_s": round(m["timing_s"]["search"], 2), "train_total_s": round(t_train, 2),
                      "test_auc": round(m["auc"], 5), "best_params": m["best_params"], "device": a.device}),
          flush=True)


if __name__ == "__main__":
    main()
