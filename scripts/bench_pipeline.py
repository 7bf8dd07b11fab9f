#!/usr/bin/env python
"""The reference's training job end to end (src/model_train_test/model_tree_train_test.py main():
leakage drop -> 80/20 split -> RFE to 20 features with step 1 -> RandomizedSearchCV 20 x 3-fold ->
refit -> evaluation -> artifacts), fed device-resident from the GPU preprocessing:

  raw CSV --GPU reader--> DeviceFrame --clean / stage 2 / features--> tree DeviceFrame
          --tree_training_matrix (HBM)--> split, RFE (repacked bins), search folds, eval (device gathers)

Default: the notebook's scale (~100k raw rows). ``--full``: the reference's production job --
2.9M x 143 raw rows (clean_data.py full), ~2.3M training rows; the shipped checkpoint was trained on
that job (root sum_hessian -> ~2.28M rows). The synthetic raw schema yields fewer
model columns than the reference's 106, so the tree set is padded on the device with generated
stand-in columns up to 106 -- the reference's 87 sequential RFE fits plus 61 search fits.
``--also-pandas`` times the pandas hand-off (``to_pandas``, host matrix) of the same job for comparison.
Prints one JSON line with the stage timings."""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402


def log(msg: str) -> None:
    print(f"[bench_pipeline] {msg}", file=sys.stderr, flush=True)


def pad_columns(tree, n_target: int, n_have: int, seed: int = 7):
    """Device-generated stand-ins (lognormal, 10% missing) for LendingClub columns the synthetic raw
    schema does not model, appended until ``n_target`` features enter RFE."""
    import torch

    from cobalt_smart_lender_ai_amd.prep.device_frame import DCol

    pad = max(0, n_target - n_have)
    g = torch.Generator(device=tree.device).manual_seed(seed)
    cols = {}
    for k in range(pad):
        v = torch.exp(torch.randn(tree.n, generator=g, device=tree.device, dtype=torch.float64))
        v[torch.rand(tree.n, generator=g, device=tree.device) < 0.1] = float("nan")
        cols[f"synthetic_extra_{k}"] = DCol("f", v, "float64")
    return (tree.assign(**cols) if cols else tree), pad


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--raw-rows", type=int, default=None)
    ap.add_argument("--full", action="store_true", help="the reference's full-data job (2.9M raw rows)")
    ap.add_argument("--rfe-features", type=int, default=106)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--n-iter", type=int, default=20)
    ap.add_argument("--csv", default=None, help="raw CSV path (written if missing)")
    ap.add_argument("--also-pandas", action="store_true")
    a = ap.parse_args()
    rows = a.raw_rows or (2_900_000 if a.full else 100_000)

    import pyarrow as pa
    import pyarrow.csv as pcsv
    import torch

    from cobalt_smart_lender_ai_amd.config import LEAKAGE_COLUMNS, TrainConfig
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.pipeline.train_tree import run_training
    from cobalt_smart_lender_ai_amd.prep.clean import clean_data_flow
    from cobalt_smart_lender_ai_amd.prep.features import clean_lending_data, feature_engineer_lending_data

    ref_date = "2025-07-04"
    out: dict = {"metric": "reference training job wall time (prep + RFE + RandomizedSearchCV + refit + eval)",
                 "config": "pipeline-full" if a.full else "pipeline-100k", "device": a.device}
    if a.device.startswith("cuda"):  # the CLI's default: raw CSV -> GPU reader -> device-resident stages
        from cobalt_smart_lender_ai_amd.prep.device_prep import run_device_prep

        csv = Path(a.csv or f"/tmp/cobalt_raw_{rows}.csv")
        if not csv.exists():
            t = time.perf_counter()
            raw = make_raw_lendingclub(rows, seed=0, n_cols=143)
            pcsv.write_csv(pa.Table.from_pandas(raw, preserve_index=False), str(csv))
            out["raw_shape"] = list(raw.shape)
            del raw
            log(f"raw CSV {csv} ({csv.stat().st_size / 1e9:.2f} GB) written in {time.perf_counter() - t:.1f} s")
        dev = torch.device(a.device)
        run_device_prep(str(csv), device=dev, reference_date=ref_date)  # warm-up (kernels, allocator)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = run_device_prep(str(csv), device=dev, reference_date=ref_date)
        tree = res["tree"]
        n_feat = len([c for c in tree.columns if c != "loan_default" and c not in LEAKAGE_COLUMNS])
        tree, pad = pad_columns(tree, a.rfe_features, n_feat)
        torch.cuda.synchronize(dev)
        t_prep = time.perf_counter() - t0
        out["prep_stages_s"] = {k: round(v, 3) for k, v in res["timings"].items()}
        del res
    else:
        raw = make_raw_lendingclub(rows, seed=0)
        t0 = time.perf_counter()
        df = clean_data_flow(raw, device=a.device)
        df = clean_lending_data(df, reference_date=ref_date, device=a.device)
        tree, _ = feature_engineer_lending_data(df, device=a.device)
        t_prep = time.perf_counter() - t0
        n_feat = len([c for c in tree.columns if c != "loan_default" and c not in LEAKAGE_COLUMNS])
        pad = max(0, a.rfe_features - n_feat)
        rng = np.random.default_rng(7)
        for k in range(pad):
            v = rng.lognormal(0, 1, len(tree)).astype(np.float32)
            v[rng.random(len(tree)) < 0.1] = np.nan
            tree[f"synthetic_extra_{k}"] = v
    log(f"prep {t_prep:.2f} s, tree {tree.shape}, {n_feat} model features + {pad} stand-ins")
    cfg = TrainConfig(device=a.device)
    cfg.search_n_iter = a.n_iter
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        m = run_training(tree, cfg, local_dir=d, device=a.device)
        t_train = time.perf_counter() - t0
    log(f"training job {t_train:.2f} s: {m['timing_s']}")
    fits = m["rfe_fit_s"]
    out.update({
        "rows": int(tree.shape[0]), "train_rows": int(round(tree.shape[0] * 0.8)),
        "features_into_rfe": n_feat + pad, "padded_features": pad, "rfe_fits": n_feat + pad - 20 + 1,
        "search_fits": a.n_iter * 3 + 1, "hand_off": m["hand_off"],
        "prep_s": round(t_prep, 3), "stages_s": {k: round(v, 3) for k, v in m["timing_s"].items()},
        "rfe_fit_s_first": round(fits[0], 4) if fits else None,
        "rfe_fit_s_last": round(fits[-1], 4) if fits else None,
        "rfe_fit_last_over_first": round(fits[-1] / fits[0], 3) if fits else None,
        "train_total_s": round(t_train, 3), "job_total_s": round(t_prep + t_train, 3),
        "test_auc": round(m["auc"], 5), "best_params": m["best_params"],
        "selected_features": m["selected_features"]})
    if a.also_pandas and a.device.startswith("cuda"):
        with tempfile.TemporaryDirectory() as d:
            t0 = time.perf_counter()
            df = tree.to_pandas()
            t_conv = time.perf_counter() - t0
            mp_ = run_training(df, cfg, local_dir=d, device=a.device)
            t_pd = time.perf_counter() - t0
        out["pandas_hand_off"] = {"to_pandas_s": round(t_conv, 3), "train_total_s": round(t_pd, 3),
                                  "stages_s": {k: round(v, 3) for k, v in mp_["timing_s"].items()},
                                  "same_features": mp_["selected_features"] == m["selected_features"],
                                  "same_best_params": mp_["best_params"] == m["best_params"],
                                  "same_auc": mp_["auc"] == m["auc"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
