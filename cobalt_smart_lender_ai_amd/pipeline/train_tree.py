"""End-to-end tree-model training pipeline (reference: src/model_train_test/model_tree_train_test.py
``main()``).

Steps, in the reference order: drop the 14 leakage columns -> 80/20 split (``random_state=22``,
not stratified) -> ``scale_pos_weight = neg/pos`` on the training labels -> RFE to 20 features ->
randomized search (20 candidates x stratified 3-fold ROC-AUC) -> test evaluation (report, AUC,
confusion matrix) -> figures -> ``xgb_model_tree.pkl`` (XGBoost-compatible pickle) +
``selected_features_tree.txt`` + ``metrics.json`` in the artifact store (``models/xgboost/``) and
the local ``models/`` directory.

Deliberate, documented difference: rows whose ``loan_default`` is missing (loan statuses outside the
reference's map, e.g. "Does not meet the credit policy...") are dropped before the split, since a
NaN label has no defined gradient (XGBoost rejects such labels).
"""
from __future__ import annotations

import json
import logging
import time
from dataclasses import asdict
from pathlib import Path

import numpy as np
import pandas as pd

from ..config import (BEST_MODEL_FILENAME, FEATURES_FILENAME, LEAKAGE_COLUMNS, METRICS_JSON, TrainConfig)
from ..dataio.artifacts import ArtifactStore
from ..metrics import classification as cls_metrics
from ..metrics.auc import roc_auc
from ..models import gbdt
from ..models.booster import dump_pickle_bytes
from ..select.rfe import rfe
from ..select.search import randomized_search
from ..select.split import train_test_split_indices
from ..utils import plots

log = logging.getLogger(__name__)


def _matrix(df: pd.DataFrame) -> np.ndarray:
    return df.to_numpy(dtype=np.float32, na_value=np.nan)


def run_training(df_tree: pd.DataFrame, cfg: TrainConfig | None = None, store: ArtifactStore | None = None,
                 local_dir: str | Path = "models", device=None, rfe_params: dict | None = None,
                 pool=None) -> dict:
    """``pool``: a :class:`~..parallel.taskpool.GpuTaskPool` for the search's task-parallel fits.
    Without one, ``cfg.fits_in_parallel`` > 1 (None = all visible GPUs) creates a pool here -- before
    this function's own GPU work, so the workers are spawned from a process without HIP state. Only
    for GPU work and only if this process has not initialised HIP yet (``can_auto_pool``; ``cli
    train`` guarantees it); otherwise the fits run in this process."""
    from ..parallel.taskpool import GpuTaskPool, can_auto_pool, resolve_workers

    cfg = cfg or TrainConfig()
    own_pool = None
    if pool is None and resolve_workers(cfg.fits_in_parallel) > 1 and can_auto_pool(device):
        pool = own_pool = GpuTaskPool(resolve_workers(cfg.fits_in_parallel))
    try:
        return _run_training(df_tree, cfg, store, local_dir, device, rfe_params, pool)
    finally:
        if own_pool is not None:
            own_pool.close()


def _run_training(df_tree: pd.DataFrame, cfg: TrainConfig, store: ArtifactStore | None, local_dir, device,
                  rfe_params: dict | None, pool) -> dict:
    t0 = time.perf_counter()
    df = df_tree.drop(columns=LEAKAGE_COLUMNS, errors="ignore")
    n_nan = int(df["loan_default"].isna().sum())
    if n_nan:
        log.info("Dropping %d rows with a missing loan_default label", n_nan)
        df = df.loc[df["loan_default"].notna()]
    X = df.drop(columns=["loan_default"])
    y = df["loan_default"].to_numpy(dtype=np.float32)
    tr, te = train_test_split_indices(len(df), cfg.test_size, cfg.split_random_state)
    Xtr, Xte, ytr, yte = X.iloc[tr], X.iloc[te], y[tr], y[te]
    log.info("Train shape: %s, Test shape: %s", Xtr.shape, Xte.shape)
    spw = float((ytr == 0).sum() / max((ytr == 1).sum(), 1))
    log.info("scale_pos_weight=%.4f", spw)

    names, types = gbdt._feature_info(Xtr)
    # ---- RFE to exactly n features (XGBoost defaults: 100 trees, depth 6, eta 0.3)
    base_rfe = dict(gbdt.XGB_DEFAULTS, scale_pos_weight=spw, random_state=cfg.rfe_random_state)
    base_rfe.update(rfe_params or {})
    tr_rfe = time.perf_counter()
    r = rfe(_matrix(Xtr), ytr, base_rfe, n_features_to_select=cfg.rfe_n_features, step=cfg.rfe_step,
            device=device, feature_names=names)
    selected = r.selected(names)
    t_rfe = time.perf_counter() - tr_rfe
    log.info("Selected %d features: %s", len(selected), selected)

    # ---- randomized search on the selected features
    base = dict(gbdt.XGB_DEFAULTS, scale_pos_weight=spw, random_state=cfg.base_random_state)
    ts = time.perf_counter()
    sr = randomized_search(_matrix(Xtr[selected]), ytr, cfg.search_space, base, n_iter=cfg.search_n_iter,
                           cv=cfg.search_cv_folds, random_state=cfg.search_random_state, device=device,
                           n_gpus=1, pool=pool)
    t_search = time.perf_counter() - ts
    log.info("Best score (AUC): %s", sr.best_score_)
    log.info("Best params: %s", sr.best_params_)
    best = sr.best_estimator_
    best.feature_names = list(selected)
    best.feature_types = [types[names.index(c)] for c in selected] if types else None

    # ---- evaluation
    proba = best.predict_proba(_matrix(Xte[selected]), device=device)
    proba = np.asarray(proba.cpu().numpy() if hasattr(proba, "cpu") else proba)
    pred = (proba > 0.5).astype(np.int64)
    report = cls_metrics.classification_report(yte.astype(np.int64), pred, output_dict=True)
    auc = roc_auc(yte, proba)
    cm = cls_metrics.confusion_matrix(yte.astype(np.int64), pred)
    log.info("Classification Report:\n %s", cls_metrics.classification_report(yte.astype(np.int64), pred))
    log.info("ROC AUC: %.4f", auc)

    # ---- artifacts
    local = Path(local_dir)
    local.mkdir(parents=True, exist_ok=True)
    sk_params = {**{k: v for k, v in base.items() if k in ("scale_pos_weight", "random_state")},
                 **sr.best_params_, "eval_metric": "logloss", "use_label_encoder": False}
    sk_state = {k: v for k, v in sk_params.items() if k != "use_label_encoder"}
    sk_state["kwargs"] = {"use_label_encoder": False}
    pkl = dump_pickle_bytes(best, sk_state)
    (local / BEST_MODEL_FILENAME).write_bytes(pkl)
    feats_txt = "".join(f"{f}\n" for f in selected) + "\n# Features selected via RFE + XGBoost hyperparam search.\n"
    (local / FEATURES_FILENAME).write_text(feats_txt)
    metrics = {"auc": float(auc), "classification_report": report,
               "best_params": {k: (v.item() if hasattr(v, "item") else v) for k, v in sr.best_params_.items()}}
    metrics_txt = json.dumps(metrics, indent=2)
    (local / METRICS_JSON).write_text(metrics_txt)
    fig_cm = plots.confusion_matrix_figure(cm)
    fig_imp = plots.feature_importance_figure(selected, best.feature_importances("gain"))
    fig_cm.savefig(local / "confusion_matrix.png")
    fig_imp.savefig(local / "feature_importance.png")
    if store is not None:
        out = cfg.output_path
        store.put_bytes(out + BEST_MODEL_FILENAME, pkl)
        store.put_bytes(out + FEATURES_FILENAME, feats_txt.encode())
        store.put_bytes(out + METRICS_JSON, metrics_txt.encode())
        store.save_figure(fig_cm, out + "confusion_matrix.png")
        store.save_figure(fig_imp, out + "feature_importance.png")
    plots.close(fig_cm)
    plots.close(fig_imp)
    metrics["timing_s"] = {"rfe": t_rfe, "search": t_search, "total": time.perf_counter() - t0}
    metrics["selected_features"] = selected
    metrics["config"] = {k: v for k, v in asdict(cfg).items() if k != "search_space"}
    return metrics
