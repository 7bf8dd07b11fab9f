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

The tree dataset may be a pandas frame (the reference's hand-off: ``pd.read_csv`` of the tree CSV,
``model_tree_train_test.py:77``) or a :class:`~..prep.device_frame.DeviceFrame` straight from the
device preprocessing: then the feature matrix is built in HBM (``tree_training_matrix``), the split,
RFE repacking, search folds and evaluation rows are device gathers, and only labels, split indices and
the small per-fit results touch the host. Both hand-offs train the same models (tested).
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


def _host_inputs(df_tree: pd.DataFrame):
    df = df_tree.drop(columns=LEAKAGE_COLUMNS, errors="ignore")
    n_nan = int(df["loan_default"].isna().sum())
    if n_nan:
        log.info("Dropping %d rows with a missing loan_default label", n_nan)
        df = df.loc[df["loan_default"].notna()]
    X = df.drop(columns=["loan_default"])
    names, types = gbdt._feature_info(X)
    return _matrix(X), df["loan_default"].to_numpy(dtype=np.float32), names, types


def _device_inputs(frame):
    """(X [N, F] float32 device matrix, y host labels, names, XGBoost feature types) of a DeviceFrame,
    typed as the pandas hand-off would be (bool -> "i", integer -> "int", else "float")."""
    import torch

    from ..prep.device_prep import tree_training_matrix

    n0 = frame.n
    X, y, names = tree_training_matrix(frame, drop=LEAKAGE_COLUMNS)
    if X.shape[0] != n0:
        log.info("Dropping %d rows with a missing loan_default label", n0 - X.shape[0])
    types = []
    for c in names:
        col = frame[c]
        if col.dtype == "bool":
            types.append("i")
        elif col.dtype == "int64" and (col.kind == "b" or not bool(torch.isnan(col.data).any())):
            types.append("int")
        else:
            types.append("float")
    return X, y.cpu().numpy().astype(np.float32), names, types


def _rows(X, idx):
    if isinstance(X, np.ndarray):
        return X[idx]
    import torch

    return X.index_select(0, torch.as_tensor(np.asarray(idx, dtype=np.int64), device=X.device))


def _cols(X, idx):
    if isinstance(X, np.ndarray):
        return np.ascontiguousarray(X[:, idx])
    import torch

    return X.index_select(1, torch.as_tensor(np.asarray(idx, dtype=np.int64), device=X.device)).contiguous()


def run_training(df_tree, cfg: TrainConfig | None = None, store: ArtifactStore | None = None,
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


def _run_training(df_tree, cfg: TrainConfig, store: ArtifactStore | None, local_dir, device,
                  rfe_params: dict | None, pool) -> dict:
    from ..prep.device_frame import DeviceFrame

    t0 = time.perf_counter()
    on_device = isinstance(df_tree, DeviceFrame)
    X, y, names, types = _device_inputs(df_tree) if on_device else _host_inputs(df_tree)
    if on_device and device is None:
        device = X.device
    tr, te = train_test_split_indices(len(y), cfg.test_size, cfg.split_random_state)
    Xtr, Xte, ytr, yte = _rows(X, tr), _rows(X, te), y[tr], y[te]
    log.info("Train shape: %s, Test shape: %s", tuple(Xtr.shape), tuple(Xte.shape))
    spw = float((ytr == 0).sum() / max((ytr == 1).sum(), 1))
    log.info("scale_pos_weight=%.4f", spw)
    t_split = time.perf_counter() - t0

    # ---- RFE to exactly n features (XGBoost defaults: 100 trees, depth 6, eta 0.3)
    base_rfe = dict(gbdt.XGB_DEFAULTS, scale_pos_weight=spw, random_state=cfg.rfe_random_state)
    base_rfe.update(rfe_params or {})
    tr_rfe = time.perf_counter()
    r = rfe(Xtr, ytr, base_rfe, n_features_to_select=cfg.rfe_n_features, step=cfg.rfe_step,
            device=device, feature_names=names)
    selected = r.selected(names)
    sel_idx = [names.index(c) for c in selected]
    t_rfe = time.perf_counter() - tr_rfe
    log.info("Selected %d features: %s", len(selected), selected)

    # ---- randomized search on the selected features
    base = dict(gbdt.XGB_DEFAULTS, scale_pos_weight=spw, random_state=cfg.base_random_state)
    ts = time.perf_counter()
    sr = randomized_search(_cols(Xtr, sel_idx), ytr, cfg.search_space, base, n_iter=cfg.search_n_iter,
                           cv=cfg.search_cv_folds, random_state=cfg.search_random_state, device=device,
                           n_gpus=1, pool=pool)
    t_search = time.perf_counter() - ts
    log.info("Best score (AUC): %s", sr.best_score_)
    log.info("Best params: %s", sr.best_params_)
    best = sr.best_estimator_
    best.feature_names = list(selected)
    best.feature_types = [types[i] for i in sel_idx] if types else None

    # ---- evaluation
    te0 = time.perf_counter()
    proba = best.predict_proba(_cols(Xte, sel_idx), device=device)
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
    metrics["timing_s"] = {"inputs_split": t_split, "rfe": t_rfe, "search": t_search,
                           "eval_artifacts": time.perf_counter() - te0, "total": time.perf_counter() - t0}
    metrics["rfe_fit_s"] = [h["fit_s"] for h in r.history]
    metrics["hand_off"] = "device" if on_device else "pandas"
    metrics["selected_features"] = selected
    metrics["config"] = {k: v for k, v in asdict(cfg).items() if k != "search_space"}
    return metrics
