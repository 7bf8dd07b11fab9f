"""NN challenger pipeline (reference: notebooks/04_model_training.ipynb cells 31-44).

Steps in the notebook's order: read the NN dataset -> drop the leakage columns plus
``last_pymnt_d_days_NA`` -> MinMaxScaler on all features -> 80/20 split (``random_state=22``) ->
GBDT with XGBoost defaults (``random_state=42``) on the scaled split -> top-20 features by gain
importance -> re-split the UNSCALED top-20 frame -> SMOTE(random_state=123) + MinMaxScaler fit on the
resampled rows -> ``build_and_train_nn`` -> report / AUC / confusion matrix -> save the model
(safetensors), the scaler (JSON) and ``selected_features_nn.txt``.

``reproduce_reference=True`` (default) keeps the notebook's behaviour of training on the unscaled,
non-resampled ``X_train`` and scoring the AUC on thresholded predictions; both
the thresholded and the probability AUC are reported. ``reproduce_reference=False`` trains on the
SMOTE-resampled, scaled rows the notebook prepared.
"""
from __future__ import annotations

import json
import logging
import time
from dataclasses import asdict, dataclass
from pathlib import Path

import numpy as np
import pandas as pd

from ..config import LEAKAGE_COLUMNS
from ..dataio.artifacts import ArtifactStore
from ..metrics import classification as cls_metrics
from ..metrics.auc import roc_auc
from ..models import gbdt
from ..nn.mlp import MLPConfig, fit_many
from ..nn.smote import SMOTE, MinMaxScaler
from ..select.split import train_test_split_indices

log = logging.getLogger(__name__)

NN_OUTPUT_PATH = "models/nn/"
FEATURES_COMMENT = ("# Features selected using XGBoost (Some of these features are in Log scale. Refer to notebook 03 "
                    "for more details.) used for training the Neural Network model.")


@dataclass
class NNTrainConfig:
    test_size: float = 0.2
    split_random_state: int = 22
    importance_random_state: int = 42
    n_features: int = 20
    smote_random_state: int = 123
    reproduce_reference: bool = True
    output_path: str = NN_OUTPUT_PATH
    seed: int = 0
    mlp: MLPConfig | None = None


def run_nn_training(df_nn: pd.DataFrame, cfg: NNTrainConfig | None = None, store: ArtifactStore | None = None,
                    local_dir: str | Path = "models", device=None, gbdt_params: dict | None = None) -> dict:
    cfg = cfg or NNTrainConfig()
    mcfg = cfg.mlp or MLPConfig(seed=cfg.seed)
    t0 = time.perf_counter()
    df = df_nn.drop(columns=LEAKAGE_COLUMNS + ["last_pymnt_d_days_NA"], errors="ignore")
    df = df.loc[df["loan_default"].notna()]
    X = df.drop(columns=["loan_default"]).astype(np.float64)
    y = df["loan_default"].to_numpy(dtype=np.float32)
    Xs = pd.DataFrame(MinMaxScaler().fit_transform(X), columns=X.columns)
    tr, te = train_test_split_indices(len(df), cfg.test_size, cfg.split_random_state)
    params = dict(gbdt.XGB_DEFAULTS, random_state=cfg.importance_random_state, **(gbdt_params or {}))
    imp_model = gbdt.train(Xs.iloc[tr].to_numpy(np.float32), y[tr], params, device=device,
                           feature_names=list(X.columns))
    imp = imp_model.feature_importances("gain")
    order = np.argsort(-imp, kind="stable")
    top = [X.columns[i] for i in order[: cfg.n_features]]
    log.info("Selected top %d features: %s", cfg.n_features, top)

    Xr = X[top]
    Xtr, Xte, ytr, yte = Xr.iloc[tr], Xr.iloc[te], y[tr], y[te]
    Xsm, ysm = SMOTE(random_state=cfg.smote_random_state, device=device).fit_resample(Xtr, ytr)
    scaler = MinMaxScaler().fit(Xsm)
    if cfg.reproduce_reference:
        fit_X, fit_y, val_X = Xtr.to_numpy(np.float32), ytr, Xte.to_numpy(np.float32)
    else:
        fit_X, fit_y = scaler.transform(Xsm).astype(np.float32), np.asarray(ysm, dtype=np.float32)
        val_X = scaler.transform(Xte).astype(np.float32)
    tt = time.perf_counter()
    models, hists = fit_many(fit_X, fit_y, val_X, yte, mcfg, seeds=(mcfg.seed,), device=device, feature_names=top)
    t_train = time.perf_counter() - tt
    model, history = models[0], hists[0]

    proba = model.predict_proba(val_X, device=device)
    pred = (proba > 0.5).astype(np.int64)
    yi = yte.astype(np.int64)
    report = cls_metrics.classification_report(yi, pred, output_dict=True)
    log.info("Classification Report:\n%s", cls_metrics.classification_report(yi, pred))
    auc_thresholded = roc_auc(yte, pred.astype(np.float32))
    auc_proba = roc_auc(yte, proba)
    log.info("ROC AUC (thresholded, as the notebook): %.4f; on probabilities: %.4f", auc_thresholded, auc_proba)
    cm = cls_metrics.confusion_matrix(yi, pred)

    local = Path(local_dir)
    local.mkdir(parents=True, exist_ok=True)
    model.save(local / "nn_model.safetensors")
    (local / "scaler_nn.json").write_text(scaler.to_json())
    feats_txt = "".join(f"{f}\n" for f in top) + "\n" + FEATURES_COMMENT
    (local / "selected_features_nn.txt").write_text(feats_txt)
    metrics = {"auc_thresholded": float(auc_thresholded), "auc": float(auc_proba), "classification_report": report,
               "confusion_matrix": cm.tolist(), "history": history, "selected_features": top,
               "train_rows": int(len(fit_y)), "smote_rows": int(len(ysm)), "train_seconds": t_train,
               "total_seconds": time.perf_counter() - t0,
               "config": {k: v for k, v in asdict(cfg).items() if k != "mlp"} | {"mlp": asdict(mcfg)}}
    (local / "metrics_nn.json").write_text(json.dumps(metrics, indent=2, default=float))
    if store is not None:
        out = cfg.output_path
        for name in ("nn_model.safetensors", "scaler_nn.json", "selected_features_nn.txt", "metrics_nn.json"):
            store.upload_file(local / name, out + name)
    return metrics
