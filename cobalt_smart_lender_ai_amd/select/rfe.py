"""Recursive feature elimination (K27) on the GPU GBDT.

Reference: ``RFE(XGBClassifier(eval_metric='logloss', scale_pos_weight=spw, random_state=42),
n_features_to_select=20, step=1)`` (src/model_train_test/model_tree_train_test.py:111-125) -- ~87
sequential XGBoost fits, each re-sketching and re-binning its column subset.

Here the matrix is sketched and binned ONCE (cut points are per feature, so a subset's cuts equal
the full matrix's); every elimination step is a masked fit on the same device-resident bins
(``train_binned(feature_mask=...)``), eliminating the ``step`` lowest-importance features
(``np.argsort`` of the gain importances, as sklearn's RFE does) until ``n_features_to_select``
remain, then refitting on the survivors.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field

import numpy as np

from ..models import gbdt
from ..models.booster import Booster

log = logging.getLogger(__name__)


@dataclass
class RFEResult:
    support_: np.ndarray
    ranking_: np.ndarray
    n_features_: int
    estimator_: Booster
    history: list[dict] = field(default_factory=list)

    def selected(self, names: list[str]) -> list[str]:
        return [n for n, s in zip(names, self.support_) if s]


def rfe(X, y, params: gbdt.GBDTParams | dict, n_features_to_select: int = 20, step: int = 1,
        device=None, feature_names: list[str] | None = None, importance_type: str = "gain",
        binned: gbdt.BinnedData | None = None, step_score=None) -> RFEResult:
    """``step_score(booster, support)`` (optional) is called for every fitted subset, from all
    features down to the final one -- the hook RFECV scores the elimination path with."""
    if isinstance(params, dict):
        params = gbdt.GBDTParams.from_kwargs(**params)
    bd = binned if binned is not None else gbdt.bin_dataset(X, max_bin=params.max_bin,
                                                            sketch_rows=params.sketch_rows, device=device)
    F = bd.n_features
    support = np.ones(F, dtype=bool)
    ranking = np.ones(F, dtype=np.int64)
    hist = []
    step = max(1, int(step))
    while support.sum() > n_features_to_select:
        feats = np.nonzero(support)[0]
        t0 = time.perf_counter()
        bst = gbdt.train_binned(bd, y, params, feature_mask=support, feature_names=feature_names)
        if step_score is not None:
            step_score(bst, support.copy())
        imp_full = bst.feature_importances(importance_type)
        imp = imp_full[feats]
        ranks = np.argsort(imp)
        thr = min(step, int(support.sum()) - n_features_to_select)
        drop = feats[ranks][:thr]
        support[drop] = False
        ranking[~support] += 1
        hist.append({"n_features": int(len(feats)), "dropped": drop.tolist(), "fit_s": time.perf_counter() - t0})
        log.debug("RFE: %d features, dropped %s", len(feats), drop.tolist())
    est = gbdt.train_binned(bd, y, params, feature_mask=support, feature_names=feature_names)
    if step_score is not None:
        step_score(est, support.copy())
    return RFEResult(support, ranking, int(support.sum()), est, hist)
