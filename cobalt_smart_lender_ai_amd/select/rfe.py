"""Recursive feature elimination (K27) on the GPU GBDT.

Reference: ``RFE(XGBClassifier(eval_metric='logloss', scale_pos_weight=spw, random_state=42),
n_features_to_select=20, step=1)`` (src/model_train_test/model_tree_train_test.py:111-125) -- ~87
sequential XGBoost fits, each re-sketching and re-binning its column subset.

Here the matrix is sketched and binned ONCE (cut points are per feature, so a subset's cuts equal
the full matrix's). Every elimination step fits on the surviving columns only: the device-resident
bins are repacked to them (``gbdt.subset_features``: a gather of N x F' bytes, far cheaper than a
fit), so a fit's cost falls with the feature count -- 21 features run the 32-byte-record fast path
instead of the 106-feature one -- while its trees equal a ``feature_mask`` fit on the full matrix
(``repack=False``, tested). The ``step`` lowest-importance features (``np.argsort`` of the gain
importances, as sklearn's RFE does) are eliminated until ``n_features_to_select`` remain, then the
survivors are refit. Boosters are returned over the full feature space.
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
        binned: gbdt.BinnedData | None = None, step_score=None, repack: bool = True) -> RFEResult:
    """``step_score(booster, support)`` (optional) is called for every fitted subset, from all
    features down to the final one -- the hook RFECV scores the elimination path with.
    ``repack=False``: masked fits on the full-width matrix (the same trees, at the full width's cost)."""
    if isinstance(params, dict):
        params = gbdt.GBDTParams.from_kwargs(**params)
    bd = binned if binned is not None else gbdt.bin_dataset(X, max_bin=params.max_bin,
                                                            sketch_rows=params.sketch_rows, device=device)
    F = bd.n_features
    support = np.ones(F, dtype=bool)
    ranking = np.ones(F, dtype=np.int64)
    hist = []
    step = max(1, int(step))
    yt = y
    if bd.device.type == "cuda":  # labels go to the device once, not once per fit
        yt = gbdt._to_tensor(y, bd.device).reshape(-1)

    def fit(sup: np.ndarray):
        feats = np.nonzero(sup)[0]
        if not repack or len(feats) == F:
            return gbdt.train_binned(bd, yt, params, feature_mask=sup, feature_names=feature_names)
        sub = gbdt.subset_features(bd, feats)
        names = [feature_names[i] for i in feats] if feature_names is not None else None
        b = gbdt.train_binned(sub, yt, params, feature_names=names)
        return gbdt.expand_features(b, feats, F, feature_names)

    while support.sum() > n_features_to_select:
        feats = np.nonzero(support)[0]
        t0 = time.perf_counter()
        bst = fit(support)
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
    est = fit(support)
    if step_score is not None:
        step_score(est, support.copy())
    return RFEResult(support, ranking, int(support.sum()), est, hist)
