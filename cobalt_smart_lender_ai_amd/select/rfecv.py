"""RFECV (notebook N4): recursive elimination with cross-validated choice of the feature count.

Reference: ``RFECV(XGBClassifier(scale_pos_weight, eval_metric='logloss'), step=5,
cv=StratifiedKFold(3), scoring='roc_auc', min_features_to_select=20, n_jobs=-1)``
(notebooks/04_model_training.ipynb cell 13; the notebook run was interrupted).

scikit-learn 1.7 semantics: on every fold an RFE down to ``min_features_to_select`` scores each
subset of its elimination path on the held-out rows; fold scores are summed per path position and
the SMALLEST feature count among the best sums is chosen; a final RFE on all rows selects that many.
Each fold is sketched/binned once (masked fits on the same device-resident bins).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ..metrics.auc import roc_auc
from ..models import gbdt
from ..models.booster import Booster
from .rfe import rfe
from .split import stratified_kfold_indices


@dataclass
class RFECVResult:
    support_: np.ndarray
    ranking_: np.ndarray
    n_features_: int
    estimator_: Booster
    cv_results_: dict = field(default_factory=dict)

    def selected(self, names: list[str]) -> list[str]:
        return [n for n, s in zip(names, self.support_) if s]


def rfecv(X, y, params: gbdt.GBDTParams | dict, step: int = 5, cv: int = 3, min_features_to_select: int = 1,
          device=None, feature_names: list[str] | None = None) -> RFECVResult:
    if isinstance(params, dict):
        params = gbdt.GBDTParams.from_kwargs(**params)
    X = np.asarray(X, dtype=np.float32)
    y = np.asarray(y, dtype=np.float32)
    F = X.shape[1]
    k_min = min(min_features_to_select, F)
    folds = stratified_kfold_indices(y, cv)
    scores, n_feats = [], None
    for tr, va in folds:
        path_scores, path_n = [], []

        def score(bst, support, va=va):
            p = bst.predict_proba(X[va], device=device)
            path_scores.append(roc_auc(y[va], np.asarray(p.cpu().numpy() if hasattr(p, "cpu") else p)))
            path_n.append(int(support.sum()))

        rfe(X[tr], y[tr], params, n_features_to_select=k_min, step=step, device=device,
            feature_names=feature_names, step_score=score)
        scores.append(path_scores)
        n_feats = path_n
    scores = np.asarray(scores)
    n_rev = np.asarray(n_feats)[::-1]
    best_n = int(n_rev[np.argmax(scores.sum(0)[::-1])])
    final = rfe(X, y, params, n_features_to_select=best_n, step=step, device=device, feature_names=feature_names)
    rev = scores[:, ::-1]
    res = {"mean_test_score": rev.mean(0), "std_test_score": rev.std(0), "n_features": n_rev}
    for i in range(rev.shape[0]):
        res[f"split{i}_test_score"] = rev[i]
    return RFECVResult(final.support_, final.ranking_, final.n_features_, final.estimator_, res)
