"""TreeExplainer-style API over the GPU TreeSHAP kernel (reference: ``shap.TreeExplainer`` in
src/api/cobalt_fast_api.py:46,100 and notebooks/04_model_training.ipynb cells 24-26).

``TreeExplainer(model).shap_values(X)`` returns path-dependent (``feature_perturbation=
"tree_path_dependent"``) SHAP values in margin space, ``expected_value`` is the cover-weighted mean
leaf sum (the API's ``base_value``). ``shap`` itself is not a dependency: the summary / bar /
waterfall / force views the notebook draws are produced with matplotlib from the same arrays.
"""
from __future__ import annotations

import numpy as np

from ..models.booster import Booster


def _booster(model) -> Booster:
    if isinstance(model, Booster):
        return model
    if hasattr(model, "get_booster"):
        return model.get_booster()
    raise TypeError("expected a Booster or a fitted GBDTClassifier")


class TreeExplainer:
    def __init__(self, model, device=None):
        self.booster = _booster(model)
        self.device = device
        self.expected_value = float(self.booster.expected_value())
        self.feature_names = list(self.booster.feature_names or [f"f{i}" for i in range(self.booster.num_feature)])

    def shap_values(self, X) -> np.ndarray:
        names = self.booster.feature_names
        if hasattr(X, "columns") and names:
            X = X[names]
        Xn = X.to_numpy(dtype=np.float32, na_value=np.nan) if hasattr(X, "to_numpy") else np.asarray(X, np.float32)
        phi = self.booster.shap_values(Xn, device=self.device)
        return np.asarray(phi.cpu().numpy() if hasattr(phi, "cpu") else phi, dtype=np.float64)

    def __call__(self, X) -> "Explanation":
        vals = self.shap_values(X)
        data = X.to_numpy(dtype=np.float64, na_value=np.nan) if hasattr(X, "to_numpy") else np.asarray(X, np.float64)
        return Explanation(vals, np.full(len(vals), self.expected_value), data, self.feature_names)


class Explanation:
    def __init__(self, values, base_values, data, feature_names):
        self.values = np.asarray(values)
        self.base_values = np.asarray(base_values)
        self.data = np.asarray(data)
        self.feature_names = list(feature_names)

    def __getitem__(self, i) -> "Explanation":
        return Explanation(self.values[i], self.base_values[i], self.data[i], self.feature_names)

    def mean_abs(self) -> np.ndarray:
        return np.abs(self.values).mean(0)


def _plt():
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    return plt


def bar_plot(exp: Explanation, max_display: int = 10):
    """Global importance: mean |SHAP| per feature (shap.plots.bar)."""
    plt = _plt()
    m = exp.mean_abs()
    order = np.argsort(-m, kind="stable")[:max_display][::-1]
    fig, ax = plt.subplots(figsize=(8, 0.4 * len(order) + 1.5))
    ax.barh([exp.feature_names[i] for i in order], m[order], color="#008bfb")
    ax.set_xlabel("mean(|SHAP value|)")
    fig.tight_layout()
    return fig


def summary_plot(exp: Explanation, max_display: int = 20, seed: int = 0):
    """Beeswarm-style summary (shap.summary_plot): one row per feature, points coloured by the
    feature value's within-feature rank."""
    plt = _plt()
    m = exp.mean_abs()
    order = np.argsort(-m, kind="stable")[:max_display][::-1]
    rng = np.random.default_rng(seed)
    fig, ax = plt.subplots(figsize=(9, 0.45 * len(order) + 1.5))
    for row, f in enumerate(order):
        v = exp.values[:, f]
        x = exp.data[:, f]
        ok = ~np.isnan(x)
        col = np.full(len(x), 0.5)
        if ok.any():
            r = np.argsort(np.argsort(x[ok]))
            col[ok] = r / max(len(r) - 1, 1)
        ax.scatter(v, row + rng.uniform(-0.3, 0.3, len(v)), c=col, cmap="coolwarm", s=4, alpha=0.6)
    ax.set_yticks(range(len(order)), [exp.feature_names[i] for i in order])
    ax.axvline(0, color="grey", lw=0.8)
    ax.set_xlabel("SHAP value (impact on model output)")
    fig.tight_layout()
    return fig


def force_data(exp: Explanation, i: int) -> dict:
    """The numbers behind shap's force plot for row ``i`` (base, prediction, sorted contributions)."""
    v = exp.values[i]
    order = np.argsort(-np.abs(v), kind="stable")
    return {"base_value": float(exp.base_values[i]), "output": float(exp.base_values[i] + v.sum()),
            "contributions": [{"feature": exp.feature_names[j], "value": float(exp.data[i, j]),
                               "shap": float(v[j])} for j in order]}
