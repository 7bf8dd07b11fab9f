"""Streamlit-independent pieces of the UI client (reference: src/streamlit_ui/cobalt_streamlit.py).

* ``single_payload`` -- the /predict JSON body the single-borrower form builds (:49-84): numeric
  fields, dummy checkboxes as 0/1, the hardship select expanded into four one-hot keys, and the two
  underscore keys renamed to the model's space-containing names.
* ``ApiClient``      -- thin ``requests`` wrapper for /predict, /predict_bulk_csv and
  /feature_importance_bulk (:87, :143, :162).
* ``waterfall_figure`` -- the SHAP waterfall chart (the reference calls ``shap.plots.waterfall``,
  max_display=10 :104-111; ``shap`` is not a dependency here, so the chart is drawn directly with
  matplotlib from the API's ``shap_values``/``base_value``).
* ``importance_figure`` -- the bulk "Top 10 Important Features" bar chart (:164-172).
"""
from __future__ import annotations

import os
from typing import Any

import numpy as np

API_URL = os.environ.get("API_URL", "http://cobalt-lender-api:8000")

NUMERIC_COLS = ["loan_amnt", "term", "installment", "fico_range_low", "last_fico_range_high", "open_il_12m",
                "open_il_24m", "max_bal_bc", "num_rev_accts", "pub_rec_bankruptcies", "emp_length_num",
                "earliest_cr_line_days"]
DUMMY_COLS = ["grade_E", "home_ownership_MORTGAGE", "verification_status_Verified", "application_type_Joint_App",
              "hardship_status_BROKEN", "hardship_status_COMPLETE", "hardship_status_COMPLETED",
              "hardship_status_No_Hardship"]
ALL_COLS = NUMERIC_COLS + DUMMY_COLS
HARDSHIP_CHOICES = ["ACTIVE", "BROKEN", "COMPLETE", "COMPLETED", "No_Hardship"]
FORM_DEFAULTS = {"loan_amnt": 10000.0, "term": 36, "installment": 300.0, "fico_range_low": 660.0,
                 "last_fico_range_high": 700.0, "open_il_12m": 1.0, "open_il_24m": 2.0, "max_bal_bc": 2000.0,
                 "num_rev_accts": 10.0, "pub_rec_bankruptcies": 0.0, "emp_length_num": 3.0,
                 "earliest_cr_line_days": 4000.0}
_RENAMES = {"application_type_Joint_App": "application_type_Joint App",
            "hardship_status_No_Hardship": "hardship_status_No Hardship"}


def single_payload(numeric: dict[str, float], grade_e: bool = False, mortgage: bool = False,
                   verified: bool = False, joint: bool = False, hardship: str = "ACTIVE") -> dict[str, Any]:
    if hardship not in HARDSHIP_CHOICES:
        raise ValueError(f"hardship must be one of {HARDSHIP_CHOICES}")
    d: dict[str, Any] = {k: numeric.get(k, FORM_DEFAULTS[k]) for k in NUMERIC_COLS}
    d["grade_E"] = int(grade_e)
    d["home_ownership_MORTGAGE"] = int(mortgage)
    d["verification_status_Verified"] = int(verified)
    d["application_type_Joint_App"] = int(joint)
    for s in HARDSHIP_CHOICES[1:]:
        d[f"hardship_status_{s}"] = 1 if hardship == s else 0
    for old, new in _RENAMES.items():
        d[new] = d.pop(old)
    return d


class ApiClient:
    def __init__(self, base_url: str | None = None, session=None, timeout: float = 60.0):
        import requests

        self.base = (base_url or API_URL).rstrip("/")
        self.http = session or requests.Session()
        self.timeout = timeout

    def predict(self, payload: dict) -> dict:
        r = self.http.post(f"{self.base}/predict", json=payload, timeout=self.timeout)
        r.raise_for_status()
        return r.json()

    def predict_bulk_csv(self, name: str, data: bytes) -> list[dict]:
        r = self.http.post(f"{self.base}/predict_bulk_csv", files={"file": (name, data, "text/csv")},
                           timeout=self.timeout)
        r.raise_for_status()
        return r.json()["predictions"]

    def feature_importance_bulk(self, rows: list[dict]) -> list[dict]:
        r = self.http.post(f"{self.base}/feature_importance_bulk", json={"data": rows}, timeout=self.timeout)
        r.raise_for_status()
        return r.json()["top_features"]


def waterfall_figure(shap_values, base_value: float, data, feature_names: list[str], max_display: int = 10):
    """SHAP waterfall: bars accumulate from E[f(x)] to f(x); the smallest |phi| beyond
    ``max_display - 1`` features are folded into one "other features" bar."""
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    phi = np.asarray(shap_values, dtype=np.float64).reshape(-1)
    x = np.asarray(data, dtype=np.float64).reshape(-1)
    order = np.argsort(-np.abs(phi), kind="stable")
    keep = order[: max_display - 1] if len(order) > max_display else order
    rest = np.setdiff1d(order, keep)
    labels = [f"{x[i]:.4g} = {feature_names[i]}" for i in keep]
    vals = list(phi[keep])
    if len(rest):
        labels.append(f"{len(rest)} other features")
        vals.append(float(phi[rest].sum()))
    # draw from the bottom (smallest) up, as the shap plot does
    labels, vals = labels[::-1], vals[::-1]
    fx = base_value + phi.sum()
    lefts = []
    acc = base_value
    for v in vals:  # cumulative from the bottom bar upward
        lefts.append(acc)
        acc += v
    fig, ax = plt.subplots(figsize=(10, 6))
    ys = np.arange(len(vals))
    colors = ["#ff0051" if v > 0 else "#008bfb" for v in vals]
    ax.barh(ys, vals, left=lefts, color=colors)
    for y, l, v in zip(ys, lefts, vals):
        ax.text(l + v, y, f"{v:+.2f}", va="center", ha="left" if v > 0 else "right", fontsize=8)
    ax.set_yticks(ys, labels)
    ax.axvline(base_value, color="grey", lw=0.8, ls="--")
    ax.axvline(fx, color="black", lw=0.8)
    ax.set_xlabel(f"E[f(X)] = {base_value:.3f}    f(x) = {fx:.3f}")
    fig.tight_layout()
    return fig


def importance_figure(top_features: list[dict]):
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    feats = [d["feature"] for d in top_features]
    imps = [d["importance"] for d in top_features]
    fig, ax = plt.subplots()
    ax.barh(feats[::-1], imps[::-1])
    ax.set_xlabel("Importance (gain)")
    ax.set_title("Top 10 Important Features")
    fig.tight_layout()
    return fig
