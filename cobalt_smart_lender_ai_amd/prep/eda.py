"""Exploratory helpers from the cleaning notebook.

* ``null_data_summary`` -- notebooks/01_data_cleaning.ipynb cell 28: columns with nulls, sorted by
  count, as ``[Column, Percentage]`` rows above a threshold (null counts on the device, K1).
* ``zscore`` / ``zscore_outlier_counts`` -- cells 39/41: ``scipy.stats.zscore`` (population std,
  ddof=0; NaN propagates as in scipy's default ``nan_policy='propagate'``) and the outlier counts
  ``|z| > t`` for t in 2.0, 2.25, 2.5, 2.75. Moments come from the fused column-moment kernel.
* ``describe`` -- cell 19's ``describe()`` for numeric columns (count/mean/std/min/quartiles/max),
  count/sum/sumsq/min/max on the device, quartiles by device sort.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from ..ops import prep_ops
from . import frame


def null_data_summary(df: pd.DataFrame, threshold_percentage: float = 50, device=None) -> pd.DataFrame:
    dev = frame.resolve_device(device)
    nulls = frame.null_counts(df, dev).sort_values(ascending=False, kind="stable")
    nulls = nulls[nulls > 0].reset_index()
    nulls.columns = ["Column", "Percentage"]
    nulls["Percentage"] = nulls["Percentage"] / len(df) * 100
    return nulls[nulls["Percentage"] > threshold_percentage]


def zscore(values, device=None) -> np.ndarray:
    """``scipy.stats.zscore`` of a 1-D array/Series (ddof=0)."""
    dev = frame.resolve_device(device)
    x = torch.as_tensor(np.asarray(values, dtype=np.float64)).reshape(1, -1).to(dev)
    m = prep_ops.col_moments(x).cpu().numpy()[0]
    cnt, s, s2 = m[0], m[1], m[2]
    a = x.cpu().numpy()[0]
    if cnt < len(a):  # scipy propagates NaN through the moments
        return np.full_like(a, np.nan)
    mean = s / cnt
    var = max(s2 / cnt - mean * mean, 0.0)
    # two-pass correction for the cancellation of sumsq (exact for the moments scipy computes)
    var = float(np.mean((a - mean) ** 2)) if var < 1e-12 * max(mean * mean, 1.0) else var
    return (a - mean) / np.sqrt(var)


def zscore_outlier_counts(values, thresholds=(2.0, 2.25, 2.5, 2.75), device=None) -> dict[float, int]:
    z = np.abs(zscore(values, device))
    return {float(t): int(np.sum(z > t)) for t in thresholds}


def describe(df: pd.DataFrame, device=None) -> pd.DataFrame:
    dev = frame.resolve_device(device)
    num = frame.numeric_columns(df)
    if not num:
        return pd.DataFrame()
    X = frame.to_device(df, num, dev)
    mo = prep_ops.col_moments(X).cpu().numpy()
    cnt, s, s2, mn, mx = mo.T
    mean = np.where(cnt > 0, s / np.maximum(cnt, 1), np.nan)
    var = np.where(cnt > 1, (s2 - cnt * mean * mean) / np.maximum(cnt - 1, 1), np.nan)
    xs = torch.sort(X, dim=1).values.cpu().numpy()
    q = {}
    for name, p in (("25%", 0.25), ("50%", 0.5), ("75%", 0.75)):
        vals = []
        for c in range(len(num)):
            n = int(cnt[c])
            if n == 0:
                vals.append(np.nan)
                continue
            pos = p * (n - 1)  # pandas/numpy linear interpolation
            lo, hi = int(np.floor(pos)), int(np.ceil(pos))
            vals.append(xs[c, lo] + (xs[c, hi] - xs[c, lo]) * (pos - lo))
        q[name] = vals
    out = pd.DataFrame({"count": cnt, "mean": mean, "std": np.sqrt(np.maximum(var, 0)),
                        "min": np.where(cnt > 0, mn, np.nan), **q, "max": np.where(cnt > 0, mx, np.nan)},
                       index=num).T
    return out
