"""Batch-scoring automation (reference: src/api/automation_test.py).

The reference script carves a 10-row, label-free sample of the 20 model columns out of the tree
dataset (``train_test_split(test_size=10, random_state=42)``) into
``data/data-input-automation/test_sample.csv``, then waits for an external job to write
``data/3-outputs/latest_output.csv`` and asks for a manual comparison. Here both halves exist:
``make_sample`` writes the input and returns the held-back labels, and ``score_file`` is the
automated job (engine-scored probabilities appended as ``prob_default``).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pandas as pd

from ..config import DEPLOYED_FEATURES


def make_sample(df_tree: pd.DataFrame, out_csv: str | Path, n: int = 10, random_state: int = 42,
                columns: list[str] | None = None) -> pd.Series:
    from ..select.split import train_test_split_indices

    cols = columns or list(DEPLOYED_FEATURES)
    _, te = train_test_split_indices(len(df_tree), test_size=n, random_state=random_state)
    X = df_tree[cols].iloc[te]
    p = Path(out_csv)
    p.parent.mkdir(parents=True, exist_ok=True)
    X.to_csv(p, index=False)
    return df_tree["loan_default"].iloc[te].reset_index(drop=True)


def score_file(booster, in_csv: str | Path, out_csv: str | Path, device=None) -> pd.DataFrame:
    df = pd.read_csv(in_csv)
    names = booster.feature_names or list(df.columns)
    X = df[names].to_numpy(dtype=np.float32, na_value=np.nan)
    prob = booster.predict_proba(X, device=device)
    prob = prob.cpu().numpy() if hasattr(prob, "cpu") else np.asarray(prob)
    out = df.assign(prob_default=prob.astype(np.float64))
    p = Path(out_csv)
    p.parent.mkdir(parents=True, exist_ok=True)
    out.to_csv(p, index=False)
    return out
