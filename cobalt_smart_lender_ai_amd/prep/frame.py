"""Bridge between pandas frames and the column-major device tensors used by ``ops/prep_ops``.

String parsing stays on the host (pandas/pyarrow); every numeric pass over the frame
(null counts, row filters, log transforms, imputation, dedupe hashing, one-hot) runs on the device
tensor when a GPU is present.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from ..ops import prep_ops


def resolve_device(device: str | torch.device | None) -> torch.device:
    if device is None:
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


def numeric_columns(df: pd.DataFrame) -> list[str]:
    return [c for c in df.columns if pd.api.types.is_numeric_dtype(df[c].dtype) and not pd.api.types.is_bool_dtype(df[c].dtype)]


def to_device(df: pd.DataFrame, cols: list[str], device: torch.device) -> torch.Tensor:
    """Column-major float64 [C, N] tensor of ``df[cols]``."""
    if not cols:
        return torch.zeros((0, len(df)), dtype=torch.float64, device=device)
    a = np.empty((len(cols), len(df)), dtype=np.float64)
    for i, c in enumerate(cols):
        a[i] = df[c].to_numpy(dtype=np.float64, na_value=np.nan)
    return torch.from_numpy(a).to(device)


def null_counts(df: pd.DataFrame, device: torch.device) -> pd.Series:
    """``df.isnull().sum()`` with the numeric columns counted on the device (K1)."""
    num = numeric_columns(df)
    out = {}
    if num:
        cnt = prep_ops.col_null_counts(to_device(df, num, device)).cpu().numpy()
        out.update(dict(zip(num, cnt.tolist())))
    for c in df.columns:
        if c not in out:
            out[c] = int(df[c].isna().sum())
    return pd.Series([out[c] for c in df.columns], index=df.columns, dtype=np.int64)


def row_null_counts(df: pd.DataFrame, subset: list[str] | None, device: torch.device) -> np.ndarray:
    """Per-row NaN count over ``subset`` (all columns when None); numeric part on the device (K2)."""
    cols = list(df.columns) if subset is None else [c for c in df.columns if c in set(subset)]
    num = [c for c in numeric_columns(df) if c in set(cols)]
    total = np.zeros(len(df), dtype=np.int64)
    if num:
        total += prep_ops.row_null_counts(to_device(df, num, device)).cpu().numpy().astype(np.int64)
    other = [c for c in cols if c not in set(num)]
    if other:
        total += df[other].isna().to_numpy().sum(1)
    return total


def duplicated(df: pd.DataFrame, device: torch.device) -> np.ndarray:
    """``df.duplicated(keep='first')``: device row hashing of the numeric block (K9) combined with
    pandas hashing of the other columns, then exact verification of every candidate pair."""
    if len(df) == 0:
        return np.zeros(0, dtype=bool)
    num = numeric_columns(df)
    other = [c for c in df.columns if c not in set(num)]
    X = to_device(df, num, device)
    extra = None
    if other:
        extra = torch.from_numpy(pd.util.hash_pandas_object(df[other].astype(object).where(df[other].notna(), None),
                                                            index=False).to_numpy().view(np.int64).copy())
    dup, (a, b) = prep_ops.duplicated_numeric(X, extra)
    dup = dup.cpu().numpy()
    if other and dup.any():
        a, b = a.cpu().numpy(), b.cpu().numpy()
        left = df[other].iloc[a].reset_index(drop=True)
        right = df[other].iloc[b].reset_index(drop=True)
        same = ((left == right) | (left.isna() & right.isna())).all(1).to_numpy()
        dup[b[~same]] = False
    return dup
