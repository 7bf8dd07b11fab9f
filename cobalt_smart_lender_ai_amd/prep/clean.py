"""Stage-1 cleaning of the raw LendingClub export (reference: src/data_preprocessing/clean_data.py
and notebooks/01_data_cleaning.ipynb; behaviour spec in SURVEY.md App. A.1).

Two presets reproduce the two reference variants:

* ``"script"`` (default, CLI parity with ``clean_data.py``): drop the two ``Unnamed`` index columns,
  drop rows with a NaN in any column that has fewer than 10 NaNs, fill ``hardship_status`` with
  "No Hardship", parse ``term`` / ``int_rate``, drop columns > 70% null, drop seven bookkeeping
  columns, zero-fill three counters, drop duplicate rows.
* ``"notebook"``: no small-null row drop; ``mths_since_last_delinq`` := 999 where missing and
  ``acc_now_delinq == 0`` then rows still missing it are dropped; only four columns dropped.

Column null counts, the row filter and the duplicate scan run on the GPU (K1, K2, K9) via
``prep/frame.py``; string parsing is host-side.
"""
from __future__ import annotations

import logging

import pandas as pd

from . import frame

log = logging.getLogger(__name__)

INDEX_COLUMNS = ["Unnamed: 0.1", "Unnamed: 0"]
SCRIPT_UNNECESSARY = ["next_pymnt_d", "last_pymnt_d", "last_credit_pull_d", "mths_since_recent_revol_delinq",
                      "il_util", "all_util", "mths_since_recent_bc_dlq"]
NOTEBOOK_UNNECESSARY = ["next_pymnt_d", "last_pymnt_d", "il_util", "all_util"]
ZERO_FILL = ["inq_last_12m", "open_acc_6m", "chargeoff_within_12_mths"]


def drop_columns_with_missing_values(df: pd.DataFrame, threshold_percentage: float = 70.0,
                                     device=None) -> pd.DataFrame:
    """Drop columns whose null share is strictly above ``threshold_percentage`` percent (C3)."""
    dev = frame.resolve_device(device)
    share = frame.null_counts(df, dev) / max(len(df), 1) * 100.0
    drop = share[share > threshold_percentage].index.tolist()
    log.info("Dropping columns with >%s%% missing: %s", threshold_percentage, drop)
    return df.drop(columns=drop)


def _parse_term(s: pd.Series) -> pd.Series:
    if pd.api.types.is_numeric_dtype(s.dtype):
        return s
    return s.str.replace(" months", "", regex=False).str.strip().astype(int)


def _parse_percent(s: pd.Series) -> pd.Series:
    if pd.api.types.is_numeric_dtype(s.dtype):
        return s
    return s.str.replace("%", "", regex=False).astype(float) / 100


def clean_data_flow(df: pd.DataFrame, preset: str = "script", device=None,
                    null_threshold: float = 70.0) -> pd.DataFrame:
    """Apply the stage-1 cleaning steps in the reference order; returns a new frame."""
    if preset not in ("script", "notebook"):
        raise ValueError(f"unknown preset {preset!r}")
    dev = frame.resolve_device(device)
    out = df.drop(columns=INDEX_COLUMNS, errors="ignore")

    if preset == "script":
        nulls = frame.null_counts(out, dev)
        subset = nulls.index[nulls < 10].tolist()
        bad = frame.row_null_counts(out, subset, dev) > 0
        out = out.loc[~bad]
    if "hardship_status" in out.columns:
        out = out.assign(hardship_status=out["hardship_status"].fillna("No Hardship"))
    if "term" in out.columns:
        out = out.assign(term=_parse_term(out["term"]))
    if "int_rate" in out.columns:
        out = out.assign(int_rate=_parse_percent(out["int_rate"]))
    out = drop_columns_with_missing_values(out, null_threshold, dev)
    if preset == "notebook" and "mths_since_last_delinq" in out.columns:
        # notebooks/01_data_cleaning.ipynb:9926-9934, after the >70% column drop (:9194)
        fill = out["mths_since_last_delinq"].isna()
        if "acc_now_delinq" in out.columns:
            fill &= out["acc_now_delinq"] == 0
        out = out.assign(mths_since_last_delinq=out["mths_since_last_delinq"].mask(fill, 999))
        out = out.loc[out["mths_since_last_delinq"].notna()]
    unnecessary = SCRIPT_UNNECESSARY if preset == "script" else NOTEBOOK_UNNECESSARY
    out = out.drop(columns=[c for c in unnecessary if c in out.columns])
    fills = {c: 0 for c in ZERO_FILL if c in out.columns}
    if fills:
        out = out.fillna(fills)
    before = len(out)
    out = out.loc[~frame.duplicated(out, dev)]
    log.info("Duplicates removed: %d", before - len(out))
    return out
