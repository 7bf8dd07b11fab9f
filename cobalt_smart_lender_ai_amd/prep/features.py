"""Stage-2 cleaning + feature engineering (reference: src/data_preprocessing/feature_engineering.py,
notebooks/03_feature_engineering.ipynb; behaviour spec in SURVEY.md App. A.2).

Produces the two datasets of the reference:

* the **tree** dataset: masked log1p of the skewed columns + ``get_dummies(drop_first=True)`` of six
  categorical columns (NaNs kept for the GBDT's learned default direction);
* the **NN** dataset: same log transform, then ``<col>_NA`` indicators + median imputation for every
  numeric column with nulls (``dti`` handled separately with ``no_income``/``dti_NA``), then label
  encoding of the remaining string columns.

GPU work (when available): masked log1p over all selected columns in one launch (K6, instead of
the reference's per-element Python ``Series.apply``), per-column null counts (K1), exact medians
(K4, device sort), fused fill + indicator (K3/K5), one-hot scatter (K7), row NaN counts for the
``dropna(thresh=...)`` filter (K2). Dictionary encoding (K8) and date/regex parsing stay host-side.
"""
from __future__ import annotations

import logging
from datetime import datetime

import numpy as np
import pandas as pd
import torch

from ..ops import prep_ops
from . import frame

log = logging.getLogger(__name__)

LEAKAGE_STAGE2 = ["recoveries", "collection_recovery_fee", "debt_settlement_flag"]
USELESS_STAGE2 = ["id", "url", "title", "zip_code", "addr_state", "emp_title", "issue_d", "initial_list_status",
                  "hardship_flag", "sub_grade", "next_pymnt_d", "last_credit_pull_d", "pymnt_plan"]
LOAN_STATUS_MAP = {"Fully Paid": 0, "Current": 0, "Issued": 0, "In Grace Period": 0, "Late (16-30 days)": 0,
                   "Late (31-120 days)": 1, "Charged Off": 1, "Default": 1}
LOG_COLUMNS = [
    "loan_amnt", "funded_amnt", "funded_amnt_inv", "int_rate", "installment", "annual_inc", "dti", "fico_range_low",
    "fico_range_high", "mths_since_last_delinq", "open_acc", "total_acc", "total_pymnt", "total_pymnt_inv",
    "total_rec_prncp", "total_rec_int", "total_rec_late_fee", "last_pymnt_amnt", "acc_now_delinq", "tot_coll_amt",
    "tot_cur_bal", "total_rev_hi_lim", "earliest_cr_line_days", "acc_open_past_24mths", "avg_cur_bal",
    "bc_open_to_buy", "mo_sin_old_rev_tl_op", "mo_sin_rcnt_rev_tl_op", "mo_sin_rcnt_tl", "mort_acc",
    "mths_since_recent_bc", "mths_since_recent_inq", "mths_since_recent_revol_delinq", "num_accts_ever_120_pd",
    "num_actv_bc_tl", "num_actv_rev_tl", "num_bc_sats", "num_bc_tl", "num_il_tl", "num_op_rev_tl", "num_rev_accts",
    "num_rev_tl_bal_gt_0", "num_sats", "num_tl_op_past_12m", "pub_rec_bankruptcies", "tot_hi_cred_lim",
    "total_bal_ex_mort", "total_bc_limit", "total_il_high_credit_limit", "revol_util",
]
DUMMY_COLUMNS = ["grade", "home_ownership", "verification_status", "purpose", "application_type", "hardship_status"]


def clean_lending_data(df: pd.DataFrame, reference_date: datetime | str | None = None, device=None,
                       row_nan_limit: int = 20, preset: str = "script") -> pd.DataFrame:
    """Stage-2 cleaning: drop leakage/useless columns, drop rows with more than ``row_nan_limit`` NaNs,
    parse ``emp_length``/``revol_util``/``earliest_cr_line``, map ``loan_status`` -> ``loan_default``.

    ``reference_date`` pins the reference's ``datetime.today()`` (App. B.2) for reproducible days.
    The ``notebook`` preset keeps ``next_pymnt_d``/``last_credit_pull_d`` at this stage (03:1367).
    """
    dev = frame.resolve_device(device)
    drop = LEAKAGE_STAGE2 + [c for c in USELESS_STAGE2
                             if not (preset == "notebook" and c in ("next_pymnt_d", "last_credit_pull_d"))]
    out = df.drop(columns=drop, errors="ignore")
    keep_min = out.shape[1] - row_nan_limit
    non_na = out.shape[1] - frame.row_null_counts(out, None, dev)
    out = out.loc[non_na >= keep_min]

    if "emp_length" in out.columns:
        el = out["emp_length"].replace("< 1 year", "0")
        num = pd.to_numeric(el.astype("string").str.extract(r"(\d+)")[0], errors="coerce").astype("float64")
        out = out.drop(columns=["emp_length"]).assign(emp_length_num=num)
    if "revol_util" in out.columns and not pd.api.types.is_numeric_dtype(out["revol_util"].dtype):
        out = out.assign(revol_util=out["revol_util"].str.replace("%", "", regex=False).astype(float) / 100)
    if "earliest_cr_line" in out.columns:
        today = pd.Timestamp(reference_date) if reference_date is not None else pd.Timestamp(datetime.today())
        dates = pd.to_datetime(out["earliest_cr_line"], format="%b-%Y", errors="coerce")
        out = out.drop(columns=["earliest_cr_line"]).assign(earliest_cr_line_days=(today - dates).dt.days)
    if "loan_status" in out.columns:
        out = out.drop(columns=["loan_status"]).assign(loan_default=out["loan_status"].map(LOAN_STATUS_MAP))
    return out


def _log_transform(df: pd.DataFrame, dev: torch.device) -> pd.DataFrame:
    cols = [c for c in LOG_COLUMNS if c in df.columns and pd.api.types.is_numeric_dtype(df[c].dtype)]
    if not cols:
        return df.copy()
    X = frame.to_device(df, cols, dev)
    mom = prep_ops.col_moments(X).cpu().numpy()   # count, sum, sumsq, min, max
    # skip all-missing columns and columns without any positive value (reference rule)
    sel = [i for i in range(len(cols)) if mom[i, 0] > 0 and mom[i, 4] > 0]
    prep_ops.masked_log1p_(X, sel)
    Xh = X.cpu().numpy()
    out = df.copy()
    for i in sel:
        out[cols[i]] = Xh[i]
    return out


def _dummies(df: pd.DataFrame, dev: torch.device) -> pd.DataFrame:
    missing = [c for c in DUMMY_COLUMNS if c not in df.columns]
    if missing:
        raise KeyError(f"None of {missing} are in the columns")
    base = df.drop(columns=DUMMY_COLUMNS)
    blocks = []
    for c in DUMMY_COLUMNS:
        s = df[c]
        levels = sorted(s.dropna().unique().tolist(), key=lambda v: (str(type(v)), v))
        if len(levels) <= 1:
            continue
        code_of = {v: i for i, v in enumerate(levels)}
        codes = s.map(code_of).fillna(-1).astype(np.int32).to_numpy()
        oh = prep_ops.onehot(torch.from_numpy(codes).to(dev), len(levels), True).cpu().numpy().astype(bool)
        blocks.append(pd.DataFrame(oh, index=df.index, columns=[f"{c}_{v}" for v in levels[1:]]))
    return pd.concat([base] + blocks, axis=1) if blocks else base


def _nn_dataset(df_log: pd.DataFrame, dev: torch.device) -> pd.DataFrame:
    nn = df_log.copy()
    nulls = frame.null_counts(nn, dev)
    with_nulls = [c for c in nulls.index[nulls > 0] if c != "dti" and pd.api.types.is_numeric_dtype(nn[c].dtype)]
    if with_nulls:
        X = frame.to_device(nn, with_nulls, dev)
        med = prep_ops.median(X)
        ind = prep_ops.fill_with_indicator_(X, list(range(len(with_nulls))), med.cpu().tolist(), True)
        Xh, Ih = X.cpu().numpy(), ind.cpu().numpy().astype(np.int64)
        # one concat for the filled columns and the _NA block (per-column inserts fragment the frame:
        # pandas PerformanceWarning at the reference's ~30 imputed columns)
        filled = pd.DataFrame({c: Xh[j] for j, c in enumerate(with_nulls)}, index=nn.index)
        na = pd.DataFrame({c + "_NA": Ih[j] for j, c in enumerate(with_nulls)}, index=nn.index)
        order = list(nn.columns) + list(na.columns)
        nn = pd.concat([nn.drop(columns=with_nulls), filled, na], axis=1)[order]
    nn["no_income"] = (nn["annual_inc"].isna() | (nn["annual_inc"] == 0)).astype(int)
    nn["dti_NA"] = df_log["dti"].isna().astype(int)
    dti_med = prep_ops.median(frame.to_device(nn, ["dti"], dev)).cpu().numpy()[0]
    nn["dti"] = nn["dti"].fillna(dti_med)
    obj = nn.select_dtypes(include=["object", "category", "string"]).columns.tolist()
    for c in obj:
        vals = nn[c].astype(str)
        uniq = np.unique(vals.to_numpy())
        nn[c] = np.searchsorted(uniq, vals.to_numpy()).astype(np.int64)
    return nn


def feature_engineer_lending_data(df: pd.DataFrame, device=None) -> tuple[pd.DataFrame, pd.DataFrame]:
    """Return ``(df_tree, df_nn)`` as the reference's ``feature_engineer_lending_data``."""
    dev = frame.resolve_device(device)
    df_log = _log_transform(df, dev)
    df_tree = _dummies(df_log, dev)
    df_nn = _nn_dataset(df_log, dev)
    return df_tree, df_nn
