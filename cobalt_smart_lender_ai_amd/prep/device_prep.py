"""Stage 1 -> stage 2 -> feature engineering on a :class:`~.device_frame.DeviceFrame` (full-scale,
device-resident path; the pandas path in ``prep/clean.py`` / ``prep/features.py`` is its oracle).

Same semantics as the reference, step for step:

* ``device_clean_data_flow``  = src/data_preprocessing/clean_data.py:87-158 (+ notebook preset);
* ``device_clean_lending_data`` = src/data_preprocessing/feature_engineering.py:44-101;
* ``device_feature_engineer``  = src/data_preprocessing/feature_engineering.py:103-184 (tree + NN sets).

String parses run once per distinct value (host) and are gathered per row on the device; log1p,
imputation, indicators, one-hot, medians, null counts, row filters and dedupe are device kernels.
``tree_training_matrix`` hands the tree set to the GBDT's binning without leaving HBM.
"""
from __future__ import annotations

import logging
import re
import time
from datetime import datetime

import numpy as np
import pandas as pd
import torch

from ..ops import prep_ops
from .clean import INDEX_COLUMNS, NOTEBOOK_UNNECESSARY, SCRIPT_UNNECESSARY, ZERO_FILL
from .device_frame import DCol, DeviceFrame, gather_vocab
from .features import DUMMY_COLUMNS, LEAKAGE_STAGE2, LOAN_STATUS_MAP, LOG_COLUMNS, USELESS_STAGE2

log = logging.getLogger(__name__)


def _col(df: DeviceFrame, name: str) -> DCol:
    """A column, hashed strings ("h") decoded to dictionary codes (only stages that need the values)."""
    return df.as_categorical(name)


# ------------------------------------------------------------------------------------------ stage 1
def _parse_term(c: DCol, n_missing: int) -> DCol:
    if c.kind != "c":
        return c
    if n_missing:
        raise ValueError("cannot convert float NaN to integer")  # pandas .astype(int) on a missing term
    tab = np.array([int(str(v).replace(" months", "").strip()) for v in c.vocab], dtype=np.float64)
    return DCol("f", gather_vocab(c, tab), "int64")


def _parse_percent(c: DCol) -> DCol:
    if c.kind != "c":
        return c
    tab = np.array([float(str(v).replace("%", "")) for v in c.vocab], dtype=np.float64) / 100
    return DCol("f", gather_vocab(c, tab), "float64")


def _fill_cat(c: DCol, value: str) -> DCol:
    if c.kind == "c":
        vocab = list(c.vocab)
        if value not in vocab:
            vocab.append(value)
        k = vocab.index(value)
        return DCol("c", torch.where(c.data < 0, torch.full_like(c.data, k), c.data), "object", vocab)
    if c.kind == "f" and bool(torch.isnan(c.data).all()):  # an all-missing column read as float64
        return DCol("c", torch.zeros_like(c.data, dtype=torch.int32), "object", [value])
    return c


def device_clean_data_flow(df: DeviceFrame, preset: str = "script", null_threshold: float = 70.0) -> DeviceFrame:
    """Stage-1 cleaning (reference: clean_data.py ``clean_data_flow``; prep/clean.py is the oracle)."""
    if preset not in ("script", "notebook"):
        raise ValueError(f"unknown preset {preset!r}")
    out = df.drop(INDEX_COLUMNS)
    if preset == "script":
        nulls = out.null_counts()
        subset = [c for c, k in nulls.items() if k < 10]
        out = out.take(out.row_null_counts(subset) == 0)
    if "hardship_status" in out:
        out = out.assign(hardship_status=_fill_cat(_col(out, "hardship_status"), "No Hardship"))
    if "term" in out:
        term = _col(out, "term")
        nm = int(term.null_mask().sum()) if term.kind == "c" else 0
        out = out.assign(term=_parse_term(term, nm))
    if "int_rate" in out:
        out = out.assign(int_rate=_parse_percent(_col(out, "int_rate")))
    nulls = out.null_counts()
    drop = [c for c, k in nulls.items() if k / max(len(out), 1) * 100.0 > null_threshold]
    log.info("Dropping columns with >%s%% missing: %s", null_threshold, drop)
    out = out.drop(drop)
    if preset == "notebook" and "mths_since_last_delinq" in out:
        c = out["mths_since_last_delinq"]
        fill = torch.isnan(c.data)
        if "acc_now_delinq" in out:
            fill &= out["acc_now_delinq"].data == 0
        out = out.assign(mths_since_last_delinq=DCol("f", torch.where(fill, 999.0, c.data), "float64"))
        out = out.take(~torch.isnan(out["mths_since_last_delinq"].data))
    unnecessary = SCRIPT_UNNECESSARY if preset == "script" else NOTEBOOK_UNNECESSARY
    out = out.drop([c for c in unnecessary if c in out])
    for z in ZERO_FILL:
        if z in out and out[z].kind == "f":
            c = out[z]
            out = out.assign(**{z: DCol("f", torch.nan_to_num(c.data, nan=0.0), c.dtype)})
    before = len(out)
    out = out.take(~out.duplicated())
    log.info("Duplicates removed: %d", before - len(out))
    return out


# ------------------------------------------------------------------------------------------ stage 2
_DIGITS = re.compile(r"(\d+)")


def _emp_length_table(vocab: list) -> np.ndarray:
    out = np.full(len(vocab), np.nan)
    for i, v in enumerate(vocab):
        s = "0" if v == "< 1 year" else str(v)
        m = _DIGITS.search(s)
        if m:
            out[i] = float(m.group(1))
    return out


def device_clean_lending_data(df: DeviceFrame, reference_date: datetime | str | None = None, row_nan_limit: int = 20,
                              preset: str = "script") -> DeviceFrame:
    """Stage-2 cleaning (reference: feature_engineering.py ``clean_lending_data``)."""
    drop = LEAKAGE_STAGE2 + [c for c in USELESS_STAGE2
                             if not (preset == "notebook" and c in ("next_pymnt_d", "last_credit_pull_d"))]
    out = df.drop(drop)
    keep_min = out.shape[1] - row_nan_limit
    non_na = out.shape[1] - out.row_null_counts(None)
    out = out.take(non_na >= keep_min)
    if "emp_length" in out:
        c = _col(out, "emp_length")
        if c.kind == "c":
            num = gather_vocab(c, _emp_length_table(c.vocab))
        else:  # numeric emp_length: astype("string") -> the digits of its text
            num = torch.floor(c.data).where(~torch.isnan(c.data), c.data)
        out = out.drop(["emp_length"]).assign(emp_length_num=DCol("f", num, "float64"))
    if "revol_util" in out and out["revol_util"].kind in ("c", "h"):
        out = out.assign(revol_util=_parse_percent(_col(out, "revol_util")))
    if "earliest_cr_line" in out:
        c = _col(out, "earliest_cr_line")
        today = pd.Timestamp(reference_date) if reference_date is not None else pd.Timestamp(datetime.today())
        if c.kind == "c":
            dates = pd.to_datetime(pd.Series(c.vocab, dtype=object), format="%b-%Y", errors="coerce")
            tab = (today - dates).dt.days.to_numpy(dtype=np.float64, na_value=np.nan)
            days = gather_vocab(c, tab)
        else:
            days = torch.full((len(out),), float("nan"), dtype=torch.float64, device=out.device)
        dt = "int64" if not bool(torch.isnan(days).any()) else "float64"
        out = out.drop(["earliest_cr_line"]).assign(earliest_cr_line_days=DCol("f", days, dt))
    if "loan_status" in out:
        c = _col(out, "loan_status")
        if c.kind == "c":
            tab = np.array([LOAN_STATUS_MAP.get(v, np.nan) for v in c.vocab], dtype=np.float64)
            lab = gather_vocab(c, tab)
        else:
            lab = torch.full((len(out),), float("nan"), dtype=torch.float64, device=out.device)
        dt = "int64" if not bool(torch.isnan(lab).any()) else "float64"
        out = out.drop(["loan_status"]).assign(loan_default=DCol("f", lab, dt))
    return out


# ------------------------------------------------------------------------------------------ features
def _log_transform(df: DeviceFrame) -> DeviceFrame:
    cols = [c for c in LOG_COLUMNS if c in df and df[c].kind == "f"]
    if not cols:
        return df.copy()
    X = torch.stack([df[c].data for c in cols])              # [C, N] float64
    mom = prep_ops.col_moments(X).cpu().numpy()               # count, sum, sumsq, min, max
    sel = [i for i in range(len(cols)) if mom[i, 0] > 0 and mom[i, 4] > 0]
    prep_ops.masked_log1p_(X, sel)                            # K6: one launch for every column
    return df.assign(**{cols[i]: DCol("f", X[i], "float64") for i in sel})


def _sorted_levels(c: DCol) -> tuple[list, torch.Tensor]:
    """Present levels sorted as pandas/Python sort them, and code -> rank (-1 missing) on the device."""
    if c.kind == "c":
        present = torch.unique(c.data[c.data >= 0]).cpu().numpy()
        vals = [c.vocab[k] for k in present]
        order = sorted(range(len(vals)), key=lambda i: (str(type(vals[i])), vals[i]))
        rank = np.full(len(c.vocab) + 1, -1, dtype=np.int32)
        for r, i in enumerate(order):
            rank[present[i]] = r
        rt = torch.from_numpy(rank).to(c.data.device)
        return [vals[i] for i in order], rt[torch.where(c.data < 0, len(c.vocab), c.data.long())]
    x = c.data.to(torch.float64)
    u = torch.unique(x[~torch.isnan(x)])                      # sorted
    codes = torch.searchsorted(u, torch.nan_to_num(x, nan=0.0)).to(torch.int32)
    codes = torch.where(torch.isnan(x), -1, codes)
    vals = u.cpu().numpy().tolist()
    if c.dtype in ("int64", "bool"):
        vals = [int(v) for v in vals]
    return vals, codes


def _dummies(df: DeviceFrame) -> DeviceFrame:
    missing = [c for c in DUMMY_COLUMNS if c not in df]
    if missing:
        raise KeyError(f"None of {missing} are in the columns")
    out = df.drop(DUMMY_COLUMNS)
    for c in DUMMY_COLUMNS:
        levels, codes = _sorted_levels(_col(df, c))
        if len(levels) <= 1:
            continue
        oh = prep_ops.onehot(codes, len(levels), True)        # K7: [N, L-1] uint8 (drop_first)
        out = out.assign(**{f"{c}_{v}": DCol("b", oh[:, j].contiguous(), "bool") for j, v in enumerate(levels[1:])})
    return out


def _nn_dataset(df_log: DeviceFrame) -> DeviceFrame:
    nn = df_log.copy()
    nulls = nn.null_counts()
    with_nulls = [c for c, k in nulls.items() if k > 0 and c != "dti" and nn[c].numeric]
    if with_nulls:
        X = torch.stack([nn[c].data.to(torch.float64) for c in with_nulls])
        med = prep_ops.median(X)                               # K4: device sort
        ind = prep_ops.fill_with_indicator_(X, list(range(len(with_nulls))), med.cpu().tolist(), True)  # K3/K5
        for j, c in enumerate(with_nulls):
            nn = nn.assign(**{c + "_NA": DCol("b", ind[j].to(torch.uint8), "int64")})
            nn = nn.assign(**{c: DCol("f", X[j], "float64")})
    inc = nn["annual_inc"].data
    nn = nn.assign(no_income=DCol("b", (torch.isnan(inc) | (inc == 0)).to(torch.uint8), "int64"))
    nn = nn.assign(dti_NA=DCol("b", torch.isnan(df_log["dti"].data).to(torch.uint8), "int64"))
    dti = nn["dti"].data
    dmed = prep_ops.median(dti.to(torch.float64).unsqueeze(0))[0]
    nn = nn.assign(dti=DCol("f", torch.where(torch.isnan(dti), dmed, dti), "float64"))
    for c in [k for k, v in nn.cols.items() if v.kind in ("c", "h")]:
        col = _col(nn, c)
        # LabelEncoder().fit_transform(astype(str)): missing values are the string "nan"
        strs = [str(v) for v in col.vocab] + ["nan"]
        present = torch.unique(torch.where(col.data < 0, len(col.vocab), col.data.long())).cpu().numpy()
        uniq = sorted({strs[k] for k in present})
        pos = {s: i for i, s in enumerate(uniq)}
        tab = np.array([pos.get(s, -1) for s in strs], dtype=np.float64)
        t = torch.from_numpy(tab).to(col.data.device)
        enc = t[torch.where(col.data < 0, len(col.vocab), col.data.long())]
        nn = nn.assign(**{c: DCol("f", enc, "int64")})
    return nn


def device_feature_engineer(df: DeviceFrame) -> tuple[DeviceFrame, DeviceFrame]:
    """``(tree, nn)`` datasets (reference: feature_engineering.py ``feature_engineer_lending_data``)."""
    df_log = _log_transform(df)
    return _dummies(df_log), _nn_dataset(df_log)


def tree_training_matrix(tree: DeviceFrame, drop: list[str] = (), label: str = "loan_default"
                         ) -> tuple[torch.Tensor, torch.Tensor, list[str]]:
    """Float32 device matrix + labels of the tree set for the GBDT (rows with a missing label dropped;
    see pipeline/train_tree.py), without leaving HBM."""
    lab = tree[label].data
    keep = ~torch.isnan(lab)
    t = tree.take(keep) if not bool(keep.all()) else tree
    names = [c for c in t.columns if c != label and c not in set(drop)]
    return t.matrix(names), t[label].data.to(torch.float32), names


def run_device_prep(src, device="cuda", reference_date=None, preset: str = "script", engine: str = "auto") -> dict:
    """Raw CSV (path or bytes) -> cleaned -> stage 2 -> (tree, nn) DeviceFrames, with stage timings.
    ``engine``: the CSV reader (DeviceFrame.read_csv: "auto" = on the GPU when there is one)."""
    dev = torch.device(device)
    t = {}
    ing: dict = {}
    t0 = time.perf_counter()
    raw = DeviceFrame.read_csv(src, dev, engine=engine, timings=ing)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t["ingest"] = time.perf_counter() - t0
    for k in ("read", "tokenize", "parse", "columns"):
        if k in ing:
            t["ingest_" + k] = ing[k]
    t1 = time.perf_counter()
    c1 = device_clean_data_flow(raw, preset=preset)
    t["stage1"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    c2 = device_clean_lending_data(c1, reference_date=reference_date, preset=preset)
    t["stage2"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    tree, nn = device_feature_engineer(c2)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t["features"] = time.perf_counter() - t1
    t["total"] = time.perf_counter() - t0
    return {"raw_shape": raw.shape, "clean": c1, "stage2": c2, "tree": tree, "nn": nn, "timings": t}
