"""Preprocessing semantics against a literal pandas oracle written here."""
import warnings

import numpy as np
import pandas as pd
import pytest
import torch

from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
from cobalt_smart_lender_ai_amd.ops import prep_ops
from cobalt_smart_lender_ai_amd.prep import clean, features

REF_DATE = "2025-07-04"


# ----------------------------------------------------------------------------- pandas oracles
def oracle_stage1(df):
    d = df.drop(columns=["Unnamed: 0.1", "Unnamed: 0"], errors="ignore")
    d = d.dropna(subset=d.columns[d.isnull().sum() < 10])
    d["hardship_status"] = d["hardship_status"].fillna("No Hardship")
    d["term"] = d["term"].str.replace(" months", "").astype(int)
    d["int_rate"] = d["int_rate"].str.replace("%", "").astype(float) / 100
    pct = d.isnull().sum() / len(d) * 100
    d = d.drop(columns=pct[pct > 70].index.tolist())
    for c in ["next_pymnt_d", "last_pymnt_d", "last_credit_pull_d", "mths_since_recent_revol_delinq", "il_util",
              "all_util", "mths_since_recent_bc_dlq"]:
        if c in d.columns:
            d = d.drop(columns=[c])
    for c in ["inq_last_12m", "open_acc_6m", "chargeoff_within_12_mths"]:
        if c in d.columns:
            d[c] = d[c].fillna(0)
    return d.drop_duplicates()


def oracle_stage2(df):
    d = df.drop(columns=features.LEAKAGE_STAGE2 + features.USELESS_STAGE2, errors="ignore")
    d = d.dropna(thresh=d.shape[1] - 20)
    d["emp_length"] = d["emp_length"].replace("< 1 year", "0")
    d["emp_length_num"] = pd.to_numeric(d["emp_length"].str.extract(r"(\d+)")[0], errors="coerce")
    d = d.drop(columns=["emp_length"])
    d["revol_util"] = d["revol_util"].str.replace("%", "", regex=False).astype(float) / 100
    dt = pd.to_datetime(d["earliest_cr_line"], format="%b-%Y", errors="coerce")
    d["earliest_cr_line_days"] = (pd.Timestamp(REF_DATE) - dt).dt.days
    d = d.drop(columns=["earliest_cr_line"])
    d["loan_default"] = d["loan_status"].map(features.LOAN_STATUS_MAP)
    return d.drop(columns=["loan_status"])


def oracle_fe(df):
    lg = df.copy()
    for c in features.LOG_COLUMNS:
        if c in lg.columns:
            if lg[c].notnull().sum() == 0 or (lg[c].dropna() <= 0).all():
                continue
            lg[c] = lg[c].apply(lambda x: np.log1p(x) if pd.notnull(x) and x > 0 else x)
    tree = pd.get_dummies(lg.copy(), columns=features.DUMMY_COLUMNS, drop_first=True)
    nn = lg.copy()
    for c in nn.isnull().sum()[lambda s: s > 0].index:
        if c == "dti" or not np.issubdtype(nn[c].dtype, np.number):
            continue
        nn[c + "_NA"] = nn[c].isnull().astype(int)
        nn[c] = nn[c].fillna(nn[c].median())
    nn["no_income"] = ((nn["annual_inc"].isnull()) | (nn["annual_inc"] == 0)).astype(int)
    nn["dti_NA"] = lg["dti"].isnull().astype(int)
    nn["dti"] = nn["dti"].fillna(nn["dti"].median())
    from sklearn.preprocessing import LabelEncoder

    for c in nn.select_dtypes(include=["object", "category"]).columns:
        nn[c] = LabelEncoder().fit_transform(nn[c].astype(str))
    return tree, nn


@pytest.fixture(scope="module")
def raw():
    return make_raw_lendingclub(3000, seed=7)


def _eq(a, b):
    a = a.reset_index(drop=True)
    b = b.reset_index(drop=True)
    assert list(a.columns) == list(b.columns)
    pd.testing.assert_frame_equal(a, b, check_dtype=False, check_exact=False, rtol=1e-12)


def test_stage1_matches_oracle(raw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        _eq(clean.clean_data_flow(raw, device="cpu"), oracle_stage1(raw))


def test_stage2_and_fe_match_oracle(raw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        s1 = oracle_stage1(raw)
        s2 = features.clean_lending_data(s1, reference_date=REF_DATE, device="cpu")
        _eq(s2, oracle_stage2(s1))
        tree, nn = features.feature_engineer_lending_data(s2, device="cpu")
        otree, onn = oracle_fe(oracle_stage2(s1))
    _eq(tree, otree)
    _eq(nn, onn)


def test_duplicates_and_small_null_rows_removed(raw):
    out = clean.clean_data_flow(raw, device="cpu")
    assert not out.duplicated().any()
    assert len(out) < len(raw) - 3  # 3 injected duplicates + rows with NaN in 1-9-null columns


def test_notebook_preset_fills_delinquency(raw):
    out = clean.clean_data_flow(raw, preset="notebook", device="cpu")
    assert out["mths_since_last_delinq"].notna().all()
    assert (out["mths_since_last_delinq"] == 999).any()


def test_prep_ops_host_semantics():
    X = torch.tensor([[1.0, np.nan, 3.0, 4.0], [np.nan, np.nan, 0.0, -2.0]], dtype=torch.float64)
    assert prep_ops.col_null_counts(X).tolist() == [1, 2]
    assert prep_ops.row_null_counts(X).tolist() == [1, 2, 0, 0]
    med = prep_ops.median(X)
    assert med[0].item() == 3.0 and med[1].item() == -1.0
    Y = X.clone()
    prep_ops.masked_log1p_(Y, [0, 1])
    assert Y[0, 0].item() == np.log1p(1.0) and Y[1, 3].item() == -2.0 and np.isnan(Y[1, 0].item())
    oh = prep_ops.onehot(torch.tensor([0, 2, -1, 1], dtype=torch.int32), 3, True)
    assert oh.tolist() == [[0, 0], [0, 1], [0, 0], [1, 0]]
    Z = torch.tensor([[1.0, 1.0, 2.0, 1.0], [np.nan, np.nan, 0.0, np.nan]], dtype=torch.float64)
    dup, _ = prep_ops.duplicated_numeric(Z)
    assert dup.tolist() == [False, True, False, True]


def test_eda_helpers_match_pandas_scipy():
    from scipy import stats

    from cobalt_smart_lender_ai_amd.prep import eda

    rng = np.random.default_rng(3)
    df = pd.DataFrame({"a": rng.normal(100, 20, 500), "b": rng.random(500), "s": ["x"] * 500})
    df.loc[rng.random(500) < 0.3, "b"] = np.nan
    ours = eda.null_data_summary(df, threshold_percentage=0, device="cpu")
    assert list(ours["Column"]) == ["b"] and ours["Percentage"].iloc[0] == pytest.approx(df["b"].isna().mean() * 100)
    np.testing.assert_allclose(eda.zscore(df["a"], device="cpu"), stats.zscore(df["a"]), rtol=1e-10)
    z = np.abs(stats.zscore(df["a"]))
    assert eda.zscore_outlier_counts(df["a"], device="cpu") == {t: int((z > t).sum()) for t in (2.0, 2.25, 2.5, 2.75)}
    d = eda.describe(df, device="cpu")
    ref = df.describe()
    np.testing.assert_allclose(d[["a", "b"]].to_numpy(), ref[["a", "b"]].to_numpy(), rtol=1e-9)


def test_notebook_preset_matches_pandas_oracle():
    raw = make_raw_lendingclub(4000, seed=9)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ours = clean.clean_data_flow(raw, preset="notebook", device="cpu")
        d = raw.drop(columns=["Unnamed: 0.1", "Unnamed: 0"], errors="ignore")
        d["hardship_status"] = d["hardship_status"].fillna("No Hardship")
        d["term"] = d["term"].str.replace(" months", "").astype(int)
        d["int_rate"] = d["int_rate"].str.replace("%", "").astype(float) / 100
        pct = d.isnull().sum() / len(d) * 100
        d = d.drop(columns=pct[pct > 70].index.tolist())
        if "mths_since_last_delinq" in d.columns:
            m = d["mths_since_last_delinq"].isna() & (d["acc_now_delinq"] == 0)
            d.loc[m, "mths_since_last_delinq"] = 999
            d = d.dropna(subset=["mths_since_last_delinq"])
        d = d.drop(columns=[c for c in clean.NOTEBOOK_UNNECESSARY if c in d.columns])
        for c in ["inq_last_12m", "open_acc_6m", "chargeoff_within_12_mths"]:
            if c in d.columns:
                d[c] = d[c].fillna(0)
        d = d.drop_duplicates()
    pd.testing.assert_frame_equal(ours.reset_index(drop=True), d.reset_index(drop=True), check_dtype=False)


def test_read_table_pandas_typing_duplicates_and_nullable_bools():
    """the CSV readers behind read_table type a frame like pandas.read_csv -- repeated
    header names become a, a.1, a.2 (pandas' renaming) instead of collapsing into one column, and a
    true/false column with missing values is pandas' object True / False / NaN (not float64); the
    CSV writer renders it as pandas does."""
    import io

    import pandas as pd

    from cobalt_smart_lender_ai_amd.prep.csv_gpu import dedup_names
    from cobalt_smart_lender_ai_amd.prep.device_frame import DeviceFrame

    assert dedup_names(["a", "b", "a", "a", "a.1"]) == ["a", "b", "a.2", "a.3", "a.1"]
    data = b"a,b,a,flag,flagn,a.1\n1,x,2.5,True,True,7\n2,y,3.5,False,,8\n3,,4.5,True,False,9\n"
    ref = pd.read_csv(io.BytesIO(data), float_precision="round_trip")
    got = DeviceFrame.read_csv(data, "cpu", engine="arrow").to_pandas()
    assert list(got.columns) == list(ref.columns)
    pd.testing.assert_frame_equal(got, ref)
    assert ref["flagn"].dtype == object
