"""Synthetic raw LendingClub export (strings and all) for the preprocessing pipeline.

Mirrors the raw 100k-sample schema the reference cleans (notebooks/01_data_cleaning.ipynb:2985;
SURVEY.md §2.3): two ``Unnamed`` index columns, ``" 36 months"`` terms, ``"13.56%"`` rates and
utilisations, ``"10+ years"`` / ``"< 1 year"`` employment lengths, ``"Aug-2003"`` dates, the full
``loan_status`` vocabulary, mostly-null hardship/joint columns (> 70% null), a few columns with
1-9 nulls, and injected duplicate rows -- so every branch of App. A.1/A.2 is exercised.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

MONTHS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]
STATUS = ["Fully Paid", "Current", "Charged Off", "Late (31-120 days)", "In Grace Period", "Late (16-30 days)",
          "Default", "Issued", "Does not meet the credit policy. Status:Fully Paid"]
STATUS_P = [0.47, 0.36, 0.14, 0.012, 0.006, 0.003, 0.001, 0.006, 0.002]
PURPOSE = ["debt_consolidation", "credit_card", "home_improvement", "other", "major_purchase", "medical",
           "small_business", "car", "vacation", "moving", "house", "wedding", "renewable_energy"]


# Further numeric columns of the LendingClub export (names from its data dictionary), used to widen the
# synthetic frame to the real export's 143 columns (``n_cols``); (name, missing share, generator kind)
EXTRA_NUMERIC = [
    ("tot_coll_amt", 0.03, "logn"), ("tot_cur_bal", 0.03, "logn"), ("total_rev_hi_lim", 0.03, "logn"),
    ("acc_open_past_24mths", 0.02, "pois4"), ("avg_cur_bal", 0.03, "logn"), ("bc_open_to_buy", 0.04, "logn"),
    ("bc_util", 0.04, "pct"), ("mo_sin_old_il_acct", 0.06, "pois120"), ("mo_sin_rcnt_rev_tl_op", 0.03, "pois12"),
    ("mo_sin_rcnt_tl", 0.03, "pois8"), ("mths_since_recent_bc", 0.04, "pois24"),
    ("mths_since_recent_inq", 0.12, "pois6"), ("num_accts_ever_120_pd", 0.03, "pois0"),
    ("num_actv_bc_tl", 0.03, "pois4"), ("num_actv_rev_tl", 0.03, "pois6"), ("num_bc_sats", 0.03, "pois4"),
    ("num_bc_tl", 0.03, "pois8"), ("num_il_tl", 0.03, "pois8"), ("num_op_rev_tl", 0.03, "pois8"),
    ("num_rev_tl_bal_gt_0", 0.03, "pois6"), ("num_sats", 0.03, "pois12"), ("num_tl_120dpd_2m", 0.06, "pois0"),
    ("num_tl_30dpd", 0.03, "pois0"), ("num_tl_90g_dpd_24m", 0.03, "pois0"), ("num_tl_op_past_12m", 0.03, "pois2"),
    ("pct_tl_nvr_dlq", 0.03, "pct"), ("percent_bc_gt_75", 0.04, "pct"), ("tax_liens", 0.0, "pois0"),
    ("tot_hi_cred_lim", 0.03, "logn"), ("total_bal_ex_mort", 0.03, "logn"), ("total_bc_limit", 0.03, "logn"),
    ("total_il_high_credit_limit", 0.03, "logn"), ("open_act_il", 0.3, "pois2"), ("open_rv_12m", 0.3, "pois1"),
    ("open_rv_24m", 0.3, "pois2"), ("total_bal_il", 0.3, "logn"), ("total_cu_tl", 0.3, "pois1"),
    ("inq_fi", 0.3, "pois1"), ("collections_12_mths_ex_med", 0.0, "pois0"), ("delinq_amnt", 0.0, "pois0"),
    ("mths_since_last_major_derog", 0.74, "pois40"), ("mths_since_last_record", 0.84, "pois60"),
    ("policy_code", 0.0, "one"), ("revol_bal_joint", 0.95, "logn"), ("sec_app_fico_range_low", 0.95, "fico"),
    ("sec_app_fico_range_high", 0.95, "fico"), ("sec_app_inq_last_6mths", 0.95, "pois1"),
    ("sec_app_mort_acc", 0.95, "pois1"), ("sec_app_open_acc", 0.95, "pois12"), ("sec_app_revol_util", 0.95, "pct"),
    ("sec_app_open_act_il", 0.95, "pois2"), ("sec_app_num_rev_accts", 0.95, "pois12"),
    ("sec_app_chargeoff_within_12_mths", 0.95, "pois0"), ("sec_app_collections_12_mths_ex_med", 0.95, "pois0"),
    ("dti_joint", 0.93, "dti"), ("deferral_term", 0.95, "three"), ("hardship_amount", 0.95, "logn"),
    ("hardship_length", 0.95, "three"), ("hardship_dpd", 0.95, "pois8"),
    ("orig_projected_additional_accrued_interest", 0.96, "logn"), ("hardship_payoff_balance_amount", 0.95, "logn"),
    ("hardship_last_payment_amount", 0.95, "logn"), ("settlement_amount", 0.97, "logn"),
    ("settlement_percentage", 0.97, "pct"), ("settlement_term", 0.97, "pois12"), ("out_prncp_inv", 0.0, "logn"),
    ("total_pymnt_inv", 0.0, "logn"), ("member_id", 1.0, "one"), ("open_il_6m", 0.3, "pois1"),
    ("mths_since_rcnt_il", 0.32, "pois20"), ("sec_app_mths_since_last_major_derog", 0.98, "pois40"),
    ("num_tl_120dpd_6m", 0.06, "pois0"), ("settlement_days", 0.97, "pois30"),
]


def _extra_column(rng: np.random.Generator, n: int, kind: str) -> np.ndarray:
    if kind == "logn":
        v = np.round(np.exp(8 + 1.2 * rng.standard_normal(n)))
    elif kind.startswith("pois"):
        v = rng.poisson(float(kind[4:]) or 0.05, n).astype(float)
    elif kind == "pct":
        v = np.clip(np.round(60 + 30 * rng.standard_normal(n), 1), 0, 100)
    elif kind == "fico":
        v = np.clip(np.round((690 + 40 * rng.standard_normal(n)) / 5) * 5, 540, 850)
    elif kind == "dti":
        v = np.round(np.clip(18 + 8 * rng.standard_normal(n), 0, 60), 2)
    elif kind == "three":
        v = np.full(n, 3.0)
    else:
        v = np.ones(n)
    return v


def make_raw_lendingclub(n: int, seed: int = 0, n_dups: int = 3, n_cols: int | None = None) -> pd.DataFrame:
    """``n`` raw rows (+ ``n_dups`` exact duplicates); ``n_cols`` widens the frame with further numeric
    LendingClub columns (EXTRA_NUMERIC) up to that many columns (the full export has 143)."""
    rng = np.random.default_rng(seed)
    grade = rng.choice(list("ABCDEFG"), n, p=[0.19, 0.29, 0.28, 0.14, 0.06, 0.03, 0.01])
    gi = np.searchsorted(np.array(list("ABCDEFG")), grade)
    loan = np.clip(np.round(np.exp(9.45 + 0.6 * rng.standard_normal(n)) / 25) * 25, 1000, 40000)
    term = np.where(rng.random(n) < 0.3, 60, 36)
    rate = np.clip(0.065 + 0.035 * gi + 0.01 * rng.standard_normal(n), 0.05, 0.31)
    r = rate / 12
    inst = np.round(loan * r / (1 - (1 + r) ** (-term)), 2)
    fico = np.clip(np.round((700 + 33 * rng.standard_normal(n) - 5 * gi) / 5) * 5, 640, 845)
    status = rng.choice(STATUS, n, p=STATUS_P)
    bad = np.isin(status, ["Charged Off", "Late (31-120 days)", "Default"])
    last_fico = np.where(bad, 575 + 75 * rng.standard_normal(n), 712 + 48 * rng.standard_normal(n))
    last_fico = np.clip(np.floor(last_fico / 5) * 5 + 4, 300, 850)
    emp = rng.choice(["10+ years", "< 1 year", "1 year", "2 years", "3 years", "4 years", "5 years", "6 years",
                      "7 years", "8 years", "9 years"], n)
    emp = np.where(rng.random(n) < 0.07, None, emp)
    yr = rng.integers(1970, 2016, n)
    mo = rng.integers(0, 12, n)
    ecl = np.array([f"{MONTHS[m]}-{y}" for m, y in zip(mo, yr)], dtype=object)
    issue = np.array([f"{MONTHS[m]}-{y}" for m, y in zip(rng.integers(0, 12, n), rng.integers(2012, 2020, n))],
                     dtype=object)
    annual = np.round(np.exp(11.1 + 0.5 * rng.standard_normal(n)), -2)
    annual[rng.random(n) < 0.002] = 0
    dti = np.round(np.clip(18 + 8 * rng.standard_normal(n), 0, 60), 2)
    dti[annual == 0] = np.nan
    new = rng.random(n) >= 0.296
    il12 = np.where(new, rng.poisson(0.7, n), np.nan)
    il24 = np.where(new, il12 + rng.poisson(0.9, n), np.nan)
    maxbal = np.where(new, np.round(np.exp(8.4 + 0.9 * rng.standard_normal(n))), np.nan)
    util = np.clip(50 + 25 * rng.standard_normal(n), 0, 120).round(1)
    util_s = np.array([f"{u}%" for u in util], dtype=object)
    util_s[rng.random(n) < 0.001] = None
    hard = np.where(rng.random(n) < 0.049, rng.choice(["ACTIVE", "BROKEN", "COMPLETE", "COMPLETED"], n), None)
    joint = rng.random(n) < 0.072
    mths_delinq = np.where(rng.random(n) < 0.5, rng.integers(0, 120, n).astype(float), np.nan)
    acc_now = np.where(rng.random(n) < 0.995, 0, 1)
    df = pd.DataFrame({
        "Unnamed: 0.1": np.arange(n), "Unnamed: 0": np.arange(n),
        "id": np.arange(10_000_000, 10_000_000 + n),
        "loan_amnt": loan, "funded_amnt": loan, "funded_amnt_inv": loan - rng.integers(0, 2, n) * 25,
        "term": np.array([f" {t} months" for t in term], dtype=object),
        "int_rate": np.array([f"{x * 100:.2f}%" for x in rate], dtype=object),
        "installment": inst, "grade": grade,
        "sub_grade": np.array([f"{g}{k}" for g, k in zip(grade, rng.integers(1, 6, n))], dtype=object),
        "emp_title": rng.choice(["Teacher", "Manager", "Nurse", "Driver", None], n),
        "emp_length": emp,
        "home_ownership": rng.choice(["MORTGAGE", "RENT", "OWN", "ANY", "NONE"], n, p=[0.49, 0.4, 0.1, 0.007, 0.003]),
        "annual_inc": annual,
        "verification_status": rng.choice(["Not Verified", "Source Verified", "Verified"], n),
        "issue_d": issue, "loan_status": status, "pymnt_plan": "n",
        "url": np.array([f"https://lc/loan/{i}" for i in range(n)], dtype=object),
        "purpose": rng.choice(PURPOSE, n), "title": rng.choice(["Debt consolidation", "Other", None], n),
        "zip_code": rng.choice(["100xx", "941xx", "606xx"], n), "addr_state": rng.choice(["NY", "CA", "IL"], n),
        "dti": dti, "delinq_2yrs": rng.poisson(0.3, n).astype(float),
        "earliest_cr_line": ecl, "fico_range_low": fico, "fico_range_high": fico + 4,
        "inq_last_6mths": rng.poisson(0.6, n).astype(float),
        "mths_since_last_delinq": mths_delinq,
        "open_acc": rng.poisson(11, n).astype(float), "pub_rec": rng.poisson(0.2, n).astype(float),
        "revol_bal": np.round(np.exp(9 + rng.standard_normal(n))), "revol_util": util_s,
        "total_acc": rng.poisson(24, n).astype(float),
        "initial_list_status": rng.choice(["w", "f"], n),
        "out_prncp": np.where(status == "Current", loan * rng.random(n), 0.0),
        "total_pymnt": loan * rng.random(n), "total_rec_prncp": loan * rng.random(n) * 0.8,
        "total_rec_int": loan * rng.random(n) * 0.2, "total_rec_late_fee": np.where(rng.random(n) < 0.03, 15.0, 0.0),
        "recoveries": np.where(bad, loan * 0.05, 0.0), "collection_recovery_fee": np.where(bad, 10.0, 0.0),
        "last_pymnt_d": issue, "last_pymnt_amnt": inst * rng.random(n),
        "next_pymnt_d": np.where(status == "Current", "Apr-2020", None),
        "last_credit_pull_d": issue, "last_fico_range_high": last_fico, "last_fico_range_low": last_fico - 4,
        "acc_now_delinq": acc_now.astype(float),
        "open_acc_6m": np.where(new, rng.poisson(1.0, n), np.nan), "open_il_12m": il12, "open_il_24m": il24,
        "max_bal_bc": maxbal, "il_util": np.where(new, rng.integers(0, 120, n), np.nan),
        "all_util": np.where(new, rng.integers(0, 120, n), np.nan),
        "inq_last_12m": np.where(new, rng.poisson(2, n), np.nan),
        "chargeoff_within_12_mths": np.where(rng.random(n) < 0.001, np.nan, 0.0),
        "mo_sin_old_rev_tl_op": rng.poisson(180, n).astype(float),
        "mort_acc": rng.poisson(1.5, n).astype(float),
        "num_rev_accts": np.where(rng.random(n) < 0.024, np.nan, 1 + rng.poisson(12.8, n)),
        "pub_rec_bankruptcies": np.where(rng.random(n) < 0.0005, np.nan, rng.binomial(1, 0.11, n)),
        "mths_since_recent_bc_dlq": np.where(rng.random(n) < 0.75, np.nan, rng.integers(0, 100, n)),
        "mths_since_recent_revol_delinq": np.where(rng.random(n) < 0.65, np.nan, rng.integers(0, 100, n)),
        "application_type": np.where(joint, "Joint App", "Individual"),
        "annual_inc_joint": np.where(joint, annual * 1.6, np.nan),
        "hardship_flag": np.where(hard != None, "Y", "N"),  # noqa: E711
        "hardship_status": hard,
        "debt_settlement_flag": rng.choice(["N", "Y"], n, p=[0.98, 0.02]),
    })
    if n_cols is not None and n_cols > df.shape[1]:
        extra = {}
        for name, miss, kind in EXTRA_NUMERIC[: n_cols - df.shape[1]]:
            v = _extra_column(rng, n, kind)
            if miss >= 1.0:
                v[:] = np.nan
            elif miss > 0:
                v[rng.random(n) < miss] = np.nan
            extra[name] = v
        df = pd.concat([df, pd.DataFrame(extra)], axis=1)
    # a few columns with 1-9 NaNs (exercises the script preset's row drop)
    for c, k in (("delinq_2yrs", 3), ("inq_last_6mths", 5), ("open_acc", 2)):
        df.loc[rng.choice(n, k, replace=False), c] = np.nan
    if n_dups and n > n_dups:
        dup_rows = df.iloc[rng.choice(n, n_dups, replace=False)].copy()
        df = pd.concat([df, dup_rows], ignore_index=True)
        # duplicates share their index columns too (exact copies), as real duplicate exports do
    return df
