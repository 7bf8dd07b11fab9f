"""Synthetic LendingClub-shaped data (there is no network, so no real dataset in the tests/bench).

``make_lendingclub`` draws the 20 deployed model features of the reference
(src/api/cobalt_fast_api.py:60-79) with the marginals recorded in the reference
notebooks (means/medians/ranges, ~29.6% nulls on the 2015+ "open_il/max_bal"
fields, 2.4% on num_rev_accts, 6.95% on emp_length, ~7.2% joint applications, ~95.1% "No Hardship")
and a logistic ground truth calibrated to the reference's 12.9% default rate. ``last_fico_range_high``
is drawn conditionally on the label, reproducing its dominance in the shipped model (App. B.13).

By default the six features the reference model splits in log1p space (App. B.1: loan_amnt,
installment, fico_range_low, num_rev_accts, pub_rec_bankruptcies, earliest_cr_line_days) are
returned log1p-transformed (``x>0`` only), i.e. the layout of the reference's tree dataset.

Randomness is counter based (splitmix64 of (seed, stream, global row)), so a row's values depend only
on its global index: every data-parallel rank can generate its own shard on its own GPU and the
union is bit-identical to the single-GPU dataset.
"""
from __future__ import annotations

import math

import torch

FEATURES = [
    "loan_amnt", "term", "installment", "fico_range_low", "last_fico_range_high", "open_il_12m", "open_il_24m",
    "max_bal_bc", "num_rev_accts", "pub_rec_bankruptcies", "emp_length_num", "earliest_cr_line_days", "grade_E",
    "home_ownership_MORTGAGE", "verification_status_Verified", "application_type_Joint App",
    "hardship_status_BROKEN", "hardship_status_COMPLETE", "hardship_status_COMPLETED",
    "hardship_status_No Hardship",
]
FEATURE_TYPES = ["float", "int", "float", "float", "float", "float", "float", "float", "float", "float", "float",
                 "float", "i", "i", "i", "i", "i", "i", "i", "i"]
LOG1P_FEATURES = ["loan_amnt", "installment", "fico_range_low", "num_rev_accts", "pub_rec_bankruptcies",
                  "earliest_cr_line_days"]

_M64 = (1 << 64) - 1


def _i64(c: int) -> int:
    c &= _M64
    return c - (1 << 64) if c >= (1 << 63) else c


_C1 = _i64(0x9E3779B97F4A7C15)
_C2 = _i64(0xBF58476D1CE4E5B9)
_C3 = _i64(0x94D049BB133111EB)


def _srl(x: torch.Tensor, k: int) -> torch.Tensor:
    """Logical right shift of int64 viewed as uint64."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def _mix(x: torch.Tensor) -> torch.Tensor:
    x = x + _C1
    x = (x ^ _srl(x, 30)) * _C2
    x = (x ^ _srl(x, 27)) * _C3
    return x ^ _srl(x, 31)


class _Rng:
    def __init__(self, seed: int, rows: torch.Tensor):
        self.base = _mix(rows ^ _i64(seed * 0x100000001B3))
        self.k = 0

    def uniform(self) -> torch.Tensor:
        self.k += 1
        h = _mix(self.base ^ _i64(self.k * 0xD1B54A32D192ED03))
        return (_srl(h, 11).to(torch.float64) + 0.5) * (1.0 / 9007199254740992.0)

    def normal(self) -> torch.Tensor:
        u1, u2 = self.uniform(), self.uniform()
        return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)

    def poisson(self, lam: torch.Tensor | float, kmax: int = 40) -> torch.Tensor:
        u = self.uniform()
        lam_t = torch.as_tensor(lam, dtype=torch.float64, device=u.device).expand_as(u)
        p = torch.exp(-lam_t)
        cdf = p.clone()
        k = torch.zeros_like(u)
        for i in range(1, kmax):
            more = u > cdf
            if not bool(more.any()):
                break
            k = k + more.to(torch.float64)
            p = p * lam_t / i
            cdf = cdf + p
        return k

    def choice(self, probs: list[float]) -> torch.Tensor:
        u = self.uniform()
        edges = torch.tensor(list(_cumsum(probs)), dtype=torch.float64, device=u.device)
        return torch.bucketize(u, edges[:-1], right=True)


def _cumsum(ps):
    s = 0.0
    for p in ps:
        s += p
        yield s


# logit intercept calibrated (2^20 rows, seed 0) to a 12.9% default rate
_INTERCEPT = -2.86


def make_lendingclub(n_rows: int, seed: int = 0, row_offset: int = 0, device: str | torch.device = "cpu",
                     log_space: bool = True, dtype: torch.dtype = torch.float32,
                     chunk: int = 1 << 22) -> tuple[torch.Tensor, torch.Tensor]:
    """Return ``(X [n, 20], y [n])``; rows are global indices ``row_offset .. row_offset+n-1``."""
    dev = torch.device(device)
    X = torch.empty((n_rows, len(FEATURES)), dtype=dtype, device=dev)
    y = torch.empty(n_rows, dtype=dtype, device=dev)
    for s in range(0, n_rows, chunk):
        e = min(n_rows, s + chunk)
        xs, ys = _gen(row_offset + s, e - s, seed, dev, log_space)
        X[s:e] = xs.to(dtype)
        y[s:e] = ys.to(dtype)
    return X, y


def _gen(first: int, n: int, seed: int, dev: torch.device, log_space: bool):
    rows = torch.arange(first, first + n, dtype=torch.int64, device=dev)
    r = _Rng(seed, rows)
    f64 = torch.float64
    nan = torch.tensor(float("nan"), dtype=f64, device=dev)

    grade = r.choice([0.19, 0.29, 0.28, 0.14, 0.06, 0.03, 0.01]).to(f64)            # A..G
    loan = torch.exp(9.45 + 0.6 * r.normal()).clamp(700, 40000)
    loan = torch.round(loan / 25.0) * 25.0
    p60 = (0.12 + 0.45 * (loan > 20000).to(f64) + 0.05 * grade).clamp(0, 0.95)
    term = torch.where(r.uniform() < p60, 60.0, 36.0)
    rate = (0.065 + 0.035 * grade + 0.01 * r.normal()).clamp(0.05, 0.31) / 12.0
    installment = loan * rate / (1 - torch.pow(1 + rate, -term))
    installment = torch.round(installment * 100) / 100
    fico = (690.0 + 5.0 * torch.floor(r.poisson(torch.clamp(3.5 - 0.35 * grade, min=0.3)) * 2.0)
            + 10 * r.normal().abs() - 4 * grade).clamp(640, 845)
    fico = torch.round(fico / 5.0) * 5.0
    new_fields = r.uniform() >= 0.296                                                  # 2015+ loans
    il12 = r.poisson(0.70)
    il24 = il12 + r.poisson(0.92)
    maxbal = torch.where(r.uniform() < 0.03, torch.zeros_like(loan), torch.exp(8.4 + 0.9 * r.normal()).clamp(1, 94246))
    maxbal = torch.round(maxbal)
    nra = (1 + r.poisson(12.8)).clamp(1, 92)
    bk = torch.where(r.uniform() < 0.885, 0.0, torch.where(r.uniform() < 0.9, 1.0, 2.0 + r.poisson(0.3)))
    emp = torch.where(r.uniform() < 0.33, 10.0, torch.floor(r.uniform() * 10.0))
    ecl = (6500.0 + 2700.0 * r.normal()).clamp(1000, 25000).round()
    mortgage = (r.uniform() < 0.49).to(f64)
    verified = (r.uniform() < 0.28 + 0.04 * grade).to(f64)
    joint = (r.uniform() < 0.072).to(f64)
    dti_z = r.normal()

    risk = (_INTERCEPT + 0.42 * grade + 0.35 * (term == 60).to(f64) - 0.010 * (fico - 700) + 0.12 * il12
            + 0.25 * dti_z + 0.25 * bk - 0.12 * mortgage + 0.15 * verified - 0.02 * emp
            - 0.00002 * (ecl - 6500) + 0.000008 * (loan - 15000) + 0.6 * r.normal())
    y = (r.uniform() < torch.sigmoid(risk)).to(f64)

    # hardship status (ACTIVE is the dropped first level of the one-hot)
    hu = r.uniform()
    hard_rate = torch.where(y == 1, torch.full_like(hu, 0.16), torch.full_like(hu, 0.031))
    hs = torch.where(hu >= hard_rate, 4.0, torch.floor(r.uniform() * 4.0).clamp(0, 3))  # 0 ACTIVE 1 BROKEN 2 COMPLETE 3 COMPLETED 4 none
    hs = torch.where((hs == 1) & (y == 0) & (r.uniform() < 0.6), 3.0, hs)

    # post-origination FICO: the reference model's dominant (leaky) feature
    lf = torch.where(y == 1, 575.0 + 75.0 * r.normal(), 712.0 + 48.0 * r.normal()).clamp(300, 850)
    lf = torch.floor(lf / 5.0) * 5.0 + 4.0
    lf = torch.where(r.uniform() < 0.004, torch.zeros_like(lf), lf.clamp(max=850))

    cols = [loan, term, installment, fico, lf,
            torch.where(new_fields, il12, nan), torch.where(new_fields, il24, nan),
            torch.where(new_fields, maxbal, nan),
            torch.where(r.uniform() < 0.024, nan, nra),
            torch.where(r.uniform() < 0.0005, nan, bk),
            torch.where(r.uniform() < 0.0695, nan, emp),
            ecl, (grade == 4).to(f64), mortgage, verified, joint,
            (hs == 1).to(f64), (hs == 2).to(f64), (hs == 3).to(f64), (hs == 4).to(f64)]
    X = torch.stack(cols, 1)
    if log_space:
        for name in LOG1P_FEATURES:
            j = FEATURES.index(name)
            v = X[:, j]
            X[:, j] = torch.where(v > 0, torch.log1p(v), v)
    return X, y


def train_test_split_rows(n: int, test_frac: float = 0.2) -> tuple[int, int]:
    n_test = int(round(n * test_frac))
    return n - n_test, n_test
