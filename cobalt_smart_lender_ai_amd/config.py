"""Configuration: dataclasses whose defaults equal the reference's hard-coded literals.

Reference constants: S3 bucket / object keys (src/data_preprocessing/clean_data.py:15-23,
src/data_preprocessing/feature_engineering.py:17-20, src/model_train_test/model_tree_train_test.py:
26-31, src/api/cobalt_fast_api.py:19-21), training hyper-parameters (model_tree_train_test.py:82-164),
API port 8000 / UI port 8001 (cobalt_fast_api.py:148-150, src/streamlit_ui/Dockerfile). Every field
can be overridden from a YAML file (``load_yaml``) or ``COBALT_*`` environment variables.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

BUCKET_NAME = "cobalt-lending-ai-data-lake"
RAW_DATA_KEY_FULL = "dataset/1-raw/LendingClubFullData2007-2020Q3"
CLEAN_DATA_KEY_FULL = "dataset/2-intermediate/full_dataset_cleaned_01.csv"
RAW_DATA_KEY_SAMPLE = "dataset/1-raw/100kSampleData"
CLEAN_DATA_KEY_SAMPLE = "dataset/2-intermediate/sample_100k_cleaned.csv"
CLEAN_DATA_KEY_TREE = "dataset/2-intermediate/full_dataset_cleaned_02_tree.csv"
CLEAN_DATA_KEY_NN = "dataset/2-intermediate/full_dataset_cleaned_02_nn.csv"
MODEL_OUTPUT_PATH = "models/xgboost/"
BEST_MODEL_FILENAME = "xgb_model_tree.pkl"
FEATURES_FILENAME = "selected_features_tree.txt"
METRICS_JSON = "metrics.json"
S3_MODEL_KEY = "models/xgboost/xgb_model_tree.pkl"

LEAKAGE_COLUMNS = [
    "total_rec_late_fee", "total_rec_prncp", "out_prncp", "last_pymnt_amnt", "last_pymnt_d", "funded_amnt_inv",
    "funded_amnt", "out_prncp_inv", "total_pymnt", "total_pymnt_inv", "last_pymnt_d_days",
    "last_credit_pull_d_days", "issue_d_days", "total_rec_int",
]

DEPLOYED_FEATURES = [
    "loan_amnt", "term", "installment", "fico_range_low", "last_fico_range_high", "open_il_12m", "open_il_24m",
    "max_bal_bc", "num_rev_accts", "pub_rec_bankruptcies", "emp_length_num", "earliest_cr_line_days", "grade_E",
    "home_ownership_MORTGAGE", "verification_status_Verified", "application_type_Joint App",
    "hardship_status_BROKEN", "hardship_status_COMPLETE", "hardship_status_COMPLETED",
    "hardship_status_No Hardship",
]

SEARCH_SPACE: dict[str, list] = {
    "n_estimators": [100, 200, 300],
    "max_depth": [3, 5, 7, 9],
    "learning_rate": [0.01, 0.05, 0.1],
    "subsample": [0.8, 1.0],
    "colsample_bytree": [0.5, 0.8, 1.0],
    "gamma": [0, 1, 5],
}


@dataclass
class PrepConfig:
    bucket: str = BUCKET_NAME
    null_col_threshold_pct: float = 70.0        # clean_data.py:130
    row_nan_limit: int = 20                     # feature_engineering.py:66 (thresh = ncols - 20)
    preset: str = "script"                      # "script" (clean_data.py) or "notebook" (01_data_cleaning)
    reference_date: str | None = None           # pin datetime.today() for earliest_cr_line_days
    device: str | None = None


@dataclass
class TrainConfig:
    bucket: str = BUCKET_NAME
    input_key: str = CLEAN_DATA_KEY_TREE
    output_path: str = MODEL_OUTPUT_PATH
    test_size: float = 0.2                      # model_tree_train_test.py:95
    split_random_state: int = 22
    rfe_n_features: int = 20                    # :117
    rfe_step: int = 1
    rfe_random_state: int = 42
    search_n_iter: int = 20                     # :149
    search_cv_folds: int = 3
    search_random_state: int = 22
    base_random_state: int = 78
    search_space: dict[str, list] = field(default_factory=lambda: dict(SEARCH_SPACE))
    device: str | None = None
    fits_in_parallel: int | None = None         # task-parallel fits across GPUs (None = all visible)


@dataclass
class ServeConfig:
    model_path: str = "models/xgb_model_tree.pkl"
    s3_bucket: str = BUCKET_NAME
    s3_model_key: str = S3_MODEL_KEY
    source: str = "local"                       # "local" or "s3"
    host: str = "0.0.0.0"
    port: int = 8000
    max_batch: int = 512
    max_wait_ms: float = 1.0
    device: str | None = None
    use_graphs: bool = True
    scorer_socket: str | None = None            # set: score through serve/scorer.py (multi-worker)


def _coerce(v: str, typ: Any):
    if typ in (int, "int"):
        return int(v)
    if typ in (float, "float"):
        return float(v)
    if typ in (bool, "bool"):
        return v.lower() in ("1", "true", "yes")
    return v


def from_env(cls, prefix: str = "COBALT_"):
    """Instantiate ``cls`` with overrides from environment variables ``<prefix><FIELD>``."""
    kw = {}
    for f in dataclasses.fields(cls):
        key = prefix + f.name.upper()
        if key in os.environ:
            t = f.type if not isinstance(f.type, str) else f.type.split("|")[0].strip()
            kw[f.name] = _coerce(os.environ[key], t)
    return cls(**kw)


def load_yaml(cls, path: str | Path):
    import yaml

    data = yaml.safe_load(Path(path).read_text()) or {}
    names = {f.name for f in dataclasses.fields(cls)}
    return cls(**{k: v for k, v in data.items() if k in names})
