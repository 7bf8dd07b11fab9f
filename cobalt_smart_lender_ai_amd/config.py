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


# ------------------------------------------------------------------------------------------------
# Environment knobs: EVERY ``COBALT_*`` variable the package reads, in one documented registry.
# scope "native" = read by the HIP/C++ library through csrc/knobs.cpp (knob_int / knob_str, the only
# getenv calls of csrc/); "python" = read by the Python package; "test" = fault injection and test-only
# switches. tests/test_knobs.py checks that the native registry and every COBALT_* name in the source
# tree appear here. Defaults are the measured-best settings (docs/PERF.md); knobs of rejected
# experiments are deleted together with their code.
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Knob:
    default: str
    scope: str
    doc: str


KNOBS: dict[str, Knob] = {
    # -- trainer tuning / diagnostics (native) --
    "COBALT_STAMPS": Knob("", "native", "file: in-kernel launch / probe timestamps of sampled trees (scripts/stamp_summary.py)"),
    "COBALT_HIST_ABLATE": Knob("0", "native", "timing-only ablations of the histogram / partition / root passes (wrong models)"),
    "COBALT_HIST_CHUNK": Knob("auto", "native", "rows per histogram work item at levels >= 1 (~n/1536, 1024..4096)"),
    "COBALT_HIST_CHUNK0": Knob("auto", "native", "rows per root histogram item when the root pass is not fused"),
    "COBALT_ROOT_CHUNK": Knob("auto", "native", "rows per item of the fused gradient + root-histogram pass (whole rounds of 2 blocks per CU)"),
    "COBALT_PART_CHUNK": Knob("auto", "native", "rows per partition item (4096 while a level fits one block per CU, else 8192; <= 8192)"),
    "COBALT_EVAL_FG": Knob("auto", "native", "features per split-evaluation group (0 = one block per node; 8 above 32 features)"),
    "COBALT_EVAL_PART": Knob("1", "native", "split evaluation fused into the partition pass while a level fits one block per CU (0 off, 2 forced)"),
    "COBALT_HIST_PAIR": Knob("1", "native", "lane-pair record gathers in the histogram levels (16 < F <= 24)"),
    "COBALT_MAX_COPY_SHIFT": Knob("4", "native", "log2 of the per-lane LDS histogram copies of a low-cardinality feature (0..6)"),
    "COBALT_WT": Knob("auto", "native", "write-through stores: bit 0 histogram slabs, bit 1 partition row ids, bit 2 the root pass's (g, h) (7 below 4M rows, else 5)"),
    "COBALT_MARGIN_IN_RECORD": Knob("1", "native", "binary labels, <= 20 features, >= 4M rows: the root pass keeps every row's margin in its 32-byte record (0 off, 2 at any row count)"),
    "COBALT_PART_POS": Knob("1", "native", "row partition in position-ordered blocks whose row-id loads need no plan (0: node-ordered items)"),
    "COBALT_BIN_SCALAR": Knob("", "native", "force the generic binning kernel for 32-byte records (tests)"),
    "COBALT_PRED_WALK": Knob("4", "native", "trees walked at once per predictor thread (2 / 4 / 8)"),
    # -- data parallelism --
    "COBALT_IPC_FUSED": Knob("1", "native", "IPC exchange fused into the split evaluation (0: separate exchange kernel + fused eval/partition)"),
    "COBALT_DP_OWNER": Knob("1", "native", "node ownership on the three deepest levels over the fused IPC exchange"),
    "COBALT_EVAL_BLOCKS": Knob("1", "native", "over the fused IPC exchange: the fused evaluation + partition pass with one evaluator block per node (0: k_eval + k_partition)"),
    "COBALT_CU_BUDGET": Knob("", "native", "CUs of this rank's CU-masked stream (set by parallel/cumask.py)"),
    "COBALT_DP_TRANSPORT": Knob("auto", "python", "native communicator: auto (IPC within a node), ipc or rccl"),
    "COBALT_DIST_BACKEND": Knob("auto", "python", "torch.distributed backend override (gloo for ranks sharing one GPU)"),
    "COBALT_DIST_NATIVE": Knob("auto", "python", "create the trainer's native communicator with a gloo bootstrap (1)"),
    "COBALT_IPC_SLOT_MB": Knob("64", "python", "IPC send-slot capacity per rank"),
    "COBALT_IPC_TIMEOUT_S": Knob("120", "python", "in-kernel exchange deadline before the group fails on every rank"),
    "COBALT_IPC_CONNECT_TIMEOUT_S": Knob("30", "python", "deadline of the IPC connect self-test"),
    "COBALT_COLLECTIVE_TIMEOUT_S": Knob("1800", "python", "host watchdog deadline for one enqueued segment of trees"),
    "COBALT_SHARED_CU_MASK": Knob("auto", "python", "CU-masked streams for ranks sharing one GPU (default for 2-8 ranks)"),
    "COBALT_CU_MASK_LAYOUT": Knob("blocked", "python", "CU masks of ranks sharing one GPU: blocked (contiguous bits, every XCC covered) or interleaved"),
    "COBALT_TEST_PLACEMENT": Knob("0", "test", "parallel/dp_check.py: record the XCCs / CUs a rank's masked stream runs on"),
    "COBALT_BENCH_SHARED_DEVICE": Knob("0", "python", "bench.py: every rank on cuda:0 (the 1-GPU multi-rank rehearsal)"),
    # -- trainer / serving (python) --
    "COBALT_LABEL_IN_RECORD": Knob("1", "python", "0/1 labels ride in the row records' padding (weights derived from them)"),
    "COBALT_TRAINER_CACHE": Knob("1", "python", "keep one trainer context per process for back-to-back fits of the same shapes"),
    "COBALT_SEARCH_STREAMS": Knob("4", "python", "HIP streams of the randomized search's concurrent fits"),
    "COBALT_PRED_TILE": Knob("2048", "python", "tree nodes per LDS tile of the GPU predictor"),
    "COBALT_SK_TIMING": Knob("0", "python", "per-stage times of the device quantile sketch to stderr"),
    "COBALT_NATIVE_LIB": Knob("", "python", "load this native library instead of _lib/libcobalt_hip.so (A/B builds, host-ASan build)"),
    "COBALT_OFFLOAD_ARCH": Knob("gfx950", "python", "offload architecture of the native build"),
    "COBALT_RCCL_LIB": Knob("auto", "python", "path of librccl for the native RCCL communicator"),
    "COBALT_ARTIFACT_URI": Knob("data-lake", "python", "artifact store: a local directory or s3://bucket"),
    "COBALT_MODEL_PATH": Knob("models/xgb_model_tree.pkl", "python", "model the API serves"),
    "COBALT_SOURCE": Knob("local", "python", "model source of the API (s3 with boto3)"),
    "COBALT_SCORER_SOCKET": Knob("", "python", "unix socket of the GPU scorer process behind `serve --workers N`"),
    "COBALT_SERVE_WORKERS": Knob("1", "python", "HTTP worker processes of `serve`"),
    # -- fault injection / tests --
    "COBALT_FAULT_AFTER_TREES": Knob("0", "test", "a rank fails (or stalls, with COBALT_FAULT_STALL_S) after this many trees"),
    "COBALT_FAULT_RANK": Knob("-1", "test", "the rank COBALT_FAULT_AFTER_TREES applies to (-1: every rank)"),
    "COBALT_FAULT_STALL_S": Knob("0", "test", "the faulting rank stalls this long once instead of dying"),
    "COBALT_FAULT_CORRUPT_RANK": Knob("-1", "test", "this rank perturbs a tree's root totals (replica-divergence test)"),
    "COBALT_FAULT_CORRUPT_TREE": Knob("1", "test", "the tree COBALT_FAULT_CORRUPT_RANK perturbs"),
    "COBALT_REFERENCE_PKL": Knob("", "test", "path of the reference's shipped model for the golden tests"),
    "COBALT_REFERENCE_UI": Knob("", "test", "path of the reference Streamlit script for the UI replay test"),
    "COBALT_RECORD_UI": Knob("", "test", "record the UI replay's exchanges"),
}


def knob(name: str, default: str | None = None) -> str | None:
    """The value of a registered ``COBALT_*`` knob (``default`` when unset)."""
    if name not in KNOBS:
        raise KeyError(f"{name} is not a registered knob (config.KNOBS)")
    return os.environ.get(name, default)
