"""Device-resident preprocessing (prep/device_frame.py, prep/device_prep.py) against the pandas path
(prep/clean.py + prep/features.py, the reference's semantics: src/data_preprocessing/clean_data.py:87-158,
feature_engineering.py:44-184). The frame runs on CPU tensors here and on the GPU in
tests/test_gpu_prep.py (>= 1M rows)."""
import numpy as np
import pandas as pd
import pytest

from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
from cobalt_smart_lender_ai_amd.prep import device_prep as dp
from cobalt_smart_lender_ai_amd.prep.clean import clean_data_flow
from cobalt_smart_lender_ai_amd.prep.features import clean_lending_data, feature_engineer_lending_data

REF_DATE = "2025-07-04"


def assert_frames_equal(a: pd.DataFrame, b: pd.DataFrame, rtol: float = 1e-15) -> None:
    """Same columns in the same order, same rows, same values (NaN == NaN; floats to a few ulp),
    compatible dtypes."""
    assert list(a.columns) == list(b.columns)
    assert len(a) == len(b)
    for c in a.columns:
        x, y = a[c], b[c]
        if x.dtype == object or y.dtype == object:
            xs = x.astype(object).where(x.notna(), None).tolist()
            ys = y.astype(object).where(y.notna(), None).tolist()
            assert xs == ys, c
            continue
        assert (x.dtype == bool) == (y.dtype == bool), (c, x.dtype, y.dtype)
        assert np.issubdtype(x.dtype, np.integer) == np.issubdtype(y.dtype, np.integer), (c, x.dtype, y.dtype)
        xv, yv = x.to_numpy(np.float64), y.to_numpy(np.float64)
        if np.issubdtype(x.dtype, np.floating) or np.issubdtype(y.dtype, np.floating):
            # device libm log1p may differ from glibc's in the last bit: a few ulp, no more
            assert np.allclose(xv, yv, rtol=rtol, atol=0.0, equal_nan=True), c
        else:
            assert np.array_equal(xv, yv, equal_nan=True), c


def pandas_path(csv, preset="script"):
    raw = pd.read_csv(csv, low_memory=False, float_precision="round_trip")
    c1 = clean_data_flow(raw, preset=preset, device="cpu")
    c2 = clean_lending_data(c1, reference_date=REF_DATE, device="cpu", preset=preset)
    tree, nn = feature_engineer_lending_data(c2, device="cpu")
    return c1, c2, tree, nn


def device_path(csv, device, preset="script"):
    r = dp.run_device_prep(csv, device=device, reference_date=REF_DATE, preset=preset)
    return r["clean"].to_pandas(), r["stage2"].to_pandas(), r["tree"].to_pandas(), r["nn"].to_pandas()


@pytest.mark.parametrize("preset", ["script", "notebook"])
def test_device_frame_pipeline_equals_pandas_path(tmp_path, preset):
    raw = make_raw_lendingclub(20_000, seed=4, n_dups=5)
    csv = tmp_path / "raw.csv"
    raw.to_csv(csv, index=False)
    for got, ref in zip(device_path(str(csv), "cpu", preset), pandas_path(csv, preset)):
        assert_frames_equal(got, ref)


def test_tree_training_matrix(tmp_path):
    raw = make_raw_lendingclub(5_000, seed=5)
    csv = tmp_path / "raw.csv"
    raw.to_csv(csv, index=False)
    r = dp.run_device_prep(str(csv), device="cpu", reference_date=REF_DATE)
    X, y, names = dp.tree_training_matrix(r["tree"], drop=["id"])
    ref = r["tree"].to_pandas()
    ref = ref[ref["loan_default"].notna()]
    assert "loan_default" not in names and "id" not in names
    assert np.array_equal(X.numpy(), ref[names].to_numpy(np.float32), equal_nan=True)
    assert np.array_equal(y.numpy(), ref["loan_default"].to_numpy(np.float32))


def test_device_frame_pipeline_143_columns(tmp_path):
    """The full export's width (143 columns: mostly-null joint / hardship / settlement fields that
    stage 1 drops, LC numeric columns that the log transform covers)."""
    raw = make_raw_lendingclub(8_000, seed=6, n_cols=143)
    assert raw.shape[1] == 143
    csv = tmp_path / "raw.csv"
    raw.to_csv(csv, index=False)
    for got, ref in zip(device_path(str(csv), "cpu"), pandas_path(csv)):
        assert_frames_equal(got, ref)


def test_prep_flow_device_engine_writes_the_pandas_artifacts(tmp_path):
    """Both CLI stages with the device-resident engine (on CPU tensors here) write the same CSV
    artifacts as the pandas engine."""
    from cobalt_smart_lender_ai_amd.config import CLEAN_DATA_KEY_FULL, CLEAN_DATA_KEY_NN, CLEAN_DATA_KEY_TREE, \
        RAW_DATA_KEY_FULL
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore
    from cobalt_smart_lender_ai_amd.pipeline.prep_flow import run_clean, run_features

    raw = make_raw_lendingclub(6_000, seed=9)
    outs = {}
    for engine in ("pandas", "device"):
        st = LocalStore(tmp_path / engine)
        st.write_csv(raw, RAW_DATA_KEY_FULL)
        run_clean(st, use_sample=False, device="cpu", engine=engine)
        run_features(st, device="cpu", reference_date=REF_DATE, engine=engine)
        outs[engine] = [st.read_csv(k) for k in (CLEAN_DATA_KEY_FULL, CLEAN_DATA_KEY_TREE, CLEAN_DATA_KEY_NN)]
    # pandas.read_csv's default float parser is not correctly rounded (the device engine's pyarrow
    # reader is), so CSV round trips of the stage-1 artifact may differ in the last few bits
    for a, b in zip(outs["device"], outs["pandas"]):
        assert_frames_equal(a, b, rtol=1e-14)
