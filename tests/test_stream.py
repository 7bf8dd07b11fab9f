"""Streamed ingestion (models/stream.py): a chunked fit equals the in-core fit of the same rows."""
import numpy as np
import pandas as pd
import pytest
import torch

from cobalt_smart_lender_ai_amd.dataio import synth
from cobalt_smart_lender_ai_amd.models import gbdt, stream

PARAMS = dict(n_estimators=4, max_depth=4, learning_rate=0.3, gamma=0.5, subsample=0.9, random_state=2)


def _data(n, seed=4):
    X, y = synth.make_lendingclub(n, seed=seed)
    return X.numpy(), y.numpy()


def test_stream_equals_in_core_host():
    X, y = _data(6000)
    p = gbdt.GBDTParams(sketch_rows=1000, **PARAMS)  # sampled sketch: the stride crosses chunk borders
    ref = gbdt.train(X, y, p, device="cpu").save_raw("ubj")
    src = stream.array_chunks(X, y, 777)
    out = stream.train_stream(src, p, device="cpu").save_raw("ubj")
    assert out == ref
    # row count given up front (two passes instead of three)
    assert stream.train_stream(src, p, n_rows=len(X), device="cpu").save_raw("ubj") == ref


def test_stream_csv_source(tmp_path):
    X, y = _data(3000, seed=6)
    cols = list(synth.FEATURES)
    df = pd.DataFrame(X, columns=cols)
    df["loan_default"] = y
    path = tmp_path / "rows.csv.gz"
    df.to_csv(path, index=False, compression="gzip")
    p = gbdt.GBDTParams(**PARAMS)
    src = stream.csv_chunks(str(path), cols, "loan_default", rows_per_chunk=512)
    out = stream.train_stream(src, p, device="cpu")
    back = pd.read_csv(path)
    ref = gbdt.train(back[cols].to_numpy(np.float32), back["loan_default"].to_numpy(np.float32), p, device="cpu")
    assert out.save_raw("ubj") == ref.save_raw("ubj")


def test_stream_row_count_mismatch():
    X, y = _data(1000)
    with pytest.raises(ValueError):
        stream.bin_stream(stream.array_chunks(X, y, 300), n_rows=999, device="cpu")


@pytest.mark.gpu
def test_stream_equals_in_core_gpu():
    X, y = _data(300_000, seed=8)
    p = gbdt.GBDTParams(n_estimators=6, max_depth=6, learning_rate=0.2, random_state=1, sketch_rows=50_000)
    ref = gbdt.train(X, y, p, device="cuda").save_raw("ubj")
    out = stream.train_stream(stream.array_chunks(X, y, 65_537), p, device="cuda").save_raw("ubj")
    assert out == ref
