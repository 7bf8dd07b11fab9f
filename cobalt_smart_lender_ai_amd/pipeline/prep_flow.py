"""Data-lake stages of the preprocessing pipeline (reference: src/data_preprocessing/clean_data.py
``main`` :161-175 and feature_engineering.py ``main`` :186-204).

Stage 1  raw CSV (sample or full)  -> ``clean_data_flow``               -> cleaned CSV
Stage 2  cleaned full CSV          -> ``clean_lending_data`` + features -> tree CSV + NN CSV

``engine="device"`` (the default on a GPU) runs a stage device-resident: the CSV is parsed once
(pyarrow) into a :class:`~..prep.device_frame.DeviceFrame` in HBM, every step runs on the GPU and
only the artifact CSV goes back to the host (prep/device_prep.py; 29x the pandas path on the
2.9M x 143 export, profiles/configs/prep-full.json). ``engine="pandas"`` runs the reference-shaped
pandas path (its numeric passes still on ``device``). The store is any
:class:`~..dataio.artifacts.ArtifactStore` (local directory mirror of the bucket, or S3).
"""
from __future__ import annotations

import logging

import pandas as pd

from ..config import (CLEAN_DATA_KEY_FULL, CLEAN_DATA_KEY_NN, CLEAN_DATA_KEY_SAMPLE, CLEAN_DATA_KEY_TREE,
                      RAW_DATA_KEY_FULL, RAW_DATA_KEY_SAMPLE)
from ..dataio.artifacts import ArtifactStore
from ..prep.clean import clean_data_flow
from ..prep.features import clean_lending_data, feature_engineer_lending_data

log = logging.getLogger(__name__)


def _engine(engine: str | None, device) -> str:
    import torch

    if engine in ("device", "pandas"):
        return engine
    dev = torch.device(device) if device is not None else None
    if dev is not None:
        return "device" if dev.type == "cuda" else "pandas"
    return "device" if torch.cuda.is_available() else "pandas"


def read_table(store: ArtifactStore, key: str, device=None) -> pd.DataFrame:
    """``store.read_csv(key)`` -- parsed on the GPU when one is used (prep/csv_gpu.py: a 3.3 GB
    full-data tree CSV in well under a second instead of about a minute), then handed over as a pandas
    frame equal to ``pd.read_csv``'s (the reference job's read, model_tree_train_test.py:77): pandas'
    default float conversion is reproduced on the device (float_precision="high"); a file the device
    reader refuses (ragged rows, values pandas types as text) is read by pandas itself."""
    import torch

    dev = torch.device(device) if device is not None else (
        torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    if dev.type != "cuda":
        return store.read_csv(key)
    from ..prep.csv_gpu import CsvLayoutError
    from ..prep.device_frame import DeviceFrame

    try:
        return DeviceFrame.read_csv(store.get_bytes(key), dev, float_precision="high").to_pandas()
    except CsvLayoutError:
        return store.read_csv(key)


def _write_frame(store: ArtifactStore, dfr, key: str) -> None:
    """The artifact CSV of a device frame: formatted on the GPU (byte-identical to pandas.to_csv,
    prep/csv_gpu.frame_to_csv_bytes), pandas off the GPU."""
    from ..prep.csv_gpu import frame_to_csv_bytes

    data = frame_to_csv_bytes(dfr)
    if data is None:
        store.write_csv(dfr.to_pandas(), key)
    else:
        store.put_bytes(key, data)


def run_clean(store: ArtifactStore, use_sample: bool = True, device=None, preset: str = "script",
              engine: str | None = None):
    """Stage 1. Returns the cleaned frame (a DeviceFrame with the device engine)."""
    key_in = RAW_DATA_KEY_SAMPLE if use_sample else RAW_DATA_KEY_FULL
    key_out = CLEAN_DATA_KEY_SAMPLE if use_sample else CLEAN_DATA_KEY_FULL
    log.info("Loading %s dataset from %s", "SAMPLE" if use_sample else "FULL", key_in)
    if _engine(engine, device) == "device":
        from ..prep.device_frame import DeviceFrame
        from ..prep.device_prep import device_clean_data_flow

        out = device_clean_data_flow(DeviceFrame.read_csv(store.get_bytes(key_in), device or "cuda"), preset=preset)
        log.info("Saving cleaned data (%d rows x %d cols) to %s", *out.shape, key_out)
        _write_frame(store, out, key_out)
        return out
    df = store.read_csv(key_in)
    out = clean_data_flow(df, preset=preset, device=device)
    log.info("Saving cleaned data (%d rows x %d cols) to %s", len(out), out.shape[1], key_out)
    store.write_csv(out, key_out)
    return out


def run_features(store: ArtifactStore, device=None, reference_date=None,
                 key_in: str = CLEAN_DATA_KEY_FULL, engine: str | None = None):
    """Stage 2 + feature engineering. Returns (tree, nn) (DeviceFrames with the device engine)."""
    if _engine(engine, device) == "device":
        from ..prep.device_frame import DeviceFrame
        from ..prep.device_prep import device_clean_lending_data, device_feature_engineer

        dfr = device_clean_lending_data(DeviceFrame.read_csv(store.get_bytes(key_in), device or "cuda"),
                                        reference_date=reference_date)
        tree, nn = device_feature_engineer(dfr)
        log.info("Tree dataset %s, NN dataset %s (device-resident)", tree.shape, nn.shape)
        _write_frame(store, tree, CLEAN_DATA_KEY_TREE)
        _write_frame(store, nn, CLEAN_DATA_KEY_NN)
        return tree, nn
    df = store.read_csv(key_in)
    df_clean = clean_lending_data(df, reference_date=reference_date, device=device)
    df_tree, df_nn = feature_engineer_lending_data(df_clean, device=device)
    log.info("NaN values in tree dataset:\n%s", df_tree.isnull().sum().sort_values(ascending=False).head())
    log.info("NaN values in NN dataset:\n%s", df_nn.isnull().sum().sort_values(ascending=False).head())
    store.write_csv(df_tree, CLEAN_DATA_KEY_TREE)
    store.write_csv(df_nn, CLEAN_DATA_KEY_NN)
    return df_tree, df_nn
