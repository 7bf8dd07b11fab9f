"""Data-lake stages of the preprocessing pipeline (reference: src/data_preprocessing/clean_data.py
``main`` :161-175 and feature_engineering.py ``main`` :186-204).

Stage 1  raw CSV (sample or full)  -> ``clean_data_flow``               -> cleaned CSV
Stage 2  cleaned full CSV          -> ``clean_lending_data`` + features -> tree CSV + NN CSV

Both stages run their numeric work on the active device (``prep_ops``); the store is any
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


def run_clean(store: ArtifactStore, use_sample: bool = True, device=None, preset: str = "script") -> pd.DataFrame:
    key_in = RAW_DATA_KEY_SAMPLE if use_sample else RAW_DATA_KEY_FULL
    key_out = CLEAN_DATA_KEY_SAMPLE if use_sample else CLEAN_DATA_KEY_FULL
    log.info("Loading %s dataset from %s", "SAMPLE" if use_sample else "FULL", key_in)
    df = store.read_csv(key_in)
    out = clean_data_flow(df, preset=preset, device=device)
    log.info("Saving cleaned data (%d rows x %d cols) to %s", len(out), out.shape[1], key_out)
    store.write_csv(out, key_out)
    return out


def run_features(store: ArtifactStore, device=None, reference_date=None,
                 key_in: str = CLEAN_DATA_KEY_FULL) -> tuple[pd.DataFrame, pd.DataFrame]:
    df = store.read_csv(key_in)
    df_clean = clean_lending_data(df, reference_date=reference_date, device=device)
    df_tree, df_nn = feature_engineer_lending_data(df_clean, device=device)
    log.info("NaN values in tree dataset:\n%s", df_tree.isnull().sum().sort_values(ascending=False).head())
    log.info("NaN values in NN dataset:\n%s", df_nn.isnull().sum().sort_values(ascending=False).head())
    store.write_csv(df_tree, CLEAN_DATA_KEY_TREE)
    store.write_csv(df_nn, CLEAN_DATA_KEY_NN)
    return df_tree, df_nn
