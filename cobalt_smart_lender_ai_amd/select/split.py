"""Row splits with index parity to scikit-learn (K26).

The reference splits with ``train_test_split(test_size=0.2, random_state=22)`` (not stratified,
src/model_train_test/model_tree_train_test.py:95-97) and cross-validates with
``StratifiedKFold(3)`` (no shuffle, :153). Indices are produced host-side with scikit-learn's own
generators so a given ``random_state`` selects exactly the reference's rows; only the index arrays
travel to the device.
"""
from __future__ import annotations

import numpy as np


def train_test_split_indices(n: int, test_size: float | int = 0.2, random_state: int | None = 22,
                             shuffle: bool = True, stratify=None) -> tuple[np.ndarray, np.ndarray]:
    from sklearn.model_selection import train_test_split

    idx = np.arange(n)
    tr, te = train_test_split(idx, test_size=test_size, random_state=random_state, shuffle=shuffle,
                              stratify=stratify)
    return np.asarray(tr), np.asarray(te)


def stratified_kfold_indices(y, n_splits: int = 3, shuffle: bool = False,
                             random_state: int | None = None) -> list[tuple[np.ndarray, np.ndarray]]:
    from sklearn.model_selection import StratifiedKFold

    y = np.asarray(y)
    skf = StratifiedKFold(n_splits=n_splits, shuffle=shuffle, random_state=random_state if shuffle else None)
    return [(np.asarray(a), np.asarray(b)) for a, b in skf.split(np.zeros(len(y)), y)]
