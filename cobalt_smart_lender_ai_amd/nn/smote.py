"""SMOTE oversampling (K29) and MinMaxScaler (K30) for the NN challenger.

Reference: ``SMOTE(random_state=123).fit_resample(X_train, y_train)`` then ``MinMaxScaler`` fit on
the resampled rows (notebooks/04_model_training.ipynb cell 38). imblearn is not installed here; this
re-implements its documented algorithm and random-number sequence:

* per minority class: k+1 nearest neighbours of every class row among the class rows, first
  column (the row itself) dropped;
* ``rs = RandomState(random_state)``; ``idx = rs.randint(0, n_class*k, n_new)``;
  ``steps = rs.uniform(size=n_new)``; ``rows, cols = divmod(idx, k)``;
  ``new = X[rows] + steps * (X[nn[rows, cols]] - X[rows])``;
* output = original rows followed by the synthetic rows of each class, in class order.

The neighbour search runs on the GPU (``csrc/knn.hip``: fp32 MFMA distance tiles + register
top-k), on CPU with scikit-learn's NearestNeighbors. Parity with imblearn itself is unpinned (not
importable); the algorithm is tested against a scikit-learn oracle.
"""
from __future__ import annotations

import ctypes
import json

import numpy as np
import torch

from .. import _native

_native.register("cobalt_knn", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p])
_native.register("cobalt_smote_interp", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p])
_KNN_K = (1, 2, 3, 4, 5, 6, 7, 8, 11, 16)


def _device(device) -> torch.device:
    if device is not None:
        return torch.device(device)
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def kneighbors(Q: np.ndarray, R: np.ndarray, k: int, device=None) -> tuple[np.ndarray, np.ndarray]:
    """Indices [nq, k] and Euclidean distances of the k nearest rows of R for every row of Q,
    ordered by (distance, index)."""
    dev = _device(device)
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    R = np.ascontiguousarray(R, dtype=np.float32)
    if dev.type == "cuda":
        if k not in _KNN_K:
            raise ValueError(f"k must be one of {_KNN_K}")
        Qd, Rd = torch.as_tensor(Q, device=dev), torch.as_tensor(R, device=dev)
        idx = torch.empty((Q.shape[0], k), dtype=torch.int32, device=dev)
        dist = torch.empty((Q.shape[0], k), dtype=torch.float32, device=dev)
        rc = _native.lib().cobalt_knn(Qd.data_ptr(), Q.shape[0], Rd.data_ptr(), R.shape[0], Q.shape[1], k,
                                      idx.data_ptr(), dist.data_ptr(), _native.stream_handle())
        _native.check(rc, "cobalt_knn")
        return idx.cpu().numpy().astype(np.int64), np.sqrt(dist.cpu().numpy())
    from sklearn.neighbors import NearestNeighbors

    nn = NearestNeighbors(n_neighbors=k).fit(R.astype(np.float64))
    d, i = nn.kneighbors(Q.astype(np.float64))
    return i, d


class SMOTE:
    def __init__(self, sampling_strategy="auto", random_state=None, k_neighbors: int = 5, device=None):
        if sampling_strategy != "auto":
            raise NotImplementedError("only sampling_strategy='auto' (the reference's setting)")
        self.random_state = random_state
        self.k_neighbors = k_neighbors
        self.device = device

    def fit_resample(self, X, y):
        cols = getattr(X, "columns", None)
        Xn = np.asarray(X.to_numpy() if hasattr(X, "to_numpy") else X, dtype=np.float64)
        yn = np.asarray(y.to_numpy() if hasattr(y, "to_numpy") else y)
        classes, counts = np.unique(yn, return_counts=True)
        n_max = counts.max()
        outs_X, outs_y = [Xn], [yn]
        self.sampling_strategy_ = {c: int(n_max - n) for c, n in zip(classes, counts) if n < n_max}
        for cls, n_new in self.sampling_strategy_.items():
            if n_new == 0:
                continue
            Xc = Xn[yn == cls]
            k = self.k_neighbors
            nn, _ = kneighbors(Xc, Xc, k + 1, self.device)
            nn = nn[:, 1:]
            rs = np.random.RandomState(self.random_state) if not isinstance(self.random_state, np.random.RandomState) \
                else self.random_state
            idx = rs.randint(low=0, high=nn.size, size=n_new)
            steps = rs.uniform(size=n_new)
            rows = np.floor_divide(idx, nn.shape[1])
            cidx = np.mod(idx, nn.shape[1])
            outs_X.append(self._interp(Xc, nn, rows, cidx, steps))
            outs_y.append(np.full(n_new, cls, dtype=yn.dtype))
        Xr = np.vstack(outs_X)
        yr = np.hstack(outs_y)
        if cols is not None:
            import pandas as pd

            Xr = pd.DataFrame(Xr, columns=cols)
            yr = pd.Series(yr, name=getattr(y, "name", None))
        return Xr, yr

    def _interp(self, Xc, nn, rows, cols, steps) -> np.ndarray:
        dev = _device(self.device)
        if dev.type == "cuda":
            F = Xc.shape[1]
            Xd = torch.as_tensor(np.ascontiguousarray(Xc), device=dev)
            nnd = torch.as_tensor(nn.astype(np.int32), device=dev).contiguous()
            rd = torch.as_tensor(rows.astype(np.int64), device=dev)
            cd = torch.as_tensor(cols.astype(np.int64), device=dev)
            sd = torch.as_tensor(steps.astype(np.float64), device=dev)
            out = torch.empty((len(rows), F), dtype=torch.float64, device=dev)
            rc = _native.lib().cobalt_smote_interp(Xd.data_ptr(), F, nnd.data_ptr(), nn.shape[1], rd.data_ptr(),
                                                   cd.data_ptr(), sd.data_ptr(), len(rows), out.data_ptr(),
                                                   _native.stream_handle())
            _native.check(rc, "cobalt_smote_interp")
            return out.cpu().numpy()
        return Xc[rows] + steps[:, None] * (Xc[nn[rows, cols]] - Xc[rows])


class MinMaxScaler:
    """Column min/max scaling to [0, 1] (sklearn semantics: constant columns map to 0; NaN ignored
    in the fit and passed through)."""

    def fit(self, X):
        Xn = np.asarray(X.to_numpy() if hasattr(X, "to_numpy") else X, dtype=np.float64)
        self.data_min_ = np.nanmin(Xn, axis=0)
        self.data_max_ = np.nanmax(Xn, axis=0)
        rng = self.data_max_ - self.data_min_
        rng[rng == 0.0] = 1.0
        self.scale_ = 1.0 / rng
        self.min_ = -self.data_min_ * self.scale_
        self.n_features_in_ = Xn.shape[1]
        if hasattr(X, "columns"):
            self.feature_names_in_ = np.asarray(X.columns, dtype=object)
        return self

    def transform(self, X):
        Xn = np.asarray(X.to_numpy() if hasattr(X, "to_numpy") else X, dtype=np.float64)
        return Xn * self.scale_ + self.min_

    def fit_transform(self, X):
        return self.fit(X).transform(X)

    def inverse_transform(self, X):
        return (np.asarray(X, dtype=np.float64) - self.min_) / self.scale_

    def to_json(self) -> str:
        return json.dumps({k: getattr(self, k).tolist() for k in ("data_min_", "data_max_", "scale_", "min_")}
                          | {"feature_names_in_": list(getattr(self, "feature_names_in_", []))})

    @classmethod
    def from_json(cls, s: str) -> "MinMaxScaler":
        d = json.loads(s)
        m = cls()
        for k in ("data_min_", "data_max_", "scale_", "min_"):
            setattr(m, k, np.asarray(d[k], dtype=np.float64))
        if d.get("feature_names_in_"):
            m.feature_names_in_ = np.asarray(d["feature_names_in_"], dtype=object)
        m.n_features_in_ = len(m.scale_)
        return m
