"""Scoring engine: batched probability + TreeSHAP on the GPU with hipGraph-captured buckets.

The reference scores one HTTP request at a time with ``xgb_model.predict_proba`` and
``shap.TreeExplainer.shap_values`` (src/api/cobalt_fast_api.py:90-108). Here a request batch is
padded to a bucket size (1, 8, 64, 512, 4096) whose whole pipeline -- predictor kernel + TreeSHAP kernel
(+ its fixed-order chunk reduction) -- was captured once into a hipGraph (``torch.cuda.CUDAGraph``
over the library's own launches on the capture stream). Serving a batch is then: one H2D copy into
the bucket's static input (from pinned staging), one graph replay, one D2H copy. Larger batches are split into bucket
sized pieces. On a CPU-only host the engine runs the NumPy reference path instead.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass

import numpy as np
import torch

from ..models.booster import Booster, predict_margin_host, sigmoid32, treeshap_host

BUCKETS = (1, 8, 64, 512, 4096)


@dataclass
class _Bucket:
    size: int
    x: torch.Tensor          # [B, F] float32 (static graph input)
    prob: torch.Tensor       # [B] float32
    phi: torch.Tensor | None  # [B, F] float64
    x_pin: torch.Tensor | None = None     # pinned host staging of x / prob / phi (async copies)
    prob_pin: torch.Tensor | None = None
    phi_pin: torch.Tensor | None = None
    graph_prob: torch.cuda.CUDAGraph | None = None
    graph_full: torch.cuda.CUDAGraph | None = None


class ScoringEngine:
    def __init__(self, booster: Booster, device: str | torch.device | None = None, use_graphs: bool = True,
                 buckets: tuple[int, ...] = BUCKETS):
        self.booster = booster
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.F = booster.num_feature
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self._lock = threading.Lock()
        self._buckets: dict[int, _Bucket] = {}
        self.expected_value = float(booster.expected_value())
        if self.device.type == "cuda":
            from ..ops import predict_ops

            self._ops = predict_ops
            predict_ops.gpu_forest(booster, self.device, None, with_shap=True)  # pack once
            self._stream = torch.cuda.Stream(self.device)
            for b in buckets:
                self._buckets[b] = self._make_bucket(b)

    # ------------------------------------------------------------------ graph capture
    def _run_prob(self, bk: _Bucket) -> None:
        self._ops.predict_gpu(self.booster, bk.x, None, out_prob=bk.prob)

    def _run_full(self, bk: _Bucket) -> None:
        self._ops.predict_gpu(self.booster, bk.x, None, out_prob=bk.prob)
        self._ops.treeshap_gpu(self.booster, bk.x, bk.phi)

    def _make_bucket(self, size: int) -> _Bucket:
        dev = self.device
        bk = _Bucket(size=size, x=torch.zeros((size, self.F), dtype=torch.float32, device=dev),
                     prob=torch.zeros(size, dtype=torch.float32, device=dev),
                     phi=torch.zeros((size, self.F), dtype=torch.float64, device=dev),
                     x_pin=torch.zeros((size, self.F), dtype=torch.float32).pin_memory(),
                     prob_pin=torch.zeros(size, dtype=torch.float32).pin_memory(),
                     phi_pin=torch.zeros((size, self.F), dtype=torch.float64).pin_memory())
        if not self.use_graphs:
            return bk
        with torch.cuda.device(dev), torch.cuda.stream(self._stream):
            # warm up outside capture (loads kernels, sets LDS attributes)
            self._run_full(bk)
            torch.cuda.synchronize(dev)
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=self._stream):
                self._run_prob(bk)
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, stream=self._stream):
                self._run_full(bk)
        bk.graph_prob, bk.graph_full = g1, g2
        return bk

    # ---------------------------------------------------------------------- scoring
    def _bucket_for(self, n: int) -> _Bucket:
        for b in sorted(self._buckets):
            if n <= b:
                return self._buckets[b]
        return self._buckets[max(self._buckets)]

    def score(self, X: np.ndarray, with_shap: bool = True) -> tuple[np.ndarray, np.ndarray | None]:
        """Return (prob_default [N] float32, shap [N, F] float64 or None)."""
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float32))
        if X.ndim != 2 or X.shape[1] != self.F:
            raise ValueError(f"expected [N, {self.F}] features, got {X.shape}")
        N = X.shape[0]
        if self.device.type != "cuda":
            p = sigmoid32(predict_margin_host(self.booster, X))
            return p, (treeshap_host(self.booster, X) if with_shap else None)
        probs = np.empty(N, dtype=np.float32)
        phis = np.empty((N, self.F), dtype=np.float64) if with_shap else None
        with self._lock, torch.cuda.device(self.device), torch.cuda.stream(self._stream):
            s = 0
            while s < N:
                bk = self._bucket_for(N - s)
                e = min(N, s + bk.size)
                n = e - s
                xp = bk.x_pin.numpy()
                xp[:n] = X[s:e]
                if n < bk.size:
                    xp[n:] = 0.0
                bk.x.copy_(bk.x_pin, non_blocking=True)
                if self.use_graphs:
                    (bk.graph_full if with_shap else bk.graph_prob).replay()
                elif with_shap:
                    self._run_full(bk)
                else:
                    self._run_prob(bk)
                bk.prob_pin[:n].copy_(bk.prob[:n], non_blocking=True)
                if with_shap:
                    bk.phi_pin[:n].copy_(bk.phi[:n], non_blocking=True)
                self._stream.synchronize()
                probs[s:e] = bk.prob_pin.numpy()[:n]
                if with_shap:
                    phis[s:e] = bk.phi_pin.numpy()[:n]
                s = e
            self._stream.synchronize()
        return probs, phis

    def predict_proba(self, X: np.ndarray) -> np.ndarray:
        return self.score(X, with_shap=False)[0]
