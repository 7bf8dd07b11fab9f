"""Streamed ("external memory") ingestion for GBDT training.

The reference reads the whole CSV into pandas RAM (``clean_data.py:44-67``,
``model_tree_train_test.py:37-46``). Here a training set can arrive as a re-iterable stream of row
chunks (CSV pages, Arrow batches, NumPy shards) and only its quantised form is ever resident:

* pass 1 (only when the row count is not given) counts rows;
* pass 2 keeps the rows whose GLOBAL index is a multiple of the sketch stride -- exactly the sample
  the in-core path draws -- so the quantile cuts (K12) and therefore the trees are identical to
  an in-core fit of the same rows. On a GPU with every row sketched (the default, SKETCH_AUTO) that
  sample only places the device sketch's bucket boundaries, and two more passes (bucket histogram,
  candidate gather: ``sketch.stream_exact_cuts``) give the all-row cuts of the in-core fit;
* pass 3 uploads each chunk through a pair of pinned staging buffers (the host parses chunk k+1
  while the device copies and bins chunk k) and quantises it in place into the preallocated row
  records + feature-major bins (``cobalt_bin_matrix_ld``, K13): 32 B + F B per row on the device
  instead of 4F B of fp32 (100M x 20 features: 5.2 GB of the 288 GB HBM), no per-chunk copies.
"""
from __future__ import annotations

import time
from typing import Callable, Iterable, Iterator

import numpy as np
import torch

from . import sketch
from .gbdt import SKETCH_AUTO, SKETCH_SAMPLE_ROWS, BinnedData, GBDTParams, _resolve_device, train_binned

Chunk = tuple  # (X [n, F] float32, y [n])
ChunkSource = Callable[[], Iterable[Chunk]]


def array_chunks(X, y, rows_per_chunk: int) -> ChunkSource:
    """A chunk source over in-memory arrays (tests, NumPy memory maps)."""
    def gen() -> Iterator[Chunk]:
        for s in range(0, len(X), rows_per_chunk):
            yield X[s:s + rows_per_chunk], y[s:s + rows_per_chunk]
    return gen


def csv_chunks(path: str, feature_columns: list[str], label_column: str, rows_per_chunk: int = 1 << 20,
               **read_csv_kw) -> ChunkSource:
    """A chunk source over a (possibly compressed) CSV: only ``rows_per_chunk`` rows are parsed at a time."""
    import pandas as pd

    cols = list(feature_columns) + [label_column]

    def gen() -> Iterator[Chunk]:
        for df in pd.read_csv(path, usecols=cols, chunksize=rows_per_chunk, **read_csv_kw):
            X = df[list(feature_columns)].to_numpy(dtype=np.float32, na_value=np.nan)
            yield X, df[label_column].to_numpy(dtype=np.float32)
    return gen


def _as_np(a, dtype) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy().astype(dtype, copy=False)
    if hasattr(a, "to_numpy"):
        return a.to_numpy(dtype=dtype)
    return np.asarray(a, dtype=dtype)


class _PinnedUploader:
    """Two pinned staging buffers used alternately; a buffer is refilled only after the device copy
    that last read it has completed, so host parsing overlaps the device's copy + binning."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.buf: list[torch.Tensor | None] = [None, None]
        self.ev: list[torch.cuda.Event | None] = [None, None]
        self.k = 0

    def put(self, x: np.ndarray) -> torch.Tensor:
        i = self.k & 1
        self.k += 1
        if self.ev[i] is not None:
            self.ev[i].synchronize()
        n = x.size
        if self.buf[i] is None or self.buf[i].numel() < n:
            self.buf[i] = torch.empty(max(n, 1), dtype=torch.float32, pin_memory=True)
        stage = self.buf[i][:n]
        stage.copy_(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32).reshape(-1)))
        out = stage.to(self.dev, non_blocking=True).view(x.shape)
        ev = torch.cuda.Event()
        ev.record()
        self.ev[i] = ev
        return out


def stream_cuts(source: ChunkSource, *, n_rows: int | None = None, max_bin: int = 256,
                sketch_rows: int | None = SKETCH_AUTO,
                device=None, dist=None, row_offset: int = 0, n_rows_global: int | None = None):
    """Quantile cuts of a chunk stream: the in-core fit's cuts for the same ``sketch_rows`` (default
    SKETCH_AUTO, as ``gbdt.bin_dataset``). On a GPU
    with every row sketched (``sketch_rows`` SKETCH_AUTO / None / 0) the bucketed device sketch runs
    over the stream, one chunk on the device at a time (sketch.stream_exact_cuts: two more passes);
    otherwise the rows whose GLOBAL index is a multiple of the sketch stride are gathered (SKETCH_AUTO
    on the CPU: 2^18 rows). Returns ``(cuts, nbins, n_rows, n_rows_global, n_features)``."""
    dev = _resolve_device(device, None)
    world = dist.world if dist is not None else 1
    if n_rows is None:
        n_rows = sum(len(c[0]) for c in source())
    N = int(n_rows)
    n_glob = n_rows_global if n_rows_global is not None else (
        int(dist.allreduce_scalar(N, "sum", dev)) if world > 1 else N)
    # (up to 2^18 rows the strided sample is every row already: the cheaper full sort)
    exact_dev = dev.type == "cuda" and (sketch_rows is None or sketch_rows == 0 or
                                        (sketch_rows < 0 and n_glob > SKETCH_SAMPLE_ROWS))
    if exact_dev:  # the boundary sample of sketch.device_exact_cuts (same global rows)
        stride = sketch.sample_stride(n_glob, sketch.BOUNDARY_SAMPLE_ROWS)
    else:
        if sketch_rows is not None and sketch_rows < 0:
            sketch_rows = SKETCH_SAMPLE_ROWS
        stride = sketch.sample_stride(n_glob, sketch_rows or 0)
    F = None
    parts, seen = [], 0
    miss = None  # per-feature NaN presence over the WHOLE stream (decides 255 vs 256 bins)
    for Xc, _ in source():
        Xc = _as_np(Xc, np.float32)
        F = Xc.shape[1] if F is None else F
        first = (-(row_offset + seen)) % stride
        parts.append(Xc[first::stride])
        m = np.isnan(Xc).any(0)
        miss = m if miss is None else (miss | m)
        seen += len(Xc)
    if seen != N:
        raise ValueError(f"the stream yielded {seen} rows, expected {N}")
    samp = torch.as_tensor(np.concatenate(parts) if parts else np.zeros((0, F or 0), np.float32), device=dev)
    has_missing = torch.as_tensor(miss if miss is not None else np.zeros(F or 0, bool), device=dev)
    if world > 1:
        samp = dist.allgather_rows(samp)
        hm = has_missing.to(torch.float32).to(dist._coll_device(dev))
        dist.allreduce(hm, "max")
        has_missing = hm.to(dev) > 0
    if exact_dev:
        def chunks():
            up = _PinnedUploader(dev)
            for Xc, _ in source():
                yield up.put(_as_np(Xc, np.float32))

        cuts, nbins = sketch.stream_exact_cuts(chunks, N, F, samp, has_missing, max_bin,
                                               dist=dist if world > 1 else None, device=dev)
    else:
        cuts, nbins = sketch.compute_cuts(samp, max_bin, None, has_missing)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return cuts, nbins, N, n_glob, F


def bin_stream(source: ChunkSource, *, n_rows: int | None = None, max_bin: int = 256,
               sketch_rows: int | None = SKETCH_AUTO,
               device=None, dist=None, row_offset: int = 0,
               n_rows_global: int | None = None) -> tuple[BinnedData, torch.Tensor]:
    """Quantise a chunk stream; returns the binned matrix and the labels (on ``device``)."""
    dev = _resolve_device(device, None)
    ts = time.perf_counter()
    cuts, nbins, N, n_glob, F = stream_cuts(source, n_rows=n_rows, max_bin=max_bin, sketch_rows=sketch_rows,
                                            device=dev, dist=dist, row_offset=row_offset,
                                            n_rows_global=n_rows_global)
    t_sketch = time.perf_counter() - ts
    tb = time.perf_counter()
    bd = BinnedData(dev, N, n_glob, F, row_offset, cuts, nbins, t_sketch=t_sketch)
    y = torch.empty(N, dtype=torch.float32, device=dev)
    if dev.type == "cuda":
        from ..ops import gbdt_ops

        bd.records = torch.zeros((N, gbdt_ops.row_stride(F)), dtype=torch.uint8, device=dev)
        bd.binsT = torch.empty((F, N), dtype=torch.uint8, device=dev)
        up = _PinnedUploader(dev)
        r0 = 0
        for Xc, yc in source():
            Xc = _as_np(Xc, np.float32)
            n = len(Xc)
            gbdt_ops.bin_matrix_into(up.put(Xc), cuts, nbins, bd.records, bd.binsT, r0)
            y[r0:r0 + n] = torch.from_numpy(_as_np(yc, np.float32)).to(dev, non_blocking=False)
            r0 += n
        torch.cuda.synchronize(dev)
    else:
        bins = np.empty((N, F), dtype=np.uint8)
        c_np, nb_np = cuts.cpu().numpy(), nbins.cpu().numpy()
        r0 = 0
        for Xc, yc in source():
            Xc = _as_np(Xc, np.float32)
            n = len(Xc)
            bins[r0:r0 + n] = sketch.bin_matrix_host(Xc, c_np, nb_np)
            y[r0:r0 + n] = torch.from_numpy(_as_np(yc, np.float32))
            r0 += n
        bd.bins_host = bins
    bd.t_bin = time.perf_counter() - tb
    return bd, y


def train_stream(source: ChunkSource, params: GBDTParams | dict | None = None, *, n_rows: int | None = None,
                 device=None, dist=None, row_offset: int = 0, n_rows_global: int | None = None, **kw):
    """``gbdt.train`` for a chunk stream (same trees as the in-core fit of the same rows)."""
    if params is None:
        params = GBDTParams()
    elif isinstance(params, dict):
        params = GBDTParams.from_kwargs(**params)
    bd, y = bin_stream(source, n_rows=n_rows, max_bin=params.max_bin, sketch_rows=params.sketch_rows,
                       device=device, dist=dist, row_offset=row_offset, n_rows_global=n_rows_global)
    return train_binned(bd, y, params, dist=dist, **kw)
