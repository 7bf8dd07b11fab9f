"""Gradient-boosted decision trees for binary credit-default classification.

Public API:

* :func:`train` — fit a :class:`~.booster.Booster` on a feature matrix (GPU: hand-written gfx950
  kernels, optionally data-parallel across ranks; CPU: the NumPy reference trainer).
* :class:`GBDTClassifier` — an sklearn-compatible estimator with the constructor arguments and
  attributes of ``xgboost.XGBClassifier`` used by the reference (``n_estimators``, ``max_depth``,
  ``learning_rate``, ``gamma``, ``subsample``, ``colsample_bytree``, ``scale_pos_weight``,
  ``random_state``, ``eval_metric``, ``feature_importances_``, ``get_booster()``, ``predict_proba``),
  so it drops into sklearn's RFE / RandomizedSearchCV exactly where the reference used XGBClassifier
  (src/model_train_test/model_tree_train_test.py:111-164).

A fit = quantile sketch (K12) + binning (K13) + ``n_estimators`` boosting rounds of depthwise
histogram trees (K14-K20). See ``csrc/gbdt.hip`` for the device design.
"""
from __future__ import annotations

import ctypes
import json
import logging
import math
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Sequence

import numpy as np
import torch

from . import gbdt_host, sketch
from .booster import Booster, dump_pickle_bytes, sigmoid32, trees_from_heap_nodes
from ..config import knob

log = logging.getLogger(__name__)

XGB_DEFAULTS = dict(n_estimators=100, max_depth=6, learning_rate=0.3, gamma=0.0, min_child_weight=1.0,
                    reg_lambda=1.0, reg_alpha=0.0, subsample=1.0, colsample_bytree=1.0, max_bin=256,
                    scale_pos_weight=1.0, random_state=0, base_score=None)


@dataclass
class GBDTParams:
    n_estimators: int = 100
    max_depth: int = 6
    learning_rate: float = 0.3
    gamma: float = 0.0
    min_child_weight: float = 1.0
    reg_lambda: float = 1.0
    reg_alpha: float = 0.0
    subsample: float = 1.0
    colsample_bytree: float = 1.0
    max_bin: int = 256
    scale_pos_weight: float = 1.0
    random_state: int = 0
    base_score: float | None = None
    # rows of the strided global sample the quantile sketch uses; None / 0 = every row (exact weighted
    # quantiles; on the GPU the device sketch of csrc/sketch.hip, exact under data parallelism too);
    # SKETCH_AUTO (default) = every row on a GPU (XGBoost hist's semantics: the device sketch, ~4 ms at
    # 10M rows; up to 2^18 rows the full sort), a 2^18-row strided sample on the CPU; streams / external
    # memory: see models/stream.stream_cuts
    sketch_rows: int | None = -1
    # quantile-sketch weights: "sample" = the sample weights (XGBoost hist semantics, the reference's
    # tree_method), "hessian" = first-round hessians (sample weight x scale_pos_weight for positives,
    # XGBoost approx semantics); sketch_mode "summary" merges per-rank QuantileSummary objects
    # instead of all-gathering the global sample (see models/sketch.py)
    sketch_weight: str = "sample"
    sketch_mode: str = "sample"
    # fixed-point gradient precision: 17 bits (default; one packed u64 LDS atomic per cell) or 25 bits
    # ("wide": g and h summed in separate int64 cells, 256x finer steps; 32-byte records, <= 24 features
    # on the GPU; the CPU trainer implements both exactly -- docs/PERF.md "Gradient precision")
    grad_bits: int = 17

    @classmethod
    def from_kwargs(cls, **kw) -> "GBDTParams":
        names = {f for f in cls.__dataclass_fields__}
        alias = {"eta": "learning_rate", "lambda": "reg_lambda", "alpha": "reg_alpha", "min_split_loss": "gamma",
                 "seed": "random_state"}
        out = {}
        for k, v in kw.items():
            k = alias.get(k, k)
            if k in names and v is not None:
                out[k] = v
        return cls(**out)


@dataclass
class FitReport:
    """Timings and sizes of one fit (for logs / bench)."""
    n_rows: int = 0
    n_rows_global: int = 0
    n_features: int = 0
    n_trees: int = 0
    device: str = "cpu"
    world: int = 1
    t_sketch: float = 0.0
    t_bin: float = 0.0
    t_boost: float = 0.0
    t_total: float = 0.0
    phases: dict[str, float] = field(default_factory=dict)   # filled when ``sync_phases`` is set
    sync_phases: bool = False
    extra: dict[str, Any] = field(default_factory=dict)

    def mark(self, name: str, t_prev: float, dev: torch.device) -> float:
        """Record the wall time since ``t_prev`` under ``name`` (device-synchronised when profiling)."""
        if not self.sync_phases:
            return t_prev
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        now = time.perf_counter()
        self.phases[name] = self.phases.get(name, 0.0) + (now - t_prev)
        return now


def _to_tensor(X, device, dtype=torch.float32) -> torch.Tensor:
    if isinstance(X, torch.Tensor):
        return X.to(device=device, dtype=dtype).contiguous()
    if hasattr(X, "to_numpy"):
        X = X.to_numpy(dtype=np.float32, na_value=np.nan) if hasattr(X, "columns") else X.to_numpy()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(X, dtype=np.float32)), device=device).to(dtype).contiguous()


def _resolve_device(device: str | torch.device | None, X) -> torch.device:
    if device is None:
        if isinstance(X, torch.Tensor):
            return X.device
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def feature_masks(n_trees: int, n_feat: int, colsample: float, seed: int) -> np.ndarray:
    """Per-tree column masks for ``colsample_bytree`` (all ones when 1.0)."""
    m = np.ones((n_trees, n_feat), dtype=np.uint8)
    if colsample >= 1.0:
        return m
    k = max(1, int(math.floor(colsample * n_feat)))
    rng = np.random.default_rng(seed + 0x5EED)
    for t in range(n_trees):
        m[t] = 0
        m[t, rng.choice(n_feat, size=k, replace=False)] = 1
    return m


@dataclass
class BinnedData:
    """A quantised training matrix: cuts + bins, reusable across fits on the same rows (RFE steps,
    search candidates). GPU: row records [N, stride] + feature-major bins [F, N]; host: uint8 [N, F]."""
    device: torch.device
    n_rows: int
    n_rows_global: int
    n_features: int
    row_offset: int
    cuts: torch.Tensor
    nbins: torch.Tensor
    records: torch.Tensor | None = None
    binsT: torch.Tensor | None = None
    bins_host: np.ndarray | None = None
    t_sketch: float = 0.0
    t_bin: float = 0.0


def _allreduce_max_flags(flags: torch.Tensor, dist, dev) -> torch.Tensor:
    t = flags.to(torch.float32).to(dist._coll_device(dev))
    dist.allreduce(t, "max")
    return t.to(dev) > 0


def _summary_cuts(samp: torch.Tensor, wsamp: torch.Tensor | None, max_bin: int, has_missing: torch.Tensor,
                  dist, dev, on_device: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """sketch_mode="summary": every rank summarises its own sample, the summaries are all-gathered
    (a few KB per feature instead of the raw rows) and merged identically on every rank. Integer
    weights are scaled by the GLOBAL max weight, so one unit means the same weight on every rank.
    ``on_device``: the summary is built where the sample lives (:func:`sketch.device_summary`; the
    full-data sketch), else by the host :class:`sketch.QuantileSummary`."""
    w_max = None
    if wsamp is not None:
        w_max = float(wsamp.max()) if wsamp.numel() else 0.0
        if dist is not None and dist.world > 1:
            w_max = dist.allreduce_scalar(w_max, "max", dev)
        w_max = w_max if w_max > 0 else 1.0
    if on_device:
        off, vals, wts = sketch.device_summary(samp, wsamp, w_max=w_max)
    else:
        summ = sketch.QuantileSummary.build(samp.cpu().numpy(), None if wsamp is None else wsamp.cpu().numpy(),
                                            w_max=w_max)
        off, vals, wts, _ = summ.to_arrays()
    if dist is not None and dist.world > 1:
        per = int(dist.allreduce_scalar(float(len(vals)), "max", dev))  # common padded length
        ent = torch.full((per, 2), float("nan"), dtype=torch.float64)
        ent[: len(vals), 0] = torch.from_numpy(vals.astype(np.float64))
        ent[: len(vals), 1] = torch.from_numpy(wts.astype(np.float64))
        offs = torch.from_numpy(off.astype(np.float64))[:, None]
        all_ent = dist.allgather_rows(ent.to(dist._coll_device(dev))).cpu().numpy()
        all_off = dist.allgather_rows(offs.to(dist._coll_device(dev))).cpu().numpy()[:, 0].astype(np.int64)
        F1 = len(off)
        parts = []
        for r in range(dist.world):
            o = all_off[r * F1:(r + 1) * F1]
            e = all_ent[r * per:r * per + int(o[-1])]
            parts.append(sketch.QuantileSummary.from_arrays(o, e[:, 0].astype(np.float32), e[:, 1].astype(np.int64),
                                                            np.zeros(F1 - 1, dtype=bool)))
        summ = sketch.QuantileSummary.merge(parts)
    else:
        summ = sketch.QuantileSummary.from_arrays(off, vals, wts, np.zeros(len(off) - 1, dtype=bool))
    summ.has_missing = has_missing.cpu().numpy().astype(bool)
    c, nb = summ.cuts(max_bin)
    return torch.from_numpy(c).to(dev), torch.from_numpy(nb).to(dev)


SKETCH_AUTO = -1
SKETCH_SAMPLE_ROWS = 1 << 18


def resolve_sketch_rows(sketch_rows: int | None, dev, n_rows_global: int | None = None) -> int | None:
    """SKETCH_AUTO -> None (every row, the device sketch) on a CUDA device above 2^18 rows; the
    2^18-row sample elsewhere (up to 2^18 rows that sample IS every row, by the cheaper full sort)."""
    if sketch_rows is not None and sketch_rows < 0:
        big = n_rows_global is None or n_rows_global > SKETCH_SAMPLE_ROWS
        return None if (torch.device(dev).type == "cuda" and big) else SKETCH_SAMPLE_ROWS
    return sketch_rows


def bin_dataset(X, *, max_bin: int = 256, sketch_rows: int | None = SKETCH_AUTO, device=None, dist=None,
                n_rows_global: int | None = None, row_offset: int = 0, sketch_weights=None,
                sketch_mode: str = "sample") -> BinnedData:
    """Weighted quantile sketch (K12) on a global strided sample + binning (K13).

    ``sketch_rows`` None / 0: every row (XGBoost ``hist`` sketches all rows), exact weighted quantiles.
    On a GPU this is the bucketed device sketch (``sketch.device_exact_cuts``): under data parallelism
    its bucket histograms are all-reduced and the target buckets' candidates all-gathered, so every rank
    gets the full data's cuts without gathering the raw rows. On the CPU under data parallelism each
    rank summarises its shard and the summaries are merged (``sketch_mode="summary"``).
    ``sketch_weights`` ([N_local], optional): per-row sketch weights (see models/sketch.py).
    A feature gets 256 bins only if it has no missing value in the FULL data (all ranks).
    ``SKETCH_AUTO``: every row on a GPU, the 2^18-row sample on the CPU."""
    dev = _resolve_device(device, X)
    world = dist.world if dist is not None else 1
    Xt = _to_tensor(X, dev)
    N, F = Xt.shape
    n_glob = n_rows_global if n_rows_global is not None else (
        int(dist.allreduce_scalar(N, "sum", dev)) if world > 1 else N)
    sketch_rows = resolve_sketch_rows(sketch_rows, dev, n_glob)
    ts = time.perf_counter()
    has_missing = torch.isnan(Xt).any(0) if N else torch.zeros(F, dtype=torch.bool, device=dev)
    full = not sketch_rows
    if full and dev.type == "cuda" and sketch_mode != "summary":
        # every row, exactly (csrc/sketch.hip: bucket histograms + per-bucket selection, no row sort;
        # under data parallelism four device all-reduces -- the missing flags ride in the first -- so
        # the cuts are the full data's)
        sw = _to_tensor(sketch_weights, dev).reshape(-1) if sketch_weights is not None else None
        cuts, nbins = sketch.device_exact_cuts(Xt, max_bin, sw, has_missing if world == 1 else None,
                                               dist=dist if world > 1 else None, row_offset=row_offset,
                                               n_rows_global=n_glob)
        torch.cuda.synchronize(dev)
        t_sketch = time.perf_counter() - ts
        tb = time.perf_counter()
        bd = BinnedData(dev, N, n_glob, F, row_offset, cuts, nbins, t_sketch=t_sketch)
        _bin_device(bd, Xt, cuts, nbins)
        torch.cuda.synchronize(dev)
        bd.t_bin = time.perf_counter() - tb
        return bd
    if world > 1:
        has_missing = _allreduce_max_flags(has_missing, dist, dev)
    stride = 1 if full else sketch.sample_stride(n_glob, sketch_rows)
    samp = sketch.local_sample(Xt, row_offset, stride)
    wsamp = None
    if sketch_weights is not None:
        wsamp = sketch.local_sample(_to_tensor(sketch_weights, dev).reshape(-1, 1), row_offset, stride)[:, 0]
    if sketch_mode == "summary" or (full and world > 1):
        cuts, nbins = _summary_cuts(samp, wsamp, max_bin, has_missing, dist, dev, on_device=full)
    else:
        if world > 1:
            samp = dist.allgather_rows(samp)
            if wsamp is not None:
                wsamp = dist.allgather_rows(wsamp.reshape(-1, 1), pad_value=0.0)[:, 0]
        cuts, nbins = sketch.compute_cuts(samp, max_bin, wsamp, has_missing)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_sketch = time.perf_counter() - ts
    tb = time.perf_counter()
    bd = BinnedData(dev, N, n_glob, F, row_offset, cuts, nbins, t_sketch=t_sketch)
    if dev.type == "cuda":
        _bin_device(bd, Xt, cuts, nbins)
        torch.cuda.synchronize(dev)
    else:
        bd.bins_host = sketch.bin_matrix_host(Xt.cpu().numpy(), cuts.cpu().numpy(), nbins.cpu().numpy())
    bd.t_bin = time.perf_counter() - tb
    return bd


def _bin_device(bd: BinnedData, Xt: torch.Tensor, cuts: torch.Tensor, nbins: torch.Tensor) -> None:
    """Binning on the GPU: row records (32 bytes for <= 24 features) + feature-major bins.
    (Packed 16-byte records were measured slower in round 5 -- the per-feature bit-field extracts cost
    the histogram gathers more than the halved bytes saved: profiles/round5/packed_vs_32byte.txt.)"""
    from ..ops import gbdt_ops

    bd.records, bd.binsT = gbdt_ops.bin_matrix(Xt, cuts, nbins)


def sketch_weights_for(params: "GBDTParams", y, sample_weight=None, device=None):
    """Per-row sketch weights for ``params.sketch_weight`` (None = unweighted)."""
    mode = getattr(params, "sketch_weight", "sample")
    if mode == "sample":
        return sample_weight
    if mode != "hessian":
        raise ValueError(f"sketch_weight must be 'sample' or 'hessian', got {mode!r}")
    yt = _to_tensor(y, device).reshape(-1)
    w = _to_tensor(sample_weight, device).reshape(-1) if sample_weight is not None else torch.ones_like(yt)
    spw = float(params.scale_pos_weight if params.scale_pos_weight is not None else 1.0)
    return w * torch.where(yt == 1.0, torch.tensor(spw, device=yt.device), torch.tensor(1.0, device=yt.device))


def subset_rows(bd: BinnedData, rows: np.ndarray) -> BinnedData:
    """Rows ``rows`` of a binned matrix with the same cuts (CV folds re-use one binning)."""
    idx = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=bd.device)
    out = BinnedData(bd.device, len(rows), len(rows), bd.n_features, 0, bd.cuts, bd.nbins)
    if bd.records is not None:
        out.records = bd.records.index_select(0, idx).contiguous()
        out.binsT = bd.binsT.index_select(1, idx).contiguous()
    else:
        out.bins_host = bd.bins_host[np.asarray(rows)]
    return out


def subset_features(bd: BinnedData, feats) -> BinnedData:
    """The binned matrix restricted to the feature columns ``feats`` (ascending indices), repacked:
    row records of the narrower width (32 bytes for <= 24 features: the fused fast path) and the
    matching feature-major rows -- a device gather of ``N x len(feats)`` bytes, no re-sketch (cuts
    are per feature). A fit on it grows exactly the trees of a ``feature_mask`` fit on ``bd``
    (same bins, same colsample draws, same tie order), at the cost of the narrower matrix."""
    f = np.asarray(feats, dtype=np.int64)
    idx = torch.as_tensor(f, device=bd.device)
    out = BinnedData(bd.device, bd.n_rows, bd.n_rows_global, len(f), bd.row_offset,
                     bd.cuts.index_select(0, idx).contiguous(), bd.nbins.index_select(0, idx).contiguous())
    if bd.records is not None:
        from ..ops import gbdt_ops

        rec = torch.zeros((bd.n_rows, gbdt_ops.row_stride(len(f))), dtype=torch.uint8, device=bd.device)
        rec[:, : len(f)] = bd.records.index_select(1, idx)
        out.records = rec
        out.binsT = bd.binsT.index_select(0, idx).contiguous()
    else:
        out.bins_host = np.ascontiguousarray(bd.bins_host[:, f])
    return out


def expand_features(bst: Booster, feats, n_features: int, feature_names: Sequence[str] | None = None,
                    feature_types: Sequence[str] | None = None) -> Booster:
    """A booster fitted on :func:`subset_features` columns, re-expressed over the full feature space
    (split indices mapped back; leaves keep index 0 as XGBoost writes them)."""
    from .booster import Tree

    f = np.asarray(feats, dtype=np.int32)
    trees = []
    for t in bst.trees:
        si = np.where(t.left_children != -1, f[t.split_indices], 0).astype(np.int32)
        trees.append(Tree(t.left_children, t.right_children, t.parents, si, t.split_conditions, t.default_left,
                          t.base_weights, t.loss_changes, t.sum_hessian))
    return Booster(trees, list(feature_names) if feature_names is not None else None,
                   list(feature_types) if feature_types is not None else None, bst.base_score, int(n_features),
                   bst.objective, dict(bst.train_params), dict(bst.attributes))


def check_grad_bits(grad_bits: int, n_features: int, device_type: str) -> None:
    """``grad_bits`` is 17 or 25; the GPU's wide (25-bit) cells need the 32-byte row records of <= 24
    features (csrc/gbdt.hip cobalt_gbdt_create refuses the rest with -6)."""
    if grad_bits not in gbdt_host.GRAD_BITS:
        raise ValueError(f"grad_bits must be one of {gbdt_host.GRAD_BITS}")
    if grad_bits > 17 and device_type == "cuda" and n_features > 24:
        raise ValueError(f"grad_bits={grad_bits} on the GPU supports <= 24 features (32-byte row records); "
                         f"got {n_features}: use grad_bits=17")


def check_gpu_shape(max_depth: int, n_rows: int) -> None:
    """The GPU trainer's limits (csrc/gbdt.hip cobalt_gbdt_create: -1 / -5), named before any device work."""
    if not 1 <= max_depth <= 10:
        raise ValueError(f"the GPU trainer supports max_depth 1-10 (got {max_depth}); use the host trainer "
                         "(device='cpu') for deeper trees")
    if n_rows >= (1 << 31) - 1:
        raise ValueError(f"{n_rows} rows exceed one GPU fit's int32 row ids: shard them over ranks "
                         "(data parallel) or stream them (models.external.train_external)")


def train(X, y, params: GBDTParams | dict | None = None, *, sample_weight=None, device=None,
          feature_names: Sequence[str] | None = None, feature_types: Sequence[str] | None = None,
          dist=None, n_rows_global: int | None = None, row_offset: int = 0,
          report: FitReport | None = None, init_booster: Booster | None = None,
          checkpoint_path: str | None = None, checkpoint_every: int = 0, resume: bool = True,
          exact_fp64: bool = False) -> Booster:
    """Fit a binary:logistic GBDT. With ``dist`` (a :class:`~..parallel.dist.DistContext`) each rank
    passes its local row shard (``row_offset`` = global index of its first row).

    ``init_booster`` continues boosting from an existing model for ``n_estimators`` MORE trees
    (XGBoost's ``xgb_model=``). ``checkpoint_path`` + ``checkpoint_every`` write the model every that
    many trees (atomic replace, rank 0); with ``resume`` an existing checkpoint there is loaded and
    training continues to ``n_estimators`` trees in total -- bit-identical to an uninterrupted fit,
    because sampling is keyed by the global tree index and the margins are re-predicted in tree order.

    ``exact_fp64`` (CPU only): unquantised fp64 gradients and histograms -- the accuracy reference of
    the fixed-point trainer (tests/test_quantization.py)."""
    if params is None:
        params = GBDTParams()
    elif isinstance(params, dict):
        params = GBDTParams.from_kwargs(**params)
    t0 = time.perf_counter()
    ckpt = Checkpointer(checkpoint_path, checkpoint_every, params, dist) if checkpoint_path else None
    total = None
    if ckpt is not None and resume and init_booster is None:
        init_booster = ckpt.load()
        if init_booster is not None:
            total = int(params.n_estimators)
            log.info("resuming from %s at tree %d of %d", checkpoint_path, init_booster.num_trees, total)
    dev = _resolve_device(device, X)
    # the trainer's shape limits, before the sketch (and its data-parallel collectives) and the binning;
    # train_binned checks them again for pre-binned inputs
    check_grad_bits(int(params.grad_bits), int(X.shape[1]), dev.type)
    if dev.type == "cuda":
        check_gpu_shape(int(params.max_depth), int(X.shape[0]))
    init_margin = None
    if init_booster is not None:
        from ..ops import predict_ops

        Xt = _to_tensor(X, dev)
        init_margin = predict_ops.predict_margin(init_booster, Xt, dev)
        if not isinstance(init_margin, torch.Tensor):
            init_margin = torch.as_tensor(init_margin)
        init_margin = init_margin.to(dev, torch.float32).contiguous()
    bd = bin_dataset(X, max_bin=params.max_bin, sketch_rows=params.sketch_rows, device=device, dist=dist,
                     n_rows_global=n_rows_global, row_offset=row_offset,
                     sketch_weights=sketch_weights_for(params, y, sample_weight, dev),
                     sketch_mode=params.sketch_mode)
    bst = train_binned(bd, y, params, sample_weight=sample_weight, feature_names=feature_names,
                       feature_types=feature_types, dist=dist, report=report, init_booster=init_booster,
                       init_margin=init_margin, total_trees=total, checkpoint=ckpt, exact_fp64=exact_fp64)
    if report is not None:
        report.t_total = time.perf_counter() - t0
    return bst


def train_binned(bd: BinnedData, y, params: GBDTParams | dict | None = None, *, sample_weight=None,
                 feature_names: Sequence[str] | None = None, feature_types: Sequence[str] | None = None,
                 feature_mask: np.ndarray | None = None, dist=None, report: FitReport | None = None,
                 init_booster: Booster | None = None, init_margin: torch.Tensor | None = None,
                 total_trees: int | None = None, checkpoint: "Checkpointer | None" = None,
                 exact_fp64: bool = False) -> Booster:
    """Boost on pre-binned data. ``feature_mask`` (bool [F]) restricts the fit to a feature subset
    (the trees still index the full feature space, so a subset fit costs no re-binning).
    ``init_booster`` + ``init_margin`` (its margins on these rows) continue an existing model: grow
    ``total_trees - init_booster.num_trees`` trees (default ``n_estimators`` more)."""
    if params is None:
        params = GBDTParams()
    elif isinstance(params, dict):
        params = GBDTParams.from_kwargs(**params)
    dev = bd.device
    world = dist.world if dist is not None else 1
    grad_bits = int(params.grad_bits)
    N, F = bd.n_rows, bd.n_features
    check_grad_bits(grad_bits, F, dev.type)
    if dev.type == "cuda":
        check_gpu_shape(int(params.max_depth), N)
    rep = report if report is not None else FitReport()
    tp = rep.mark("pre", time.perf_counter(), dev)
    yt = _to_tensor(y, dev).reshape(-1)
    if yt.shape[0] != N:
        raise ValueError("X and y row counts differ")
    spw = float(params.scale_pos_weight if params.scale_pos_weight is not None else 1.0)
    # (python scalars, not device tensors: no host-to-device copies; the same float32 values)
    pw = torch.where(yt == 1.0, spw, 1.0).to(torch.float32)
    wt = (_to_tensor(sample_weight, dev).reshape(-1) * pw) if sample_weight is not None else pw
    wt = wt.to(torch.float32).contiguous()

    T0 = init_booster.num_trees if init_booster is not None else 0
    if init_booster is not None and init_margin is None:
        raise ValueError("init_booster needs init_margin (its margins on the training rows)")
    # base score = weighted label mean (XGBoost boost_from_average for binary:logistic) and the largest
    # weight (the fixed-point scales); under data parallelism both in ONE collective: [sum w, sum w y,
    # every rank's max weight in its own slot] summed on the device
    need_bs = init_booster is None and params.base_score is None
    labels_binary = None  # known after the one-rank read below
    if world > 1:
        buf = torch.zeros(2 + world, dtype=torch.float64, device=dev)
        if need_bs:
            buf[0] = wt.double().sum()
            buf[1] = (wt.double() * yt.double()).sum()
        if N:
            buf[2 + dist.rank] = wt.max().double()
        if hasattr(dist, "device_allreduce") and dev.type == "cuda":
            dist.device_allreduce(buf, "sum")
        else:
            t = buf.to(dist._coll_device(dev))
            dist.allreduce(t, "sum")
            buf = t.to(dev)
        sw, swy, wmax = (float(v) for v in (buf[0], buf[1], buf[2:].max()))
    else:  # one device -> host read for the three (and whether the labels are 0 / 1, for the trainer)
        wd = wt.double()
        z = torch.zeros((), dtype=torch.float64, device=dev)
        sw, swy, wmax, y01 = torch.stack([wd.sum() if need_bs else z, (wd * yt.double()).sum() if need_bs else z,
                                          wd.max() if N else z + 1.0,
                                          ((yt == 0) | (yt == 1)).all().double()]).tolist()
        labels_binary = y01 != 0.0
    if init_booster is not None:
        base_score = float(init_booster.base_score)
    elif params.base_score is None:
        base_score = min(max(swy / sw if sw > 0 else 0.5, 1e-6), 1 - 1e-6)
    else:
        base_score = float(params.base_score)
    base_score = float(np.float32(base_score))
    base_margin = Booster([], base_score=base_score, num_feature=F).base_margin
    gscale, hscale = gbdt_host.quant_scales(wmax, grad_bits)

    T_new = (int(total_trees) - T0) if total_trees is not None else int(params.n_estimators)
    if T_new < 0:
        raise ValueError("the initial model already has more trees than requested")
    T = T0 + T_new  # global tree indices [T0, T) are grown; masks/RNG are keyed by the global index
    fmask_np = feature_masks(T, F, float(params.colsample_bytree), int(params.random_state))
    if feature_mask is not None:
        fm_sub = np.asarray(feature_mask, dtype=bool)
        active = np.nonzero(fm_sub)[0]
        fmask_np = np.zeros((T, F), dtype=np.uint8)
        sub = feature_masks(T, len(active), float(params.colsample_bytree), int(params.random_state))
        fmask_np[:, active] = sub
    seg = checkpoint.every if checkpoint is not None and checkpoint.every > 0 else max(T_new, 1)
    trees_so_far = list(init_booster.trees) if init_booster is not None else []
    names = list(feature_names) if feature_names is not None else (
        list(init_booster.feature_names) if init_booster is not None and init_booster.feature_names else None)
    ftypes = list(feature_types) if feature_types is not None else (
        list(init_booster.feature_types) if init_booster is not None and init_booster.feature_types else None)

    def make_booster(trees):
        return Booster(trees=list(trees), feature_names=names, feature_types=ftypes, base_score=base_score,
                       num_feature=F,
                       train_params=dict(eta=hp.eta, gamma=hp.gamma, max_depth=hp.max_depth,
                                         min_child_weight=hp.min_child_weight, reg_lambda=hp.reg_lambda,
                                         reg_alpha=hp.reg_alpha, subsample=hp.subsample,
                                         colsample_bytree=float(params.colsample_bytree),
                                         max_bin=int(params.max_bin), scale_pos_weight=spw, seed=hp.seed))

    def segment_done(new_nodes: np.ndarray, end: int) -> None:
        trees_so_far.extend(trees_from_heap_nodes(new_nodes, hp.max_depth))
        if checkpoint is not None:
            checkpoint.save(make_booster(trees_so_far))
        fault_after = int(knob("COBALT_FAULT_AFTER_TREES", "0") or 0)
        fault_rank = int(knob("COBALT_FAULT_RANK", "-1") or -1)
        if fault_after and end >= fault_after and end < T and (fault_rank < 0 or fault_rank == (dist.rank if dist else 0)):
            stall = float(knob("COBALT_FAULT_STALL_S", "0") or 0)
            if stall > 0:  # a slow (not dead) rank: once, then it carries on
                if not getattr(segment_done, "stalled", False):
                    segment_done.stalled = True
                    time.sleep(stall)
            else:
                raise InjectedFault(f"injected fault after tree {end}")
    hp = gbdt_host.HostGbdtParams(max_depth=int(params.max_depth), eta=float(params.learning_rate),
                                  reg_lambda=float(params.reg_lambda), reg_alpha=float(params.reg_alpha),
                                  gamma=float(params.gamma), min_child_weight=float(params.min_child_weight),
                                  subsample=float(params.subsample), seed=int(params.random_state),
                                  gscale=1.0 if exact_fp64 else gscale, hscale=1.0 if exact_fp64 else hscale,
                                  quant=not exact_fp64, qbits=grad_bits)
    if exact_fp64 and dev.type != "cpu":
        raise ValueError("exact_fp64 is the host (CPU) reference trainer")
    tp = rep.mark("labels_weights", tp, dev)
    tb = time.perf_counter()
    if dev.type == "cuda":
        from ..ops import gbdt_ops

        margin = (init_margin.to(dev, torch.float32).clone().contiguous() if init_margin is not None
                  else torch.full((N,), base_margin, dtype=torch.float32, device=dev))
        comm = dist.native_comm if dist is not None else None
        if world > 1 and comm is None:
            raise RuntimeError("data-parallel GPU training needs the native RCCL communicator")
        tr = gbdt_ops.GpuGbdtTrainer(n_rows=N, n_feat=F, max_depth=hp.max_depth, max_trees=T, eta=hp.eta,
                                     reg_lambda=hp.reg_lambda, reg_alpha=hp.reg_alpha, gamma=hp.gamma,
                                     min_child_weight=hp.min_child_weight, subsample=hp.subsample,
                                     gscale=gscale, hscale=hscale, base_margin=base_margin,
                                     seed=hp.seed, row_offset=bd.row_offset, world_size=world, comm=comm,
                                     grad_bits=grad_bits)
        fm = torch.as_tensor(fmask_np, device=dev).contiguous()
        tr.set_data(bd.records, bd.binsT, bd.cuts.contiguous(), bd.nbins.to(torch.int32).contiguous(),
                    yt.contiguous(), wt, margin, fm)
        # 0/1 labels and no sample weights: the labels ride in the row records' padding and the weights
        # follow from them (8 fewer bytes per row in every gradient pass); COBALT_LABEL_IN_RECORD=0 off
        if (sample_weight is None and knob("COBALT_LABEL_IN_RECORD", "1") != "0"
                and bd.records.shape[1] == 32 and F <= 23
                and (labels_binary if labels_binary is not None else bool(((yt == 0) | (yt == 1)).all()))):
            tr.set_binary_labels(float(np.float32(spw)))
        tp = rep.mark("trainer_setup", tp, dev)
        completed = False
        try:
            if T0:
                tr.set_start(T0)
            if world > 1:
                # COBALT_FAULT_CORRUPT_RANK=r [COBALT_FAULT_CORRUPT_TREE=t]: rank r grows a different tree t
                # (its root totals perturbed), which the in-flight replica check must catch on every rank
                cr = int(knob("COBALT_FAULT_CORRUPT_RANK", "-1") or -1)
                if cr == dist.rank:
                    tr.set_fault(int(knob("COBALT_FAULT_CORRUPT_TREE", "1") or 1))
            head = None
            if checkpoint is None and T - T0 >= 64 and _own_device(world):
                # Two grow calls: the first part's trees are fetched (on a side stream) and converted on
                # the host while the GPU grows the last ones -- the host's ~1 ms per 300 trees of
                # fetch + conversion leaves the fit's critical path.
                tail = min(32, (T - T0) // 4)
                head = T - tail
                tr.grow(T0, head - T0)
                ev = torch.cuda.Event()
                ev.record()
                tr.grow(head, T - head)
                rep.extra["plan"] = tr.plan()
                if world > 1:
                    _watch_segment(dist, dev, T0, head, tr, ev)
                else:
                    ev.synchronize()
                trees_so_far.extend(trees_from_heap_nodes(tr.fetch(T0, head - T0, _side_stream(dev)), hp.max_depth))
            for s0 in ([head] if head is not None else range(T0, T, seg)):
                s1 = min(T, s0 + seg)
                if head is None:
                    tr.grow(s0, s1 - s0)
                    rep.extra["plan"] = tr.plan()
                if world > 1:  # fail fast (abort the communicator) if a peer rank dies mid-segment
                    _watch_segment(dist, dev, s0, s1, tr)
                tp = rep.mark("grow", tp, dev)
                seg_nodes = tr.fetch(s0, s1 - s0)
                if world > 1 and tr.replica_error():
                    raise ReplicaDivergence(f"data-parallel replicas diverged before tree {s1} (rank {dist.rank}): "
                                            "the ranks' split decisions differ (in-flight digest check)")
                tp = rep.mark("fetch", tp, dev)
                segment_done(seg_nodes, s1)
                tp = rep.mark("convert", tp, dev)
            completed = True
        finally:
            tr.close(park=completed)  # a completed fit's context is kept for the next fit of these shapes
        tp = rep.mark("close", tp, dev)
        rep.extra["margin"] = margin  # training margins incl. every tree (device tensor)
    else:
        cuts_np = bd.cuts.cpu().numpy()
        nb_np = bd.nbins.cpu().numpy()
        margin_np = (init_margin.cpu().numpy().astype(np.float32).copy() if init_margin is not None
                     else np.full(N, np.float32(base_margin), dtype=np.float32))
        y_np = yt.cpu().numpy()
        w_np = wt.cpu().numpy()
        allreduce = None
        if world > 1:
            def allreduce(a: np.ndarray) -> np.ndarray:
                t = torch.from_numpy(np.ascontiguousarray(a))
                dist.allreduce(t, "sum")
                return t.numpy()
        for s0 in range(T0, T, seg):
            s1 = min(T, s0 + seg)
            recs = []
            for t in range(s0, s1):
                gq, hq = gbdt_host.gradients_host(margin_np, y_np, w_np, hp, t, bd.row_offset)
                recs.append(gbdt_host.grow_tree_host(bd.bins_host, cuts_np, nb_np, gq, hq, margin_np, hp,
                                                     fmask_np[t], allreduce))
            segment_done(np.stack(recs), s1)
        rep.extra["margin"] = margin_np
    t_boost = time.perf_counter() - tb
    tp = rep.mark("to_trees", tp, dev)
    bst = make_booster(trees_so_far)
    if report is not None:
        report.n_rows, report.n_rows_global, report.n_features, report.n_trees = N, bd.n_rows_global, F, T
        report.device, report.world = str(dev), world
        report.t_sketch, report.t_bin, report.t_boost = bd.t_sketch, bd.t_bin, t_boost
        report.extra["cuts"] = bd.cuts
        report.extra["nbins"] = bd.nbins
    return bst


_side_streams: dict = {}


def _own_device(world: int) -> bool:
    """Whether the fit may take a second stream of its own (the fetch overlap): one process only. Ranks
    that share a device (the one-GPU rehearsals) are time-sliced or CU-partitioned, and their exchange
    kernels wait on each other inside the GPU: an extra stream per process deadlocked unmasked ranks for
    the 120 s exchange deadline (tests/test_00gpu_dp_ipc.py, a CU budget without masks) and slowed
    CU-masked ranks 9x (2 ranks, 2M rows: 945.6 vs 102.7 ms per fit,
    profiles/round6/ab_sketch_side_stream.txt). Data-parallel fits on separate GPUs would not share
    queues, but that configuration cannot be rehearsed on one GPU, so they keep one stream too."""
    return world <= 1


def _side_stream(dev) -> torch.cuda.Stream:
    """A second stream of ``dev`` (created once) for copies that must not wait on the trainer's stream."""
    key = torch.device(dev).index or 0
    if key not in _side_streams:
        _side_streams[key] = torch.cuda.Stream(torch.device("cuda", key))
    return _side_streams[key]


def _watch_segment(dist, dev, s0: int, s1: int, tr=None, ev=None) -> None:
    """Wait for trees [s0, s1) -- the work before ``ev`` (default: everything enqueued so far) -- with
    the data-parallel watchdog (a dead or failed peer aborts the communicator instead of hanging)."""
    from .. import _native
    from ..parallel import dist as pdist

    if ev is None:
        ev = torch.cuda.Event()
        ev.record()
    comm = dist.native_comm
    lib = _native.lib()

    def comm_error():
        e = lib.cobalt_comm_async_error(ctypes.c_void_p(comm)) if comm else 0
        return e
    # a replica divergence does not stop the stream (every rank keeps exchanging in step): the segment
    # finishes and the caller raises ReplicaDivergence after it, on every rank
    pdist.wait_with_watchdog(ev.query, timeout_s=pdist.collective_timeout_s(), comm_error=comm_error if comm else None,
                             abort=lambda: pdist.abort_native_comm(dist), what=f"trees {s0}..{s1 - 1}")


class InjectedFault(RuntimeError):
    """Raised by the fault-injection hook (``COBALT_FAULT_AFTER_TREES`` [+ ``COBALT_FAULT_RANK``])."""


class ReplicaDivergence(RuntimeError):
    """Data-parallel ranks grew different trees (a stale or corrupted exchange on some rank). Raised on
    every rank of the fit: each one's digest check compares the ranks' summed digests with its own."""


class Checkpointer:
    """Periodic model checkpoints of a fit (checkpoint-per-N-trees + resume).

    The checkpoint is the XGBoost UBJSON model of the trees grown so far (loadable by any consumer
    of the format) plus a JSON sidecar with the fit parameters; both are replaced atomically
    (write + ``os.replace``). Only rank 0 writes under data parallelism; every rank reads on resume."""

    def __init__(self, path: str, every: int, params: GBDTParams, dist=None):
        self.path = str(path)
        self.every = int(every)
        self.params = params
        self.rank = dist.rank if dist is not None else 0

    def _meta(self, n_trees: int) -> dict:
        keys = ("max_depth", "learning_rate", "gamma", "min_child_weight", "reg_lambda", "reg_alpha", "subsample",
                "colsample_bytree", "max_bin", "scale_pos_weight", "random_state", "n_estimators")
        return {"n_trees": n_trees, "params": {k: getattr(self.params, k) for k in keys}}

    def save(self, booster: Booster) -> None:
        if self.rank != 0:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(booster.save_raw("ubj"))
        os.replace(tmp, self.path)
        with open(tmp + ".json", "w") as fh:
            json.dump(self._meta(booster.num_trees), fh)
        os.replace(tmp + ".json", self.path + ".json")

    def load(self) -> Booster | None:
        if not os.path.exists(self.path):
            return None
        meta_p = self.path + ".json"
        if os.path.exists(meta_p):
            with open(meta_p) as fh:
                meta = json.load(fh)
            want = self._meta(meta["n_trees"])["params"]
            diff = {k: (meta["params"].get(k), v) for k, v in want.items()
                    if k != "n_estimators" and meta["params"].get(k) != v}
            if diff:
                raise ValueError(f"checkpoint {self.path} was written with different parameters: {diff}")
        with open(self.path, "rb") as fh:
            return Booster.load_raw(fh.read())


def _feature_info(X) -> tuple[list[str] | None, list[str] | None]:
    if hasattr(X, "columns"):
        names = [str(c) for c in X.columns]
        types = []
        for c in X.columns:
            dt = X[c].dtype
            if dt == bool or str(dt) == "bool":
                types.append("i")
            elif np.issubdtype(dt, np.integer):
                types.append("int")
            else:
                types.append("float")
        return names, types
    return None, None


class GBDTClassifier:
    """sklearn-compatible drop-in for ``xgboost.XGBClassifier`` backed by this framework's trainer."""

    _param_names = ["n_estimators", "max_depth", "learning_rate", "gamma", "min_child_weight", "reg_lambda",
                    "reg_alpha", "subsample", "colsample_bytree", "max_bin", "scale_pos_weight", "random_state",
                    "base_score", "eval_metric", "use_label_encoder", "device", "importance_type", "n_jobs",
                    "sketch_rows", "sketch_weight"]

    def __init__(self, n_estimators=None, max_depth=None, learning_rate=None, gamma=None, min_child_weight=None,
                 reg_lambda=None, reg_alpha=None, subsample=None, colsample_bytree=None, max_bin=None,
                 scale_pos_weight=None, random_state=None, base_score=None, eval_metric=None,
                 use_label_encoder=None, device=None, importance_type=None, n_jobs=None, sketch_rows=None,
                 sketch_weight=None):
        self.n_estimators = n_estimators
        self.max_depth = max_depth
        self.learning_rate = learning_rate
        self.gamma = gamma
        self.min_child_weight = min_child_weight
        self.reg_lambda = reg_lambda
        self.reg_alpha = reg_alpha
        self.subsample = subsample
        self.colsample_bytree = colsample_bytree
        self.max_bin = max_bin
        self.scale_pos_weight = scale_pos_weight
        self.random_state = random_state
        self.base_score = base_score
        self.eval_metric = eval_metric
        self.use_label_encoder = use_label_encoder
        self.device = device
        self.importance_type = importance_type
        self.n_jobs = n_jobs
        self.sketch_rows = sketch_rows
        self.sketch_weight = sketch_weight

    # sklearn protocol
    def get_params(self, deep: bool = True) -> dict[str, Any]:
        return {k: getattr(self, k) for k in self._param_names}

    def set_params(self, **params) -> "GBDTClassifier":
        for k, v in params.items():
            if k not in self._param_names:
                raise ValueError(f"invalid parameter {k!r}")
            setattr(self, k, v)
        return self

    def __sklearn_tags__(self):
        from sklearn.utils import Tags, ClassifierTags, TargetTags, InputTags
        return Tags(estimator_type="classifier", target_tags=TargetTags(required=True),
                    classifier_tags=ClassifierTags(), input_tags=InputTags(allow_nan=True))

    _estimator_type = "classifier"

    def _train_params(self) -> GBDTParams:
        kw = {k: v for k, v in self.get_params().items() if v is not None}
        return GBDTParams.from_kwargs(**{k: v for k, v in {**XGB_DEFAULTS, **kw}.items()})

    def fit(self, X, y, sample_weight=None, xgb_model=None, **_):
        """``xgb_model`` (a Booster, a fitted classifier or a model/pickle path) continues boosting
        from that model for ``n_estimators`` more trees, as XGBoost's ``fit(xgb_model=...)``."""
        names, types = _feature_info(X)
        init = None
        if xgb_model is not None:
            if isinstance(xgb_model, Booster):
                init = xgb_model
            elif hasattr(xgb_model, "get_booster"):
                init = xgb_model.get_booster()
            else:
                from pathlib import Path

                raw = Path(xgb_model).read_bytes()
                if raw[:1] == b"\x80":
                    from .booster import load_pickle_bytes

                    init = load_pickle_bytes(raw)[1]
                else:
                    init = Booster.load_raw(raw)
        y_np = np.asarray(y.to_numpy() if hasattr(y, "to_numpy") else y).reshape(-1)
        self.classes_ = np.unique(y_np)
        if len(self.classes_) > 2:
            raise ValueError("GBDTClassifier supports binary targets")
        self.n_classes_ = 2
        yb = (y_np == self.classes_[-1]).astype(np.float32) if len(self.classes_) == 2 else y_np.astype(np.float32)
        rep = FitReport()
        self._Booster = train(X, yb, self._train_params(), sample_weight=sample_weight, device=self.device,
                              feature_names=names, feature_types=types, report=rep, init_booster=init)
        self.fit_report_ = rep
        self.n_features_in_ = self._Booster.num_feature
        if names is not None:
            self.feature_names_in_ = np.array(names, dtype=object)
        return self

    def get_booster(self) -> Booster:
        if not hasattr(self, "_Booster"):
            raise ValueError("need to call fit or load_model beforehand")
        return self._Booster

    def _matrix(self, X) -> np.ndarray | torch.Tensor:
        if isinstance(X, torch.Tensor):
            return X
        if hasattr(X, "columns") and getattr(self, "feature_names_in_", None) is not None:
            X = X[list(self.feature_names_in_)]
        return np.asarray(X.to_numpy(dtype=np.float32, na_value=np.nan) if hasattr(X, "to_numpy") else X,
                          dtype=np.float32)

    def predict_proba(self, X) -> np.ndarray:
        p = self.get_booster().predict_proba(self._matrix(X), device=self.device)
        p = p.cpu().numpy() if isinstance(p, torch.Tensor) else np.asarray(p)
        return np.stack([1.0 - p, p], axis=1)

    def predict(self, X) -> np.ndarray:
        p = self.predict_proba(X)[:, 1]
        pred = (p > 0.5).astype(np.int64)
        return self.classes_[pred] if getattr(self, "classes_", None) is not None and len(self.classes_) == 2 else pred

    def score(self, X, y) -> float:
        from ..metrics.classification import accuracy_score

        return accuracy_score(np.asarray(y), self.predict(X))

    @property
    def feature_importances_(self) -> np.ndarray:
        return self.get_booster().feature_importances(self.importance_type or "gain")

    # checkpoint I/O (reference: joblib.dump(best_model_tree) -> xgb_model_tree.pkl)
    def sklearn_state_params(self) -> dict[str, Any]:
        p = {k: getattr(self, k) for k in ["n_estimators", "max_depth", "learning_rate", "gamma", "min_child_weight",
                                           "reg_alpha", "reg_lambda", "subsample", "colsample_bytree",
                                           "scale_pos_weight", "base_score", "random_state", "max_bin", "device",
                                           "importance_type", "n_jobs", "eval_metric"]}
        p["kwargs"] = {"use_label_encoder": self.use_label_encoder} if self.use_label_encoder is not None else {}
        return p

    def save_pickle(self, path) -> None:
        from pathlib import Path

        Path(path).write_bytes(dump_pickle_bytes(self.get_booster(), self.sklearn_state_params()))

    @classmethod
    def load_pickle(cls, path) -> "GBDTClassifier":
        from pathlib import Path
        from .booster import load_pickle_bytes

        st, bst = load_pickle_bytes(Path(path).read_bytes())
        kw = {k: st.get(k) for k in cls._param_names if k in st and k not in ("use_label_encoder",)}
        if isinstance(kw.get("scale_pos_weight"), np.floating):
            kw["scale_pos_weight"] = float(kw["scale_pos_weight"])
        m = cls(**kw)
        m._Booster = bst
        m.classes_ = np.array([0, 1])
        m.n_classes_ = 2
        m.n_features_in_ = bst.num_feature
        if bst.feature_names:
            m.feature_names_in_ = np.array(bst.feature_names, dtype=object)
        return m

    def save_model(self, path) -> None:
        self.get_booster().save_model(path)

    def load_model(self, path) -> None:
        self._Booster = Booster.load_model(path)
        self.classes_ = np.array([0, 1])
        self.n_classes_ = 2


# XGBoost-compatible alias used by the reference-shaped CLIs
XGBClassifier = GBDTClassifier
