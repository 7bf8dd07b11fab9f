"""Weighted quantile sketch -> per-feature cut points (K12 in SURVEY.md §2.4).

Replaces XGBoost's weighted-quantile sketch (``max_bin=256``, ``sketch_ratio=2`` in the reference
checkpoint Config) that ``XGBClassifier.fit`` runs before building ``GHistIndexMatrix``
(reference: src/model_train_test/model_tree_train_test.py:111-118,159 -> ``tree_method=hist``).

Semantics (identical on CPU and GPU -- only sort, compare, gather and INTEGER arithmetic, so a
sample yields bit-identical cuts on either device and on any number of ranks):

* cuts live in a ``[F, 256]`` float32 table; ``nbins[f]`` entries are used and the last used entry is
  the sentinel ``FLT_MAX``. ``bin(x) = #{cuts <= x}`` clamped to ``nbins-1``; NaN is the missing bin.
* up to ``maxb_f = min(max_bin, 256)`` bins for a feature without missing values, ``min(max_bin, 255)``
  for one with them: bins are uint8 and code 255 is the missing bin of features that have missing
  values (a 256-bin feature never sees a NaN, so its code 255 is the real bin 255; every split on it
  is learnt with ``default_left = 0``, so the trainer's "missing" branch for code 255 coincides with
  the value branch -- see csrc/gbdt.hip HistLanes.full).
* a feature with ``k <= maxb_f`` distinct sample values gets one bin per value: cuts are the
  distinct values ``u_1..u_{k-1}`` (value ``u_i`` lands in bin ``i``);
* otherwise cuts are weighted quantiles: with the sample sorted by value and integer weights
  ``w_i`` (cumulative ``C_i``, total ``W``), cut ``j`` (``j = 1..maxb_f-1``) is the first value whose
  ``C_i * maxb_f > j * W``, de-duplicated and strictly above the minimum. With unit weights this is
  the order statistic ``x[floor(j*n/maxb_f)]``.

Weights: XGBoost's ``hist`` updater sketches with the SAMPLE weights (``GHistIndexMatrix`` is built
from ``HistBatch(max_bin)``; only ``approx`` passes the gradient hessians), and ``scale_pos_weight``
lives in the objective, not in the sample weights -- so the reference's cuts are sample-weighted
(unweighted without ``sample_weight``). That is the default (``sketch_weight="sample"``).
``sketch_weight="hessian"`` weights each row by its first-round hessian ``p0(1-p0) * w * spw^y``;
``p0`` is the same for every row at round 0, so this is ``w * spw^y`` up to a constant (XGBoost's
``approx`` semantics). Weights are quantised to integers (``round(w / w_max * 2^20)``) so the
cumulative sums are exact and device-independent.

Sampling: ``sample_stride`` picks rows whose GLOBAL index is a multiple of ``ceil(N/sketch_rows)``,
so every rank of a data-parallel job contributes a disjoint part of the same global sample and the
cuts do not depend on the number of ranks. For jobs whose sample would be too large to all-gather,
:class:`QuantileSummary` is a mergeable per-rank summary (``merge`` is exact for the values it keeps,
and the cuts of merged summaries agree with the exact weighted quantiles within the summary's rank
error).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from ..config import knob

FLT_MAX = float(np.finfo(np.float32).max)
MAX_BINS = 256        # bins of a feature without missing values (uint8 codes 0..255)
MAX_BINS_U8 = 255     # bins of a feature with missing values (code 255 = missing)
WEIGHT_SCALE = 1 << 20
# rows of the strided sample whose order statistics bound the exact device sketch's buckets (any sample
# gives the same cuts; <= 32768 rows per feature sort in LDS in one kernel, csrc/sketch.hip)
BOUNDARY_SAMPLE_ROWS = 1 << 15


def sample_stride(n_global: int, sketch_rows: int) -> int:
    if sketch_rows <= 0 or n_global <= sketch_rows:
        return 1
    return int(math.ceil(n_global / sketch_rows))


def local_sample(X: torch.Tensor, row_offset: int, stride: int) -> torch.Tensor:
    """Rows of the local shard ``X`` whose global index is a multiple of ``stride``."""
    if stride == 1:
        return X
    first = (-row_offset) % stride
    return X[first::stride]


def quantize_weights(w: torch.Tensor | None, n: int, device) -> torch.Tensor:
    """Integer sketch weights (int64): ``round(w / max(w) * 2^20)``, or ones when ``w`` is None."""
    if w is None:
        return torch.ones(n, dtype=torch.int64, device=device)
    wd = w.to(device=device, dtype=torch.float64).reshape(-1)
    if wd.numel() == 0:
        return torch.zeros(0, dtype=torch.int64, device=device)
    if bool((wd < 0).any()) or not bool(torch.isfinite(wd).all()):
        raise ValueError("sketch weights must be finite and >= 0")
    m = float(wd.max())
    if m <= 0:
        return torch.ones(n, dtype=torch.int64, device=device)
    return torch.round(wd * (WEIGHT_SCALE / m)).to(torch.int64)


def feature_max_bins(max_bin: int, has_missing: torch.Tensor) -> torch.Tensor:
    """Per-feature bin budget: 256 (capped by max_bin) without missing values, else 255."""
    mb = int(max_bin)
    if mb < 2:
        raise ValueError("max_bin must be >= 2")
    full = min(mb, MAX_BINS)
    miss = min(mb, MAX_BINS_U8)
    return torch.where(has_missing.to(torch.bool), torch.tensor(miss, device=has_missing.device),
                       torch.tensor(full, device=has_missing.device)).to(torch.int64)


def _row_cumsum(x: torch.Tensor, block: int = 1024) -> torch.Tensor:
    """Inclusive int64 prefix sums along dim 1 of a [F, S] tensor, as a two-level scan over blocks of
    ``block`` columns (torch's single-pass scan of a few long rows ran at 0.6 ms for 20 x 2^18 on the
    GPU: one block per row). Integer arithmetic: identical to ``torch.cumsum(x, 1)``."""
    F, S = x.shape
    x = x.to(torch.int64)
    if S <= 4 * block:
        return torch.cumsum(x, 1)
    nb = -(-S // block)
    pad = nb * block - S
    xb = torch.nn.functional.pad(x, (0, pad)).view(F, nb, block)
    inner = torch.cumsum(xb, 2)
    base = torch.cumsum(inner[:, :, -1], 1) - inner[:, :, -1]                   # exclusive block prefixes
    return (inner + base[:, :, None]).view(F, nb * block)[:, :S]


def compute_cuts(sample: torch.Tensor, max_bin: int = 256, weights: torch.Tensor | None = None,
                 has_missing: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """Cut table ``[F, 256]`` float32 and ``nbins [F]`` int32 from a ``[S, F]`` float32 sample.

    ``weights`` ([S], >= 0, optional): per-row sketch weights (see module doc). ``has_missing``
    ([F] bool): whether each feature has missing values in the FULL data (default: in the sample);
    it decides between 255 and 256 bins. Runs on the sample's device (rocPRIM radix sort through
    ``torch.sort`` on GPU)."""
    S, F = sample.shape
    dev = sample.device
    if has_missing is None:
        has_missing = torch.isnan(sample).any(0) if S else torch.zeros(F, dtype=torch.bool, device=dev)
    has_missing = has_missing.to(dev)
    maxb = feature_max_bins(max_bin, has_missing)                              # [F] int64
    if S == 0:
        return (torch.full((F, 256), FLT_MAX, dtype=torch.float32, device=dev),
                torch.ones(F, dtype=torch.int32, device=dev))
    # feature-major first: one contiguous segment per feature for the segmented sort
    srt = torch.sort(sample.to(torch.float32).t().contiguous(), dim=1)         # NaN last
    xs = srt.values                                                            # [F, S]
    valid = ~torch.isnan(xs)
    cnt = valid.sum(1)                                                          # [F]
    dflag = valid.clone()
    dflag[:, 1:] &= xs[:, 1:] != xs[:, :-1]
    nd = dflag.sum(1)                                                           # distinct count
    rank = _row_cumsum(dflag) - 1
    exact = nd <= maxb
    # Both paths are computed for every feature and selected per feature after, and the cut slots are
    # written by scatters into a trash column 256 instead of nonzero() gathers: no host synchronisation
    # (each one cost a device round trip inside the timed fit; 10M-row bench sketch 3.2 ms before).
    trash = torch.full((F, 257), FLT_MAX, dtype=torch.float32, device=dev)

    # exact path: one bin per distinct value (slot rank - 1 <= 254 for the distinct values of rank >= 1)
    ex = exact[:, None] & dflag & (rank >= 1)
    cuts_ex = trash.clone().scatter_(1, torch.where(ex, rank - 1, 256), xs)
    nb_ex = torch.where(nd > 0, nd, torch.ones_like(nd))

    # weighted-quantile path
    wq = quantize_weights(weights, S, dev)                                      # [S] int64
    ws = wq[srt.indices] * valid                                                # [F, S], 0 for NaN
    cum = _row_cumsum(ws)                                                       # exact int64
    W = cum[:, -1]                                                              # [F]
    k = torch.arange(1, MAX_BINS, device=dev, dtype=torch.int64)                # j = 1..255
    # first i with cum_i * maxb > j * W  ==  searchsorted(cum * maxb, j * W, right)
    idx = torch.searchsorted((cum * maxb[:, None]).contiguous(), (k[None, :] * W[:, None]).contiguous(),
                             right=True)
    idx = torch.minimum(idx, (cnt - 1).clamp(min=0)[:, None])
    q = xs.gather(1, idx)                                                       # [F, 255]
    inb = k[None, :] < maxb[:, None]                                            # j < maxb_f
    keep = inb & (q > xs[:, :1])
    keep[:, 1:] &= q[:, 1:] != q[:, :-1]
    pos = torch.cumsum(keep.to(torch.int64), 1) - 1
    cuts_q = trash.scatter_(1, torch.where(keep, pos, 256), q)
    nbq = keep.sum(1) + 1
    cuts = torch.where(exact[:, None], cuts_ex[:, :256], cuts_q[:, :256]).contiguous()
    nb = torch.where(exact, nb_ex, nbq)
    # sentinel in the last used slot
    cuts.scatter_(1, (nb - 1).clamp(min=0)[:, None], FLT_MAX)
    # -0.0 and +0.0 sort as equal, so which one a cut inherits depends on the sort implementation
    # (CPU vs rocPRIM); canonicalise so model files are byte-identical across devices.
    cuts = cuts + 0.0
    return cuts, nb.to(torch.int32)


def weighted_quantile_cuts_np(x: np.ndarray, w: np.ndarray | None, maxb: int) -> np.ndarray:
    """NumPy oracle of one feature's quantile-path cuts (float32 values, float weights)."""
    x = np.asarray(x, dtype=np.float32)
    ok = ~np.isnan(x)
    order = np.argsort(x, kind="stable")
    order = order[ok[order]]
    xs = x[order]
    if w is None:
        wq = np.ones(len(x), dtype=np.int64)
    else:
        wd = np.asarray(w, dtype=np.float64)
        wq = np.round(wd * (WEIGHT_SCALE / wd.max())).astype(np.int64)
    cum = np.cumsum(wq[order])
    W = int(cum[-1])
    out = []
    for j in range(1, maxb):
        i = int(np.searchsorted(cum * maxb, j * W, side="right"))
        i = min(i, len(xs) - 1)
        v = xs[i]
        if v > xs[0] and (not out or v != out[-1]):
            out.append(v)
    return np.asarray(out, dtype=np.float32)


class QuantileSummary:
    """Mergeable weighted quantile summary of one rank's rows (all features), for data-parallel jobs
    whose global sample is too large to all-gather (SURVEY.md §2.7 "all-gather quantile summaries").

    Per feature it keeps at most ``size`` (value, weight) entries: the sorted distinct values with
    their summed integer weights, pruned by cumulative weight to evenly spaced ranks (each kept value
    carries the weight of the values folded into it). ``merge`` concatenates summaries and re-prunes;
    ``cuts`` runs the same weighted-quantile rule as :func:`compute_cuts` on the merged entries.
    Rank error of a prune: at most ``W / size`` per step, so cuts from summaries of ``size >= 8 *
    max_bin`` stay within ~1/8 bin of the exact weighted quantiles."""

    def __init__(self, values: list[np.ndarray], weights: list[np.ndarray], has_missing: np.ndarray):
        self.values, self.weights, self.has_missing = values, weights, np.asarray(has_missing, dtype=bool)

    @staticmethod
    def _prune(v: np.ndarray, w: np.ndarray, size: int) -> tuple[np.ndarray, np.ndarray]:
        if len(v) <= size:
            return v, w
        cum = np.cumsum(w)
        W = cum[-1]
        # group boundaries at evenly spaced cumulative weight; each group is represented by its
        # LAST value with the group's total weight (keeps the max value exactly)
        grp = np.minimum((cum * size - 1) // W, size - 1) if W > 0 else np.zeros(len(v), dtype=np.int64)
        last = np.r_[grp[1:] != grp[:-1], True]
        gw = np.add.reduceat(w, np.r_[0, np.nonzero(last)[0][:-1] + 1])
        return v[last], gw.astype(np.int64)

    @classmethod
    def build(cls, X: np.ndarray, w: np.ndarray | None = None, size: int = 2048,
              w_max: float | None = None) -> "QuantileSummary":
        """Summary of the rows ``X`` [n, F]. ``w_max``: the weight that maps to ``2^20`` integer units.
        Summaries that are merged must share it (the GLOBAL max weight under data parallelism --
        one unit must mean the same weight on every rank); default: the local max."""
        X = np.asarray(X, dtype=np.float32)
        n, F = X.shape
        if w is None:
            wq = np.ones(n, dtype=np.int64)
        else:
            wd = np.asarray(w, np.float64).reshape(-1)
            scale = w_max if w_max is not None else (float(wd.max()) if wd.size else 1.0)
            wq = np.round(wd * (WEIGHT_SCALE / max(float(scale), 1e-300))).astype(np.int64)
        vals, wts, miss = [], [], np.zeros(F, dtype=bool)
        for f in range(F):
            x = X[:, f]
            ok = ~np.isnan(x)
            miss[f] = not ok.all()
            u, inv = np.unique(x[ok], return_inverse=True)
            ws = np.bincount(inv, weights=wq[ok], minlength=len(u)).astype(np.int64)
            v2, w2 = cls._prune(u, ws, size)
            vals.append(v2)
            wts.append(w2)
        return cls(vals, wts, miss)

    @classmethod
    def merge(cls, parts: list["QuantileSummary"], size: int = 2048) -> "QuantileSummary":
        F = len(parts[0].values)
        vals, wts = [], []
        for f in range(F):
            v = np.concatenate([p.values[f] for p in parts])
            w = np.concatenate([p.weights[f] for p in parts])
            u, inv = np.unique(v, return_inverse=True)
            ws = np.bincount(inv, weights=w, minlength=len(u)).astype(np.int64)
            v2, w2 = cls._prune(u, ws, size)
            vals.append(v2)
            wts.append(w2)
        return cls(vals, wts, np.any([p.has_missing for p in parts], axis=0))

    def cuts(self, max_bin: int = 256) -> tuple[np.ndarray, np.ndarray]:
        F = len(self.values)
        cuts = np.full((F, 256), np.float32(FLT_MAX), dtype=np.float32)
        nb = np.ones(F, dtype=np.int32)
        for f in range(F):
            maxb = min(max_bin, MAX_BINS_U8 if self.has_missing[f] else MAX_BINS)
            v, w = self.values[f], self.weights[f]
            if len(v) == 0:
                continue
            if len(v) <= maxb:
                c = v[1:]
            else:
                cum = np.cumsum(w)
                W = int(cum[-1])
                out = []
                for j in range(1, maxb):
                    i = min(int(np.searchsorted(cum * maxb, j * W, side="right")), len(v) - 1)
                    if v[i] > v[0] and (not out or v[i] != out[-1]):
                        out.append(v[i])
                c = np.asarray(out, dtype=np.float32)
            cuts[f, : len(c)] = c
            nb[f] = len(c) + 1
            cuts[f, nb[f] - 1] = np.float32(FLT_MAX)
        return cuts + np.float32(0.0), nb

    def to_arrays(self) -> tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Flat (offsets, values, weights, has_missing) for a collective."""
        off = np.r_[0, np.cumsum([len(v) for v in self.values])].astype(np.int64)
        return off, np.concatenate(self.values).astype(np.float32), np.concatenate(self.weights), self.has_missing

    @classmethod
    def from_arrays(cls, off, vals, wts, miss) -> "QuantileSummary":
        return cls([vals[off[f]:off[f + 1]] for f in range(len(off) - 1)],
                   [wts[off[f]:off[f + 1]] for f in range(len(off) - 1)], miss)


def device_summary(X: torch.Tensor, w: torch.Tensor | None = None, size: int = 8192,
                   w_max: float | None = None) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """:class:`QuantileSummary` arrays (offsets, values, int64 weights) of EVERY row of ``X`` [n, F],
    computed on ``X``'s device: one batched sort per feature column (rocPRIM via ``torch.sort``), the
    distinct values' integer weights by a segmented sum, and the same cumulative-weight prune as
    :meth:`QuantileSummary._prune` -- so only ``<= size`` entries per feature leave the device. The
    full-data sketch of a data-parallel fit merges these per-rank summaries (``w_max`` = the global
    max weight, see :meth:`QuantileSummary.build`)."""
    n, F = X.shape
    dev = X.device
    if w is None:
        wq = torch.ones(n, dtype=torch.int64, device=dev)
    else:
        wd = w.to(device=dev, dtype=torch.float64).reshape(-1)
        scale = w_max if w_max is not None else (float(wd.max()) if wd.numel() else 1.0)
        wq = torch.round(wd * (WEIGHT_SCALE / max(float(scale), 1e-300))).to(torch.int64)
    offs, vals, wts = [0], [], []
    for f in range(F):
        x = X[:, f].to(torch.float32)
        ok = ~torch.isnan(x)
        xv = x[ok]
        if xv.numel() == 0:
            offs.append(offs[-1])
            continue
        xs, order = torch.sort(xv)
        ws = wq[ok][order]
        new = torch.ones_like(xs, dtype=torch.bool)
        new[1:] = xs[1:] != xs[:-1]
        gid = torch.cumsum(new.to(torch.int64), 0) - 1
        u = xs[new]
        uw = torch.zeros(u.numel(), dtype=torch.int64, device=dev).scatter_add_(0, gid, ws)
        if u.numel() > size:  # prune by cumulative weight (QuantileSummary._prune, on the device)
            cum = torch.cumsum(uw, 0)
            W = int(cum[-1])
            grp = torch.clamp((cum * size - 1) // max(W, 1), max=size - 1) if W > 0 else torch.zeros_like(cum)
            last = torch.ones_like(grp, dtype=torch.bool)
            last[:-1] = grp[1:] != grp[:-1]
            cl = cum[last]
            gw = torch.diff(cl, prepend=torch.zeros(1, dtype=torch.int64, device=dev))
            u, uw = u[last], gw
        vals.append(u.cpu().numpy())
        wts.append(uw.cpu().numpy())
        offs.append(offs[-1] + int(u.numel()))
    off = np.asarray(offs, dtype=np.int64)
    v = np.concatenate(vals).astype(np.float32) if vals else np.zeros(0, np.float32)
    ww = np.concatenate(wts).astype(np.int64) if wts else np.zeros(0, np.int64)
    return off, v, ww


def bin_matrix_host(X: np.ndarray, cuts: np.ndarray, nbins: np.ndarray) -> np.ndarray:
    """NumPy binning (oracle of ``cobalt_bin_matrix``): uint8 [N, F], NaN -> 255."""
    X = np.asarray(X, dtype=np.float32)
    N, F = X.shape
    out = np.empty((N, F), dtype=np.uint8)
    for f in range(F):
        nb = int(nbins[f])
        c = cuts[f, :nb]
        b = np.searchsorted(c, X[:, f], side="right")
        b = np.minimum(b, nb - 1)
        b = np.where(np.isnan(X[:, f]), 255, b)
        out[:, f] = b.astype(np.uint8)
    return out


def full_bin_mask(nbins) -> np.ndarray:
    """Features whose uint8 code 255 is a real bin (256 bins, no missing values)."""
    return np.asarray(nbins) >= MAX_BINS


def _sk_lib():
    from .. import _native

    lib = _native.lib()
    if not getattr(lib, "_sk_declared", False):
        import ctypes

        V, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        lib.cobalt_sk_hist.restype = I
        lib.cobalt_sk_hist.argtypes = [V, I64, I64, I, V, V, V, I, V, V, V, V, V]
        lib.cobalt_sk_gather.restype = I
        lib.cobalt_sk_gather.argtypes = [V, I64, I64, I, V, V, V, V, V, I, V, V, I, V, V]
        lib.cobalt_sk_select.restype = I
        lib.cobalt_sk_select.argtypes = [V, V, V, I, V, V, V, V, V, V, V, V, V]
        lib.cobalt_sk_transpose.restype = I
        lib.cobalt_sk_transpose.argtypes = [V, I64, I, V, V]
        lib.cobalt_sk_exact.restype = I
        lib.cobalt_sk_exact.argtypes = [I, V, V, V, V, V, V, V, V, V, V]
        lib.cobalt_sk_bounds_build.restype = I
        lib.cobalt_sk_bounds_build.argtypes = [V, I, I, V, V, V]
        lib.cobalt_sk_reduce.restype = I
        lib.cobalt_sk_reduce.argtypes = [V, V, V, I, I, V, V, V, V, V]
        lib.cobalt_sk_plan_layout.restype = I
        lib.cobalt_sk_plan_layout.argtypes = [I, V]
        lib.cobalt_sk_plan.restype = I
        lib.cobalt_sk_plan.argtypes = [I, V, V, V, V, V, V, V, V, V]
        lib.cobalt_sk_blkoff.restype = I
        lib.cobalt_sk_blkoff.argtypes = [I, V, I, V, I, V, V, V]
        lib.cobalt_sk_assemble.restype = I
        lib.cobalt_sk_assemble.argtypes = [I, V, V, V, V, V, V, V, V, V]
        lib.cobalt_sk_sample_bounds.restype = I
        lib.cobalt_sk_sample_bounds.argtypes = [V, I64, I64, I, I, V, V, V]
        for name in ("cobalt_sk_bounds", "cobalt_sk_buckets", "cobalt_sk_sort_cap", "cobalt_sk_sample_cap"):
            getattr(lib, name).restype = I
            getattr(lib, name).argtypes = []
        lib._sk_declared = True
    return lib


def _ptr(t):
    return None if t is None else int(t.data_ptr())


def device_exact_cuts(X: torch.Tensor, max_bin: int = 256, weights: torch.Tensor | None = None,
                      has_missing: torch.Tensor | None = None, *, dist=None, row_offset: int = 0,
                      n_rows_global: int | None = None, w_max: float | None = None,
                      sample_rows: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """:func:`compute_cuts` over EVERY row of ``X`` [N, F] (a CUDA tensor), bit for bit, without sorting
    the rows (csrc/sketch.hip): sample boundaries split each feature's value axis into buckets, one
    pass histograms the rows per bucket, the target ranks are located by prefix sums, and only the
    rows of the few buckets that hold a target are gathered and sorted (in LDS, per bucket).

    Under data parallelism (``dist``) every rank passes its shard and the ranks exchange four
    fixed-layout SUM all-reduces on the device (``dist.device_allreduce``; no size exchanges, no
    padding): (1) the global strided sample, placed by global sample index, with the missing-value flags
    and the weight scale; (2) the bucket counts (+ weight sums), summed, and every rank's value range by
    rank slot; (2b) every rank's rows of the few selected bucket segments, by rank slot -- where its
    candidates go inside each global segment; (3) the candidates, written straight into the global
    segment layout. Every rank then computes the full data's cuts.
    ``w_max`` scales the weights (default: the global max)."""
    import os

    N, F = X.shape
    dev = X.device
    timing = knob("COBALT_SK_TIMING") == "1"  # per-stage times (device-synchronised) to stderr
    marks = []

    def mark(name):
        if timing:
            torch.cuda.synchronize(dev)
            marks.append((name, __import__("time").perf_counter()))
    mark("start")
    world = dist.world if dist is not None else 1
    n_glob = n_rows_global if n_rows_global is not None else N
    X = X.to(torch.float32)
    stride = sample_stride(n_glob, BOUNDARY_SAMPLE_ROWS if sample_rows is None else sample_rows)
    samp = local_sample(X, row_offset, stride)
    wd = weights.to(device=dev, dtype=torch.float64).reshape(-1) if weights is not None else None
    if wd is not None:
        if bool((wd < 0).any()) or not bool(torch.isfinite(wd).all()):
            raise ValueError("sketch weights must be finite and >= 0")
        if w_max is None:
            w_max = float(wd.max()) if wd.numel() else 0.0
    if world > 1:
        # collective 1: the global sample + missing flags + weight scale (folded into the one exchange)
        samp, has_missing, w_max = _global_sample(dist, dev, X, samp, row_offset, stride, n_glob, has_missing,
                                                  w_max if wd is not None else None)
    elif has_missing is None:
        has_missing = torch.isnan(X).any(0) if N else torch.zeros(F, dtype=torch.bool, device=dev)
    wq = None
    if wd is not None:
        scale = WEIGHT_SCALE / w_max if w_max and w_max > 0 else 0.0
        wq = (torch.round(wd * scale) if scale else torch.ones_like(wd)).to(torch.int32).contiguous()
    return _exact_core(lambda: iter([(X, wq)]), True, N, F, dev, samp, has_missing, max_bin, dist, wq is not None,
                       mark, marks, timing)


def _global_sample(dist, dev, X, samp, row_offset: int, stride: int, n_glob: int, has_missing, w_max):
    """Collective 1 of the data-parallel exact sketch: ONE int32 SUM all-reduce of a fixed layout --
    the global strided sample (row g of the data, g % stride == 0, at sample index g // stride: the
    ranks' rows are disjoint, so the sum of bit patterns IS the sample, NaN and -0.0 included), then
    the F missing-value counts (unless ``has_missing`` is given), then every rank's float64 ``w_max``
    bits in its own two slots. Returns (global sample [S, F], has_missing [F] bool, global w_max)."""
    R, r = dist.world, dist.rank
    N, F = X.shape
    S = (n_glob - 1) // stride + 1 if n_glob > 0 else 0
    first = (-row_offset) % stride
    g0 = (row_offset + first) // stride
    ns = samp.shape[0]
    buf = torch.zeros(S * F + F + 2 * R, dtype=torch.int32, device=dev)
    if ns:
        buf[g0 * F:(g0 + ns) * F] = samp.contiguous().view(torch.int32).reshape(-1)
    if has_missing is None and N:
        buf[S * F:S * F + F] = torch.isnan(X).any(0).to(torch.int32)
    if w_max is not None:
        buf[S * F + F + 2 * r:S * F + F + 2 * r + 2] = torch.tensor([float(w_max)], dtype=torch.float64).view(
            torch.int32).to(dev)
    dist.device_allreduce(buf, "sum")
    gsamp = buf[:S * F].view(torch.float32).reshape(S, F)
    hm = has_missing.to(dev).to(torch.bool) if has_missing is not None else buf[S * F:S * F + F] > 0
    wm = None
    if w_max is not None:
        wm = float(buf[S * F + F:].cpu().view(torch.float64).max())
    return gsamp, hm, wm


def _fkey64(v: torch.Tensor) -> torch.Tensor:
    """Order-preserving integer key of float32 values (int64, ascending with the value; -0 < +0)."""
    b = v.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return torch.where(b >= 0x80000000, 0xFFFFFFFF - b, b + 0x80000000)


def _fkey64_inv(k: torch.Tensor) -> torch.Tensor:
    b = torch.where(k >= 0x80000000, k - 0x80000000, 0xFFFFFFFF - k)
    return (b - ((b >= 0x80000000).to(torch.int64) << 32)).to(torch.int32).view(torch.float32)


def _allreduce_buckets(dist, dev, cnt_loc, w_loc, vmin, vmax):
    """Collective 2 of the data-parallel exact sketch: ONE int64 SUM all-reduce of the bucket counts
    (and weight sums), summed in place -- F x NB cells whatever the rank count -- plus every rank's value
    range as order keys in its own 2F slots. Returns the global counts, weight sums, min / max. (Each
    rank's offset inside the few selected buckets comes from collective 2b, _segment_offsets: per-rank
    slots of the whole F x NB table would grow the message with the rank count -- ~111 MB per rank at 8
    ranks for the 106-feature RFE fits with weights.)"""
    R, r = dist.world, dist.rank
    F, NB = cnt_loc.shape
    FN = F * NB
    nw = FN if w_loc is not None else 0
    buf = torch.zeros(FN + nw + R * 2 * F, dtype=torch.int64, device=dev)
    buf[:FN] = cnt_loc.reshape(-1)
    if w_loc is not None:
        buf[FN:FN + nw] = w_loc.reshape(-1)
    base = FN + nw + r * 2 * F
    buf[base:base + F] = _fkey64(vmin)
    buf[base + F:base + 2 * F] = _fkey64(vmax)
    dist.device_allreduce(buf, "sum")
    cnt_h = buf[:FN].reshape(F, NB)
    w_h = buf[FN:FN + nw].reshape(F, NB) if w_loc is not None else None
    keys = buf[FN + nw:].reshape(R, 2 * F)
    vmin_g = _fkey64_inv(keys[:, :F].amin(0))
    vmax_g = _fkey64_inv(keys[:, F:].amax(0))
    return cnt_h, w_h, vmin_g, vmax_g


def _segment_offsets(dist, dev, loc_sizes):
    """Collective 2b: this rank's rows of every selected bucket segment (the same segments on every rank:
    the selection depends only on the global counts) in its own slot of one R x nseg int64 SUM
    all-reduce; returns the rows of the lower ranks per segment -- where this rank's candidates start
    inside the segment's global layout. Issued also when nseg == 0 (one cell), so every data-parallel
    sketch runs the same number of collectives."""
    R, r = dist.world, dist.rank
    nseg = int(loc_sizes.numel())
    buf = torch.zeros(max(R * nseg, 1), dtype=torch.int64, device=dev)
    if nseg:
        buf[r * nseg:(r + 1) * nseg] = loc_sizes
    dist.device_allreduce(buf, "sum")
    if not nseg:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    per = buf.reshape(R, nseg)
    return (torch.cumsum(per, 0) - per)[r]


def stream_exact_cuts(chunks, n_rows: int, n_features: int, samp: torch.Tensor, has_missing: torch.Tensor,
                      max_bin: int = 256, *, dist=None, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """:func:`device_exact_cuts` of data that arrives in chunks (``chunks()`` yields CUDA [n_c, F]
    float32 tensors; it is iterated twice): every row sketched, bit for bit the in-core cuts, with
    one chunk on the device at a time. ``samp``: a (global, strided) sample for the bucket boundaries;
    unweighted."""
    import os

    dev = torch.device(device)
    timing = knob("COBALT_SK_TIMING") == "1"
    marks = []

    def mark(name):
        if timing:
            torch.cuda.synchronize(dev)
            marks.append((name, __import__("time").perf_counter()))
    mark("start")
    return _exact_core(lambda: ((c, None) for c in chunks()), False, int(n_rows), int(n_features), dev, samp,
                       has_missing, max_bin, dist, False, mark, marks, timing)


def _sk_transpose(lib, X, stream):
    """[n, F] float32 (CUDA) -> feature-major [F, n]."""
    from .. import _native

    N, F = X.shape
    if X.is_contiguous() and 0 < F <= 32 and N:
        XT = torch.empty((F, N), dtype=torch.float32, device=X.device)
        _native.check(lib.cobalt_sk_transpose(X.data_ptr(), N, F, XT.data_ptr(), stream), "cobalt_sk_transpose")
        return XT
    return X.t().contiguous()


# the device plan's arrays, in the order of csrc/sketch.hip SkArr (their int64 word offsets inside the
# plan workspace come from cobalt_sk_plan_layout)
_PLAN_ARRS = ("sel", "fstat", "fbase", "summary", "q0", "thr", "pre", "tb", "need", "slot", "seg_feat", "seg_bucket",
              "loc_sizes", "glob_sizes", "loc_off", "glob_off", "tgt_off", "want", "ndist", "tpos", "tprefix", "tthr",
              "tmaxb")
_plan_offsets: dict = {}


def _plan_layout(lib, F: int) -> list:
    off = _plan_offsets.get(F)
    if off is None:
        import ctypes

        buf = (ctypes.c_int64 * (len(_PLAN_ARRS) + 1))()
        n = lib.cobalt_sk_plan_layout(F, ctypes.addressof(buf))
        if n != len(_PLAN_ARRS):
            raise RuntimeError(f"cobalt_sk_plan_layout: {n} arrays, expected {len(_PLAN_ARRS)}")
        off = _plan_offsets[F] = list(buf)
    return off


def _exact_core(chunks, single, N, F, dev, samp, has_missing, max_bin, dist, weighted, mark, marks, timing):
    """The bucketed exact sketch over the rows of ``chunks()`` ((X_chunk, int32 weights or None)
    pairs; ``single``: one chunk, its transpose and pass-1 slabs are reused by the gather).

    Everything between the passes runs on the device (csrc/sketch.hip: k_sk_bounds, k_sk_reduce,
    k_sk_plan1-3, k_sk_blkoff, k_sk_assemble) with ONE host read -- the plan's sizes, which the candidate
    buffers and the collectives need; only the rare fallbacks (a segment beyond the LDS sort) run torch
    code here."""
    import ctypes

    from .. import _native

    lib = _sk_lib()
    if F == 0:
        return (torch.empty((0, 256), dtype=torch.float32, device=dev), torch.empty(0, dtype=torch.int32, device=dev))
    world = dist.world if dist is not None else 1
    NBND, NB, CAP = lib.cobalt_sk_bounds(), lib.cobalt_sk_buckets(), lib.cobalt_sk_sort_cap()
    stream = _native.stream_handle()
    chk = _native.check
    maxb = feature_max_bins(max_bin, has_missing.to(dev)).contiguous()              # [F] int64

    # 1. boundaries: <= NBND - 1 distinct values of the global strided sample -- sorted in LDS straight
    # from the (strided) sample view (k_sk_sample_bounds), or torch.sort + k_sk_bounds beyond its cap
    S = samp.shape[0]
    bounds = torch.empty((F, NBND), dtype=torch.float32, device=dev)
    m = torch.empty(F, dtype=torch.int32, device=dev)
    if 0 < S <= lib.cobalt_sk_sample_cap():
        sp = samp if samp.dtype == torch.float32 else samp.to(torch.float32)
        chk(lib.cobalt_sk_sample_bounds(sp.data_ptr(), sp.stride(0), sp.stride(1), S, F, bounds.data_ptr(),
                                        m.data_ptr(), stream), "cobalt_sk_sample_bounds")
        mark("sort")
    elif S:
        sv = torch.sort((samp.t() + 0.0).contiguous(), dim=1).values                 # [F, S], NaN last
        mark("sort")
        chk(lib.cobalt_sk_bounds_build(sv.data_ptr(), F, S, bounds.data_ptr(), m.data_ptr(), stream),
            "cobalt_sk_bounds_build")
    else:
        bounds.fill_(float("inf"))
        m.zero_()
    mark("bounds")

    # 2. bucket histograms (row counts; weight sums when weighted) + min / max valid value, per chunk;
    # the slabs are summed on the device (k_sk_reduce)
    def chunk_hist(XT, n, wq, bid=None):
        nblk = max(1, min(64, -(-n // 65536)))
        cnt_slab = torch.empty((nblk, F, NB), dtype=torch.int32, device=dev)
        w_slab = torch.empty((nblk, F, NB), dtype=torch.int64, device=dev) if wq is not None else None
        bmm = torch.empty((nblk, F, 2), dtype=torch.float32, device=dev)
        if n:
            rc = lib.cobalt_sk_hist(XT.data_ptr(), n, n, F, _ptr(wq), bounds.data_ptr(), m.data_ptr(), nblk,
                                    cnt_slab.data_ptr(), _ptr(w_slab), bmm.data_ptr(), _ptr(bid), stream)
            chk(rc, "cobalt_sk_hist")
        return nblk, cnt_slab, w_slab, bmm

    cnt_loc = torch.zeros((F, NB), dtype=torch.int64, device=dev)
    w_loc = torch.zeros((F, NB), dtype=torch.int64, device=dev) if weighted else None
    vmin = torch.full((F,), float("inf"), dtype=torch.float32, device=dev)
    vmax = torch.full((F,), float("-inf"), dtype=torch.float32, device=dev)
    kept = None
    for Xc, wq in chunks():
        Xc = Xc.to(torch.float32)
        n = Xc.shape[0]
        XT = _sk_transpose(lib, Xc, stream)
        mark("transpose")
        # one chunk (the in-core sketch): pass 1 also keeps every value's bucket, so the candidate pass
        # reads 2 bytes per value instead of searching the boundaries again
        bid = torch.empty((F, n), dtype=torch.int16, device=dev) if single and n else None
        nblk, cnt_slab, w_slab, bmm = chunk_hist(XT, n, wq, bid)
        if n:
            chk(lib.cobalt_sk_reduce(cnt_slab.data_ptr(), _ptr(w_slab), bmm.data_ptr(), nblk, F, cnt_loc.data_ptr(),
                                     _ptr(w_loc), vmin.data_ptr(), vmax.data_ptr(), stream), "cobalt_sk_reduce")
        if single:
            kept = (XT, n, wq, nblk, cnt_slab, bid)
    cnt_h, w_h = cnt_loc, w_loc
    if world > 1:  # collective 2
        cnt_h, w_h, vmin, vmax = _allreduce_buckets(dist, dev, cnt_loc, w_loc, vmin, vmax)
    cnt_h, vmin, vmax = cnt_h.contiguous(), vmin.contiguous(), vmax.contiguous()
    mark("hist")

    # 3. the plan (k_sk_plan1-3): targets j * W / maxb, their buckets (an equal bucket IS the value), the
    # selected open buckets as segments with their local / global offsets; one host read of the sizes
    off = _plan_layout(lib, F)
    ws = torch.empty(off[-1], dtype=torch.int64, device=dev)

    def arr(name, dtype, count):
        k = _PLAN_ARRS.index(name)
        return ws[off[k]:off[k + 1]].view(dtype)[:count]

    summ = (ctypes.c_int64 * 8)()
    chk(lib.cobalt_sk_plan(F, cnt_h.data_ptr(), _ptr(w_h), cnt_loc.data_ptr(), bounds.data_ptr(), maxb.data_ptr(),
                           vmax.data_ptr(), ws.data_ptr(), ctypes.addressof(summ), stream), "cobalt_sk_plan")
    nseg, T, tot_loc, tot_glob, any_unc, nbig_t, nbig_w = (int(x) for x in summ[:7])
    slot = arr("slot", torch.int32, F * NB)
    glob_off = arr("glob_off", torch.int64, nseg + 1)
    mark("targets")

    # 4. candidates: the rows of the selected buckets, per segment (a second walk over the chunks;
    # each block writes at its offset from the chunk's per-block bucket counts, k_sk_blkoff). Data
    # parallel: straight into the GLOBAL segment layout (this rank's rows of segment s start at
    # glob_off[s] + the lower ranks' rows of s), zeros elsewhere, and collective 3 sums the ranks'
    # buffers: values and weights in one int32 buffer [tot | tot].
    if world > 1:
        tot_loc = tot = tot_glob
        cbuf = torch.zeros(max(2 * tot if weighted else tot, 1), dtype=torch.int32, device=dev)
        cval = cbuf[:max(tot, 1)].view(torch.float32)
        cw = cbuf[tot:2 * tot] if weighted else None
        start = glob_off[:-1] + _segment_offsets(dist, dev, arr("loc_sizes", torch.int64, nseg))  # collective 2b
    else:
        cval = torch.empty(max(tot_loc, 1), dtype=torch.float32, device=dev)
        cw = torch.empty(max(tot_loc, 1), dtype=torch.int32, device=dev) if weighted else None
        start = arr("loc_off", torch.int64, nseg + 1)[:-1]
    if nseg and N:
        cursor = start.clone()
        for Xc, wq in (iter([(None, None)]) if single else chunks()):
            bid = None
            if single:
                XT, n, wq, nblk, cnt_slab, bid = kept
            else:
                Xc = Xc.to(torch.float32)
                n = Xc.shape[0]
                XT = _sk_transpose(lib, Xc, stream)
                nblk, cnt_slab, _, _ = chunk_hist(XT, n, wq)
            if not n:
                continue
            blk_off = torch.empty((nblk, nseg), dtype=torch.int64, device=dev)
            chk(lib.cobalt_sk_blkoff(F, ws.data_ptr(), nseg, cnt_slab.data_ptr(), nblk, cursor.data_ptr(),
                                     blk_off.data_ptr(), stream), "cobalt_sk_blkoff")
            rc = lib.cobalt_sk_gather(XT.data_ptr(), n, n, F, _ptr(wq), bounds.data_ptr(), m.data_ptr(),
                                      slot.data_ptr(), blk_off.data_ptr(), nseg, cval.data_ptr(), _ptr(cw), nblk,
                                      _ptr(bid), stream)
            chk(rc, "cobalt_sk_gather")
    if world > 1 and nseg:  # collective 3: every rank's candidates, already in the global layout
        dist.device_allreduce(cbuf, "sum")

    mark("gather")
    # 5. select the open targets from their bucket's sorted candidates (k_sk_select); for the features
    # that may be exact (one bin per distinct value), also their segments' distinct values
    out = torch.empty(max(T, 1), dtype=torch.float32, device=dev)
    ndist = arr("ndist", torch.int32, max(nseg, 1))
    dval = torch.empty_like(cval)
    if nseg and (T or any_unc):
        tgt_off = arr("tgt_off", torch.int32, nseg + 1)
        prefix = arr("tprefix", torch.int64, T)
        tthr = arr("tthr", torch.int64, T)
        tmaxb = arr("tmaxb", torch.int64, T)
        rc = lib.cobalt_sk_select(cval.data_ptr(), _ptr(cw), glob_off.data_ptr(), nseg, tgt_off.data_ptr(),
                                  prefix.data_ptr(), tthr.data_ptr(), tmaxb.data_ptr(), out.data_ptr(),
                                  arr("want", torch.uint8, nseg).data_ptr(), dval.data_ptr(), ndist.data_ptr(), stream)
        chk(rc, "cobalt_sk_select")
        if nbig_t:  # rare: segments beyond the LDS sort with targets -- sorted here
            glob_sizes = arr("glob_sizes", torch.int64, nseg)
            for s in torch.nonzero(glob_sizes > CAP).reshape(-1).tolist():
                t0, t1 = int(tgt_off[s]), int(tgt_off[s + 1])
                if t0 == t1:
                    continue
                o0, o1 = int(glob_off[s]), int(glob_off[s + 1])
                vs, order = torch.sort(cval[o0:o1])
                ws_ = (cw[o0:o1][order].to(torch.int64) if cw is not None else torch.ones_like(order))
                cum = torch.cumsum(ws_, 0)
                key = ((prefix[t0:t1, None] + cum[None, :]) * tmaxb[t0:t1, None]).contiguous()
                i = torch.searchsorted(key, tthr[t0:t1, None].contiguous(), right=True)[:, 0].clamp(max=o1 - o0 - 1)
                out[t0:t1] = vs[i]

    mark("select")
    # 6. the cut tables (k_sk_exact: one bin per distinct value where a feature has <= maxb of them;
    # k_sk_assemble: the quantile path, the choice between them, the sentinel)
    cuts_ex = torch.full((F, 257), FLT_MAX, dtype=torch.float32, device=dev)
    nd = torch.empty(F, dtype=torch.int64, device=dev)
    chk(lib.cobalt_sk_exact(F, cnt_h.data_ptr(), bounds.data_ptr(), slot.data_ptr(), glob_off.data_ptr(),
                            ndist.data_ptr(), dval.data_ptr(), maxb.data_ptr(), cuts_ex.data_ptr(), nd.data_ptr(),
                            stream), "cobalt_sk_exact")
    if nbig_w:  # rare: an exact-candidate feature with a segment beyond the LDS sort -- distinct values here
        uncertain = arr("fstat", torch.int64, 5 * F).view(F, 5)[:, 4] > 0
        nz = cnt_h > 0
        slot2 = slot.view(F, NB)
        for f in torch.nonzero(uncertain & (nd < 0)).reshape(-1).tolist():
            eqnz = nz[f, 1::2][:NBND]
            segs = torch.nonzero(slot2[f] >= 0).reshape(-1)
            parts = [bounds[f][eqnz]]
            for bb in segs.tolist():
                s = int(slot2[f, bb])
                parts.append(cval[int(glob_off[s]):int(glob_off[s + 1])])
            dv = torch.unique(torch.cat(parts))                                            # sorted
            nd[f] = dv.numel()
            if dv.numel() <= int(maxb[f]):
                row = torch.full((257,), FLT_MAX, dtype=torch.float32, device=dev)
                row[: dv.numel() - 1] = dv[1:]
                cuts_ex[f] = row
    cuts = torch.empty((F, 256), dtype=torch.float32, device=dev)
    nbv = torch.empty(F, dtype=torch.int32, device=dev)
    chk(lib.cobalt_sk_assemble(F, ws.data_ptr(), out.data_ptr(), vmin.data_ptr(), maxb.data_ptr(), nd.data_ptr(),
                               cuts_ex.data_ptr(), cuts.data_ptr(), nbv.data_ptr(), stream), "cobalt_sk_assemble")
    mark("assemble")
    if timing:
        import sys

        print("[sketch] " + " ".join(f"{marks[i][0]}={1e3 * (marks[i][1] - marks[i - 1][1]):.3f}ms"
                                     for i in range(1, len(marks))) + f" candidates={tot_loc} segments={nseg}",
              file=sys.stderr)
    return cuts, nbv


