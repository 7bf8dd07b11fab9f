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

FLT_MAX = float(np.finfo(np.float32).max)
MAX_BINS = 256        # bins of a feature without missing values (uint8 codes 0..255)
MAX_BINS_U8 = 255     # bins of a feature with missing values (code 255 = missing)
WEIGHT_SCALE = 1 << 20


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
