"""Quantile sketch -> per-feature cut points (K12 in SURVEY.md §2.4).

Replaces XGBoost's weighted-quantile sketch (``max_bin=256``, ``sketch_ratio=2`` in the reference
checkpoint Config) that ``XGBClassifier.fit`` runs before building ``GHistIndexMatrix``.

Semantics (identical on CPU and GPU — only sort, compare, gather and integer arithmetic, so a
sample yields bit-identical cuts on either device and on any number of ranks):

* cuts live in a ``[F, 256]`` float32 table; ``nbins[f]`` entries are used and the last used entry is
  the sentinel ``FLT_MAX``. ``bin(x) = #{cuts <= x}`` clamped to ``nbins-1``; NaN is the missing bin.
* a feature with ``k <= max_bins`` distinct sample values gets one bin per value: cuts are the
  distinct values ``u_1..u_{k-1}`` (value ``u_i`` lands in bin ``i``);
* otherwise cuts are the de-duplicated order statistics ``x[floor(j*n/max_bins)]``, ``j=1..max_bins-1``,
  strictly above the minimum.

``max_bins = min(max_bin, 255)``: bin id 255 is reserved for missing values (uint8 storage).
A split at bin ``j`` has threshold ``cuts[f, j]`` (``x < cut`` goes left), exactly XGBoost's
``split_condition`` convention.

Sampling: ``sample_stride`` picks rows whose GLOBAL index is a multiple of ``ceil(N/sketch_rows)``,
so every rank of a data-parallel job contributes a disjoint part of the same global sample.
"""
from __future__ import annotations

import math

import numpy as np
import torch

FLT_MAX = float(np.finfo(np.float32).max)
MAX_BINS_U8 = 255


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


def compute_cuts(sample: torch.Tensor, max_bin: int = 256) -> tuple[torch.Tensor, torch.Tensor]:
    """Cut table ``[F, 256]`` float32 and ``nbins [F]`` int32 from a ``[S, F]`` float32 sample.

    Runs on the sample's device (rocPRIM radix sort through ``torch.sort`` on GPU).
    """
    maxb = int(min(max_bin, MAX_BINS_U8))
    if maxb < 2:
        raise ValueError("max_bin must be >= 2")
    S, F = sample.shape
    dev = sample.device
    cuts = torch.full((F, 256), FLT_MAX, dtype=torch.float32, device=dev)
    if S == 0:
        return cuts, torch.ones(F, dtype=torch.int32, device=dev)
    xs = torch.sort(sample.to(torch.float32), dim=0).values.t().contiguous()  # [F, S], NaN last
    valid = ~torch.isnan(xs)
    cnt = valid.sum(1)                                                          # [F]
    dflag = valid.clone()
    dflag[:, 1:] &= xs[:, 1:] != xs[:, :-1]
    nd = dflag.sum(1)                                                           # distinct count
    rank = torch.cumsum(dflag.to(torch.int64), 1) - 1
    exact = nd <= maxb

    # exact path: one bin per distinct value
    ex = exact[:, None] & dflag & (rank >= 1)
    fi, pi = ex.nonzero(as_tuple=True)
    cuts[fi, rank[fi, pi] - 1] = xs[fi, pi]
    nb = torch.where(nd > 0, nd, torch.ones_like(nd))

    # quantile path
    if bool((~exact).any()):
        k = torch.arange(1, maxb, device=dev, dtype=torch.int64)
        idx = torch.div(k[None, :] * cnt[:, None], maxb, rounding_mode="floor").clamp_(max=S - 1)
        q = xs.gather(1, idx)                                                   # [F, maxb-1]
        keep = q > xs[:, :1]
        keep[:, 1:] &= q[:, 1:] != q[:, :-1]
        pos = torch.cumsum(keep.to(torch.int64), 1) - 1
        qf = (~exact)[:, None] & keep
        fi, pi = qf.nonzero(as_tuple=True)
        # rows of the quantile path: reset first, then scatter
        qrows = (~exact).nonzero(as_tuple=True)[0]
        cuts[qrows] = FLT_MAX
        cuts[fi, pos[fi, pi]] = q[fi, pi]
        nbq = keep.sum(1) + 1
        nb = torch.where(exact, nb, nbq)
    # sentinel in the last used slot
    cuts.scatter_(1, (nb - 1).clamp(min=0)[:, None], FLT_MAX)
    # -0.0 and +0.0 sort as equal, so which one a cut inherits depends on the sort implementation
    # (CPU vs rocPRIM); canonicalise so model files are byte-identical across devices.
    cuts = cuts + 0.0
    return cuts, nb.to(torch.int32)


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
