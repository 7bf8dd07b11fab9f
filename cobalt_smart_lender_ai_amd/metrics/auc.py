"""ROC-AUC (K24) with exact tie handling, on CPU or GPU tensors.

Replaces ``sklearn.metrics.roc_auc_score`` at src/model_train_test/model_tree_train_test.py:175 and
in the RandomizedSearchCV scorer (``scoring='roc_auc'``, :151). Mann-Whitney form:
``AUC = (sum of positive average ranks - P(P+1)/2) / (P * N)``, ranks averaged over ties — identical
to sklearn's trapezoidal ROC integral. The sort is rocPRIM's radix sort through ``torch.sort``;
the rank/tie reduction runs as device tensor ops (no host round trip until the final scalar).

Data parallel: :func:`roc_auc_distributed` all-gathers the (score, label) shards, or, with
``bins`` set, all-reduces a 2 x bins score histogram (approximate, for 10^9-row scoring).
"""
from __future__ import annotations

import numpy as np
import torch


def _t(x, device=None) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x if device is None else x.to(device)
    return torch.as_tensor(np.asarray(x), device=device)


def roc_auc(y_true, y_score) -> float:
    s = _t(y_score).reshape(-1).to(torch.float64)
    y = _t(y_true, s.device).reshape(-1).to(torch.float64)
    n = s.numel()
    if n == 0:
        raise ValueError("empty input")
    P = float(y.sum())
    Nn = float(n - P)
    if P == 0 or Nn == 0:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
    order = torch.argsort(s, stable=True)
    ss = s[order]
    ys = y[order]
    _, inv, counts = torch.unique_consecutive(ss, return_inverse=True, return_counts=True)
    ends = torch.cumsum(counts, 0).to(torch.float64)               # 1-based rank of each group's last item
    avg_rank = ends - (counts.to(torch.float64) - 1.0) / 2.0        # average 1-based rank in the group
    pos_rank_sum = float((avg_rank[inv] * ys).sum())
    return (pos_rank_sum - P * (P + 1) / 2.0) / (P * Nn)


def roc_auc_distributed(y_true: torch.Tensor, y_score: torch.Tensor, ctx, bins: int | None = None) -> float:
    if ctx is None or ctx.world == 1:
        return roc_auc(y_true, y_score)
    if bins is None:
        ys = ctx.allgather_rows(y_true.reshape(-1, 1).to(torch.float32), pad_value=-1.0).reshape(-1)
        ss = ctx.allgather_rows(y_score.reshape(-1, 1).to(torch.float32), pad_value=0.0).reshape(-1)
        keep = ys >= 0
        return roc_auc(ys[keep], ss[keep])
    s = y_score.reshape(-1).to(torch.float64).clamp(0, 1)
    idx = torch.clamp((s * bins).long(), max=bins - 1)
    h = torch.zeros((2, bins), dtype=torch.float64, device=s.device)
    yb = y_true.reshape(-1).to(torch.long)
    h.index_put_((yb, idx), torch.ones_like(s), accumulate=True)
    h = ctx.allreduce(h if ctx.backend == "nccl" else h.cpu(), "sum").to(s.device)
    neg, pos = h[0], h[1]
    cneg = torch.cumsum(neg, 0) - neg                               # negatives strictly below the bin
    auc_num = float((pos * (cneg + 0.5 * neg)).sum())
    return auc_num / float(pos.sum() * neg.sum())
