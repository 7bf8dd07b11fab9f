"""Randomized hyper-parameter search with stratified K-fold ROC-AUC scoring (K28).

Reference: ``RandomizedSearchCV(XGBClassifier(eval_metric='logloss', scale_pos_weight=spw,
random_state=78), param_distributions, n_iter=20, scoring='roc_auc', cv=StratifiedKFold(3),
n_jobs=-1, random_state=22)`` (src/model_train_test/model_tree_train_test.py:132-164) = 60 fits +
1 refit spread over CPU worker processes.

Here: the candidate list comes from scikit-learn's ``ParameterSampler`` (same ``random_state`` ->
same 20 candidates); each fold's training rows are sketched + binned once and reused by all 20
candidates; fits run on the GPU, concurrently on several HIP streams of one device, or task-parallel
with one worker process per GPU (``n_gpus``). The best candidate (highest mean AUC, first on ties -- sklearn's
``rank_test_score`` argmin) is refit on all training rows.
"""
from __future__ import annotations

import dataclasses
import logging
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..metrics.auc import roc_auc
from ..models import gbdt
from ..models.booster import Booster
from .split import stratified_kfold_indices
from ..config import knob

log = logging.getLogger(__name__)


@dataclass
class SearchResult:
    best_params_: dict
    best_score_: float
    best_index_: int
    best_estimator_: Booster
    cv_results_: dict = field(default_factory=dict)


def sample_candidates(param_distributions: dict, n_iter: int, random_state: int | None) -> list[dict]:
    from sklearn.model_selection import ParameterSampler

    return [dict(p) for p in ParameterSampler(param_distributions, n_iter=n_iter, random_state=random_state)]


def _fold_scores(X, y, folds, base: dict, candidates: list[dict], device, streams: int | None = None) -> np.ndarray:
    """[n_candidates, n_folds] AUC matrix; one binning per fold. On a GPU the (fold, candidate) fits
    run concurrently on ``streams`` HIP streams (one host thread each; the fits of a 3-fold search
    on ~100k rows are launch/latency bound, so several in flight fill the device)."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    Xn = X if isinstance(X, (np.ndarray, torch.Tensor)) else np.asarray(X, dtype=np.float32)
    yn = np.asarray(y.cpu().numpy() if isinstance(y, torch.Tensor) else y, dtype=np.float32)
    scores = np.zeros((len(candidates), len(folds)))
    params0 = gbdt.GBDTParams.from_kwargs(**base)
    on_dev = isinstance(Xn, torch.Tensor) and Xn.is_cuda

    def rows(idx):  # a fold's rows: a device gather when the matrix is device-resident
        return Xn.index_select(0, torch.as_tensor(idx, device=Xn.device)) if on_dev else Xn[idx]

    bds = [gbdt.bin_dataset(rows(tr), max_bin=params0.max_bin, sketch_rows=params0.sketch_rows, device=device)
           for tr, _ in folds]
    # labels and validation rows of every fold, staged once (not once per candidate)
    ytr = [torch.as_tensor(yn[tr], device=bd.device) if bd.device.type == "cuda" else yn[tr]
           for (tr, _), bd in zip(folds, bds)]
    Xva = [rows(va) for _, va in folds]

    def fit(i: int, k: int, bd=None) -> None:
        _, va = folds[k]
        p = gbdt.GBDTParams.from_kwargs(**{**base, **candidates[i]})
        bst = gbdt.train_binned(bd if bd is not None else bds[k], ytr[k], p)
        prob = bst.predict_proba(Xva[k], device=str(bds[k].device))
        scores[i, k] = roc_auc(yn[va], prob)

    tasks = [(i, k) for k in range(len(folds)) for i in range(len(candidates))]
    dev = bds[0].device if bds else torch.device("cpu")
    n_streams = streams if streams is not None else int(knob("COBALT_SEARCH_STREAMS", "4"))
    if dev.type != "cuda" or n_streams <= 1:
        for i, k in tasks:
            fit(i, k)
        return scores
    local = __import__("threading").local()

    def run(task) -> None:
        if not hasattr(local, "stream"):
            torch.cuda.set_device(dev)
            local.stream = torch.cuda.Stream(dev)
            local.bds = {}
        i, k = task
        with torch.cuda.stream(local.stream):
            if k not in local.bds:  # the trainer writes each fit's gradient pairs into the row records:
                # every worker needs its own copy (the feature-major bins stay shared, read-only)
                local.bds[k] = dataclasses.replace(bds[k], records=bds[k].records.clone())
            fit(i, k, local.bds[k])
            local.stream.synchronize()

    torch.cuda.synchronize(dev)  # the binned folds are complete before other streams read them
    with ThreadPoolExecutor(n_streams) as ex:
        list(ex.map(run, tasks))
    return scores


def _worker(args):
    """Pool task: the fold scores of a candidate subset on this worker's GPU (parallel/taskpool.py)."""
    from ..parallel.taskpool import worker_device

    X, y, folds, base, cands, dev_type = args
    return _fold_scores(X, y, folds, base, cands, worker_device(dev_type))


def randomized_search(X, y, param_distributions: dict, base_params: dict, n_iter: int = 20, cv: int = 3,
                      random_state: int | None = 22, device=None, n_gpus: int | None = 1,
                      pool=None) -> SearchResult:
    """``pool`` (a :class:`~..parallel.taskpool.GpuTaskPool`, created before this process touched the
    GPU) runs the (candidate x fold) fits task-parallel, candidates dealt round-robin to its workers;
    otherwise ``n_gpus`` > 1 (None = all visible) creates one for this call."""
    from ..parallel.taskpool import GpuTaskPool, can_auto_pool, visible_gpus

    if isinstance(X, torch.Tensor) and X.is_cuda:  # device-resident matrix: fits stay in this process
        X = X.to(torch.float32).contiguous()
        if pool is not None:
            log.info("randomized_search: device-resident matrix, fits run on this process's streams")
            pool = None
        n_gpus = 1
    else:
        X = np.asarray(X.cpu().numpy() if isinstance(X, torch.Tensor) else X, dtype=np.float32)
    y = np.asarray(y.cpu().numpy() if isinstance(y, torch.Tensor) else y, dtype=np.float32)
    cands = sample_candidates(param_distributions, n_iter, random_state)
    folds = stratified_kfold_indices(y, cv)
    t0 = time.perf_counter()
    own = None
    if pool is None:
        ngpu = visible_gpus() if n_gpus is None else min(int(n_gpus), visible_gpus())
        if ngpu > 1 and can_auto_pool(device):
            pool = own = GpuTaskPool(ngpu, ngpu)
    try:
        if pool is not None:
            nw = pool.workers
            shards = [list(range(i, len(cands), nw)) for i in range(nw)]
            shards = [sh for sh in shards if sh]
            dev_type = torch.device(device).type if device is not None else "cuda"
            parts = pool.map(_worker, [(X, y, folds, base_params, [cands[j] for j in sh], dev_type) for sh in shards])
            scores = np.zeros((len(cands), len(folds)))
            for sh, part in zip(shards, parts):
                scores[sh] = part
        else:
            scores = _fold_scores(X, y, folds, base_params, cands, device)
    finally:
        if own is not None:
            own.close()
    mean = scores.mean(1)
    # sklearn ranks with method="min": equal scores share the best rank
    order = np.argsort(-mean, kind="stable")
    ranks = np.empty(len(mean), dtype=np.int64)
    prev, r = None, 0
    for pos, i in enumerate(order):
        if prev is None or mean[i] != prev:
            r = pos + 1
            prev = mean[i]
        ranks[i] = r
    best = int(np.argmin(ranks))
    best_params = cands[best]
    bst = gbdt.train(X, y, gbdt.GBDTParams.from_kwargs(**{**base_params, **best_params}), device=device)
    res = {"params": cands, "mean_test_score": mean, "std_test_score": scores.std(1), "rank_test_score": ranks,
           "search_seconds": time.perf_counter() - t0}
    for k in range(scores.shape[1]):
        res[f"split{k}_test_score"] = scores[:, k]
    return SearchResult(best_params, float(mean[best]), best, bst, res)
