"""Task-parallel model selection (reference RandomizedSearchCV(n_jobs=-1),
src/model_train_test/model_tree_train_test.py:148-157): pooled fits score exactly like one process."""
import numpy as np

from cobalt_smart_lender_ai_amd.dataio import synth
from cobalt_smart_lender_ai_amd.parallel.taskpool import GpuTaskPool, resolve_workers, visible_gpus
from cobalt_smart_lender_ai_amd.select import search
from cobalt_smart_lender_ai_amd.select.split import stratified_kfold_indices

SPACE = {"max_depth": [3, 5], "learning_rate": [0.1, 0.3], "subsample": [0.8, 1.0], "n_estimators": [5, 8]}


def test_resolve_workers_defaults_to_visible_gpus():
    assert resolve_workers(None) == max(1, visible_gpus())
    assert resolve_workers(3) == 3


def test_pooled_search_equals_single_process_cpu():
    X, y = synth.make_lendingclub(4_000, seed=23)
    X, y = X.numpy(), y.numpy()
    base = dict(n_estimators=5, scale_pos_weight=3.0, random_state=78)
    cands = search.sample_candidates(SPACE, 5, 22)
    folds = stratified_kfold_indices(y, 3)
    ref = search._fold_scores(X, y, folds, base, cands, "cpu")
    with GpuTaskPool(2, n_gpus=0) as pool:
        res = search.randomized_search(X, y, SPACE, base, n_iter=5, cv=3, random_state=22, device="cpu", pool=pool)
    got = np.stack([res.cv_results_[f"split{k}_test_score"] for k in range(3)], 1)
    assert np.array_equal(got, ref)
    assert res.best_index_ == int(np.argmax(ref.mean(1)))


def test_no_automatic_pool_for_cpu_work_or_an_initialised_process(monkeypatch):
    """run_training / randomized_search create a pool on their own only for GPU work from
    a process without HIP state; a CPU request stays in-process (and on the CPU in pool workers)."""
    import torch

    from cobalt_smart_lender_ai_amd.parallel import taskpool

    assert not taskpool.can_auto_pool("cpu")
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    assert not taskpool.can_auto_pool("cuda")
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    assert taskpool.can_auto_pool("cuda")
    monkeypatch.setitem(taskpool._SLOT, "gpu", 0)
    assert taskpool.worker_device("cpu") == "cpu"
