"""Task-parallel search on the GPU: worker processes (several per device on a 1-GPU box) score the
(candidate x fold) fits exactly like the single-process search. The file sorts before every other
test so the pool is spawned before this process initialises HIP (spawning from an initialised
process is refused on the pool)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_gpu_pooled_search_equals_single_process():
    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.parallel.taskpool import GpuTaskPool
    from cobalt_smart_lender_ai_amd.select import search
    from cobalt_smart_lender_ai_amd.select.split import stratified_kfold_indices

    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in this process; run this file on its own")
    X, y = synth.make_lendingclub(30_000, seed=23)
    X, y = X.numpy(), y.numpy()
    space = {"max_depth": [3, 5, 7], "learning_rate": [0.05, 0.1, 0.3], "subsample": [0.8, 1.0],
             "colsample_bytree": [0.5, 1.0]}
    base = dict(n_estimators=30, scale_pos_weight=3.0, random_state=78)
    with GpuTaskPool(3) as pool:  # 3 workers on cuda:0
        res = search.randomized_search(X, y, space, base, n_iter=6, cv=3, random_state=22, device="cuda",
                                       pool=pool)
    got = np.stack([res.cv_results_[f"split{k}_test_score"] for k in range(3)], 1)
    ref = search._fold_scores(X, y, stratified_kfold_indices(y, 3), base, search.sample_candidates(space, 6, 22),
                              "cuda", streams=1)
    assert np.array_equal(got, ref)
