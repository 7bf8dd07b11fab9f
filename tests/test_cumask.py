"""CU-mask policy for data-parallel ranks that share one GPU (parallel/cumask.py): masks only from 2
to MAX_MASKED_RANKS ranks (6+ masked ranks deadlock at the in-kernel exchange, measured in
profiles/round4/dp_shared_gpu.txt), overridable by COBALT_SHARED_CU_MASK; the interleaved masks are
disjoint and cover every CU."""
from cobalt_smart_lender_ai_amd.parallel import cumask


def test_mask_policy(monkeypatch):
    monkeypatch.delenv("COBALT_SHARED_CU_MASK", raising=False)
    assert [cumask.want_shared_mask(w) for w in (1, 2, 5, 6, 8)] == [False, True, True, False, False]
    monkeypatch.setenv("COBALT_SHARED_CU_MASK", "1")
    assert cumask.want_shared_mask(8) and not cumask.want_shared_mask(1)
    monkeypatch.setenv("COBALT_SHARED_CU_MASK", "0")
    assert not cumask.want_shared_mask(3)


def test_interleaved_masks_partition_the_cus():
    n_cu = 256
    for world in (2, 3, 5):
        seen = 0
        for r in range(world):
            words = cumask.interleaved_mask(r, world, n_cu)
            bits = sum(w << (32 * i) for i, w in enumerate(words))
            assert bits & seen == 0
            seen |= bits
        assert seen == (1 << n_cu) - 1
