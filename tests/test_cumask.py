"""CU-mask policy for data-parallel ranks that share one GPU (parallel/cumask.py): masks for 2 to
MAX_MASKED_RANKS (8) ranks, overridable by COBALT_SHARED_CU_MASK; the default blocked masks are
disjoint, cover every CU and give every rank CUs in all 8 XCCs under the measured bit -> XCC mapping
(bit i -> XCC i mod 8, profiles/round5/qdiag_masks.txt), which the former interleaved layout did not
for 6 ranks (the 6-rank deadlock)."""
from cobalt_smart_lender_ai_amd.parallel import cumask


def _bits(words):
    return sum(w << (32 * i) for i, w in enumerate(words))


def _xccs(bits, n_cu=256, n_xcc=8):
    return {i % n_xcc for i in range(n_cu) if (bits >> i) & 1}


def test_mask_policy(monkeypatch):
    monkeypatch.delenv("COBALT_SHARED_CU_MASK", raising=False)
    assert [cumask.want_shared_mask(w) for w in (1, 2, 5, 6, 8, 9)] == [False, True, True, True, True, False]
    monkeypatch.setenv("COBALT_SHARED_CU_MASK", "1")
    assert cumask.want_shared_mask(9) and not cumask.want_shared_mask(1)
    monkeypatch.setenv("COBALT_SHARED_CU_MASK", "0")
    assert not cumask.want_shared_mask(3)


def test_blocked_masks_partition_the_cus_and_cover_every_xcc():
    n_cu = 256
    for world in range(2, 33):
        seen = 0
        for r in range(world):
            bits = _bits(cumask.blocked_mask(r, world, n_cu))
            assert bits & seen == 0
            assert _xccs(bits, n_cu) == set(range(8)), (world, r)
            seen |= bits
        assert seen == (1 << n_cu) - 1


def test_interleaved_masks_leave_xccs_empty_when_world_shares_a_factor_with_8():
    n_cu = 256
    for world in (3, 5, 7):
        assert all(_xccs(_bits(cumask.interleaved_mask(r, world, n_cu))) == set(range(8)) for r in range(world))
    for world in (2, 4, 6):  # the 6-rank deadlock of rounds 4-5
        assert all(len(_xccs(_bits(cumask.interleaved_mask(r, world, n_cu)))) < 8 for r in range(world))
