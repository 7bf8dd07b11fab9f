"""Weighted quantile sketch (K12): NumPy oracle parity, 256-bin features, data-parallel invariance and
the mergeable summary (reference: XGBClassifier hist, max_bin=256 -- the shipped pkl's Config,
src/model_train_test/model_tree_train_test.py:111-118)."""
import numpy as np
import pytest
import torch

from cobalt_smart_lender_ai_amd.models import gbdt, sketch


def _mixed(n, seed=0):
    rng = np.random.default_rng(seed)
    X = np.stack([
        rng.lognormal(9, 0.6, n),                      # continuous, no missing -> 256 bins
        rng.normal(size=n),                            # continuous, with missing -> 255 bins
        rng.integers(0, 12, n).astype(float),          # low cardinality -> one bin per value
        (rng.random(n) < 0.3).astype(float),           # binary
    ], 1).astype(np.float32)
    X[rng.random(n) < 0.1, 1] = np.nan
    return X


def test_unweighted_cuts_are_order_statistics():
    X = _mixed(50_000, 1)
    c, nb = sketch.compute_cuts(torch.from_numpy(X), 256)
    c1, nb1 = sketch.compute_cuts(torch.from_numpy(X), 256, weights=torch.ones(len(X)))
    assert torch.equal(c, c1) and torch.equal(nb, nb1)
    for f, maxb in ((0, 256), (1, 255)):
        xs = np.sort(X[~np.isnan(X[:, f]), f])
        ref = []
        for j in range(1, maxb):
            v = xs[(j * len(xs)) // maxb]
            if v > xs[0] and (not ref or v != ref[-1]):
                ref.append(v)
        assert int(nb[f]) == len(ref) + 1
        assert np.array_equal(c[f, : len(ref)].numpy(), np.asarray(ref, np.float32))
    assert int(nb[0]) == 256 and int(nb[1]) == 255  # 256 real bins only without missing values
    assert int(nb[2]) == 12 and int(nb[3]) == 2


def test_weighted_cuts_match_numpy_oracle():
    X = _mixed(40_000, 2)
    rng = np.random.default_rng(3)
    w = np.where(rng.random(len(X)) < 0.13, 6.74642229, 1.0) * rng.uniform(0.5, 1.5, len(X))
    c, nb = sketch.compute_cuts(torch.from_numpy(X), 256, weights=torch.from_numpy(w))
    for f, maxb in ((0, 256), (1, 255)):
        ref = sketch.weighted_quantile_cuts_np(X[:, f], w, maxb)
        assert int(nb[f]) == len(ref) + 1
        assert np.array_equal(c[f, : len(ref)].numpy(), ref)
    # heavier weights pull the cuts: a weighted sketch differs from the unweighted one
    cu, _ = sketch.compute_cuts(torch.from_numpy(X), 256)
    assert not torch.equal(c[0], cu[0])


def test_hessian_sketch_weights_scale_positives():
    y = np.array([0, 1, 1, 0], np.float32)
    p = gbdt.GBDTParams(scale_pos_weight=6.5, sketch_weight="hessian")
    w = gbdt.sketch_weights_for(p, y, None, "cpu")
    assert np.allclose(w.numpy(), [1, 6.5, 6.5, 1])
    assert gbdt.sketch_weights_for(gbdt.GBDTParams(), y, None, "cpu") is None
    with pytest.raises(ValueError):
        gbdt.sketch_weights_for(gbdt.GBDTParams(sketch_weight="bogus"), y, None, "cpu")


def test_sketch_auto_resolution():
    """SKETCH_AUTO (the default): every row on a GPU above 2^18 rows (the exact device sketch), the
    2^18-row sample on the CPU and for small data (where that sample is every row); explicit values
    pass through."""
    auto, samp = gbdt.SKETCH_AUTO, gbdt.SKETCH_SAMPLE_ROWS
    assert gbdt.GBDTParams().sketch_rows == auto
    assert gbdt.resolve_sketch_rows(auto, "cuda", 10_000_000) is None
    assert gbdt.resolve_sketch_rows(auto, "cuda", None) is None
    assert gbdt.resolve_sketch_rows(auto, "cuda", samp) == samp
    assert gbdt.resolve_sketch_rows(auto, "cpu", 10_000_000) == samp
    for v in (None, 0, 4096):
        assert gbdt.resolve_sketch_rows(v, "cuda", 10_000_000) == v


def test_host_binning_and_training_with_256_bin_features():
    X = _mixed(20_000, 4)
    y = (np.nan_to_num(X[:, 1]) + 0.002 * X[:, 0] / 1e3 > 0.5).astype(np.float32)
    bd = gbdt.bin_dataset(X, device="cpu")
    assert int(bd.nbins[0]) == 256
    assert bd.bins_host[:, 0].max() == 255          # code 255 is a real bin of feature 0
    assert np.isnan(X[:, 1]).any() and (bd.bins_host[np.isnan(X[:, 1]), 1] == 255).all()
    b = gbdt.train(X, y, gbdt.GBDTParams(n_estimators=5, max_depth=4), device="cpu")
    from cobalt_smart_lender_ai_amd.models.booster import predict_margin_host

    rep = gbdt.FitReport()
    b = gbdt.train(X, y, gbdt.GBDTParams(n_estimators=5, max_depth=4), device="cpu", report=rep)
    assert np.array_equal(rep.extra["margin"], predict_margin_host(b, X))
    for t in b.trees:  # splits on the no-missing 256-bin feature send missing values right
        sel = (t.left_children != -1) & (t.split_indices == 0)
        assert (t.default_left[sel] == 0).all()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("weighted", [False, True])
def test_data_parallel_cuts_equal_single_rank(world, weighted):
    from cobalt_smart_lender_ai_amd.parallel import loopback
    from cobalt_smart_lender_ai_amd.parallel.dist import shard_range

    n = 30_000
    X = _mixed(n, 5)
    X[n - 7, 0] = np.nan  # one missing value on the LAST rank only: every rank must use 255 bins
    w = np.random.default_rng(6).uniform(0.1, 3.0, n) if weighted else None
    ref = gbdt.bin_dataset(X, device="cpu", sketch_rows=4096, sketch_weights=w)
    assert int(ref.nbins[0]) == 255

    def rank_fn(ctx):
        s, e = shard_range(n, ctx.rank, ctx.world)
        bd = gbdt.bin_dataset(X[s:e], device="cpu", sketch_rows=4096, dist=ctx, n_rows_global=n, row_offset=s,
                              sketch_weights=None if w is None else w[s:e])
        return bd.cuts, bd.nbins

    for c, nb in loopback.run_ranks(world, rank_fn, device="cpu"):
        assert torch.equal(c, ref.cuts) and torch.equal(nb, ref.nbins)


def test_quantile_summary_merge_is_rank_consistent_and_accurate():
    from cobalt_smart_lender_ai_amd.parallel import loopback
    from cobalt_smart_lender_ai_amd.parallel.dist import shard_range

    n = 60_000
    X = _mixed(n, 7)
    exact = sketch.compute_cuts(torch.from_numpy(X), 256)

    def rank_fn(ctx):
        s, e = shard_range(n, ctx.rank, ctx.world)
        bd = gbdt.bin_dataset(X[s:e], device="cpu", sketch_rows=n, dist=ctx, n_rows_global=n, row_offset=s,
                              sketch_mode="summary")
        return bd.cuts, bd.nbins

    outs = loopback.run_ranks(4, rank_fn, device="cpu")
    for c, nb in outs[1:]:
        assert torch.equal(c, outs[0][0]) and torch.equal(nb, outs[0][1])
    c, nb = outs[0]
    # low-cardinality features are exact; continuous ones within ~1/8 bin of the exact quantiles
    assert torch.equal(c[2:], exact[0][2:]) and torch.equal(nb[2:], exact[1][2:])
    for f in (0, 1):
        xs = np.sort(X[~np.isnan(X[:, f]), f])
        k = int(nb[f]) - 1
        ranks = np.searchsorted(xs, c[f, :k].numpy(), side="left") / len(xs)
        target = np.arange(1, k + 1) / (k + 1)
        assert np.max(np.abs(ranks - target)) < 2.0 / 256


def _rank_error_ok(X, w, c, nb, f, tol):
    """Cuts of feature f sit within ``tol`` (fraction of the total weight) of the weighted quantiles."""
    ok = ~np.isnan(X[:, f])
    order = np.argsort(X[ok, f], kind="stable")
    xs = X[ok, f][order]
    ws = (np.ones(ok.sum()) if w is None else w[ok][order]).astype(np.float64)
    cum = np.cumsum(ws) / ws.sum()
    k = int(nb[f]) - 1
    ranks = cum[np.searchsorted(xs, c[f, :k].numpy(), side="left") - 1]
    target = np.arange(1, k + 1) / (k + 1)
    return np.max(np.abs(ranks - target)) < tol


def test_weighted_summary_merge_uses_the_global_weight_scale():
    """each rank scaled its integer weights by its OWN max weight, so merged summaries mixed
    units. With ranks whose weights differ by 50x, the merged cuts must still be the weighted
    quantiles of the union (exact for low-cardinality features), identical on every rank; a rank with
    an empty shard must not break the merge."""
    from cobalt_smart_lender_ai_amd.parallel import loopback

    n = 48_000
    X = _mixed(n, 8)
    w = np.random.default_rng(9).uniform(0.5, 1.5, n)
    w[n // 2:] *= 50.0  # ranks 2-3 carry 50x the weight of ranks 0-1 ...
    X[n // 2:, :2] += np.float32(3.0)  # ... and hold shifted values, so the weighting moves the cuts
    exact = sketch.compute_cuts(torch.from_numpy(X), 256, weights=torch.from_numpy(w))
    bounds = [(0, n // 4), (n // 4, n // 2), (n // 2, 3 * n // 4), (3 * n // 4, n), (n, n)]  # rank 4: empty

    def rank_fn(ctx):
        s, e = bounds[ctx.rank]
        bd = gbdt.bin_dataset(X[s:e], device="cpu", sketch_rows=n, dist=ctx, n_rows_global=n, row_offset=s,
                              sketch_mode="summary", sketch_weights=w[s:e])
        return bd.cuts, bd.nbins

    outs = loopback.run_ranks(5, rank_fn, device="cpu")
    for c, nb in outs[1:]:
        assert torch.equal(c, outs[0][0]) and torch.equal(nb, outs[0][1])
    c, nb = outs[0]
    assert torch.equal(c[2:], exact[0][2:]) and torch.equal(nb[2:], exact[1][2:])
    for f in (0, 1):
        assert _rank_error_ok(X, w, c, nb, f, 0.006)


def test_device_summary_equals_host_summary():
    X = _mixed(30_000, 10)
    w = np.random.default_rng(11).uniform(0.2, 2.0, len(X))
    for wt in (None, w):
        host = sketch.QuantileSummary.build(X, wt, size=1024).to_arrays()
        dev = sketch.device_summary(torch.from_numpy(X), None if wt is None else torch.from_numpy(wt), size=1024)
        for a, b in zip(host[:3], dev):
            assert np.array_equal(a, b)


def test_full_data_sketch_single_rank_is_exact_and_ranks_agree():
    """sketch_rows=None: every row is sketched -- exact weighted quantiles (the NumPy oracle) on one
    rank; under data parallelism the per-rank device summaries merge to the same cuts on every rank,
    within the summary's rank error of the exact ones."""
    from cobalt_smart_lender_ai_amd.parallel import loopback
    from cobalt_smart_lender_ai_amd.parallel.dist import shard_range

    n = 40_000
    X = _mixed(n, 12)
    w = np.random.default_rng(13).uniform(0.5, 3.0, n)
    one = gbdt.bin_dataset(X, device="cpu", sketch_rows=None, sketch_weights=w)
    for f, maxb in ((0, 256), (1, 255)):
        ref = sketch.weighted_quantile_cuts_np(X[:, f], w, maxb)
        assert int(one.nbins[f]) == len(ref) + 1
        assert np.array_equal(one.cuts[f, : len(ref)].numpy(), ref)

    def rank_fn(ctx):
        s, e = shard_range(n, ctx.rank, ctx.world)
        bd = gbdt.bin_dataset(X[s:e], device="cpu", sketch_rows=None, dist=ctx, n_rows_global=n, row_offset=s,
                              sketch_weights=w[s:e])
        return bd.cuts, bd.nbins

    outs = loopback.run_ranks(4, rank_fn, device="cpu")
    for c, nb in outs[1:]:
        assert torch.equal(c, outs[0][0]) and torch.equal(nb, outs[0][1])
    c, nb = outs[0]
    assert torch.equal(c[2:], one.cuts[2:]) and torch.equal(nb[2:], one.nbins[2:])
    for f in (0, 1):
        assert _rank_error_ok(X, w, c, nb, f, 0.004)


def _adversarial_frames(n, dev, seed=0):
    """Feature columns that stress the bucketed exact sketch: continuous, heavy duplicates, rare
    values the strided sample misses, low cardinality with a few unsampled extra values (the
    'uncertain' distinct-count path), NaNs, -0.0 / +0.0, a constant and an all-NaN column, and a column
    whose sampled rows hold a single value (one huge open bucket: the host fallback sort)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    cols = []
    cols.append(torch.randn(n, generator=g) * 1000)
    cols.append(torch.round(torch.randn(n, generator=g) * 3))                       # heavy duplicates
    x = torch.randint(0, 40, (n,), generator=g).float()
    rare = torch.rand(n, generator=g) < 5e-5
    cols.append(torch.where(rare, 1000.0 + torch.arange(n).float(), x))              # rare unsampled values
    x = torch.randint(0, 100, (n,), generator=g).float()
    cols.append(torch.where(torch.arange(n) % 7919 == 3, 100.5 + (torch.arange(n) % 5).float(), x))  # uncertain
    x = torch.randn(n, generator=g)
    cols.append(torch.where(torch.rand(n, generator=g) < 0.3, torch.tensor(float("nan")), x))
    x = torch.where(torch.rand(n, generator=g) < 0.5, torch.tensor(-0.0), torch.tensor(0.0))
    cols.append(torch.where(torch.rand(n, generator=g) < 0.5, x, torch.randn(n, generator=g)))
    cols.append(torch.full((n,), 3.25))
    cols.append(torch.full((n,), float("nan")))
    stride = sketch.sample_stride(n, 1 << 16)
    cols.append(torch.where(torch.arange(n) % stride == 0, torch.tensor(0.0), 1.0 + torch.rand(n, generator=g)))
    return torch.stack(cols, 1).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_device_exact_cuts_equal_the_full_sort(weighted):
    """The bucketed full-data sketch (csrc/sketch.hip) returns compute_cuts' cuts over EVERY row, bit
    for bit: the LendingClub-shaped features at 2M rows and the adversarial columns at 600k rows, with
    unit weights and with hessian-style weights (including zero-weight rows)."""
    from cobalt_smart_lender_ai_amd.dataio import synth

    dev = torch.device("cuda", 0)
    X1, y1 = synth.make_lendingclub(2_000_000, seed=4, device=dev)
    X2 = _adversarial_frames(600_000, dev)
    for X, y in ((X1, y1), (X2, None)):
        w = None
        if weighted:
            if y is not None:
                w = torch.where(y == 1, 6.5, 1.0).to(dev)
            else:
                w = (torch.arange(X.shape[0], device=dev) % 11).float()  # zero weights on every 11th row
        want_c, want_n = sketch.compute_cuts(X, 256, w)
        got_c, got_n = sketch.device_exact_cuts(X, 256, w)
        assert torch.equal(got_n, want_n), (got_n, want_n)
        for f in range(X.shape[1]):
            nb = int(want_n[f])
            assert torch.equal(got_c[f, :nb].view(torch.int32), want_c[f, :nb].view(torch.int32)), f


@pytest.mark.gpu
def test_stream_exact_cuts_equal_in_core():
    """The bucketed sketch over a chunk stream (sketch.stream_exact_cuts: one chunk on the device at a
    time, pass-2 offsets carried across chunks) returns the in-core device sketch's cuts, and a streamed
    fit with the default sketch (every row on a GPU) grows the in-core fit's trees."""
    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.models import stream

    dev = torch.device("cuda", 0)
    X2 = _adversarial_frames(400_000, dev, seed=3)
    for X in (X2,):
        hm = torch.isnan(X).any(0)
        want_c, want_n = sketch.device_exact_cuts(X, 256, None, hm)
        samp = sketch.local_sample(X, 0, sketch.sample_stride(X.shape[0], 1 << 16))
        bounds = [0, 70_001, 150_000, 333_333, X.shape[0]]

        def chunks():
            for a, b in zip(bounds[:-1], bounds[1:]):
                yield X[a:b].contiguous()

        got_c, got_n = sketch.stream_exact_cuts(chunks, X.shape[0], X.shape[1], samp, hm, 256, device=dev)
        assert torch.equal(got_n, want_n)
        for f in range(X.shape[1]):
            nb = int(want_n[f])
            assert torch.equal(got_c[f, :nb].view(torch.int32), want_c[f, :nb].view(torch.int32)), f
    Xh, yh = synth.make_lendingclub(300_000, seed=9)
    Xh, yh = Xh.numpy(), yh.numpy()
    params = dict(n_estimators=4, max_depth=6, learning_rate=0.3, random_state=2)
    ref = gbdt.train(torch.from_numpy(Xh).cuda(), torch.from_numpy(yh).cuda(), params, device="cuda")
    got = stream.train_stream(stream.array_chunks(Xh, yh, 70_000), params, n_rows=len(Xh), device="cuda")
    assert got.save_raw("ubj") == ref.save_raw("ubj")


def test_device_plan_layout_holds_every_array():
    """The device sketch's plan workspace (csrc/sketch.hip sk_plan_layout, carved by models/sketch.py
    _exact_core): one region per array in SkArr order, each large enough for its worst case -- every
    bucket of every feature a segment, every rank of every feature an open target (host-only check)."""
    from cobalt_smart_lender_ai_amd import _native

    if not _native.available():
        pytest.skip("native library not built")
    lib = sketch._sk_lib()
    NB, T = lib.cobalt_sk_buckets(), 255
    size = {"sel": 1, "fstat": 8, "fbase": 8, "summary": 8, "q0": 4, "thr": 8, "pre": 8, "tb": 4, "need": 1,
            "slot": 4, "seg_feat": 4, "seg_bucket": 4, "loc_sizes": 8, "glob_sizes": 8, "loc_off": 8, "glob_off": 8,
            "tgt_off": 4, "want": 1, "ndist": 4, "tpos": 4, "tprefix": 8, "tthr": 8, "tmaxb": 8}
    assert tuple(size) == sketch._PLAN_ARRS
    for F in (1, 20, 106):
        off = sketch._plan_layout(lib, F)
        count = {"sel": F * NB, "fstat": 5 * F, "fbase": 4 * F, "summary": 8, "q0": F * T, "thr": F * T, "pre": F * T,
                 "tb": F * T, "need": F * T, "slot": F * NB, "seg_feat": F * NB, "seg_bucket": F * NB,
                 "loc_sizes": F * NB, "glob_sizes": F * NB, "loc_off": F * NB + 1, "glob_off": F * NB + 1,
                 "tgt_off": F * NB + 1, "want": F * NB, "ndist": F * NB, "tpos": F * T, "tprefix": F * T,
                 "tthr": F * T, "tmaxb": F * T}
        for i, name in enumerate(sketch._PLAN_ARRS):
            assert (off[i + 1] - off[i]) * 8 >= count[name] * size[name], (F, name)
