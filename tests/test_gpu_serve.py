"""GPU scoring engine: hipGraph-replayed buckets == eager kernels == NumPy host reference
(reference behaviour: src/api/cobalt_fast_api.py:90-108 predict_proba + TreeExplainer)."""
import asyncio

import numpy as np
import pytest
import torch

from cobalt_smart_lender_ai_amd import _native
from cobalt_smart_lender_ai_amd.models.booster import predict_margin_host, sigmoid32, treeshap_host
from cobalt_smart_lender_ai_amd.serve.batcher import MicroBatcher
from cobalt_smart_lender_ai_amd.serve.engine import ScoringEngine

pytestmark = pytest.mark.gpu


def _rows(n, F, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, F)).astype(np.float32) * np.float32(300) + np.float32(500)
    X[:, 12:] = (rng.random((n, F - 12)) < 0.3).astype(np.float32)
    X[rng.random((n, F)) < 0.05] = np.nan
    return X


@pytest.fixture(scope="module")
def engines(reference_booster):
    g = ScoringEngine(reference_booster, device="cuda:0", use_graphs=True)
    e = ScoringEngine(reference_booster, device="cuda:0", use_graphs=False)
    return g, e


def test_native_library_is_loaded(engines):
    assert _native.available() and _native.loaded_path() is not None


@pytest.mark.parametrize("n", [1, 7, 64, 700, 5000])
def test_graph_buckets_match_eager_and_host(engines, reference_booster, n):
    g, e = engines
    X = _rows(n, reference_booster.num_feature, seed=n)
    pg, sg = g.score(X)
    pe, se = e.score(X)
    np.testing.assert_array_equal(pg, pe)
    np.testing.assert_array_equal(sg, se)
    ph = sigmoid32(predict_margin_host(reference_booster, X))
    np.testing.assert_allclose(pg, ph, rtol=0, atol=2e-7)
    k = min(n, 64)
    sh = treeshap_host(reference_booster, X[:k])
    np.testing.assert_allclose(sg[:k], sh, rtol=1e-9, atol=1e-9)
    # local accuracy: sum(phi) + E[f] == margin
    m = predict_margin_host(reference_booster, X).astype(np.float64)
    np.testing.assert_allclose(sg.sum(1) + g.expected_value, m, atol=2e-4)


def test_prob_only_replay(engines, reference_booster):
    g, _ = engines
    X = _rows(300, reference_booster.num_feature, seed=11)
    p, s = g.score(X, with_shap=False)
    assert s is None
    np.testing.assert_array_equal(p, g.score(X)[0])


def test_micro_batcher_concurrent_requests(engines, reference_booster):
    g, _ = engines
    X = _rows(200, reference_booster.num_feature, seed=5)
    ref_p, ref_s = g.score(X)

    async def go():
        b = MicroBatcher(g, max_batch=64, max_wait_ms=2.0)
        await b.start()
        res = await asyncio.gather(*[b.submit(X[i]) for i in range(len(X))])
        await b.stop()
        return res, b.stats

    res, stats = asyncio.run(go())
    np.testing.assert_array_equal(np.array([r[0] for r in res], dtype=np.float32), ref_p)
    np.testing.assert_array_equal(np.stack([r[1] for r in res]), ref_s)
    assert stats.rows == 200 and stats.batches < 200


def test_shap_is_batch_size_invariant(engines, reference_booster):
    """A row's SHAP values are bit-identical scored alone, in a bucket, or in a split bulk batch."""
    g, e = engines
    X = _rows(5000, reference_booster.num_feature, seed=21)
    full = g.score(X)[1]
    for i in (0, 17, 4999):
        np.testing.assert_array_equal(g.score(X[i:i + 1])[1][0], full[i])
        np.testing.assert_array_equal(e.score(X[i:i + 3])[1][0], full[i])


def test_shap_pattern_tables_equal_direct_kernel(reference_booster):
    """Fast-TreeSHAP pattern tables give bit-identical values to the direct EXTEND/UNWIND kernel."""
    from cobalt_smart_lender_ai_amd.ops import predict_ops

    gf = predict_ops.gpu_forest(reference_booster, torch.device("cuda", 0), None, with_shap=True)
    assert gf.table is not None
    X = torch.as_tensor(_rows(3000, reference_booster.num_feature, seed=33), device="cuda")
    a = torch.zeros((3000, reference_booster.num_feature), dtype=torch.float64, device="cuda")
    b = torch.zeros_like(a)
    predict_ops.treeshap_gpu(reference_booster, X, a)
    predict_ops._FORCE_DIRECT_SHAP = True
    try:
        predict_ops.treeshap_gpu(reference_booster, X, b)
    finally:
        predict_ops._FORCE_DIRECT_SHAP = False
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_large_batch_predictor_matches_host(reference_booster):
    """The row-block predictor (k_predict, batches past the small-batch path) against the host
    predictor on NaN-bearing rows: the interleaved tree walks keep the fp32 tree-order sum."""
    import torch

    from cobalt_smart_lender_ai_amd.ops import predict_ops

    n = predict_ops._SMALL_ROWS + 12_345
    X = _rows(n, reference_booster.num_feature, seed=11)
    Xd = torch.from_numpy(X).cuda()
    margin = torch.empty(n, dtype=torch.float32, device="cuda")
    prob = torch.empty(n, dtype=torch.float32, device="cuda")
    predict_ops.predict_gpu(reference_booster, Xd, None, out_margin=margin, out_prob=prob)
    mh = predict_margin_host(reference_booster, X)
    np.testing.assert_array_equal(margin.cpu().numpy(), mh)


@pytest.mark.gpu
def test_batch_scoring_chunks_match_host(reference_booster):
    """Chunked batch scoring (device-resident in place, device-resident through graph staging, and
    host-streamed; several chunks plus a ragged tail) equals the host predictor: graphs replay on
    the scorer's stream, ordered after the chunk copy and before the result copy."""
    import torch

    from cobalt_smart_lender_ai_amd.serve.batch_score import score_device_matrix, score_shard

    n, chunk = 200_003, 1 << 16
    X = _rows(n, reference_booster.num_feature, seed=5)
    ref = sigmoid32(predict_margin_host(reference_booster, X))
    Xd = torch.from_numpy(X).cuda()
    Xd.mul_(1.0)  # pending work on the current stream when the scorer starts
    pd = score_device_matrix(reference_booster, Xd, chunk=chunk).cpu().numpy()
    np.testing.assert_allclose(pd, ref, rtol=0, atol=2e-7)
    # the same (X, out) buffers again: direct launches, then a capture, then replays of that graph,
    # which read X's CURRENT contents
    out = torch.empty(n, dtype=torch.float32, device=Xd.device)
    for _ in range(3):
        np.testing.assert_array_equal(score_device_matrix(reference_booster, Xd, out, chunk=chunk).cpu().numpy(), pd)
    assert any(g is not None for g in reference_booster.__dict__["_score_graphs"].values())
    X2 = X.copy()
    X2[: n // 2] = X[n // 2: 2 * (n // 2)]
    Xd.copy_(torch.from_numpy(X2))
    ref2 = sigmoid32(predict_margin_host(reference_booster, X2))
    np.testing.assert_allclose(score_device_matrix(reference_booster, Xd, out, chunk=chunk).cpu().numpy(), ref2,
                               rtol=0, atol=2e-7)
    Xd.copy_(torch.from_numpy(X))
    # column-major input takes the GraphScorer staging path (static buffer + replay per chunk)
    Xc = Xd.t().contiguous().t()
    assert Xc.stride(1) != 1
    np.testing.assert_array_equal(score_device_matrix(reference_booster, Xc, chunk=chunk).cpu().numpy(), pd)
    ph = score_shard(reference_booster, X, chunk=chunk)
    np.testing.assert_array_equal(ph, pd)


@pytest.mark.gpu
def test_deep_trees_grow_the_lds_tile():
    """Trees larger than the default 2048-node tile (depth 12, host-trained: the GPU trainer stops at
    depth 10 = 2047 nodes) get a larger per-model tile; both predictor paths equal the host predictor."""
    import torch

    from cobalt_smart_lender_ai_amd.models import gbdt
    from cobalt_smart_lender_ai_amd.ops import predict_ops

    rng = np.random.default_rng(3)
    Xt = rng.normal(size=(40_000, 16)).astype(np.float32)
    yt = ((Xt[:, 0] * Xt[:, 1] + np.sin(3 * Xt[:, 2]) + rng.normal(size=40_000)) > 0).astype(np.float32)
    bst = gbdt.train(Xt, yt, {"max_depth": 12, "n_estimators": 4, "min_child_weight": 0.0, "gamma": 0.0},
                     device="cpu")
    assert predict_ops.tile_capacity(bst) > predict_ops.TILE_NODES
    for n in (5000, predict_ops._SMALL_ROWS + 77):
        X = rng.normal(size=(n, 16)).astype(np.float32)
        X[rng.random((n, 16)) < 0.05] = np.nan
        Xd = torch.from_numpy(X).cuda()
        margin = torch.empty(n, dtype=torch.float32, device="cuda")
        predict_ops.predict_gpu(bst, Xd, None, out_margin=margin)
        np.testing.assert_array_equal(margin.cpu().numpy(), predict_margin_host(bst, X))


def test_host_stream_scorer_files_equal_device_path(reference_booster, tmp_path):
    """The host/disk-resident pipeline (memory-mapped shards -> pinned slots -> H2D -> graph -> D2H)
    scores exactly what the device-resident path scores, across file boundaries, partial last
    chunks and slot reuse."""
    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.serve import batch_score as bs

    parts, paths = [], []
    for i, n in enumerate([1_300_000, 700_001, 1_000_000]):
        X = synth.make_lendingclub(n, seed=i, row_offset=i * 2_000_000)[0].numpy()
        p = tmp_path / f"s{i}.npy"
        np.save(p, X)
        parts.append(X)
        paths.append(str(p))
    meta = bs.score_files(reference_booster, paths, tmp_path / "out", 0, 1, "cuda", chunk=300_000, slots=3,
                          stage_threads=4)
    assert meta["rows"] == 3_000_001
    got = bs.gather_scores(tmp_path / "out")
    Xd = torch.from_numpy(np.concatenate(parts)).cuda()
    ref = bs.score_device_matrix(reference_booster, Xd).cpu().numpy()
    assert np.array_equal(got, ref)


def test_bulk_csv_device_parse_equals_pandas_path(reference_booster, monkeypatch):
    """/predict_bulk_csv with a large upload on a GPU engine: parsed by the GPU CSV reader and scored
    from HBM -- the response equals the pandas path's (the reference's pd.read_csv + predict_proba)."""
    import io

    import pandas as pd
    from fastapi.testclient import TestClient

    from cobalt_smart_lender_ai_amd.config import DEPLOYED_FEATURES, ServeConfig
    from cobalt_smart_lender_ai_amd.serve import app as app_mod

    n = 12_000
    X = _rows(n, len(DEPLOYED_FEATURES), seed=11)
    df = pd.DataFrame(X.astype(np.float64), columns=DEPLOYED_FEATURES)
    df["term"] = np.where(np.arange(n) % 2 == 0, 36, 60)  # an integer column (int64 in both parsers)
    buf = io.StringIO()
    df.to_csv(buf, index=False)
    body = buf.getvalue().encode()
    assert len(body) >= 1 << 20
    app = app_mod.create_app(ServeConfig(device="cuda:0"), booster=reference_booster)
    with TestClient(app) as c:
        files = {"file": ("x.csv", body, "text/csv")}
        monkeypatch.setattr(app_mod, "GPU_CSV_MIN_BYTES", 1 << 40)
        host = c.post("/predict_bulk_csv", files=files)
        monkeypatch.setattr(app_mod, "GPU_CSV_MIN_BYTES", 0)
        calls = []
        real = app_mod._score_device
        monkeypatch.setattr(app_mod, "_score_device",
                            lambda b, Xd, lock=None: calls.append(Xd.shape) or real(b, Xd, lock))
        dev = c.post("/predict_bulk_csv", files=files)
    assert host.status_code == 200 and dev.status_code == 200, (host.text[:200], dev.text[:200])
    assert calls == [(n, len(DEPLOYED_FEATURES))]  # the device path ran
    hp, dp = host.json()["predictions"], dev.json()["predictions"]
    assert len(hp) == len(dp) == n
    diff = [(i, k, hp[i][k], dp[i].get(k)) for i in range(n) for k in hp[i] if hp[i][k] != dp[i].get(k)]
    assert not diff, (len(diff), diff[:8])
    assert dev.json() == host.json()


def test_concurrent_predict_and_repeated_bulk_device_requests(reference_booster, monkeypatch):
    """Same-size device-parsed bulk uploads (the caching allocator hands them the same addresses) next
    to concurrent /predict requests whose micro-batcher replays the engine's hipGraphs: every request
    succeeds and every bulk answer is the same (advisor finding: the bulk scorer captured a graph on a
    worker thread outside the engine lock; it is now serialised with the engine and never captures)."""
    import concurrent.futures as cf
    import io

    import pandas as pd
    from fastapi.testclient import TestClient

    from cobalt_smart_lender_ai_amd.config import DEPLOYED_FEATURES, ServeConfig
    from cobalt_smart_lender_ai_amd.serve import app as app_mod

    n = 12_000
    X = _rows(n, len(DEPLOYED_FEATURES), seed=5)
    buf = io.StringIO()
    pd.DataFrame(X.astype(np.float64), columns=DEPLOYED_FEATURES).to_csv(buf, index=False)
    files = {"file": ("x.csv", buf.getvalue().encode(), "text/csv")}
    monkeypatch.setattr(app_mod, "GPU_CSV_MIN_BYTES", 0)
    row = {f: float(v) for f, v in zip(DEPLOYED_FEATURES, np.nan_to_num(X[0]))}
    row["application_type_Joint App"] = row.pop("application_type_Joint App")
    app = app_mod.create_app(ServeConfig(device="cuda:0", use_graphs=True), booster=reference_booster)
    with TestClient(app) as c:
        def bulk(_):
            r = c.post("/predict_bulk_csv", files=files)
            return r.status_code, [p["prob_default"] for p in r.json()["predictions"]] if r.status_code == 200 else r.text

        def single(_):
            return c.post("/predict", json=row).status_code, None

        with cf.ThreadPoolExecutor(8) as ex:
            futs = [ex.submit(bulk if k % 2 == 0 else single, k) for k in range(24)]
            res = [f.result() for f in futs]
    codes = [r[0] for r in res]
    assert codes == [200] * len(codes), res[:3]
    outs = [r[1] for k, r in enumerate(res) if k % 2 == 0]
    assert all(o == outs[0] for o in outs)
