"""Host/disk-resident batch scoring (BASELINE.json "1B-row scoring ... on 8xMI355X"): rank sharding
of memory-mapped shard files, rehearsed with 2 gloo ranks on the CPU (reference: the bulk path of
src/api/cobalt_fast_api.py:113-126, scaled out)."""
import os
import socket

import numpy as np
import pytest
import torch

from cobalt_smart_lender_ai_amd.serve import batch_score as bs


@pytest.mark.parametrize("sizes", [[10, 7, 0, 13], [1], [5, 5, 5, 5, 5]])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_segments_cover_every_row_once(sizes, world):
    total = sum(sizes)
    seen = np.zeros(total, dtype=np.int64)
    starts = np.r_[0, np.cumsum(sizes)]
    prev_end = 0
    for r in range(world):
        for fi, b, e, g in bs.rank_segments(sizes, r, world):
            assert 0 <= b < e <= sizes[fi] and g == starts[fi] + b
            assert g == prev_end  # ranks own contiguous, ordered ranges
            prev_end = g + (e - b)
            seen[g:g + (e - b)] += 1
    assert (seen == 1).all()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, model_bytes, paths, out_dir):
    import torch.distributed as tdist

    from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    _, b = load_pickle_bytes(model_bytes)
    bs.score_files(b, paths, out_dir, rank, world, device="cpu", chunk=4000)
    tdist.barrier()
    tdist.destroy_process_group()


def test_two_rank_gloo_rehearsal_matches_host_predictor(tmp_path, reference_model_bytes):
    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes, predict_margin_host, sigmoid32

    rng = np.random.default_rng(0)
    paths, parts = [], []
    for i, n in enumerate([9000, 4000, 7001]):
        X = synth.make_lendingclub(n, seed=i, log_space=bool(i % 2))[0].numpy()
        X[rng.random(X.shape) < 0.01] = np.nan
        p = tmp_path / f"shard_{i}.npy"
        np.save(p, X)
        paths.append(str(p))
        parts.append(X)
    out_dir = tmp_path / "out"
    torch.multiprocessing.spawn(_rank_main, args=(2, _port(), reference_model_bytes, paths, str(out_dir)), nprocs=2)
    got = bs.gather_scores(out_dir)
    _, b = load_pickle_bytes(reference_model_bytes)
    ref = sigmoid32(predict_margin_host(b, np.concatenate(parts)))
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_open_shards_refuses_pickles(tmp_path):
    p = tmp_path / "obj.npy"
    np.save(p, np.array([{"a": 1}], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):
        bs.open_shards([p])


def test_gather_ignores_stale_ranks_and_rejects_gaps(tmp_path, reference_model_bytes):
    """A 3-rank run followed by a 2-rank run into the same directory: gather uses the 2 live ranks
    only (the 3-rank run's rank 2 file is stale); a missing rank or an overlap raises. ``max_rows``
    (the CLI's one-chunk warm-up) scores only the head of a share."""
    import json

    from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes, predict_margin_host, sigmoid32

    _, b = load_pickle_bytes(reference_model_bytes)
    X = np.random.default_rng(3).normal(size=(5000, 20)).astype(np.float32) * 50 + 100
    p = tmp_path / "s.npy"
    np.save(p, X)
    out = tmp_path / "out"
    for r in range(3):
        bs.score_files(b, [str(p)], out, r, 3, device="cpu", chunk=1000)
    for r in range(2):
        bs.score_files(b, [str(p)], out, r, 2, device="cpu", chunk=1000)
    ref = sigmoid32(predict_margin_host(b, X))
    assert np.array_equal(bs.gather_scores(out), ref)
    m = json.loads((out / "scores_rank00001.json").read_text())
    m["global_offset"] += 1
    (out / "scores_rank00001.json").write_text(json.dumps(m))
    with pytest.raises(ValueError):
        bs.gather_scores(out)
    (out / "scores_rank00001.json").unlink()
    with pytest.raises(ValueError):
        bs.gather_scores(out)
    meta = bs.score_files(b, [str(p)], tmp_path / "warm", 0, 1, device="cpu", chunk=1000, max_rows=700)
    assert meta["rows"] == 700
    assert np.array_equal(np.load(tmp_path / "warm" / "scores_rank00000.npy"), ref[:700])
