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
