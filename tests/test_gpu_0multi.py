"""Data-parallel training over >= 2 GPUs (one process per GPU, RCCL): the model equals the 1-GPU fit
byte for byte. The file sorts first so its ranks are spawned before
this process initialises HIP (a spawn from an initialised process is refused on the pool). Skipped on
single-GPU hosts (the 1-rank RCCL protocol test in test_gpu_gbdt.py and
the 2-rank gloo test in test_gbdt_cpu.py cover the protocol there)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

PARAMS = dict(n_estimators=6, max_depth=7, learning_rate=0.1, gamma=1.0, subsample=0.9, colsample_bytree=0.8,
              random_state=5, scale_pos_weight=6.0)
N = 400_000


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.models import gbdt
    from cobalt_smart_lender_ai_amd.parallel import dist as pdist

    ctx = pdist.init_from_env()
    dev = torch.device("cuda", rank)
    s, e = pdist.shard_range(N, rank, world)
    X, y = synth.make_lendingclub(e - s, seed=3, row_offset=s, device=dev)
    b = gbdt.train(X, y, PARAMS, device=dev, dist=ctx, n_rows_global=N, row_offset=s)
    if rank == 0:
        with open(out, "wb") as fh:
            fh.write(b.save_raw("ubj"))
    pdist.shutdown()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")
@pytest.mark.timeout(600)
def test_two_gpu_data_parallel_equals_single_gpu(tmp_path):
    import torch.multiprocessing as mp

    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.models import gbdt

    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in this process; run this file on its own")
    out = str(tmp_path / "dp.ubj")
    mp.spawn(_worker, args=(2, _port(), out), nprocs=2, join=True)
    X, y = synth.make_lendingclub(N, seed=3, device="cuda:0")
    ref = gbdt.train(X, y, PARAMS, device="cuda:0").save_raw("ubj")
    assert open(out, "rb").read() == ref
