"""Data-parallel training over physical GPUs (one process per GPU): the model equals the 1-GPU fit byte
for byte, for every rank count an 8-GPU node runs (2, 4, 8 <= device_count) over both transports --
the IPC one-shot exchange across GPUs (gloo bootstrap + the native IPC group; the default within a
node) and RCCL (nccl bootstrap + the native RCCL communicator) -- at depth 7, so node ownership is
active on the deep levels of the IPC runs. The ranks run in spawned processes (parallel/dp_check.py);
this file sorts first so the pytest process has not initialised HIP when it spawns them. On a 1-GPU box
every case skips (tests/test_00gpu_dp_ipc.py covers processes sharing one GPU, test_gpu_gbdt.py the
1-rank protocols)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
N = 400_000


def _params(trees=6):
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    return dict(dp_check.DEFAULT_PARAMS, n_estimators=trees)


def _expected_ipc_epochs(trees: int) -> int:
    # connect self-test (4) + the exact sketch's four device all-reduces + the fit scalars' one +
    # one exchange per level per tree + the final replica-digest exchange of the fit's one grow call
    return 4 + 4 + 1 + 7 * trees + 1


@pytest.mark.timeout(900)
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_multi_gpu_data_parallel_equals_single_gpu(world, transport):
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in this process; run this file on its own")
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    ref = dp_check.run(1, N, _params())[0]
    assert ref["ok"], ref
    got = dp_check.run(world, N, _params(), transport=transport, one_gpu_per_rank=True, timeout_s=600)
    for g in got:
        assert g["ok"], g  # (a replica divergence would raise on every rank: the in-flight digest check)
        assert g["transport"] == transport, g
        assert g["model_sha256"] == ref["model_sha256"], (world, transport, g["rank"])
        if transport == "ipc":
            assert g["ipc_epochs"] == _expected_ipc_epochs(ref["trees"]), g


@pytest.mark.timeout(900)
def test_torchrun_bench_on_every_gpu():
    """The driver's multi-GPU bench command on this node's GPUs: one JSON line, every rank holds the same
    model, and the AUC equals the 1-GPU bench's on the same rows (same trees)."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in this process; run this file on its own")
    common = ["--rows", "1000000", "--steps", "1", "--warmup", "1", "--test-rows", "100000"]
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1"}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", "29631", "bench.py", "--gpus", str(n), *common],
                       cwd=ROOT, capture_output=True, text=True, timeout=800, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    multi = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    r1 = subprocess.run([sys.executable, "bench.py", *common], cwd=ROOT, capture_output=True, text=True, timeout=600,
                        env=env)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][-1])
    assert multi["n_gpus"] == n and multi["replicas_agree"] is True, multi
    assert multi["auc"] == one["auc"], (multi["auc"], one["auc"])
