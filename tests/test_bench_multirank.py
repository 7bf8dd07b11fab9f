"""The driver's multi-GPU entry point, rehearsed on CPU: ``torch.distributed.run --nproc-per-node 2
bench.py --gpus 2`` with GPUs hidden runs two gloo ranks through the same bench code path (shard
ranges, all-reduced class balance / timings, the distributed sketch, the host trainer's per-level
histogram all-reduce). Exactly one JSON line must come from rank 0, with the strong-scaling
bookkeeping of a 2-rank run, and the model it trains must score the same AUC as the 1-rank run."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
# (a strided sketch sample: on the CPU the all-row sketch of a sharded fit merges per-rank quantile
# summaries, which are within the summary's rank error of the 1-rank cuts but not equal to them; the
# GPU's all-row sketch is exact under DP -- tests/test_00gpu_dp_ipc.py)
ARGS = ["--rows", "200000", "--trees", "5", "--steps", "1", "--warmup", "0", "--test-rows", "50000",
        "--sketch-rows", "65536"]


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str) -> list[dict]:
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_bench_gloo_ranks_one_json_line_and_same_auc(world):
    one = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *ARGS], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr[-3000:]
    (ref,) = _json_lines(one.stdout)
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
                          str(world), *ARGS], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert two.returncode == 0, two.stderr[-3000:]
    lines = _json_lines(two.stdout)
    assert len(lines) == 1, two.stdout
    got = lines[0]
    assert got["n_gpus"] == world
    assert got["rows_global"] == 200000
    assert got["config"]["rows_per_gpu"] == 200000 // world
    assert got["config"]["parallelism"] == f"dp{world}"
    assert got["config"]["global_batch"] == 200000
    assert got["metric"] == ref["metric"]
    assert got["value"] > 0 and got["ms_per_step"] > 0
    assert got["auc"] == ref["auc"]
    assert got["replicas_agree"] is True  # both ranks hold the same model (digest min == max)
