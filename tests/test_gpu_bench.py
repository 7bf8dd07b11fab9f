"""The bench.py contract the round driver parses: one JSON line on rank 0 with the BASELINE metric,
the whole-job rows/s and the config (a small fit here; the driver runs the 10M-row default)."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(300)
def test_bench_prints_one_contract_json_line():
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--rows", "200000", "--trees", "5", "--steps", "2",
                          "--warmup", "1", "--test-rows", "20000"], cwd=ROOT, capture_output=True, text=True,
                         timeout=280)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    baseline = json.loads((ROOT / "BASELINE.json").read_text())
    assert d["metric"] == "rows/sec GBDT train on 10M-row LendingClub-shaped tabular; AUC parity"
    assert d["metric"] in json.dumps(baseline)
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "strong"
    assert d["value"] == pytest.approx(200_000 / (d["ms_per_step"] / 1e3), rel=1e-3)
    assert d["config"]["global_batch"] == 200_000 and d["config"]["parallelism"] == "dp1"
    assert 0.5 < d["auc"] <= 1.0


@pytest.mark.timeout(600)
def test_torchrun_one_rank_equals_plain_bench():
    """The driver's scaling harness launches bench.py through torchrun (RANK / WORLD_SIZE / MASTER_* from
    the environment, the distributed context built from them); with one rank that path must print the
    same contract line as the plain run -- same n_gpus, config and AUC (the fit is deterministic) -- so the
    N = 1 point of the scaling curve is the headline bench by construction."""
    from cobalt_smart_lender_ai_amd.parallel.dp_check import free_port

    args = ["bench.py", "--gpus", "1", "--rows", "1000000", "--trees", "20", "--steps", "1", "--warmup", "1",
            "--test-rows", "100000"]
    plain = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert plain.returncode == 0, plain.stderr[-2000:]
    tr = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                         "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args],
                        cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert tr.returncode == 0, tr.stderr[-2000:]
    a, b = ([json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")] for r in (plain, tr))
    assert len(a) == 1 and len(b) == 1, (plain.stdout[-1000:], tr.stdout[-1000:])
    a, b = a[0], b[0]
    for k in ("metric", "n_gpus", "config", "auc", "unit", "scaling", "dtype", "sketch_rows", "rows_global"):
        assert a[k] == b[k], (k, a[k], b[k])
    assert b["n_gpus"] == 1 and b["config"]["parallelism"] == "dp1" and b["dp_transport"] is None


@pytest.mark.timeout(300)
def test_bench_auc_matches_the_pinned_host_oracle():
    """bench.py at 100k rows: the GPU fit's test AUC equals the host trainer's pinned one (the same trees;
    the synthetic rows come from the device generator here, the host one there) and the JSON names the
    reference's source (bench.py PARITY_AUC)."""
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--rows", "100000", "--test-rows", "100000",
                          "--steps", "1", "--warmup", "0"], cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert "host trainer" in d["auc_parity_source"], d
    assert abs(d["auc"] - d["auc_parity_ref"]) <= 2e-5, d
    assert d["auc_parity_ok"] is True
