"""The bench's same-configuration AUC reference (bench.py PARITY_AUC, scripts/parity_oracle.py): the host
trainer (models/gbdt_host.py) with exactly the bench protocol -- 300 trees, depth 7, eta 0.05, gamma 5,
lambda 1, min_child_weight 1, 256 bins, every row sketched, spw = (n - pos) / pos, test AUC on the next
rows -- reproduces the pinned number, and every bench reference names its source. (The GPU grows this
trainer's trees byte for byte, tests/test_gpu_gbdt.py; tests/test_gpu_bench.py checks the bench's GPU
AUC against the same pin.)"""
import importlib.util
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_every_parity_reference_names_its_source():
    b = _bench()
    for key, ref in b.PARITY_AUC.items():
        assert 0.5 < ref["auc"] < 1.0 and ref["source"], key
    assert "HistGradientBoosting" in b.PARITY_AUC[(10_000_000, 300, 7, 0, 1_000_000)]["source"] or \
        "host trainer" in b.PARITY_AUC[(10_000_000, 300, 7, 0, 1_000_000)]["source"]


@pytest.mark.timeout(600)
def test_host_oracle_reproduces_the_pinned_100k_auc():
    out = subprocess.run([sys.executable, str(ROOT / "scripts" / "parity_oracle.py"), "--rows", "100000", "--test-rows",
                          "100000"], cwd=ROOT, capture_output=True, text=True, timeout=580)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    pinned = _bench().PARITY_AUC[(100_000, 300, 7, 0, 100_000)]
    assert got["auc"] == pinned["auc"], (got, pinned)
    assert "host trainer" in pinned["source"]
