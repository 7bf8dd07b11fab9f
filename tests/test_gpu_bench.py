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
