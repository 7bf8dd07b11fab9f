#!/usr/bin/env python
"""Scoring benchmarks on one GPU (reference model, 20 features):
  * ScoringEngine latency per bucket (prob only / prob + TreeSHAP, hipGraph replay incl. H2D/D2H);
  * device-resident bulk scoring throughput (rows/s) through GraphScorer chunks;
  * host-resident bulk scoring (pinned, double-buffered);
  * MLP challenger inference throughput.
Prints one JSON object."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes  # noqa: E402
from cobalt_smart_lender_ai_amd.serve.batch_score import score_device_matrix, score_shard  # noqa: E402
from cobalt_smart_lender_ai_amd.serve.engine import ScoringEngine  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)), float(np.percentile(ts, 99))


def main():
    pkl = Path(__file__).resolve().parents[1] / "src" / "api" / "models" / "xgb_model_tree.pkl"
    _, b = load_pickle_bytes(pkl.read_bytes())
    rng = np.random.default_rng(0)
    F = b.num_feature
    out = {"model": "reference xgb_model_tree.pkl (300 trees, depth 7)"}
    eng = ScoringEngine(b, device="cuda:0")
    lat = {}
    for n in (1, 64, 512, 4096):
        X = rng.random((n, F)).astype(np.float32) * 1000
        p50, p99 = timeit(lambda: eng.score(X, with_shap=False), 50)
        s50, s99 = timeit(lambda: eng.score(X, with_shap=True), 20)
        lat[n] = {"prob_p50_us": p50 * 1e6, "prob_p99_us": p99 * 1e6, "prob_shap_p50_us": s50 * 1e6,
                  "prob_shap_p99_us": s99 * 1e6, "shap_rows_per_s": n / s50}
    out["engine_latency"] = lat
    N = 50_000_000
    Xd = torch.rand((N, F), device="cuda") * 1000
    res = torch.empty(N, device="cuda")
    t, _ = timeit(lambda: score_device_matrix(b, Xd, res), 3)
    out["device_bulk_rows_per_s"] = N / t
    del Xd, res
    Nh = 20_000_000
    Xh = (rng.random((Nh, F), dtype=np.float32) * 1000)
    t0 = time.perf_counter()
    score_shard(b, Xh)
    out["host_bulk_rows_per_s"] = Nh / (time.perf_counter() - t0)
    from cobalt_smart_lender_ai_amd.nn import mlp
    p = torch.as_tensor(mlp.init_params(F), device="cuda")
    Xm = torch.rand((10_000_000, F), device="cuda")
    pm = torch.empty(10_000_000, device="cuda")
    t, _ = timeit(lambda: mlp.mlp_forward_gpu(Xm, p, pm), 5)
    out["mlp_infer_rows_per_s"] = 10_000_000 / t
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
