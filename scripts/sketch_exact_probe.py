#!/usr/bin/env python
"""Full-data exact sketch (csrc/sketch.hip, sketch.device_exact_cuts) against the sort-based
compute_cuts over every row and the 2^18-row sample path, at 10M x 20 (the headline shape): times
(best of --reps, device-synchronised) and cut equality. One JSON line."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import sketch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--only-exact", action="store_true", help="profiling: the exact path only")
a = ap.parse_args()
dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(a.rows, seed=0, device=dev)
hm = torch.isnan(X).any(0)


def timed(fn):
    out = fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return out, best * 1e3


(ce, ne), t_exact = timed(lambda: sketch.device_exact_cuts(X, 256, None, hm))
if a.only_exact:
    print(json.dumps({"rows": a.rows, "exact_ms": round(t_exact, 3)}), flush=True)
    sys.exit(0)
(cs, ns), t_sort = timed(lambda: sketch.compute_cuts(X, 256, None, hm))
samp = sketch.local_sample(X, 0, sketch.sample_stride(a.rows, 1 << 18))
(cq, nq), t_samp = timed(lambda: sketch.compute_cuts(samp, 256, None, hm))
w = torch.where(y == 1, 6.5, 1.0)
(cew, new_), t_exact_w = timed(lambda: sketch.device_exact_cuts(X, 256, w, hm))
(csw, nsw), t_sort_w = timed(lambda: sketch.compute_cuts(X, 256, w, hm))


def same(c1, n1, c2, n2):
    return bool(torch.equal(n1, n2)) and all(torch.equal(c1[f, :int(n1[f])], c2[f, :int(n1[f])])
                                             for f in range(c1.shape[0]))


print(json.dumps({"rows": a.rows, "features": X.shape[1], "exact_ms": round(t_exact, 3), "sort_ms": round(t_sort, 3),
                  "sample_2p18_ms": round(t_samp, 3), "exact_weighted_ms": round(t_exact_w, 3),
                  "sort_weighted_ms": round(t_sort_w, 3), "exact_equals_sort": same(ce, ne, cs, ns),
                  "exact_equals_sort_weighted": same(cew, new_, csw, nsw),
                  "sample_equals_full": same(cq, nq, cs, ns)}), flush=True)
