#!/usr/bin/env python
"""sha256 of the model a headline-config fit produces (for A/Bs of trainer switches that must not
change the trees, e.g. COBALT_PART_PP): one JSON line {rows, trees, sha, auc_train}."""
import argparse
import hashlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--trees", type=int, default=40)
a = ap.parse_args()
dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(a.rows, seed=0, device=dev)
pos = float(y.sum())
params = gbdt.GBDTParams(n_estimators=a.trees, max_depth=7, learning_rate=0.05, gamma=5.0, reg_lambda=1.0,
                         min_child_weight=1.0, max_bin=256, scale_pos_weight=(a.rows - pos) / pos, random_state=78)
b = gbdt.train(X, y, params, device=dev)
sha = hashlib.sha256(b.save_raw("ubj")).hexdigest()[:16]
print(json.dumps({"rows": a.rows, "trees": a.trees, "sha": sha}), flush=True)
