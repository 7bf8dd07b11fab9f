#!/usr/bin/env python
"""In-kernel stamps (COBALT_STAMPS) of one single-GPU fit (argv[1] rows, 70 trees); works with any
library build (COBALT_NATIVE_LIB) for same-box A/B of per-kernel spans."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.dataio import synth  # noqa: E402
from cobalt_smart_lender_ai_amd.models import gbdt  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda", 0)
X, y = synth.make_lendingclub(rows, seed=0, device=dev)
spw = float((y == 0).sum() / (y == 1).sum())
p = gbdt.GBDTParams(n_estimators=70, max_depth=7, learning_rate=0.05, gamma=5.0, scale_pos_weight=spw, random_state=78)
gbdt.train(X, y, p, device=dev)
torch.cuda.synchronize()
print("done", flush=True)
