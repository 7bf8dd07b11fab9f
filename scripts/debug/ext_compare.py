"""Debug: external-memory GPU vs host path -- first differing tree / sample sizes / mu."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
from cobalt_smart_lender_ai_amd.dataio import synth
from cobalt_smart_lender_ai_amd.models import external
from cobalt_smart_lender_ai_amd.models.stream import array_chunks

X, y = synth.make_lendingclub(60_000, seed=5)
X, y = X.numpy(), y.numpy()
src = array_chunks(X, y, 11_000)
params = dict(n_estimators=12, max_depth=6, learning_rate=0.3, gamma=1.0, random_state=11, scale_pos_weight=5.0,
              colsample_bytree=0.8)
rh, rd = external.ExternalReport(), external.ExternalReport()
h = external.train_external(src, params, device="cpu", sample_rate=0.25, report=rh)
d = external.train_external(src, params, device="cuda", sample_rate=0.25, report=rd)
print("samples host", rh.sample_rows)
print("samples dev ", rd.sample_rows)
print("mu host", rh.mu[:4])
print("mu dev ", rd.mu[:4])
for t, (a, b) in enumerate(zip(h.trees, d.trees)):
    same = (np.array_equal(a.split_indices, b.split_indices) and np.array_equal(a.split_conditions, b.split_conditions)
            and np.array_equal(a.sum_hessian, b.sum_hessian))
    if not same:
        print("first differing tree", t, a.num_nodes, b.num_nodes)
        print(a.split_indices[:8], b.split_indices[:8])
        print(a.sum_hessian[:4], b.sum_hessian[:4])
        print(a.split_conditions[:8], b.split_conditions[:8])
        break
else:
    print("all trees equal")
