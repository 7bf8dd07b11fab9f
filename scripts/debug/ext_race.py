"""Debug: GPU external path -- margins/sample after each pass vs host, with and without a sync after grow."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch
from cobalt_smart_lender_ai_amd.dataio import synth
from cobalt_smart_lender_ai_amd.models import external
from cobalt_smart_lender_ai_amd.models.stream import array_chunks

X, y = synth.make_lendingclub(60_000, seed=5)
X, y = X.numpy(), y.numpy()
src = array_chunks(X, y, 11_000)
params = dict(n_estimators=4, max_depth=6, learning_rate=0.3, gamma=1.0, random_state=11, scale_pos_weight=5.0,
              colsample_bytree=0.8)
hm = {}
oh = external._HostPasses.page_pass
def hpp(self, prev, mu, t):
    r = oh(self, prev, mu, t)
    hm[(prev, t)] = (self.margin.copy(), r[0], r[1].copy(), mu)
    return r
external._HostPasses.page_pass = hpp
external.train_external(src, params, device="cpu", sample_rate=0.25)

for sync in (False, True):
    gm = {}
    og = external._GpuPasses.page_pass
    def gpp(self, prev, mu, t):
        r = og(self, prev, mu, t)
        gm[(prev, t)] = (self.margin.cpu().numpy().copy(), r[0], r[1].copy(), mu)
        return r
    external._GpuPasses.page_pass = gpp
    if sync:
        ogr = external._GpuPasses.grow
        def ggr(self, t, ns):
            ogr(self, t, ns)
            torch.cuda.synchronize()
        external._GpuPasses.grow = ggr
    external.train_external(src, params, device="cuda", sample_rate=0.25)
    external._GpuPasses.page_pass = og
    print("sync", sync)
    for k in sorted(hm):
        if k in gm:
            a, b = hm[k], gm[k]
            print(k, "margin maxdiff", float(np.abs(a[0] - b[0]).max()), "ns", a[1], b[1],
                  "counts diff", int(np.abs(a[2] - b[2]).sum()), "mu", a[3], b[3])
