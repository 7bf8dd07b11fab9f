#!/usr/bin/env python
"""Summarise a COBALT_STAMPS file (per-launch in-kernel timing of the GBDT trainer, csrc/gbdt.hip).

Columns per launch: start, gap (dispatch gap after the previous launch's last wave), span (first
block start -> last wave end), dispatch spread (first -> last block start), blocks. The summary
gives, per kernel name and position in the tree, the median gap / span, and the per-tree totals."""
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
raw = []
for ln in open(path):
    if ln.startswith("#"):
        raw.append(None)
        continue
    p = ln.split()
    raw.append((p[1], int(p[2]), int(p[3]), int(p[4]), int(p[5]), [float(x) for x in p[6:12]]))
last = max(i for i, r in enumerate(raw) if r is None)  # the last grow call of the file
raw = [r for r in raw[last + 1:] if r is not None and r[4] > 0]
# split into trees at each gradient launch; rows: (name, start_us, gap_us, span_us, spread_us, blocks)
trees, cur, prev_end = [], [], None
for name, st, en, ls, nb, pr in raw:
    if name in ("k_grad_hist", "k_grad", "k_tree_begin"):
        if cur:
            trees.append(cur)
        cur, prev_end, t0 = [], st, st
    cur.append((name, (st - t0) * 0.01, (st - prev_end) * 0.01, (en - st) * 0.01, (ls - st) * 0.01, nb,
                [x * 0.01 if x >= 0 else -1 for x in pr]))
    prev_end = en
if cur:
    trees.append(cur)
pos = defaultdict(list)
for t in trees:
    for i, r in enumerate(t):
        pos[(i, r[0])].append(r)
print(f"trees={len(trees)}  launches/tree={np.median([len(t) for t in trees]):.0f}")
print(f"{'#':>3} {'kernel':16} {'gap_us':>7} {'span_us':>8} {'spread':>7} {'blocks':>7}  probes (us after block start)")
tot_gap = tot_span = 0.0
for (i, name), rs in sorted(pos.items()):
    g = np.median([r[2] for r in rs]); s = np.median([r[3] for r in rs]); d = np.median([r[4] for r in rs])
    b = np.median([r[5] for r in rs])
    tot_gap += g; tot_span += s
    pr = np.median(np.array([r[6] for r in rs]), axis=0)
    pstr = " ".join(f"{x:6.2f}" for x in pr if x >= 0)
    print(f"{i:3d} {name:16} {g:7.2f} {s:8.2f} {d:7.2f} {b:7.0f}  {pstr}")
tree_us = [t[-1][1] + t[-1][3] - t[0][1] for t in trees]
print(f"per tree: median wall {np.median(tree_us):.1f} us = gaps {tot_gap:.1f} + spans {tot_span:.1f}")
agg = defaultdict(lambda: [0.0, 0.0])
for (i, name), rs in pos.items():
    agg[name][0] += np.median([r[2] for r in rs]); agg[name][1] += np.median([r[3] for r in rs])
for k, (g, s) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:16} gaps {g:7.1f}  spans {s:7.1f} us/tree")
