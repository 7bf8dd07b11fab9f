#!/usr/bin/env python
"""The part of a fit before its first boosting round, from a rocprofv3 --kernel-trace CSV: every kernel
between a fit's first quantile-sketch kernel and its first gradient pass (sketch, binning, setup), with
its duration and the idle gap before it -- where the prelude's wall time goes (GPU work vs host gaps).
usage: prof_prelude.py kernel_trace.csv [fit index, default: the last complete one]"""
import sys

import pandas as pd

t = pd.read_csv(sys.argv[1]).sort_values("Start_Timestamp").reset_index(drop=True)
t["us"] = (t["End_Timestamp"] - t["Start_Timestamp"]) / 1000
t["name"] = (t["Kernel_Name"].str.replace("void ", "", regex=False).str.replace("(anonymous namespace)::", "", regex=False)
             .str.split("(").str[0].str.slice(0, 60))
base = t["name"].str.split("<").str[0]
starts = t.index[base == "k_sk_hist"].tolist()
# the first k_sk_hist of each fit: the previous kernel is not a sketch kernel
grads = t.index[base.isin(["k_grad_hist", "k_grad"])].tolist()
# a fit's first k_sk_hist: no gradient pass since the previous k_sk_hist
fits = [i for k, i in enumerate(starts) if k == 0 or any(starts[k - 1] < g < i for g in grads)]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
s = fits[which]
e = next(g for g in grads if g > s)
# back up to the fit's first kernel after the previous fit's last tree (k_apply_tree / copies)
b = s
while b > 0 and base.iloc[b - 1] not in ("k_apply_tree", "k_dig_cmp"):
    b -= 1
seg = t.loc[b:e].copy()
seg["gap_us"] = (seg["Start_Timestamp"] - seg["End_Timestamp"].shift(1)) / 1000
print(seg[["name", "us", "gap_us"]].round(1).to_string(index=False))
wall = (seg["Start_Timestamp"].iloc[-1] - seg["Start_Timestamp"].iloc[0]) / 1000
busy = seg["us"].iloc[:-1].sum()
print(f"prelude: {len(seg) - 1} kernels, wall {wall:.1f} us (first kernel -> first gradient pass), busy {busy:.1f} us, "
      f"idle {wall - busy:.1f} us")
print(seg.iloc[:-1].groupby("name")["us"].agg(["size", "sum"]).sort_values("sum", ascending=False).round(1).to_string())
