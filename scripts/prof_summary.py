#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals and the last GBDT tree's timeline."""
import sys

import pandas as pd

path = sys.argv[1]
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 1
t = pd.read_csv(path)
t["us"] = (t["End_Timestamp"] - t["Start_Timestamp"]) / 1000
t["name"] = t["Kernel_Name"].str.split("(").str[0].str.slice(0, 48)
print("== per-kernel totals (us per tree) ==")
g = t.groupby("name").agg(calls=("us", "size"), total_us=("us", "sum"), avg_us=("us", "mean"))
g["per_tree_us"] = g["total_us"] / trees
print(g.sort_values("total_us", ascending=False).head(20).round(1).to_string())
base = t["name"].str.replace("void ", "", regex=False).str.split("<").str[0]
idx = t.index[base.isin(["k_grad", "k_grad_hist"])]
if len(idx):
    last = t.loc[idx[-1]:]
    stop = last.index[base.loc[last.index].isin(["k_apply_tree", "__amd_rocclr_copyBuffer"])]
    if len(stop):
        last = last.loc[: stop[0]]
    print("== last tree timeline ==")
    print(last[["name", "us", "Grid_Size_X"]].round(1).to_string(index=False))
    print("busy_us", round(last["us"].sum(), 1), "span_us",
          round((last["End_Timestamp"].iloc[-1] - last["Start_Timestamp"].iloc[0]) / 1000, 1))
