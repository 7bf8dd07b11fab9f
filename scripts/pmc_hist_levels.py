#!/usr/bin/env python
"""Per-level LDS behaviour of k_hist at 10M rows: joins a rocprofv3 --pmc counter CSV (per dispatch)
with its kernel trace, assigns every k_hist dispatch its tree level (position after the tree's root
pass), and prints per level: median duration, LDS instructions, bank-conflict cycles per LDS
instruction."""
import sys

import pandas as pd

cc = pd.read_csv(sys.argv[1])
kt = pd.read_csv(sys.argv[2])
kt["us"] = (kt["End_Timestamp"] - kt["Start_Timestamp"]) / 1000
kt = kt.sort_values("Start_Timestamp").reset_index(drop=True)
base = kt["Kernel_Name"].str.replace("void ", "", regex=False).str.split("<").str[0].str.split("(").str[0]
level, lv = [], -1
for b in base:
    if b in ("k_grad_hist", "k_grad"):
        lv = 0
    elif b in ("k_hist",):
        lv += 1
    level.append(lv if b == "k_hist" else -1)
kt["level"] = level
piv = cc.pivot_table(index="Dispatch_Id", columns="Counter_Name", values="Counter_Value", aggfunc="sum")
m = kt.merge(piv, left_on="Dispatch_Id", right_index=True, how="inner")
h = m[m["level"] > 0]
cols = [c for c in piv.columns]
g = h.groupby("level").agg(n=("us", "size"), us=("us", "median"), **{c: (c, "median") for c in cols})
if "SQ_LDS_BANK_CONFLICT" in g and "SQ_INSTS_LDS" in g:
    g["conflict_per_lds"] = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_INSTS_LDS"]
print(g.round(3).to_string())
root = m[base.loc[m.index].isin(["k_grad_hist"])] if len(m) else m
