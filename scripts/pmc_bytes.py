#!/usr/bin/env python
"""Per-kernel bytes from a rocprofv3 --pmc counter CSV (FETCH_SIZE / WRITE_SIZE, KB per dispatch) joined
with the kernel-trace durations of the same run: MB per dispatch and the implied bandwidth.
usage: pmc_bytes.py counter_collection.csv kernel_trace.csv"""
import sys

import pandas as pd

c = pd.read_csv(sys.argv[1])
k = pd.read_csv(sys.argv[2])
c["name"] = c["Kernel_Name"].str.split("(").str[0].str.replace("void ", "", regex=False).str.slice(0, 40)
k["name"] = k["Kernel_Name"].str.split("(").str[0].str.replace("void ", "", regex=False).str.slice(0, 40)
k["us"] = (k["End_Timestamp"] - k["Start_Timestamp"]) / 1000
v = c.groupby(["name", "Counter_Name"])["Counter_Value"].mean().unstack()
d = k.groupby("name")["us"].agg(["mean", "size"])
out = v.join(d, how="inner")
for col in v.columns:
    out[col + "_MB"] = out[col] / 1024.0
    out[col + "_TBps"] = out[col] * 1024.0 / (out["mean"] * 1e-6) / 1e12
keep = [x for x in out.columns if x.endswith("_MB") or x.endswith("_TBps")] + ["mean", "size"]
print(out[keep].sort_values("mean", ascending=False).head(14).round(3).to_string())
