#!/bin/bash
# HBM traffic per trainer kernel (TCC FETCH_SIZE / WRITE_SIZE, one pass each) for a 20-tree 10M fit,
# with the kernel durations from the same runs: achieved GB/s per kernel.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
: > $R/gpurun_out/pmc_bytes_summary.txt
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmcb$i -o run -- python3 $R/bench.py --trees 20 --steps 1 --warmup 0 --test-rows 10000 "$@" > $R/gpurun_out/pmcb_$i.log 2>&1 || exit $?
  f=$(find /tmp/pmcb$i -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$set" <<'PY' >> $R/gpurun_out/pmc_bytes_summary.txt
import sys, pandas as pd
pd.set_option("display.width", 250)
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.replace("void ", "").str.split("(").str[0].str.slice(0, 26)
t = t[t["name"].str.startswith("k_")]
# counter value per dispatch (summed over the counter's instances), duration from the dispatch's timestamps
print("columns:", list(t.columns))
if "Start_Timestamp" in t.columns:
    g = t.groupby(["Dispatch_Id", "name"]).agg(v=("Counter_Value", "sum"), s=("Start_Timestamp", "first"),
                                                e=("End_Timestamp", "first")).reset_index()
    g["us"] = (g["e"] - g["s"]) / 1e3
else:
    g = t.groupby(["Dispatch_Id", "name"]).agg(v=("Counter_Value", "sum")).reset_index()
    g["us"] = float("nan")
a = g.groupby("name").agg(calls=("v", "size"), kbytes=("v", "sum"), us=("us", "sum"))
a["MB_per_call"] = a["kbytes"] / a["calls"] / 1e3
a["GB_per_s"] = a["kbytes"] * 1e3 / (a["us"] * 1e3)
print(f"== {sys.argv[2]} (KB units as reported) ==")
print(a.sort_values("us", ascending=False).round(2).to_string())
PY
done
cat $R/gpurun_out/pmc_bytes_summary.txt
