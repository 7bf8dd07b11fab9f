#!/bin/bash
# Texture-addresser (load path) busy cycles per trainer kernel: TA_TA_BUSY summed over the CUs' TA
# instances vs GRBM_GUI_ACTIVE cycles of the dispatch (10M rows x 20 trees).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmcta -o run -- python3 $R/bench.py --trees 20 --steps 1 --warmup 0 --test-rows 10000 > $R/gpurun_out/pmcta.log 2>&1 || exit $?
f=$(find /tmp/pmcta -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > $R/gpurun_out/pmc_ta_summary.txt
import sys, pandas as pd
pd.set_option("display.width", 250)
t = pd.read_csv(sys.argv[1])
t["name"] = t["Kernel_Name"].str.replace("void ", "").str.split("(").str[0].str.slice(0, 26)
t = t[t["name"].str.startswith("k_")]
g = t.groupby(["name", "Counter_Name"])["Counter_Value"].sum().unstack()
g["TA_busy_frac_per_CU"] = g["TA_TA_BUSY_sum"] / (256 * g["GRBM_GUI_ACTIVE"])
print(g.to_string(float_format=lambda v: f"{v:.4g}"))
PY
cat $R/gpurun_out/pmc_ta_summary.txt
