#!/usr/bin/env python
"""8 (and 6) data-parallel processes on ONE GPU: every rank's outcome per configuration (CU masks on /
off), for diagnosing the 8-process rehearsal. One JSON line per configuration."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cobalt_smart_lender_ai_amd.parallel import dp_check  # noqa: E402

params = dict(dp_check.DEFAULT_PARAMS, n_estimators=3)
ref = dp_check.run(1, 240_000, params)[0]
print(json.dumps({"ref_ok": ref["ok"], "fit_s": ref.get("fit_s")}), flush=True)
for procs, env in ((8, {}), (6, {}), (8, {"COBALT_SHARED_CU_MASK": "0"}), (8, {"COBALT_EVAL_PART": "0"})):
    t0 = time.time()
    env = dict(env, COBALT_IPC_TIMEOUT_S="25")
    got = dp_check.run(procs, 240_000, params, timeout_s=150, env=env)
    print(json.dumps({"procs": procs, "env": env, "wall_s": round(time.time() - t0, 1),
                      "same": [g.get("model_sha256") == ref.get("model_sha256") for g in got],
                      "ranks": [{k: (g.get(k)[:160] if isinstance(g.get(k), str) else g.get(k))
                                 for k in ("rank", "ok", "error", "message", "fit_s", "cu_budget", "ipc_epochs")}
                                for g in got]}), flush=True)
