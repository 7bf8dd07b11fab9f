#!/usr/bin/env python
"""8 (and 6) data-parallel processes on ONE GPU: every rank's outcome per configuration (CU masks on /
off), for diagnosing the 8-process rehearsal. One JSON line per configuration."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cobalt_smart_lender_ai_amd.parallel import dp_check  # noqa: E402



def _heartbeat() -> None:  # a line every 30 s while the ranks run (silent GPU commands count as hung)
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[dp8_diag] {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main() -> None:
    _heartbeat()
    trees = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=trees)
    ref = dp_check.run(1, 240_000, params)[0]
    print(json.dumps({"ref_ok": ref["ok"], "fit_s": ref.get("fit_s")}), flush=True)
    sets = {"queues": ((8, {"GPU_MAX_HW_QUEUES": "1"}), (8, {"GPU_MAX_HW_QUEUES": "2"}), (6, {}), (8, {})),
            "width": ((5, {"COBALT_IPC_TIMEOUT_S": "100"}), (6, {"COBALT_IPC_TIMEOUT_S": "100"}),
                      (6, {"COBALT_IPC_TIMEOUT_S": "100", "COBALT_SHARED_CU_MASK": "0"})),
            "eight1": ((8, {"COBALT_IPC_TIMEOUT_S": "250", "COBALT_SHARED_CU_MASK": "0"}),),
            "eight": ((8, {"COBALT_IPC_TIMEOUT_S": "250", "COBALT_SHARED_CU_MASK": "0", "GPU_MAX_HW_QUEUES": "1"}),
                      (8, {"COBALT_IPC_TIMEOUT_S": "250", "COBALT_SHARED_CU_MASK": "0"}))}
    configs = sets[sys.argv[1] if len(sys.argv) > 1 else "queues"]
    for procs, env in configs:
        t0 = time.time()
        env = dict({"COBALT_IPC_TIMEOUT_S": "25"}, **env)
        got = dp_check.run(procs, 240_000, params, timeout_s=float(env["COBALT_IPC_TIMEOUT_S"]) + 40, env=env)
        print(json.dumps({"procs": procs, "env": env, "wall_s": round(time.time() - t0, 1),
                          "same": [g.get("model_sha256") == ref.get("model_sha256") for g in got],
                          "ranks": [{k: (g.get(k)[:160] if isinstance(g.get(k), str) else g.get(k))
                                     for k in ("rank", "ok", "error", "message", "fit_s", "cu_budget", "ipc_epochs")}
                                    for g in got]}), flush=True)


if __name__ == "__main__":  # (the ranks are spawned: they re-import this file)
    main()
