#!/usr/bin/env python
"""In-kernel stamps of rank 0 in N CU-masked data-parallel processes sharing ONE GPU (IPC transport):
how long the fused exchange's evaluator blocks take to sum N ranks' slots, level by level.
usage: dp_rank_stamps.py ROWS_PER_RANK N [N ...]  (writes gpurun_out/dprs_<N>_rank<r>.txt raw stamps)"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from cobalt_smart_lender_ai_amd.parallel import dp_check  # noqa: E402


def main() -> None:
    per_rank = int(sys.argv[1])
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=70, subsample=1.0, colsample_bytree=1.0, learning_rate=0.05,
                  gamma=5.0)
    for n in (int(a) for a in sys.argv[2:]):
        out = Path("gpurun_out")
        for f in out.glob(f"dprs_{n}_rank*.txt"):
            f.unlink()
        res = dp_check.run(n, n * per_rank, params, timeout_s=300,
                           env={"COBALT_STAMPS": str(out.resolve() / f"dprs_{n}_rank{{rank}}.txt")})
        print(json.dumps({"procs": n, "ok": [r["ok"] for r in res], "fit_s": [round(r.get("fit_s", -1), 3) for r in res],
                          "sha_equal": len({r.get("model_sha256") for r in res}) == 1,
                          "plan": res[0].get("plan")}), flush=True)
        if not all(r["ok"] for r in res):
            print(json.dumps(res[0])[:3000], flush=True)
            sys.exit(1)


if __name__ == "__main__":  # (spawned ranks re-import this module)
    main()
