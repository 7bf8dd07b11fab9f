#!/usr/bin/env python
"""Node ownership A/B with DP processes sharing one GPU: fit seconds per rank with COBALT_DP_OWNER=1
(default) and 0, same model asserted. One JSON line per configuration."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cobalt_smart_lender_ai_amd.parallel import dp_check  # noqa: E402


def main() -> None:
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=60, subsample=1.0, colsample_bytree=1.0)
    for procs in (2, 4):
        res = {}
        for own in ("1", "0", "1", "0"):
            got = dp_check.run(procs, rows, params, timeout_s=400, env={"COBALT_DP_OWNER": own})
            assert all(g["ok"] for g in got), got
            res.setdefault(own, []).append(round(max(g["fit_s"] for g in got), 3))
            res.setdefault("sha_" + own, got[0]["model_sha256"][:16])
        print(json.dumps({"procs": procs, "rows": rows, **res}), flush=True)


if __name__ == "__main__":
    main()
