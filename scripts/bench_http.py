#!/usr/bin/env python
"""End-to-end REST benchmark of the scoring service (the reference's `POST /predict` with TreeSHAP,
src/api/cobalt_fast_api.py:96-108): uvicorn serving the shipped model on the GPU in a child process,
clients issuing concurrent single-row requests over HTTP/1.1 keep-alive (httpx). Reports latency
percentiles and requests/s per concurrency level, plus the micro-batch sizes the server saw
(Prometheus /metrics). Prints one JSON object."""
from __future__ import annotations

import asyncio
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
PAYLOAD = {
    "loan_amnt": 10000.0, "term": 36, "installment": 300.0, "fico_range_low": 660.0, "last_fico_range_high": 700.0,
    "open_il_12m": 1.0, "open_il_24m": 2.0, "max_bal_bc": 2000.0, "num_rev_accts": 10.0,
    "pub_rec_bankruptcies": 0.0, "emp_length_num": 3.0, "earliest_cr_line_days": 4000.0, "grade_E": 0,
    "home_ownership_MORTGAGE": 0, "verification_status_Verified": 0, "application_type_Joint App": 0,
    "hardship_status_BROKEN": 0, "hardship_status_COMPLETE": 0, "hardship_status_COMPLETED": 0,
    "hardship_status_No Hardship": 0,
}


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _request_bytes(port: int) -> bytes:
    body = json.dumps(PAYLOAD).encode()
    return (f"POST /predict HTTP/1.1\r\nHost: 127.0.0.1:{port}\r\nContent-Type: application/json\r\n"
            f"Content-Length: {len(body)}\r\n\r\n").encode() + body


async def _client(port: int, conns: int, n_per: int) -> list[float]:
    """``conns`` keep-alive connections, each sending ``n_per`` requests back to back (raw sockets and a
    pre-encoded request: the load generator must not be the bottleneck)."""
    req = _request_bytes(port)
    lat: list[float] = []

    async def one():
        r, w = await asyncio.open_connection("127.0.0.1", port)
        for _ in range(n_per):
            t = time.perf_counter()
            w.write(req)
            await w.drain()
            head = await r.readuntil(b"\r\n\r\n")
            assert head.startswith(b"HTTP/1.1 200"), head[:40]
            clen = int([ln for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0].split(b":")[1])
            await r.readexactly(clen)
            lat.append(time.perf_counter() - t)
        w.close()

    await asyncio.gather(*[one() for _ in range(conns)])
    return lat


def _client_proc(args) -> list[float]:
    port, conns, n_per = args
    return asyncio.run(_client(port, conns, n_per))


def _run_level(port: int, procs: int, conns: int, n_per: int) -> dict:
    import multiprocessing as mp

    with mp.get_context("fork").Pool(procs) as pool:
        t0 = time.perf_counter()
        parts = pool.map(_client_proc, [(port, conns, n_per)] * procs)
        dt = time.perf_counter() - t0
    a = np.concatenate([np.array(p) for p in parts]) * 1e3
    return {"concurrency": procs * conns, "requests": int(a.size), "req_per_s": round(a.size / dt, 1),
            "p50_ms": round(float(np.percentile(a, 50)), 3), "p99_ms": round(float(np.percentile(a, 99)), 3)}


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--mode", choices=["split", "replicated"], default="split",
                    help="workers > 1: `serve --workers N` (one GPU scorer process, SO_REUSEPORT workers) or "
                         "`uvicorn --workers N` with one engine per worker")
    a = ap.parse_args()
    port = _port()
    env = dict(os.environ, COBALT_MODEL_PATH=str(ROOT / "src/api/models/xgb_model_tree.pkl"),
               PYTHONPATH=str(ROOT))
    split = a.workers > 1 and a.mode == "split"
    if split:  # the CLI path: one GPU scorer process + N CPU-only SO_REUSEPORT workers
        cmd = [sys.executable, "-m", "cobalt_smart_lender_ai_amd", "serve", "--host", "127.0.0.1",
               "--port", str(port), "--log-level", "warning", "--workers", str(a.workers)]
    else:
        cmd = [sys.executable, "-m", "uvicorn", "cobalt_smart_lender_ai_amd.serve.app:create_app", "--factory",
               "--host", "127.0.0.1", "--port", str(port), "--log-level", "warning", "--workers", str(a.workers)]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env)
    url = f"http://127.0.0.1:{port}"
    try:
        import httpx

        up = 0
        for _ in range(900):  # model load + hipGraph capture at startup (every worker)
            try:
                if httpx.get(url + "/health", timeout=1.0).json().get("status") == "ok":
                    up += 1
                    if up >= 3 * a.workers:
                        break
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.2)
        else:
            raise RuntimeError("server did not come up")
        time.sleep(3.0 if a.workers > 1 and not split else 0.0)  # let the other workers finish their capture
        levels = []
        for procs, conns, n in ((1, 1, 400), (4, 4, 200), (4, 16, 100), (8, 32, 40)):
            levels.append(_run_level(port, procs, conns, n))
            print(json.dumps(levels[-1]), file=sys.stderr, flush=True)
        health = httpx.get(url + "/health").json()
        if split:  # the scorer batches for every worker: its own counters
            batches, rows = float(health["batches"]), float(health["rows"])
        else:
            metrics = httpx.get(url + "/metrics").text
            cnt = [ln for ln in metrics.splitlines() if ln.startswith("cobalt_microbatch_rows_count")]
            tot = [ln for ln in metrics.splitlines() if ln.startswith("cobalt_microbatch_rows_sum")]
            batches = float(cnt[0].split()[-1]) if cnt else 0.0
            rows = float(tot[0].split()[-1]) if tot else 0.0
    finally:
        srv.terminate()
        srv.wait(timeout=60)
    print(json.dumps({"metric": "POST /predict (probability + TreeSHAP) over HTTP, 1 MI355X", "levels": levels,
                      "server_workers": a.workers, "mode": "split" if split else "single/replicated",
                      "mean_rows_per_microbatch": round(rows / batches, 2) if batches else None,
                      "device": health.get("device"), "hipgraphs": health.get("graphs")}), flush=True)


if __name__ == "__main__":
    main()
