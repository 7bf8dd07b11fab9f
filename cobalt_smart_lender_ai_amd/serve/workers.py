"""Multi-process HTTP front end: N uvicorn servers on one port via ``SO_REUSEPORT``.

Why not ``uvicorn --workers N``: uvicorn 0.52 hands the parent's listening socket to spawned children
through ``socket.fromfd``, which yields a socket whose ``proto`` is 0, so asyncio's transport does
not recognise it as TCP and never sets ``TCP_NODELAY`` on accepted connections. Nagle plus the
client's delayed ACK then add ~40-50 ms to every keep-alive response (measured: 0.48 ms -> 44 ms p50
on a trivial FastAPI route going from 1 to 2 workers; scripts/bench_http.py). Here every worker
creates its own ``IPPROTO_TCP`` socket with ``SO_REUSEPORT``: the kernel spreads connections over
the workers' accept queues (no shared-accept thundering herd) and asyncio sets ``TCP_NODELAY``.
"""
from __future__ import annotations

import multiprocessing as mp
import signal
import socket

APP = "cobalt_smart_lender_ai_amd.serve.app:create_app"


def reuseport_socket(host: str, port: int) -> socket.socket:
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.set_inheritable(True)
    return s


def _worker(host: str, port: int, log_level: str) -> None:
    import uvicorn

    sock = reuseport_socket(host, port)
    cfg = uvicorn.Config(APP, factory=True, host=host, port=port, log_level=log_level, backlog=2048)
    uvicorn.Server(cfg).run(sockets=[sock])


def run_workers(host: str, port: int, n: int, log_level: str = "info") -> int:
    """Start ``n`` worker processes on ``host:port`` and wait; SIGTERM/SIGINT stops them all."""
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(host, port, log_level), daemon=False) for _ in range(n)]
    for p in procs:
        p.start()

    signalled = []

    def stop():
        for p in procs:
            if p.is_alive():
                p.terminate()

    def on_signal(*_):
        signalled.append(1)
        stop()

    old = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        for p in procs:
            p.join()
    finally:
        stop()
        for p in procs:
            p.join(timeout=30)
        for sig, h in old.items():
            signal.signal(sig, h)
    if signalled:  # we were asked to stop: exit codes -SIGTERM are the expected outcome
        return 0
    return max(abs(p.exitcode or 0) for p in procs)
