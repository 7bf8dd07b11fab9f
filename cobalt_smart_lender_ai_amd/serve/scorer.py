"""One GPU scoring process shared by several HTTP worker processes.

A single Python event loop tops out near ~1.7k requests/s on HTTP parsing and validation, and
several GPU-owning server processes on one device time-slice its contexts (~50 ms per request with
8 of them, docs/PERF.md). The production shape is therefore: N uvicorn workers that only speak HTTP
(CPU), and ONE scorer process that owns the GPU -- the ScoringEngine's hipGraph buckets and a
micro-batcher that now batches the requests of all workers together.

Transport: a Unix-domain stream socket, binary frames (little endian).
  request  = u32 request id | u32 rows | u8 want_shap | rows x F float32
  response = u32 request id | u32 rows | u8 status | u32 extra bytes | extra
             status 0: extra = rows float32 probabilities [+ rows x F float64 SHAP]
             status 1: extra = utf-8 error message (the engine raised; the request fails, the
                       scorer keeps serving)
  A request with 0 rows asks for the scorer's batching statistics (status 0, extra = JSON).
Each worker keeps one connection and multiplexes its in-flight requests by id.
"""
from __future__ import annotations

import asyncio
import json
import os
import struct
import sys
import time
from pathlib import Path

import numpy as np

_REQ = struct.Struct("<IIB")
_RSP = struct.Struct("<IIBI")


# ---------------------------------------------------------------------------------------- server
class _Server:
    def __init__(self, engine, max_batch: int, max_wait_ms: float):
        self.engine = engine
        self.F = engine.F
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1000.0
        self.queue: asyncio.Queue = asyncio.Queue()
        self.stats = {"batches": 0, "rows": 0, "requests": 0, "max_batch_seen": 0, "device": str(engine.device)}

    async def handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        lock = asyncio.Lock()
        try:
            while True:
                head = await reader.readexactly(_REQ.size)
                rid, n, shap = _REQ.unpack(head)
                if n == 0:
                    msg = json.dumps(self.stats).encode()
                    async with lock:
                        writer.write(_RSP.pack(rid, 0, 0, len(msg)) + msg)
                        await writer.drain()
                    continue
                X = np.frombuffer(await reader.readexactly(4 * n * self.F), dtype=np.float32).reshape(n, self.F)
                await self.queue.put((X, bool(shap), rid, writer, lock))
        except (asyncio.IncompleteReadError, ConnectionResetError):
            pass
        finally:
            writer.close()

    async def run_batches(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            items = [await self.queue.get()]
            rows = items[0][0].shape[0]
            while rows < self.max_batch and not self.queue.empty():
                items.append(self.queue.get_nowait())
                rows += items[-1][0].shape[0]
            if rows < self.max_batch and self.max_wait > 0:
                await asyncio.sleep(self.max_wait)
                while rows < self.max_batch and not self.queue.empty():
                    items.append(self.queue.get_nowait())
                    rows += items[-1][0].shape[0]
            X = np.concatenate([it[0] for it in items]) if len(items) > 1 else items[0][0]
            want = any(it[1] for it in items)
            try:
                probs, phis = await loop.run_in_executor(None, self.engine.score, X, want)
                err = None
            except Exception as e:  # noqa: BLE001
                err = repr(e).encode()
            st = self.stats
            st["batches"] += 1
            st["rows"] += rows
            st["requests"] += len(items)
            st["max_batch_seen"] = max(st["max_batch_seen"], rows)
            s = 0
            for Xi, shap, rid, writer, lock in items:
                n = Xi.shape[0]
                if err is not None:
                    frame = _RSP.pack(rid, n, 1, len(err)) + err
                else:
                    body = [probs[s:s + n].astype(np.float32).tobytes()]
                    if shap:
                        body.append(np.ascontiguousarray(phis[s:s + n], dtype=np.float64).tobytes())
                    extra = b"".join(body)
                    frame = _RSP.pack(rid, n, 0, len(extra)) + extra
                s += n
                async with lock:
                    writer.write(frame)
                    try:
                        await writer.drain()
                    except ConnectionResetError:
                        pass


async def start_server(engine, socket_path: str, max_batch: int = 512, max_wait_ms: float = 1.0):
    """Listen on ``socket_path`` with ``engine`` (in the running loop); returns the asyncio server."""
    srv = _Server(engine, max_batch, max_wait_ms)
    if os.path.exists(socket_path):
        os.unlink(socket_path)
    server = await asyncio.start_unix_server(srv.handle, path=socket_path)
    server._cobalt_batches = asyncio.get_running_loop().create_task(srv.run_batches())
    return server


def serve(socket_path: str, model_path: str | None = None, device: str | None = None, max_batch: int = 512,
          max_wait_ms: float = 1.0, ready_file: str | None = None) -> None:
    """Run the scorer (blocking): load the model, capture the engine's graphs, listen on the socket."""
    from ..config import ServeConfig, from_env
    from .app import load_model
    from .engine import ScoringEngine

    cfg = from_env(ServeConfig)
    if model_path:
        cfg.model_path = model_path
    engine = ScoringEngine(load_model(cfg), device=device or cfg.device, use_graphs=cfg.use_graphs)

    async def main():
        server = await start_server(engine, socket_path, max_batch, max_wait_ms)
        if ready_file:
            Path(ready_file).write_text(str(engine.device))
        print(f"[INFO] scorer on {engine.device} listening at {socket_path}", flush=True)
        async with server:
            await server.serve_forever()

    asyncio.run(main())


# ---------------------------------------------------------------------------------------- client
class RemoteScorer:
    """Async client of the scorer (one connection per worker process, requests multiplexed by id).
    ``submit`` has the MicroBatcher's signature, ``score_many`` serves bulk requests."""

    def __init__(self, socket_path: str, n_feat: int):
        self.path = socket_path
        self.F = n_feat
        self._reader = self._writer = None
        self._pending: dict[int, tuple[asyncio.Future, bool]] = {}
        self._next = 0
        self._task = None
        self._wlock = None

    async def start(self, timeout_s: float = 120.0) -> None:
        t0 = time.monotonic()
        while True:
            try:
                self._reader, self._writer = await asyncio.open_unix_connection(self.path)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                if time.monotonic() - t0 > timeout_s:
                    raise RuntimeError(f"scorer socket {self.path} not available")
                await asyncio.sleep(0.1)
        self._wlock = asyncio.Lock()
        self._task = asyncio.get_running_loop().create_task(self._read_loop())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            self._task = None
        if self._writer is not None:
            self._writer.close()

    async def _read_loop(self) -> None:
        try:
            while True:
                rid, n, status, nb = _RSP.unpack(await self._reader.readexactly(_RSP.size))
                extra = await self._reader.readexactly(nb)
                fut, shap = self._pending.pop(rid)
                if fut.done():
                    continue
                if status != 0:
                    fut.set_exception(RuntimeError(f"scorer failed: {extra.decode(errors='replace')}"))
                elif n == 0:
                    fut.set_result(json.loads(extra))
                else:
                    probs = np.frombuffer(extra, dtype=np.float32, count=n)
                    phis = np.frombuffer(extra, dtype=np.float64, offset=4 * n).reshape(n, self.F) if shap else None
                    fut.set_result((probs, phis))
        except (asyncio.IncompleteReadError, ConnectionResetError) as e:
            for fut, _ in self._pending.values():
                if not fut.done():
                    fut.set_exception(RuntimeError(f"scorer connection lost: {e!r}"))
            self._pending.clear()

    async def _request(self, X: np.ndarray, with_shap: bool):
        if self._task is None:
            raise RuntimeError("RemoteScorer.start() was not awaited")
        rid = self._next
        self._next = (self._next + 1) & 0xFFFFFFFF
        fut = asyncio.get_running_loop().create_future()
        self._pending[rid] = (fut, with_shap)
        async with self._wlock:
            self._writer.write(_REQ.pack(rid, X.shape[0], 1 if with_shap else 0) + X.tobytes())
            await self._writer.drain()
        return await fut

    async def score_many(self, X: np.ndarray, with_shap: bool) -> tuple[np.ndarray, np.ndarray | None]:
        X = np.ascontiguousarray(X, dtype=np.float32)
        if X.ndim != 2 or X.shape[1] != self.F:
            raise ValueError(f"expected [N, {self.F}] features, got {X.shape}")
        if X.shape[0] == 0:
            return np.empty(0, np.float32), (np.empty((0, self.F)) if with_shap else None)
        return await self._request(X, with_shap)

    async def stats(self) -> dict:
        return await self._request(np.empty((0, self.F), np.float32), False)

    async def submit(self, row: np.ndarray) -> tuple[float, np.ndarray]:
        probs, phis = await self.score_many(np.asarray(row, dtype=np.float32).reshape(1, -1), True)
        return float(probs[0]), phis[0]


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="GPU scoring process for multi-worker serving")
    ap.add_argument("--socket", required=True)
    ap.add_argument("--model", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-batch", type=int, default=512)
    ap.add_argument("--max-wait-ms", type=float, default=1.0)
    ap.add_argument("--ready-file", default=None)
    a = ap.parse_args(argv)
    serve(a.socket, a.model, a.device, a.max_batch, a.max_wait_ms, a.ready_file)
    return 0


if __name__ == "__main__":
    sys.exit(main())
