"""Asynchronous micro-batcher for single-row scoring requests.

Each ``/predict`` request is one row (reference: src/api/cobalt_fast_api.py:96-108). Concurrent
requests are queued; a single worker task drains the queue, waiting at most ``max_wait_ms`` for more
rows (up to ``max_batch``), scores them in one engine call (one hipGraph replay per bucket) on a
worker thread, and resolves every request's future with its own row of the result.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

import numpy as np

from .engine import ScoringEngine


@dataclass
class BatcherStats:
    batches: int = 0
    rows: int = 0
    max_batch_seen: int = 0
    busy_s: float = 0.0
    hist: dict[int, int] = field(default_factory=dict)


class MicroBatcher:
    def __init__(self, engine: ScoringEngine, max_batch: int = 512, max_wait_ms: float = 1.0):
        self.engine = engine
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1000.0
        self._queue: asyncio.Queue | None = None
        self._task: asyncio.Task | None = None
        self.stats = BatcherStats()
        self.on_batch = None  # optional callback(rows) per scored batch (serving metrics)

    async def start(self) -> None:
        if self._task is None:
            self._queue = asyncio.Queue()
            self._task = asyncio.create_task(self._run())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
            self._task = None

    async def submit(self, row: np.ndarray) -> tuple[float, np.ndarray]:
        if self._task is None:
            await self.start()
        fut = asyncio.get_running_loop().create_future()
        await self._queue.put((np.asarray(row, dtype=np.float32).reshape(-1), fut))
        return await fut

    async def _run(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            first = await self._queue.get()
            items = [first]
            # drain what is already queued; if that is not a full batch, give concurrent requests one
            # short window (a single sleep -- not a wait_for per item, which cost more than it saved)
            while len(items) < self.max_batch and not self._queue.empty():
                items.append(self._queue.get_nowait())
            if len(items) < self.max_batch and self.max_wait > 0:
                await asyncio.sleep(self.max_wait)
                while len(items) < self.max_batch and not self._queue.empty():
                    items.append(self._queue.get_nowait())
            X = np.stack([r for r, _ in items])
            t0 = time.perf_counter()
            try:
                probs, phis = await loop.run_in_executor(None, self.engine.score, X, True)
            except Exception as e:  # noqa: BLE001
                for _, f in items:
                    if not f.done():
                        f.set_exception(e)
                continue
            self.stats.busy_s += time.perf_counter() - t0
            self.stats.batches += 1
            self.stats.rows += len(items)
            self.stats.max_batch_seen = max(self.stats.max_batch_seen, len(items))
            self.stats.hist[len(items)] = self.stats.hist.get(len(items), 0) + 1
            if self.on_batch is not None:
                self.on_batch(len(items))
            for i, (_, f) in enumerate(items):
                if not f.done():
                    f.set_result((float(probs[i]), phis[i]))
