"""In-process multi-rank simulation of the data-parallel path (test infrastructure).

``run_ranks(world, fn)`` runs ``fn(ctx)`` on ``world`` host threads of this process, all on one
device, each thread on its own HIP stream with a :class:`LoopbackContext`: the Python-side
collectives (``allreduce``, ``allgather_rows``, ``barrier``) meet through a ``threading.Barrier``
and the native communicator is a rank of ``csrc/loopcomm.hip``'s loopback group, so the C++
trainer enqueues exactly the per-level collectives it enqueues on RCCL. This exercises the N-rank
GBDT protocol (sharded rows, global histograms, child-choice consistency) on a single GPU, where
RCCL cannot host two ranks. Not a production transport: use :mod:`.dist` (RCCL over xGMI) for that.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass, field
from typing import Any, Callable

import torch

from .dist import DistContext


class _Group:
    def __init__(self, world: int, timeout: float):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots: list[Any] = [None] * world


@dataclass
class LoopbackContext(DistContext):
    group: _Group | None = field(default=None, repr=False)

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world == 1:
            return t
        g = self.group
        g.slots[self.rank] = t.detach().to("cpu", copy=True)
        g.barrier.wait()
        vals = torch.stack(g.slots)
        red = {"sum": lambda v: v.sum(0), "max": lambda v: v.max(0).values, "min": lambda v: v.min(0).values}[op]
        out = red(vals).to(t.dtype)
        g.barrier.wait()
        t.copy_(out.to(t.device))
        return t

    def allgather_rows(self, t: torch.Tensor, pad_value: float = float("nan")) -> torch.Tensor:
        if self.world == 1:
            return t
        g = self.group
        g.slots[self.rank] = t.detach().to("cpu", copy=True)
        g.barrier.wait()
        out = torch.cat(list(g.slots), 0)
        g.barrier.wait()
        return out.to(t.device)

    def barrier(self) -> None:
        if self.world > 1:
            self.group.barrier.wait()

    def _coll_device(self, dev) -> torch.device:
        return torch.device("cpu")

    def close(self) -> None:
        if self.native_comm:
            from .. import _native

            _native.lib().cobalt_comm_destroy(ctypes.c_void_p(self.native_comm), 0)
            self.native_comm = None


def run_ranks(world: int, fn: Callable[[LoopbackContext], Any], device: str | torch.device = "cuda:0",
              timeout: float = 600.0) -> list[Any]:
    """Run ``fn(ctx)`` for ranks 0..world-1 concurrently (threads) and return their results.
    ``device="cpu"``: host-only ranks (no native communicator; the small collectives still meet)."""
    dev = torch.device(device)
    gpu = dev.type == "cuda"
    lib = None
    grp = ctypes.c_void_p()
    if gpu:
        from .. import _native

        lib = _native.lib()
        rc = lib.cobalt_comm_loop_group(world, ctypes.byref(grp))
        if rc:
            raise RuntimeError(f"cobalt_comm_loop_group failed ({rc})")
    pg = _Group(world, timeout)
    results: list[Any] = [None] * world
    errors: list[BaseException | None] = [None] * world

    def body(r: int) -> None:
        h = ctypes.c_void_p()
        ctx = None
        try:
            if gpu and lib.cobalt_comm_loop_rank(grp, r, ctypes.byref(h)):
                raise RuntimeError("cobalt_comm_loop_rank failed")
            ctx = LoopbackContext(rank=r, world=world, local_rank=dev.index or 0, backend="loopback",
                                  native_comm=h.value if gpu else None, group=pg)
            if not gpu:
                results[r] = fn(ctx)
                return
            torch.cuda.set_device(dev)
            with torch.cuda.stream(torch.cuda.Stream(dev)):
                results[r] = fn(ctx)
                torch.cuda.current_stream(dev).synchronize()
        except BaseException as e:  # noqa: BLE001
            errors[r] = e
            pg.barrier.abort()
        finally:
            if ctx is not None:
                ctx.close()

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if gpu:
        torch.cuda.synchronize(dev)
        lib.cobalt_comm_loop_group_free(grp)
    failed = [e for e in errors if e is not None]
    if failed:  # the root cause first (peers fail with barrier / communicator errors after it)
        first = next((e for e in failed if not isinstance(e, threading.BrokenBarrierError)), failed[0])
        first.rank_errors = errors
        raise first
    return results
