"""Task-parallel model selection across GPUs (SURVEY.md §2.6 "Task parallel (model-level)").

The reference spreads RandomizedSearchCV's 60 fits over CPU worker processes
(``n_jobs=-1``, src/model_train_test/model_tree_train_test.py:148-157). Here a :class:`GpuTaskPool`
holds one worker process per slot, slot ``i`` bound to GPU ``i % n_gpus``; each worker runs whole
fits (and binds its device once, on its first task). Several slots may share a GPU: a search fit on
~100k rows is launch-latency bound, so 2-4 concurrent processes per device overlap their kernels.

Create the pool BEFORE the parent process makes its first HIP call (``torch.cuda.is_available()``,
a tensor on the GPU, a kernel): a spawned child of a process with an initialised HIP runtime
inherits that state, and some pools refuse such spawns outright. :func:`visible_gpus` counts devices
without initialising HIP.
"""
from __future__ import annotations

import multiprocessing as mp
import os
from typing import Any, Callable, Iterable

_SLOT: dict[str, Any] = {}


def visible_gpus() -> int:
    """Number of visible GPUs, without initialising the HIP runtime (device_count() does not)."""
    import torch

    try:
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 0


def _init_slot(counter, n_gpus: int) -> None:
    with counter.get_lock():
        slot = counter.value
        counter.value += 1
    _SLOT["slot"] = slot
    _SLOT["gpu"] = (slot % n_gpus) if n_gpus > 0 else None
    # each worker owns its process-wide CPU thread pools: keep them small beside the GPU work
    os.environ.setdefault("OMP_NUM_THREADS", "2")


def worker_device(device_type: str = "cuda") -> str:
    """The device string of the current pool worker (``cuda:N``; ``cpu`` without GPUs or when the
    caller asked for CPU work)."""
    gpu = _SLOT.get("gpu")
    if gpu is None or device_type != "cuda":
        return "cpu"
    import torch

    torch.cuda.set_device(gpu)
    return f"cuda:{gpu}"


class GpuTaskPool:
    """``workers`` spawned worker processes over ``n_gpus`` GPUs (default: all visible)."""

    def __init__(self, workers: int, n_gpus: int | None = None):
        self.n_gpus = visible_gpus() if n_gpus is None else int(n_gpus)
        self.workers = max(1, int(workers))
        ctx = mp.get_context("spawn")
        counter = ctx.Value("i", 0)
        self._pool = ctx.Pool(self.workers, initializer=_init_slot, initargs=(counter, self.n_gpus))

    def map(self, fn: Callable, tasks: Iterable) -> list:
        return self._pool.map(fn, list(tasks), chunksize=1)

    def close(self) -> None:
        if self._pool is not None:
            self._pool.close()
            self._pool.join()
            self._pool = None

    def __enter__(self) -> "GpuTaskPool":
        return self

    def __exit__(self, *exc) -> None:
        if self._pool is not None:
            self._pool.terminate()
            self._pool.join()
            self._pool = None


def resolve_workers(fits_in_parallel: int | None) -> int:
    """``TrainConfig.fits_in_parallel``: None = one worker per visible GPU (1 without GPUs)."""
    if fits_in_parallel is None:
        return max(1, visible_gpus())
    return max(1, int(fits_in_parallel))


def can_auto_pool(device=None) -> bool:
    """Whether a caller may create a :class:`GpuTaskPool` on its own: only for GPU work, and only from
    a process that has not initialised HIP yet (its children would inherit the runtime's state, and
    the pool refuses such spawns). Otherwise the caller logs why and runs in-process."""
    import logging

    import torch

    dev_type = torch.device(device).type if device is not None else ("cuda" if visible_gpus() else "cpu")
    if dev_type != "cuda":
        return False
    if torch.cuda.is_initialized():
        logging.getLogger(__name__).warning(
            "not creating a GPU task pool: HIP is already initialised in this process (create the pool "
            "before the first GPU call and pass it in); running the fits in this process")
        return False
    return True
