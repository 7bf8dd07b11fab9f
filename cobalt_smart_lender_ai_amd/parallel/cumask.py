"""CU partitioning for several ranks that share ONE GPU (the 1-GPU rehearsal of multi-GPU data
parallelism).

On an 8-GPU node every rank owns a whole device. When N rank processes share one device instead,
their kernels compete for the same compute units, and the data-parallel exchange waits inside
kernels (the fused IPC exchange of ``csrc/gbdt.hip``): with 8 ranks the blocks of 7 ranks that are
already waiting can occupy every CU while the 8th rank's publishing block never gets one -- observed
as a 120 s group deadline at 8 processes (round 4), while 2-4 processes ran. A GPU does not preempt a
running wave for another process's queue, so the fix is the hardware's own partitioning: each rank
launches on a stream whose CU mask (``hipExtStreamCreateWithCUMask``) holds a disjoint 1/N of the
CUs, like a small GPU of its own. The mask interleaves the ranks (CU ``rank + k * N``), so every rank
has CUs in every XCD whichever way the runtime maps mask bits onto the XCDs. ``COBALT_CU_BUDGET``
tells the trainer's launch heuristics how many CUs it has (e.g. the fused evaluation + partition
pass only runs while its whole grid is resident).

Measured on one MI355X (scripts/dp8_diag.py, profiles/round4/dp_shared_gpu.txt): with masks, 2-5
processes run at full speed (5 ranks: 0.14 s per 1-tree fit, the 1-process model); from 6 processes
on, the masked fits deadlock at the in-kernel exchange (every rank times out). Unmasked, 6 and 8
processes are time-sliced by the GPU's queue scheduler -- slow (8 ranks: 12.6 s for one tree) but
every rank finishes with the 1-process model, byte for byte. So the masks are the default only up
to 5 ranks per device. None of this applies to the production layout (one process per GPU).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_HIP = None


def _hip() -> ctypes.CDLL:
    global _HIP
    if _HIP is None:
        p = Path(torch.__file__).parent / "lib" / "libamdhip64.so"
        _HIP = ctypes.CDLL(str(p) if p.exists() else "libamdhip64.so")
        _HIP.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        _HIP.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
    return _HIP


def interleaved_mask(rank: int, world: int, n_cu: int) -> list[int]:
    """32-bit mask words selecting CUs ``rank, rank + world, rank + 2 world, ...`` of ``n_cu``."""
    words = [0] * ((n_cu + 31) // 32)
    for cu in range(rank, n_cu, world):
        words[cu // 32] |= 1 << (cu % 32)
    return words


def blocked_mask(rank: int, world: int, n_cu: int) -> list[int]:
    """32-bit mask words selecting the contiguous CU range ``[rank n / world, (rank + 1) n / world)``."""
    words = [0] * ((n_cu + 31) // 32)
    for cu in range(rank * n_cu // world, (rank + 1) * n_cu // world):
        words[cu // 32] |= 1 << (cu % 32)
    return words


def shared_device_stream(rank: int, world: int, device: torch.device) -> torch.cuda.ExternalStream:
    """A stream of ``device`` restricted to this rank's 1/world of the CUs; sets ``COBALT_CU_BUDGET``
    (call before the first fit: the trainer reads it once). ``COBALT_CU_MASK_LAYOUT``: ``interleaved``
    (default: CU rank + k * world) or ``blocked`` (a contiguous range; scripts/dp_queue_diag.py)."""
    n_cu = torch.cuda.get_device_properties(device).multi_processor_count
    layout = os.environ.get("COBALT_CU_MASK_LAYOUT", "interleaved")
    words = blocked_mask(rank, world, n_cu) if layout == "blocked" else interleaved_mask(rank, world, n_cu)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = _hip().hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    os.environ["COBALT_CU_BUDGET"] = str(sum(bin(w).count("1") for w in words))
    return torch.cuda.ExternalStream(h.value, device=device)


def placement(stream: torch.cuda.ExternalStream | None, device: torch.device, blocks: int = 1024) -> dict:
    """Where a grid launched on ``stream`` runs (csrc/ipccomm.hip ``cobalt_hw_ids``): the XCCs and the
    number of distinct CUs its blocks landed on. Only call on a mask that covers every XCC (a mask that
    leaves one out never finishes the launch)."""
    from .. import _native

    out = torch.zeros(blocks, dtype=torch.int32, device=device)
    s = stream if stream is not None else torch.cuda.current_stream(device)
    rc = _native.lib().cobalt_hw_ids(ctypes.c_void_p(s.cuda_stream), blocks, ctypes.c_void_p(out.data_ptr()))
    if rc != 0:
        raise RuntimeError(f"cobalt_hw_ids failed ({rc})")
    s.synchronize()
    ids = out.cpu().numpy().astype("int64")
    return {"xccs": sorted({int(v >> 16) for v in ids}), "cus": len({int(v) for v in ids})}


MAX_MASKED_RANKS = 5


def want_shared_mask(world: int) -> bool:
    """Partition the CUs when ranks share a device (``COBALT_SHARED_CU_MASK``: default on for 2 to
    ``MAX_MASKED_RANKS`` ranks, off above -- see the module notes; "1" forces it on, "0" off)."""
    env = os.environ.get("COBALT_SHARED_CU_MASK")
    if env is not None:
        return world > 1 and env != "0"
    return 1 < world <= MAX_MASKED_RANKS
