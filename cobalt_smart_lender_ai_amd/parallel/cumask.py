"""CU partitioning for several ranks that share ONE GPU (the 1-GPU rehearsal of multi-GPU data
parallelism).

On an 8-GPU node every rank owns a whole device. When N rank processes share one device instead,
their kernels compete for the same compute units, and the data-parallel exchange waits inside
kernels (the fused IPC exchange of ``csrc/gbdt.hip``): unpartitioned, the GPU time-slices the
processes' queues (8 ranks: 12.6 s for one tree, round 4). A GPU does not preempt a running wave for
another process's queue, so the fix is the hardware's own partitioning: each rank launches on a
stream whose CU mask (``hipExtStreamCreateWithCUMask``) holds a disjoint 1/N of the CUs, like a
small GPU of its own. ``COBALT_CU_BUDGET`` tells the trainer's launch heuristics how many CUs it has.

The mask must give the rank CUs in EVERY XCC: a dispatch hands each of the 8 XCCs its round-robin
share of the grid, and the share of an XCC with no CU in the mask never runs. Measured on one MI355X
(round 5, ``scripts/dp_queue_diag.py`` with the ``cobalt_hw_ids`` placement probe,
``profiles/round5/qdiag_masks.txt``): the mask bits go to the XCCs round-robin (bit i -> XCC i mod 8),
so the former default layout -- CU ``rank + k * N`` -- gave rank r of 6 only the XCCs of r's parity and
every 6-rank fit deadlocked, while a BLOCKED layout -- a contiguous range of N-th of the bits, >= 8
consecutive bits for any N <= 32 -- covers all 8 XCCs: 6 and 8 masked ranks run at full speed (8 ranks:
32 CUs each, 4 per XCC, the 1-process model byte for byte). (With 2 and 4 ranks the interleaved masks
were not applied at all -- the probe saw every rank's blocks on all 256 CUs -- so those runs had been
time-sliced rather than partitioned.) The blocked layout is the default for 2-8 sharing ranks.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch
from ..config import knob

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
    (call before the first fit: the trainer reads it once). ``COBALT_CU_MASK_LAYOUT``: ``blocked``
    (default: a contiguous range of mask bits, every XCC covered) or ``interleaved`` (CU rank + k * world;
    leaves XCCs empty when world and 8 share a factor -- scripts/dp_queue_diag.py)."""
    n_cu = torch.cuda.get_device_properties(device).multi_processor_count
    layout = knob("COBALT_CU_MASK_LAYOUT", "blocked")
    words = interleaved_mask(rank, world, n_cu) if layout == "interleaved" else blocked_mask(rank, world, n_cu)
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


MAX_MASKED_RANKS = 8


def want_shared_mask(world: int) -> bool:
    """Partition the CUs when ranks share a device (``COBALT_SHARED_CU_MASK``: default on for 2 to
    ``MAX_MASKED_RANKS`` ranks, off above -- see the module notes; "1" forces it on, "0" off)."""
    env = knob("COBALT_SHARED_CU_MASK")
    if env is not None:
        return world > 1 and env != "0"
    return 1 < world <= MAX_MASKED_RANKS
