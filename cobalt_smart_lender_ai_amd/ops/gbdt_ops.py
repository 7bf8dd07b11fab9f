"""ctypes wrappers around the gfx950 GBDT trainer (``csrc/gbdt.hip``).

``GpuGbdtTrainer`` owns a native trainer context: its workspace (packed gradients, ping-pong row
indices, per-level histogram slots, node records) is allocated once per fit in HBM; inputs (bins,
labels, weights, margins) are PyTorch tensors on the same device. ``grow`` enqueues whole trees on
the current HIP stream without host synchronisation; ``fetch`` copies the node records back once.
"""
from __future__ import annotations

import atexit
import os
import threading

import ctypes

import numpy as np
import torch

from .. import _native
from ..models.booster import NODE_DTYPE
from ..config import knob


class GbdtConfig(ctypes.Structure):
    _fields_ = [
        ("n_rows", ctypes.c_int64),
        ("row_offset", ctypes.c_int64),
        ("n_feat", ctypes.c_int32),
        ("row_stride", ctypes.c_int32),
        ("max_depth", ctypes.c_int32),
        ("max_trees", ctypes.c_int32),
        ("chunk", ctypes.c_int32),
        ("feat_tile", ctypes.c_int32),
        ("eta", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("min_child_weight", ctypes.c_double),
        ("subsample", ctypes.c_double),
        ("gscale", ctypes.c_double),
        ("hscale", ctypes.c_double),
        ("base_margin", ctypes.c_float),
        ("world_size", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("comm", ctypes.c_void_p),
        ("grad_bits", ctypes.c_int32),  # 17 (packed u64 LDS cells) or 25 (wide int64 cells)
        ("reserved0", ctypes.c_int32),
    ]


assert ctypes.sizeof(GbdtConfig) == 136


def row_stride(n_feat: int) -> int:
    """Bytes per row record: bins padded to 8 bytes, then the packed (g, h) u64; 16-byte aligned so a
    record is one aligned 32-byte piece of a memory sector for the 20-feature model."""
    return ((n_feat + 7) // 8 * 8 + 8 + 15) // 16 * 16


def pick_chunk(n_rows: int) -> int:
    """Rows per histogram/partition work item: ~768 root items (3 resident 512-thread blocks per CU,
    so the root level runs in one wave of blocks), power of two in [1024, 16384] (16384 keeps the
    per-block packed sums below 2^30)."""
    target = max(1, -(-n_rows // 768))
    c = 1024
    while c < target and c < 16384:
        c *= 2
    return c


def pick_feat_tile(n_feat: int) -> int:
    """Features per histogram block: all of them up to 32 (64 KiB of LDS), else tiles of 32."""
    return min(row_stride(n_feat), 32)


def bin_matrix(X: torch.Tensor, cuts: torch.Tensor, nbins: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Quantise ``X`` [N, F] float32 (CUDA) -> (row records [N, stride] uint8 with the bins in the
    first F bytes, binsT [F, N] uint8)."""
    if X.device.type != "cuda":
        raise ValueError("bin_matrix expects a CUDA tensor")
    X = X.contiguous()
    N, F = X.shape
    st = row_stride(F)
    # the vectorised kernel (k_bin_rec32: 32-byte records, F % 4 == 0, 16-byte aligned rows) writes
    # every byte of every record; the generic one only the bins
    whole = (st == 32 and F % 4 == 0 and F <= 24 and X.data_ptr() % 16 == 0
             and not knob("COBALT_BIN_SCALAR"))
    bins = (torch.empty if whole else torch.zeros)((N, st), dtype=torch.uint8, device=X.device)
    binsT = torch.empty((F, N), dtype=torch.uint8, device=X.device)
    lib = _native.lib()
    rc = lib.cobalt_bin_matrix(X.data_ptr(), N, F, F, cuts.contiguous().data_ptr(),
                               nbins.to(torch.int32).contiguous().data_ptr(), bins.data_ptr(), st,
                               binsT.data_ptr(), _native.stream_handle())
    _native.check(rc, "cobalt_bin_matrix")
    return bins, binsT


def bin_matrix_into(X: torch.Tensor, cuts: torch.Tensor, nbins: torch.Tensor, records: torch.Tensor,
                    binsT: torch.Tensor, row0: int) -> None:
    """Quantise the chunk ``X`` [n, F] (CUDA) in place into rows ``row0 .. row0+n`` of preallocated
    ``records`` [N, stride] and ``binsT`` [F, N] (streamed ingestion: no per-chunk copies)."""
    X = X.contiguous()
    n, F = X.shape
    N, st = records.shape
    if binsT.shape != (F, N) or row0 < 0 or row0 + n > N or st != row_stride(F):
        raise ValueError("chunk does not fit the preallocated binned matrix")
    if not (records.is_contiguous() and binsT.is_contiguous()):
        raise ValueError("records/binsT must be contiguous")
    rc = _native.lib().cobalt_bin_matrix_ld(X.data_ptr(), n, F, F, cuts.contiguous().data_ptr(),
                                            nbins.to(torch.int32).contiguous().data_ptr(),
                                            records.data_ptr() + row0 * st, st, binsT.data_ptr() + row0, N,
                                            _native.stream_handle())
    _native.check(rc, "cobalt_bin_matrix_ld")


# ONE parked trainer context (the last finished fit's) for back-to-back fits of the same shapes
# (cobalt_gbdt_reuse): its device buffers are kept for the next fit instead of freed and reallocated
# (~2.5 ms of hipFree / hipMalloc per 10M-row fit). A fit of other shapes replaces it.
# COBALT_TRAINER_CACHE=0 disables; release_cached_trainers() frees it (also at exit).
_PARKED: dict[tuple, int] = {}
_PARKED_LOCK = threading.Lock()


def _cache_on() -> bool:
    return knob("COBALT_TRAINER_CACHE", "1") != "0"


def release_cached_trainers() -> None:
    with _PARKED_LOCK:
        hs = list(_PARKED.values())
        _PARKED.clear()
    if hs:
        lib = _native.lib()
        for h in hs:
            lib.cobalt_gbdt_destroy(ctypes.c_void_p(h))


atexit.register(release_cached_trainers)


class GpuGbdtTrainer:
    def __init__(self, *, n_rows: int, n_feat: int, max_depth: int, max_trees: int, eta: float,
                 reg_lambda: float, reg_alpha: float, gamma: float, min_child_weight: float, subsample: float,
                 gscale: float, hscale: float, base_margin: float, seed: int, row_offset: int = 0,
                 world_size: int = 1, comm: int | None = None, chunk: int | None = None,
                 feat_tile: int | None = None, grad_bits: int = 17):
        self.lib = _native.lib()
        cfg = GbdtConfig()
        cfg.n_rows = n_rows
        cfg.row_offset = row_offset
        cfg.n_feat = n_feat
        cfg.row_stride = row_stride(n_feat)
        cfg.max_depth = max_depth
        cfg.max_trees = max_trees
        cfg.chunk = chunk or pick_chunk(n_rows)
        cfg.feat_tile = feat_tile or pick_feat_tile(n_feat)
        cfg.eta = eta
        cfg.lambda_ = reg_lambda
        cfg.alpha = reg_alpha
        cfg.gamma = gamma
        cfg.min_child_weight = min_child_weight
        cfg.subsample = subsample
        cfg.gscale = gscale
        cfg.hscale = hscale
        cfg.base_margin = base_margin
        cfg.world_size = world_size
        cfg.seed = seed & ((1 << 64) - 1)
        cfg.comm = comm
        cfg.grad_bits = int(grad_bits)
        self.cfg = cfg
        self._key = (torch.cuda.current_device(), cfg.n_rows, cfg.n_feat, cfg.row_stride, cfg.max_depth,
                     cfg.max_trees, cfg.chunk, cfg.feat_tile, cfg.world_size, cfg.comm or 0, cfg.grad_bits)
        h = None
        if _cache_on():
            with _PARKED_LOCK:
                hp = _PARKED.pop(self._key, None)
            if hp is not None:
                if self.lib.cobalt_gbdt_reuse(ctypes.c_void_p(hp), ctypes.byref(cfg)) == 0:
                    h = ctypes.c_void_p(hp)
                else:
                    self.lib.cobalt_gbdt_destroy(ctypes.c_void_p(hp))
        if h is None:
            h = ctypes.c_void_p()
            rc = self.lib.cobalt_gbdt_create(ctypes.byref(cfg), ctypes.byref(h))
            _native.check(rc, "cobalt_gbdt_create")
        self.h = h
        self.max_nodes = int(self.lib.cobalt_gbdt_max_nodes(h))
        self._keep: list[torch.Tensor] = []

    def set_data(self, bins, binsT, cuts, nbins, label, weight, margin, fmask) -> None:
        ts = [bins, binsT, cuts, nbins, label, weight, margin, fmask]
        for t in ts:
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("trainer inputs must be contiguous CUDA tensors")
        self._keep = ts
        # cobalt_gbdt_set_data reads the bin counts with a blocking hipMemcpy, which is not ordered
        # after work on a non-default stream (e.g. the int32 conversion of ``nbins`` on a search
        # worker's stream): finish the caller's stream first
        torch.cuda.current_stream(bins.device).synchronize()
        rc = self.lib.cobalt_gbdt_set_data(self.h, *[t.data_ptr() for t in ts])
        _native.check(rc, "cobalt_gbdt_set_data")

    def set_binary_labels(self, spw: float) -> bool:
        """After :meth:`set_data`: hold the 0/1 labels in the row records (byte 23 of a 32-byte record,
        F <= 23) and derive each row's weight from its label (``spw`` for positives, 1 otherwise), so
        the gradient pass reads neither array. The caller guarantees binary labels and no sample
        weights. False (nothing changed) when the record layout has no room."""
        rc = self.lib.cobalt_gbdt_set_binary_labels(self.h, ctypes.c_float(spw), _native.stream_handle())
        if rc == -13:
            return False
        _native.check(rc, "cobalt_gbdt_set_binary_labels")
        return True

    def plan(self) -> dict:
        """The last grow call's launch plan (csrc/gbdt.hip cobalt_gbdt_plan)."""
        fn = getattr(self.lib, "cobalt_gbdt_plan", None)
        if fn is None or not self.h:
            return {}
        out = (ctypes.c_int32 * 7)()
        fn(self.h, out)
        return {"ipc_fused": bool(out[0]), "own_level": int(out[1]), "wide_gradients": bool(out[2]),
                "fused_eval_resident_blocks": int(out[3]),
                "eval_part_levels": [lv for lv in range(16) if (out[4] >> lv) & 1],
                "eval_block_levels": [lv for lv in range(16) if (out[5] >> lv) & 1],
                "eval_block_overflow_levels": [lv for lv in range(16) if (out[6] >> lv) & 1]}

    def replica_error(self) -> int:
        """Data-parallel replica check (csrc/gbdt.hip GbdtDev::dig): 0 = healthy, 2 = this rank's trees
        diverged from its peers' (detected at level 0 of the tree after the divergent one)."""
        fn = getattr(self.lib, "cobalt_gbdt_error", None)  # absent from pre-check libraries (A/B runs)
        return int(fn(self.h)) if (self.h and fn is not None) else 0

    def set_fault(self, tree: int) -> None:
        """Fault injection (tests): perturb tree ``tree``'s root totals on this rank only."""
        _native.check(self.lib.cobalt_gbdt_set_fault(self.h, int(tree)), "cobalt_gbdt_set_fault")

    def set_start(self, t0: int) -> None:
        """Continue boosting at global tree index ``t0`` (margins already hold trees < t0)."""
        _native.check(self.lib.cobalt_gbdt_set_start(self.h, t0), "cobalt_gbdt_set_start")

    def grow(self, t0: int, n_trees: int) -> None:
        rc = self.lib.cobalt_gbdt_grow(self.h, t0, n_trees, _native.stream_handle())
        if rc != 0 and self.cfg.comm:
            raise RuntimeError(f"cobalt_gbdt_grow failed ({rc}): {self.lib.cobalt_comm_last_error().decode()}")
        _native.check(rc, "cobalt_gbdt_grow")

    # -------------------------------------------------------------- external-memory (sampled) mode
    def set_rows(self, n: int) -> None:
        """Rows of the current sample written into the bound records (<= the created capacity)."""
        _native.check(self.lib.cobalt_gbdt_set_rows(self.h, int(n)), "cobalt_gbdt_set_rows")

    def grow_sampled(self, t: int) -> None:
        """Grow tree ``t`` from the precomputed (reweighted) gradient pairs in the bound records."""
        _native.check(self.lib.cobalt_gbdt_grow_sampled(self.h, t, _native.stream_handle()), "cobalt_gbdt_grow_sampled")

    def tree_ptr(self, t: int) -> int:
        return int(self.lib.cobalt_gbdt_tree_ptr(self.h, t))

    def fetch(self, t0: int, n: int, stream: torch.cuda.Stream | None = None) -> np.ndarray:
        """Node records of trees [t0, t0 + n) (copied on ``stream``, default the current one, and
        synchronised with it only)."""
        out = np.zeros((n, self.max_nodes), dtype=NODE_DTYPE)
        rc = self.lib.cobalt_gbdt_fetch_trees(self.h, t0, n, out.ctypes.data, _native.stream_handle(stream))
        _native.check(rc, "cobalt_gbdt_fetch_trees")
        return out

    def close(self, park: bool = True) -> None:
        """Finish with the context: parked for the next fit of the same shapes when ``park`` (a fit
        that completed: its fetch synchronised the stream, so no kernel still uses the buffers), else
        destroyed."""
        h = getattr(self, "h", None)
        if not h:
            return
        self.h = None
        self._keep = []
        if park and _cache_on() and getattr(self, "_key", None) is not None:
            with _PARKED_LOCK:
                old = list(_PARKED.values())
                _PARKED.clear()
                _PARKED[self._key] = h.value
            for o in old:
                self.lib.cobalt_gbdt_destroy(ctypes.c_void_p(o))
            return
        self.lib.cobalt_gbdt_destroy(h)

    def __del__(self):
        try:
            self.close(park=False)
        except Exception:  # noqa: BLE001
            pass
