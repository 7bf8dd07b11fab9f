"""ctypes binding of the in-tree native library ``_lib/libcobalt_hip.so``.

The library holds the hand-written gfx950 HIP kernels and the C++ runtime (trainer driver, RCCL
communicator, predictor, TreeSHAP, preprocessing kernels). PyTorch-ROCm is imported first so that
the library resolves ``libamdhip64.so.7`` to the HIP runtime PyTorch already loaded.

On a machine with a GPU, every GPU op goes through this library; if it cannot be loaded the op
raises :class:`NativeUnavailable` (there is no silent eager fallback). Host (``device="cpu"``)
execution uses the reference implementations in the ``*_host`` modules instead.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen of the HIP library)

from . import build as _build
from .config import knob

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None
_err: str | None = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_double = ctypes.c_double
c_float = ctypes.c_float
c_char_p = ctypes.c_char_p


class NativeUnavailable(RuntimeError):
    pass


# name -> (restype, [argtypes])
_SIGS: dict[str, tuple] = {
    # gbdt.hip
    "cobalt_gbdt_create": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "cobalt_heap_to_trees": (ctypes.c_int64, [c_void_p, c_int, c_int] + [c_void_p] * 10),
    "cobalt_gbdt_set_data": (c_int, [c_void_p] * 9),
    "cobalt_gbdt_grow": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "cobalt_gbdt_fetch_trees": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "cobalt_gbdt_max_nodes": (c_int, [c_void_p]),
    "cobalt_gbdt_set_start": (c_int, [c_void_p, c_int]),
    "cobalt_gbdt_set_binary_labels": (c_int, [c_void_p, c_float, c_void_p]),
    "cobalt_gbdt_destroy": (c_int, [c_void_p]),
    "cobalt_gbdt_reuse": (c_int, [c_void_p, c_void_p]),
    "cobalt_gbdt_grow_sampled": (c_int, [c_void_p, c_int, c_void_p]),
    "cobalt_gbdt_set_rows": (c_int, [c_void_p, c_int64]),
    "cobalt_gbdt_error": (c_int, [c_void_p]),
    "cobalt_gbdt_ox_init": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "cobalt_gbdt_ox_begin": (c_int, [c_void_p, c_int, c_void_p]),
    "cobalt_gbdt_ox_page": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_int, c_int, c_void_p]),
    "cobalt_gbdt_ox_level": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "cobalt_gbdt_ox_end": (c_int, [c_void_p, c_int, c_void_p]),
    "cobalt_gbdt_set_fault": (c_int, [c_void_p, c_int]),
    "cobalt_gbdt_tree_ptr": (c_void_p, [c_void_p, c_int]),
    "cobalt_ooc_page": (c_int, [c_void_p, c_int, c_int64, c_int64, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                ctypes.c_uint64, c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "cobalt_ooc_bins": (c_int, []),
    "cobalt_gbdt_plan": (c_int, [c_void_p, c_void_p]),
    "cobalt_knob_count": (c_int, []),
    "cobalt_bin_matrix": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_int,
                                  c_void_p, c_void_p]),
    "cobalt_bin_matrix_ld": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_int,
                                     c_void_p, c_int64, c_void_p]),
    # comm.cpp
    "cobalt_comm_load": (c_int, [c_char_p]),
    "cobalt_comm_last_error": (c_char_p, []),
    "cobalt_comm_unique_id": (c_int, [c_void_p]),
    "cobalt_comm_init": (c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "cobalt_comm_destroy": (c_int, [c_void_p, c_int]),
    "cobalt_comm_async_error": (c_int, [c_void_p]),
    "cobalt_comm_allreduce": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "cobalt_comm_allgather": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    # ipccomm.hip
    "cobalt_ipc_handle_bytes": (c_int, []),
    "cobalt_ipc_create": (c_int, [c_int, c_int, c_int64, c_double, ctypes.POINTER(c_void_p), c_void_p]),
    "cobalt_ipc_connect": (c_int, [c_void_p, c_void_p]),
    "cobalt_ipc_epoch": (ctypes.c_uint, [c_void_p]),
    "cobalt_ipc_set_timeout": (ctypes.c_int, [c_void_p, ctypes.c_double]),
    "cobalt_ipc_dtab_selftest": (c_int, [c_void_p, ctypes.c_uint, c_void_p]),
    "cobalt_hw_ids": (c_int, [c_void_p, c_int, c_void_p]),
    # loopcomm.hip
    "cobalt_comm_loop_group": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "cobalt_comm_loop_rank": (c_int, [c_void_p, c_int, ctypes.POINTER(c_void_p)]),
    "cobalt_comm_loop_group_free": (c_int, [c_void_p]),
}


def _declare(lib: ctypes.CDLL) -> None:
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    # optional symbols registered by other modules (predict.hip, prep.hip, ...)
    for name, (res, args) in _EXTRA_SIGS.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args


_EXTRA_SIGS: dict[str, tuple] = {}


def register(name: str, restype, argtypes) -> None:
    """Declare the C signature of an exported symbol (called at import by ops modules)."""
    _EXTRA_SIGS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name, None)
        if fn is not None:
            fn.restype = restype
            fn.argtypes = argtypes


def load(build_if_needed: bool = True) -> ctypes.CDLL:
    """Load (building first when sources changed and hipcc exists) the native library."""
    global _lib, _err
    with _lock:
        if _lib is not None:
            return _lib
        override = knob("COBALT_NATIVE_LIB")  # e.g. the host-sanitizer build (build --sanitize)
        path = Path(override) if override else _build.lib_path()
        try:
            if not override and build_if_needed and _build.is_stale() and Path(_build.HIPCC).exists():
                _build.build()
            if not path.exists():
                raise NativeUnavailable(f"{path} missing; run `python -m cobalt_smart_lender_ai_amd.build`")
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        except NativeUnavailable as e:
            _err = str(e)
            raise
        except Exception as e:  # noqa: BLE001
            _err = f"{type(e).__name__}: {e}"
            raise NativeUnavailable(_err) from e
        _declare(lib)
        _lib = lib
        return lib


def lib() -> ctypes.CDLL:
    return load()


def available() -> bool:
    try:
        load()
        return True
    except NativeUnavailable:
        return False


def gpu_available() -> bool:
    return torch.cuda.is_available()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def stream_handle(stream: torch.cuda.Stream | None = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return int(t.data_ptr())


def loaded_path() -> str | None:
    return str(_build.lib_path()) if _lib is not None else None


def rccl_path() -> str:
    """Path of the RCCL library PyTorch links (``torch/lib/librccl.so``)."""
    p = Path(torch.__file__).parent / "lib" / "librccl.so"
    if p.exists():
        return str(p)
    return knob("COBALT_RCCL_LIB", "/opt/rocm/lib/librccl.so")
