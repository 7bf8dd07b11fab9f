"""Column-store preprocessing ops (K1-K9, K11, K30) with a gfx950 path and a NumPy host path.

A numeric frame is a column-major float64 tensor ``[C, N]``. On CUDA tensors every op launches the
kernels in ``csrc/prep.hip``; on CPU tensors the same semantics run in NumPy (the test oracle).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native

_V, _I, _I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_native.register("cobalt_col_null_counts", _I, [_V, _I64, _I, _V, _V])
_native.register("cobalt_row_null_counts", _I, [_V, _I64, _I, _V, _V, _V])
_native.register("cobalt_masked_log1p", _I, [_V, _I64, _V, _I, _V])
_native.register("cobalt_fill_indicator", _I, [_V, _I64, _V, _V, _I, _V, _V])
_native.register("cobalt_row_hash", _I, [_V, _I64, _I, _V, _V])
_native.register("cobalt_rows_equal", _I, [_V, _I64, _I, _V, _V, _I64, _V, _V])
_native.register("cobalt_onehot", _I, [_V, _I64, _I, _I, _V, _V])
_native.register("cobalt_col_moments", _I, [_V, _I64, _I, _V, _V])
_native.register("cobalt_minmax_apply", _I, [_V, _I64, _I, _V, _V, _V, _V])
_native.register("cobalt_str_hash", _I, [_V, _V, _V, _I64, _V, _V])


def _cuda(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def _lib():
    return _native.lib()


def _s() -> int:
    return _native.stream_handle()


def col_null_counts(X: torch.Tensor) -> torch.Tensor:
    """[C, N] float64 -> int64 [C] NaN counts."""
    C, N = X.shape
    if _cuda(X):
        out = torch.empty(C, dtype=torch.int64, device=X.device)
        _native.check(_lib().cobalt_col_null_counts(X.data_ptr(), N, C, out.data_ptr(), _s()), "col_null_counts")
        return out
    return torch.from_numpy(np.isnan(X.numpy()).sum(1).astype(np.int64))


def row_null_counts(X: torch.Tensor, colmask: torch.Tensor | None = None) -> torch.Tensor:
    C, N = X.shape
    if _cuda(X):
        out = torch.empty(N, dtype=torch.int32, device=X.device)
        cm = colmask.to(device=X.device, dtype=torch.uint8).contiguous() if colmask is not None else None
        _native.check(_lib().cobalt_row_null_counts(X.data_ptr(), N, C, cm.data_ptr() if cm is not None else None,
                                                    out.data_ptr(), _s()), "row_null_counts")
        return out
    a = np.isnan(X.numpy())
    if colmask is not None:
        a = a[colmask.cpu().numpy().astype(bool)]
    return torch.from_numpy(a.sum(0).astype(np.int32))


def masked_log1p_(X: torch.Tensor, cols: list[int]) -> None:
    """In place: x -> log1p(x) where x > 0 on the listed columns."""
    if not cols:
        return
    if _cuda(X):
        ct = torch.tensor(cols, dtype=torch.int32, device=X.device)
        _native.check(_lib().cobalt_masked_log1p(X.data_ptr(), X.shape[1], ct.data_ptr(), len(cols), _s()),
                      "masked_log1p")
        return
    a = X.numpy()
    for c in cols:
        v = a[c]
        pos = v > 0
        v[pos] = np.log1p(v[pos])


def fill_with_indicator_(X: torch.Tensor, cols: list[int], values: list[float], indicator: bool = True):
    """In place NaN fill of ``cols`` with ``values``; returns int8 [len(cols), N] missing indicators."""
    N = X.shape[1]
    if not cols:
        return None
    if _cuda(X):
        ct = torch.tensor(cols, dtype=torch.int32, device=X.device)
        vt = torch.tensor(values, dtype=torch.float64, device=X.device)
        ind = torch.empty((len(cols), N), dtype=torch.int8, device=X.device) if indicator else None
        _native.check(_lib().cobalt_fill_indicator(X.data_ptr(), N, ct.data_ptr(), vt.data_ptr(), len(cols),
                                                   ind.data_ptr() if ind is not None else None, _s()),
                      "fill_indicator")
        return ind
    a = X.numpy()
    ind = np.zeros((len(cols), N), dtype=np.int8) if indicator else None
    for j, (c, v) in enumerate(zip(cols, values)):
        m = np.isnan(a[c])
        if ind is not None:
            ind[j] = m
        a[c][m] = v
    return torch.from_numpy(ind) if ind is not None else None


def row_hash(X: torch.Tensor) -> torch.Tensor:
    C, N = X.shape
    if _cuda(X):
        out = torch.empty(N, dtype=torch.int64, device=X.device)
        _native.check(_lib().cobalt_row_hash(X.data_ptr(), N, C, out.data_ptr(), _s()), "row_hash")
        return out
    a = np.ascontiguousarray(X.numpy().T)
    a = np.where(np.isnan(a), np.nan, a) + 0.0  # canonical NaN, -0.0 -> 0.0
    v = a.view(np.uint64) if a.size else np.zeros((N, 0), np.uint64)
    h = np.full(N, 0x243F6A8885A308D3, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for c in range(C):
            x = h ^ (v[:, c] + np.uint64(0x9E3779B97F4A7C15) * np.uint64(c + 1))
            x = x + np.uint64(0x9E3779B97F4A7C15)
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            h = x ^ (x >> np.uint64(31))
    return torch.from_numpy(h.view(np.int64))


def rows_equal(X: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    C, N = X.shape
    m = a.numel()
    if _cuda(X):
        eq = torch.empty(m, dtype=torch.uint8, device=X.device)
        _native.check(_lib().cobalt_rows_equal(X.data_ptr(), N, C, a.contiguous().data_ptr(), b.contiguous().data_ptr(),
                                               m, eq.data_ptr(), _s()), "rows_equal")
        return eq.bool()
    xa, xb = X.numpy()[:, a.numpy()], X.numpy()[:, b.numpy()]
    return torch.from_numpy(((xa == xb) | (np.isnan(xa) & np.isnan(xb))).all(0))


def duplicated_numeric(X: torch.Tensor, extra_hash: torch.Tensor | None = None) -> torch.Tensor:
    """``DataFrame.duplicated(keep='first')`` over the numeric block (optionally combined with a hash of
    the non-numeric columns, whose equality the caller verifies). Returns (dup mask, candidate pairs)."""
    N = X.shape[1]
    h = row_hash(X)
    if extra_hash is not None:
        h = h ^ (extra_hash.to(h.device) * 0x9E3779B1)
    order = torch.sort(h, stable=True).indices
    hs = h[order]
    same = torch.zeros(N, dtype=torch.bool, device=h.device)
    if N > 1:
        same[1:] = hs[1:] == hs[:-1]
    # candidate pair: each row vs the first row of its hash run
    run_start = torch.arange(N, device=h.device)
    run_start[same] = 0
    run_start = torch.cummax(run_start, 0).values
    cand = same.nonzero(as_tuple=True)[0]
    a = order[run_start[cand]]
    b = order[cand]
    eq = rows_equal(X, a, b) if cand.numel() else torch.zeros(0, dtype=torch.bool, device=h.device)
    dup = torch.zeros(N, dtype=torch.bool, device=h.device)
    dup[b[eq]] = True
    return dup, (a[eq], b[eq])


def onehot(codes: torch.Tensor, levels: int, drop_first: bool = True) -> torch.Tensor:
    n = codes.numel()
    w = levels - (1 if drop_first else 0)
    if _cuda(codes):
        out = torch.empty((n, max(w, 0)), dtype=torch.uint8, device=codes.device)
        if w > 0:
            _native.check(_lib().cobalt_onehot(codes.to(torch.int32).contiguous().data_ptr(), n, levels,
                                               int(drop_first), out.data_ptr(), _s()), "onehot")
        return out
    c = codes.numpy().astype(np.int64) - (1 if drop_first else 0)
    out = np.zeros((n, max(w, 0)), dtype=np.uint8)
    ok = (c >= 0) & (c < w)
    out[np.nonzero(ok)[0], c[ok]] = 1
    return torch.from_numpy(out)


def col_moments(X: torch.Tensor) -> torch.Tensor:
    """[C, 5] = (count, sum, sumsq, min, max) over non-NaN values."""
    C, N = X.shape
    if _cuda(X):
        out = torch.zeros((C, 5), dtype=torch.float64, device=X.device)
        out[:, 3] = float("inf")
        out[:, 4] = float("-inf")
        _native.check(_lib().cobalt_col_moments(X.data_ptr(), N, C, out.data_ptr(), _s()), "col_moments")
        return out
    a = X.numpy()
    m = ~np.isnan(a)
    cnt = m.sum(1)
    s = np.where(m, a, 0).sum(1)
    s2 = np.where(m, a * a, 0).sum(1)
    mn = np.where(cnt > 0, np.nanmin(np.where(m, a, np.inf), 1), np.inf)
    mx = np.where(cnt > 0, np.nanmax(np.where(m, a, -np.inf), 1), -np.inf)
    return torch.from_numpy(np.stack([cnt.astype(np.float64), s, s2, mn, mx], 1))


def median(X: torch.Tensor) -> torch.Tensor:
    """Exact per-column median of non-NaN values (pandas ``Series.median``: mean of the two middle
    values for even counts, NaN for empty columns). Sort on device (rocPRIM)."""
    C, N = X.shape
    xs = torch.sort(X, dim=1).values  # NaN last
    cnt = (~torch.isnan(X)).sum(1)
    lo = torch.clamp((cnt - 1) // 2, min=0)
    hi = torch.clamp(cnt // 2, min=0)
    idx_lo = lo.clamp(max=max(N - 1, 0)).unsqueeze(1)
    idx_hi = hi.clamp(max=max(N - 1, 0)).unsqueeze(1)
    if N == 0:
        return torch.full((C,), float("nan"), dtype=torch.float64, device=X.device)
    v = (xs.gather(1, idx_lo).squeeze(1) + xs.gather(1, idx_hi).squeeze(1)) / 2.0
    return torch.where(cnt > 0, v, torch.full_like(v, float("nan")))


def minmax_scale(X: torch.Tensor, mn: torch.Tensor, mx: torch.Tensor) -> torch.Tensor:
    """[C, N] -> row-major float32 [N, C] scaled to [0, 1] with the given per-column min/max."""
    C, N = X.shape
    if _cuda(X):
        out = torch.empty((N, C), dtype=torch.float32, device=X.device)
        _native.check(_lib().cobalt_minmax_apply(X.data_ptr(), N, C, mn.contiguous().data_ptr(),
                                                 mx.contiguous().data_ptr(), out.data_ptr(), _s()), "minmax")
        return out
    rng = (mx - mn).numpy()
    sc = np.where(rng > 0, 1.0 / np.where(rng > 0, rng, 1.0), 0.0)
    return torch.from_numpy(((X.numpy() - mn.numpy()[:, None]) * sc[:, None]).T.astype(np.float32))


_MASK64 = (1 << 64) - 1


def _splitmix_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def _string_hash_host(data: np.ndarray, off: np.ndarray, valid: np.ndarray | None) -> np.ndarray:
    """NumPy twin of k_str_hash (vectorised over strings, looping over 8-byte word positions)."""
    n = len(off) - 1
    b, e = off[:-1].astype(np.int64), off[1:].astype(np.int64)
    ln = e - b
    h = np.uint64(0x9E3779B97F4A7C15) ^ ln.astype(np.uint64)
    nw = (ln + 7) // 8
    dpad = np.concatenate([data, np.zeros(8, np.uint8)])
    for k in range(int(nw.max()) if n else 0):
        act = nw > k
        w = np.zeros(n, dtype=np.uint64)
        for j in range(8):
            p = b + 8 * k + j
            ok = act & (p < e)
            w |= np.where(ok, dpad[np.where(ok, p, len(data))], 0).astype(np.uint64) << np.uint64(8 * j)
        h = np.where(act, _splitmix_np(h ^ w), h)
    h = np.where(h == 0, np.uint64(1), h)
    if valid is not None:
        h = np.where(valid, h, np.uint64(0))
    return h.view(np.int64)


def string_hash(col, device) -> torch.Tensor:
    """int64 [N] hashes of an Arrow string (Chunked)Array; 0 = missing. GPU: k_str_hash per chunk."""
    import pyarrow as pa

    dev = torch.device(device)
    chunks = col.chunks if hasattr(col, "chunks") else [col]
    outs = []
    for ch in chunks:
        n = len(ch)
        if n == 0:
            continue
        large = pa.types.is_large_string(ch.type)
        bufs = ch.buffers()
        ity = np.int64 if large else np.int32
        off = np.frombuffer(bufs[1], dtype=ity, count=n + 1, offset=ch.offset * np.dtype(ity).itemsize).astype(np.int64)
        base = int(off[0])
        data = np.frombuffer(bufs[2], dtype=np.uint8)[base:int(off[-1])] if bufs[2] is not None else np.zeros(0, np.uint8)
        off = off - base
        valid = ch.is_valid().to_numpy(zero_copy_only=False) if ch.null_count else None
        if dev.type == "cuda":
            d = torch.from_numpy(np.ascontiguousarray(data)).to(dev) if len(data) else torch.zeros(1, dtype=torch.uint8,
                                                                                             device=dev)
            o = torch.from_numpy(off).to(dev)
            v = torch.from_numpy(valid.astype(np.uint8)).to(dev) if valid is not None else None
            out = torch.empty(n, dtype=torch.int64, device=dev)
            _native.check(_lib().cobalt_str_hash(d.data_ptr(), o.data_ptr(), v.data_ptr() if v is not None else None,
                                                 n, out.data_ptr(), _s()), "str_hash")
            outs.append(out)
        else:
            outs.append(torch.from_numpy(_string_hash_host(data, off, valid)))
    return torch.cat(outs) if outs else torch.zeros(0, dtype=torch.int64, device=dev)
