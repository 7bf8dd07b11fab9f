"""Inference entry points: margins, probabilities and TreeSHAP for a :class:`Booster`.

GPU path: gfx950 kernels in ``csrc/predict.hip`` (forest packed once per booster and device, cached).
CPU path: the NumPy reference implementations in ``models/booster.py``.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from ..models.booster import Booster, Tree, predict_margin_host, sigmoid32, treeshap_host
from ..config import knob

# LDS tile capacity in nodes: a model's tile is max(this, its largest tree), at most MAX_TILE_NODES
# (csrc/predict.hip kMaxTileNodes). 2048 measured best on MI355X (125M-row scoring, 300 depth-7
# trees: 1024 -> 793M, 2048 -> 810M, 3072 -> 683M, 6144 -> 490M, 8192 -> 261M rows/s) -- smaller
# tiles mean more resident blocks per CU. COBALT_PRED_TILE overrides it for sweeps.
TILE_NODES = int(knob("COBALT_PRED_TILE", "2048"))
MAX_TILE_NODES = 8192
MAX_PATH = 15

_native.register("cobalt_predict", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p])
_native.register("cobalt_treeshap", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p])
_native.register("cobalt_treeshap_chunks", ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int])
_native.register("cobalt_predict_small_rows", ctypes.c_int64, [])
_native.register("cobalt_predict_small", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p])
_SMALL_ROWS = 131072
_native.register("cobalt_shap_table_build", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p])
_native.register("cobalt_treeshap_tab", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_void_p])
SHAP_ROWS_MIN = 256  # batches from this size use the row-parallel table kernel
SHAP_ROWS_MAX_F = 48
SHAP_TABLE_MAX_K = 10             # longest path (unique features) that gets a pattern table
SHAP_TABLE_MAX_BYTES = 2 << 30    # per-model table budget on the device

PATH_ELEM = np.dtype([("lo", "<f4"), ("hi", "<f4"), ("feat", "<i4"), ("nan_ok", "<i4"), ("zero", "<f8")])


def _bfs_order(t: Tree) -> list[int]:
    order, q = [], [0]
    while q:
        nxt = []
        for j in q:
            order.append(j)
            if t.left_children[j] != -1:
                nxt += [int(t.left_children[j]), int(t.right_children[j])]
        q = nxt
    return order


def tile_capacity(b: Booster, n_trees: int | None = None) -> int:
    """LDS tile capacity (nodes) for this forest: TILE_NODES, grown to fit the largest tree."""
    trees = b.trees[: (n_trees if n_trees is not None else b.num_trees)]
    biggest = max((len(t.left_children) for t in trees), default=0)
    cap = max(TILE_NODES, -(-biggest // 64) * 64)
    if cap > MAX_TILE_NODES:
        raise ValueError(f"tree with {biggest} nodes exceeds the LDS tile ({MAX_TILE_NODES} nodes)")
    return cap


def pack_forest(b: Booster, n_trees: int | None = None,
                tile_nodes: int | None = None) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(nodes uint32 [M, 2], tree_ptr int32 [T+1], tile_ptr int32 [n_tiles+1]); trees are grouped into
    tiles of at most ``tile_nodes`` (default ``tile_capacity``) nodes."""
    tile_nodes = tile_capacity(b, n_trees) if tile_nodes is None else tile_nodes
    trees = b.trees[: (n_trees if n_trees is not None else b.num_trees)]
    metas, vals, tree_ptr = [], [], [0]
    for t in trees:
        order = _bfs_order(t)
        if len(order) > 0xFFFE:
            raise ValueError("tree too large for the packed predictor")
        nid = {j: i for i, j in enumerate(order)}
        meta = np.zeros(len(order), dtype=np.uint32)
        val = np.zeros(len(order), dtype=np.float32)
        for j, i in nid.items():
            if t.left_children[j] == -1:
                meta[i] = 0xFFFF
            else:
                l, r = nid[int(t.left_children[j])], nid[int(t.right_children[j])]
                assert r == l + 1
                f = int(t.split_indices[j])
                if f > 0x7FFF:
                    raise ValueError("feature index too large for the packed predictor")
                meta[i] = (l & 0xFFFF) | (f << 16) | (int(t.default_left[j]) << 31)
            val[i] = t.split_conditions[j]
        metas.append(meta)
        vals.append(val)
        tree_ptr.append(tree_ptr[-1] + len(order))
    M = tree_ptr[-1]
    nodes = np.zeros((M, 2), dtype=np.uint32)
    if M:
        nodes[:, 0] = np.concatenate(metas)
        nodes[:, 1] = np.concatenate(vals).view(np.uint32)
    tiles = [0]
    acc = 0
    for i in range(len(trees)):
        sz = tree_ptr[i + 1] - tree_ptr[i]
        if sz > tile_nodes:
            raise ValueError("tree exceeds the LDS tile")
        if acc + sz > tile_nodes:
            tiles.append(i)
            acc = 0
        acc += sz
    tiles.append(len(trees))
    return nodes, np.asarray(tree_ptr, dtype=np.int32), np.asarray(tiles, dtype=np.int32)


def extract_paths(b: Booster) -> tuple[np.ndarray, np.ndarray, np.ndarray, int]:
    """Leaf paths with repeated features merged (elements, path_ptr, leaf values, max unique len)."""
    elems: list[tuple] = []
    ptr = [0]
    vals: list[float] = []
    max_len = 0
    for t in b.trees:
        cov = t.sum_hessian.astype(np.float64)
        stack = [(0, [])]
        while stack:
            j, path = stack.pop()
            if t.left_children[j] == -1:
                merged: dict[int, list] = {}
                order: list[int] = []
                for (parent, f, went_left, child) in path:
                    if f not in merged:
                        merged[f] = [-np.inf, np.inf, True, 1.0]
                        order.append(f)
                    m = merged[f]
                    thr = float(t.split_conditions[parent])
                    if went_left:
                        m[1] = min(m[1], thr)
                    else:
                        m[0] = max(m[0], thr)
                    m[2] = m[2] and (bool(t.default_left[parent]) == went_left)
                    m[3] *= cov[child] / cov[parent]
                for f in order:
                    lo, hi, nan_ok, z = merged[f]
                    elems.append((np.float32(lo), np.float32(hi), f, int(nan_ok), z))
                max_len = max(max_len, len(order))
                ptr.append(len(elems))
                vals.append(float(t.split_conditions[j]))
                continue
            f = int(t.split_indices[j])
            l, r = int(t.left_children[j]), int(t.right_children[j])
            stack.append((r, path + [(j, f, False, r)]))
            stack.append((l, path + [(j, f, True, l)]))
    arr = np.array(elems, dtype=PATH_ELEM) if elems else np.zeros(0, dtype=PATH_ELEM)
    return arr, np.asarray(ptr, dtype=np.int32), np.asarray(vals, dtype=np.float64), max_len


@dataclass
class _GpuForest:
    nodes: torch.Tensor
    tree_ptr: torch.Tensor
    tile_ptr: torch.Tensor
    n_tiles: int
    n_trees: int
    tile_cap: int
    elems: torch.Tensor | None = None
    path_ptr: torch.Tensor | None = None
    path_val: torch.Tensor | None = None
    n_paths: int = 0
    max_len: int = 0
    tab_ptr: torch.Tensor | None = None   # Fast-TreeSHAP pattern tables (None: direct kernel)
    table: torch.Tensor | None = None


def gpu_forest(b: Booster, device: torch.device, n_trees: int | None = None, with_shap: bool = False) -> _GpuForest:
    cache = b.__dict__.setdefault("_gpu_cache", {})
    key = (str(device), n_trees if n_trees is not None else b.num_trees)
    gf = cache.get(key)
    if gf is None:
        cap = tile_capacity(b, n_trees)
        nodes, tptr, tiles = pack_forest(b, n_trees, cap)
        gf = _GpuForest(torch.from_numpy(nodes).to(device), torch.from_numpy(tptr).to(device),
                        torch.from_numpy(tiles).to(device), len(tiles) - 1, len(tptr) - 1, cap)
        cache[key] = gf
    if with_shap and gf.elems is None:
        el, pp, pv, ml = extract_paths(b)
        if ml > MAX_PATH:
            raise ValueError(f"path with {ml} unique features exceeds the GPU TreeSHAP limit {MAX_PATH}")
        gf.elems = torch.from_numpy(el.view(np.uint8).copy()).to(device)
        gf.path_ptr = torch.from_numpy(pp).to(device)
        gf.path_val = torch.from_numpy(pv).to(device)
        gf.n_paths = len(pv)
        gf.max_len = ml
        k = np.diff(pp).astype(np.int64)
        sizes = (np.left_shift(1, k) * k) if len(k) else np.zeros(0, np.int64)
        if len(k) and ml <= SHAP_TABLE_MAX_K and int(sizes.sum()) * 8 <= SHAP_TABLE_MAX_BYTES:
            tp = np.zeros(len(k) + 1, dtype=np.int64)
            np.cumsum(sizes, out=tp[1:])
            gf.tab_ptr = torch.from_numpy(tp).to(device)
            gf.table = torch.empty(int(tp[-1]), dtype=torch.float64, device=device)
            rc = _native.lib().cobalt_shap_table_build(gf.elems.data_ptr(), gf.path_ptr.data_ptr(),
                                                       gf.path_val.data_ptr(), gf.n_paths, ml, gf.tab_ptr.data_ptr(),
                                                       gf.table.data_ptr(), _native.stream_handle())
            _native.check(rc, "cobalt_shap_table_build")
    return gf


def _device_of(X, device) -> torch.device:
    if device is not None:
        d = torch.device(device)
    elif isinstance(X, torch.Tensor):
        d = X.device
    else:
        d = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def _as_f32(X, device: torch.device) -> torch.Tensor:
    if isinstance(X, torch.Tensor):
        return X.to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(X, dtype=np.float32)), device=device)


def predict_gpu(b: Booster, X: torch.Tensor, n_trees: int | None = None, out_margin: torch.Tensor | None = None,
                out_prob: torch.Tensor | None = None) -> None:
    """Launch the predictor on the current stream (graph-capturable: no host sync; small batches use a
    scratch buffer from the caching allocator, which a graph capture takes from its private pool)."""
    gf = gpu_forest(b, X.device, n_trees)
    N, F = X.shape
    if F < b.num_feature:
        raise ValueError(f"X has {F} features, model needs {b.num_feature}")
    lib = _native.lib()
    om = out_margin.data_ptr() if out_margin is not None else None
    op = out_prob.data_ptr() if out_prob is not None else None
    if N < _SMALL_ROWS and N * gf.n_trees <= (1 << 24):
        # tile-parallel path (see csrc/predict.hip): grid = row blocks x tree tiles
        leaves = torch.empty(N * gf.n_trees, dtype=torch.float32, device=X.device)
        rc = lib.cobalt_predict_small(X.data_ptr(), N, F, X.stride(0), gf.nodes.data_ptr(), gf.tree_ptr.data_ptr(),
                                      gf.tile_ptr.data_ptr(), gf.n_tiles, gf.tile_cap, gf.n_trees, b.base_margin,
                                      leaves.data_ptr(), om, op, _native.stream_handle())
        _native.check(rc, "cobalt_predict_small")
        return
    rc = lib.cobalt_predict(X.data_ptr(), N, F, X.stride(0), gf.nodes.data_ptr(), gf.tree_ptr.data_ptr(),
                            gf.tile_ptr.data_ptr(), gf.n_tiles, gf.tile_cap, b.base_margin, om, op,
                            _native.stream_handle())
    _native.check(rc, "cobalt_predict")


_FORCE_DIRECT_SHAP = False  # tests compare the row-parallel table kernel against the direct kernel


def treeshap_gpu(b: Booster, X: torch.Tensor, phi: torch.Tensor) -> None:
    """Write TreeSHAP values into ``phi`` [N, F] float64 on the current stream (deterministic: no
    floating-point atomics; partial sums are combined in a fixed order)."""
    gf = gpu_forest(b, X.device, None, with_shap=True)
    N, F = X.shape
    lib = _native.lib()
    for s in range(0, N, 65535):
        e = min(N, s + 65535)
        nch = int(lib.cobalt_treeshap_chunks(e - s, F, gf.n_paths))
        work = torch.empty((e - s) * nch * F, dtype=torch.float64, device=X.device) if nch > 1 else None
        wp = work.data_ptr() if work is not None else None
        if gf.table is not None and not _FORCE_DIRECT_SHAP and e - s >= SHAP_ROWS_MIN and F <= SHAP_ROWS_MAX_F:
            rc = lib.cobalt_treeshap_tab(X[s:e].data_ptr(), e - s, F, X.stride(0), gf.elems.data_ptr(),
                                         gf.path_ptr.data_ptr(), gf.n_paths, gf.max_len, gf.tab_ptr.data_ptr(),
                                         gf.table.data_ptr(), phi[s:e].data_ptr(), wp, nch, _native.stream_handle())
            _native.check(rc, "cobalt_treeshap_tab")
        else:
            rc = lib.cobalt_treeshap(X[s:e].data_ptr(), e - s, F, X.stride(0), gf.elems.data_ptr(),
                                     gf.path_ptr.data_ptr(), gf.path_val.data_ptr(), gf.n_paths, gf.max_len,
                                     phi[s:e].data_ptr(), wp, nch, _native.stream_handle())
            _native.check(rc, "cobalt_treeshap")


def predict_margin(b: Booster, X, device=None, n_trees: int | None = None):
    d = _device_of(X, device)
    if d.type == "cuda":
        Xt = _as_f32(X, d)
        out = torch.empty(Xt.shape[0], dtype=torch.float32, device=d)
        predict_gpu(b, Xt, n_trees, out_margin=out)
        return out if isinstance(X, torch.Tensor) else out.cpu().numpy()
    Xn = X.cpu().numpy() if isinstance(X, torch.Tensor) else np.asarray(X, dtype=np.float32)
    return predict_margin_host(b, Xn, n_trees)


def predict_proba(b: Booster, X, device=None):
    d = _device_of(X, device)
    if d.type == "cuda":
        Xt = _as_f32(X, d)
        out = torch.empty(Xt.shape[0], dtype=torch.float32, device=d)
        predict_gpu(b, Xt, None, out_prob=out)
        return out if isinstance(X, torch.Tensor) else out.cpu().numpy()
    return sigmoid32(predict_margin(b, X, "cpu"))


def shap_values(b: Booster, X, device=None):
    d = _device_of(X, device)
    if d.type == "cuda":
        Xt = _as_f32(X, d)
        phi = torch.zeros((Xt.shape[0], Xt.shape[1]), dtype=torch.float64, device=d)
        treeshap_gpu(b, Xt, phi)
        return phi if isinstance(X, torch.Tensor) else phi.cpu().numpy()
    Xn = X.cpu().numpy() if isinstance(X, torch.Tensor) else np.asarray(X, dtype=np.float32)
    return treeshap_host(b, Xn)
