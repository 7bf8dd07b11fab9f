"""External-memory ("out-of-core") GBDT training: quantised pages in host DRAM, a per-tree sample
on the device (BASELINE.json config "100M-row out-of-core GBDT with host-DRAM
spill (288 GB HBM per-GPU sizing)").

The in-core trainer keeps ~72 B per row on the GPU (32-byte row record, feature-major bins, margin,
label, weight, two row-index buffers), i.e. ~4 G rows per 288 GB MI355X. Beyond that -- or under a
device-memory budget -- this path keeps only the margins, labels and weights on the device (12 B per
row) and spills the rows' bins to pinned host pages in a compact format (the F bins rounded up to 4
bytes: 20 B per row for the deployed features instead of the 32-byte record, since the per-tree page
stream is bound by the H2D copy):

1. ``stream_cuts`` -- the in-core quantile sketch over the stream (the cuts of an in-core fit with the same ``sketch_rows``; by default every row for exact streaming on a GPU, a 2^18-row sample for the sampled mode);
2. every chunk is binned on the GPU and its row records are copied to a pinned host page;
3. per tree, every page streams back through ``k_ooc_page`` (double-buffered H2D on a copy stream):
   the previous tree is applied to the margins, g/h are computed, and a minimal-variance sample
   (MVS, the sampler XGBoost uses for GPU external memory: keep row i with p_i = min(1, ghat_i/mu),
   ghat = sqrt(g^2 + h^2), gradients reweighted by 1/p_i) is compacted into the trainer's records;
4. the in-core kernels grow the tree on the sample (``cobalt_gbdt_grow_sampled``).

mu for tree t comes from the exact integer ghat histogram (2048 log-spaced bins) of the previous
pass, solved on the host so that the expected sample is ``sample_rate * N`` rows (capped at
``w_max`` so the fixed-point gradient scales hold). The sample order on the GPU depends on atomic
claims, but every histogram sum is an exact integer, so the GPU path grows exactly the trees of the
host path below (tested) -- which, with ``device="cpu"``, is the oracle and the CPU fallback.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import gbdt_host, sketch
from .booster import NODE_DTYPE, Booster, trees_from_heap_nodes
from . import gbdt
from .gbdt import GBDTParams, _resolve_device, feature_masks
from .stream import ChunkSource, _as_np, _PinnedUploader, stream_cuts

OOC_BINS = 2048
_MASK64 = (1 << 64) - 1


def ooc_key(seed: int, tree: int) -> int:
    """Per-tree key of the MVS keep decision (mirrors ``key`` passed to ``k_ooc_page``)."""
    return gbdt_host.splitmix64_int((seed ^ ((0x5851F42D4C957F2D + tree * 0x632BE59BD9B4E019) & _MASK64)) & _MASK64)


def page_stride(n_feat: int) -> int:
    """Bytes per row of a spilled page: the bins, rounded up to whole 32-bit words."""
    return (n_feat + 3) // 4 * 4


def ghat_bin(v: np.ndarray) -> np.ndarray:
    """Host mirror of ``ooc_bin``: binary exponent x 16 mantissa steps (exact integer arithmetic)."""
    v = np.asarray(v, dtype=np.float64)
    f, e = np.frexp(v)
    b = (e.astype(np.int64) + 64) * 16 + np.floor((f - 0.5) * 32.0).astype(np.int64)
    b = np.clip(b, 1, OOC_BINS - 1)
    return np.where(v > 0, b, 0)


def _bin_values() -> np.ndarray:
    b = np.arange(OOC_BINS)
    e, k = b // 16 - 64, b % 16
    v = 0.5 * (np.ldexp(0.5 + k / 32.0, e) + np.ldexp(0.5 + (k + 1) / 32.0, e))
    v[0] = 0.0
    return v


def mvs_threshold(counts: np.ndarray, target: float, mu_max: float) -> float:
    """mu such that the expected MVS sample sum_i min(1, ghat_i / mu) is ``target`` rows, from the
    binned ghat counts (bisection in log space: a deterministic function of the integer counts),
    capped at ``mu_max``."""
    c = np.asarray(counts, dtype=np.float64)
    v = _bin_values()
    live = (c > 0) & (v > 0)
    if not live.any():
        return float(mu_max)
    if target >= c[live].sum():
        return float(min(v[live].min() * 0.5, mu_max))  # keep everything
    cv, vv = c[live], v[live]
    lo, hi = math.log(vv.min()) - 1.0, math.log(vv.max()) + math.log(cv.sum() / max(target, 1.0)) + 1.0
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if float((cv * np.minimum(1.0, vv / math.exp(mid))).sum()) > target:
            lo = mid
        else:
            hi = mid
    return float(min(math.exp(0.5 * (lo + hi)), mu_max))


def apply_nodes_bins(nodes: np.ndarray, bins: np.ndarray) -> np.ndarray:
    """Leaf value of every row (uint8 bins [n, F]) in one heap-ordered tree (``NODE_DTYPE``)."""
    n = len(bins)
    idx = np.zeros(n, dtype=np.int64)
    rows = np.arange(n)
    while True:
        split = nodes["status"][idx] == 2
        if not split.any():
            break
        f = np.where(split, nodes["feat"][idx], 0)
        b = bins[rows, f].astype(np.int64)
        left = np.where(b == 255, nodes["default_left"][idx] == 1, b <= nodes["bin"][idx])
        idx = np.where(split, 2 * idx + np.where(left, 1, 2), idx)
    return nodes["leaf_value"][idx].astype(np.float32)


@dataclass
class ExternalReport:
    n_rows: int = 0
    n_pages: int = 0
    host_bytes: int = 0
    device_page_bytes: int = 0
    t_sketch: float = 0.0
    t_pages: float = 0.0
    t_boost: float = 0.0
    sample_rows: list = field(default_factory=list)
    mu: list = field(default_factory=list)
    # "in-core": an exact fit whose pages all fit the HBM budget ran the in-core trainer; "paged": the
    # page passes (host-DRAM or partly HBM-resident pages)
    mode: str = "paged"


def train_external(source: ChunkSource, params: GBDTParams | dict | None = None, *, n_rows: int | None = None,
                   device=None, sample_rate: float = 0.2, device_page_bytes: int = 0, feature_names=None,
                   feature_types=None, report: ExternalReport | None = None) -> Booster:
    """Train on a chunk stream with host-resident pages (one page per chunk) and a per-tree MVS sample
    of about ``sample_rate * n_rows`` rows on the device. Pages up to ``device_page_bytes`` in total
    stay in HBM (no PCIe traffic per tree); the rest are spilled to pinned host memory."""
    if params is None:
        params = GBDTParams()
    elif isinstance(params, dict):
        params = GBDTParams.from_kwargs(**params)
    if not 0.0 < sample_rate <= 1.0:
        raise ValueError("sample_rate must be in (0, 1]")
    if int(params.grad_bits) != 17:
        # the page passes (cobalt_gbdt_ox_init / the sampled grow) keep the packed 17-bit (g, h) cells
        raise ValueError(f"out-of-core training supports grad_bits=17 only (got {params.grad_bits})")
    exact = sample_rate >= 1.0  # every row every tree: level-wise page streaming (no sample)
    dev = _resolve_device(device, None)
    if exact and dev.type == "cuda":
        # the exact pass keeps a row's node in 2^(depth + 1) - 1 <= 255 staged node slots and the feature
        # table in LDS (csrc/gbdt.hip cobalt_gbdt_ox_init): refuse before the sketch / page passes
        n_feat = None
        if int(params.max_depth) <= 7:  # the feature count from the stream's first chunk (one chunk read)
            it = iter(source())
            try:
                first = next(it, None)
            finally:  # release the half-read stream (an open file, a generator) now, not at GC
                getattr(it, "close", lambda: None)()
            n_feat = None if first is None else int(first[0].shape[1])
        if int(params.max_depth) > 7 or (n_feat is not None and n_feat > 32):
            raise ValueError(f"exact out-of-core training (sample_rate=1) supports max_depth <= 7 and <= 32 "
                             f"features (got max_depth={params.max_depth}, features={n_feat}); use sample_rate < 1")
    rep = report if report is not None else ExternalReport()
    t0 = time.perf_counter()
    if (exact and dev.type == "cuda" and n_rows is not None and n_feat is not None
            and device_page_bytes >= page_stride(n_feat) * int(n_rows) and _in_core_fits(int(n_rows), n_feat, dev, raw=True)):
        # every page would sit in HBM and so does the raw matrix: ONE pass over the stream into a device
        # matrix and the in-core fit (device sketch + binning + trees: the cuts of the streamed sketch and
        # the trees of the exact page passes, byte for byte) -- no further passes over the source
        return _train_in_core_raw(source, params, int(n_rows), n_feat, dev, feature_names, feature_types, rep)
    # the sketch: exact streaming (every row) sketches every row by default, like the in-core fit on a
    # GPU; the sampled mode keeps the 2^18-row strided sample (one pass over the stream instead of
    # three -- with a regenerated or re-read source the extra passes cost seconds at 100M rows)
    sk = params.sketch_rows
    if sk is not None and sk < 0 and not exact:
        sk = 1 << 18
    cuts, nbins, N, _, F = stream_cuts(source, n_rows=n_rows, max_bin=params.max_bin, sketch_rows=sk, device=dev)
    if F > 24:
        raise ValueError("external-memory training packs a row into one 32-byte record (<= 24 features)")
    rep.t_sketch = time.perf_counter() - t0
    rep.n_rows = N

    if exact and dev.type == "cuda" and device_page_bytes >= page_stride(F) * N and _in_core_fits(N, F, dev):
        # every page would sit in HBM: bin the stream straight into the in-core trainer's layout and grow
        # with the in-core kernels (the exact page passes grow the same trees byte for byte, but re-read
        # every page per level: 19.9 s vs 1.9 s at 100M rows)
        return _train_in_core(source, params, N, F, dev, cuts, nbins, feature_names, feature_types, rep)

    # pages: quantised row records on the host, labels on the training device
    t0 = time.perf_counter()
    pages: list[tuple[int, object]] = []
    y = torch.empty(N, dtype=torch.float32, device=dev)
    r0 = 0
    if dev.type == "cuda":
        from ..ops import gbdt_ops

        up = _PinnedUploader(dev)
        resident = 0
        ps = page_stride(F)
        for Xc, yc in source():
            Xc = _as_np(Xc, np.float32)
            rec, _ = gbdt_ops.bin_matrix(up.put(Xc), cuts, nbins)
            rec = rec[:, :ps]  # bins only: k_ooc_page rebuilds the 32-byte record of a sampled row
            if resident + rec.numel() <= device_page_bytes:  # within the HBM budget: keep it there
                resident += rec.numel()
                pages.append((r0, rec.contiguous()))
            else:
                page = torch.empty(rec.shape, dtype=torch.uint8, pin_memory=True)
                page.copy_(rec)
                pages.append((r0, page))
            y[r0:r0 + len(Xc)] = torch.from_numpy(_as_np(yc, np.float32)).to(dev)
            r0 += len(Xc)
        torch.cuda.synchronize(dev)
    else:
        c_np, nb_np = cuts.cpu().numpy(), nbins.cpu().numpy()
        for Xc, yc in source():
            Xc = _as_np(Xc, np.float32)
            pages.append((r0, sketch.bin_matrix_host(Xc, c_np, nb_np)))
            y[r0:r0 + len(Xc)] = torch.from_numpy(_as_np(yc, np.float32))
            r0 += len(Xc)
    rep.n_pages = len(pages)
    rep.host_bytes = int(sum(p.numel() if isinstance(p, torch.Tensor) else p.nbytes for _, p in pages
                             if not (isinstance(p, torch.Tensor) and p.is_cuda)))
    rep.device_page_bytes = int(sum(p.numel() for _, p in pages if isinstance(p, torch.Tensor) and p.is_cuda))
    rep.t_pages = time.perf_counter() - t0

    spw = float(params.scale_pos_weight if params.scale_pos_weight is not None else 1.0)
    w = torch.where(y == 1.0, torch.tensor(spw, device=dev), torch.tensor(1.0, device=dev)).to(torch.float32)
    if params.base_score is None:
        sw, swy = float(w.double().sum()), float((w.double() * y.double()).sum())
        base_score = min(max(swy / sw if sw > 0 else 0.5, 1e-6), 1 - 1e-6)
    else:
        base_score = float(params.base_score)
    base_score = float(np.float32(base_score))
    base_margin = Booster([], base_score=base_score, num_feature=F).base_margin
    wmax = float(w.max()) if N else 1.0
    # |g / p| and h / p are both <= max(|g|, h, mu) <= w_max once mu is capped at w_max
    gscale = hscale = float(2 ** 16) / wmax  # the page kernel clips at +-2^16 (k_ooc_page)
    T, D = int(params.n_estimators), int(params.max_depth)
    seed = int(params.random_state)
    fmask = feature_masks(T, F, float(params.colsample_bytree), seed)
    hp = gbdt_host.HostGbdtParams(max_depth=D, eta=float(params.learning_rate), reg_lambda=float(params.reg_lambda),
                                  reg_alpha=float(params.reg_alpha), gamma=float(params.gamma),
                                  min_child_weight=float(params.min_child_weight), subsample=1.0, seed=seed,
                                  gscale=gscale, hscale=hscale)
    target = sample_rate * N
    cap = int(min(N, math.ceil(target * 1.25) + 4096))

    if exact:
        t0 = time.perf_counter()
        nodes = _train_exact(pages, y, w, base_margin, F, dev, cuts, nbins, params, T, fmask, wmax)
        rep.t_boost = time.perf_counter() - t0
        rep.sample_rows = [N] * T
        names = list(feature_names) if feature_names is not None else None
        return Booster(trees=trees_from_heap_nodes(nodes, D), feature_names=names,
                       feature_types=list(feature_types) if feature_types is not None else None,
                       base_score=base_score, num_feature=F,
                       train_params=dict(eta=float(params.learning_rate), gamma=float(params.gamma), max_depth=D,
                                         min_child_weight=float(params.min_child_weight),
                                         reg_lambda=float(params.reg_lambda), reg_alpha=float(params.reg_alpha),
                                         subsample=float(params.subsample),
                                         colsample_bytree=float(params.colsample_bytree),
                                         max_bin=int(params.max_bin), scale_pos_weight=spw, seed=seed))

    t0 = time.perf_counter()
    runner = (_GpuPasses if dev.type == "cuda" else _HostPasses)(pages, y, w, base_margin, F, cap, gscale, hscale,
                                                                 dev, cuts, nbins, hp, T, fmask)
    try:
        _, counts = runner.page_pass(-1, 0.0, 0)  # statistics only: ghat of the initial margins
        for t in range(T):
            mu = mvs_threshold(counts, target, wmax)
            ns, counts = runner.page_pass(t - 1, mu, t)
            while ns > cap:  # rare: the sample outgrew its buffer -> a sparser sample of the same margins
                mu = mu * ns / cap * 1.1
                ns, _ = runner.page_pass(-1, mu, t)
            rep.sample_rows.append(int(ns))
            rep.mu.append(float(mu))
            runner.grow(t, ns)
        nodes = runner.fetch()
    finally:
        runner.close()
    rep.t_boost = time.perf_counter() - t0
    names = list(feature_names) if feature_names is not None else None
    return Booster(trees=trees_from_heap_nodes(nodes, D), feature_names=names,
                   feature_types=list(feature_types) if feature_types is not None else None,
                   base_score=base_score, num_feature=F,
                   train_params=dict(eta=hp.eta, gamma=hp.gamma, max_depth=D, min_child_weight=hp.min_child_weight,
                                     reg_lambda=hp.reg_lambda, reg_alpha=hp.reg_alpha, subsample=1.0,
                                     colsample_bytree=float(params.colsample_bytree), max_bin=int(params.max_bin),
                                     scale_pos_weight=spw, seed=seed, sampling_method="gradient_based",
                                     external_sample_rate=float(sample_rate)))


def _in_core_fits(N: int, F: int, dev: torch.device, raw: bool = False) -> bool:
    """The in-core trainer's ~72 B per row (32-byte records, feature-major bins, margins, labels,
    weights, two row-index buffers; models/gbdt.py) -- plus, with ``raw``, the float32 matrix and the
    sketch's transposed copy and bucket ids -- fit the device's free memory with headroom, and the rows
    fit its int32 row ids."""
    from ..ops import gbdt_ops

    if N >= (1 << 31) - 1:
        return False
    free, _ = torch.cuda.mem_get_info(dev)
    need = N * (gbdt_ops.row_stride(F) + F + 4 * 6 + (F * 10 if raw else 0)) + (256 << 20)
    return need <= 0.9 * free


def _train_in_core_raw(source, params: GBDTParams, N: int, F: int, dev: torch.device, feature_names, feature_types,
                       rep: ExternalReport) -> Booster:
    """Exact external-memory fit whose raw matrix fits the device: the stream is read once into a device
    [N, F] float32 matrix and the in-core trainer fits it (``gbdt.train``)."""
    from .gbdt import train

    t0 = time.perf_counter()
    up = _PinnedUploader(dev)
    X = torch.empty((N, F), dtype=torch.float32, device=dev)
    y = torch.empty(N, dtype=torch.float32, device=dev)
    r0 = 0
    for Xc, yc in source():
        Xc = _as_np(Xc, np.float32)
        if r0 + len(Xc) > N or Xc.shape[1] != F:
            raise ValueError(f"the stream yields more than n_rows={N} rows or not {F} features")
        X[r0:r0 + len(Xc)] = up.put(Xc)
        y[r0:r0 + len(Xc)] = torch.from_numpy(_as_np(yc, np.float32)).to(dev)
        r0 += len(Xc)
    if r0 != N:
        raise ValueError(f"the stream yielded {r0} rows, n_rows={N}")
    torch.cuda.synchronize(dev)
    rep.n_rows = N
    rep.n_pages = 0
    rep.host_bytes = 0
    rep.device_page_bytes = int(X.numel() * 4)
    rep.t_pages = time.perf_counter() - t0
    rep.mode = "in-core"
    t0 = time.perf_counter()
    fr = gbdt.FitReport()
    bst = train(X, y, params, device=dev, feature_names=feature_names, feature_types=feature_types, report=fr)
    torch.cuda.synchronize(dev)
    rep.t_sketch = fr.t_sketch
    rep.t_boost = time.perf_counter() - t0 - fr.t_sketch
    rep.sample_rows = [N] * int(params.n_estimators)
    return bst


def _train_in_core(source, params: GBDTParams, N: int, F: int, dev: torch.device, cuts, nbins, feature_names,
                   feature_types, rep: ExternalReport) -> Booster:
    """Exact external-memory fit whose pages all fit the HBM budget: the chunks are binned into the
    in-core row records + feature-major bins (``bin_matrix_into``: no per-chunk copies) and the in-core
    trainer grows the trees -- the same trees the exact page passes grow, at in-core speed."""
    from ..ops import gbdt_ops
    from .gbdt import BinnedData, train_binned

    t0 = time.perf_counter()
    up = _PinnedUploader(dev)
    records = torch.zeros((N, gbdt_ops.row_stride(F)), dtype=torch.uint8, device=dev)
    binsT = torch.empty((F, N), dtype=torch.uint8, device=dev)
    y = torch.empty(N, dtype=torch.float32, device=dev)
    r0 = 0
    for Xc, yc in source():
        Xc = _as_np(Xc, np.float32)
        gbdt_ops.bin_matrix_into(up.put(Xc), cuts, nbins, records, binsT, r0)
        y[r0:r0 + len(Xc)] = torch.from_numpy(_as_np(yc, np.float32)).to(dev)
        r0 += len(Xc)
    if r0 != N:
        raise ValueError(f"the stream yielded {r0} rows on the binning pass, {N} on the sketch pass")
    torch.cuda.synchronize(dev)
    rep.n_pages = 0
    rep.host_bytes = 0
    rep.device_page_bytes = int(records.numel() + binsT.numel())
    rep.t_pages = time.perf_counter() - t0
    rep.mode = "in-core"
    t0 = time.perf_counter()
    bd = BinnedData(dev, N, N, F, 0, cuts, nbins, records=records, binsT=binsT)
    bst = train_binned(bd, y, params, feature_names=feature_names, feature_types=feature_types)
    torch.cuda.synchronize(dev)
    rep.t_boost = time.perf_counter() - t0
    rep.sample_rows = [N] * int(params.n_estimators)
    return bst


class _HostPasses:
    """NumPy page passes + host tree growth: the executable specification of the GPU path."""

    def __init__(self, pages, y, w, base_margin, F, cap, gscale, hscale, dev, cuts, nbins, hp, T, fmask):
        self.pages, self.F, self.cap, self.hp, self.fmask = pages, F, cap, hp, fmask
        self.y, self.w = y.cpu().numpy().astype(np.float64), w.cpu().numpy().astype(np.float64)
        self.margin = np.full(len(self.y), np.float32(base_margin), dtype=np.float32)
        self.gscale, self.hscale = gscale, hscale
        self.cuts, self.nbins = cuts.cpu().numpy(), nbins.cpu().numpy()
        self.trees: list[np.ndarray] = []
        self.sample = None

    def page_pass(self, prev: int, mu: float, t: int):
        counts = np.zeros(OOC_BINS, dtype=np.int64)
        key = np.uint64(ooc_key(self.hp.seed, t))
        sb, sg, sh = [], [], []
        for r0, bins in self.pages:
            n = len(bins)
            sl = slice(r0, r0 + n)
            if prev >= 0:
                self.margin[sl] = (self.margin[sl] + apply_nodes_bins(self.trees[prev], bins)).astype(np.float32)
            m = self.margin[sl].astype(np.float64)
            p = 1.0 / (1.0 + np.exp(-m))
            g = (p - self.y[sl]) * self.w[sl]
            h = np.maximum(p * (1.0 - p), 1e-16) * self.w[sl]
            gh = np.sqrt(g * g + h * h)
            counts += np.bincount(ghat_bin(gh), minlength=OOC_BINS)
            if mu > 0.0:
                pk = np.where(gh >= mu, 1.0, gh / mu)
                hs = gbdt_host.splitmix64_np(key ^ np.arange(r0, r0 + n, dtype=np.uint64))
                keep = (hs >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0) < pk
                sb.append(bins[keep])
                sg.append(np.clip(np.rint(g[keep] / pk[keep] * self.gscale), -65536, 65536).astype(np.int64))
                sh.append(np.clip(np.rint(h[keep] / pk[keep] * self.hscale), 0, 65536).astype(np.int64))
        ns = 0
        if mu > 0.0:
            self.sample = (np.concatenate(sb), np.concatenate(sg), np.concatenate(sh))
            ns = len(self.sample[0])
        return ns, counts

    def grow(self, t: int, ns: int) -> None:
        bins, gq, hq = self.sample
        self.trees.append(gbdt_host.grow_tree_host(bins, self.cuts, self.nbins, gq, hq,
                                                   np.zeros(len(bins), np.float32), self.hp, self.fmask[t]))

    def fetch(self) -> np.ndarray:
        return np.stack(self.trees) if self.trees else np.zeros((0, (1 << (self.hp.max_depth + 1)) - 1), NODE_DTYPE)

    def close(self) -> None:
        pass


class _GpuPasses:
    """``k_ooc_page`` over pinned host pages (H2D of page k+1 overlaps the pass over page k) and the
    in-core trainer in sampled mode."""

    def __init__(self, pages, y, w, base_margin, F, cap, gscale, hscale, dev, cuts, nbins, hp, T, fmask):
        from .. import _native
        from ..ops import gbdt_ops

        self.native, self.lib = _native, _native.lib()
        self.pages, self.F, self.cap, self.dev, self.hp = pages, F, cap, dev, hp
        self.gscale, self.hscale = gscale, hscale
        self.y, self.w = y.contiguous(), w.contiguous()
        self.margin = torch.full((len(y),), base_margin, dtype=torch.float32, device=dev)
        st = gbdt_ops.row_stride(F)
        self.srec = torch.zeros((cap, st), dtype=torch.uint8, device=dev)
        self.sbinsT = torch.zeros((F, cap), dtype=torch.uint8, device=dev)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.hist = torch.zeros(OOC_BINS, dtype=torch.int32, device=dev)
        self.tr = gbdt_ops.GpuGbdtTrainer(n_rows=cap, n_feat=F, max_depth=hp.max_depth, max_trees=T, eta=hp.eta,
                                          reg_lambda=hp.reg_lambda, reg_alpha=hp.reg_alpha, gamma=hp.gamma,
                                          min_child_weight=hp.min_child_weight, subsample=1.0, gscale=gscale,
                                          hscale=hscale, base_margin=base_margin, seed=hp.seed)
        fm = torch.as_tensor(fmask, device=dev).contiguous()
        self.tr.set_data(self.srec, self.sbinsT, cuts.contiguous(), nbins.to(torch.int32).contiguous(),
                         torch.zeros(cap, device=dev), torch.ones(cap, device=dev), torch.zeros(cap, device=dev), fm)
        biggest = max((p.shape[0] for _, p in pages), default=1)
        self.ps = page_stride(F)
        self.stage = [torch.empty((biggest, self.ps), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(dev)
        self.T = T

    def page_pass(self, prev: int, mu: float, t: int):
        cur = torch.cuda.current_stream(self.dev)
        self.counter.zero_()
        self.hist.zero_()
        prev_ptr = self.tr.tree_ptr(prev) if prev >= 0 else None
        key = ooc_key(self.hp.seed, t)
        done = [None, None]  # events: the pass that last read each staging buffer
        for k, (r0, page) in enumerate(self.pages):
            if page.is_cuda:  # HBM-resident page: no copy
                rc = self.lib.cobalt_ooc_page(page.data_ptr(), page.shape[1], page.shape[0], r0, self.F, prev_ptr,
                                              self.tr.max_nodes,
                                              self.margin.data_ptr(), self.y.data_ptr(), self.w.data_ptr(), key, 0,
                                              float(mu), self.gscale, self.hscale, self.srec.data_ptr(),
                                              self.sbinsT.data_ptr(), self.cap, self.counter.data_ptr(),
                                              self.hist.data_ptr(), self.native.stream_handle())
                self.native.check(rc, "cobalt_ooc_page")
                continue
            buf = self.stage[k & 1]
            with torch.cuda.stream(self.copy_stream):
                if done[k & 1] is not None:
                    self.copy_stream.wait_event(done[k & 1])
                buf[: page.shape[0]].copy_(page, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            cur.wait_event(ev)
            rc = self.lib.cobalt_ooc_page(buf.data_ptr(), page.shape[1], page.shape[0], r0, self.F, prev_ptr,
                                          self.tr.max_nodes,
                                          self.margin.data_ptr(), self.y.data_ptr(), self.w.data_ptr(), key, 0,
                                          float(mu), self.gscale, self.hscale, self.srec.data_ptr(),
                                          self.sbinsT.data_ptr(), self.cap, self.counter.data_ptr(),
                                          self.hist.data_ptr(), self.native.stream_handle())
            self.native.check(rc, "cobalt_ooc_page")
            e2 = torch.cuda.Event()
            e2.record(cur)
            done[k & 1] = e2
        ns = int(self.counter.item())
        return ns, self.hist.cpu().numpy().astype(np.int64)

    def grow(self, t: int, ns: int) -> None:
        self.tr.set_rows(ns)
        self.tr.grow_sampled(t)

    def fetch(self) -> np.ndarray:
        return self.tr.fetch(0, self.T)

    def close(self) -> None:
        self.tr.close(park=False)


def _train_exact(pages, y, w, base_margin, F, dev, cuts, nbins, params, T, fmask, wmax) -> np.ndarray:
    """Every row every tree (``sample_rate=1``): the in-core fixed-point scales and dither, so the trees
    equal the in-core fit's byte for byte. GPU: level-wise page streaming (``cobalt_gbdt_ox_*``, the
    in-core split evaluation on histograms summed page by page; ~22 B per row on the device). CPU: the
    host trainer on the concatenated pages (the oracle)."""
    D = int(params.max_depth)
    gscale, hscale = gbdt_host.quant_scales(wmax)
    hp = gbdt_host.HostGbdtParams(max_depth=D, eta=float(params.learning_rate), reg_lambda=float(params.reg_lambda),
                                  reg_alpha=float(params.reg_alpha), gamma=float(params.gamma),
                                  min_child_weight=float(params.min_child_weight), subsample=float(params.subsample),
                                  seed=int(params.random_state), gscale=gscale, hscale=hscale)
    if dev.type != "cuda":
        bins = np.concatenate([p for _, p in pages]) if pages else np.zeros((0, F), np.uint8)
        bins = np.ascontiguousarray(bins[:, :F])
        margin = np.full(len(bins), np.float32(base_margin), dtype=np.float32)
        yn, wn = y.cpu().numpy(), w.cpu().numpy()
        c_np, nb_np = cuts.cpu().numpy(), nbins.cpu().numpy()
        recs = []
        for t in range(T):
            gq, hq = gbdt_host.gradients_host(margin, yn, wn, hp, t, 0)
            recs.append(gbdt_host.grow_tree_host(bins, c_np, nb_np, gq, hq, margin, hp, fmask[t]))
        return np.stack(recs) if recs else np.zeros((0, (1 << (D + 1)) - 1), NODE_DTYPE)
    from .. import _native
    from ..ops import gbdt_ops

    lib, stream = _native.lib(), _native.stream_handle
    N = len(y)
    dummy = 4096
    tr = gbdt_ops.GpuGbdtTrainer(n_rows=dummy, n_feat=F, max_depth=D, max_trees=T, eta=hp.eta, reg_lambda=hp.reg_lambda,
                                 reg_alpha=hp.reg_alpha, gamma=hp.gamma, min_child_weight=hp.min_child_weight,
                                 subsample=hp.subsample, gscale=gscale, hscale=hscale, base_margin=base_margin,
                                 seed=hp.seed)
    try:
        fm = torch.as_tensor(fmask, device=dev).contiguous()
        z = torch.zeros(dummy, device=dev)
        tr.set_data(torch.zeros((dummy, gbdt_ops.row_stride(F)), dtype=torch.uint8, device=dev),
                    torch.zeros((F, dummy), dtype=torch.uint8, device=dev), cuts.contiguous(),
                    nbins.to(torch.int32).contiguous(), z, torch.ones(dummy, device=dev), z.clone(), fm)
        margin = torch.full((N,), base_margin, dtype=torch.float32, device=dev)
        yy, ww = y.to(dev, torch.float32).contiguous(), w.to(dev, torch.float32).contiguous()
        _native.check(lib.cobalt_gbdt_ox_init(tr.h, N, margin.data_ptr(), yy.data_ptr(), ww.data_ptr()),
                      "cobalt_gbdt_ox_init")
        biggest = max((p.shape[0] for _, p in pages), default=1)
        ps = pages[0][1].shape[1] if pages else page_stride(F)
        stage = [torch.empty((biggest, ps), dtype=torch.uint8, device=dev) for _ in range(2)]
        copy_stream = torch.cuda.Stream(dev)
        # last pass reading each staging buffer: kept ACROSS passes (the next pass's first uploads
        # overwrite the buffers the previous pass's last pages are still being read from)
        done = [None, None]

        def stream_pages(mode: int, t: int) -> None:
            cur = torch.cuda.current_stream(dev)
            for k, (r0, page) in enumerate(pages):
                if page.is_cuda:
                    ptr = page.data_ptr()
                else:  # double-buffered H2D on the copy stream, overlapping the previous page's pass
                    buf = stage[k & 1]
                    with torch.cuda.stream(copy_stream):
                        if done[k & 1] is not None:
                            copy_stream.wait_event(done[k & 1])
                        buf[: page.shape[0]].copy_(page, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(copy_stream)
                    cur.wait_event(ev)
                    ptr = buf.data_ptr()
                rc = lib.cobalt_gbdt_ox_page(tr.h, ptr, page.shape[1], page.shape[0], r0, mode, t, stream())
                _native.check(rc, "cobalt_gbdt_ox_page")
                if not page.is_cuda:
                    e2 = torch.cuda.Event()
                    e2.record(cur)
                    done[k & 1] = e2

        for t in range(T):
            _native.check(lib.cobalt_gbdt_ox_begin(tr.h, t, stream()), "cobalt_gbdt_ox_begin")
            stream_pages(-1, t)
            _native.check(lib.cobalt_gbdt_ox_level(tr.h, 0, t, stream()), "cobalt_gbdt_ox_level")
            for lv in range(D - 1):
                stream_pages(lv, t)
                _native.check(lib.cobalt_gbdt_ox_level(tr.h, lv + 1, t, stream()), "cobalt_gbdt_ox_level")
            _native.check(lib.cobalt_gbdt_ox_end(tr.h, t, stream()), "cobalt_gbdt_ox_end")
        return tr.fetch(0, T)
    finally:
        tr.close(park=False)
