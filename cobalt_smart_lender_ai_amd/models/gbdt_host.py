"""Host (NumPy) implementation of the histogram GBDT trainer.

This is the executable specification of ``csrc/gbdt.hip``: same fixed-point gradient quantisation,
same histogram + subtraction scheme, same split enumeration order, tie-break and acceptance rules,
same leaf update. It serves three purposes:

* the oracle of the GPU trainer tests (given identical cuts both produce identical trees);
* the ``device="cpu"`` execution path (CPU-only hosts, CI);
* the CPU data-parallel rehearsal: with a ``torch.distributed`` gloo group the per-level histograms
  are all-reduced exactly like the GPU path all-reduces them over RCCL.

Split semantics follow XGBoost's ``hist`` updater (reference: the ``XGBClassifier`` fits at
src/model_train_test/model_tree_train_test.py:111-164): gain ``G_L²/(H_L+λ) + G_R²/(H_R+λ) -
G²/(H+λ)`` (L1-thresholded when ``alpha > 0``), both default directions for features with missing
values in the node, children need ``H >= min_child_weight``, a split needs ``loss_chg > 1e-6`` and
``loss_chg >= gamma`` (``min_split_loss``), leaf value ``-G/(H+λ) * eta``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .booster import NODE_DTYPE

FLT_MAX = np.float32(np.finfo(np.float32).max)
MASK64 = (1 << 64) - 1
QBITS = 17          # |g_q| < 2^17, h_q <= 2^17: a <= 16384-row histogram block sums to < 2^31
G_CLIP = (1 << QBITS) - 1
H_CLIP = 1 << QBITS
QBITS_WIDE = 25     # wide gradients (grad_bits=25): int64 histogram cells on the GPU
GRAD_BITS = (QBITS, QBITS_WIDE)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def splitmix64_int(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def tree_key(seed: int, tree: int) -> int:
    return splitmix64_int((seed ^ ((0xA5A5A5A5 + tree * 0x632BE59BD9B4E019) & MASK64)) & MASK64)


def dither_key(seed: int, tree: int) -> int:
    """Per-tree key of the gradient quantiser's dither (csrc/gbdt.hip quantize_gh)."""
    return splitmix64_int((tree_key(seed, tree) ^ 0xD1B54A32D192ED03) & MASK64)


def dither_uniforms(seed: int, tree: int, global_rows: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Two independent U[0,1) per row (high / low 32 bits of one splitmix64 draw)."""
    hsh = splitmix64_np(np.uint64(dither_key(seed, tree)) ^ global_rows.astype(np.uint64))
    ug = (hsh >> np.uint64(32)).astype(np.float64) * (1.0 / 4294967296.0)
    uh = (hsh & np.uint64(0xFFFFFFFF)).astype(np.float64) * (1.0 / 4294967296.0)
    return ug, uh


def row_sample_mask(seed: int, tree: int, global_rows: np.ndarray, rate: float) -> np.ndarray:
    h = splitmix64_np(np.uint64(tree_key(seed, tree)) ^ global_rows.astype(np.uint64))
    u = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return u < rate


@dataclass
class HostGbdtParams:
    max_depth: int
    eta: float
    reg_lambda: float
    reg_alpha: float
    gamma: float
    min_child_weight: float
    subsample: float
    seed: int
    gscale: float
    hscale: float
    quant: bool = True   # False: unquantised fp64 gradients and histograms (accuracy reference)
    qbits: int = QBITS   # quantised magnitude bits: 17, or 25 (wide gradients)


def quant_scales(w_max: float, bits: int = QBITS) -> tuple[float, float]:
    """Fixed-point scales: |g| <= w and h <= w/4, so both quantised magnitudes stay <= 2^bits. At 17
    bits a 16384-row histogram block sums to < 2^31 -- the packed-u64 LDS accumulation on the GPU keeps
    h in the low 32 bits (no carry into g) and g as a signed 32-bit high half; at 25 bits (wide
    gradients) the GPU sums g and h in separate int64 cells."""
    if bits not in GRAD_BITS:
        raise ValueError(f"grad_bits must be one of {GRAD_BITS}")
    w_max = float(w_max) if w_max > 0 else 1.0
    return float(2 ** bits) / w_max, float(2 ** (bits + 2)) / w_max


def _thresh_l1(g, alpha):
    return np.where(g > alpha, g - alpha, np.where(g < -alpha, g + alpha, 0.0))


def _calc_gain(g, h, lam, alpha, mcw):
    t = g if alpha == 0.0 else _thresh_l1(g, alpha)
    return np.where(h < mcw, 0.0, (t * t) / (h + lam))


def _calc_gain_pair(gl, hl, gr, hr, lam, alpha):
    """Both children's gains with one division, in the device's operation order (csrc/gbdt.hip,
    calc_gain_pair); only used where both children reach min_child_weight."""
    tl = gl if alpha == 0.0 else _thresh_l1(gl, alpha)
    tr = gr if alpha == 0.0 else _thresh_l1(gr, alpha)
    dl = hl + lam
    dr = hr + lam
    with np.errstate(divide="ignore", invalid="ignore"):
        return (tl * tl * dr + tr * tr * dl) / (dl * dr)


def _calc_weight(g: float, h: float, lam: float, alpha: float, mcw: float) -> float:
    if h < mcw or h <= 0.0:
        return 0.0
    t = g if alpha == 0.0 else float(_thresh_l1(np.float64(g), alpha))
    return -t / (h + lam)


def gradients_host(margin: np.ndarray, label: np.ndarray, weight: np.ndarray, p: HostGbdtParams, tree: int,
                   row_offset: int = 0) -> tuple[np.ndarray, np.ndarray]:
    m = margin.astype(np.float64)
    pr = 1.0 / (1.0 + np.exp(-m))
    y = label.astype(np.float64)
    w = weight.astype(np.float64)
    g = (pr - y) * w
    h = np.maximum(pr * (1.0 - pr), 1e-16) * w
    if p.subsample < 1.0:
        keep = row_sample_mask(p.seed, tree, row_offset + np.arange(len(m), dtype=np.int64), p.subsample)
        g = np.where(keep, g, 0.0)
        h = np.where(keep, h, 0.0)
    if not p.quant:
        return g, h
    # unbiased fixed point: floor(x * scale + u), u ~ U[0,1) from a per-(tree, global row) hash, so
    # E[q] = x * scale exactly -- small hessians are not flushed to 0 and the rounding error of a sum
    # averages out instead of accumulating a bias; deterministic (same on every device / rank count)
    ug, uh = dither_uniforms(p.seed, tree, row_offset + np.arange(len(m), dtype=np.int64))
    gclip, hclip = (1 << p.qbits) - 1, 1 << p.qbits
    gq = np.clip(np.floor(g * p.gscale + ug), -gclip, gclip).astype(np.int64)
    hq = np.clip(np.floor(h * p.hscale + uh), 0, hclip).astype(np.int64)
    return gq, hq


def _node_hist(bins, rows, gq, hq, fmask, nbins=None) -> np.ndarray:
    """Histogram of one node. Code 255 is the missing bin, except for 256-bin features (no missing
    values), where it is the real bin 255."""
    F = bins.shape[1]
    dt = np.int64 if np.issubdtype(gq.dtype, np.integer) else np.float64
    out = np.zeros((F + 1, 256, 2), dtype=dt)
    g = gq[rows]
    h = hq[rows]
    for f in range(F):
        if not fmask[f]:
            continue
        b = bins[rows, f].astype(np.int64)
        m = (b != 255) | (nbins is not None and int(nbins[f]) >= 256)
        out[f, :, 0] = np.bincount(b[m], weights=g[m].astype(np.float64), minlength=256)[:256].astype(dt)
        out[f, :, 1] = np.bincount(b[m], weights=h[m].astype(np.float64), minlength=256)[:256].astype(dt)
        if F < 255:  # rows with a missing value of f (exact counts; survive the subtraction trick)
            out[F, 1 + f, 0] = len(m) - int(np.count_nonzero(m))
    out[F, 0, 0] = g.sum()
    out[F, 0, 1] = h.sum()
    return out


def _eval_node(hist, G, H, nbins, fmask, p: HostGbdtParams):
    """Best split of one node: returns (gain, key, GL, HL) or None."""
    ginv, hinv = 1.0 / p.gscale, 1.0 / p.hscale
    Gd, Hd = G * ginv, H * hinv
    pg = float(_calc_gain(np.float64(Gd), np.float64(Hd), p.reg_lambda, p.reg_alpha, p.min_child_weight))
    best_gain, best_key, best_gl, best_hl = -np.inf, np.iinfo(np.int32).max, 0, 0
    F = len(nbins)
    for f in range(F):
        if not fmask[f]:
            continue
        nb = int(nbins[f])
        hg, hh = hist[f, :, 0], hist[f, :, 1]
        cg, ch = np.cumsum(hg), np.cumsum(hh)
        mg, mh = G - cg[-1].item(), H - ch[-1].item()
        b = np.arange(nb)
        cands = [(cg[:nb], ch[:nb], f * 1024 + b)]
        # fp64 mode: G - sum(bins) is not exactly 0 without missing values, so use the missing count
        has_missing = mg != 0 or mh != 0 if p.quant else (F >= 255 or hist[F, 1 + f, 0] > 0)
        if has_missing:
            cands.append((cg[:nb] - hg[:nb] + mg, ch[:nb] - hh[:nb] + mh, f * 1024 + 512 + (nb - 1 - b)))
        for GL, HL, key in cands:
            gl = GL.astype(np.float64) * ginv
            hl = HL.astype(np.float64) * hinv
            gr = (G - GL).astype(np.float64) * ginv
            hr = (H - HL).astype(np.float64) * hinv
            ok = (hl >= p.min_child_weight) & (hr >= p.min_child_weight)
            if not ok.any():
                continue
            gain = _calc_gain_pair(gl, hl, gr, hr, p.reg_lambda, p.reg_alpha) - pg
            gain = np.where(ok, gain, -np.inf)
            mx = gain.max()
            if mx == -np.inf:
                continue
            sel = np.nonzero(gain == mx)[0]
            i = sel[np.argmin(key[sel])]
            if mx > best_gain or (mx == best_gain and key[i] < best_key):
                best_gain, best_key, best_gl, best_hl = float(mx), int(key[i]), GL[i].item(), HL[i].item()
    if best_key == np.iinfo(np.int32).max:
        return None, Gd, Hd
    return (best_gain, best_key, best_gl, best_hl), Gd, Hd


def grow_tree_host(bins: np.ndarray, cuts: np.ndarray, nbins: np.ndarray, gq: np.ndarray, hq: np.ndarray,
                   margin: np.ndarray, p: HostGbdtParams, fmask: np.ndarray, allreduce=None) -> np.ndarray:
    """Grow one depthwise tree in place of ``margin`` (float32, updated with leaf values).

    Returns the heap-ordered node records (``NODE_DTYPE``). ``allreduce(arr_int64) -> arr`` sums the
    built histograms across data-parallel ranks (identity when ``None``).
    """
    D = p.max_depth
    N, F = bins.shape
    max_nodes = (1 << (D + 1)) - 1
    nodes = np.zeros(max_nodes, dtype=NODE_DTYPE)
    nodes["feat"] = -1
    nodes["bin"] = -1
    nodes[0]["status"] = 1
    nodes[0]["build"] = 1
    nodes[0]["count"] = N
    GH = np.zeros((max_nodes, 2), dtype=np.int64 if p.quant else np.float64)  # node (G, H) sums
    rows: dict[int, np.ndarray] = {0: np.arange(N, dtype=np.int64)}
    hist_prev: dict[int, np.ndarray] = {}
    for level in range(D + 1):
        first, nlev = (1 << level) - 1, 1 << level
        level_nodes = range(first, first + nlev)
        if level > 0:
            for q in range((1 << (level - 1)) - 1, first):
                if nodes[q]["status"] != 2:
                    continue
                L, R = 2 * q + 1, 2 * q + 2
                left_small = GH[L, 1] <= GH[R, 1]
                nodes[L]["build"] = 1 if left_small else 0
                nodes[R]["build"] = 0 if left_small else 1
        hist_cur: dict[int, np.ndarray] = {}
        if level < D:
            built = [n for n in level_nodes if nodes[n]["status"] == 1 and nodes[n]["build"] == 1]
            if level == 0:
                built = [0]
            nslots = 1 if level == 0 else (1 << (level - 1))
            slots = np.zeros((nslots, F + 1, 256, 2), dtype=GH.dtype)
            for n in built:
                slot = 0 if level == 0 else ((n - first) >> 1)
                slots[slot] = _node_hist(bins, rows.get(n, np.zeros(0, np.int64)), gq, hq, fmask, nbins)
            if allreduce is not None:
                slots = allreduce(slots)
            for n in level_nodes:
                if nodes[n]["status"] != 1:
                    continue
                slot = 0 if level == 0 else ((n - first) >> 1)
                if nodes[n]["build"]:
                    hist_cur[n] = slots[slot]
                else:
                    par = (n - 1) // 2
                    hist_cur[n] = hist_prev[par] - slots[slot]
            if level == 0:
                GH[0] = hist_cur[0][F, 0]
        for n in level_nodes:
            nd = nodes[n]
            if nd["status"] != 1:
                continue
            G, H = GH[n, 0].item(), GH[n, 1].item()
            if level < D:
                best, Gd, Hd = _eval_node(hist_cur[n], G, H, nbins, fmask, p)
            else:
                best, Gd, Hd = None, G * (1.0 / p.gscale), H * (1.0 / p.hscale)
            wgt = _calc_weight(Gd, Hd, p.reg_lambda, p.reg_alpha, p.min_child_weight)
            nodes[n]["sum_hess"] = np.float32(Hd)
            nodes[n]["base_weight"] = np.float32(wgt * p.eta)
            ok = False
            if best is not None:
                loss = np.float32(best[0])
                ok = bool(loss > np.float32(1e-6) and loss >= np.float32(p.gamma))
            r = rows.get(n, np.zeros(0, np.int64))
            if ok:
                gain, key, GL, HL = best
                f = key >> 10
                rr = key & 1023
                nb = int(nbins[f])
                if rr < 512:
                    j, dl = rr, 0
                else:
                    j, dl = (nb - 1 - (rr - 512)) - 1, 1
                nodes[n]["status"] = 2
                nodes[n]["feat"] = f
                nodes[n]["bin"] = j
                nodes[n]["default_left"] = dl
                nodes[n]["split_cond"] = cuts[f, j] if j >= 0 else -FLT_MAX
                nodes[n]["loss_chg"] = np.float32(gain)
                L, R = 2 * n + 1, 2 * n + 2
                nodes[L]["status"], nodes[R]["status"] = 1, 1
                GH[L] = (GL, HL)
                GH[R] = (G - GL, H - HL)
                b = bins[r, f]
                go_left = np.where(b == 255, dl == 1, b.astype(np.int64) <= j)
                rows[L] = r[go_left]
                rows[R] = r[~go_left]
                nodes[L]["count"] = len(rows[L])
                nodes[R]["count"] = len(rows[R])
            else:
                lv = np.float32(wgt * p.eta)
                nodes[n]["status"] = 3
                nodes[n]["leaf_value"] = lv
                nodes[n]["split_cond"] = lv
                if len(r):
                    margin[r] = (margin[r] + lv).astype(np.float32)
        hist_prev = hist_cur
    if p.quant:
        nodes["G"], nodes["H"] = GH[:, 0], GH[:, 1]
    return nodes
