"""Large-batch scoring (BASELINE.json config "Batch inference: 1B-row scoring via hipGraph on
8xMI355X"; SURVEY.md §2.6 batch-parallel inference, §7.3 P6).

Rows are sharded contiguously over the ranks (one process per GPU, ``torch.distributed``); each rank
streams its shard through a fixed-size device chunk whose predictor launch is captured once into a
hipGraph and replayed per chunk, double-buffered on two streams so the H2D copy of chunk k+1
overlaps the scoring of chunk k. There is no collective except the final gather of per-rank counts
/ checksums (predictions stay on each rank or go to per-rank output files).

``score_shard`` is the per-rank engine; ``score_device_matrix`` scores a device-resident matrix
(the benchmark path: data generated on the GPU, no PCIe in the loop; the chunk launches run in
place on the matrix, captured into one hipGraph).
"""
from __future__ import annotations

import numpy as np
import torch

from ..models.booster import Booster
from ..ops import predict_ops


_SCORE_GRAPH_CACHE = 8  # captured score_device_matrix graphs kept per booster


class GraphScorer:
    """A predictor launch over a static [chunk, F] device buffer, captured into a hipGraph."""

    def __init__(self, booster: Booster, chunk: int, n_feat: int, device, use_graph: bool = True):
        self.booster, self.chunk, self.device = booster, int(chunk), torch.device(device)
        self.x = torch.zeros((self.chunk, n_feat), dtype=torch.float32, device=self.device)
        self.prob = torch.empty(self.chunk, dtype=torch.float32, device=self.device)
        self.stream = torch.cuda.Stream(self.device)
        self.graph = None
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            predict_ops.predict_gpu(booster, self.x, None, out_prob=self.prob)  # warm-up: packs the forest
            self.stream.synchronize()
            if use_graph:
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, stream=self.stream):
                    predict_ops.predict_gpu(booster, self.x, None, out_prob=self.prob)

    def run(self) -> None:
        # on the scorer's stream: a graph replays on the CURRENT stream, and the chunk copies in and
        # out are ordered on this one (replaying on the default stream raced with both)
        with torch.cuda.stream(self.stream):
            if self.graph is not None:
                self.graph.replay()
            else:
                predict_ops.predict_gpu(self.booster, self.x, None, out_prob=self.prob)


def score_device_matrix(booster: Booster, X: torch.Tensor, out: torch.Tensor | None = None,
                        chunk: int = 1 << 22, capture: bool = True) -> torch.Tensor:
    """Probabilities of a device-resident [N, F] matrix.

    Row-contiguous fp32 input is scored in place: the predictor launches for every ``chunk`` rows run
    straight on views of X and ``out``. (The earlier form staged each chunk into a GraphScorer's
    static buffer: a D2D copy per chunk plus the scorer's warm-up launch, ~10% of the 125M-row
    shard.) The launch sequence is captured into a hipGraph the SECOND time the same (X, out) buffers
    are scored and replayed from then on (a serving loop over static buffers); a one-off call
    launches directly instead of paying a capture it would replay once. ``capture=False`` never
    captures (the API's bulk requests: per-request buffers, scored next to the serving engine's own
    graph replays). Other layouts go through a
    GraphScorer's static buffer chunk by chunk."""
    N, F = X.shape
    out = out if out is not None else torch.empty(N, dtype=torch.float32, device=X.device)
    if N == 0:
        return out
    if (X.dtype == torch.float32 and X.stride(1) == 1 and out.is_contiguous()
            and out.dtype == torch.float32 and out.device == X.device):
        gf = predict_ops.gpu_forest(booster, X.device)  # pack + upload the forest outside any capture
        cur = torch.cuda.current_stream(X.device)
        side = torch.cuda.Stream(X.device)
        side.wait_stream(cur)  # X (and out) may still be in flight on the caller's stream

        def launches():
            for s in range(0, N, chunk):
                e = min(N, s + chunk)
                predict_ops.predict_gpu(booster, X[s:e], None, out_prob=out[s:e])

        cache = booster.__dict__.setdefault("_score_graphs", {})
        key = (str(X.device), X.data_ptr(), X.stride(0), N, F, out.data_ptr(), int(chunk), id(gf))
        graph = cache.get(key)
        if graph is None and key in cache and capture:  # second sighting of these buffers: capture
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                launches()
            cache[key] = graph
        with torch.cuda.stream(side):
            if graph is not None:
                graph.replay()
            else:
                launches()
                if len(cache) >= _SCORE_GRAPH_CACHE:  # bounded: drop the oldest entry
                    cache.pop(next(iter(cache)))
                cache[key] = None
        side.synchronize()
        cur.wait_stream(side)
        return out
    sc = GraphScorer(booster, min(chunk, N), F, X.device)
    sc.stream.wait_stream(torch.cuda.current_stream(X.device))  # X may still be in flight there
    for s in range(0, N, sc.chunk):
        e = min(N, s + sc.chunk)
        with torch.cuda.stream(sc.stream):
            sc.x[: e - s].copy_(X[s:e], non_blocking=True)
            if e - s < sc.chunk:
                sc.x[e - s:].zero_()
        sc.run()
        with torch.cuda.stream(sc.stream):
            out[s:e].copy_(sc.prob[: e - s], non_blocking=True)
    sc.stream.synchronize()
    return out


class NpyShard:
    """A ``.npy`` shard read with ``preadv`` straight into caller buffers (the pinned staging slots).

    Memory-mapping the file instead costs a minor page fault per 4 KB the first time each page is
    touched -- ~20k faults per 80 MB chunk, which bounded the mapped path at ~3 ms per chunk (~27 GB/s)
    while the upload itself runs at ~54 GB/s. The header is parsed without unpickling anything."""

    def __init__(self, path):
        import os

        self.path = str(path)
        with open(self.path, "rb") as fh:
            ver = np.lib.format.read_magic(fh)
            rd = np.lib.format.read_array_header_1_0 if ver == (1, 0) else np.lib.format.read_array_header_2_0
            shape, fortran, dtype = rd(fh)  # literal header, nothing unpickled
            self.offset = fh.tell()
        if dtype != np.float32 or fortran or len(shape) != 2:
            raise ValueError(f"{self.path}: need a C-ordered 2-D float32 array, got {dtype} {shape}")
        self.shape = tuple(int(x) for x in shape)
        self.row_bytes = self.shape[1] * 4
        self.fd = os.open(self.path, os.O_RDONLY)

    def __len__(self) -> int:
        return self.shape[0]

    def close(self) -> None:
        import os

        if self.fd is not None:
            os.close(self.fd)
            self.fd = None

    def read_rows(self, dst: np.ndarray, r0: int, r1: int) -> None:
        """Rows [r0, r1) into dst[:r1-r0] (C-contiguous float32 [*, F])."""
        import os

        mv = memoryview(dst[: r1 - r0].reshape(-1).view(np.uint8))
        want, got = (r1 - r0) * self.row_bytes, 0
        while got < want:
            n = os.preadv(self.fd, [mv[got:want]], self.offset + r0 * self.row_bytes + got)
            if n <= 0:
                raise IOError(f"{self.path}: short read at row {r0}")
            got += n


class _ShardView:
    """Rows [b, e) of an NpyShard, sliceable like an array (for HostStreamScorer.score)."""

    def __init__(self, shard: NpyShard, b: int, e: int):
        self.shard, self.b, self.e = shard, b, e

    def __len__(self) -> int:
        return self.e - self.b


class HostStreamScorer:
    """Host-resident scoring pipeline (host DRAM / memory-mapped files -> HBM -> scores -> host).

    ``slots`` pinned staging slots rotate through four stages that overlap across chunks:
    (1) the rows of chunk k are copied from the source (an array or ``np.memmap`` view) into pinned
    slot k % slots by a thread pool (several memcpy streams -- one thread does ~10 GB/s, short of
    the ~50 GB/s PCIe Gen5 link); (2) H2D on a copy stream; (3) the predictor graph of that slot on
    the compute stream, ordered after the copy by an event; (4) D2H of the probabilities on a second
    copy stream (so chunk k's read-back never queues in front of chunk k+1's upload). A slot is
    reused only once its read-back event has completed -- the host waits on per-chunk events, never
    on a whole stream, so staging chunk k+1 overlaps the GPU work of chunks k-slots+1..k.
    """

    def __init__(self, booster: Booster, chunk: int, n_feat: int, device, slots: int = 4, stage_threads: int = 8,
                 h2d_streams: int = 2):
        from concurrent.futures import ThreadPoolExecutor

        self.booster, self.chunk, self.F = booster, int(chunk), int(n_feat)
        self.dev = torch.device(device)
        self.slots = max(2, int(slots))
        # each chunk's upload is split over several copy streams: one copy runs on one DMA engine,
        # and a single engine does not fill the host link
        self.h2d = [torch.cuda.Stream(self.dev) for _ in range(max(1, int(h2d_streams)))]
        self.d2h = torch.cuda.Stream(self.dev)
        self.comp = torch.cuda.Stream(self.dev)
        self.xh = [torch.empty((self.chunk, self.F), dtype=torch.float32).pin_memory() for _ in range(self.slots)]
        self.ph = [torch.empty(self.chunk, dtype=torch.float32).pin_memory() for _ in range(self.slots)]
        self.xh_np = [t.numpy() for t in self.xh]
        self.ph_np = [t.numpy() for t in self.ph]
        self.xd = [torch.zeros((self.chunk, self.F), dtype=torch.float32, device=self.dev) for _ in range(self.slots)]
        self.pd = [torch.empty(self.chunk, dtype=torch.float32, device=self.dev) for _ in range(self.slots)]
        self.graphs = []
        with torch.cuda.device(self.dev), torch.cuda.stream(self.comp):
            predict_ops.predict_gpu(booster, self.xd[0], None, out_prob=self.pd[0])  # packs + uploads the forest
            self.comp.synchronize()
            for k in range(self.slots):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.comp):
                    predict_ops.predict_gpu(booster, self.xd[k], None, out_prob=self.pd[k])
                self.graphs.append(g)
        self.nthreads = max(1, int(stage_threads))
        self.pool = ThreadPoolExecutor(self.nthreads) if self.nthreads > 1 else None

    def close(self) -> None:
        if self.pool is not None:
            self.pool.shutdown()
            self.pool = None

    def _stage(self, dst: np.ndarray, src, s: int, e: int) -> None:
        """Rows [s, e) of ``src`` into the pinned slot ``dst``, split over the staging threads."""
        n = e - s
        if isinstance(src, _ShardView):
            job = lambda a, b: src.shard.read_rows(dst[a:], src.b + s + a, src.b + s + b)  # noqa: E731
        else:
            job = lambda a, b: np.copyto(dst[a:b], src[s + a:s + b])  # noqa: E731
        if self.pool is None or n < 65536:
            job(0, n)
            return
        step = -(-n // self.nthreads)
        futs = [self.pool.submit(job, i, min(n, i + step)) for i in range(0, n, step)]
        for f in futs:
            f.result()

    def score(self, src, out: np.ndarray | None = None) -> np.ndarray:
        """Probabilities of the rows of ``src`` ([N, F] float32 array / memmap, or a shard view) into
        ``out`` ([N])."""
        N = len(src)
        out = np.empty(N, dtype=np.float32) if out is None else out
        busy: list[tuple[int, int, torch.cuda.Event] | None] = [None] * self.slots

        def retire(k: int) -> None:
            s, e, ev = busy[k]
            ev.synchronize()
            np.copyto(out[s:e], self.ph_np[k][: e - s])
            busy[k] = None

        # rows already in pinned host memory (torch.Tensor.pin_memory()) upload straight from the source
        direct = isinstance(src, torch.Tensor) and src.device.type == "cpu" and src.is_pinned()
        for i, s in enumerate(range(0, N, self.chunk)):
            e = min(N, s + self.chunk)
            k = i % self.slots
            if busy[k] is not None:
                retire(k)
            if not direct:
                self._stage(self.xh_np[k], src, s, e)
            n = e - s
            xsrc = src[s:e] if direct else self.xh[k][:n]
            part = -(-n // len(self.h2d))
            for j, st in enumerate(self.h2d):
                a, b = j * part, min(n, (j + 1) * part)
                if a >= b:
                    continue
                ev_in = torch.cuda.Event()
                with torch.cuda.stream(st):
                    self.xd[k][a:b].copy_(xsrc[a:b], non_blocking=True)
                    ev_in.record(st)
                self.comp.wait_event(ev_in)
            with torch.cuda.stream(self.comp):
                self.graphs[k].replay()
            ev_c = torch.cuda.Event()
            ev_c.record(self.comp)
            self.d2h.wait_event(ev_c)
            ev_out = torch.cuda.Event()
            with torch.cuda.stream(self.d2h):
                self.ph[k][:n].copy_(self.pd[k][:n], non_blocking=True)
                ev_out.record(self.d2h)
            busy[k] = (s, e, ev_out)
        for k in range(self.slots):
            if busy[k] is not None:
                retire(k)
        return out


def score_shard(booster: Booster, X_host: np.ndarray, chunk: int = 1 << 20, device=None, slots: int = 4,
                stage_threads: int = 8, h2d_streams: int = 2) -> np.ndarray:
    """Host matrix (array or memmap) -> probabilities through :class:`HostStreamScorer`."""
    dev = torch.device(device or "cuda")
    N, F = X_host.shape
    if N == 0:
        return np.empty(0, dtype=np.float32)
    sc = HostStreamScorer(booster, min(chunk, N), F, dev, slots=slots, stage_threads=stage_threads,
                          h2d_streams=h2d_streams)
    try:
        return sc.score(X_host)
    finally:
        sc.close()


# ------------------------------------------------------------------------------------------ files
def open_shards(paths) -> list[np.ndarray]:
    """Memory-map ``.npy`` shard files ([n_i, F] float32; never unpickled: ``allow_pickle=False``)."""
    arrs = [np.load(str(p), mmap_mode="r", allow_pickle=False) for p in paths]
    F = {a.shape[1] for a in arrs}
    if len(F) != 1 or any(a.ndim != 2 for a in arrs):
        raise ValueError("shards must be 2-D arrays with the same number of columns")
    return arrs


def rank_segments(sizes: list[int], rank: int, world: int) -> list[tuple[int, int, int, int]]:
    """The contiguous global row range of ``rank`` over the concatenated shards, as
    ``(file_index, begin, end, global_offset)`` segments (rows [begin, end) of that file)."""
    from ..parallel.dist import shard_range

    total = int(sum(sizes))
    r0, r1 = shard_range(total, rank, world)
    segs, off = [], 0
    for i, n in enumerate(sizes):
        b, e = max(r0, off), min(r1, off + n)
        if b < e:
            segs.append((i, b - off, e - off, b))
        off += n
    return segs


def score_files(booster: Booster, paths, out_dir, rank: int = 0, world: int = 1, device=None,
                chunk: int = 1 << 20, slots: int = 4, stage_threads: int = 8, h2d_streams: int = 2,
                max_rows: int | None = None) -> dict:
    """Score this rank's share of the shard files and write ``out_dir/scores_rank{rank:05d}.npy`` (+ a
    JSON index with the global row offset). GPU: the pipelined :class:`HostStreamScorer`; CPU: the
    host predictor (the multi-rank rehearsal of the sharding, tests/test_batch_score.py).
    ``max_rows``: score only the first rows of the share (warm-ups)."""
    import json
    from pathlib import Path

    arrs = open_shards(paths)  # validates the headers (and serves the CPU path)
    segs = rank_segments([len(a) for a in arrs], rank, world)
    if max_rows is not None:
        cut, left = [], int(max_rows)
        for i, b, e, g in segs:
            if left <= 0:
                break
            cut.append((i, b, min(e, b + left), g))
            left -= cut[-1][2] - b
        segs = cut
    n = sum(e - b for _, b, e, _ in segs)
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    out_path = out_dir / f"scores_rank{rank:05d}.npy"
    out = np.lib.format.open_memmap(str(out_path), mode="w+", dtype=np.float32, shape=(n,))
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    pos = 0
    sc = None
    try:
        if dev.type == "cuda" and n:
            sc = HostStreamScorer(booster, min(chunk, n), arrs[0].shape[1], dev, slots=slots,
                                  stage_threads=stage_threads, h2d_streams=h2d_streams)
        shards = {}
        for i, b, e, _ in segs:
            view = arrs[i][b:e]
            if sc is not None:
                if i not in shards:
                    shards[i] = NpyShard(paths[i])
                sc.score(_ShardView(shards[i], b, e), out[pos:pos + (e - b)])
            else:
                for s in range(0, e - b, chunk):
                    t = min(e - b, s + chunk)
                    p = booster.predict_proba(np.asarray(view[s:t], dtype=np.float32), device="cpu")
                    out[pos + s:pos + t] = np.asarray(p.cpu().numpy() if hasattr(p, "cpu") else p, np.float32)
            pos += e - b
        for sh in shards.values():
            sh.close()
    finally:
        if sc is not None:
            sc.close()
    out.flush()
    meta = {"rank": rank, "world": world, "rows": n, "global_offset": segs[0][3] if segs else None,
            "files": [str(p) for p in paths]}
    (out_dir / f"scores_rank{rank:05d}.json").write_text(json.dumps(meta))
    return meta


def gather_scores(out_dir) -> np.ndarray:
    """Concatenate the per-rank score files of ``out_dir`` in global row order.

    Only the ranks of the LAST job are used: the world size comes from rank 0's index, ranks
    ``0 .. world - 1`` must all be present with that world size, and their global row ranges must
    tile ``[0, total)`` without gaps or overlaps -- files left by an earlier run with more ranks are
    ignored, and an inconsistent directory raises instead of returning shifted rows."""
    import json
    from pathlib import Path

    d = Path(out_dir)
    p0 = d / "scores_rank00000.json"
    if not p0.exists():
        return np.empty(0, np.float32)
    world = int(json.loads(p0.read_text())["world"])
    metas = []
    for r in range(world):
        p = d / f"scores_rank{r:05d}.json"
        if not p.exists():
            raise ValueError(f"{d}: rank {r} of a {world}-rank job has no score index")
        m = json.loads(p.read_text())
        if int(m["world"]) != world:
            raise ValueError(f"{d}: rank {r} was written by a {m['world']}-rank job, rank 0 by a {world}-rank job")
        metas.append(m)
    live = sorted((m for m in metas if m["rows"]), key=lambda m: m["global_offset"])
    pos = 0
    for m in live:
        if int(m["global_offset"]) != pos:
            raise ValueError(f"{d}: rank {m['rank']} starts at row {m['global_offset']}, expected {pos}")
        pos += int(m["rows"])
    parts = [np.load(str(d / f"scores_rank{m['rank']:05d}.npy"), allow_pickle=False) for m in live]
    return np.concatenate(parts) if parts else np.empty(0, np.float32)


def make_shards(out_dir, rows: int, files: int, n_feat: int = 20, seed: int = 1, device=None) -> list[str]:
    """Write ``files`` synthetic LendingClub-shaped ``.npy`` shards with ``rows`` rows in total
    (generated on the GPU in pieces when one is available)."""
    from pathlib import Path

    from ..dataio import synth

    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    paths, base = [], 0
    per = -(-rows // files)
    for i in range(files):
        n = min(per, rows - base)
        if n <= 0:
            break
        p = out_dir / f"shard_{i:04d}.npy"
        mm = np.lib.format.open_memmap(str(p), mode="w+", dtype=np.float32, shape=(n, n_feat))
        for s in range(0, n, 10_000_000):
            e = min(n, s + 10_000_000)
            mm[s:e] = synth.make_lendingclub(e - s, seed=seed, row_offset=base + s, device=dev)[0][:, :n_feat].cpu().numpy()
        mm.flush()
        del mm
        paths.append(str(p))
        base += n
    return paths


def main(argv=None) -> int:
    """Batch scoring CLI (torchrun for N GPUs; rank 0 prints one JSON line with the whole-job rows/s,
    max time over ranks).

    * ``--input 'shards/*.npy'``: host/disk-resident -- every rank memory-maps the shard files, scores
      its contiguous share through the pinned pipeline and writes ``--output/scores_rankNNNNN.npy``;
    * ``--make-shards DIR --rows N --files K``: write synthetic LendingClub-shaped shards first;
    * default: ``--rows-per-gpu`` rows generated on each GPU (device-resident, hipGraph chunks)."""
    import argparse
    import glob
    import json
    import time
    from pathlib import Path

    from ..dataio import synth
    from ..models.booster import load_pickle_bytes
    from ..parallel import dist as pdist

    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-gpu", type=int, default=125_000_000)
    ap.add_argument("--model", default=str(Path(__file__).resolve().parents[2] / "src/api/models/xgb_model_tree.pkl"))
    ap.add_argument("--chunk", type=int, default=1 << 22)
    ap.add_argument("--gen-chunk", type=int, default=25_000_000)
    ap.add_argument("--input", nargs="*", default=None, help="shard .npy files or globs (host/disk-resident path)")
    ap.add_argument("--output", default="batch_scores")
    ap.add_argument("--make-shards", default=None, help="write synthetic shards into this directory first")
    ap.add_argument("--rows", type=int, default=100_000_000, help="rows of --make-shards")
    ap.add_argument("--files", type=int, default=4, help="files of --make-shards")
    ap.add_argument("--host-chunk", type=int, default=1 << 20)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--stage-threads", type=int, default=8)
    ap.add_argument("--h2d-streams", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=1, help="timed passes over the input (host path)")
    ap.add_argument("--pinned-rows", type=int, default=0,
                    help="host-resident in pinned DRAM: score this many rows held in a pinned host tensor")
    a = ap.parse_args(argv)
    ctx = pdist.init_from_env()
    dev = torch.device("cuda", ctx.local_rank)
    torch.cuda.set_device(dev)
    _, b = load_pickle_bytes(Path(a.model).read_bytes())
    if a.make_shards:
        if ctx.rank == 0:
            make_shards(a.make_shards, a.rows, a.files, b.num_feature, device=dev)
        ctx.barrier()
        if not a.input:
            a.input = [str(Path(a.make_shards) / "shard_*.npy")]
    if a.pinned_rows:
        n = a.pinned_rows
        Xp = torch.empty((n, b.num_feature), dtype=torch.float32).pin_memory()
        for s0 in range(0, n, a.gen_chunk):
            e0 = min(n, s0 + a.gen_chunk)
            Xp[s0:e0] = synth.make_lendingclub(e0 - s0, seed=1, row_offset=ctx.rank * n + s0,
                                               device=dev)[0][:, : b.num_feature].cpu()
        sc = HostStreamScorer(b, min(a.host_chunk, n), b.num_feature, dev, slots=a.slots,
                              stage_threads=a.stage_threads, h2d_streams=a.h2d_streams)
        out = np.empty(n, dtype=np.float32)
        sc.score(Xp[: min(n, a.host_chunk)], out[: min(n, a.host_chunk)])  # warm-up
        ctx.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.repeat):
            sc.score(Xp, out)
        torch.cuda.synchronize(dev)
        ctx.barrier()
        dt = ctx.allreduce_scalar((time.perf_counter() - t0) / a.repeat, "max", dev)
        sc.close()
        if ctx.rank == 0:
            print(json.dumps({"metric": "batch scoring rows/s (host-resident, pinned DRAM)", "value": n * ctx.world / dt,
                              "per_gpu": n / dt, "n_gpus": ctx.world, "rows": n * ctx.world, "seconds": dt,
                              "host_chunk": a.host_chunk, "slots": a.slots, "h2d_streams": a.h2d_streams,
                              "mean_prob_rank0": float(out.mean())}))
        pdist.shutdown()
        return 0
    if a.input:
        paths = sorted(p for g in a.input for p in (glob.glob(g) or [g]))
        arrs = open_shards(paths)
        total = sum(len(x) for x in arrs)
        # warm-up: scorer construction (pinned buffers, graphs) + ONE chunk, in a directory of this
        # rank's own (ranks must not truncate / remap each other's warm-up file)
        wchunk = min(a.host_chunk, len(arrs[0]))
        score_files(b, [paths[0]], Path(a.output) / "_warm" / f"rank{ctx.rank}", 0, 1, dev, chunk=wchunk,
                    slots=a.slots, stage_threads=a.stage_threads, max_rows=wchunk)
        ctx.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.repeat):
            meta = score_files(b, paths, a.output, ctx.rank, ctx.world, dev, chunk=a.host_chunk, slots=a.slots,
                               stage_threads=a.stage_threads, h2d_streams=a.h2d_streams)
        torch.cuda.synchronize(dev)
        ctx.barrier()
        dt = ctx.allreduce_scalar((time.perf_counter() - t0) / a.repeat, "max", dev)
        if ctx.rank == 0:
            p0 = np.load(str(Path(a.output) / "scores_rank00000.npy"), mmap_mode="r", allow_pickle=False)
            print(json.dumps({"metric": "batch scoring rows/s (host/disk-resident shards)", "value": total / dt,
                              "per_gpu": total / dt / ctx.world, "n_gpus": ctx.world, "rows": total,
                              "seconds": dt, "files": len(paths), "host_chunk": a.host_chunk, "slots": a.slots,
                              "stage_threads": a.stage_threads, "h2d_streams": a.h2d_streams, "mean_prob_rank0": float(np.mean(p0[:10_000_000]))}))
        pdist.shutdown()
        return 0
    n = a.rows_per_gpu
    X = torch.empty((n, b.num_feature), dtype=torch.float32, device=dev)
    for s in range(0, n, a.gen_chunk):  # generate in pieces: bounded scratch memory
        e = min(n, s + a.gen_chunk)
        X[s:e] = synth.make_lendingclub(e - s, seed=1, row_offset=ctx.rank * n + s, device=dev)[0][:, : b.num_feature]
    out = torch.empty(n, dtype=torch.float32, device=dev)
    score_device_matrix(b, X[: min(n, a.chunk)], out[: min(n, a.chunk)], chunk=a.chunk)  # warm-up / graph
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    score_device_matrix(b, X, out, chunk=a.chunk)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    dt = ctx.allreduce_scalar(time.perf_counter() - t0, "max", dev)
    mean_p = ctx.allreduce_scalar(float(out.double().sum()), "sum", dev) / (n * ctx.world)
    if ctx.rank == 0:
        print(json.dumps({"metric": "batch scoring rows/s", "value": n * ctx.world / dt, "n_gpus": ctx.world,
                          "rows": n * ctx.world, "seconds": dt, "mean_prob": mean_p, "chunk": a.chunk}))
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
