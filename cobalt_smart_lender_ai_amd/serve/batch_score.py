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
                        chunk: int = 1 << 22) -> torch.Tensor:
    """Probabilities of a device-resident [N, F] matrix.

    Row-contiguous fp32 input is scored in place: the predictor launches for every ``chunk`` rows run
    straight on views of X and ``out``, captured into one hipGraph and replayed once. (The earlier
    form staged each chunk into a GraphScorer's static buffer: a D2D copy per chunk plus the
    scorer's warm-up launch, ~10% of the 125M-row shard.) Other layouts go through a GraphScorer's
    static buffer chunk by chunk."""
    N, F = X.shape
    out = out if out is not None else torch.empty(N, dtype=torch.float32, device=X.device)
    if N == 0:
        return out
    if (X.dtype == torch.float32 and X.stride(1) == 1 and out.is_contiguous()
            and out.dtype == torch.float32 and out.device == X.device):
        predict_ops.gpu_forest(booster, X.device)  # pack + upload the forest outside the capture
        cur = torch.cuda.current_stream(X.device)
        side = torch.cuda.Stream(X.device)
        side.wait_stream(cur)  # X (and out) may still be in flight on the caller's stream
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            for s in range(0, N, chunk):
                e = min(N, s + chunk)
                predict_ops.predict_gpu(booster, X[s:e], None, out_prob=out[s:e])
        with torch.cuda.stream(side):
            graph.replay()
        side.synchronize()
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


def score_shard(booster: Booster, X_host: np.ndarray, chunk: int = 1 << 20, device=None) -> np.ndarray:
    """Host matrix -> probabilities with pinned double-buffered H2D copies overlapping the graphs."""
    dev = torch.device(device or "cuda")
    N, F = X_host.shape
    out = np.empty(N, dtype=np.float32)
    if N == 0:
        return out
    chunk = min(chunk, N)
    scorers = [GraphScorer(booster, chunk, F, dev) for _ in range(2)]
    pinned = [torch.empty((chunk, F), dtype=torch.float32).pin_memory() for _ in range(2)]
    res = [torch.empty(chunk, dtype=torch.float32).pin_memory() for _ in range(2)]
    pending: list[tuple[int, int, int]] = []
    Xh = np.ascontiguousarray(X_host, dtype=np.float32)
    # staging copies through NumPy views of the pinned buffers (np.copyto runs at memcpy speed;
    # Tensor.copy_ on CPU is far slower for a plain contiguous copy). Splitting the copy over 4-8
    # threads did not help on the MI355X box (156-178M rows/s vs 174M), so the copy is not the bound.
    pinned_np = [p.numpy() for p in pinned]
    for k, s in enumerate(range(0, N, chunk)):
        b = k & 1
        e = min(N, s + chunk)
        sc = scorers[b]
        sc.stream.synchronize()  # buffer b free again (its previous chunk is done)
        for (ps, pe, pb) in [p for p in pending if p[2] == b]:
            out[ps:pe] = res[pb][: pe - ps].numpy()
            pending.remove((ps, pe, pb))
        np.copyto(pinned_np[b][: e - s], Xh[s:e])
        with torch.cuda.stream(sc.stream):
            sc.x[: e - s].copy_(pinned[b][: e - s], non_blocking=True)
            if e - s < chunk:
                sc.x[e - s:].zero_()
        sc.run()
        with torch.cuda.stream(sc.stream):
            res[b][: e - s].copy_(sc.prob[: e - s], non_blocking=True)
        pending.append((s, e, b))
    for sc in scorers:
        sc.stream.synchronize()
    for (ps, pe, pb) in pending:
        out[ps:pe] = res[pb][: pe - ps].numpy()
    return out


def main(argv=None) -> int:
    """``python -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu N`` (torchrun for N GPUs):
    scores synthetic LendingClub-shaped rows generated on each GPU with the given (or shipped) model
    and prints one JSON line with the whole-job rows/s (max time over ranks)."""
    import argparse
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
    a = ap.parse_args(argv)
    ctx = pdist.init_from_env()
    dev = torch.device("cuda", ctx.local_rank)
    torch.cuda.set_device(dev)
    _, b = load_pickle_bytes(Path(a.model).read_bytes())
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
