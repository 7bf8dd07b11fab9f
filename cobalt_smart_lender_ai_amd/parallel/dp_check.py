"""Multi-process data-parallel harness: N rank processes train one GBDT on row shards and report the
model digest, so N-rank fits can be compared byte for byte with a 1-rank fit (and a dead rank's
peers can be shown to fail fast).

On a 1-GPU box every rank shares ``cuda:0``: the torch group is ``gloo`` (bootstrap / small
metadata) and the histogram all-reduce runs on the IPC one-shot group (``csrc/ipccomm.hip``), the
only GPU transport that accepts several processes on one device. On a multi-GPU node
``--one-gpu-per-rank`` gives rank r ``cuda:r`` (``--transport rccl`` for the RCCL A/B).

The parent process never touches HIP (ranks are spawned, and the results come back as JSON files),
so it can run inside a pytest session before other GPU tests initialise the runtime.

``python -m cobalt_smart_lender_ai_amd.parallel.dp_check --procs 2 --rows 300000``

(The reference has no distributed training; this is the multi-rank rehearsal of the DP design,
SURVEY.md §2.6 / §4 "Distributed tests".)
"""
from __future__ import annotations

import argparse
import hashlib
import json
import multiprocessing as mp
import os
import socket
import tempfile
import time
import traceback
from pathlib import Path
from ..config import knob

DEFAULT_PARAMS = dict(n_estimators=6, max_depth=7, learning_rate=0.1, gamma=1.0, subsample=0.9, colsample_bytree=0.8,
                      random_state=5, scale_pos_weight=6.0)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_main(rank: int, world: int, port: int, out_dir: str, rows: int, params: dict, transport: str,
              one_gpu_per_rank: bool, checkpoint_every: int, seed: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank if one_gpu_per_rank else 0), LOCAL_WORLD_SIZE=str(world))
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    if "{rank}" in knob("COBALT_STAMPS", ""):  # per-rank stamp files (diagnostics)
        os.environ["COBALT_STAMPS"] = knob("COBALT_STAMPS").replace("{rank}", str(rank))
    res: dict = {"rank": rank, "world": world, "ok": False}
    t0 = time.monotonic()
    ctx = None
    try:
        import torch

        from ..dataio import synth
        from ..models import gbdt
        from . import dist as pdist

        from . import cumask

        dev = torch.device("cuda", rank if one_gpu_per_rank else 0)
        torch.cuda.set_device(dev)
        stream = None
        if not one_gpu_per_rank and cumask.want_shared_mask(world):
            # ranks sharing the device each get their own 1/world of the CUs (see parallel/cumask.py)
            stream = cumask.shared_device_stream(rank, world, dev)
            res["cu_budget"] = int(knob("COBALT_CU_BUDGET"))
            if knob("COBALT_TEST_PLACEMENT") == "1":
                res["placement"] = cumask.placement(stream, dev)
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            if world > 1:
                backend = "nccl" if (one_gpu_per_rank and transport == "rccl") else "gloo"
                ctx = pdist.init_from_env(backend=backend, native=True, transport=transport)
                res["transport"] = ctx.transport
            s, e = pdist.shard_range(rows, rank, world)
            X, y = synth.make_lendingclub(e - s, seed=seed, row_offset=s, device=dev)
            ck = str(Path(out_dir) / "ckpt.ubj") if checkpoint_every else None
            t1 = time.monotonic()
            rep = gbdt.FitReport()
            b = gbdt.train(X, y, params, device=dev, dist=ctx, n_rows_global=rows, row_offset=s,
                           checkpoint_path=ck, checkpoint_every=checkpoint_every, resume=False, report=rep)
            torch.cuda.synchronize(dev)
            res["fit_s"] = time.monotonic() - t1
            res["plan"] = rep.extra.get("plan")
        raw = b.save_raw("ubj")
        res["model_sha256"] = hashlib.sha256(raw).hexdigest()
        res["trees"] = b.num_trees
        if ctx is not None and ctx.native_comm and ctx.transport == "ipc":
            from .. import _native
            import ctypes

            res["ipc_epochs"] = int(_native.lib().cobalt_ipc_epoch(ctypes.c_void_p(ctx.native_comm)))
        if rank == 0:
            (Path(out_dir) / "model.ubj").write_bytes(raw)
        res["ok"] = True
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        res["error"] = type(e).__name__
        res["message"] = str(e)[:2000]
        res["traceback"] = traceback.format_exc()[-4000:]
        if type(e).__name__ == "InjectedFault":
            # a crashed rank: no clean shutdown, the peers must notice on their own
            res["elapsed_s"] = time.monotonic() - t0
            (Path(out_dir) / f"rank{rank}.json").write_text(json.dumps(res))
            os._exit(3)
    res["elapsed_s"] = time.monotonic() - t0
    (Path(out_dir) / f"rank{rank}.json").write_text(json.dumps(res))
    try:
        from . import dist as pdist

        pdist.shutdown()
    except Exception:  # noqa: BLE001
        pass
    os._exit(0 if res["ok"] else 1)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def run(procs: int, rows: int = 300_000, params: dict | None = None, *, transport: str = "ipc",
        one_gpu_per_rank: bool = False, out_dir: str | None = None, timeout_s: float = 600,
        env: dict | None = None, checkpoint_every: int = 0, seed: int = 3) -> list[dict]:
    """Spawn ``procs`` ranks, wait (``timeout_s``), and return their result dicts (rank order).
    ``env`` is applied to the children (e.g. fault injection: ``COBALT_FAULT_AFTER_TREES``)."""
    params = dict(DEFAULT_PARAMS if params is None else params)
    out = out_dir or tempfile.mkdtemp(prefix="cobalt_dp_")
    ctx = mp.get_context("spawn")
    port = free_port()
    saved = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update({k: str(v) for k, v in (env or {}).items()})
    try:
        ps = [ctx.Process(target=rank_main, args=(r, procs, port, out, rows, params, transport, one_gpu_per_rank,
                                                  checkpoint_every, seed)) for r in range(procs)]
        for p in ps:
            p.start()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    deadline = time.monotonic() + timeout_s
    for p in ps:
        p.join(max(1.0, deadline - time.monotonic()))
    for p in ps:
        if p.is_alive():
            p.terminate()
            p.join(10)
            if p.is_alive():
                p.kill()
    results = []
    for r in range(procs):
        f = Path(out) / f"rank{r}.json"
        results.append(json.loads(f.read_text()) if f.exists() else {"rank": r, "ok": False, "error": "no result",
                                                                      "exitcode": ps[r].exitcode})
    # one progress line per multi-rank run (long GPU test sessions show they are alive)
    print(f"[dp_check] {procs} rank(s), {rows} rows: ok={[g.get('ok') for g in results]} "
          f"fit_s={[round(g.get('fit_s', -1), 2) for g in results]} plan={results[0].get('plan')}", flush=True)
    return results


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--rows", type=int, default=300_000)
    ap.add_argument("--trees", type=int, default=DEFAULT_PARAMS["n_estimators"])
    ap.add_argument("--transport", default="ipc", choices=["ipc", "rccl"])
    ap.add_argument("--one-gpu-per-rank", action="store_true")
    a = ap.parse_args(argv)
    params = dict(DEFAULT_PARAMS, n_estimators=a.trees)
    ref = run(1, a.rows, params)[0]
    got = run(a.procs, a.rows, params, transport=a.transport, one_gpu_per_rank=a.one_gpu_per_rank)
    same = all(g.get("model_sha256") == ref.get("model_sha256") for g in got)
    print(json.dumps({"reference": ref, "ranks": got, "identical": same}, indent=1))


if __name__ == "__main__":
    main()
