#!/usr/bin/env python
"""Headline benchmark: rows/s of GBDT training on 10M-row LendingClub-shaped data (+ AUC).

Metric and config come from BASELINE.json: "rows/sec GBDT train on 10M-row LendingClub-shaped
tabular; AUC parity", with the deployed hyper-parameters of the reference model (300 trees, depth 7,
eta 0.05, gamma 5, lambda 1, min_child_weight 1, max_bin 256, scale_pos_weight = neg/pos,
binary:logistic, 20 features). One step = one complete fit (quantile sketch + binning + 300
boosting rounds + model fetch), i.e. BASELINE.md's ``rows_per_s = N_train_rows / wall_seconds(fit)``.

Data: synthetic LendingClub-shaped rows (no dataset download is possible) generated on each GPU for
its own shard by global row index. Scaling mode "strong" (the default) keeps the BASELINE config's
10M GLOBAL rows and shards them over the ranks, so every N trains the same model on the same data
(BASELINE.json configs[2]: "10M-row GBDT data-parallel ... on 8xMI355X"). "weak" (opt-in,
``--scaling weak``) gives every rank a 10M-row shard instead (N x 10M global rows); its JSON line
says so in ``scaling`` and ``rows_global``. Strong scaling of a 300-tree x 7-level boosting run is
bounded by its 2,100 sequential level steps (each needs one histogram all-reduce under DP), see
docs/PERF.md.

Launch: ``python bench.py`` (1 GPU) or ``torchrun --nproc-per-node N bench.py --gpus N``.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
from cobalt_smart_lender_ai_amd.config import knob

BASELINE_ROWS_PER_S = None  # the reference publishes no throughput (BASELINE.json "published": {})

# AUC parity (within +-0.002 of a CPU histogram GBDT trained on the same synthetic rows with
# the same hyper-parameters). The reference of a configuration (training rows, trees, depth, seed, test
# rows -- the test AUC is on the next test_rows rows) is the host trainer (models/gbdt_host.py, NumPy,
# CPU) with EXACTLY the bench's config -- gamma 5, min_child_weight 1 on the hessian, lambda 1, 256 bins,
# every row sketched, spw = neg/pos -- run by scripts/parity_oracle.py (profiles/configs/parity-oracle-*.json):
# its 17-bit fixed-point trainer (the trees the GPU grows) and its unquantised float64 trainer. The
# independent cross-check is scikit-learn's HistGradientBoostingClassifier on the same rows
# (scripts/bench_configs.py cpu-hist-gbdt-10m), whose config differs (below).
_HOST_ORACLE = "cobalt host trainer (models/gbdt_host.py, NumPy, CPU), same config, scripts/parity_oracle.py"
_SKLEARN_XCHECK = {"engine": "sklearn HistGradientBoostingClassifier (16 threads; profiles/configs/cpu-hist-gbdt-10m.json)",
                   "config_differences": "no min_split_loss (gamma); min_samples_leaf=1 instead of min_child_weight=1 "
                                         "on the hessian; 255 value bins + a missing bin; its own quantile binning"}
PARITY_AUC = {
    (10_000_000, 300, 7, 0, 1_000_000): {"auc": 0.951044, "source": _HOST_ORACLE + ", 17-bit (the GPU's trees)",
                                         "fit_s": 6290.5, "exact_fp64_auc": 0.95104,
                                         "exact_fp64_source": _HOST_ORACLE + ", unquantised float64 gradients",
                                         "cross_check": dict(_SKLEARN_XCHECK, auc=0.95106),
                                         "records": "profiles/configs/parity-oracle-10000000_{17,fp64}.json"},
    (2_000_000, 300, 7, 0, 1_000_000): {"auc": 0.95069, "source": _HOST_ORACLE + ", 17-bit (the GPU's trees)",
                                        "fit_s": 1023.6},
    # (pinned by tests/test_parity_oracle.py on the CPU and tests/test_gpu_bench.py on the GPU)
    (100_000, 300, 7, 0, 100_000): {"auc": 0.945837, "source": _HOST_ORACLE + ", 17-bit (the GPU's trees)",
                                    "fit_s": 50.3},
}
PARITY_TOL = 0.002


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=10_000_000, help="training rows (global for strong scaling)")
    ap.add_argument("--test-rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=300)
    ap.add_argument("--depth", type=int, default=7)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--profile-fit", action="store_true", help="print per-phase timings to stderr")
    ap.add_argument("--sketch-rows", type=int, default=0,
                    help="rows of the quantile-sketch sample; 0 (default) = every row, the exact device sketch "
                         "(XGBoost hist's all-row semantics; csrc/sketch.hip)")
    ap.add_argument("--grad-bits", type=int, default=17, choices=[17, 25],
                    help="fixed-point gradient bits: 17 (packed u64 histogram cells, default) or 25 (int64 cells)")
    a = ap.parse_args()

    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc
    from cobalt_smart_lender_ai_amd.models import gbdt
    from cobalt_smart_lender_ai_amd.parallel import dist as pdist

    # COBALT_BENCH_SHARED_DEVICE=1: every rank on cuda:0 (the 1-GPU multi-process rehearsal); each rank
    # then launches on its own CU-masked share of the device (parallel/cumask.py)
    shared = knob("COBALT_BENCH_SHARED_DEVICE") == "1"
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if shared and torch.cuda.is_available():
        from cobalt_smart_lender_ai_amd.parallel import cumask

        torch.cuda.set_device(0)
        if cumask.want_shared_mask(env_world):
            torch.cuda.set_stream(cumask.shared_device_stream(int(os.environ.get("RANK", "0")), env_world,
                                                              torch.device("cuda", 0)))
    ctx = pdist.init_from_env()
    world, rank = ctx.world, ctx.rank
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev_index = 0 if shared else ctx.local_rank
    dev = torch.device("cuda", dev_index) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)

    n_global = a.rows if a.scaling == "strong" else a.rows * world
    start, end = pdist.shard_range(n_global, rank, world)
    X, y = synth.make_lendingclub(end - start, seed=a.seed, row_offset=start, device=dev)
    pos = ctx.allreduce_scalar(float(y.sum()), "sum", dev)
    spw = (n_global - pos) / pos
    params = gbdt.GBDTParams(n_estimators=a.trees, max_depth=a.depth, learning_rate=0.05, gamma=5.0,
                             reg_lambda=1.0, min_child_weight=1.0, max_bin=256, scale_pos_weight=spw,
                             random_state=78, sketch_rows=a.sketch_rows or None, grad_bits=a.grad_bits)

    def fit():
        rep = gbdt.FitReport(sync_phases=a.profile_fit)
        b = gbdt.train(X, y, params, device=dev, dist=ctx if world > 1 else None, n_rows_global=n_global,
                       row_offset=start, report=rep, feature_names=synth.FEATURES,
                       feature_types=synth.FEATURE_TYPES)
        return b, rep

    fallback = None
    for _ in range(a.warmup):
        diverged = False
        try:
            fit()
        except (gbdt.ReplicaDivergence, pdist.CollectiveTimeout) as e:
            # divergence: raised on every rank of the same fit (in-flight digest check); a timed-out
            # in-kernel exchange: every rank's deadline passes (the peers stop publishing), the group
            # is aborted and the GPU work drained
            if world == 1 or ctx.transport != "ipc":
                raise
            print(f"[bench] rank {rank}: {type(e).__name__}: {e}", file=sys.stderr)
            diverged = type(e).__name__
        # every rank agrees before acting on it, so the ranks' collectives stay in step
        if world > 1 and ctx.allreduce_scalar(1.0 if diverged else 0.0, "max", dev) > 0.5:
            fallback = f"ipc exchange failed in warm-up ({diverged or 'on a peer'}); RCCL"
            pdist.switch_transport(ctx, "rccl")
    ctx.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    reps = []
    booster = None
    for _ in range(a.steps):
        booster, rep = fit()
        reps.append(rep)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.allreduce_scalar(elapsed, "max", dev)

    # (outside the timed region) data parallel: every rank must hold the same model -- a 52-bit digest
    # of the last fit's UBJSON, compared by a min / max all-reduce
    replicas_agree = None
    if world > 1 and booster is not None:
        import hashlib

        h = float(int.from_bytes(hashlib.sha256(booster.save_raw("ubj")).digest()[:8], "little") >> 12)
        replicas_agree = ctx.allreduce_scalar(h, "min", dev) == ctx.allreduce_scalar(h, "max", dev)
        if not replicas_agree and rank == 0:
            print("[bench] ERROR: data-parallel ranks hold different models", file=sys.stderr)

    auc = None
    if rank == 0 and booster is not None:
        Xt, yt = synth.make_lendingclub(a.test_rows, seed=a.seed, row_offset=n_global, device=dev)
        p = booster.predict_proba(Xt, device=dev)
        auc = float(roc_auc(yt, p))
    parity = PARITY_AUC.get((n_global, a.trees, a.depth, a.seed, a.test_rows))
    parity_ref = parity["auc"] if parity else None
    auc_parity_ok = None if (auc is None or parity_ref is None) else abs(auc - parity_ref) <= PARITY_TOL
    if auc_parity_ok is False:
        print(f"[bench] WARNING: AUC {auc:.5f} drifted from the CPU reference {parity_ref:.5f} by more than "
              f"{PARITY_TOL}", file=sys.stderr)
    ms = elapsed / max(a.steps, 1) * 1e3
    value = n_global * a.steps / elapsed
    if a.profile_fit and rank == 0:
        for r in reps:
            print(f"[bench] sketch {r.t_sketch*1e3:.1f} ms  bin {r.t_bin*1e3:.1f} ms  boost {r.t_boost*1e3:.1f} ms"
                  f"  total {r.t_total*1e3:.1f} ms  phases "
                  + " ".join(f"{k}={v*1e3:.1f}" for k, v in r.phases.items()), file=sys.stderr)
    if rank == 0:
        out = {
            "metric": "rows/sec GBDT train on 10M-row LendingClub-shaped tabular; AUC parity",
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None if BASELINE_ROWS_PER_S is None else value / BASELINE_ROWS_PER_S,
            "dtype": "fp32",
            "precision": f"fp32 features; fp64 gradient math quantised to {a.grad_bits}-bit dithered (unbiased) fixed "
                         "point; exact int64 histogram sums; fp64 split gains",
            "data": "synthetic LendingClub-shaped (20 deployed features, 12.9% positives), generated on device",
            "config": {
                "model": f"GBDT binary:logistic, {a.trees} trees depth {a.depth} eta 0.05 gamma 5 lambda 1 max_bin 256 "
                         "spw=neg/pos",
                "global_batch": n_global,
                "rows_per_gpu": end - start,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "n_features": len(synth.FEATURES),
                "trees": a.trees,
                "max_depth": a.depth,
            },
            "rows_global": n_global,
            "sketch_rows": a.sketch_rows or "all",
            "dp_transport": ctx.transport if world > 1 else None,
            "dp_transport_fallback": fallback,
            # csrc/gbdt.hip node ownership: deep levels evaluated by the subtree's owner rank only
            "dp_node_ownership": (f"levels {max((world - 1).bit_length(), a.depth - 3)}-{a.depth - 1}"
                                  if world > 1 and ctx.transport == "ipc" and knob("COBALT_DP_OWNER", "1") != "0"
                                  and knob("COBALT_IPC_FUSED", "1") != "0" else None),
            "replica_check": "in-flight per-tree digest of every rank's split decisions" if world > 1 else None,
            "replicas_agree": replicas_agree,
            "auc": None if auc is None else round(auc, 5),
            "auc_parity_ref": parity_ref,
            "auc_parity_source": parity["source"] if parity else None,
            "auc_parity_ok": auc_parity_ok,
            "auc_parity_detail": {k: v for k, v in parity.items() if k not in ("auc", "source")} if parity else None,
            "test_rows": a.test_rows,
            "fit_breakdown_ms": {
                "sketch": round(sum(r.t_sketch for r in reps) / len(reps) * 1e3, 3),
                "bin": round(sum(r.t_bin for r in reps) / len(reps) * 1e3, 3),
                "boost": round(sum(r.t_boost for r in reps) / len(reps) * 1e3, 3),
            } if reps else None,
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
