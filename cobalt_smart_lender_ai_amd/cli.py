"""Command-line entry point: ``python -m cobalt_smart_lender_ai_amd <command>``.

Commands mirror the reference's scripts:

  synth     write a synthetic LendingClub-shaped raw CSV into the store (offline stand-in for the
            Kaggle download, reference README "Data" section)
  clean     stage 1 (clean_data.py; ``--full`` = ``python clean_data.py full``)
  features  stage 2 (feature_engineering.py)
  train     tree model training (model_tree_train_test.py)
  train-nn  NN challenger (notebook 04 cells 31-44)
  serve     FastAPI scoring service (cobalt_fast_api.py, uvicorn)
  dictionary  descriptions of columns from the LendingClub data dictionary workbook (LCDataDictionary.xlsx)

The artifact store is ``--store`` or ``$COBALT_ARTIFACT_URI`` (a local directory or ``s3://bucket``).
"""
from __future__ import annotations

import argparse
import json
import logging
import sys
from .config import knob


def _store(args):
    from .dataio.artifacts import get_store

    return get_store(args.store)


def cmd_synth(args) -> int:
    from .config import RAW_DATA_KEY_FULL, RAW_DATA_KEY_SAMPLE
    from .dataio.synth_raw import make_raw_lendingclub

    st = _store(args)
    df = make_raw_lendingclub(args.rows, seed=args.seed)
    st.write_csv(df, RAW_DATA_KEY_FULL if args.full else RAW_DATA_KEY_SAMPLE)
    if args.both:
        st.write_csv(df, RAW_DATA_KEY_SAMPLE if args.full else RAW_DATA_KEY_FULL)
    print(f"[INFO] wrote {len(df)} synthetic raw rows")
    return 0


def cmd_clean(args) -> int:
    from .pipeline.prep_flow import run_clean

    run_clean(_store(args), use_sample=not args.full, device=args.device, preset=args.preset, engine=args.engine)
    return 0


def cmd_features(args) -> int:
    from .pipeline.prep_flow import run_features

    run_features(_store(args), device=args.device, reference_date=args.reference_date, engine=args.engine)
    return 0


def cmd_train(args) -> int:
    from .config import TrainConfig
    from .pipeline.train_tree import run_training

    st = _store(args)
    cfg = TrainConfig(device=args.device)
    if args.n_iter is not None:
        cfg.search_n_iter = args.n_iter
    if args.gpus is not None:
        cfg.fits_in_parallel = args.gpus
    from .parallel.taskpool import GpuTaskPool, resolve_workers

    # the search's worker processes are spawned first, before this process touches the GPU
    nw = resolve_workers(cfg.fits_in_parallel)
    pool = GpuTaskPool(nw) if nw > 1 else None
    try:
        from .pipeline.prep_flow import read_table

        df = read_table(st, cfg.input_key, args.device)
        m = run_training(df, cfg, store=st, local_dir=args.local_dir, device=args.device, pool=pool)
    finally:
        if pool is not None:
            pool.close()
    print(json.dumps({k: m[k] for k in ("auc", "best_params", "timing_s", "selected_features")}, indent=2))
    return 0


def cmd_train_nn(args) -> int:
    from .config import CLEAN_DATA_KEY_NN
    from .nn.mlp import MLPConfig
    from .pipeline.train_nn import NNTrainConfig, run_nn_training

    st = _store(args)
    cfg = NNTrainConfig(reproduce_reference=not args.use_smote, mlp=MLPConfig(epochs=args.epochs))
    from .pipeline.prep_flow import read_table

    m = run_nn_training(read_table(st, CLEAN_DATA_KEY_NN, args.device), cfg, store=st, local_dir=args.local_dir,
                        device=args.device)
    print(json.dumps({k: m[k] for k in ("auc", "auc_thresholded", "selected_features", "train_seconds")}, indent=2))
    return 0


def cmd_serve(args) -> int:
    import os
    import subprocess
    import sys
    import tempfile

    import uvicorn

    # One Python event loop tops out near ~1.7k requests/s on HTTP parsing and validation. With
    # --workers N > 1 the N uvicorn workers stay CPU-only and forward rows to ONE scorer process that
    # owns the GPU (serve/scorer.py): one engine, one set of hipGraphs, and micro-batches that pool the
    # requests of every worker.
    scorer = None
    if args.workers > 1 and not knob("COBALT_SCORER_SOCKET"):
        sock = os.path.join(tempfile.mkdtemp(prefix="cobalt_scorer_"), "scorer.sock")
        cmd = [sys.executable, "-m", "cobalt_smart_lender_ai_amd.serve.scorer", "--socket", sock]
        if args.device:
            cmd += ["--device", args.device]
        scorer = subprocess.Popen(cmd)
        os.environ["COBALT_SCORER_SOCKET"] = sock  # inherited by the spawned workers
    try:
        if args.workers > 1:
            from .serve.workers import run_workers  # SO_REUSEPORT workers (see there: TCP_NODELAY)

            return run_workers(args.host, args.port, args.workers, args.log_level)
        uvicorn.run("cobalt_smart_lender_ai_amd.serve.app:create_app", factory=True, host=args.host,
                    port=args.port, log_level=args.log_level)
    finally:
        if scorer is not None:
            scorer.terminate()
            scorer.wait(timeout=30)
    return 0


def cmd_dvc(args) -> int:
    """DVC-compatible versioning of raw data files (dataio/dvc.py): add / status / push / pull."""
    from .dataio import dvc

    st = _store(args)
    for target in args.targets:
        if args.action == "add":
            print(dvc.add(target))
        elif args.action == "status":
            for p, s in dvc.status(target).items():
                print(f"{s}\t{p}")
        elif args.action == "push":
            print("\n".join(dvc.push(target, st, prefix=args.prefix)))
        else:
            print("\n".join(str(p) for p in dvc.pull(target, st, prefix=args.prefix)))
    return 0


def cmd_dictionary(args) -> int:
    from .dataio import dictionary, synth

    dd = dictionary.load_data_dictionary(args.xlsx)
    cols = args.columns or synth.FEATURES
    for c, desc in dictionary.describe_columns(cols, dd).items():
        print(f"{c}\t{desc}")
    return 0


def main(argv: list[str] | None = None) -> int:
    logging.basicConfig(level=logging.INFO, format="[%(levelname)s] %(message)s")
    p = argparse.ArgumentParser(prog="cobalt_smart_lender_ai_amd")
    p.add_argument("--store", default=None, help="artifact store (dir or s3://bucket)")
    p.add_argument("--device", default=None, help="cuda:N or cpu (default: cuda:0 when available)")
    sub = p.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("synth")
    s.add_argument("--rows", type=int, default=100_000)
    s.add_argument("--seed", type=int, default=0)
    s.add_argument("--full", action="store_true")
    s.add_argument("--both", action="store_true", help="write the same frame under sample and full keys")
    s.set_defaults(fn=cmd_synth)
    s = sub.add_parser("clean")
    s.add_argument("--full", action="store_true")
    s.add_argument("--preset", default="script", choices=["script", "notebook"])
    s.add_argument("--engine", default=None, choices=["device", "pandas"],
                   help="device-resident frame (default on a GPU) or the pandas path")
    s.set_defaults(fn=cmd_clean)
    s = sub.add_parser("features")
    s.add_argument("--reference-date", default=None)
    s.add_argument("--engine", default=None, choices=["device", "pandas"])
    s.set_defaults(fn=cmd_features)
    s = sub.add_parser("train")
    s.add_argument("--local-dir", default="models")
    s.add_argument("--n-iter", type=int, default=None)
    s.add_argument("--gpus", type=int, default=None)
    s.set_defaults(fn=cmd_train)
    s = sub.add_parser("train-nn")
    s.add_argument("--local-dir", default="models")
    s.add_argument("--epochs", type=int, default=50)
    s.add_argument("--use-smote", action="store_true", help="train on the SMOTE-resampled, scaled rows")
    s.set_defaults(fn=cmd_train_nn)
    s = sub.add_parser("serve")
    s.add_argument("--host", default="0.0.0.0")
    s.add_argument("--port", type=int, default=8000)
    s.add_argument("--workers", type=int, default=int(__import__("os").environ.get("COBALT_SERVE_WORKERS", "1")))
    s.add_argument("--log-level", default="info")
    s.set_defaults(fn=cmd_serve)
    s = sub.add_parser("dvc", help="DVC-compatible data versioning: add | status | push | pull")
    s.add_argument("action", choices=["add", "status", "push", "pull"])
    s.add_argument("targets", nargs="+", help="data files (add) or .dvc pointers")
    s.add_argument("--prefix", default="dataset/", help="remote key prefix (the reference's DVC remote path)")
    s.set_defaults(fn=cmd_dvc)
    s = sub.add_parser("dictionary", help="column descriptions (default: the 20 deployed model features)")
    s.add_argument("--xlsx", required=True, help="path to LCDataDictionary.xlsx")
    s.add_argument("columns", nargs="*")
    s.set_defaults(fn=cmd_dictionary)
    args = p.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
