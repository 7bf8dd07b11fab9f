#!/usr/bin/env python
"""Full-scale preprocessing: pandas path vs the device-resident path (reference
src/data_preprocessing/clean_data.py:87-158 + feature_engineering.py:44-184 on the ~2.9M-row export).

A synthetic raw LendingClub export (``--rows`` x 143 columns, strings and all; dataio/synth_raw.py) is
written as CSV (not timed), then
  * pandas path:  pandas.read_csv -> clean_data_flow -> clean_lending_data -> feature_engineer (CPU);
  * device path:  pyarrow CSV reader -> DeviceFrame in HBM -> the same three stages on the GPU ->
                  the tree set's float32 matrix -> GBDT quantile sketch + binning (still in HBM).
Both produce identical frames (checked on the tree set); prints one JSON line."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def log(msg: str) -> None:
    print(f"[bench_prep] {msg}", file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_900_000)
    ap.add_argument("--cols", type=int, default=143)
    ap.add_argument("--csv", default="/tmp/cobalt_raw_full.csv")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--skip-pandas", action="store_true")
    a = ap.parse_args()

    import pandas as pd
    import pyarrow as pa
    import pyarrow.csv as pcsv
    import torch

    from cobalt_smart_lender_ai_amd.config import LEAKAGE_COLUMNS
    from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub
    from cobalt_smart_lender_ai_amd.models import gbdt
    from cobalt_smart_lender_ai_amd.prep import device_prep as dp
    from cobalt_smart_lender_ai_amd.prep.clean import clean_data_flow
    from cobalt_smart_lender_ai_amd.prep.features import clean_lending_data, feature_engineer_lending_data

    ref_date = "2025-07-04"
    t = time.perf_counter()
    raw = make_raw_lendingclub(a.rows, seed=0, n_cols=a.cols)
    shape = raw.shape
    pcsv.write_csv(pa.Table.from_pandas(raw, preserve_index=False), a.csv)
    del raw
    size_gb = Path(a.csv).stat().st_size / 1e9
    log(f"raw {shape} -> {a.csv} ({size_gb:.2f} GB) in {time.perf_counter() - t:.1f} s")

    dev = torch.device(a.device)
    res = dp.run_device_prep(a.csv, device=dev, reference_date=ref_date)  # warm-up (kernels, allocator)
    del res
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    res = dp.run_device_prep(a.csv, device=dev, reference_date=ref_date)
    tb = time.perf_counter()
    X, y, names = dp.tree_training_matrix(res["tree"], drop=[c for c in LEAKAGE_COLUMNS])
    bd = gbdt.bin_dataset(X, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_dev = time.perf_counter() - t0
    t_bins = time.perf_counter() - tb
    dtimes = {k: round(v, 3) for k, v in res["timings"].items()}
    log(f"device path {t_dev:.2f} s {dtimes} + matrix/binning {t_bins:.2f} s; tree {res['tree'].shape}")
    write = None
    if dev.type == "cuda":  # the artifact CSVs of the prep stages (clean_data.py / feature_engineering.py saves)
        from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes
        write = {}
        for key in ("clean", "tree", "nn"):
            tw = time.perf_counter()
            wt = {}
            blob = frame_to_csv_bytes(res[key], timings=wt)
            write[key + "_s"] = round(time.perf_counter() - tw, 3)
            write[key + "_mb"] = round(len(blob) / 1e6, 1)
            write[key + "_phases"] = {k: round(v, 3) for k, v in wt.items() if k.endswith("_s")}
        sub = res["tree"].take(torch.arange(res["tree"].n, device=dev) < res["tree"].n // 10)
        tw = time.perf_counter()
        pd_blob = sub.to_pandas().to_csv(index=False).encode()
        write["pandas_tree_10pct_s"] = round(time.perf_counter() - tw, 3)
        write["pandas_tree_10pct_equal"] = pd_blob == bytes(frame_to_csv_bytes(sub))
        log(f"GPU CSV write {write}")
    arrow_ingest = None
    if dev.type == "cuda":  # the host-parsed ingest it replaces (pyarrow C++ reader + uploads), for reference
        del res["clean"], res["stage2"]
        ta = time.perf_counter()
        from cobalt_smart_lender_ai_amd.prep.device_frame import DeviceFrame
        DeviceFrame.read_csv(a.csv, dev, engine="arrow")
        torch.cuda.synchronize(dev)
        arrow_ingest = round(time.perf_counter() - ta, 3)
        log(f"pyarrow ingest (previous engine) {arrow_ingest:.2f} s")

    out = {"metric": "preprocessing wall time, raw CSV -> tree/NN datasets (+ GBDT bins on device)",
           "raw_rows": shape[0], "raw_cols": shape[1], "csv_gb": round(size_gb, 3),
           "tree_shape": list(res["tree"].shape), "nn_shape": list(res["nn"].shape),
           "device_s": round(t_dev, 3), "device_stages_s": dtimes, "device_matrix_and_bins_s": round(t_bins, 3),
           "gbdt_features": len(names), "device": str(dev), "arrow_engine_ingest_s": arrow_ingest,
           "artifact_csv_write": write}
    if not a.skip_pandas:
        t0 = time.perf_counter()
        df = pd.read_csv(a.csv, low_memory=False, float_precision="round_trip")
        t1 = time.perf_counter()
        log(f"pandas read_csv {t1 - t0:.1f} s")
        c1 = clean_data_flow(df, device="cpu")
        t2 = time.perf_counter()
        log(f"pandas stage 1 {t2 - t1:.1f} s")
        c2 = clean_lending_data(c1, reference_date=ref_date, device="cpu")
        t3 = time.perf_counter()
        log(f"pandas stage 2 {t3 - t2:.1f} s")
        tree, nn = feature_engineer_lending_data(c2, device="cpu")
        t4 = time.perf_counter()
        log(f"pandas features {t4 - t3:.1f} s")
        sys.path.insert(0, str(ROOT / "tests"))
        from test_device_prep import assert_frames_equal

        assert_frames_equal(res["tree"].to_pandas(), tree)
        assert_frames_equal(res["nn"].to_pandas(), nn)
        out.update(pandas_s=round(t4 - t0, 3),
                   pandas_stages_s={"read_csv": round(t1 - t0, 3), "stage1": round(t2 - t1, 3),
                                    "stage2": round(t3 - t2, 3), "features": round(t4 - t3, 3)},
                   speedup=round((t4 - t0) / t_dev, 2), frames_equal=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
