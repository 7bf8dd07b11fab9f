#!/usr/bin/env python
"""GPU CSV ingest timing on a synthetic raw LendingClub export: per-phase and slowest columns."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cobalt_smart_lender_ai_amd.dataio.synth_raw import make_raw_lendingclub  # noqa: E402
from cobalt_smart_lender_ai_amd.prep.device_frame import DeviceFrame  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1_000_000
path = "/tmp/cobalt_csv_probe.csv"
if not Path(path).exists():
    import pyarrow as pa
    import pyarrow.csv as pcsv
    pcsv.write_csv(pa.Table.from_pandas(make_raw_lendingclub(n, seed=0, n_cols=143), preserve_index=False), path)
for rep in range(2):
    t = {}
    t0 = time.perf_counter()
    DeviceFrame.read_csv(path, "cuda", engine="gpu", timings=t)
    torch.cuda.synchronize()
    print(f"gpu ingest {time.perf_counter() - t0:.3f} s", {k: (round(v, 4) if isinstance(v, float) else v)
                                                           for k, v in t.items() if k != "column_times"}, flush=True)
for ct in t.get("column_times", []):
    print(f"  {ct[0]*1e3:8.1f} ms  {ct[1]:30s} kind={ct[2]} vocab={ct[3]}")
fr = DeviceFrame.read_csv(path, "cuda", engine="gpu")
from cobalt_smart_lender_ai_amd.prep.csv_gpu import frame_to_csv_bytes  # noqa: E402

for rep in range(2):
    wt = {}
    t0 = time.perf_counter()
    blob = frame_to_csv_bytes(fr, timings=wt)
    print(f"gpu write {time.perf_counter() - t0:.3f} s {len(blob) / 1e6:.1f} MB",
          {k: round(v, 4) for k, v in wt.items() if k.endswith("_s")}, flush=True)
if "--no-arrow" not in sys.argv:
    t0 = time.perf_counter()
    DeviceFrame.read_csv(path, "cuda", engine="arrow")
    torch.cuda.synchronize()
    print(f"arrow ingest {time.perf_counter() - t0:.3f} s")
