#!/usr/bin/env python
"""Summarise a rocprofv3 kernel + memory-copy trace of the host-resident scoring pipeline: per-kind
totals, link throughput, and how much of the H2D copy time overlaps predictor kernels."""
import csv
import glob
import sys

root = sys.argv[1]
kt = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
mt = glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True)
kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for f in kt for r in csv.DictReader(open(f))]
cps = []
for f in mt:
    for r in csv.DictReader(open(f)):
        cps.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "?")),
                    int(r.get("Bytes", r.get("Size", 0)) or 0)))
pred = sorted((s, e) for s, e, n in kern if "predict" in n)
print(f"kernels: {len(kern)}  predictor launches: {len(pred)}  copies: {len(cps)}")
for kind in sorted({c[2] for c in cps}):
    sel = [c for c in cps if c[2] == kind]
    t = sum(e - s for s, e, _, _ in sel) / 1e9
    b = sum(c[3] for c in sel)
    big = [c for c in sel if c[3] >= 1 << 20]
    bt = sum(e - s for s, e, _, _ in big) / 1e9
    print(f"{kind:28s} n={len(sel):6d} bytes={b/1e9:8.3f} GB busy={t*1e3:9.2f} ms"
          + (f"  >=1MiB copies: {sum(c[3] for c in big)/max(bt,1e-12)/1e9:6.1f} GB/s" if big else ""))
if pred:
    pt = sum(e - s for s, e in pred) / 1e9
    span = (max(e for _, e in pred) - min(s for s, _ in pred)) / 1e9
    print(f"predictor busy {pt*1e3:.2f} ms over a {span*1e3:.2f} ms span")
    h2d = [(s, e) for s, e, k, b in cps if "HOST_TO_DEVICE" in k.upper() and b >= 1 << 20]
    ov = 0
    for s, e in h2d:
        for ps, pe in pred:
            ov += max(0, min(e, pe) - max(s, ps))
    tot = sum(e - s for s, e in h2d)
    if tot:
        print(f"H2D copy time overlapped with predictor kernels: {ov/tot*100:.1f}%")
    lo = min(min(s for s, _ in pred), min((s for s, _, _, _ in cps), default=1 << 62))
    hi = max(max(e for _, e in pred), max((e for _, e, _, _ in cps), default=0))
    print(f"pipeline span (first copy/kernel -> last): {(hi-lo)/1e6:.2f} ms")
