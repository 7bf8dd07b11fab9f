#!/usr/bin/env python
"""Per-kernel register / spill / occupancy table of a HIP source, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (cross-compiles for gfx950; no GPU needed).
usage: kernel_resources.py csrc/gbdt.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-c", src,
                    "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"remark: (?:.*?)(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]|"
                  r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
print(f"{'kernel':70s} {'VGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'scratch':>7s} {'occ':>4s} {'LDS':>6s}")
for c in rows:
    if pat and not pat.search(c["name"]):
        continue
    print(f"{c['name'][:70]:70s} {c.get('VGPRs','?'):>5s} {c.get('VGPRs Spill','?'):>6s} {c.get('SGPRs Spill','?'):>6s} "
          f"{c.get('ScratchSize','?'):>7s} {c.get('Occupancy','?'):>4s} {c.get('LDS Size','?'):>6s}")
