#!/usr/bin/env python
"""Host-side bandwidth probe for the host-resident scoring path: multi-threaded np.copyto into a
pinned buffer, and preadv of a page-cached shard file into it (GB/s)."""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

path = sys.argv[1]
n_mb = 800
src = np.ones(n_mb << 18, dtype=np.float32)
dst_t = torch.empty(n_mb << 18, dtype=torch.float32).pin_memory()
dst = dst_t.numpy()
for th in (1, 4, 8, 16):
    pool = ThreadPoolExecutor(th)
    step = len(src) // th
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        list(pool.map(lambda i: np.copyto(dst[i:i + step], src[i:i + step]), range(0, len(src), step)))
        best = min(best, time.perf_counter() - t)
    print(f"copyto  threads={th:2d}  {n_mb / 1024 / best:6.1f} GB/s")
fd = os.open(path, os.O_RDONLY)
mv = memoryview(dst.view(np.uint8))
nb = len(mv)
for th in (1, 4, 8, 16):
    pool = ThreadPoolExecutor(th)
    step = nb // th
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        list(pool.map(lambda i: os.preadv(fd, [mv[i:i + step]], 128 + i), range(0, nb, step)))
        best = min(best, time.perf_counter() - t)
    print(f"preadv  threads={th:2d}  {n_mb / 1024 / best:6.1f} GB/s")
x = torch.empty(n_mb << 18, dtype=torch.float32, device="cuda")
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); x.copy_(dst_t, non_blocking=True); torch.cuda.synchronize()
print(f"H2D pinned single copy {n_mb / 1024 / (time.perf_counter() - t):6.1f} GB/s")
