"""Probe: f1 level-0 chunk schedule (STORMCK_COMMIT_CHUNKS="first,growth") A/B'd in one
process on one arena, schedules interleaved per round (GPU box, repo root)."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import commit as sc  # noqa: E402
from storm_amd import engine  # noqa: E402

BLOCK, FANOUT, REV = 32768, 1200, 1
SCHED = ["32768,3", "32768,6", "32768,10", "16384,6", "16384,10", "65536,4", "1048576,1"]

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n = 1 << 20
b0, size, last = sc.pointer_forest(n, BLOCK, FANOUT, slot=BLOCK, revision=REV)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(arena.data_ptr() + BLOCK, BLOCK, n, 0, 0x53544F524D)
torch.cuda.synchronize()
out = np.zeros(len(b0), dtype=np.uint64)
ref = None
t_end = time.perf_counter() + 1.5
while time.perf_counter() < t_end:
    sc.commit_device(arena.data_ptr(), b0, REV, last, out=out)
res = {s: [] for s in SCHED}
for r in range(12):
    for s in SCHED:
        os.environ["STORMCK_COMMIT_CHUNKS"] = s
        sc.commit_device(arena.data_ptr(), b0, REV, last, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            sc.commit_device(arena.data_ptr(), b0, REV, last, out=out)
        torch.cuda.synchronize()
        res[s].append((time.perf_counter() - t0) / 3 * 1e3)
        if ref is None:
            ref = out.copy()
        elif not np.array_equal(out, ref):
            raise SystemExit(f"checksums differ under schedule {s}")
    print("round", r, flush=True)
for s in SCHED:
    v = res[s]
    print(f"{s:>12}  median {statistics.median(v):.3f} ms  min {min(v):.3f} ms", flush=True)
