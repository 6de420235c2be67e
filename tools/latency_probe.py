"""Probe: latency-path kernels (GPU box, repo root). Single blocks.Checksum calls
(k_xxh64_single), small device batches (k_xxh64_wide, one workgroup per block), and
one top-of-tree Merkle level (k_pointer_level_wide), each timed back-to-back."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import blocks, engine  # noqa: E402

BLOCK = 32768
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.current_stream(dev)
rng = np.random.default_rng(7)
host = rng.integers(0, 256, size=65536, dtype=np.uint8)
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    blocks.Checksum(host[:BLOCK])
for size in (72, 4096, 30000, 31808, BLOCK, 65536):
    one = host[:size].copy()
    k = 3000
    t0 = time.perf_counter()
    for _ in range(k):
        blocks.Checksum(one)
    print(f"single call {size:>6} B: {(time.perf_counter() - t0) / k * 1e6:7.2f} us", flush=True)

arena = torch.empty((128, BLOCK), dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(arena.data_ptr(), BLOCK, 128, 0, 0x53544F524D, st.cuda_stream)
out = torch.empty(128, dtype=torch.int64, device=dev)
for n in (1, 16, 128):
    for _ in range(20):
        engine.checksum_device(arena.data_ptr(), BLOCK, n, out.data_ptr(), BLOCK, 0, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 500
    e0.record(st)
    for _ in range(k):
        engine.checksum_device(arena.data_ptr(), BLOCK, n, out.data_ptr(), BLOCK, 0, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    print(f"device batch n={n:>3}: {e0.elapsed_time(e1) / k * 1e3:7.2f} us per launch", flush=True)

cs = torch.randint(-2**62, 2**62, (1200 * 12,), dtype=torch.int64, device=dev)
par = torch.empty(12, dtype=torch.int64, device=dev)
for m in (1200, 1200 * 12):
    for _ in range(20):
        engine.pointer_level_device(cs.data_ptr(), m, 0, 1, 2, 1200, par.data_ptr(), st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 500
    e0.record(st)
    for _ in range(k):
        engine.pointer_level_device(cs.data_ptr(), m, 0, 1, 2, 1200, par.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    print(f"pointer level m={m:>6}: {e0.elapsed_time(e1) / k * 1e3:7.2f} us per launch", flush=True)
