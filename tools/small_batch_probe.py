"""Probe: device batches of 1, 16 and 128 uniform 32 KiB-slot blocks (31,808 B hashed,
storm's objectlist size), the k_xxh64_wide range (one workgroup per block). us per
launch, back-to-back on one stream, HIP events, after a 1 s clock settle."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import engine  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.current_stream(dev).cuda_stream
L, SLOT = 31808, 32768
buf = torch.empty((128, SLOT), dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(buf.data_ptr(), SLOT, 128, 0, 0x53544F524D)
out = torch.empty(128, dtype=torch.int64, device=dev)
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    engine.checksum_device(buf.data_ptr(), SLOT, 128, out.data_ptr(), L, 0, st)
    torch.cuda.synchronize()
for n in (1, 16, 128):
    k = 400
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        engine.checksum_device(buf.data_ptr(), SLOT, n, out.data_ptr(), L, 0, st)
    e1.record()
    torch.cuda.synchronize()
    print(f"n={n}: {e0.elapsed_time(e1) / k * 1e3:.1f} us")
