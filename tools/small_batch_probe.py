"""Probe: device batches of uniform 32 KiB-slot blocks (31,808 B hashed, storm's
objectlist size). Default sizes 1, 16, 128 (k_xxh64_wide, one workgroup per block);
`python tools/small_batch_probe.py 1200 1600 2048 ...` for other sizes. us per launch,
back-to-back on one stream, HIP events, after a 1 s clock settle."""
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
sizes = [int(a) for a in sys.argv[1:]] or [1, 16, 128]
nmax = max(sizes)
buf = torch.empty((nmax, SLOT), dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(buf.data_ptr(), SLOT, nmax, 0, 0x53544F524D)
out = torch.empty(nmax, dtype=torch.int64, device=dev)
d_lens = 0
if os.environ.get("PROBE_LENS"):  # per-block lengths: storm's leaf / node sizes in turn
    mix = torch.tensor([31808, 30000, 32768, 28808], dtype=torch.int32)
    lens_t = mix.repeat(nmax // 4 + 1)[:nmax].to(dev)
    d_lens = lens_t.data_ptr()
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    engine.checksum_device(buf.data_ptr(), SLOT, nmax, out.data_ptr(), L, d_lens, st)
    torch.cuda.synchronize()
for n in sizes:
    k = 400
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        engine.checksum_device(buf.data_ptr(), SLOT, n, out.data_ptr(), L, d_lens, st)
    e1.record()
    torch.cuda.synchronize()
    print(f"n={n}: {e0.elapsed_time(e1) / k * 1e3:.1f} us")
