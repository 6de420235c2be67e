"""Probe (GPU box): one Merkle level at storm's fan-out, timed with HIP events, for the
level sizes of the c3 / c4 shard trees (16M and 8M leaves) and a 1M-leaf commit.
Run once per kernel: STORMCK_POINTER_RING=0 selects the register-quad k_pointer_level."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import _lib  # noqa: E402

if os.environ.get("MERKLE_PROBE_LIB"):  # A/B: a variant build of the library
    _lib.LIB_PATH = os.path.abspath(os.environ["MERKLE_PROBE_LIB"])
from storm_amd import engine  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.current_stream(dev)
kind = os.environ.get("MERKLE_PROBE_LIB", "") + " " + {"0": "register-quad", "1": "ring (1 wave)"}.get(os.environ.get("STORMCK_POINTER_RING", ""), "ring (wave pair)")
cs = torch.randint(-2**62, 2**62, (16 << 20,), dtype=torch.int64, device=dev)
par = torch.empty(16384, dtype=torch.int64, device=dev)
for m in (16 << 20, 8 << 20, 1 << 20, 300 * 1200, 12 * 1200, 1200):
    for _ in range(20):
        engine.pointer_level_device(cs.data_ptr(), m, 0, 1, 2, 1200, par.data_ptr(), st.cuda_stream)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = 50
        e0.record(st)
        for _ in range(k):
            engine.pointer_level_device(cs.data_ptr(), m, 0, 1, 2, 1200, par.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / k * 1e3)
    ts.sort()
    nodes = (m + 1199) // 1200
    print(f"{kind:14s} level of {m:>9} children ({nodes:>6} nodes): median {ts[2]:8.2f} us "
          f"(min {ts[0]:.2f}, max {ts[-1]:.2f}); child bytes {m * 8 / (ts[2] * 1e-6) / 1e9:.1f} GB/s", flush=True)
