"""How the routing model's host-pool cap follows the host leg it is learned from (design
tool): c5-size (38 MB) host-leg batches on the pool, one after another, each call's time
beside the cap the model holds after it, and the cap the median call implies.

    python tools/learn_probe.py
"""
import ctypes
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from storm_amd import _lib, blocks, engine  # noqa: E402


def main():
    import torch
    torch.cuda.init()
    engine.init(0)
    L = _lib.lib
    n, stride = 1202, 32768
    lens = np.array([31808] * 1200 + [30000, 72], dtype=np.uint32)
    raw = np.zeros(n * stride + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    buf = raw[off:off + n * stride]
    buf[:] = np.random.default_rng(1).integers(0, 256, buf.size, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint64)
    bp, lp, op = buf.ctypes.data, lens.ctypes.data, out.ctypes.data
    hashed = int(lens.sum())
    threads = os.cpu_count()
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    for label, nt in (("pool", 0), ("1 thread", 1)):
        ts = []
        for k in range(60):
            t0 = time.perf_counter()
            _lib.check(L.stormck_checksum_host_leg(bp, stride, lp, 0, n, op, nt))
            dt = time.perf_counter() - t0
            ts.append(dt)
            r = blocks.RouteRates()
            if k % 6 == 0 or k == 59:
                print(f"{label:8s} call {k:2d}: {dt * 1e6:7.1f} us = {hashed / dt / 1e3:6.1f} GB/s   model: "
                      f"host_thread {r['host_thread']:8.0f}  host_cached {r['host_cached']:8.0f}", flush=True)
        med = statistics.median(ts)
        ts_s = sorted(ts)
        print(f"{label}: median {med * 1e6:.1f} us ({hashed / (med * 1e6 - (10 if nt != 1 else 0)) :.0f} B/us net of "
              f"fork/join), p10 {ts_s[6] * 1e6:.1f}, p90 {ts_s[54] * 1e6:.1f}, max {ts_s[-1] * 1e6:.1f} us", flush=True)
    print("threads visible", threads, ctypes.sizeof(ctypes.c_void_p))


if __name__ == "__main__":
    main()
