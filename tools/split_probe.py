"""Split-leg phase probe (design tool): one registered host batch hashed by the host pool
alone and by the split, N times each, with STORMCK_TRACE=1 so the library prints each
split's phases (worker start, first chunk issued / back, device end, host end) to stderr.

    STORMCK_TRACE=1 python tools/split_probe.py [blocks] [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from storm_amd import _lib, blocks, engine  # noqa: E402


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1202
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    torch.cuda.init()
    engine.init(0)
    stride = 32768
    raw = np.zeros(n * stride + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    buf = raw[off:off + n * stride]
    buf[:] = np.random.default_rng(1).integers(0, 256, size=buf.size, dtype=np.uint8)
    lens = np.full(n, 31808, dtype=np.uint32)
    blocks.RegisterHostMemory(buf)
    want = blocks.ChecksumBatchHost(buf, n, stride, lens=lens)
    res = {}
    for leg in ("host", "split", "split_fixed", "routed", "host"):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            if leg == "host":
                got = blocks.ChecksumBatchHost(buf, n, stride, lens=lens)
            elif leg == "split":
                got, done = blocks.ChecksumBatchSplit(buf, n, stride, lens=lens)
            elif leg == "split_fixed":
                got, done = blocks.ChecksumBatchSplit(buf, n, stride, lens=lens, device_blocks=max(1, n // 16))
            else:
                got, used = blocks.ChecksumBatchLeg(buf, n, stride, lens=lens)
            ts.append(time.perf_counter() - t0)
            assert np.array_equal(got, want)
        ts.sort()
        res[leg] = round(ts[len(ts) // 2] * 1e6, 1)
        print(leg, res[leg], "us", flush=True)
    print("rates", blocks.RouteRates(), flush=True)
    blocks.UnregisterHostMemory(buf)


if __name__ == "__main__":
    main()
