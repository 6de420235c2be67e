"""Device-side rates of the split leg's chunk paths (design tool): the whole call given to
the device (fixed share = n), so the time is the device part's alone.

  batch  stormck_checksum_split on registered strided rows: claims below 32 MiB are read
         in place by the kernels, larger ones go through the copy engine;
  commit stormck_commit_split with every leaf on the device: the kernels gather the
         leaves in place at their arena offsets (one pointer block per 1,200 leaves stays
         on the host).

    python tools/split_rate_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from storm_amd import blocks, engine  # noqa: E402
from storm_amd import commit as sc  # noqa: E402


def med(f, reps=7):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    import torch
    torch.cuda.init()
    engine.init(0)
    blocks.SetRouteRates(None, freeze=True)
    stride = 32768
    for n in (128, 520, 1200, 2048, 4096, 8192, 16384):
        raw = np.zeros(n * stride + 4096, dtype=np.uint8)
        off = (-raw.ctypes.data) % 4096
        buf = raw[off:off + n * stride]
        buf[::4096] = 7
        lens = np.full(n, 31808, dtype=np.uint32)
        blocks.RegisterHostMemory(buf)
        t_b = med(lambda: blocks.ChecksumBatchSplit(buf, n, stride, lens=lens, device_blocks=n))
        blocks.UnregisterHostMemory(buf)
        b, size, last = sc.pointer_forest(n, 31808, 1200, slot=stride, revision=1)
        raw2 = np.zeros(size + 4096, dtype=np.uint8)
        off2 = (-raw2.ctypes.data) % 4096
        arena = raw2[off2:off2 + size]
        blocks.RegisterHostMemory(arena)
        t_c = med(lambda: sc.commit_split(arena, b.copy(), 1, last, device_leaves=n))
        t_h = med(lambda: sc.commit_host(arena, b.copy(), 1, last, threads=1))
        blocks.UnregisterHostMemory(arena)
        mb = n * 31808 / 1e6
        print(f"n={n:6d} {mb:8.1f} MB  batch split(device only) {t_b * 1e6:9.1f} us = {mb / t_b / 1e3:5.1f} GB/s"
              f"   commit split(device leaves) {t_c * 1e6:9.1f} us = {mb / t_c / 1e3:5.1f} GB/s"
              f"   commit host 1 thread {t_h * 1e6:9.1f} us", flush=True)
    blocks.SetRouteRates(None)


if __name__ == "__main__":
    main()
