"""The routed commit against the split it picks, on storm's c5 forest with one host thread
(design tool): the two called alternately on the same registered arena, medians of 40
each, then the same with torch's null-stream work and the caller's stream query in play.

    python tools/commit_pair_probe.py
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from storm_amd import _lib, blocks, engine  # noqa: E402
from storm_amd import commit as sc  # noqa: E402


def main():
    import torch
    torch.cuda.set_device(0)
    engine.init(0)
    L = _lib.lib
    b0, size, last = sc.pointer_forest(1200, 31808, 1200, slot=32768, revision=1)
    pages = (size + 4095) // 4096 * 4096
    raw = np.zeros(pages + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    arena = raw[off:off + pages]
    arena[:] = np.random.default_rng(2).integers(0, 256, arena.size, dtype=np.uint8)
    blocks.RegisterHostMemory(arena)
    ap = arena.ctypes.data
    hbm = torch.from_numpy(arena).to("cuda")  # torch work on the null stream, as in bench.py
    torch.cuda.synchronize()

    def one(kind, stream=None):
        b = b0.copy()
        out = np.zeros(len(b), dtype=np.uint64)
        la = ctypes.c_uint64(last)
        used, done = ctypes.c_uint32(0), ctypes.c_uint64(0)
        t0 = time.perf_counter()
        if kind == "routed_1":
            rc = L.stormck_commit(ap, b.ctypes.data, len(b), 1, ctypes.byref(la), out.ctypes.data, stream, 1,
                                  ctypes.byref(used))
        else:
            rc = L.stormck_commit_split(ap, b.ctypes.data, len(b), 1, ctypes.byref(la), out.ctypes.data, None, 0, 1,
                                        _lib.SPLIT_BALANCED, ctypes.byref(done))
        dt = time.perf_counter() - t0
        _lib.check(rc)
        return dt, used.value, done.value

    for k in range(3):
        one("routed_1")
        one("split_1")
    for label, stream in (("null stream", None), ("own stream", torch.cuda.Stream().cuda_stream)):
        res = {"routed_1": [], "split_1": []}
        legs, dones = set(), []
        for k in range(40):
            for kind in (("routed_1", "split_1") if k % 2 == 0 else ("split_1", "routed_1")):
                dt, used, done = one(kind, stream)
                res[kind].append(dt)
                if kind == "routed_1":
                    legs.add(used)
                else:
                    dones.append(done)
        med = {k: sorted(v)[len(v) // 2] * 1e6 for k, v in res.items()}
        print(f"{label}: routed_1 {med['routed_1']:.1f} us (legs {sorted(legs)})  split_1 {med['split_1']:.1f} us "
              f"(device leaves ~{int(np.median(dones))})  rates {blocks.RouteRates()}", flush=True)
    del hbm
    blocks.UnregisterHostMemory(arena)


if __name__ == "__main__":
    main()
