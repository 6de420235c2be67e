"""End-to-end host-memory checksum rate (H2D + kernel + D2H), for DESIGN.md.

storm's blocks live in host memory (cache.data backed by pkg/memdev / pkg/filedev,
/root/reference/cache/cache.go:36-40), so a drop-in call starts and ends there.
Measures blocks.ChecksumBatchGPU (the device leg of ChecksumBatch) over a host buffer of synthetic 32 KiB blocks:
  * pageable memory (library stages through pinned buffers with parallel memcpy)
  * registered memory (stormck_host_register: DMA straight from the caller's pages)
and, for reference, the raw pinned H2D copy rate. Results are checked bit-exact
against the device-resident path on the same blocks.

    python tools/e2e_bench.py [--gib 8] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOCK = 32768


def aligned_empty(nbytes: int, align: int = 1 << 21):
    """uint8 array whose data starts on an `align` boundary. Kernels reading host memory
    in place need 256-byte aligned rows to run at the PCIe link rate (38 GiB/s at
    +16 B vs 51 GiB/s aligned, profiles/r01_probe_host_gather.txt); numpy only aligns
    to 16 B. storm's cache.data, a large Go allocation, is page-aligned."""
    import numpy as np
    raw = np.empty(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from storm_amd import _lib, blocks, engine

    dev = torch.device("cuda:0")
    n = int(a.gib * 2**30) // BLOCK
    d = torch.empty((n, BLOCK), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(d.data_ptr(), BLOCK, n, 0, 0x53544F524D)
    ref = engine.checksum_tensor(d)
    torch.cuda.synchronize()
    host = aligned_empty(n * BLOCK).reshape(n, BLOCK)
    torch.from_numpy(host).copy_(d)
    want = ref.cpu().numpy().view(np.uint64)
    del d
    torch.cuda.empty_cache()

    def timed(fn):
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            best = min(best, time.perf_counter() - t0)
        return best, out

    res = {"blocks": n, "block_bytes": BLOCK, "gib": round(n * BLOCK / 2**30, 3)}
    blocks.ChecksumBatchGPU(host[:64], 64, BLOCK, length=BLOCK)  # warm the context / staging
    t, out = timed(lambda: blocks.ChecksumBatchGPU(host, n, BLOCK, length=BLOCK))
    assert np.array_equal(out, want), "pageable host path mismatch"
    res["pageable_gib_s"] = round(n * BLOCK / t / 2**30, 2)

    _lib.check(_lib.lib.stormck_host_register(host.ctypes.data, host.nbytes))
    try:
        t, out = timed(lambda: blocks.ChecksumBatchGPU(host, n, BLOCK, length=BLOCK))
        assert np.array_equal(out, want), "registered host path mismatch"
        res["registered_gib_s"] = round(n * BLOCK / t / 2**30, 2)
        # raw H2D copy of the same registered bytes, 256 MiB chunks, for reference
        buf = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        chunk = 256 << 20
        flat = torch.from_numpy(host.reshape(-1))

        def h2d():
            for off in range(0, host.nbytes, chunk):
                m = min(chunk, host.nbytes - off)
                buf[:m].copy_(flat[off:off + m], non_blocking=True)
            torch.cuda.synchronize()

        t, _ = timed(h2d)
        res["raw_h2d_registered_gib_s"] = round(host.nbytes / t / 2**30, 2)
    finally:
        _lib.check(_lib.lib.stormck_host_unregister(host.ctypes.data))
    # f2/f3: batched cold read + verify from a file device (page-cache resident image,
    # storm's filedev), blocks read in a random address order into cache slots
    import tempfile
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), suffix=".img") as f:
        host.tofile(f.name)
        fd = os.open(f.name, os.O_RDONLY)
        try:
            addrs = np.random.default_rng(1).permutation(n).astype(np.uint64)
            lens = np.full(n, BLOCK, dtype=np.uint32)
            exp = want[addrs.astype(np.int64)]
            slots = np.empty((n, BLOCK), dtype=np.uint8)
            blocks.ReadVerifyBatch(fd, addrs[:256], lens[:256], exp[:256], slots, BLOCK)  # warm
            t, r = timed(lambda: blocks.ReadVerifyBatch(fd, addrs, lens, exp, slots, BLOCK))
            assert r == (n, 0), r
            res["read_verify_file_random_gib_s"] = round(n * BLOCK / t / 2**30, 2)
            res["read_verify_note"] = "parallel pread (16 threads) from page cache on a reader thread, 1 GiB ahead of the pipelined H2D + verify"
        finally:
            os.close(fd)
    # f3 cold read from storage: the same image opened with O_DIRECT (no page cache),
    # read into page-aligned registered slots (full blocks, no staging copy), random
    # block order and in address order (runs of consecutive blocks: one pread per MiB)
    import mmap
    img = os.path.join(os.environ.get("E2E_IMAGE_DIR", os.getcwd()), f"e2e_odirect_{os.getpid()}.img")
    host.tofile(img)
    mm = mmap.mmap(-1, n * BLOCK)
    slots_d = np.frombuffer(mm, dtype=np.uint8).reshape(n, BLOCK)
    blocks.RegisterHostMemory(slots_d)
    try:
        fd = os.open(img, os.O_RDONLY | os.O_DIRECT)
        try:
            lens = np.full(n, BLOCK, dtype=np.uint32)
            for name, addrs in (("random", np.random.default_rng(2).permutation(n).astype(np.uint64)),
                                ("sequential", np.arange(n, dtype=np.uint64))):
                exp = want[addrs.astype(np.int64)]
                blocks.ReadVerifyBatch(fd, addrs[:256], lens[:256], exp[:256], slots_d, BLOCK)  # warm
                t, r = timed(lambda: blocks.ReadVerifyBatch(fd, addrs, lens, exp, slots_d, BLOCK))
                assert r == (n, 0), r
                res[f"read_verify_odirect_{name}_gib_s"] = round(n * BLOCK / t / 2**30, 2)
            # the storage alone: the same O_DIRECT reads with nothing verified (32 threads)
            import concurrent.futures as cf
            order = np.random.default_rng(3).permutation(n)

            def raw_read(part):
                for i in part:
                    os.preadv(fd, [memoryview(mm)[int(i) * BLOCK:(int(i) + 1) * BLOCK]], int(order[i]) * BLOCK)

            parts = np.array_split(np.arange(n), 32)
            t0 = time.perf_counter()
            with cf.ThreadPoolExecutor(32) as ex:
                list(ex.map(raw_read, parts))
            res["raw_odirect_random_read_gib_s"] = round(n * BLOCK / (time.perf_counter() - t0) / 2**30, 2)
            res["odirect_note"] = ("image file on " + os.path.dirname(img) + "; see profiles/*fs_probe.txt for the "
                                   "filesystem (overlay); O_DIRECT bypasses the page cache")
        finally:
            os.close(fd)
    finally:
        blocks.UnregisterHostMemory(slots_d)
        os.unlink(img)
    # f1 commit on a registered HOST arena (storm's cache.data in place, kernels over
    # PCIe via stormck_host_device_pointer), and the zero-copy device-entry hash rate
    from storm_amd import commit as sc
    nl = 32768
    bf, size, last = sc.pointer_forest(nl, BLOCK, 1200, slot=BLOCK, revision=1)
    arena = aligned_empty(size)
    arena[:] = 0
    arena[BLOCK:BLOCK + nl * BLOCK] = host[:nl].reshape(-1) if nl <= n else 0
    blocks.RegisterHostMemory(arena)
    try:
        d_arena = blocks.HostDevicePointer(arena)
        sc.commit_device(d_arena, bf, 1, last)  # warm
        t, (cs, _) = timed(lambda: sc.commit_device(d_arena, bf, 1, last))
        res["commit_registered_host_arena_gib_s"] = round(int(bf["length"].sum()) / t / 2**30, 2)
        res["commit_registered_host_arena_ms"] = round(t * 1e3, 2)
        o1 = torch.empty(nl, dtype=torch.int64, device=dev)

        def zc():
            engine.checksum_device(d_arena + BLOCK, BLOCK, nl, o1.data_ptr(), BLOCK)
            torch.cuda.synchronize()

        t, _ = timed(zc)
        res["zero_copy_device_entry_gib_s"] = round(nl * BLOCK / t / 2**30, 2)
        assert np.array_equal(o1.cpu().numpy().view(np.uint64), want[:nl]), "zero-copy hash mismatch"
        assert np.array_equal(cs[:nl], want[:nl]), "host-arena commit mismatch"
    finally:
        blocks.UnregisterHostMemory(arena)
    # single-call latency (blocks.Checksum on one buffer: <= 64 KiB is one launch that
    # reads pinned staging over PCIe and writes the checksum to pinned memory)
    for size in (0, 72, 4096, 30000, BLOCK, 65536):
        one = host[0, :size].copy()
        blocks.Checksum(one)
        k = 2000
        t0 = time.perf_counter()
        for _ in range(k):
            blocks.Checksum(one)
        res[f"single_call_us_{size}B"] = round((time.perf_counter() - t0) / k * 1e6, 2)
    # the same hash with the block already in HBM, one block per launch, back-to-back
    # launches timed by events: the serial XXH64 chain of one block on one quad of lanes
    d1 = torch.from_numpy(host[0].copy()).to(dev)
    o1 = torch.empty(1, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for size in (72, BLOCK):
        engine.checksum_device(d1.data_ptr(), BLOCK, 1, o1.data_ptr(), size, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            engine.checksum_device(d1.data_ptr(), BLOCK, 1, o1.data_ptr(), size, stream=st)
        e1.record()
        torch.cuda.synchronize()
        res[f"device_one_block_us_{size}B"] = round(e0.elapsed_time(e1) / 200 * 1e3, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
