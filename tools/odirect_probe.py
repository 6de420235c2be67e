"""Probe (GPU box): batched cold read + verify from an O_DIRECT descriptor
(stormck_read_verify_fd) at several reader-thread counts, random and address order,
into page-aligned registered slots. Also a raw O_DIRECT read of the same blocks with
a C-level thread pool (os.preadv releases the GIL), nothing verified."""
import mmap
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import blocks, engine  # noqa: E402

BLOCK = 32768
n = int(float(os.environ.get("ODIRECT_GIB", "8")) * 2**30) // BLOCK
import torch  # noqa: E402

dev = torch.device("cuda:0")
d = torch.empty((n, BLOCK), dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(d.data_ptr(), BLOCK, n, 0, 0x53544F524D)
cs = engine.checksum_tensor(d).cpu().numpy().view(np.uint64)
img = os.path.join(os.getcwd(), f"odirect_probe_{os.getpid()}.img")
mm = mmap.mmap(-1, n * BLOCK)
host = np.frombuffer(mm, dtype=np.uint8).reshape(n, BLOCK)
torch.from_numpy(host).copy_(d)
del d
torch.cuda.empty_cache()
fd = os.open(img, os.O_RDWR | os.O_CREAT | os.O_DIRECT, 0o600)
try:
    for off in range(0, n * BLOCK, 1 << 26):
        os.pwrite(fd, memoryview(mm)[off:off + (1 << 26)], off)
    os.fsync(fd)
    blocks.RegisterHostMemory(host)
    lens = np.full(n, BLOCK, dtype=np.uint32)
    for name, addrs in (("random", np.random.default_rng(2).permutation(n).astype(np.uint64)),
                        ("in order", np.arange(n, dtype=np.uint64))):
        exp = cs[addrs.astype(np.int64)]
        for threads in [int(t) for t in os.environ.get("ODIRECT_THREADS", "1,2,4,8,16,32,64").split(",")]:
            if threads:
                os.environ["STORMCK_READ_THREADS"] = str(threads)
            else:  # 0: the library's own choice
                os.environ.pop("STORMCK_READ_THREADS", None)
            best = 1e9
            for _ in range(2):
                t0 = time.perf_counter()
                r = blocks.ReadVerifyBatch(fd, addrs, lens, exp, host, BLOCK)
                best = min(best, time.perf_counter() - t0)
                assert r == (n, 0), r
            label = f"{threads:4d}" if threads else "auto"
            print(f"O_DIRECT read+verify, {name:8s}, {label} readers: {n * BLOCK / best / 2**30:6.2f} GiB/s",
                  flush=True)
    blocks.UnregisterHostMemory(host)
finally:
    os.close(fd)
    os.unlink(img)
