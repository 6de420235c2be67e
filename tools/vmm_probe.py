"""VMM arena diagnostics (round 4): a fresh process allocates arenas through
stormck_device_alloc_placed in a given sequence of (mode, chunk), fills each with the
synthetic generator, checksums it, compares with the oracle, reads the bytes back and
reports where they differ. Usage: python tools/vmm_probe.py mode:chunk [mode:chunk ...]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as o  # noqa: E402
from storm_amd import engine  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
n, stride = 12288, 32768
want_bytes = o.fill_synthetic(n, stride, 7)
want = o.checksum_batch(want_bytes, n, stride, stride, threads=16)
for spec in sys.argv[1:]:
    mode, chunk = (int(x) for x in spec.split(":"))
    ptr, mapped = engine.device_alloc_placed(n * stride, mode, chunk)
    engine.fill_synthetic_device(ptr, stride, n, 7, o.SYNTH_SEED)
    out = torch.empty(n, dtype=torch.int64, device="cuda:0")
    engine.checksum_device(ptr, stride, n, out.data_ptr(), stride)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    bad = np.nonzero(got != want)[0]
    host = np.empty(n * stride, dtype=np.uint8)
    rc = hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(host.nbytes), 2)
    diff = np.nonzero(host != want_bytes)[0]
    mb = sorted(set((diff // (1 << 20)).tolist()))
    print(f"{spec}: va 0x{ptr:x} chunk {mapped} bad blocks {bad.size} (first {bad[:4].tolist()}, last "
          f"{bad[-4:].tolist()}); memcpy rc {rc}, differing bytes {diff.size} in MiB {mb[:8]}..{mb[-4:] if mb else []}",
          flush=True)
    engine.device_free(ptr)
