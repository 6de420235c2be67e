"""Probe (GPU box): one c5-size host-memory batch (1,202 x 31,808 B in 32 KiB slots,
registered) through the host leg and the routed call, with STORMCK_TRACE=1 so the library
prints each pass (threads, blocks, microseconds): where the routed call's time goes."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from storm_amd import _lib, engine  # noqa: E402

engine.init(0)
L = _lib.lib
nb, blk = 1202, 32768
raw = np.zeros(nb * blk + 4096, dtype=np.uint8)
off = (-raw.ctypes.data) % 4096
a = raw[off:off + nb * blk]
a[:] = 5
_lib.check(L.stormck_host_register(a.ctypes.data, a.nbytes))
out = np.zeros(nb, dtype=np.uint64)
leg = ctypes.c_uint32()
for k in range(6):
    for name in ("host_leg", "routed"):
        t0 = time.perf_counter()
        if name == "host_leg":
            rc = L.stormck_checksum_host_leg(a.ctypes.data, blk, None, 31808, nb, out.ctypes.data, 0)
        else:
            rc = L.stormck_checksum_batch(a.ctypes.data, blk, None, 31808, nb, out.ctypes.data, 0, ctypes.byref(leg))
        dt = (time.perf_counter() - t0) * 1e6
        _lib.check(rc)
        print(f"{name} {dt:.1f} us leg {leg.value}", file=sys.stderr, flush=True)
r = _lib.RouteRates()
_lib.check(L.stormck_route_get_rates(ctypes.byref(r)))
print(r.as_dict(), file=sys.stderr)
_lib.check(L.stormck_host_unregister(a.ctypes.data))
