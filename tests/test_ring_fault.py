"""A stalled ring kernel is a reported error, never a checksum.

The small-batch kernels (k_xxh64_wide_multi, k_commit_level_multi) stage blocks
through an LDS ring whose waits are bounded (kernels.h pipe_wait). A wait that
expires must not produce a value: in checksum mode it would land in a parent Pointer
(/root/reference/cache/trace.go:282,307) and in verify mode it would read as a match
(blocks/checksum.go:20-27). The debug knob STORMCK_DEBUG_STALL_CHUNK=2 makes one
stager wave of workgroup 0 never report chunk 2, so the chain's wait expires; every
entry point that can take a ring kernel must then fail loudly:

* host-synchronous calls (checksum / verify of host blocks, the f1 commit) return
  STORMCK_EHIP naming the kernel, and hand no checksums over;
* the asynchronous device call leaves the stalled workgroup's outputs unwritten and
  stormck_device_status() reports the fault (once; it is then cleared).

The knob is read once per process, so the stalled calls run in a child process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from oracle import oracle as o
from storm_amd import _lib, commit as sc, engine
L = _lib.lib
res = {}
dev = torch.device("cuda", 0)
engine.init(0)
n, B = 1200, 32768  # <= 5 per CU: k_xxh64_wide_multi, 5 blocks per workgroup, 8 chunks per block
host = o.fill_synthetic(n, B, 0)
want = o.checksum_batch(host, n, B, B, threads=8)

# 1. host batch: EHIP naming the kernel, the caller's output untouched
out = np.full(n, 0x5A5A5A5A5A5A5A5A, dtype=np.uint64)
rc = L.stormck_checksum_host(host.ctypes.data, B, None, B, n, out.ctypes.data)
res["host"] = [rc, _lib.last_error(), bool((out == 0x5A5A5A5A5A5A5A5A).all())]

# 2. host verify against the correct checksums: EHIP, not "no mismatch"
fb, nb = ctypes.c_uint64(7), ctypes.c_uint64(7)
rc = L.stormck_verify_host(host.ctypes.data, B, None, B, n, want.ctypes.data, ctypes.byref(fb), ctypes.byref(nb))
res["verify_host"] = [rc, _lib.last_error()]

# 3. device batch: async call succeeds, workgroup 0's blocks keep the sentinel, every
#    other block is right, and the status call reports the fault once
buf = torch.from_numpy(host.reshape(n, B)).to(dev)
d_out = torch.full((n,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
rc = L.stormck_checksum_device(buf.data_ptr(), B, None, B, n, d_out.data_ptr(), st)
rc2 = L.stormck_device_status(st)
msg2 = _lib.last_error()
rc3 = L.stormck_device_status(st)  # cleared after the report
got = d_out.cpu().numpy().view(np.uint64)
res["device"] = [rc, rc2, msg2, rc3, bool((got[:5] == 0x5A5A5A5A5A5A5A5A).all()), bool((got[5:] == want[5:]).all())]

# 4. device verify: the stalled workgroup reports no mismatch, the status call catches it
bad = want.copy()
bad[2] ^= 1  # a mismatch inside the stalled workgroup, which therefore goes unseen ...
bad[900] ^= 1  # ... and one outside it, which is reported
d_exp = torch.from_numpy(bad.view(np.int64)).to(dev)
d_res = torch.zeros(2, dtype=torch.int64, device=dev)
rc = L.stormck_verify_device(buf.data_ptr(), B, None, B, n, d_exp.data_ptr(), d_res.data_ptr(), st)
rc2 = L.stormck_device_status(st)
r = d_res.cpu().tolist()
res["verify_device"] = [rc, rc2, r]

# 5. f1 commit of storm's per-revision forest (1,200 leaves: k_commit_level_multi)
b, size, last = sc.pointer_forest(n, 31808, 1200, slot=B, revision=1)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
engine.fill_synthetic_device(arena.data_ptr() + B, B, n, 0, o.SYNTH_SEED)
torch.cuda.synchronize()
cs = np.zeros(len(b), dtype=np.uint64)
la = ctypes.c_uint64(last)
rc = L.stormck_commit_device(arena.data_ptr(), b.ctypes.data, len(b), 1, ctypes.byref(la), cs.ctypes.data, None)
res["commit"] = [rc, _lib.last_error()]

# 6. a batch that takes no ring kernel (one workgroup per block) is unaffected
small = 64
d_small = torch.zeros(small, dtype=torch.int64, device=dev)
rc = L.stormck_checksum_device(buf.data_ptr(), B, None, B, small, d_small.data_ptr(), st)
rc2 = L.stormck_device_status(st)
res["clean"] = [rc, rc2, bool((d_small.cpu().numpy().view(np.uint64) == want[:small]).all())]
print("RESULT " + json.dumps(res))
"""


def _child(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=200)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:]
    return json.loads(line[0][len("RESULT "):])


@pytest.mark.timeout(240)
def test_stalled_ring_kernel_fails_loudly():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    r = _child({"STORMCK_DEBUG_STALL_CHUNK": "2"})
    rc, msg, untouched = r["host"]
    assert rc == _lib.EHIP and "k_xxh64_wide_multi" in msg and "stalled" in msg, r["host"]
    assert untouched, "a stalled host batch handed checksums to the caller"
    rc, msg = r["verify_host"]
    assert rc == _lib.EHIP and "k_xxh64_wide_multi" in msg, r["verify_host"]
    rc, rc2, msg2, rc3, sentinel, rest = r["device"]
    assert rc == _lib.OK and rc2 == _lib.EHIP and "k_xxh64_wide_multi" in msg2 and rc3 == _lib.OK, r["device"]
    assert sentinel, "the stalled workgroup wrote checksums"
    assert rest, "the other workgroups' checksums are wrong"
    rc, rc2, res = r["verify_device"]
    assert rc == _lib.OK and rc2 == _lib.EHIP, r["verify_device"]
    assert res == [900, 1], res  # the mismatch in the stalled workgroup is the one not seen
    rc, msg = r["commit"]
    assert rc == _lib.EHIP and "k_commit_level_multi" in msg, r["commit"]
    assert r["clean"] == [_lib.OK, _lib.OK, True], r["clean"]


@pytest.mark.timeout(240)
def test_ring_kernels_report_no_fault_without_the_knob():
    """The same child without the knob: every call succeeds and is right."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    env = {k: v for k, v in os.environ.items() if k != "STORMCK_DEBUG_STALL_CHUNK"}
    r = _child({"STORMCK_DEBUG_STALL_CHUNK": "0"} if "STORMCK_DEBUG_STALL_CHUNK" in env else {})
    assert r["host"][0] == _lib.OK and not r["host"][2]
    assert r["verify_host"][0] == _lib.OK
    rc, rc2, _, rc3, sentinel, rest = r["device"]
    assert (rc, rc2, rc3, sentinel, rest) == (_lib.OK, _lib.OK, _lib.OK, False, True)
    assert r["verify_device"] == [_lib.OK, _lib.OK, [2, 2]]
    assert r["commit"][0] == _lib.OK
    assert r["clean"] == [_lib.OK, _lib.OK, True]
