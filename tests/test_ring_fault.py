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
  stormck_device_status() reports the fault (once; it is then cleared); a device
  verify counts the stalled workgroup's blocks as mismatches (fails closed).

Faults are per stream: with STORMCK_DEBUG_STALL_STREAM only one stream's launches
stall, and a caller on another stream (device, host or verify calls, from another
thread, in either order) sees no fault and gets correct checksums, while the stalled
caller still gets STORMCK_EHIP from its own status check.

The knobs are read once per process, so the stalled calls run in a child process."""
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

# 4. device verify: the stalled workgroup counts as 5 mismatches (fails closed), and the
#    status call reports the fault
bad = want.copy()
bad[2] ^= 1  # a mismatch inside the stalled workgroup (whose 5 blocks all count as bad) ...
bad[900] ^= 1  # ... and one outside it
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
    assert res == [0, 6], res  # the stalled workgroup's 5 blocks fail closed, plus block 900
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


CHILD_STREAMS = r"""
import ctypes, json, os, sys, threading
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from oracle import oracle as o
from storm_amd import _lib, engine
L = _lib.lib
dev = torch.device("cuda", 0)
engine.init(0)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
# only stream A's ring launches stall (read at the first ring launch of the process)
os.environ["STORMCK_DEBUG_STALL_CHUNK"] = "2"
os.environ["STORMCK_DEBUG_STALL_STREAM"] = str(sa.cuda_stream)
n, B = 1200, 32768  # k_xxh64_wide_multi
host = o.fill_synthetic(n, B, 0)
want = o.checksum_batch(host, n, B, B, threads=8)
buf = torch.from_numpy(host.reshape(n, B)).to(dev)
torch.cuda.synchronize()
SENT = 0x5A5A5A5A5A5A5A5A
res = {}

def launch(stream):
    d = torch.full((n,), SENT, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    rc = L.stormck_checksum_device(buf.data_ptr(), B, None, B, n, d.data_ptr(), stream.cuda_stream)
    return rc, d

def ok_b(d):
    return bool((d.cpu().numpy().view(np.uint64) == want).all())

# order 1: A launches (stalls), B launches; B checks first, then A
rca, da = launch(sa)
rcb, db = launch(sb)
sb_rc = L.stormck_device_status(sb.cuda_stream)
# a host-synchronous call (the library's own staging streams) in between: clean
out = np.zeros(n, dtype=np.uint64)
h_rc = L.stormck_checksum_host(host.ctypes.data, B, None, B, n, out.ctypes.data)
sa_rc = L.stormck_device_status(sa.cuda_stream)
sa_msg = _lib.last_error()
sa_rc2 = L.stormck_device_status(sa.cuda_stream)
res["order1"] = [rca, rcb, sb_rc, ok_b(db), h_rc, bool((out == want).all()), sa_rc, sa_msg, sa_rc2]

# order 2: A checks first, then B
rca, da = launch(sa)
rcb, db = launch(sb)
sa_rc = L.stormck_device_status(sa.cuda_stream)
sb_rc = L.stormck_device_status(sb.cuda_stream)
res["order2"] = [sa_rc, sb_rc, ok_b(db), bool((da.cpu().numpy().view(np.uint64)[:5] == SENT).all())]

# two threads, one stream each, both ring launches in flight together; B verifies too
barrier = threading.Barrier(2)
tres = {}

def worker(name, stream):
    barrier.wait()
    rc, d = launch(stream)
    exp = torch.from_numpy(want.view(np.int64)).to(dev)
    r = torch.zeros(2, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    rv = L.stormck_verify_device(buf.data_ptr(), B, None, B, n, exp.data_ptr(), r.data_ptr(), stream.cuda_stream)
    barrier.wait()  # both launched before either checks
    st = L.stormck_device_status(stream.cuda_stream)
    tres[name] = [rc, rv, st, ok_b(d), r.cpu().tolist()]

ta = threading.Thread(target=worker, args=("a", sa))
tb = threading.Thread(target=worker, args=("b", sb))
ta.start(); tb.start(); ta.join(); tb.join()
res["threads"] = tres
print("RESULT " + json.dumps(res))
"""


@pytest.mark.timeout(240)
def test_ring_faults_stay_on_their_stream():
    """A stall forced on stream A only: callers on stream B (device checksum and
    verify, a host batch, another thread) see OK and correct results in either
    order, and A's own status check still reports its fault."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    env = dict(os.environ)
    env.pop("STORMCK_DEBUG_STALL_CHUNK", None)
    env.pop("STORMCK_DEBUG_STALL_STREAM", None)
    p = subprocess.run([sys.executable, "-c", CHILD_STREAMS, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=200)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:]
    r = json.loads(line[0][len("RESULT "):])
    rca, rcb, sb_rc, b_ok, h_rc, h_ok, sa_rc, sa_msg, sa_rc2 = r["order1"]
    assert (rca, rcb) == (_lib.OK, _lib.OK)
    assert sb_rc == _lib.OK and b_ok, r["order1"]  # B is clean although A's kernel stalled first
    assert h_rc == _lib.OK and h_ok, r["order1"]  # and so is a host batch on the library's streams
    assert sa_rc == _lib.EHIP and "k_xxh64_wide_multi" in sa_msg and sa_rc2 == _lib.OK, r["order1"]
    sa_rc, sb_rc, b_ok, a_sentinel = r["order2"]
    assert sa_rc == _lib.EHIP and sb_rc == _lib.OK and b_ok and a_sentinel, r["order2"]
    a, b = r["threads"]["a"], r["threads"]["b"]
    assert a[0] == _lib.OK and a[1] == _lib.OK and a[2] == _lib.EHIP, a
    assert a[4][1] >= 5, a  # A's verify fails closed on its stalled workgroup (two launches stalled)
    assert b == [_lib.OK, _lib.OK, _lib.OK, True, [1200, 0]], b
