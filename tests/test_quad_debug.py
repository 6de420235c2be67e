"""Quad merges must see all four lanes of their quad.

Every kernel merges a block's four XXH64 accumulators across the lanes of its quad with
DPP (kernels.h quad_bcast: update_dpp, bound_ctrl = false, old = 0). A source lane that
is not in exec then reads as 0: the checksum is silently wrong. A round-3 variant hit
exactly this (DESIGN_LOG.md §4, "Quad merges"). The debug build (tools/libstormck_debug.so,
-DSTORMCK_DEBUG_QUAD) counts every merge made with a partially active quad. This test
runs every kernel family of the shipped dispatch through that build in a child process,
checks each result against the oracle, and requires the count to be zero. Its self-test
kernel merges with 3 lanes of every quad off, so the counter is seen to work."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _debug_lib():
    from storm_amd import build as sb
    return sb.DEBUG_LIB


def test_debug_build_exports_the_counter():
    import ctypes
    if not os.path.exists(_debug_lib()):
        pytest.fail("debug build missing: python -c 'import __graft_entry__ as g; g.build()'")
    lib = ctypes.CDLL(_debug_lib())
    assert hasattr(lib, "stormck_debug_partial_quads") and hasattr(lib, "stormck_debug_partial_quad_selftest")
    from storm_amd import _lib
    assert not hasattr(ctypes.CDLL(_lib.LIB_PATH), "stormck_debug_partial_quads")


CHILD = r"""
import ctypes, json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from oracle import oracle as o
from storm_amd import _lib, commit as sc, engine
L = _lib.lib
cnt = L.stormck_debug_partial_quads
cnt.argtypes, cnt.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
def count(reset=1):
    c = ctypes.c_uint64(0)
    _lib.check(cnt(ctypes.byref(c), reset))
    return c.value
dev = torch.device("cuda", 0)
engine.init(0)
res = {"lib": _lib.LIB_PATH}
count()
_lib.check(L.stormck_debug_partial_quad_selftest())
res["selftest"] = count()
rng = np.random.default_rng(5)
bad = []
# every batch class of launch_checksum: wide, wide-multi (5 / 8 per CU), quad spread,
# quad, LDS-DMA 1/3/8 waves and the persistent skewed form; uniform, per-block lengths,
# gathered offsets, unaligned rows; checksum and verify
for n, slot in [(1, 4096), (100, 4096), (1200, 32768), (2000, 32768), (3000, 8192), (8000, 4096), (9300, 32768),
                (12000, 4096), (30000, 1024), (60000, 2048)]:
    host = o.fill_synthetic(n, slot, 0)
    d = torch.from_numpy(host.reshape(n, slot)).to(dev)
    want = o.checksum_batch(host, n, slot, slot, threads=8)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_device(d.data_ptr(), slot, n, out.data_ptr(), slot)
    if not np.array_equal(out.cpu().numpy().view(np.uint64), want): bad.append(("uniform", n))
    lens = rng.integers(0, slot + 1, size=n).astype(np.uint32)
    dl = torch.from_numpy(lens.view(np.int32)).to(dev)
    engine.checksum_device(d.data_ptr(), slot, n, out.data_ptr(), 0, dl.data_ptr())
    if not np.array_equal(out.cpu().numpy().view(np.uint64), o.checksum_batch(host, n, slot, 0, lens=lens)):
        bad.append(("lens", n))
    perm = rng.permutation(n).astype(np.uint64)
    offs = perm * np.uint64(slot) + np.uint64(4) * (perm % np.uint64(4))  # some rows unaligned
    glens = np.minimum(lens, np.uint32(slot - 12))
    do = torch.from_numpy(offs.view(np.int64)).to(dev)
    dgl = torch.from_numpy(glens.view(np.int32)).to(dev)
    engine.checksum_gather_device(d.data_ptr(), do.data_ptr(), n, out.data_ptr(), 0, dgl.data_ptr())
    flat = host.reshape(-1)
    gw = np.array([o.xxh64(flat[int(a):int(a) + int(l)]) for a, l in zip(offs[:64], glens[:64])], dtype=np.uint64)
    if not np.array_equal(out.cpu().numpy().view(np.uint64)[:64], gw): bad.append(("gather", n))
    exp = torch.from_numpy(want.view(np.int64)).to(dev)
    r = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d.data_ptr(), slot, n, exp.data_ptr(), r.data_ptr(), slot)
    if r.cpu().tolist() != [n, 0]: bad.append(("verify", n))
    del d
# f1 commits (wide, multi, quad and LDS-DMA levels) and Merkle levels (wide, producer/chain)
for nl, ln, fan in [(2, 31808, 1200), (1200, 31808, 1200), (5000, 32768, 1200), (999, 1000, 10)]:
    b, size, last = sc.pointer_forest(nl, ln, fan, slot=32768 if fan == 1200 else 1024, revision=1)
    slot = 32768 if fan == 1200 else 1024
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + nl * slot] = o.fill_synthetic(nl, slot, 1)
    ref, rb = arena.copy(), b.copy()
    wcs, _ = o.commit(ref, rb, 1, last)
    da = torch.from_numpy(arena).to(dev)
    cs, _ = sc.commit_device(da.data_ptr(), b, 1, last)
    if not np.array_equal(cs, wcs) or not np.array_equal(da.cpu().numpy(), ref): bad.append(("commit", nl))
for m in [1200 * 12, 1200 * 4000 + 7]:
    leaf = o.synth_leaf_checksums(m, 3 + m)
    dleaf = torch.from_numpy(leaf.view(np.int64)).to(dev)
    par = torch.empty((m + 1199) // 1200, dtype=torch.int64, device=dev)
    engine.pointer_level_device(dleaf.data_ptr(), m, 1 << 40, 5, 2, 1200, par.data_ptr())
    got = par.cpu().numpy().view(np.uint64)
    ent = [(int(leaf[k]), (1 << 40) + k, 5, 2) for k in range(0, 1200)]
    if int(got[0]) != o.xxh64(o.pack_pointer_block_py(ent, 1200)): bad.append(("pointer", m))
# f4 key tags
keys = o.fill_synthetic(4096, 48, 2)
dk = torch.from_numpy(keys).to(dev)
tags = torch.empty(4096, dtype=torch.int64, device=dev)
engine.key_tags_device(dk.data_ptr(), 4096, tags.data_ptr(), stride=48, length=48)
if not np.array_equal(tags.cpu().numpy().view(np.uint64), o.checksum_batch(keys, 4096, 48, 48)): bad.append(("keys", 4096))
res["bad"] = bad
res["partial"] = count()
print("RESULT " + json.dumps(res))
"""


@pytest.mark.gpu
@pytest.mark.timeout(280)
def test_every_kernel_family_merges_full_quads():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(_debug_lib()), "debug build missing"
    env = dict(os.environ, STORMCK_LIBRARY=_debug_lib())
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=250)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:]
    r = json.loads(line[0][len("RESULT "):])
    assert r["lib"].endswith("libstormck_debug.so"), r
    assert r["selftest"] == 16, r  # one partial merge per quad of the self-test wave
    assert r["bad"] == [], r
    assert r["partial"] == 0, r
