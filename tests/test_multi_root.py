"""Multi-GPU in one process through the C-ABI (stormck_shard_plan / stormck_merkle_root_multi,
include/stormck.h): storm is one process, so its cgo shim reaches
every GPU of a node from it.

CPU: the planning (shard ranges, node-address disjointness, device dealing) against the
process-per-GPU convention of storm_amd/dist.py, the stormck_shard layout, argument errors,
and the loud failure without a device. GPU: device-resident shards hashed and combined by the
library (d_blocks set) against the oracle, on one device holding every shard and on every
visible device; the full-size c4 roots from the 64M checksums are in tests/test_c4_gpu.py.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from storm_amd import dist as sdist

FANOUT, REV = 1200, 1


def _nodes(n, f):
    t, m = 0, n
    while m > 1:
        m = (m + f - 1) // f
        t += m
    return t


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8, 64])
def test_plan_is_the_process_per_gpu_convention(world):
    """Shard s of the C planner = rank s of storm_amd/dist.py: the same leaf range, node
    address base and combining-node address, for sizes that do and do not divide."""
    from storm_amd import multi
    for n_total in (0, 1, 7, 12345, 1_000_003, 64 << 20):
        shards, root_addr = multi.plan(n_total, world, list(range(min(world, 8))))
        assert root_addr == sdist.global_root_addr(n_total)
        for s, sh in enumerate(shards):
            lo, hi = sdist.shard_range(n_total, world, s)
            assert (sh.leaf_addr_base, sh.n) == (lo, hi - lo)
            assert sh.node_addr_base == sdist.shard_node_addr_base(n_total, lo)
            assert not sh.d_blocks and not sh.d_checksums and not sh.stream and sh.stride == 0 and sh.len == 0


@pytest.mark.parametrize("fanout", [3, 10, 1200])
def test_planned_node_addresses_are_disjoint(fanout):
    """Every shard's interior nodes (node_addr_base + [0, nodes)) lie above the leaves, below
    the combining node, and apart from every other shard's."""
    from storm_amd import multi
    for n_total in (2, 17, 12345, 1_000_003):
        for world in (1, 2, 5, 8):
            shards, root_addr = multi.plan(n_total, world, [0])
            spans = sorted((sh.node_addr_base, sh.node_addr_base + _nodes(sh.n, fanout)) for sh in shards if sh.n)
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b <= c
            assert all(a >= n_total and b <= root_addr for a, b in spans)
            leaves = sorted((sh.leaf_addr_base, sh.leaf_addr_base + sh.n) for sh in shards)
            assert leaves[0][0] == 0 and leaves[-1][1] == n_total
            assert all(b == c for (_, b), (c, _) in zip(leaves, leaves[1:]))


def test_plan_deals_shards_to_devices_in_runs():
    from storm_amd import multi
    dev = lambda n_shards, devices: [sh.device for sh in multi.plan(1000, n_shards, devices)[0]]  # noqa: E731
    assert dev(8, [0, 1, 2, 3, 4, 5, 6, 7]) == list(range(8))
    assert dev(8, [0]) == [0] * 8
    assert dev(8, [3, 5]) == [3, 3, 3, 3, 5, 5, 5, 5]
    assert dev(2, [0, 1, 2, 3]) == [0, 2]
    assert dev(5, [0, 1]) == [0, 0, 0, 1, 1]


def test_shard_struct_matches_the_header():
    """ctypes' stormck_shard against the C compiler's layout of include/stormck.h."""
    from storm_amd._lib import ShardStruct
    from tests.conftest import ROOT
    src = r"""
#include <stddef.h>
#include <stdio.h>
#include "stormck.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(stormck_shard), offsetof(stormck_shard, d_blocks),
           offsetof(stormck_shard, stride), offsetof(stormck_shard, n), offsetof(stormck_shard, d_checksums),
           offsetof(stormck_shard, leaf_addr_base), offsetof(stormck_shard, node_addr_base),
           offsetof(stormck_shard, stream), offsetof(stormck_shard, device), offsetof(stormck_shard, len));
    return 0;
}
"""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(ShardStruct)] + [getattr(ShardStruct, f).offset for f, _ in ShardStruct._fields_]
    assert got == want == [64, 0, 8, 16, 24, 32, 40, 48, 56, 60]


def test_argument_errors():
    from storm_amd import _lib
    from storm_amd._lib import PointerStruct, ShardStruct
    L = _lib.lib
    sh = (ShardStruct * 2)()
    r, t = PointerStruct(), ctypes.c_uint8()
    dv = (ctypes.c_int * 1)(0)
    cases = [
        ("plan no shards", lambda: L.stormck_shard_plan(10, 0, dv, 1, sh, None)),
        ("plan null shards", lambda: L.stormck_shard_plan(10, 2, dv, 1, None, None)),
        ("plan no devices", lambda: L.stormck_shard_plan(10, 2, None, 0, sh, None)),
        ("plan 65 devices", lambda: L.stormck_shard_plan(10, 2, (ctypes.c_int * 65)(), 65, sh, None)),
        ("plan huge", lambda: L.stormck_shard_plan(1 << 63, 2, dv, 1, sh, None)),
        ("root null", lambda: L.stormck_merkle_root_multi(sh, 2, 1, 20, 1200, None, ctypes.byref(t), None, None)),
        ("fanout 1", lambda: L.stormck_merkle_root_multi(sh, 2, 1, 20, 1, ctypes.byref(r), ctypes.byref(t), None,
                                                         None)),
        ("no shards", lambda: L.stormck_merkle_root_multi(sh, 0, 1, 20, 1200, ctypes.byref(r), ctypes.byref(t), None,
                                                          None)),
        ("shards > fanout", lambda: L.stormck_merkle_root_multi((ShardStruct * 3)(), 3, 1, 20, 2, ctypes.byref(r),
                                                                ctypes.byref(t), None, None)),
        ("null shards", lambda: L.stormck_merkle_root_multi(None, 2, 1, 20, 1200, ctypes.byref(r), ctypes.byref(t),
                                                            None, None)),
    ]
    for name, fn in cases:
        assert fn() == _lib.EINVAL, name
        assert _lib.last_error(), name


def _layout_model(devices_of_shards):
    """What the gather must hold: ranks = distinct devices by first appearance, R = most shards
    on one device, shard s in row (rank * R + its place among its device's shards)."""
    devs, place, seen = [], [], {}
    for d in devices_of_shards:
        if d not in seen:
            seen[d] = 0
            devs.append(d)
        place.append(seen[d])
        seen[d] += 1
    R = max(seen.values())
    return devs, R, [devs.index(d) * R + p for d, p in zip(devices_of_shards, place)]


@pytest.mark.parametrize("seed", range(12))
def test_gather_layout_for_many_devices(seed):
    """stormck_multi_layout (the layout stormck_merkle_root_multi gathers with) for 1-8
    devices and up to 64 shards dealt in runs or interleaved: the C layout equals the model,
    and a CPU rehearsal of the D-rank all-gather (each device's R send rows, zero where it has
    fewer shards, concatenated in rank order) hands the combining node every shard's root in
    shard order, so the global root is the oracle's for any dealing. The one step this does
    not run is RCCL itself; one-GPU runs cover it at D = 1 (test_one_device_holds_every_shard)."""
    from oracle import oracle as o
    from storm_amd import multi
    rng = np.random.default_rng(seed)
    n_dev = int(rng.integers(1, 9))
    pool = [int(d) for d in rng.choice(16, size=n_dev, replace=False)]
    n_shards = int(rng.integers(1, 65))
    n_total = int(rng.integers(n_shards, 40 * n_shards))
    shards, root_addr = multi.plan(n_total, n_shards, pool)
    if seed % 2:  # interleaved dealing instead of the planner's runs
        for sh in shards:
            sh.device = int(rng.choice(pool))
    on = [sh.device for sh in shards]
    devs, R, rows = multi.layout(shards)
    assert (devs, R, rows) == _layout_model(on)
    assert len(set(rows)) == n_shards and max(rows) < len(devs) * R
    # rehearse the exchange with the oracle's shard roots
    cs = o.checksum_batch(o.fill_synthetic(n_total, 64, 0), n_total, 64, 64, threads=4)
    roots = [o.merkle_root(cs[sh.leaf_addr_base:sh.leaf_addr_base + sh.n], sh.leaf_addr_base, sh.node_addr_base,
                           REV, 10) for sh in shards]
    send = {d: [(0, 0, 0, 0)] * R for d in devs}
    seen = {d: 0 for d in devs}
    for sh, r in zip(shards, roots):
        send[sh.device][seen[sh.device]] = r
        seen[sh.device] += 1
    table = [row for d in devs for row in send[d]]  # ncclAllGather: rank order
    gathered = [table[rows[s]] for s in range(n_shards)]
    assert gathered == roots
    assert o.combine_roots(gathered, REV, root_addr, 1200) == o.combine_roots(roots, REV, root_addr, 1200)


def test_gather_layout_errors():
    from storm_amd import _lib, multi
    from storm_amd._lib import ShardStruct
    L = _lib.lib
    sh = (ShardStruct * 2)()
    d, nd, r, tr = (ctypes.c_int32 * 64)(), ctypes.c_uint32(), ctypes.c_uint32(), (ctypes.c_uint32 * 2)()
    assert L.stormck_multi_layout(None, 2, d, ctypes.byref(nd), ctypes.byref(r), tr) == _lib.EINVAL
    assert L.stormck_multi_layout(sh, 0, d, ctypes.byref(nd), ctypes.byref(r), tr) == _lib.EINVAL
    assert L.stormck_multi_layout(sh, 2, None, ctypes.byref(nd), ctypes.byref(r), tr) == _lib.EINVAL
    sh[1].device = -1
    assert L.stormck_multi_layout(sh, 2, d, ctypes.byref(nd), ctypes.byref(r), tr) == _lib.EINVAL
    assert "negative" in _lib.last_error()
    many = [multi.shard(k, 1, 8, k, 1000 + k) for k in range(65)]
    with pytest.raises(_lib.StormckError, match="64 devices"):
        multi.layout(many)
    assert multi.layout(many[:64])[:2] == (list(range(64)), 1)


def _has_gpu():
    from storm_amd import _lib
    return _lib.device_count() > 0


@pytest.mark.skipif("_has_gpu()")
def test_no_device_fails_loudly():
    from storm_amd import _lib, multi
    shards, ra = multi.plan(100, 2, [0])
    with pytest.raises(_lib.NoDeviceError):
        multi.merkle_root_multi(shards, REV, ra)


# ---------------------------------------------------------------------------- GPU
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    assert _lib.device_count() > 0, "GPU visible to torch but libstormck finds no gfx950 device"
    return torch.device("cuda:0")


def _expected(n_total, world, stride, length, fanout, first=0):
    """Oracle: the leaf checksums of logical blocks first..first+n_total-1, each shard's root
    and the combined root under the shard convention."""
    from oracle import oracle as o
    host = o.fill_synthetic(n_total, stride, first)
    cs = o.checksum_batch(host, n_total, stride, length, threads=8)
    rows = []
    for lo, hi in sdist.plan(n_total, world):
        rows.append(o.merkle_root(cs[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), REV, fanout))
    return cs, rows, o.combine_roots(rows, REV, sdist.global_root_addr(n_total), fanout)


def _device_shards(n_total, world, devices, stride, length, first=0, streams=False):
    """Planned shards whose blocks (logical first + lo ..) are generated on their devices;
    returns (shards, root_addr, per-shard checksum tensors, keep-alive list)."""
    from oracle import oracle as o
    from storm_amd import engine, multi
    shards, root_addr = multi.plan(n_total, world, devices)
    outs, keep = [], []
    for sh in shards:
        d = torch.device("cuda", sh.device)
        blocks = torch.empty((max(sh.n, 1), stride), dtype=torch.uint8, device=d)
        with torch.cuda.device(d):
            engine.fill_synthetic_device(blocks.data_ptr(), stride, sh.n, first + sh.leaf_addr_base, o.SYNTH_SEED)
        cs = torch.full((max(sh.n, 1),), -1, dtype=torch.int64, device=d)
        st = torch.cuda.Stream(device=d) if streams else None
        multi.set_buffers(sh, cs.data_ptr(), blocks.data_ptr(), stride, length, st.cuda_stream if st else 0)
        outs.append(cs)
        keep += [blocks, st]
    torch.cuda.synchronize()
    return shards, root_addr, outs, keep


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_total,stride,length,fanout,streams", [
    (1, 3000, 4096, 4096, 10, False),
    (2, 5001, 4096, 4000, 10, True),
    (3, 40_000, 1024, 1024, 1200, False),
    (8, 25_000, 2048, 2048, 10, True),
    (8, 5, 512, 500, 10, False),      # shards of 0 and 1 leaves: Free and Leaf roots
    (10, 12_345, 768, 728, 10, False),  # `-tags test` block sizes and fan-out: as many shards as it holds
    (16, 12_345, 768, 728, 1200, True),  # more shards than the c4 world
])
def test_one_device_holds_every_shard(dev, world, n_total, stride, length, fanout, streams):
    """Device list [0]: the library hashes each shard's blocks, builds each shard tree,
    gathers the rows through a one-rank RCCL communicator and combines them: leaf checksums,
    shard roots and the global root equal the oracle's."""
    from storm_amd import engine, multi
    cs_want, rows_want, root_want = _expected(n_total, world, stride, length, fanout)
    shards, root_addr, outs, keep = _device_shards(n_total, world, [0], stride, length, streams=streams)
    root, rows = multi.merkle_root_multi(shards, REV, root_addr, fanout)
    assert rows == rows_want
    assert root == root_want
    for sh, cs in zip(shards, outs):
        got = engine.u64(cs)[:sh.n]
        assert np.array_equal(got, cs_want[sh.leaf_addr_base:sh.leaf_addr_base + sh.n])
    # the call is repeatable (cached communicator and buffers) and leaves the streams usable
    root2, rows2 = multi.merkle_root_multi(shards, REV, root_addr, fanout)
    assert (root2, rows2) == (root, rows)
    del keep


@pytest.mark.gpu
def test_precomputed_leaf_checksums(dev):
    """d_blocks NULL: the leaf checksums are read from d_checksums (what bench.py's in-process
    mode passes after hashing its arena passes), and nothing is written to them."""
    from oracle import oracle as o
    from storm_amd import multi
    n_total, world = 30_001, 4
    leaves = o.synth_leaf_checksums(n_total)
    t = torch.from_numpy(leaves.view(np.int64).copy()).to(dev)
    shards, root_addr = multi.plan(n_total, world, [0])
    for sh in shards:
        multi.set_buffers(sh, t[sh.leaf_addr_base:].data_ptr())
    root, rows = multi.merkle_root_multi(shards, REV, root_addr)
    want_rows = [o.merkle_root(leaves[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), REV)
                 for lo, hi in sdist.plan(n_total, world)]
    assert rows == want_rows
    assert root == o.combine_roots(want_rows, REV, sdist.global_root_addr(n_total))
    assert np.array_equal(t.cpu().numpy().view(np.uint64), leaves)


@pytest.mark.gpu
def test_more_shards_than_the_combining_node_holds(dev):
    """The combining node is one pointer block: at most `fanout` shard roots."""
    from storm_amd import _lib, multi
    shards, ra = multi.plan(100, 11, [0])
    with pytest.raises(_lib.StormckError, match="1..fanout"):
        multi.merkle_root_multi(shards, REV, ra, 10)


@pytest.mark.gpu
def test_bad_shard_device_is_named(dev):
    from storm_amd import _lib, multi
    shards, ra = multi.plan(100, 2, [0])
    keep = torch.empty(100, dtype=torch.int64, device=dev)
    for sh in shards:
        multi.set_buffers(sh, keep[sh.leaf_addr_base:].data_ptr())
    shards[1].device = 4096  # every shard is checked before any device work
    with pytest.raises(_lib.StormckError, match=r"shards\[1\].device = 4096"):
        multi.merkle_root_multi(shards, REV, ra)
    shards, ra = multi.plan(100, 2, [0])  # n > 0 without checksums
    with pytest.raises(_lib.StormckError, match=r"d_checksums is null"):
        multi.merkle_root_multi(shards, REV, ra)


@pytest.mark.gpu
def test_every_visible_device(dev):
    """One shard per visible device (8 on an MI355X node: RCCL over xGMI), plus two shards per
    device; skipped on a one-GPU box, where the one-device tests above cover the code path."""
    from storm_amd import engine, multi
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one visible device")
    for world in (n, 2 * n):
        cs_want, rows_want, root_want = _expected(40_000, world, 2048, 2048, FANOUT, first=77)
        shards, root_addr, outs, keep = _device_shards(40_000, world, list(range(n)), 2048, 2048, first=77,
                                                       streams=True)
        root, rows = multi.merkle_root_multi(shards, REV, root_addr)
        assert rows == rows_want and root == root_want
        for sh, cs in zip(shards, outs):
            assert np.array_equal(engine.u64(cs)[:sh.n], cs_want[sh.leaf_addr_base:sh.leaf_addr_base + sh.n])
        del keep
