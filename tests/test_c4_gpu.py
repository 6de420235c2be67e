"""c3 / c4 at full size on one GPU (BASELINE.json configs[2], configs[3]).

c4 is 64M x 32 KiB blocks sharded 8M per GPU over 8 GPUs, with the shard roots
gathered and combined. Its arithmetic does not depend on which GPU a shard runs on,
so this test runs the 8 shards one after another on one GPU, exactly as each rank of
bench.py would: the shard streams through a 2M-block arena (4 passes, the arena
regenerated with the pass's own logical blocks), the shard tree is built on the
device (k_pointer_level*), and the 8 roots are combined on the device
(k_pointer_node). Checked against tests/golden/c3c4_roots.json, computed with
libxxhash by oracle/gen_golden.py --c4 (roots for world 1, 2, 4 and 8, and the c3 root
of the first 16M blocks), plus the digest of all 64M checksums.
"""
import numpy as np
import pytest

from tests.conftest import hx, load_golden

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

torch = pytest.importorskip("torch")

BLOCK, FANOUT, REV = 32768, 1200, 1


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    assert _lib.device_count() > 0, "GPU visible to torch but libstormck finds no gfx950 device"
    return torch.device("cuda:0")


def _row(root):
    from storm_amd import engine
    t = engine.as_tuple(root)
    return ["0x%016x" % v for v in t[:3]] + [t[3]]


@pytest.fixture(scope="module")
def c4_checksums(dev):
    """All 64M checksums, computed shard by shard as the c4 ranks do."""
    from oracle import oracle as o
    from storm_amd import dist as sdist
    from storm_amd import engine
    fx = load_golden("c3c4_roots.json")
    n_total, world, arena_n = fx["c4"]["n_total"], 8, 2 << 20  # bench.py --arena default
    arena = torch.empty((arena_n, BLOCK), dtype=torch.uint8, device=dev)
    cs = torch.empty(n_total, dtype=torch.int64, device=dev)
    for r in range(world):
        lo, hi = sdist.shard_range(n_total, world, r)
        for first in range(lo, hi, arena_n):
            cnt = min(arena_n, hi - first)
            engine.fill_synthetic_device(arena.data_ptr(), BLOCK, cnt, first, o.SYNTH_SEED)
            engine.checksum_device(arena.data_ptr(), BLOCK, cnt, cs[first:].data_ptr(), BLOCK)
    torch.cuda.synchronize()
    del arena
    torch.cuda.empty_cache()
    return cs


def test_c4_checksums_digest(c4_checksums):
    from oracle import oracle as o
    fx = load_golden("c3c4_roots.json")["c4"]
    host = c4_checksums.cpu().numpy().view(np.uint64)
    assert [int(v) for v in host[::1 << 20]] == [hx(v) for v in fx["every_1048576th"]]
    assert o.xxh64(host.astype("<u8")) == hx(fx["digest"])


@pytest.mark.parametrize("world", [8, 4, 2, 1])
def test_c4_shard_roots_and_global_root(dev, c4_checksums, world):
    """Per-shard device trees + the device combine = the libxxhash roots (world 8 is
    c4 itself: 8 shards of 8M; world 1 is the strong-scaling series' N = 1 point, all
    64M leaves in one tree)."""
    from storm_amd import dist as sdist
    from storm_amd import engine
    fx = load_golden("c3c4_roots.json")["c4"]
    n_total = fx["n_total"]
    want = fx["worlds"][str(world)]
    roots = []
    for r in range(world):
        lo, hi = sdist.shard_range(n_total, world, r)
        roots.append(engine.merkle_root_tensor(c4_checksums[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo),
                                               REV, FANOUT))
    table = torch.stack(roots)
    groot = engine.combine_roots_tensor(table, REV, sdist.global_root_addr(n_total), FANOUT)
    torch.cuda.synchronize()
    assert [_row(r) for r in roots] == want["shard_roots"]
    assert _row(groot) == want["global_root"]


def test_c3_root_of_the_first_16m_blocks(dev, c4_checksums):
    """bench.py's N = 1 line: the shard tree of blocks 0..16M-1 (c3)."""
    from storm_amd import engine
    fx = load_golden("c3c4_roots.json")["c3"]
    root = engine.merkle_root_tensor(c4_checksums[:fx["n"]], fx["leaf_addr_base"], fx["node_addr_base"], REV, FANOUT)
    torch.cuda.synchronize()
    assert _row(root) == fx["root"]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c4_roots_through_the_c_abi_multi_entry(dev, c4_checksums, world):
    """The one-process multi-GPU entry (stormck_merkle_root_multi, what storm's cgo shim
    calls) with device list [0]: the planned shards' trees over slices of the 64M checksums,
    the RCCL gather (a one-rank communicator here) and the device combine reproduce the c4
    world-N shard roots and global root (world 1: the strong-scaling N = 1 point)."""
    from storm_amd import multi
    fx = load_golden("c3c4_roots.json")["c4"]
    want = fx["worlds"][str(world)]
    shards, root_addr = multi.plan(fx["n_total"], world, [0])
    for sh in shards:
        multi.set_buffers(sh, c4_checksums[sh.leaf_addr_base:].data_ptr())
    root, rows = multi.merkle_root_multi(shards, REV, root_addr, FANOUT)
    fmt = lambda r: ["0x%016x" % v for v in r[:3]] + [r[3]]  # noqa: E731
    assert [fmt(r) for r in rows] == want["shard_roots"]
    assert fmt(root) == want["global_root"]
