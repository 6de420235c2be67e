"""f1 — level-synchronous batched commit (storm Cache.Commit data phase,
/root/reference/cache/cache.go:87-137 + trace.go:274-320).

CPU: the oracle's serial commit loop reproduces the libxxhash fixture built by an
independent restatement (oracle/gen_golden.py gen_commit), and the host forest
builder reproduces the fixture's layout. GPU: stormck_commit_device matches the
fixture, the oracle on random forests (fan-out 10 and 1200, relocations, mixed
lengths), and at full size (1M dirty 32 KiB leaves) every origin verifies.
"""
import struct

import numpy as np
import pytest

from oracle import oracle as o
from storm_amd import commit as sc
from tests.conftest import hx, load_golden


def fixture_forest():
    g = load_golden("commit.json")
    rng = np.random.default_rng(g["leaf_bytes_seed"])
    slot, n = g["slot"], g["n_leaves"]
    lens = [int(x) for x in rng.choice([72, 256, 536, 728, 1000, 1024], size=n)]
    assert lens == g["leaf_lens"]
    b, size, last = sc.pointer_forest(n, lens, g["fanout"], slot=slot, revision=g["revision"])
    existing = rng.random(len(b)) < 0.3
    assert [int(x) for x in existing] == g["existing"]
    b["birth_revision"][existing] = g["revision"]
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + n * slot] = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    assert o.xxh64(arena) == hx(g["initial_arena_xxh64"])
    return g, b, arena, last


def singularity_step(arena, revision, last):
    # cache/cache.go:71-73: Revision++, Checksum = 0, Checksum = BlockChecksum(singularity)
    struct.pack_into("<Q", arena, 16, revision + 1)
    struct.pack_into("<Q", arena, 64, last)
    struct.pack_into("<Q", arena, 0, 0)
    return o.xxh64(arena[:72])


def test_oracle_commit_matches_fixture():
    g, b, arena, last = fixture_forest()
    cs, last2 = o.commit(arena, b, g["revision"], last)
    assert [int(v) for v in cs] == [hx(v) for v in g["checksums"]]
    assert [int(v) for v in b["address"]] == g["addresses"]
    assert last2 == g["last_allocated"]
    assert o.xxh64(arena[72:]) == hx(g["final_arena_xxh64"])
    assert singularity_step(arena, g["revision"], last2) == hx(g["singularity_checksum"])


def test_forest_shape():
    b, size, last = sc.pointer_forest(25, 100, 10, slot=1024, revision=1)
    # 25 leaves -> 3 pointer blocks -> 1 root pointer block
    assert len(b) == 25 + 3 + 1 and last == 29
    assert list(b["parent"][:25]) == [25 + i // 10 for i in range(25)]
    assert list(b["parent"][25:28]) == [28] * 3 and b["parent"][28] == sc.NO_PARENT
    assert b["origin_pointer"][28] == sc.SING_SPACE_POINTER and b["origin_type"][28] == sc.SING_SPACE_TYPE
    assert b["origin_pointer"][13] == b["data_offset"][26] + 24 * 3
    assert b["origin_type"][13] == b["data_offset"][26] + 240 + 3
    assert set(b["type"][:25]) == {sc.LEAF} and set(b["type"][25:]) == {sc.POINTER}
    assert sc.DIRTY_DTYPE.itemsize == 56


def _random_forest(n, fanout, slot, how, rng=None):
    rng = rng or np.random.default_rng(n * 7 + fanout)
    choices = [72, 256, 536, 728, 1000, 1024] if slot < 2048 else [72, 28808, 30000, 31808, 32768, 4097]
    lens = rng.choice(choices, size=n)
    b, size, last = sc.pointer_forest(n, lens, fanout, slot=slot, revision=9, first_address=100)
    b["birth_revision"][rng.random(len(b)) < 0.4] = 3
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + n * slot] = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    return arrange(b, how, rng), arena, last


@pytest.mark.parametrize("threads", [1, 0])
def test_host_leg_matches_fixture(threads):
    """stormck_commit_host (the host leg of the routed commit; no device needed)."""
    g, b, arena, last = fixture_forest()
    cs, last2 = sc.commit_host(arena, b, g["revision"], last, threads=threads)
    assert [int(v) for v in cs] == [hx(v) for v in g["checksums"]]
    assert [int(v) for v in b["address"]] == g["addresses"]
    assert last2 == g["last_allocated"]
    assert o.xxh64(arena[72:]) == hx(g["final_arena_xxh64"])
    assert singularity_step(arena, g["revision"], last2) == hx(g["singularity_checksum"])


@pytest.mark.parametrize("threads", [1, 3, 0])
@pytest.mark.parametrize("how", ["shuffled", "upper_shuffled", "children_first"])
@pytest.mark.parametrize("n,fanout,slot", [(1, 10, 1024), (11, 10, 1024), (999, 10, 1024), (1201, 1200, 32768),
                                            (999, 10, 1032), (20000, 10, 1024)])
def test_host_leg_random_forests(n, fanout, slot, how, threads):
    """The host leg against storm's serial loop (the C oracle) on the device tests'
    forests: relocations, mixed lengths, unaligned slots, any caller order."""
    bp, arena, last = _random_forest(n, fanout, slot, how)
    ref_arena, ref_b = arena.copy(), bp.copy()
    want_cs, want_last = o.commit(ref_arena, ref_b, 9, last)
    cs, last2 = sc.commit_host(arena, bp, 9, last, threads=threads)
    assert np.array_equal(cs, want_cs)
    assert np.array_equal(bp["address"], ref_b["address"])
    assert np.array_equal(bp["birth_revision"], ref_b["birth_revision"])
    assert last2 == want_last
    assert np.array_equal(arena, ref_arena)


def test_host_leg_argument_errors():
    """The device leg's validation, messages and no-change-on-error rule."""
    from storm_amd import _lib
    b, size, last = sc.pointer_forest(25, 100, 10, slot=1024, revision=1)
    arena = np.zeros(size, dtype=np.uint8)
    for field, value, text in [("parent", 10 ** 6, "parent index out of range"),
                               ("origin_pointer", 5, "8-byte aligned")]:
        bad = b.copy()
        bad[field][3] = value
        keep = bad.copy()
        with pytest.raises(_lib.StormckError, match=text):
            sc.commit_host(arena, bad, 1, last)
        assert np.array_equal(bad, keep)
    cyc = b.copy()
    cyc["parent"][28] = 3  # root -> leaf 3 -> ... -> root
    with pytest.raises(_lib.StormckError, match="cycle"):
        sc.commit_host(arena, cyc, 1, last)


# ---------------------------------------------------------------------------
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def device_commit(arena: np.ndarray, b: np.ndarray, revision: int, last: int, dev):
    d = torch.from_numpy(arena.copy()).to(dev)
    cs, last2 = sc.commit_device(d.data_ptr(), b, revision, last)
    return d.cpu().numpy(), cs, last2


@pytest.mark.gpu
def test_device_commit_matches_fixture(dev):
    g, b, arena, last = fixture_forest()
    out, cs, last2 = device_commit(arena, b, g["revision"], last, dev)
    assert [int(v) for v in cs] == [hx(v) for v in g["checksums"]]
    assert [int(v) for v in b["address"]] == g["addresses"]
    assert last2 == g["last_allocated"]
    assert o.xxh64(out[72:]) == hx(g["final_arena_xxh64"])
    assert singularity_step(out, g["revision"], last2) == hx(g["singularity_checksum"])


def arrange(b: np.ndarray, how: str, rng) -> np.ndarray:
    """Permute the dirty list and remap parent indices. "shuffled": parents may precede
    children; "upper_shuffled": level 0 (the leaves) stays a prefix in index order, the
    pointer blocks after it are shuffled; "children_first": as built."""
    n_leaves = int((b["type"] == sc.LEAF).sum())
    if how == "children_first":
        return b.copy()
    if how == "shuffled":
        perm = rng.permutation(len(b))
    else:
        perm = np.concatenate([np.arange(n_leaves), n_leaves + rng.permutation(len(b) - n_leaves)])
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(b))
    bp = b[perm].copy()
    has = bp["parent"] >= 0
    bp["parent"][has] = inv[bp["parent"][has]]
    return bp


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["shuffled", "upper_shuffled", "children_first"])
@pytest.mark.parametrize("n,fanout,slot", [(1, 10, 1024), (10, 10, 1024), (11, 10, 1024), (999, 10, 1024),
                                            (5000, 1200, 32768), (1201, 1200, 32768),
                                            # 8- but not 16-byte aligned slots: register-quad commit kernel
                                            (999, 10, 1032), (3000, 1200, 32776),
                                            # level 0 in several growing chunks (32K, 96K, rest)
                                            (140000, 10, 1024)])
def test_device_commit_random_forests(dev, n, fanout, slot, how):
    """The commit must not depend on the caller's order beyond the documented
    (height, index) rule; the library takes a different route per arrangement (level 0
    a prefix or not, upper levels in height order or not)."""
    rng = np.random.default_rng(n * 7 + fanout)
    choices = [72, 256, 536, 728, 1000, 1024] if slot < 2048 else [72, 28808, 30000, 31808, 32768, 4097]
    lens = rng.choice(choices, size=n)
    b, size, last = sc.pointer_forest(n, lens, fanout, slot=slot, revision=9, first_address=100)
    b["birth_revision"][rng.random(len(b)) < 0.4] = 3
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + n * slot] = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    bp = arrange(b, how, rng)
    ref_arena, ref_b = arena.copy(), bp.copy()
    want_cs, want_last = o.commit(ref_arena, ref_b, 9, last)
    out, cs, last2 = device_commit(arena, bp, 9, last, dev)
    assert np.array_equal(cs, want_cs)
    assert np.array_equal(bp["address"], ref_b["address"]) and np.array_equal(bp["birth_revision"], ref_b["birth_revision"])
    assert last2 == want_last
    assert np.array_equal(out, ref_arena)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [12000, 20000, 36864])
def test_device_commit_streaming_level_mixed_lengths(dev, n):
    """Levels from 39 blocks per CU take the LDS-DMA commit kernel (on 256 CUs: 12,000
    leaves in 3-wave workgroups, 20,000 in 1-wave ones, 36,864 in 3-wave ones again
    where 8-wave ones would put two workgroups on some CUs): leaves of mixed storm lengths
    (workgroups whose blocks run out of stripes at different tiles), a third relocating,
    shuffled dirty list; vs the oracle's serial commit."""
    rng = np.random.default_rng(n)
    slot = 32768
    lens = rng.choice([72, 28808, 30000, 31808, 32768, 4097, 512], size=n)
    b, size, last = sc.pointer_forest(n, lens, 1200, slot=slot, revision=4, first_address=7)
    b["birth_revision"][::3] = 2
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + n * slot] = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    perm = rng.permutation(len(b))
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(b))
    bp = b[perm].copy()
    has = bp["parent"] >= 0
    bp["parent"][has] = inv[bp["parent"][has]]
    ref_arena, ref_b = arena.copy(), bp.copy()
    want_cs, want_last = o.commit(ref_arena, ref_b, 4, last)
    out, cs, last2 = device_commit(arena, bp, 4, last, dev)
    assert np.array_equal(cs, want_cs)
    assert np.array_equal(bp["address"], ref_b["address"]) and last2 == want_last
    assert np.array_equal(out, ref_arena)


@pytest.mark.gpu
def test_commit_on_registered_host_arena(dev):
    """f1 on storm's cache.data where it lives: a registered host arena, reached in
    place through stormck_host_device_pointer (kernels read blocks and write origins
    over PCIe). Same result as the oracle's serial commit, byte for byte."""
    from storm_amd import blocks as sb
    rng = np.random.default_rng(77)
    n, slot = 3000, 32768
    lens = rng.choice([72, 28808, 30000, 31808, 32768], size=n)
    b, size, last = sc.pointer_forest(n, lens, 1200, slot=slot, revision=6)
    b["birth_revision"][::4] = 3
    arena = np.zeros(size, dtype=np.uint8)
    arena[slot:slot + n * slot] = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    ref_arena, ref_b = arena.copy(), b.copy()
    want_cs, want_last = o.commit(ref_arena, ref_b, 6, last)
    sb.RegisterHostMemory(arena)
    try:
        d_arena = sb.HostDevicePointer(arena)
        assert d_arena != 0
        cs, last2 = sc.commit_device(d_arena, b, 6, last)
        torch.cuda.synchronize()
    finally:
        sb.UnregisterHostMemory(arena)
    assert np.array_equal(cs, want_cs) and last2 == want_last
    assert np.array_equal(b["address"], ref_b["address"])
    assert np.array_equal(arena, ref_arena)


@pytest.mark.gpu
@pytest.mark.slow
def test_device_commit_1m_leaves_properties(dev):
    """1M dirty 32 KiB leaves + 835 pointer blocks (fan-out 1200), all in HBM: after the
    commit every block's origin holds {its checksum, address, birth} and its type, and
    every checksum equals an independent batch hash of the block."""
    from storm_amd import engine
    n, slot, rev = 1 << 20, 32768, 1
    b, size, last = sc.pointer_forest(n, slot, 1200, slot=slot, revision=rev)
    b["birth_revision"][::3] = rev  # a third of the blocks relocate
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + slot, slot, n, 0, o.SYNTH_SEED)
    torch.cuda.synchronize()
    cs, last2 = sc.commit_device(arena.data_ptr(), b, rev, last)
    assert last2 == last + len(range(0, len(b), 3))
    # independent re-hash of every committed block (gather kernel) after the commit
    offs = torch.from_numpy(b["data_offset"].view(np.int64)).to(dev)
    lens = torch.from_numpy(b["length"].view(np.int32)).to(dev)
    again = torch.empty(len(b), dtype=torch.int64, device=dev)
    engine.checksum_gather_device(arena.data_ptr(), offs.data_ptr(), len(b), again.data_ptr(), 0, lens.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(again.cpu().numpy().view(np.uint64), cs)
    # origins: 24-byte Pointer + type byte
    a = arena.view(torch.int64)
    optr = torch.from_numpy((b["origin_pointer"] // 8).astype(np.int64)).to(dev)
    got = torch.stack([a[optr], a[optr + 1], a[optr + 2]], 1).cpu().numpy().view(np.uint64)
    assert np.array_equal(got[:, 0], cs)
    assert np.array_equal(got[:, 1], b["address"]) and np.array_equal(got[:, 2], b["birth_revision"])
    types = arena[torch.from_numpy(b["origin_type"].astype(np.int64)).to(dev)].cpu().numpy()
    assert np.array_equal(types, b["type"])
    # leaves match the oracle on a sample
    host = arena[slot:slot + 64 * slot].cpu().numpy()
    assert np.array_equal(o.checksum_batch(host, 64, slot, slot), cs[:64])


@pytest.mark.gpu
def test_routed_commit_legs(dev):
    """stormck_commit (the Go binding's CommitBatch): an HBM arena takes the device leg,
    an unregistered host arena the host leg, a registered one the leg of the cost model
    (storm's 3-block commit: host); every leg equal to storm's serial loop (the oracle)."""
    from storm_amd import _lib, blocks
    cases = []
    for n, fanout, slot in [(2, 1200, 32768), (1200, 1200, 32768), (999, 10, 1024)]:
        bp, arena, last = _random_forest(n, fanout, slot, "shuffled")
        ref_arena, ref_b = arena.copy(), bp.copy()
        want_cs, want_last = o.commit(ref_arena, ref_b, 9, last)
        cases.append((bp, arena, last, ref_arena, ref_b, want_cs, want_last))
    for kind in ("hbm", "pageable", "registered"):
        for k, (bp0, arena0, last, ref_arena, ref_b, want_cs, want_last) in enumerate(cases):
            bp = bp0.copy()
            if kind == "hbm":
                d = torch.from_numpy(arena0.copy()).to(dev)
                cs, last2, leg = sc.commit(d.data_ptr(), bp, 9, last)
                got = d.cpu().numpy()
                assert leg == _lib.LEG_DEVICE
            else:
                raw = np.zeros(arena0.nbytes + 8192, dtype=np.uint8)
                off = (-raw.ctypes.data) % 4096
                host = raw[off:off + arena0.nbytes]
                host[:] = arena0
                if kind == "registered":
                    blocks.RegisterHostMemory(host)
                try:
                    cs, last2, leg = sc.commit(host.ctypes.data, bp, 9, last)
                finally:
                    if kind == "registered":
                        blocks.UnregisterHostMemory(host)
                got = host
                if kind == "pageable" or k == 0:
                    assert leg == _lib.LEG_HOST, (kind, k)
            assert np.array_equal(cs, want_cs), (kind, k)
            assert np.array_equal(bp["address"], ref_b["address"]) and last2 == want_last
            assert np.array_equal(got, ref_arena), (kind, k)
