"""GPU parity of the LDS-DMA kernel for per-block lengths and gathered offsets
(k_xxh64_glds_var, storm_amd/csrc/kernels.h): the batch shape storm produces, dirty
slots of cache.data with mixed Sizeof(T) (/root/reference/cache/cache.go:36-40,
blocks/objectlist/block.go:29-40, blocks/blob/block.go:25-29). Every block is compared
with the C oracle (XXH64 seed 0 = blocks.Checksum, blocks/checksum.go:15-17).

* all 4M blocks of a gather over a 128 GiB arena of 32 KiB slots, lengths drawn from
  storm's leaf and node sizes (31,808 / 30,000 / 32,768 / 28,808 B), in a shuffled slot
  order: the persistent, 4 KiB-skewed form;
* the edges, in each workgroup shape (2 waves, 8 waves, persistent 8 waves): lengths
  0..31 (no stripe), whole tiles, partial last tiles, blocks of more than 64 tiles,
  8-byte- and byte-aligned gathered starts (not staged: hashed from global memory by
  their quad), runs of such blocks long enough that whole waves have no tile, a
  partial last workgroup; verify with planted mismatches on the per-block-length path.
"""
import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

STORM_LENS = np.array([31808, 30000, 32768, 28808], dtype=np.uint32)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.timeout(600)
def test_gather_4m_blocks_storm_lengths(dev):
    from storm_amd import engine
    n, slot = 4 << 20, 32768
    rng = np.random.default_rng(3)
    perm = rng.permutation(n).astype(np.uint64)  # block i lives in slot perm[i]
    lens = STORM_LENS[rng.integers(0, 4, size=n)]
    arena = torch.empty((n, slot), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr(), slot, n, 5, o.SYNTH_SEED)
    d_offs = torch.from_numpy((perm * np.uint64(slot)).view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    engine.checksum_gather_device(arena.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    e0.record()
    engine.checksum_gather_device(arena.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"gather 4M storm-length blocks: {ms:.3f} ms, {int(lens.sum()) / (ms * 1e-3) / 1e9:.0f} GB/s")
    got = _u64(out)
    lens_by_slot = np.empty(n, dtype=np.uint32)
    lens_by_slot[perm] = lens
    want_by_slot = np.empty(n, dtype=np.uint64)
    piece = 1 << 17
    for c0 in range(0, n, piece):
        host = arena[c0:c0 + piece].cpu().numpy()
        want_by_slot[c0:c0 + piece] = o.checksum_batch(host, piece, slot, 0, lens=lens_by_slot[c0:c0 + piece],
                                                       threads=16)
    bad = np.nonzero(got != want_by_slot[perm])[0]
    assert bad.size == 0, f"{bad.size} of {n} blocks differ from the oracle, first {int(bad[0])}"


def _edge_layout(rng, n, slot, unaligned_share, long_runs):
    """Per-block lengths and gathered offsets inside slots of `slot` bytes."""
    kinds = rng.integers(0, 6, size=n)
    lens = np.empty(n, dtype=np.int64)
    room = slot - 16
    lens[kinds == 0] = rng.integers(0, 32, size=int((kinds == 0).sum()))                  # no stripe
    k1 = kinds == 1
    lens[k1] = np.minimum(rng.integers(1, room // 512 + 1, size=int(k1.sum())) * 512, room)  # whole tiles
    k2 = kinds >= 2
    lens[k2] = rng.integers(32, room + 1, size=int(k2.sum()))                              # partial last tile
    extra = np.zeros(n, dtype=np.int64)
    u = rng.random(n) < unaligned_share
    extra[u] = rng.choice([8, 1, 4, 12], size=int(u.sum()))
    for start, length, kind in long_runs:  # whole waves without a staged block
        if kind == "unaligned":
            extra[start:start + length] = 8
        else:
            lens[start:start + length] = rng.integers(0, 32, size=length)
    lens = np.minimum(lens, slot - extra)
    offs = np.arange(n, dtype=np.int64) * slot + extra
    return lens.astype(np.uint32), offs.astype(np.uint64)


EDGE_CASES = [
    # n, slot bytes: 2-wave workgroups; blocks up to ~65 KiB (more than 64 tiles)
    (16_391, 66_560),
    # 8-wave workgroups, one group each
    (30_011, 8_192),
    # persistent 8-wave workgroups, waves 4 KiB apart (the host's tile estimate for
    # per-block lengths is 32 KiB per block, so this batch size takes it)
    (2_000_003, 1_024),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,slot", EDGE_CASES)
def test_var_kernel_edges(dev, n, slot):
    from storm_amd import engine
    rng = np.random.default_rng(n)
    runs = [(1024, 300, "unaligned"), (n // 2, 257, "short")]
    lens, offs = _edge_layout(rng, n, slot, 0.03, runs)
    host = rng.integers(0, 256, size=n * slot + 64, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    want = o.checksum_gather(host, offs, lens=lens, threads=16)
    bad = np.nonzero(_u64(out) != want)[0]
    assert bad.size == 0, (n, slot, bad.size, bad[:8], lens[bad[:8]], offs[bad[:8]] % 16)
    # the same blocks through base + stride with per-block lengths (aligned rows: the
    # same kernel without offsets), then verify with planted mismatches
    want_s = o.checksum_batch(host, n, slot, 0, lens=lens, threads=16)
    out_s = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_device(d.data_ptr(), slot, n, out_s.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    bad = np.nonzero(_u64(out_s) != want_s)[0]
    assert bad.size == 0, (n, slot, "stride", bad.size, bad[:8])
    planted = np.sort(rng.choice(n, size=5, replace=False))
    exp = want_s.copy()
    exp[planted] ^= np.uint64(1)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d.data_ptr(), slot, n, torch.from_numpy(exp.view(np.int64)).to(dev).data_ptr(),
                         res.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [int(planted[0]), 5]
    # a uniform length through gathered offsets (the gather entry point without lengths)
    L = int(min(lens.max(), slot - 16)) // 3 + 5
    aligned_offs = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    d_aoffs = torch.from_numpy(aligned_offs.view(np.int64)).to(dev)
    engine.checksum_gather_device(d.data_ptr(), d_aoffs.data_ptr(), n, out.data_ptr(), L, 0)
    torch.cuda.synchronize()
    want_u = o.checksum_batch(host, n, slot, L, threads=16)
    bad = np.nonzero(_u64(out) != want_u)[0]
    assert bad.size == 0, (n, slot, "uniform gather", bad.size, bad[:8])


@pytest.mark.timeout(600)
def test_gather_locality_order_repeats(dev):
    """The locality order (kernels.h k_order_*) on a gather that repeats slots: 1.2M
    draws with replacement from 1.25M slots of 16 KiB, so 32 MiB regions hold ~2,048
    entries each, some more than the in-LDS sort takes (left in placement order) and
    some fewer (sorted), with equal offsets in one region."""
    from storm_amd import engine
    slots, slot, n = 1_250_000, 16384, 1_200_000
    rng = np.random.default_rng(11)
    slot_len = rng.integers(0, slot + 1, size=slots).astype(np.uint32)
    pick = rng.integers(0, slots, size=n).astype(np.uint64)
    lens = slot_len[pick]
    arena = torch.empty((slots, slot), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr(), slot, slots, 7, o.SYNTH_SEED)
    d_offs = torch.from_numpy((pick * np.uint64(slot)).view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(arena.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    counts = np.bincount((pick * np.uint64(slot) >> np.uint64(25)).astype(np.int64))
    assert counts.max() > 2048 and counts.min() <= 2048  # both sides of the sort limit
    want_by_slot = np.empty(slots, dtype=np.uint64)
    piece = 1 << 17
    for c0 in range(0, slots, piece):
        host = arena[c0:c0 + piece].cpu().numpy()
        m = host.shape[0]
        want_by_slot[c0:c0 + m] = o.checksum_batch(host, m, slot, 0, lens=slot_len[c0:c0 + m], threads=16)
    bad = np.nonzero(_u64(out) != want_by_slot[pick])[0]
    assert bad.size == 0, f"{bad.size} of {n} blocks differ from the oracle, first {int(bad[0])}"


@pytest.mark.timeout(300)
def test_length_bound_picks_the_kernel_not_the_result(dev):
    """With per-block lengths the caller may pass the longest length as `len`: batches of
    short blocks (storm's `-tags test` sizes) then take the register quad kernel instead
    of k_xxh64_glds_var (stormck.hip kVarMinLen). Every bound, none included, gives the
    oracle's checksums, gathered and strided."""
    from storm_amd import engine
    n, slot = 300_000, 1024
    rng = np.random.default_rng(17)
    lens = rng.choice([256, 536, 728], size=n).astype(np.uint32)
    host = rng.integers(0, 256, size=n * slot, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    offs = (rng.permutation(n).astype(np.uint64) * np.uint64(slot))
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    want_s = o.checksum_batch(host, n, slot, 0, lens=lens, threads=16)
    want_g = o.checksum_gather(host, offs, lens=lens, threads=16)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    for bound in (0, 728, 100, 1 << 20):  # none, exact, below the real longest, far above
        engine.checksum_device(d.data_ptr(), slot, n, out.data_ptr(), bound, d_lens.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(_u64(out), want_s), ("strided", bound)
        engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), bound, d_lens.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(_u64(out), want_g), ("gather", bound)
