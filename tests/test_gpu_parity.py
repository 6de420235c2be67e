"""GPU parity: the gfx950 kernels through the C-ABI vs the oracle and the golden
fixtures. Bit-exact (integer work). Runs on the MI355X box: pytest -m gpu.

Reference behaviour pinned: blocks.Checksum / BlockChecksum / VerifyChecksum
(/root/reference/blocks/checksum.go:10-27) = XXH64 seed 0 over the block bytes.
"""
import os

import numpy as np
import pytest

from tests.conftest import hx, load_golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    assert _lib.device_count() > 0, "GPU visible to torch but libstormck finds no gfx950 device"
    return torch.device("cuda:0")


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


# ---------------------------------------------------------------------------
# known answers / lengths / tails
# ---------------------------------------------------------------------------

def test_kat_lengths_device(dev):
    from storm_amd import engine
    rows = load_golden("kat.json")["rows"]
    stride = max(r["len"] for r in rows) + 8
    stride = (stride + 15) // 16 * 16
    for pattern in ("zeros", "iota"):
        host = np.zeros((len(rows), stride), dtype=np.uint8)
        if pattern == "iota":
            host[:] = (np.arange(stride) & 0xFF).astype(np.uint8)
        lens = torch.tensor([r["len"] for r in rows], dtype=torch.int32, device=dev)
        out = engine.checksum_tensor(_to_dev(host, dev), lens=lens)
        torch.cuda.synchronize()
        assert [int(v) for v in _u64(out)] == [hx(r[pattern]) for r in rows]


@pytest.fixture(params=["host", "gpu"])
def single(request, dev, monkeypatch):
    """Runs a single-call test through both legs: blocks.Checksum (the host latency leg,
    stormck_checksum) and the device single call (stormck_checksum_gpu,
    k_xxh64_single). BlockChecksum / VerifyChecksum call the module's Checksum."""
    from storm_amd import blocks
    if request.param == "gpu":
        monkeypatch.setattr(blocks, "Checksum", blocks.ChecksumGPU)
    return request.param


def test_public_answers_single_call(single):
    from storm_amd import blocks
    for s, v in load_golden("kat.json")["public"].items():
        assert blocks.Checksum(s.encode()) == hx(v)


def test_single_call_latency_path_lengths(dev):
    """stormck_checksum_gpu (one blocks.Checksum call on the device): slices up to 64 KiB
    go through the one-launch kernel that reads pinned host memory (every staging round
    count 1..16, clamped last round), longer ones through the host pipeline. Unaligned
    Python views exercise the host-side copy."""
    from oracle import oracle as o
    from storm_amd import blocks
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=(1 << 17) + 64, dtype=np.uint8)
    lengths = list(range(0, 100)) + [72, 255, 256, 4095, 4096, 4097, 28808, 30000, 31808, 32768,
                                     65535, 65536, 65537, 100000, 1 << 17]
    for L in lengths:
        for off in (0, 3):
            sl = data[off:off + L]  # numpy view: off = 3 hands the library an unaligned pointer
            assert blocks.ChecksumGPU(sl) == o.xxh64(sl), (L, off)
            assert blocks.Checksum(sl) == o.xxh64(sl), (L, off)


def test_single_call_length_limits(dev):
    """The device single call takes up to the 256 MiB staging chunk (a batch of one
    through the host pipeline) and refuses longer slices with EINVAL; the single-call
    leg blocks.Checksum hashes any length (stormck.h)."""
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    rng = np.random.default_rng(6)
    big = rng.integers(0, 256, size=(256 << 20) + 1, dtype=np.uint8)
    want = o.xxh64(big[:256 << 20])
    assert blocks.ChecksumGPU(big[:256 << 20]) == want
    with pytest.raises(_lib.StormckError) as e:
        blocks.ChecksumGPU(big)
    assert e.value.code == _lib.EINVAL and "256 MiB" in str(e.value)
    assert blocks.Checksum(big) == o.xxh64(big)


# ---------------------------------------------------------------------------
# c1: 1K synthetic 32 KiB blocks; generator parity
# ---------------------------------------------------------------------------

def test_synth_c1_device(dev):
    from storm_amd import engine
    g = load_golden("synth_c1.json")
    n, stride = g["n"], g["stride"]
    buf = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), stride, n, 0, hx(g["seed"]))
    out = engine.checksum_tensor(buf)
    torch.cuda.synchronize()
    assert [int(v) for v in _u64(out)] == [hx(v) for v in g["checksums"]]
    words = buf.cpu().numpy().view("<u8")
    for s in g["generator_samples"]:
        assert int(words[s["block"], s["word"]]) == hx(s["value"])


def test_synth_vs_oracle_random_lengths(dev):
    """Random lengths/offsets (ragged, unaligned) vs the C oracle."""
    from oracle import oracle as o
    from storm_amd import engine
    rng = np.random.default_rng(11)
    n, stride = 3000, 4096 + 64
    host = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    lens = rng.integers(0, 4096, size=n).astype(np.uint32)
    lens[:40] = np.arange(40)
    offs = (np.arange(n, dtype=np.uint64) * stride + rng.integers(0, 57, size=n).astype(np.uint64))
    want = np.array([o.xxh64(host[int(offs[i]):int(offs[i]) + int(lens[i])]) for i in range(n)], dtype=np.uint64)
    d = _to_dev(host, dev)
    d_offs = _to_dev(offs.view(np.int64), dev)
    d_lens = _to_dev(lens.view(np.int32), dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), want)
    # uniform length, odd base alignment through the strided entry point
    out2 = torch.empty(n - 1, dtype=torch.int64, device=dev)
    engine.checksum_device(d.data_ptr() + 3, stride, n - 1, out2.data_ptr(), 1000)
    torch.cuda.synchronize()
    want2 = o.checksum_batch(host[3:], n - 1, stride, 1000)
    assert np.array_equal(_u64(out2), want2)


@pytest.mark.parametrize("n", [1, 7, 128, 129, 1202, 1280, 1281])
def test_wide_path_premultiplied_staging(dev, n):
    """Batches of <= 128 blocks take k_xxh64_wide: blocks whose start is 8-byte aligned
    (shift 0 or 8 within their 16-byte cover) are staged with their stripe words
    premultiplied by P2; other starts, and covers over 32 KiB, take the plain path.
    129 to 5 blocks per CU (1,280 on MI355X; 1,202 = a storm commit batch) take
    k_xxh64_wide_multi, 5 staged blocks per workgroup; 1,281 the register-quad kernel.
    Random starts 0..56 mod 16 and lengths up to 32 KiB (incl. 32760 at shift 8, the
    largest premultiplied stage), checksum and verify, vs the C oracle."""
    from oracle import oracle as o
    from storm_amd import engine
    rng = np.random.default_rng(100 + n)
    stride = 32768 + 64
    host = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    lens = rng.integers(0, 32769, size=n).astype(np.uint32)
    shifts = rng.integers(0, 57, size=n).astype(np.uint64)
    if n >= 7:
        lens[:7] = [0, 31, 32, 33, 32760, 32768, 4096]
        shifts[:7] = [8, 8, 0, 8, 8, 0, 24]
    offs = np.arange(n, dtype=np.uint64) * stride + shifts
    want = np.array([o.xxh64(host[int(offs[i]):int(offs[i]) + int(lens[i])]) for i in range(n)], dtype=np.uint64)
    d = _to_dev(host, dev)
    d_offs = _to_dev(offs.view(np.int64), dev)
    d_lens = _to_dev(lens.view(np.int32), dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), want)
    # uniform length on an 8-byte (not 16-byte) aligned base: every block at shift 8
    out2 = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_device(d.data_ptr() + 8, stride, n, out2.data_ptr(), 30000)
    torch.cuda.synchronize()
    want2 = o.checksum_batch(host[8:], n, stride, 30000)
    assert np.array_equal(_u64(out2), want2)
    # verify through the same kernel (VERIFY=true)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    exp = _to_dev(want2.view(np.int64), dev)
    engine.verify_device(d.data_ptr() + 8, stride, n, exp.data_ptr(), res.data_ptr(), 30000)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [n, 0]
    bad = want2.copy()
    bad[n - 1] ^= 1
    engine.verify_device(d.data_ptr() + 8, stride, n, _to_dev(bad.view(np.int64), dev).data_ptr(), res.data_ptr(),
                         30000)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [n - 1, 1]


@pytest.mark.parametrize("length", [512, 513, 520, 1000, 8192, 28808, 30000, 31808, 32768])
def test_uniform_fast_path_lengths(dev, length):
    """Uniform-length 16-byte-aligned batches of every batch-size class: <= 128 blocks
    (one workgroup per block), below 36 blocks per CU (register quad), up to kBigW
    (LDS-staged streaming kernel in 8-, 3- or 1-wave workgroups, whichever loads the
    busiest CU least), then 8-wave workgroups: whole tiles, remainder stripes and tails,
    partial last workgroup."""
    from oracle import oracle as o
    from storm_amd import engine
    rng = np.random.default_rng(length)
    stride = (length + 15) // 16 * 16 + 16 * (length % 3)
    for n in (1, 63, 64, 65, 1000):
        host = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
        out = engine.checksum_tensor(_to_dev(host, dev), length=length)
        torch.cuda.synchronize()
        want = o.checksum_batch(host, n, stride, length)
        assert np.array_equal(_u64(out), want), (length, n)
        if n == 65:  # verify through the one-workgroup-per-block kernel
            exp = torch.from_numpy(want.view(np.int64).copy()).to(dev)
            exp[64] ^= 1
            exp[9] ^= 1
            res = torch.zeros(2, dtype=torch.int64, device=dev)
            engine.verify_device(_to_dev(host, dev).data_ptr(), stride, n, exp.data_ptr(), res.data_ptr(), length)
            torch.cuda.synchronize()
            assert _u64(res).tolist() == [9, 2], length
    # verify through the same path
    d = _to_dev(host, dev)
    exp = torch.from_numpy(want.view(np.int64).copy()).to(dev)
    exp[999] ^= 1
    exp[500] ^= 1
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d.data_ptr(), stride, 1000, exp.data_ptr(), res.data_ptr(), length)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [500, 2]
    # streaming-kernel batches: device-generated blocks, partial last workgroups, then
    # verify. On 256 CUs 9,300 and 10,257 take 3-wave workgroups, 16,389 1-wave ones,
    # 24,641 and 32,768 the 8-wave ones, 36,864 3-wave ones again.
    for n in (9300, 10240 + 17, 16384 + 5, 24576 + 65, 32768, 36864):
        big = torch.empty((n, stride), dtype=torch.uint8, device=dev)
        engine.fill_synthetic_device(big.data_ptr(), stride, n, length, 0x1234)
        out = engine.checksum_tensor(big, length=length)
        torch.cuda.synchronize()
        want = o.checksum_batch(big.cpu().numpy(), n, stride, length, threads=8)
        assert np.array_equal(_u64(out), want), (length, n)
        exp = torch.from_numpy(want.view(np.int64).copy()).to(dev)
        exp[n - 1] ^= 1
        exp[min(10000, n // 2)] ^= 1
        exp[7] ^= 1
        res = torch.zeros(2, dtype=torch.int64, device=dev)
        engine.verify_device(big.data_ptr(), stride, n, exp.data_ptr(), res.data_ptr(), length)
        torch.cuda.synchronize()
        assert _u64(res).tolist() == [7, 3], (length, n)
        del big


@pytest.mark.parametrize("shift,n", [(0, 700), (8, 700), (8, 1900), (0, 2049), (8, 3500), (0, 4096), (8, 4097)])
def test_wide_multi_ring_long_blocks(dev, shift, n):
    """Batches of up to 16 blocks per CU take k_xxh64_wide_multi, whose pipelined staging
    streams each block through a 4-slot ring (kernels.h multi_stage_hash_pipe): 4 KiB
    chunks at 5 and 8 blocks per workgroup (700, 1,900 blocks), 2 KiB chunks at 16
    (2,049 .. 4,096 blocks); 4,097 takes the register-quad kernel, for comparison. Random
    per-block lengths up to 64 KiB - 8 (covers of up to 16 / 32 chunks, stripes and tails
    straddling chunk and ring-wrap boundaries, empty blocks), 16- and 8-byte-aligned
    starts; then uniform 32 KiB blocks (storm's blob, a cover of 2,048 or 2,049 pieces) in
    the same batch-size class; every block vs the C oracle, and verify finds planted
    mismatches."""
    from oracle import oracle as o
    from storm_amd import engine
    rng = np.random.default_rng(n + shift)
    stride = 65552
    lens = rng.integers(0, 65536 - 8, size=n).astype(np.uint32)
    lens[:6] = [0, 1, 32, 4096 - shift, 4096 - shift + 31, 65536 - 16]
    host = rng.integers(0, 256, size=shift + n * stride + 64, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_device(d.data_ptr() + shift, stride, n, out.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    want = o.checksum_batch(host[shift:], n, stride, 0, lens=lens, threads=8)
    bad = np.nonzero(_u64(out) != want)[0]
    assert bad.size == 0, (shift, bad[:8], lens[bad[:8]])
    exp = want.copy()
    exp[[5, n - 1]] ^= np.uint64(1)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d.data_ptr() + shift, stride, n, torch.from_numpy(exp.view(np.int64)).to(dev).data_ptr(),
                         res.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [5, 2], (shift, n)
    m, L = min(n, 4100), 32768
    blob = rng.integers(0, 256, size=shift + m * L + 64, dtype=np.uint8)
    d2 = torch.from_numpy(blob).to(dev)
    out2 = torch.empty(m, dtype=torch.int64, device=dev)
    engine.checksum_device(d2.data_ptr() + shift, L, m, out2.data_ptr(), L)
    torch.cuda.synchronize()
    want2 = o.checksum_batch(blob[shift:], m, L, L, threads=8)
    assert np.array_equal(_u64(out2), want2), shift
    exp = want2.copy()
    exp[[3, m - 2]] ^= np.uint64(1)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d2.data_ptr() + shift, L, m, torch.from_numpy(exp.view(np.int64)).to(dev).data_ptr(),
                         res.data_ptr(), L)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [3, 2]


def test_mixed_c5(dev):
    from storm_amd import engine
    g = load_golden("mixed.json")
    lens = g["lens"]
    n, stride = len(lens), g["stride"]
    buf = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), stride, n, g["first"], hx(g["seed"]))
    out = engine.checksum_tensor(buf, lens=torch.tensor(lens, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    assert [int(v) for v in _u64(out)] == [hx(v) for v in g["checksums"]]


def test_empty_and_zero(dev):
    from storm_amd import blocks, engine
    assert blocks.Checksum(b"") == 0xEF46DB3751D8E999
    assert blocks.ChecksumGPU(b"") == 0xEF46DB3751D8E999
    engine.checksum_device(0, 0, 0, 0, 0)  # n == 0 is a no-op
    buf = torch.zeros((4, 64), dtype=torch.uint8, device=dev)
    out = engine.checksum_tensor(buf, length=0)
    torch.cuda.synchronize()
    assert all(int(v) == 0xEF46DB3751D8E999 for v in _u64(out))


# ---------------------------------------------------------------------------
# full-size configs: c2 (1M blocks, 32 GiB resident) and c3 (16M blocks via a
# 4M-block arena, 4 passes) against the libxxhash digests + oracle spot checks
# ---------------------------------------------------------------------------

def _digest_check(dev, n_total, arena_blocks):
    from oracle import oracle as o
    from storm_amd import engine
    digests = load_golden("synth_digests.json")["digests"][str(n_total)]
    stride = 32768
    arena = torch.empty((arena_blocks, stride), dtype=torch.uint8, device=dev)
    cs = torch.empty(n_total, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(n_total)
    for first in range(0, n_total, arena_blocks):
        cnt = min(arena_blocks, n_total - first)
        engine.fill_synthetic_device(arena.data_ptr(), stride, cnt, first, o.SYNTH_SEED)
        engine.checksum_device(arena.data_ptr(), stride, cnt, cs[first:].data_ptr(), stride)
        torch.cuda.synchronize()
        # spot-check 64 random blocks of this pass with the oracle on the host
        idx = rng.integers(0, cnt, size=64)
        sample = arena[torch.from_numpy(idx).to(dev)].cpu().numpy()
        want = o.checksum_batch(sample, 64, stride, stride)
        assert np.array_equal(_u64(cs[first + torch.from_numpy(idx).to(dev)]), want)
    host = _u64(cs)
    assert [int(v) for v in host[:8]] == [hx(v) for v in digests["first8"]]
    assert [int(v) for v in host[::65536]] == [hx(v) for v in digests["every_65536th"]]
    assert o.xxh64(host.astype("<u8").tobytes()) == hx(digests["digest"])
    del arena


@pytest.mark.slow
@pytest.mark.parametrize("length", [28808, 32768])
def test_large_batch_skewed_kernel(dev, length):
    """Batches that give every CU thousands of tiles take the persistent, 4 KiB-skewed
    streaming kernel (k_xxh64_glds_skew). 2.3M blocks, not a multiple of the 128-block
    group, at a storm length with remainder stripes and a tail (28808 B: 56 tiles + 4
    stripes + 8 B) and at 32 KiB: equal to the oracle on EVERY block (the arena comes
    back to the host in 4 GiB pieces), equal to the per-block-length (quad) path, and
    verify finds planted mismatches."""
    from oracle import oracle as o
    from storm_amd import engine
    n, stride = 2_300_003, 32768
    arena = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr(), stride, n, 77, o.SYNTH_SEED)
    fast = engine.checksum_tensor(arena, length=length)
    lens = torch.full((n,), length, dtype=torch.int32, device=dev)
    quad = engine.checksum_tensor(arena, lens=lens)
    torch.cuda.synchronize()
    assert torch.equal(fast, quad)
    got = _u64(fast)
    piece = 1 << 17
    for c0 in range(0, n, piece):
        cnt = min(piece, n - c0)
        host = arena[c0:c0 + cnt].cpu().numpy()
        want = o.checksum_batch(host, cnt, stride, length, threads=16)
        bad = np.nonzero(got[c0:c0 + cnt] != want)[0]
        assert bad.size == 0, f"{bad.size} blocks differ from the oracle, first {c0 + int(bad[0])}"
    exp = fast.clone()
    exp[n - 1] ^= 1
    exp[1_000_000] ^= 1
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(arena.data_ptr(), stride, n, exp.data_ptr(), res.data_ptr(), length)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [1_000_000, 2]
    del arena, lens


@pytest.mark.slow
def test_c2_1m_blocks_digest(dev):
    _digest_check(dev, 1 << 20, 1 << 20)


@pytest.mark.slow
def test_c3_16m_blocks_digest(dev):
    _digest_check(dev, 1 << 24, 1 << 22)


# ---------------------------------------------------------------------------
# verify (blocks.VerifyChecksum batched)
# ---------------------------------------------------------------------------

def test_verify_device_and_host(dev):
    from storm_amd import blocks, engine
    n, stride = 5000, 1024
    buf = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), stride, n, 77, 0x1234)
    good = engine.checksum_tensor(buf)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(buf.data_ptr(), stride, n, good.data_ptr(), res.data_ptr(), stride)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [n, 0]
    bad = good.clone()
    for i in (4321, 17, 4999):
        bad[i] ^= 1
    engine.verify_device(buf.data_ptr(), stride, n, bad.data_ptr(), res.data_ptr(), stride)
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [17, 3]
    # host path: corrupt one byte of block 123
    host = buf.cpu().numpy().copy()
    exp = _u64(good)
    assert blocks.VerifyChecksumBatchGPU(host, n, stride, exp, length=stride) == (n, 0)
    host[123, 5] ^= 0xFF
    assert blocks.VerifyChecksumBatchGPU(host, n, stride, exp, length=stride) == (123, 1)


def test_host_batch_paths(dev):
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    rng = np.random.default_rng(3)
    n, stride = 20000, 32768  # 625 MiB: several 256 MiB pipeline chunks
    host = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
    want = o.checksum_batch(host, n, stride, stride, threads=8)
    assert np.array_equal(blocks.ChecksumBatchGPU(host, n, stride, length=stride), want)
    lens = rng.integers(0, stride + 1, size=n)
    want_l = o.checksum_batch(host, n, stride, lens=lens, threads=8)
    assert np.array_equal(blocks.ChecksumBatchGPU(host, n, stride, lens=lens), want_l)
    # registered (pinned) memory is DMA'd directly
    _lib.check(_lib.lib.stormck_host_register(host.ctypes.data, host.nbytes))
    try:
        assert np.array_equal(blocks.ChecksumBatchGPU(host, n, stride, length=stride), want)
    finally:
        _lib.check(_lib.lib.stormck_host_unregister(host.ctypes.data))


# ---------------------------------------------------------------------------
# Go API mirror, with the reference's relational tests
# ---------------------------------------------------------------------------

def test_pointer_block_checksum_sequence(single):
    # /root/reference/blocks/pointer/block_test.go:11-35
    from storm_amd import blocks, layouts
    seq = [hx(v) for v in load_golden("layouts.json")["pointer_block_test_sequence"]]
    b = layouts.PointerBlock()
    got = [blocks.BlockChecksum(b)]
    b.Pointers[0].Checksum = 2
    got.append(blocks.BlockChecksum(b))
    b.PointedBlockTypes[0] = blocks.LeafBlockType
    got.append(blocks.BlockChecksum(b))
    b.PointedBlockTypes[1] = blocks.LeafBlockType
    got.append(blocks.BlockChecksum(b))
    b.Pointers[1].Address = 2
    got.append(blocks.BlockChecksum(b))
    b.Pointers[2].Checksum = 4
    got.append(blocks.BlockChecksum(b))
    assert got == seq
    assert len(set(got)) == len(got)  # every field change changes the checksum


def test_zero_blocks_and_singularity(single):
    from storm_amd import blocks, layouts
    g = load_golden("layouts.json")
    for tag in ("prod", "test"):
        test_tag = tag == "test"
        f = layouts.TEST_FANOUT if test_tag else None
        types = {
            "singularity": layouts.SingularityBlock,
            "pointer": layouts.pointer_block(f or layouts.POINTERS_PER_BLOCK),
            "spacelist": layouts.spacelist_block(f or layouts.SPACES_PER_BLOCK),
            "objectlist": layouts.objectlist_block(f or layouts.CHUNKS_PER_BLOCK),
            "blob": layouts.BlobBlock,
        }
        for name, T in types.items():
            assert blocks.BlockChecksum(T()) == hx(g["zero_block_checksums"][tag][name]), (tag, name)
    # singularity round trip (cache/cache_test.go:23-42): checksum over the block with Checksum = 0
    s = layouts.SingularityBlock.from_buffer_copy(bytes.fromhex(g["singularity_example"]["bytes_hex"]))
    s.Checksum = 0
    cs = blocks.BlockChecksum(s)
    assert cs == hx(g["singularity_example"]["checksum"])
    s.Checksum = cs
    copy = layouts.SingularityBlock.from_buffer_copy(bytes(s))
    copy.Checksum = 0
    assert blocks.VerifyChecksum(0, bytes(copy), cs) is None


def test_verify_checksum_error_format(single):
    # blocks/checksum.go:25-26: "checksum mismatch for block %d, computed: %#v, expected: %#v"
    from storm_amd import blocks
    err = blocks.VerifyChecksum(42, b"abc", 0)
    assert isinstance(err, blocks.ChecksumMismatchError)
    assert str(err) == "checksum mismatch for block 42, computed: 0x44bc2cf5ad770999, expected: 0x0"
    assert blocks.VerifyChecksum(42, b"abc", 0x44BC2CF5AD770999) is None


def test_blob_block_change_changes_checksum(single):
    # blocks/blob/block_test.go:13-49
    from storm_amd import blocks, layouts
    g = load_golden("layouts.json")["blob_test_block"]
    b = layouts.BlobBlock()
    before = blocks.BlockChecksum(b)
    raw = bytes.fromhex(g["first_128_hex"])
    ctypes_buf = (layouts.ctypes.c_uint8 * 128).from_buffer(b.Data)
    ctypes_buf[:] = raw
    after = blocks.BlockChecksum(b)
    assert after != before
    assert after == hx(g["checksum"])


# ---------------------------------------------------------------------------
# Merkle pointer tree
# ---------------------------------------------------------------------------

def test_merkle_roots_device(dev):
    from oracle import oracle as o
    from storm_amd import engine
    g = load_golden("merkle.json")
    for c in g["cases"]:
        leaf = o.synth_leaf_checksums(c["n"], hx(g["seed"]))
        d_leaf = _to_dev(leaf.view(np.int64), dev)
        root = engine.merkle_root_tensor(d_leaf, c["leaf_addr_base"], c["node_addr_base"], c["rev"], c["fanout"])
        r = engine.as_tuple(root)
        assert list(r[:3]) == [hx(v) for v in c["root"]], c
        assert r[3] == c["root_type"], c


def test_pack_pointer_blocks_materialised(dev):
    """Materialised pointer blocks hash to the fused level kernel's checksums."""
    from oracle import oracle as o
    from storm_amd import engine
    for fanout, m in ((1200, 5000), (10, 95)):
        leaf = o.synth_leaf_checksums(m)
        d_leaf = _to_dev(leaf.view(np.int64), dev)
        pm = (m + fanout - 1) // fanout
        size = o.pointer_block_size(fanout)
        stride = (size + 15) // 16 * 16
        blocks_buf = torch.zeros((pm, stride), dtype=torch.uint8, device=dev)
        engine.pack_pointer_blocks_device(d_leaf.data_ptr(), m, 900, 3, 2, fanout, blocks_buf.data_ptr(), stride)
        fused = torch.empty(pm, dtype=torch.int64, device=dev)
        engine.pointer_level_device(d_leaf.data_ptr(), m, 900, 3, 2, fanout, fused.data_ptr())
        via_bytes = engine.checksum_tensor(blocks_buf, length=size)
        torch.cuda.synchronize()
        assert np.array_equal(_u64(fused), _u64(via_bytes))
        host = blocks_buf.cpu().numpy()
        for j in range(pm):
            ent = [(int(leaf[k]), 900 + k, 3, 2) for k in range(j * fanout, min(m, (j + 1) * fanout))]
            assert bytes(host[j, :size]) == o.pack_pointer_block_py(ent, fanout)


@pytest.mark.parametrize("m", [257 * 1200, 300 * 1200 + 1, 4000 * 1200 - 7, 320 * 1200])
def test_pointer_level_ring_kernel(dev, m):
    """Levels of more than 256 nodes at storm's fan-out take k_pointer_level_pc (a
    producer wave and a chain wave per 16 nodes, premultiplied words staged in LDS). Shapes: full last wave (320
    nodes), a last wave holding 1 node and 15 idle quads (257), a last node with one
    child (300 + 1), and a ragged 4,000-node level; addresses and revision above 2^32.
    Equal to the materialised pointer blocks hashed by the batch kernels on every node,
    and to the oracle's packer + XXH64 on a sample."""
    from oracle import oracle as o
    from storm_amd import engine
    fanout, base, rev = 1200, (1 << 40) + 5, (1 << 33) + 1
    leaf = o.synth_leaf_checksums(m, 0x1234 + m)
    d_leaf = _to_dev(leaf.view(np.int64), dev)
    pm = (m + fanout - 1) // fanout
    fused = torch.empty(pm, dtype=torch.int64, device=dev)
    engine.pointer_level_device(d_leaf.data_ptr(), m, base, rev, 2, fanout, fused.data_ptr())
    size = o.pointer_block_size(fanout)
    stride = (size + 15) // 16 * 16
    blk = torch.zeros((pm, stride), dtype=torch.uint8, device=dev)
    engine.pack_pointer_blocks_device(d_leaf.data_ptr(), m, base, rev, 2, fanout, blk.data_ptr(), stride)
    via_bytes = engine.checksum_tensor(blk, length=size)
    torch.cuda.synchronize()
    got = _u64(fused)
    assert np.array_equal(got, _u64(via_bytes))
    for jn in sorted({0, 1, 15, 16, pm // 2, pm - 2, pm - 1}):
        ent = [(int(leaf[k]), base + k, rev, 2) for k in range(jn * fanout, min(m, (jn + 1) * fanout))]
        assert int(got[jn]) == o.xxh64(o.pack_pointer_block_py(ent, fanout)), jn


@pytest.mark.parametrize("knobs", [{"STORMCK_POINTER_RING": "1"}, {"STORMCK_POINTER_C": "2"},
                                   {"STORMCK_POINTER_C": "4"}, {"STORMCK_POINTER_C": "4", "STORMCK_POINTER_SIMD": "0"},
                                   {"STORMCK_POINTER_C": "0"}])
def test_pointer_level_probe_kernels(dev, knobs):
    """The Merkle level kernels behind probe knobs, which only the probe build
    (tools/libstormck_probes.so, -DSTORMCK_PROBES) has; each runs in a child that loads
    it (STORMCK_LIBRARY): the ring mode knob (STORMCK_POINTER_RING=1), 2 and 4 chain waves per
    workgroup with SIMD-ranked roles (pc_role<true>) or by wave index, and the C chosen
    per level (0). Ragged 13,982-, 6,991- and 300-node levels (the c3 and c4 shard
    levels); every node equal to the product library's default kernel in this process."""
    import subprocess
    import sys
    from oracle import oracle as o
    from storm_amd import engine
    from tests.conftest import ROOT
    fanout, base, rev = 1200, (1 << 40) + 5, (1 << 33) + 1
    sizes = [16 << 20, 8 << 20, 300 * 1200 + 1]
    want = []
    for m in sizes:
        leaf = o.synth_leaf_checksums(m, 0x77 + m)
        d_leaf = _to_dev(leaf.view(np.int64), dev)
        par = torch.empty((m + fanout - 1) // fanout, dtype=torch.int64, device=dev)
        engine.pointer_level_device(d_leaf.data_ptr(), m, base, rev, 2, fanout, par.data_ptr())
        torch.cuda.synchronize()
        want.append(_u64(par))
    code = ("import sys, numpy as np, torch\n"
            "from oracle import oracle as o\n"
            "from storm_amd import engine\n"
            f"for m in {sizes}:\n"
            f"    leaf = o.synth_leaf_checksums(m, 0x77 + m)\n"
            "    d = torch.from_numpy(leaf.view(np.int64)).to('cuda:0')\n"
            "    par = torch.empty((m + 1199) // 1200, dtype=torch.int64, device='cuda:0')\n"
            f"    engine.pointer_level_device(d.data_ptr(), m, {base}, {rev}, 2, 1200, par.data_ptr())\n"
            "    torch.cuda.synchronize()\n"
            "    np.save(sys.stdout.buffer, par.cpu().numpy().view(np.uint64))\n")
    from storm_amd import build as sb
    assert os.path.exists(sb.PROBES_LIB), "probe build missing: storm_amd.build.build_probes_lib()"
    env = dict(os.environ, STORMCK_LIBRARY=sb.PROBES_LIB, **knobs)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import io
    buf = io.BytesIO(r.stdout)
    for m, w in zip(sizes, want):
        got = np.load(buf)
        assert np.array_equal(got, w), (knobs, m, int((got != w).sum()))


def test_combine_roots_device(dev):
    from storm_amd import engine
    g = load_golden("merkle.json")["combine"]
    rows = [[hx(v) for v in r[:3]] + [r[3]] for r in g["shard_roots"]]
    table = torch.tensor(np.array(rows, dtype=np.uint64).view(np.int64), device=dev)
    groot = engine.combine_roots_tensor(table, g["rev"], 2 * g["n_total"], g["fanout"])
    r = engine.as_tuple(groot)
    assert list(r[:3]) == [hx(v) for v in g["global_root"][:3]]
    assert r[3] == g["global_root"][3]


def test_one_hip_runtime_whatever_the_import_order(dev):
    """storm_amd imported before torch must still share torch's HIP runtime
    (storm_amd/_lib.py loads torch first): a fresh process computes on both."""
    import subprocess
    import sys
    code = ("from storm_amd import blocks\n"
            "import torch\n"
            "x = torch.ones(4, device='cuda:0')\n"
            "assert blocks.ChecksumGPU(b'abc') == 0x44BC2CF5AD770999\n"
            "assert float(x.sum()) == 4.0\n"
            "print('ok')\n")
    from tests.conftest import ROOT
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_key_tags_f4(dev):
    """f4: xxhash.Sum64(key) for storm keys (keystore/keystore.go:33,66): 48-byte keys
    as in keystore/benchmark_test.go:27-32, and packed ragged keys of 1..256 bytes
    (objectlist.MaxKeyComponentLength) at arbitrary alignment; lane-per-key kernel ==
    oracle == the general quad path."""
    from oracle import oracle as o
    from storm_amd import engine
    rng = np.random.default_rng(48)
    n = 30000
    keys = rng.integers(0, 256, size=(n, 48), dtype=np.uint8)
    d = _to_dev(keys, dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.key_tags_device(d.data_ptr(), n, out.data_ptr(), stride=48, length=48)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), o.checksum_batch(keys, n, 48, 48))
    lens = rng.integers(1, 257, size=n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    packed = rng.integers(0, 256, size=int(lens.sum()), dtype=np.uint8)
    want = np.array([o.xxh64(packed[int(offs[i]):int(offs[i]) + int(lens[i])]) for i in range(n)], dtype=np.uint64)
    dp, do, dl = _to_dev(packed, dev), _to_dev(offs.view(np.int64), dev), _to_dev(lens.view(np.int32), dev)
    engine.key_tags_device(dp.data_ptr(), n, out.data_ptr(), d_offsets=do.data_ptr(), d_lens=dl.data_ptr())
    quad = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(dp.data_ptr(), do.data_ptr(), n, quad.data_ptr(), 0, dl.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), want)
    assert np.array_equal(_u64(quad), want)
    # fixed strides through the LDS-DMA batch path (+ the lane-kernel remainder):
    # stride 48/64/256, key lengths below the stride, n not a multiple of 64
    for stride, klen, m in ((48, 48, 64 * 100 + 17), (64, 40, 64 * 9), (256, 256, 64 * 3 + 63), (16, 5, 1000)):
        k2 = rng.integers(0, 256, size=(m, stride), dtype=np.uint8)
        d2 = _to_dev(k2, dev)
        o2 = torch.empty(m, dtype=torch.int64, device=dev)
        engine.key_tags_device(d2.data_ptr(), m, o2.data_ptr(), stride=stride, length=klen)
        torch.cuda.synchronize()
        assert np.array_equal(_u64(o2), o.checksum_batch(k2, m, stride, klen)), (stride, klen, m)
    # compile-time-stride ring (strides 16..64): every key length up to the stride (all
    # tail shapes of the b128-only LDS tail), full waves of 8 batches, a partial last
    # wave (3 batches) and a lane-kernel remainder (7 keys)
    m = 64 * 8 * 5 + 64 * 3 + 7
    for stride in (16, 32, 48, 64):
        k2 = rng.integers(0, 256, size=(m, stride), dtype=np.uint8)
        d2 = _to_dev(k2, dev)
        o2 = torch.empty(m, dtype=torch.int64, device=dev)
        for klen in range(0, stride + 1):
            engine.key_tags_device(d2.data_ptr(), m, o2.data_ptr(), stride=stride, length=klen)
            torch.cuda.synchronize()
            assert np.array_equal(_u64(o2), o.checksum_batch(k2, m, stride, klen)), (stride, klen)


def test_read_verify_fd_f2(dev, tmp_path):
    """f2/f3: batched cold read + verify from a file device (cache.fetchBlock =
    Store.ReadBlock + VerifyChecksum, cache/cache.go:139-167): data lands in the
    slots, clean blocks verify, corrupted ones are found, short reads are errors."""
    import os
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    rng = np.random.default_rng(7)
    nblocks, bs = 2048, 32768
    image = rng.integers(0, 256, size=(nblocks, bs), dtype=np.uint8)
    path = tmp_path / "dev.img"
    image.tofile(path)
    n = 1500
    addresses = rng.choice(nblocks, size=n, replace=False).astype(np.uint64)
    lens = rng.choice([72, 28808, 30000, 31808, 32768, 536], size=n).astype(np.uint32)
    expected = np.array([o.xxh64(image[a, :l]) for a, l in zip(addresses, lens)], dtype=np.uint64)
    dst = np.zeros((n, bs), dtype=np.uint8)
    fd = os.open(path, os.O_RDONLY)
    try:
        assert blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst, bs) == (n, 0)
        for i in range(0, n, 97):
            assert np.array_equal(dst[i, :lens[i]], image[addresses[i], :lens[i]])
        bad = expected.copy()
        bad[[900, 12]] ^= 1
        assert blocks.ReadVerifyBatch(fd, addresses, lens, bad, dst, bs) == (12, 2)
        with pytest.raises(_lib.StormckError):
            blocks.ReadVerifyBatch(fd, [nblocks + 5], [100], [0], dst, bs)
        dst2 = np.zeros((n, bs), dtype=np.uint8)
        assert blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst2, bs, full_block=True) == (n, 0)
        assert np.array_equal(dst2[5], image[addresses[5]])
    finally:
        os.close(fd)


def test_read_verify_fd_across_super_chunks(dev, tmp_path, monkeypatch):
    """f2: the reader pool runs ahead of the verifier across super-chunk boundaries
    (STORMCK_READ_SUPER_BYTES shrinks them from 1 GiB to 3 blocks here, ~700 of
    them). Clean batches verify in both read modes, and mismatches in late chunks keep
    their lowest index and count. A read past the end of the file names the lowest
    failing index."""
    import os
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    rng = np.random.default_rng(23)
    nblocks, bs = 1024, 4096
    image = rng.integers(0, 256, size=(nblocks, bs), dtype=np.uint8)
    path = tmp_path / "dev.img"
    image.tofile(path)
    n = 2100
    addresses = np.concatenate([np.arange(100, 400), rng.integers(0, nblocks, size=n - 300)]).astype(np.uint64)
    lens = rng.integers(1, bs + 1, size=n).astype(np.uint32)
    expected = np.array([o.xxh64(image[a, :l]) for a, l in zip(addresses, lens)], dtype=np.uint64)
    monkeypatch.setenv("STORMCK_READ_SUPER_BYTES", str(3 * bs))
    fd = os.open(path, os.O_RDONLY)
    try:
        for full in (False, True):
            dst = np.zeros((n, bs), dtype=np.uint8)
            got = blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst, bs, block_size=bs, full_block=full)
            assert got == (n, 0)
            assert np.array_equal(dst[250], image[addresses[250]]) if full else \
                np.array_equal(dst[250, :lens[250]], image[addresses[250], :lens[250]])
        bad = expected.copy()
        bad[[2050, 1777, 1778]] ^= 1
        assert blocks.ReadVerifyBatch(fd, addresses, lens, bad, dst, bs, block_size=bs) == (1777, 3)
        far = addresses.copy()
        far[[1900, 1500]] = nblocks + 7
        with pytest.raises(_lib.StormckError, match="block index 1500"):
            blocks.ReadVerifyBatch(fd, far, lens, expected, dst, bs, block_size=bs)
    finally:
        os.close(fd)


READER_CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as o
from storm_amd import blocks
rng = np.random.default_rng(5)
nblocks, bs, n = 512, 4096, 900
image = rng.integers(0, 256, size=(nblocks, bs), dtype=np.uint8)
path = os.path.join(sys.argv[2], "dev.img")
image.tofile(path)
addresses = rng.integers(0, nblocks, size=n).astype(np.uint64)
lens = rng.integers(1, bs + 1, size=n).astype(np.uint32)
expected = np.array([o.xxh64(image[a, :l]) for a, l in zip(addresses, lens)], dtype=np.uint64)
dst = np.zeros((n, bs), dtype=np.uint8)
fd = os.open(path, os.O_RDONLY)
ok = blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst, bs, block_size=bs) == (n, 0)
bad = expected.copy(); bad[[700, 33]] ^= 1
ok = ok and blocks.ReadVerifyBatch(fd, addresses, lens, bad, dst, bs, block_size=bs) == (33, 2)
print("RESULT", ok)
"""


@pytest.mark.parametrize("limit", ["0", "2"])
def test_read_verify_survives_reader_thread_failure(dev, tmp_path, limit):
    """Creating the reader pool can fail (thread limit): the call carries on with the
    readers already started, or reads on the calling thread when there are none, and
    never lets the exception leave the C ABI. STORMCK_DEBUG_READER_LIMIT makes creation
    fail after `limit` readers (read once per process: a child process)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, STORMCK_DEBUG_READER_LIMIT=limit, STORMCK_READ_SUPER_BYTES=str(64 * 4096))
    p = subprocess.run([sys.executable, "-c", READER_CHILD, root, str(tmp_path)], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
    assert "RESULT True" in p.stdout, p.stdout[-2000:]


def _odirect_dir(tmp_path):
    """A directory whose filesystem takes O_DIRECT (tmpfs does not), or None."""
    import os
    for d in (str(tmp_path), os.getcwd(), os.path.expanduser("~")):
        probe = os.path.join(d, f".odirect_{os.getpid()}")
        try:
            fd = os.open(probe, os.O_RDWR | os.O_CREAT | os.O_DIRECT, 0o600)
        except OSError:
            continue
        os.close(fd)
        os.unlink(probe)
        return d
    return None


def test_read_verify_o_direct_into_registered_slots(dev, tmp_path):
    """f3: the device image opened with O_DIRECT (no page cache, pkg/filedev with the
    reference's O_DIRECT TODO, persistence/init.go:54), read into page-aligned,
    registered slots (full blocks; the verify DMAs straight from them). Addresses mix
    runs of consecutive blocks (one pread per run) and random ones; clean blocks verify,
    a corrupted block on the device is found, misaligned slots are refused."""
    import mmap
    import os
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    d = _odirect_dir(tmp_path)
    if d is None:
        pytest.skip("no O_DIRECT-capable filesystem on this box")
    rng = np.random.default_rng(17)
    nblocks, bs = 4096, 32768
    image = rng.integers(0, 256, size=(nblocks, bs), dtype=np.uint8)
    path = os.path.join(d, f"odirect_dev_{os.getpid()}.img")
    image.tofile(path)
    n = 3000
    runs = np.concatenate([np.arange(100, 164), np.arange(2000, 2040), np.arange(4000, 4096)])
    rest = np.setdiff1d(np.arange(nblocks), runs)
    addresses = np.concatenate([runs, rng.choice(rest, size=n - runs.size, replace=False)]).astype(np.uint64)
    lens = rng.choice([72, 28808, 30000, 31808, 32768], size=n).astype(np.uint32)
    expected = o.checksum_batch(image[addresses.astype(np.int64)], n, bs, lens=lens, threads=8)
    mm = mmap.mmap(-1, n * bs)  # page-aligned slots
    dst = np.frombuffer(mm, dtype=np.uint8).reshape(n, bs)
    blocks.RegisterHostMemory(dst)
    fd = os.open(path, os.O_RDWR | os.O_DIRECT)
    try:
        assert blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst, bs) == (n, 0)
        for i in (0, 63, 64, 200, 2999):
            assert np.array_equal(dst[i], image[int(addresses[i])])  # whole blocks landed
        # corrupt block 2010 on the device itself (an O_DIRECT write of one aligned block)
        blk = mmap.mmap(-1, bs)
        blk.write(image[2010].tobytes())
        blk[5] ^= 0xFF
        os.pwrite(fd, blk, 2010 * bs)
        first = int(np.nonzero(addresses == 2010)[0][0])
        assert blocks.ReadVerifyBatch(fd, addresses, lens, expected, dst, bs) == (first, 1)
        misaligned = np.frombuffer(mm, dtype=np.uint8)[16:16 + (n - 1) * bs].reshape(n - 1, bs)
        with pytest.raises(_lib.StormckError) as e:
            blocks.ReadVerifyBatch(fd, addresses[:10], lens[:10], expected[:10], misaligned, bs)
        assert e.value.code == _lib.EINVAL and "aligned" in str(e.value)
    finally:
        os.close(fd)
        blocks.UnregisterHostMemory(dst)
        os.unlink(path)


def test_quad_paths_verify_and_gather_variants(dev):
    """Register-quad kernel in every shape: verify with per-block lengths (LENS+VERIFY),
    gather with offsets and a uniform length (OFFS only), verify through offsets is
    covered by the commit tests; host verify with per-block lengths."""
    from oracle import oracle as o
    from storm_amd import blocks, engine
    rng = np.random.default_rng(99)
    n, stride = 4000, 2048
    host = rng.integers(0, 256, size=(n, stride), dtype=np.uint8)
    lens = rng.integers(0, stride + 1, size=n).astype(np.uint32)
    want = o.checksum_batch(host, n, stride, lens=lens)
    d = _to_dev(host, dev)
    d_lens = _to_dev(lens.view(np.int32), dev)
    exp = torch.from_numpy(want.view(np.int64).copy()).to(dev)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(d.data_ptr(), stride, n, exp.data_ptr(), res.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [n, 0]
    exp[3999] ^= 1
    exp[1234] ^= 1
    engine.verify_device(d.data_ptr(), stride, n, exp.data_ptr(), res.data_ptr(), 0, d_lens.data_ptr())
    torch.cuda.synchronize()
    assert _u64(res).tolist() == [1234, 2]
    # gather: reversed order, uniform length
    offs = (np.arange(n, dtype=np.uint64)[::-1] * stride).copy()
    d_offs = _to_dev(offs.view(np.int64), dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 777)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), o.checksum_batch(host, n, stride, 777)[::-1])
    # host verify with per-block lengths
    bad = want.copy()
    bad[77] ^= 1
    assert blocks.VerifyChecksumBatchGPU(host, n, stride, want, lens=lens) == (n, 0)
    assert blocks.VerifyChecksumBatchGPU(host, n, stride, bad, lens=lens) == (77, 1)


def test_device_entry_points_are_graph_capturable(dev):
    """The device entry points allocate and synchronise nothing, so a batch checksum
    + Merkle root can be captured into a HIP graph once and replayed on new data
    (launch-bound small batches: one graph launch instead of several kernels)."""
    from oracle import oracle as o
    from storm_amd import engine
    n, stride = 2048, 32768
    buf = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    ws = torch.empty(engine.merkle_workspace_bytes(n, 1200) // 8 + 1, dtype=torch.int64, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), stride, n, 0, 1)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):  # warm-up outside capture
        engine.checksum_tensor(buf, out=out)
        engine.merkle_root_tensor(out, 0, n, 1, 1200, ws)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        engine.checksum_tensor(buf, out=out)
        root = engine.merkle_root_tensor(out, 0, n, 1, 1200, ws)
    for seed in (7, 8):
        engine.fill_synthetic_device(buf.data_ptr(), stride, n, 0, seed)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        want = o.checksum_batch(buf.cpu().numpy(), n, stride, stride)
        assert np.array_equal(_u64(out), want)
        assert engine.as_tuple(root) == o.merkle_root(want, 0, n, 1, 1200)


PLACEMENT_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from oracle import oracle as o
from storm_amd import _lib, engine, commit as sc
torch.cuda.init()
engine.init(0)
n, stride = 12288, 32768
want = o.checksum_batch(o.fill_synthetic(n, stride, 7), n, stride, stride, threads=8)
for mode in (2, 0):
    ptr, mapped = engine.device_alloc_placed(n * stride, mode)
    try:
        assert ptr % 4096 == 0 and mapped == 0
        engine.fill_synthetic_device(ptr, stride, n, 7, o.SYNTH_SEED)
        out = torch.empty(n, dtype=torch.int64, device="cuda")
        engine.checksum_device(ptr, stride, n, out.data_ptr(), stride)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, bad.size, bad[:8])
        # the routed entries know the arena for device memory: the batch refuses it, the
        # commit takes the device leg (host threads never dereference it)
        cs = np.zeros(4, dtype=np.uint64)
        rc = _lib.lib.stormck_checksum_batch(ptr, stride, None, stride, 4, cs.ctypes.data, 0, None)
        assert rc == _lib.EINVAL and "device memory" in _lib.last_error(), (mode, rc, _lib.last_error())
        b, size, last = sc.pointer_forest(8, 1000, 10, slot=stride, revision=1)
        host = o.fill_synthetic(size // stride, stride, 7).reshape(-1).copy()
        b_ref = b.copy()
        cs_ref, last_ref = o.commit(host, b_ref, 1, last)
        got, last_got, leg = sc.commit(ptr, b, 1, last)
        assert leg == _lib.LEG_DEVICE and last_got == last_ref, mode
        assert np.array_equal(b, b_ref)
        assert np.array_equal(got, cs_ref), mode
    finally:
        engine.device_free(ptr)
print("placement modes ok")
"""


def test_arena_placement_modes_probe_build(dev):
    """The arena placement modes measured and rejected in round 4 (stormck_device_alloc_placed:
    plain hipMalloc and a contiguous allocation; DESIGN_LOG.md) live in the probe build only.
    Through it, in a child process: a 384 MiB arena in either mode hashes like the oracle
    through the LDS-DMA kernel and frees cleanly, and the routed entry points recognise the
    arena as device memory (the batch refuses it, the commit takes the device leg and
    matches the oracle) rather than handing it to host threads. Any wrong checksum fails.
    (The VMM mode was deleted in round 6: it twice read wrong blocks and served no purpose.)"""
    import subprocess
    import sys
    from storm_amd import build as sb
    from tests.conftest import ROOT
    env = dict(os.environ, STORMCK_LIBRARY=sb.PROBES_LIB)
    r = subprocess.run([sys.executable, "-c", PLACEMENT_CHILD, ROOT], cwd=ROOT, capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0 and "placement modes ok" in r.stdout, r.stdout + r.stderr

