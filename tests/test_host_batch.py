"""Host-memory batches: the host leg (stormck_checksum_host_leg / _verify_host_leg) and
the routed batch (stormck_checksum_batch / _verify_batch) that the Go shim's
ChecksumBatch / VerifyChecksumBatch call.

A batch in host memory crosses PCIe on the device leg (~52 GiB/s end to end), while
host threads hash the same bytes four blocks at a time; the routed entry takes the leg
the library's cost model predicts is fastest (the split leg, both at
once, has its own tests in tests/test_split_gpu.py), as stormck_commit does for a commit
(/root/reference/cache/cache.go:87-137).

CPU: the host leg against the C oracle (blocks.Checksum = XXH64 seed 0,
/root/reference/blocks/checksum.go:15-17) on uniform, per-block, short, tail and
unaligned blocks, any thread count, and verify with planted mismatches. GPU: the routed
entry on both legs against the oracle, and its leg for batches the model decides
clearly.
"""
import numpy as np
import pytest

from oracle import oracle as o
from storm_amd import _lib, blocks


def _rows(n, stride, seed, offset=0):
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, size=n * stride + offset + 64, dtype=np.uint8)
    return raw[offset:offset + n * stride]


@pytest.mark.parametrize("threads", [1, 3, 0])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 9, 257])
def test_host_leg_uniform(n, threads):
    stride = 1024
    buf = _rows(n, stride, n)
    for length in (stride, 1000, 33, 31, 0):
        want = o.checksum_batch(buf, n, stride, length)
        assert np.array_equal(blocks.ChecksumBatchHost(buf, n, stride, length, threads=threads), want), length


@pytest.mark.parametrize("threads", [1, 0])
def test_host_leg_per_block_lengths_and_alignment(threads):
    n, stride = 1001, 4096
    rng = np.random.default_rng(7)
    lens = rng.integers(0, stride + 1, size=n).astype(np.uint32)
    lens[:8] = [0, 1, 31, 32, 33, 63, 64, stride]
    for offset in (0, 1, 8, 13):  # unaligned starts: the host leg reads any alignment
        buf = _rows(n, stride, 11, offset)
        want = o.checksum_batch(buf, n, stride, lens=lens)
        assert np.array_equal(blocks.ChecksumBatchHost(buf, n, stride, lens=lens, threads=threads), want), offset


def test_host_leg_storm_lengths_multithreaded():
    # storm's production Sizeof(T) mix over 32 KiB slots, enough bytes to split over threads
    n, stride = 600, 32768
    rng = np.random.default_rng(5)
    lens = rng.choice([72, 28808, 30000, 31808, 32768], size=n).astype(np.uint32)
    buf = _rows(n, stride, 5)
    want = o.checksum_batch(buf, n, stride, lens=lens, threads=8)
    for threads in (1, 2, 16, 0):
        assert np.array_equal(blocks.ChecksumBatchHost(buf, n, stride, lens=lens, threads=threads), want), threads


def test_host_leg_verify():
    n, stride = 777, 2048
    buf = _rows(n, stride, 3)
    want = o.checksum_batch(buf, n, stride, stride)
    assert blocks.VerifyChecksumBatchHost(buf, n, stride, want, stride) == (n, 0)
    bad = want.copy()
    for i in (500, 13, 776):
        bad[i] ^= 1
    for threads in (1, 0):
        assert blocks.VerifyChecksumBatchHost(buf, n, stride, bad, stride, threads=threads) == (13, 3)
    assert blocks.VerifyChecksumBatchHost(buf, 0, stride, [], stride) == (0, 0)
    assert blocks.ChecksumBatchHost(buf, 0, stride, stride).size == 0


def test_host_leg_needs_no_device_but_the_routed_batch_does():
    """Decided: the routed entry points keep STORMCK_ENODEV without a
    gfx950 device, even where their cost model would pick the host leg. They are the GPU
    engine's batch calls, and a library that quietly hashed on the CPU when its device is
    missing is the silent fallback this build must not have. The operational consequence,
    stated in INTEGRATION.md §2: a `-tags stormck` storm on a box whose GPU is absent or
    claimed fails ChecksumBatch / VerifyChecksumBatch / CommitBatch with the library's
    error (cache.Commit returns it) instead of committing; such a box runs storm built
    without the tag. The host leg itself (stormck_checksum_host_leg, stormck_commit_host)
    needs no device and stays callable for a caller that chooses it explicitly."""
    from tests.test_abi import _has_gpu
    if _has_gpu():
        pytest.skip("a device is present")
    buf = _rows(4, 64, 1)
    assert np.array_equal(blocks.ChecksumBatchHost(buf, 4, 64, 64), o.checksum_batch(buf, 4, 64, 64))
    with pytest.raises(_lib.NoDeviceError):
        blocks.ChecksumBatch(buf, 4, 64, 64)
    with pytest.raises(_lib.NoDeviceError):
        blocks.VerifyChecksumBatch(buf, 4, 64, [0] * 4, 64)


@pytest.mark.gpu
def test_routed_batch_both_legs():
    import torch
    torch.cuda.init()
    # a few blocks: the host leg (a device call costs more than hashing them)
    n, stride = 8, 32768
    buf = _rows(n, stride, 21)
    want = o.checksum_batch(buf, n, stride, stride)
    got, leg = blocks.ChecksumBatchLeg(buf, n, stride, stride)
    assert leg == _lib.LEG_HOST and np.array_equal(got, want)
    # a large batch with one host thread allowed: the model's choice, either way exact
    n = 8192  # 256 MiB
    buf = _rows(n, stride, 22)
    lens = np.random.default_rng(22).choice([28808, 30000, 31808, 32768], size=n).astype(np.uint32)
    want = o.checksum_batch(buf, n, stride, lens=lens, threads=8)
    legs = set()
    for threads in (1, 0):
        got, leg = blocks.ChecksumBatchLeg(buf, n, stride, lens=lens, host_threads=threads)
        assert leg in (_lib.LEG_HOST, _lib.LEG_DEVICE) and np.array_equal(got, want), (threads, leg)
        legs.add(leg)
        bad = want.copy()
        bad[4321] ^= 1
        bad[99] ^= 1
        fb, nb, vleg = blocks.VerifyChecksumBatchLeg(buf, n, stride, bad, lens=lens, host_threads=threads)
        assert (fb, nb) == (99, 2) and vleg == leg
    # the device leg itself on the same bytes
    assert np.array_equal(blocks.ChecksumBatchGPU(buf, n, stride, lens=lens), want)


@pytest.mark.gpu
def test_routed_batch_rejects_device_memory():
    import torch
    t = torch.zeros((4, 64), dtype=torch.uint8, device="cuda")
    out = np.zeros(4, dtype=np.uint64)
    rc = _lib.lib.stormck_checksum_batch(t.data_ptr(), 64, None, 64, 4, out.ctypes.data, 0, None)
    assert rc == _lib.EINVAL and "device memory" in _lib.last_error()
