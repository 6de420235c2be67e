"""One host batch over several devices from one process (stormck_checksum_host_multi /
stormck_verify_host_multi): storm is one Go process, so this is how its batched callers
(cache/cache.go:87-137 commit, :139-167 cold verify) would use every GPU of a node, each
device's range over its own PCIe link. The box has one GPU, so the ranges here share
device 0 (listed several times), which exercises the split, the worker threads, the
per-range offsets and the merge of verify results; every checksum is compared with the
C oracle (XXH64 seed 0 = blocks.Checksum, blocks/checksum.go:15-17)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return 0


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_checksum_and_verify_over_listed_devices(dev, devices):
    from storm_amd import blocks
    rng = np.random.default_rng(len(devices))
    n, stride = 3001, 32768
    host = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    want = o.checksum_batch(host, n, stride, stride, threads=8)
    assert np.array_equal(blocks.ChecksumBatch(host, n, stride, stride, devices=devices), want)
    # per-block lengths (every range starts at its own offset into lens)
    lens = rng.integers(0, stride + 1, size=n).astype(np.uint32)
    want_l = o.checksum_batch(host, n, stride, 0, lens=lens, threads=8)
    assert np.array_equal(blocks.ChecksumBatch(host, n, stride, lens=lens, devices=devices), want_l)
    # verify: all good, then mismatches in the first and last ranges
    assert blocks.VerifyChecksumBatch(host, n, stride, want, stride, devices=devices) == (n, 0)
    bad = want.copy()
    for i in (n - 1, n // 2 + 1, 17):
        bad[i] ^= np.uint64(1)
    assert blocks.VerifyChecksumBatch(host, n, stride, bad, stride, devices=devices) == (17, 3)


def test_registered_buffer_over_listed_devices(dev):
    """A registered (portable) buffer is DMA'd straight to every listed device."""
    from storm_amd import blocks
    n, stride = 2048, 32768
    raw = np.empty(n * stride + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    host = raw[off:off + n * stride]  # page-aligned pageable memory, registered below
    host[:] = np.random.default_rng(9).integers(0, 256, size=host.size, dtype=np.uint8)
    blocks.RegisterHostMemory(host)
    try:
        want = o.checksum_batch(host, n, stride, stride, threads=8)
        assert np.array_equal(blocks.ChecksumBatch(host, n, stride, stride, devices=[0, 0, 0, 0]), want)
    finally:
        blocks.UnregisterHostMemory(host)


def test_fewer_blocks_than_devices_and_empty(dev):
    from storm_amd import blocks
    data = np.arange(3 * 64, dtype=np.uint8)
    want = o.checksum_batch(data, 3, 64, 64)
    assert np.array_equal(blocks.ChecksumBatch(data, 3, 64, 64, devices=[0] * 8), want)
    assert np.array_equal(blocks.ChecksumBatch(data, 1, 64, 64, devices=[0, 0]), want[:1])
    assert blocks.ChecksumBatch(data, 0, 64, 64, devices=[0, 0]).size == 0


def test_bad_device_index_names_it(dev):
    from storm_amd import _lib, blocks
    n_dev = _lib.device_count()
    with pytest.raises(_lib.StormckError) as e:
        blocks.ChecksumBatch(bytes(128), 2, 64, 64, devices=[0, n_dev + 3])
    assert e.value.code == _lib.EINVAL and f"devices[1] = {n_dev + 3}" in str(e.value)


def test_errors_name_the_failing_range(dev):
    """A range that fails (here: blocks overlapping their stride) reports its device and
    block range; the calling thread keeps its current device."""
    from storm_amd import _lib
    L = _lib.lib
    buf = np.zeros(64 * 100, dtype=np.uint8)
    lens = np.full(100, 32, dtype=np.uint32)
    lens[80] = 200  # longer than the 64-byte stride: the range holding block 80 refuses
    out = np.zeros(100, dtype=np.uint64)
    devs = (ctypes.c_int * 2)(0, 0)
    before = torch.cuda.current_device()
    rc = L.stormck_checksum_host_multi(buf.ctypes.data, 64, lens.ctypes.data, 0, 100, out.ctypes.data, devs, 2)
    assert rc == _lib.EINVAL
    msg = _lib.last_error()
    assert "device 0 (blocks 50..100)" in msg and "stride" in msg, msg
    assert torch.cuda.current_device() == before


def test_every_visible_device(dev):
    """On a node with several GPUs: one range per physical device (each worker thread
    selects its own device, cu count and staging; pinned DMA to a second device), for
    pageable and registered buffers, and the caller's current device is unchanged.
    Skipped on a one-GPU box (the driver's 8-GPU node runs it)."""
    from storm_amd import blocks
    count = torch.cuda.device_count()
    if count < 2:
        pytest.skip("one device")
    devices = list(range(count))
    n, stride = 4099, 32768
    raw = np.empty(n * stride + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    host = raw[off:off + n * stride]
    host[:] = np.random.default_rng(21).integers(0, 256, size=host.size, dtype=np.uint8)
    want = o.checksum_batch(host, n, stride, stride, threads=8)
    torch.cuda.set_device(count - 1)
    assert np.array_equal(blocks.ChecksumBatch(host, n, stride, stride, devices=devices), want)
    bad = want.copy()
    bad[[n - 1, 5]] ^= np.uint64(1)
    assert blocks.VerifyChecksumBatch(host, n, stride, bad, stride, devices=devices) == (5, 2)
    blocks.RegisterHostMemory(host)
    try:
        assert np.array_equal(blocks.ChecksumBatch(host, n, stride, stride, devices=devices[::-1]), want)
    finally:
        blocks.UnregisterHostMemory(host)
    assert torch.cuda.current_device() == count - 1
    from storm_amd import _lib
    cur = ctypes.c_int(-1)
    torch.cuda.synchronize()
    assert _lib.lib.stormck_device_count(ctypes.byref(cur)) == 0 and cur.value == count
    torch.cuda.set_device(0)
