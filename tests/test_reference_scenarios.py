"""storm's own cache / persistence tests, restated on the checksum path.

The reference tests its checksum path through the layers that call it:
cache/cache_test.go, persistence/store_test.go and persistence/init_test.go. Those
layers (the cache, the store, memdev) are out of scope here (DESIGN_LOG.md §0). What they
assert about checksums is in scope. Each test below follows one reference test. It
keeps that test's block contents and its checksum checks, and runs them through this
library's boundary:

* the host leg (`blocks.Checksum` / `BlockChecksum` / `VerifyChecksum`), on the CPU;
* the device legs, `-m gpu`:
  * `ReadVerifyBatch` reads from a device file laid out like storm's memdev;
  * `VerifyChecksumBatch` and `ChecksumBatch` over host buffers.

Expected checksums come from the oracle (test infrastructure), never from the library
under test. The reference's tests build with the `test` tag (fan-out 10,
params_testing.go), so the pointer blocks here use both that fan-out and production's
1,200.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as o
from storm_amd import blocks, layouts

# persistence/init.go:16-19
MIN_N_BLOCKS = 32
STORM_SUBJECT = 0b0100001000000000100000010010000100010010110000100010010001000101
FANOUTS = [layouts.TEST_FANOUT, layouts.POINTERS_PER_BLOCK]


def image(block) -> bytes:
    """photon.NewFromValue(b).B: the struct's bytes, padding included."""
    return bytes(memoryview(block).cast("B"))


def initialize(n_blocks: int, storm_id: int) -> layouts.SingularityBlock:
    """persistence.Initialize (init.go:33-55): a fresh singularity block whose checksum
    is BlockChecksum over itself, taken while its Checksum field is still 0."""
    s = layouts.SingularityBlock()
    s.StormID = storm_id | STORM_SUBJECT
    s.NBlocks = n_blocks
    s.Checksum = blocks.BlockChecksum(s)
    return s


def with_checksum(s, checksum):
    """A copy of singularity block `s` with its Checksum field set to `checksum`."""
    c = layouts.SingularityBlock.from_buffer_copy(image(s))
    c.Checksum = checksum
    return c


def initialize_zeroed(s):
    return with_checksum(s, 0)


def validate_singularity(address: int, s: layouts.SingularityBlock):
    """validateSingularityBlock (persistence/store.go:73-81): verify a copy with
    Checksum = 0 against the stored checksum. Returns the Go error value (None = ok)."""
    if s.StormID & STORM_SUBJECT != STORM_SUBJECT:
        return ValueError("device does not contain storm storage system")
    return blocks.VerifyChecksum(address, image(initialize_zeroed(s)), s.Checksum)


# ---------------------------------------------------------------- host leg (CPU)


def test_init_singularity_checksum():
    """persistence/init_test.go:17-41 (TestInit): read back, zero Checksum, re-hash."""
    s = initialize(MIN_N_BLOCKS, 0x1234_5678_9ABC_DEF0)
    stored = s.Checksum
    s.Checksum = 0
    assert s.StormID & STORM_SUBJECT == STORM_SUBJECT
    assert (s.Revision, s.LastAllocatedBlock, s.SpacePointer.Address) == (0, 0, 0)
    assert s.SpaceBlockType == blocks.FreeBlockType
    assert blocks.BlockChecksum(s) == stored == o.xxh64(image(s))


def test_overwrite_changes_checksum():
    """init_test.go:43-78 (TestOverwrite): re-initialising draws a new StormID, so the
    checksum changes while NBlocks / LastAllocatedBlock stay."""
    a, b = initialize(MIN_N_BLOCKS, 1), initialize(MIN_N_BLOCKS, 2)
    assert a.Checksum != b.Checksum and a.StormID != b.StormID
    assert (a.NBlocks, a.LastAllocatedBlock) == (b.NBlocks, b.LastAllocatedBlock)
    assert a.Checksum == o.xxh64(image(initialize_zeroed(a)))


def test_store_validation():
    """persistence/store_test.go:16-99: OpenStore's checksum step on the singularity
    block, for each of the reference's four cases."""
    s = initialize(MIN_N_BLOCKS, 7)
    assert validate_singularity(0, s) is None  # TestValidInitialization

    bad = layouts.SingularityBlock.from_buffer_copy(image(s))
    bad.Checksum = 0  # TestInvalidChecksum (:26-48)
    err = validate_singularity(0, bad)
    assert isinstance(err, blocks.ChecksumMismatchError)
    assert str(err) == (f"checksum mismatch for block 0, computed: {o.xxh64(image(initialize_zeroed(s))):#x}, "
                        "expected: 0x0")

    # TestInvalidBlockNumber (:50-73) recomputes the checksum WITHOUT zeroing the
    # field first, so the stored value hashes the old checksum in and the open fails
    # at the checksum step already, before the block-count check (store.go:27-31).
    nb = layouts.SingularityBlock.from_buffer_copy(image(s))
    nb.NBlocks += 1
    nb.Checksum = blocks.BlockChecksum(nb)
    assert nb.Checksum == o.xxh64(image(with_checksum(nb, s.Checksum)))
    assert isinstance(validate_singularity(0, nb), blocks.ChecksumMismatchError)

    # TestExpandingDevWorks (:75-99) zeroes it first: the checksum step passes.
    ex = layouts.SingularityBlock.from_buffer_copy(image(s))
    ex.NBlocks -= 1
    ex.Checksum = 0
    ex.Checksum = blocks.BlockChecksum(ex)
    assert validate_singularity(0, ex) is None

    foreign = layouts.SingularityBlock.from_buffer_copy(image(s))
    foreign.StormID = 0  # store.go:74-76: not a storm device, checked before the checksum
    assert isinstance(validate_singularity(0, foreign), ValueError)


@pytest.mark.parametrize("fanout", FANOUTS)
def test_fetch_block_by_address(fanout):
    """cache/cache_test.go:44-94 (TestFetchBlockByAddress): a pointer block with
    Pointers[3].Address = 21 on the device at address 1. The fetch verifies against
    BlockChecksum of that content. Rewriting it to 22 changes the checksum, and a
    verify of the new bytes against the old checksum fails with storm's message."""
    pb = layouts.pointer_block(fanout)()
    pb.Pointers[3].Address = 21
    cs21 = blocks.BlockChecksum(pb)
    assert cs21 == o.xxh64(image(pb))
    assert blocks.VerifyChecksum(1, image(pb), cs21) is None
    pb.Pointers[3].Address = 22
    cs22 = blocks.BlockChecksum(pb)
    assert cs22 != cs21 and cs22 == o.xxh64(image(pb))
    err = blocks.VerifyChecksum(1, image(pb), cs21)
    assert str(err) == f"checksum mismatch for block 1, computed: {cs22:#x}, expected: {cs21:#x}"


class PaddedStruct(ctypes.Structure):
    """cache_test.go:260-265: u64, byte, u64 -- 7 bytes of padding after Field2."""

    _fields_ = [("Field1", ctypes.c_uint64), ("Field2", ctypes.c_uint8), ("Field3", ctypes.c_uint64)]


def test_padding_is_hashed():
    """cache_test.go:267-300 (TestNewBlocksProduceConsistentResult): new blocks are
    zeroed, padding included, so equal fields give equal images and equal checksums.
    The checksum covers the padding: a dirty padding byte changes it."""
    assert ctypes.sizeof(PaddedStruct) == 24
    a, b = PaddedStruct(1, 2, 3), PaddedStruct(1, 2, 3)
    assert image(a) == image(b)
    assert blocks.BlockChecksum(a) == blocks.BlockChecksum(b) == o.xxh64(image(a))
    dirty = bytearray(image(a))
    dirty[9] = 0xA5  # a padding byte
    d = PaddedStruct.from_buffer_copy(bytes(dirty))
    assert (d.Field1, d.Field2, d.Field3) == (1, 2, 3)
    assert blocks.BlockChecksum(d) != blocks.BlockChecksum(a)
    assert blocks.BlockChecksum(d) == o.xxh64(bytes(dirty))


# ---------------------------------------------------------------- device legs (GPU)


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    assert _lib.device_count() > 0, "GPU visible to torch but libstormck finds no gfx950 device"
    return torch


def write_dev(path, fanout, n_blocks=MIN_N_BLOCKS):
    """A memdev-like device file: the singularity block at address 0, and the new
    pointer block of cache_test.go:204-258 (all zero) at address 1."""
    s = initialize(n_blocks, 11)
    s.LastAllocatedBlock = 1
    s.Checksum = 0
    s.Checksum = blocks.BlockChecksum(s)
    pb = layouts.pointer_block(fanout)()
    dev = bytearray(n_blocks * blocks.BLOCK_SIZE)
    dev[:ctypes.sizeof(s)] = image(s)
    dev[blocks.BLOCK_SIZE:blocks.BLOCK_SIZE + ctypes.sizeof(pb)] = image(pb)
    with open(path, "wb") as f:
        f.write(dev)
    return s, pb


@pytest.mark.gpu
@pytest.mark.parametrize("fanout", FANOUTS)
def test_checksum_is_verified_when_fetching(gpu, tmp_path, fanout):
    """cache/cache_test.go:204-258 (TestChecksumIsVerifiedWhenFetching), cold-cache
    part. The block is read from the device and verified on the GPU. A pointer with
    Checksum 0 fails; the right checksum passes."""
    path = os.path.join(tmp_path, "dev")
    _, pb = write_dev(path, fanout)
    size = ctypes.sizeof(pb)
    want = o.xxh64(image(pb))
    dst = np.zeros(2 * blocks.BLOCK_SIZE, dtype=np.uint8)
    fd = os.open(path, os.O_RDONLY)
    try:
        assert blocks.ReadVerifyBatch(fd, [1], [size], [0], dst, blocks.BLOCK_SIZE) == (0, 1)
        assert blocks.ReadVerifyBatch(fd, [1], [size], [want], dst, blocks.BLOCK_SIZE) == (1, 0)
        assert bytes(dst[:size]) == image(pb)
        # one batch holding both fetches: the first is the bad one
        assert blocks.ReadVerifyBatch(fd, [1, 1], [size, size], [0, want], dst, blocks.BLOCK_SIZE) == (0, 1)
        assert blocks.ReadVerifyBatch(fd, [1, 1], [size, size], [want, 0], dst, blocks.BLOCK_SIZE) == (1, 1)
    finally:
        os.close(fd)


@pytest.mark.gpu
def test_store_validation_on_device(gpu, tmp_path):
    """persistence/store_test.go's four cases as one device batch. Each singularity
    image is verified with its Checksum field zeroed against the stored value
    (store.go:78-80). Only InvalidChecksum and InvalidBlockNumber fail."""
    s = initialize(MIN_N_BLOCKS, 7)
    bad = layouts.SingularityBlock.from_buffer_copy(image(s))
    bad.Checksum = 0
    nb = layouts.SingularityBlock.from_buffer_copy(image(s))
    nb.NBlocks += 1
    nb.Checksum = blocks.BlockChecksum(nb)
    ex = layouts.SingularityBlock.from_buffer_copy(image(s))
    ex.NBlocks -= 1
    ex.Checksum = 0
    ex.Checksum = blocks.BlockChecksum(ex)
    cases = [s, bad, nb, ex]
    size = ctypes.sizeof(layouts.SingularityBlock)
    buf = np.zeros((len(cases), 128), dtype=np.uint8)
    for i, c in enumerate(cases):
        buf[i, :size] = np.frombuffer(image(initialize_zeroed(c)), dtype=np.uint8)
    expected = [c.Checksum for c in cases]
    assert blocks.VerifyChecksumBatch(buf, len(cases), 128, expected, length=size) == (1, 2)
    got = blocks.ChecksumBatch(buf, len(cases), 128, length=size)
    assert [int(v) for v in got] == [o.xxh64(bytes(buf[i, :size])) for i in range(len(cases))]
    assert [blocks.VerifyChecksum(0, bytes(buf[i, :size]), expected[i]) is None for i in range(4)] == \
        [True, False, False, True]


# keystore/keystore_test.go:38-47 (TestSetGet): "Key intentionally takes 2.5 chunks."
SETGET_KEY = bytes(range(0x50))


def test_keystore_set_get_tag():
    """The tree tag of TestSetGet's 80-byte key, xxhash.Sum64(key)
    (keystore/keystore.go:33,66), on the host leg that keyTag binds
    (integration/go/keystore/keytag_stormck.go)."""
    assert blocks.Checksum(SETGET_KEY) == o.xxh64(SETGET_KEY)


@pytest.mark.gpu
def test_keystore_storing_batches_tags(gpu):
    """keystore_test.go:74-140 (TestStoringBatches): 1,500 batches of 5 random 48-byte
    keys. Their tags on the device, at a fixed stride and packed with TestSetGet's key
    and ragged neighbours, match xxhash.Sum64 of each key."""
    from storm_amd import engine
    torch = gpu
    rng = np.random.default_rng(74)
    keys = rng.integers(0, 256, size=(1500 * 5, 48), dtype=np.uint8)
    d_keys = torch.from_numpy(keys.reshape(-1)).cuda()
    out = torch.zeros(len(keys), dtype=torch.int64, device="cuda")
    engine.key_tags_device(d_keys.data_ptr(), len(keys), out.data_ptr(), stride=48, length=48)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    assert [int(v) for v in got] == [o.xxh64(bytes(k)) for k in keys]

    packed = [SETGET_KEY] + [bytes(keys[i, :1 + i % 48]) for i in range(300)] + [bytes(256 * [0xAB])]
    offs = np.cumsum([0] + [len(k) for k in packed[:-1]]).astype(np.uint64)
    lens = np.array([len(k) for k in packed], dtype=np.uint32)
    d_buf = torch.from_numpy(np.frombuffer(b"".join(packed), dtype=np.uint8).copy()).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    out2 = torch.zeros(len(packed), dtype=torch.int64, device="cuda")
    engine.key_tags_device(d_buf.data_ptr(), len(packed), out2.data_ptr(), d_offsets=d_offs.data_ptr(),
                           d_lens=d_lens.data_ptr())
    torch.cuda.synchronize()
    assert [int(v) for v in out2.cpu().numpy().view(np.uint64)] == [o.xxh64(k) for k in packed]
