"""storm block layouts (which bytes BlockChecksum hashes) — CPU, host logic only.

Mirrors /root/reference/blocks/types_test.go:18-32 (every block fits BlockSize)
and pins the Go amd64 sizes/offsets the hashed byte ranges depend on.
"""
import ctypes

import pytest

from storm_amd import layouts
from storm_amd.blocks import BLOCK_SIZE, BlockType
from tests.conftest import load_golden


@pytest.mark.parametrize("tag", ["prod", "test"])
def test_sizes_match_go(tag):
    want = load_golden("layouts.json")["sizes"][tag]
    assert layouts.hashed_sizes(test_tag=(tag == "test")) == want


def test_every_block_fits_block_size():
    # blocks/types_test.go:18-32
    for size in layouts.hashed_sizes().values():
        assert size <= BLOCK_SIZE
    assert BLOCK_SIZE == 32768


def test_block_type_values():
    # blocks/types.go:7-15
    assert (BlockType.FREE, BlockType.POINTER, BlockType.LEAF) == (0, 1, 2)


def test_field_offsets():
    S = layouts.SingularityBlock
    assert (S.SpacePointer.offset, S.SpaceBlockType.offset, S.LastAllocatedBlock.offset) == (32, 56, 64)
    O = layouts.ObjectListBlock
    assert (O.KeyTagReminders.offset, O.ObjectLinks.offset, O.ChunkPointers.offset, O.NextChunkPointers.offset,
            O.ChunkPointerStates.offset, O.NUsedChunks.offset, O.FreeChunkIndex.offset) == \
        (19200, 24000, 28800, 30000, 31200, 31800, 31802)
    assert ctypes.sizeof(layouts.Space) == 72
    P = layouts.PointerBlock
    assert P.PointedBlockTypes.offset == 28800
    assert layouts.BlobBlock.NUsedSlots.offset == 32760


def test_blob_test_block_bytes():
    # /root/reference/blocks/blob/block_test.go:39-45: the byte image of 4 Object[item]s
    g = load_golden("layouts.json")["blob_test_block"]
    want = bytes.fromhex(g["first_128_hex"])
    expected_rows = [
        [0x1, 0x2, 0x3, 0x1], [0x4, 0x5, 0x6, 0x2], [0x7, 0x8, 0x9, 0x0], [0xa, 0xb, 0xc, 0x1]]
    for k, row in enumerate(expected_rows):
        for q, v in enumerate(row):
            assert want[32 * k + 8 * q] == v
            assert want[32 * k + 8 * q + 1: 32 * k + 8 * q + 8] == bytes(7)
