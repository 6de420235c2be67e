"""storm block layouts as ctypes structures (Go amd64 layout, padding included).

``blocks.BlockChecksum`` hashes ``unsafe.Sizeof(T)`` bytes of the live struct,
padding bytes included (/root/reference/blocks/checksum.go:10-12), so the exact
layout decides which bytes are hashed. ctypes uses the C layout rules, which for
these field types (u64 / u16 / byte and arrays of them) coincide with Go's.

Production fan-outs come from ``params.go``; the ``//go:build test`` variants
(``params_testing.go``) shrink them to 10, which changes the hashed
sizes: pointer 256, objectlist 536, spacelist 728 bytes.
"""
from __future__ import annotations

import ctypes
from ctypes import c_uint8, c_uint16, c_uint64
from functools import lru_cache

from .blocks import BLOCK_SIZE, Pointer

# /root/reference/blocks/pointer/params.go:6, objectlist/params.go:6, spacelist/params.go:6
POINTERS_PER_BLOCK = 1200
CHUNKS_PER_BLOCK = 600
SPACES_PER_BLOCK = 400
# params_testing.go under the `test` build tag
TEST_FANOUT = 10

OBJECTLIST_CHUNK_SIZE = 32  # objectlist/block.go:9


@lru_cache(maxsize=None)
def pointer_block(pointers_per_block: int = POINTERS_PER_BLOCK):
    """pointer.Block (/root/reference/blocks/pointer/block.go:10-13)."""

    class PointerBlock(ctypes.Structure):
        _fields_ = [
            ("Pointers", Pointer * pointers_per_block),
            ("PointedBlockTypes", c_uint8 * pointers_per_block),
        ]

    PointerBlock.__name__ = f"PointerBlock{pointers_per_block}"
    return PointerBlock


class BlobBlock(ctypes.Structure):
    """blob.Block (/root/reference/blocks/blob/block.go:25-29): 32768 bytes."""

    _fields_ = [("Data", c_uint8 * (BLOCK_SIZE - 8)), ("NUsedSlots", c_uint64)]


@lru_cache(maxsize=None)
def objectlist_block(chunks_per_block: int = CHUNKS_PER_BLOCK):
    """objectlist.Block (/root/reference/blocks/objectlist/block.go:29-40)."""

    class ObjectListBlock(ctypes.Structure):
        _fields_ = [
            ("Blob", c_uint8 * (chunks_per_block * OBJECTLIST_CHUNK_SIZE)),
            ("KeyTagReminders", c_uint64 * chunks_per_block),
            ("ObjectLinks", c_uint64 * chunks_per_block),
            ("ChunkPointers", c_uint16 * chunks_per_block),
            ("NextChunkPointers", c_uint16 * chunks_per_block),
            ("ChunkPointerStates", c_uint8 * chunks_per_block),
            ("NUsedChunks", c_uint16),
            ("FreeChunkIndex", c_uint16),
        ]

    ObjectListBlock.__name__ = f"ObjectListBlock{chunks_per_block}"
    return ObjectListBlock


class Space(ctypes.Structure):
    """spacelist.Space (/root/reference/blocks/spacelist/block.go:21-29): 72 bytes (5 padding)."""

    _fields_ = [
        ("SpaceIDTagReminder", c_uint64),
        ("NextObjectID", c_uint64),
        ("KeyStorePointer", Pointer),
        ("ObjectStorePointer", Pointer),
        ("KeyStoreBlockType", c_uint8),
        ("ObjectStoreBlockType", c_uint8),
        ("State", c_uint8),
    ]


@lru_cache(maxsize=None)
def spacelist_block(spaces_per_block: int = SPACES_PER_BLOCK):
    """spacelist.Block (/root/reference/blocks/spacelist/block.go:32-36)."""

    class SpaceListBlock(ctypes.Structure):
        _fields_ = [("Spaces", Space * spaces_per_block), ("NUsedSpaces", c_uint16)]

    SpaceListBlock.__name__ = f"SpaceListBlock{spaces_per_block}"
    return SpaceListBlock


class SingularityBlock(ctypes.Structure):
    """singularity.Block (/root/reference/blocks/singularity/block.go:8-19): 72 bytes.

    Hashed with Checksum = 0 (/root/reference/cache/cache.go:71-73,
    /root/reference/persistence/store.go:78-80)."""

    _fields_ = [
        ("Checksum", c_uint64),
        ("StormID", c_uint64),
        ("Revision", c_uint64),
        ("NBlocks", c_uint64),
        ("SpacePointer", Pointer),
        ("SpaceBlockType", c_uint8),
        ("LastAllocatedBlock", c_uint64),
    ]


PointerBlock = pointer_block()
ObjectListBlock = objectlist_block()
SpaceListBlock = spacelist_block()


def hashed_sizes(test_tag: bool = False) -> dict:
    """unsafe.Sizeof of every storm block type (bytes BlockChecksum hashes)."""
    f = TEST_FANOUT if test_tag else None
    return {
        "singularity": ctypes.sizeof(SingularityBlock),
        "pointer": ctypes.sizeof(pointer_block(f or POINTERS_PER_BLOCK)),
        "spacelist": ctypes.sizeof(spacelist_block(f or SPACES_PER_BLOCK)),
        "objectlist": ctypes.sizeof(objectlist_block(f or CHUNKS_PER_BLOCK)),
        "blob": ctypes.sizeof(BlobBlock),
    }
