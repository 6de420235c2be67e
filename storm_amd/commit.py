"""f1 — level-synchronous batched commit of a dirty block forest (host side).

Mirrors storm's Cache.Commit data phase (/root/reference/cache/cache.go:87-137)
and the post-commit pointer writes (/root/reference/cache/trace.go:274-320):
every dirty block is described by its blockMetadata + BlockOrigin
(cache/types.go) as a ``stormck_dirty_block`` record, and libstormck commits the
whole forest one height level per launch (include/stormck.h
``stormck_commit_device``).

``pointer_forest`` builds the dirty forest storm produces when N leaves under a
pointer tree change (the shape TraceTagForUpdating walks: slot = tag % fanout per
level), rooted at the singularity's SpacePointer; tests and tools/commit_bench.py
use it.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib

NO_ORIGIN = (1 << 64) - 1
NO_PARENT = -1
LEAF, POINTER = 2, 1

# stormck_dirty_block (56 bytes, include/stormck.h)
DIRTY_DTYPE = np.dtype([
    ("data_offset", "<u8"), ("origin_pointer", "<u8"), ("origin_type", "<u8"), ("parent", "<i8"),
    ("address", "<u8"), ("birth_revision", "<u8"), ("length", "<u4"), ("type", "u1"), ("reserved", "u1", (3,)),
], align=True)
assert DIRTY_DTYPE.itemsize == 56

# singularity.Block field offsets (/root/reference/blocks/singularity/block.go:8-19)
SING_CHECKSUM, SING_REVISION, SING_SPACE_POINTER, SING_SPACE_TYPE, SING_LAST_ALLOCATED = 0, 16, 32, 56, 64
SING_SIZE = 72


def pointer_block_size(fanout: int) -> int:
    return (25 * fanout + 7) & ~7


def commit_device(d_arena: int, blocks: np.ndarray, revision: int, last_allocated: int,
                  stream: int = 0, out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, int]:
    """Commit the dirty forest (updates blocks' address/birth_revision in place).
    Returns (checksums uint64[n], new last_allocated_block). ``out`` (uint64[n]) may be
    passed to reuse the checksum array across commits, as a long-lived caller would."""
    if blocks.dtype != DIRTY_DTYPE or not blocks.flags["C_CONTIGUOUS"]:
        raise ValueError("blocks must be a contiguous DIRTY_DTYPE array")
    n = blocks.shape[0]
    if out is None:
        out = np.zeros(n, dtype=np.uint64)
    elif out.dtype != np.uint64 or out.shape != (n,) or not out.flags["C_CONTIGUOUS"]:
        raise ValueError("out must be a contiguous uint64 array of len(blocks)")
    la = ctypes.c_uint64(last_allocated)
    _lib.check(_lib.lib.stormck_commit_device(d_arena, blocks.ctypes.data if n else None, n, revision,
                                              ctypes.byref(la), out.ctypes.data if n else None, stream or None))
    return out, la.value


def pointer_forest(n_leaves: int, leaf_lens, fanout: int, slot: int = 32768, revision: int = 1,
                   existing: Optional[np.ndarray] = None, first_address: int = 1) -> Tuple[np.ndarray, int, int]:
    """Dirty forest of `n_leaves` leaves under pointer blocks of `fanout`, rooted at the
    singularity (arena slot 0; its SpacePointer / SpaceBlockType are the root's origin).

    Arena layout (``slot`` bytes per block, storm's cache.data image): slot 0 = the
    singularity, slots 1..n_leaves = leaves, then pointer blocks level by level.
    Leaf i sits in parent j = i // fanout at slot k = i % fanout (pointer.Block.Pointers[k]
    / PointedBlockTypes[k]). New blocks carry (address, birth_revision) = (allocated,
    revision + 1) as cache.newBlock assigns them (cache/cache.go:169-180); blocks
    flagged in ``existing`` carry an older birth revision, so commit relocates them.

    Returns (blocks, arena_bytes, last_allocated_block)."""
    lens = np.broadcast_to(np.asarray(leaf_lens, dtype=np.uint32), (n_leaves,))
    pbs = pointer_block_size(fanout)
    if pbs > slot or int(lens.max(initial=0)) > slot:
        raise ValueError("block larger than a slot")
    levels = []  # number of pointer blocks per level
    m = n_leaves
    while m > 1:
        m = (m + fanout - 1) // fanout
        levels.append(m)
    total = n_leaves + sum(levels)
    b = np.zeros(total, dtype=DIRTY_DTYPE)
    # data offsets: leaves first, then pointer blocks level by level
    b["data_offset"] = (np.arange(total, dtype=np.uint64) + 1) * np.uint64(slot)
    b["length"][:n_leaves] = lens
    b["length"][n_leaves:] = pbs
    b["type"][:n_leaves] = LEAF
    b["type"][n_leaves:] = POINTER
    # origins: child c of a level sits in parent c // fanout at slot c % fanout
    start, count = 0, n_leaves
    for lv_count in levels:
        parent_start = start + count
        c = np.arange(count, dtype=np.int64)
        par = parent_start + c // fanout
        k = (c % fanout).astype(np.uint64)
        b["parent"][start:start + count] = par
        poff = b["data_offset"][par]
        b["origin_pointer"][start:start + count] = poff + np.uint64(24) * k
        b["origin_type"][start:start + count] = poff + np.uint64(24 * fanout) + k
        start, count = parent_start, lv_count
    # the single top block hangs off the singularity
    b["parent"][start] = NO_PARENT
    b["origin_pointer"][start] = SING_SPACE_POINTER
    b["origin_type"][start] = SING_SPACE_TYPE
    # metadata as newBlock assigned it
    b["address"] = np.arange(first_address, first_address + total, dtype=np.uint64)
    b["birth_revision"] = revision + 1
    last = first_address + total - 1
    if existing is not None:
        ex = np.asarray(existing, dtype=bool)
        b["birth_revision"][ex] = revision  # born in an earlier revision -> relocated on commit
    return b, (total + 1) * slot, last
