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


def commit_host(arena: np.ndarray, blocks: np.ndarray, revision: int, last_allocated: int, threads: int = 0,
                out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, int]:
    """The host leg (stormck_commit_host) on a host uint8 arena: the same commit on
    `threads` library pool threads (0 = the pool, 1 = storm's serial loop)."""
    _check_blocks(blocks)
    if arena.dtype != np.uint8 or not arena.flags["C_CONTIGUOUS"]:
        raise ValueError("arena must be a contiguous uint8 array")
    n = blocks.shape[0]
    out = _out(out, n)
    la = ctypes.c_uint64(last_allocated)
    _lib.check(_lib.lib.stormck_commit_host(arena.ctypes.data, blocks.ctypes.data if n else None, n, revision,
                                            ctypes.byref(la), out.ctypes.data if n else None, threads))
    return out, la.value


def commit(arena_ptr: int, blocks: np.ndarray, revision: int, last_allocated: int, stream: int = 0,
           host_threads: int = 0, out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, int, int]:
    """The routed commit (stormck_commit): an HBM arena takes the device leg, a registered
    host arena the leg the library's cost model picks, an unregistered one the host leg.
    Returns (checksums, new last_allocated_block, leg: _lib.LEG_HOST / LEG_DEVICE)."""
    _check_blocks(blocks)
    n = blocks.shape[0]
    out = _out(out, n)
    la, leg = ctypes.c_uint64(last_allocated), ctypes.c_uint32(0)
    _lib.check(_lib.lib.stormck_commit(arena_ptr, blocks.ctypes.data if n else None, n, revision, ctypes.byref(la),
                                       out.ctypes.data if n else None, stream or None, host_threads, ctypes.byref(leg)))
    return out, la.value, leg.value


def commit_split(arena: np.ndarray, blocks: np.ndarray, revision: int, last_allocated: int, devices=None,
                 host_threads: int = 0, device_leaves: Optional[int] = None,
                 out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, int, int]:
    """The split commit (stormck_commit_split) on a registered host arena: the leaves
    hashed by host threads from the front and the devices from the back at once, in place.
    ``device_leaves``: None = balanced by the library's rates; else exactly the last
    ``device_leaves`` leaves of the commit order go to the devices. Returns (checksums, new
    last_allocated_block, leaves the devices hashed)."""
    _check_blocks(blocks)
    if arena.dtype != np.uint8 or not arena.flags["C_CONTIGUOUS"]:
        raise ValueError("arena must be a contiguous uint8 array")
    n = blocks.shape[0]
    out = _out(out, n)
    la, done = ctypes.c_uint64(last_allocated), ctypes.c_uint64(0)
    d = (ctypes.c_int * len(devices))(*[int(x) for x in devices]) if devices else None
    _lib.check(_lib.lib.stormck_commit_split(arena.ctypes.data, blocks.ctypes.data if n else None, n, revision,
                                             ctypes.byref(la), out.ctypes.data if n else None, d,
                                             len(devices) if devices else 0, host_threads,
                                             _lib.SPLIT_BALANCED if device_leaves is None else device_leaves,
                                             ctypes.byref(done)))
    return out, la.value, done.value


def plan_commit(blocks: np.ndarray, registered: bool = True, host_threads: int = 0, n_devices: int = 1):
    """The routed commit's decision alone (stormck_route_plan_commit; no device needed):
    (leg, (host_us, device_us, split_us))."""
    _check_blocks(blocks)
    n = blocks.shape[0]
    leg, us = ctypes.c_uint32(0), (ctypes.c_double * 3)()
    _lib.check(_lib.lib.stormck_route_plan_commit(blocks.ctypes.data if n else None, n,
                                                  _lib.MEM_PINNED if registered else _lib.MEM_PAGEABLE,
                                                  host_threads, n_devices, ctypes.byref(leg), us))
    return leg.value, tuple(us)


def _check_blocks(blocks: np.ndarray) -> None:
    if blocks.dtype != DIRTY_DTYPE or not blocks.flags["C_CONTIGUOUS"]:
        raise ValueError("blocks must be a contiguous DIRTY_DTYPE array")


def _out(out: Optional[np.ndarray], n: int) -> np.ndarray:
    if out is None:
        return np.zeros(n, dtype=np.uint64)
    if out.dtype != np.uint64 or out.shape != (n,) or not out.flags["C_CONTIGUOUS"]:
        raise ValueError("out must be a contiguous uint64 array of len(blocks)")
    return out


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


# ---------------------------------------------------------------------------
# storm's Cache.commitData on the GPU: the Python mirror of the Go binding
# integration/go/cache/commit_stormck.go (same steps, same order, same errors).
# ---------------------------------------------------------------------------
#
# The caller is storm's cache (cache/cache.go:16-53) with the stormck patch
# (integration/go/cache/trace_types.patch): every blockMetadata whose PostCommitFunc is
# set also records what that closure captured, as
#   meta.commit_origin  BlockOrigin (where the parent keeps this block's Pointer/type)
#   meta.commit_parent  parentBlockMeta (the block holding the origin, or None)
#   meta.commit_size    unsafe.Sizeof(T) of the block (the bytes BlockChecksum hashes)
#   meta.commit_type    the BlockType the closure stores (Leaf / Pointer)
# and the cache exposes what commitData touches: .dirty (the dirty set), .data
# (cache.data), .blocks' .data / .address / .birth_revision / .n_commits /
# .n_references / .state / .post_commit, .origin_offsets(origin) -> (pointer, type)
# offsets into cache.data or None (the singularity), .write_origin(...),
# .revision() / .last_allocated() / .set_last_allocated(v), .store.write_block(addr,
# bytes) and .find_cached_block(addr, birth).

USED_STATE, INVALID_STATE = 1, 2  # cache/types.go:10-15


class StillReferenced(RuntimeError):
    """A dirty block keeps NReferences > 0 after all its dirty children commit: storm's
    commitData (cache/cache.go:88-90) would sweep forever; the binding refuses."""


def cache_records(cache):
    """The dirty forest as stormck_dirty_block records (commit_stormck.go collectDirty).

    Records: the dirty set in its iteration order, then every ancestor reached through a
    recorded parent that is not in it yet (storm adds those to the dirty set only when a
    child's PostCommitFunc runs, trace.go:278-281,302-305). Returns (records, metas in
    record order, indices of records whose origin lies outside cache.data)."""
    metas = list(cache.dirty)
    index = {id(m): i for i, m in enumerate(metas)}
    k = 0
    while k < len(metas):
        m = metas[k]
        p = m.commit_parent if m.post_commit is not None else None
        if p is not None and id(p) not in index:
            index[id(p)] = len(metas)
            metas.append(p)
        k += 1
    recs = np.zeros(len(metas), dtype=DIRTY_DTYPE)
    external = []
    for i, m in enumerate(metas):
        r = recs[i]
        r["data_offset"] = m.data
        r["address"] = m.address
        r["birth_revision"] = m.birth_revision
        r["origin_pointer"] = NO_ORIGIN
        r["origin_type"] = NO_ORIGIN
        r["parent"] = NO_PARENT
        if m.post_commit is None:  # committed and written, nothing stored anywhere
            continue
        r["length"] = m.commit_size
        r["type"] = m.commit_type
        off = cache.origin_offsets(m.commit_origin)
        if off is None:
            external.append(i)  # the singularity's SpacePointer: stored by the host afterwards
        else:
            r["origin_pointer"], r["origin_type"] = off
        if m.commit_parent is not None:
            r["parent"] = index[id(m.commit_parent)]
    return recs, metas, external


def commit_heights(recs: np.ndarray) -> np.ndarray:
    """Height of every record above the blocks with no dirty child (the library's level:
    stormck_commit_device commits height 0, then 1, ... in record order)."""
    n = len(recs)
    h = np.zeros(n, dtype=np.int64)
    par = recs["parent"]
    for i in range(n):
        cur, d, steps = i, 0, 0
        while par[cur] >= 0:
            cur = int(par[cur])
            d += 1
            steps += 1
            if steps > n:
                raise ValueError("parent links form a cycle")
            if h[cur] >= d:
                break
            h[cur] = d
    return h


def check_references(metas, recs: np.ndarray, heights: np.ndarray) -> None:
    """storm's reference accounting over the whole forest, before anything changes: a
    child's PostCommitFunc lowers its parent's NReferences by the child's NCommits and
    adds them to the parent's (trace.go:278-281), so in children-first order every block
    must reach NReferences == 0 (cache.go:88-90)."""
    refs = [m.n_references for m in metas]
    commits = [m.n_commits for m in metas]
    for i in np.argsort(heights, kind="stable"):
        if refs[i] != 0:
            raise StillReferenced(f"dirty block at address {metas[i].address} keeps {refs[i]} references")
        p = int(recs["parent"][i])
        if p >= 0:
            refs[p] -= commits[i]
            commits[p] += commits[i]


def commit_cache(cache, run_commit) -> np.ndarray:
    """Cache.commitData through the level-synchronous commit (cache/cache.go:87-137).

    run_commit(records, revision, last_allocated) -> (checksums, last_allocated) runs
    stormck_commit_device on cache.data (in Go: blocks.CommitBatch over the registered
    arena), updating records' address / birth_revision in place. Then, as storm's loop
    leaves them: the relocations into the metadata and LastAllocatedBlock, the root's
    Pointer into the singularity, every block written at its address, NCommits /
    NReferences zero, PostCommitFuncs consumed, and each relocated block's Data swapped
    into the slot of its new address (cache.go:96-107), in commit order. Returns the
    checksums in record order."""
    recs, metas, external = cache_records(cache)
    if len(metas) == 0:
        return np.zeros(0, dtype=np.uint64)
    heights = commit_heights(recs)
    check_references(metas, recs, heights)
    before = recs["address"].copy()
    cs, last = run_commit(recs, cache.revision(), cache.last_allocated())
    cache.set_last_allocated(last)
    order = np.lexsort((np.arange(len(metas)), heights))  # the library's commit order
    for i in order:
        m = metas[i]
        m.address = int(recs["address"][i])
        m.birth_revision = int(recs["birth_revision"][i])
    for i in external:
        m = metas[i]
        cache.write_origin(m.commit_origin, int(cs[i]), m.address, m.birth_revision, int(recs["type"][i]))
    for i in order:
        m = metas[i]
        cache.store.write_block(m.address, cache.data[m.data:m.data + cache.bs])
        cache.dirty.pop(m, None)
        m.post_commit = None
        m.n_commits = 0
        m.n_references = 0
    for i in order:
        m = metas[i]
        if m.address != int(before[i]):
            m.state = INVALID_STATE
            m2 = cache.find_cached_block(m.address, m.birth_revision)
            m2.state = USED_STATE
            m2.data, m.data = m.data, m2.data
    return cs
