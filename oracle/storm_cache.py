"""TEST INFRASTRUCTURE (oracle): storm's cache layer as far as Cache.Commit needs it.

A pure-Python restatement of the reference's metadata, tracing and commit loop, so the
stormck commit binding (storm_amd/commit.py commit_cache, the Python mirror of
integration/go/cache/commit_stormck.go) can be held against storm's own sequential
commit on the same simulated state. Only tests import this module. It restates:

  cache/types.go:17-31      blockMetadata (+ the commit record the stormck build keeps,
                            integration/go/cache/trace_types.patch), BlockOrigin
  cache/cache.go:16-53      Cache / New: cache.data, metadata, addressingOffsets, singularity
  cache/cache.go:57-85      Commit: commitData, then Revision++ and the singularity checksum
  cache/cache.go:87-111     commitData: sweep the dirty set, commit blocks with NReferences == 0,
                            relocate + swap Data with the slot of the new address
  cache/cache.go:113-137    commitBlock: relocation, WriteBlock, PostCommitFunc, NCommits = 0
  cache/cache.go:139-167    fetchBlock: ReadBlock + VerifyChecksum (a cold block)
  cache/cache.go:169-241    newBlock / findCachedBlock (free, invalid, unreferenced slots)
  cache/cache.go:243-255    dirtyBlock / invalidateBlock
  cache/trace.go:48-259     TraceTagForUpdating: Free, Leaf and Pointer cases (no split)
  cache/trace.go:261-320    the two PostCommitFunc constructors
  cache/trace.go:322-345    Trace.Commit / Trace.Release
  persistence/init.go:33-56 Initialize (singularity at address 0)

Differences that do not change what Commit computes: Go's map iteration order is
random, so the sweep here takes an explicit order (each pass visits a snapshot of the
dirty set sorted by `order_key`); addressingOffsets is a seeded numpy permutation
(Go's math/rand is not restated); blocks.Checksum is the C oracle's XXH64.

Block images are byte ranges of cache.data (photon views): pointer.Block of `fanout`
entries (Pointers[F] 24 B each, then PointedBlockTypes[F], blocks/pointer/block.go:10-13),
leaves of `leaf_len` bytes whose first 25 bytes can hold the origin of a nested tree
{Pointer, BlockType} (as keystore's trees hang off leaves of a parent tree).
"""
from __future__ import annotations

import struct
from typing import Callable, Dict, List, Optional

import numpy as np

from oracle import oracle as o

FREE_TYPE, POINTER_TYPE, LEAF_TYPE = 0, 1, 2          # blocks/types.go:7-15
FREE_STATE, USED_STATE, INVALID_STATE = 0, 1, 2       # cache/types.go:10-15
SING_SIZE = 72                                        # blocks/singularity/block.go:8-19
S_CHECKSUM, S_STORMID, S_REVISION, S_NBLOCKS, S_SPACE_PTR, S_SPACE_TYPE, S_LAST = 0, 8, 16, 24, 32, 56, 64


def pointer_block_size(fanout: int) -> int:
    return (25 * fanout + 7) & ~7


class Origin:
    """BlockOrigin (cache/types.go:27-31): where a block's Pointer and BlockType live.
    `where` is "data" (byte offsets into cache.data) or "singularity" (offsets into the
    singularity image, which is not part of cache.data)."""

    def __init__(self, where: str, pointer: int, btype: int):
        self.where, self.pointer, self.btype = where, pointer, btype

    def shifted(self, delta: int) -> "Origin":
        return Origin(self.where, self.pointer + delta, self.btype + delta)


class Meta:
    """blockMetadata (cache/types.go:17-25). data = byte offset of its Data slice in
    cache.data. commit_* = the record the stormck build keeps beside PostCommitFunc."""

    def __init__(self, data: int):
        self.data = data
        self.address = 0
        self.birth_revision = 0
        self.n_commits = 0
        self.n_references = 0
        self.state = FREE_STATE
        self.post_commit: Optional[Callable[[], None]] = None
        self.commit_origin: Optional[Origin] = None
        self.commit_parent: Optional["Meta"] = None
        self.commit_size = 0
        self.commit_type = FREE_TYPE


class Store:
    """persistence.Store over an in-memory device: address -> block image."""

    def __init__(self, block_size: int, n_blocks: int):
        self.block_size, self.n_blocks = block_size, n_blocks
        self.dev: Dict[int, bytes] = {}
        self.writes: List[int] = []

    def write_block(self, address: int, data) -> None:
        b = bytes(data)
        self.dev[address] = b + bytes(self.block_size - len(b))
        self.writes.append(address)

    def read_block(self, address: int, n: int) -> bytes:
        return self.dev.get(address, bytes(self.block_size))[:n]


def initialize(store: Store, storm_id: int = 0x4200812112C24445) -> None:
    """persistence.Initialize: the singularity at address 0, checksummed with Checksum = 0."""
    s = bytearray(SING_SIZE)
    struct.pack_into("<QQ", s, S_STORMID, storm_id, 0)
    struct.pack_into("<Q", s, S_NBLOCKS, store.n_blocks)
    struct.pack_into("<Q", s, S_CHECKSUM, o.xxh64(bytes(s)))
    store.write_block(0, s)


class Trace:
    """cache.Trace (trace.go:322-345)."""

    def __init__(self, c: "Cache", meta: Meta, pointer_blocks: List[Meta], parent: Optional["Trace"]):
        self.c, self.meta, self.pointer_blocks, self.parent = c, meta, pointer_blocks, parent

    def commit(self) -> None:
        self.meta.n_references -= 1
        self.c.dirty_block(self.meta, 1)

    def release(self) -> None:
        self.meta.n_references -= 1
        for m in self.pointer_blocks:
            m.n_references -= 1
        if self.parent is not None:
            self.parent.release()


class Cache:
    """cache.Cache (cache/cache.go:16-53)."""

    def __init__(self, store: Store, n_slots: int, fanout: int, leaf_len: int, seed: int = 0):
        self.store, self.fanout, self.leaf_len = store, fanout, leaf_len
        self.bs = store.block_size
        self.n_blocks = n_slots
        raw = np.zeros(n_slots * self.bs + 4096, dtype=np.uint8)  # cache.data, page-aligned (as Go's large make)
        off = (-raw.ctypes.data) % 4096
        self.data = raw[off:off + n_slots * self.bs]
        self.blocks = [Meta(i * self.bs) for i in range(n_slots)]
        self.addressing = np.random.default_rng(seed).permutation(n_slots).astype(np.int64)
        self.dirty: Dict[Meta, None] = {}  # insertion-ordered set
        self.sing = bytearray(store.read_block(0, SING_SIZE))

    # --- the singularity --------------------------------------------------------
    def sget(self, off: int) -> int:
        return struct.unpack_from("<Q", self.sing, off)[0]

    def sset(self, off: int, v: int) -> None:
        struct.pack_into("<Q", self.sing, off, v)

    def space_origin(self) -> Origin:
        return Origin("singularity", S_SPACE_PTR, S_SPACE_TYPE)

    # --- origins (*origin.Pointer / *origin.BlockType) --------------------------
    def _buf(self, origin: Origin):
        return self.sing if origin.where == "singularity" else self.data

    def read_origin(self, origin: Origin):
        buf = self._buf(origin)
        cs, addr, birth = struct.unpack_from("<QQQ", bytes(buf[origin.pointer:origin.pointer + 24]))
        return cs, addr, birth, int(buf[origin.btype])

    def write_origin(self, origin: Origin, cs: int, addr: int, birth: int, btype: int) -> None:
        buf = self._buf(origin)
        buf[origin.pointer:origin.pointer + 24] = np.frombuffer(struct.pack("<QQQ", cs, addr, birth), np.uint8) \
            if isinstance(buf, np.ndarray) else struct.pack("<QQQ", cs, addr, birth)
        buf[origin.btype] = btype

    # what the stormck binding reads (storm_amd/commit.py commit_cache)
    def origin_offsets(self, origin: Origin):
        return (origin.pointer, origin.btype) if origin.where == "data" else None

    def revision(self) -> int:
        return self.sget(S_REVISION)

    def last_allocated(self) -> int:
        return self.sget(S_LAST)

    def set_last_allocated(self, v: int) -> None:
        self.sset(S_LAST, v)

    def checksum(self, off: int, n: int) -> int:  # blocks.BlockChecksum over Sizeof(T) bytes
        return o.xxh64(self.data[off:off + n])

    # --- cache.go ------------------------------------------------------------------
    def commit(self, order_key: Callable[[Meta], object] = None) -> None:
        """Cache.Commit (cache.go:57-85) with storm's own commitData."""
        self.commit_data(order_key)
        self.finish_commit()

    def finish_commit(self) -> None:
        self.sset(S_REVISION, self.sget(S_REVISION) + 1)
        self.sset(S_CHECKSUM, 0)
        self.sset(S_CHECKSUM, o.xxh64(bytes(self.sing)))
        self.store.write_block(0, self.sing)

    def commit_data(self, order_key=None) -> None:
        """cache.go:87-111. Each pass visits a snapshot of the dirty set (Go ranges over a
        map it is inserting into; any visiting order is a storm order)."""
        while self.dirty:
            snapshot = list(self.dirty)
            if order_key is not None:
                snapshot.sort(key=order_key)
            progressed = False
            for meta in snapshot:
                if meta not in self.dirty or meta.n_references > 0:
                    continue
                progressed = True
                addr_before = meta.address
                self.commit_block(meta)
                if meta.address != addr_before:
                    meta.state = INVALID_STATE
                    meta2 = self.find_cached_block(meta.address, meta.birth_revision)
                    meta2.state = USED_STATE
                    meta2.data, meta.data = meta.data, meta2.data
            if not progressed:
                raise RuntimeError("storm would spin: every dirty block is still referenced")

    def commit_block(self, meta: Meta) -> None:
        """cache.go:113-137."""
        rev = self.sget(S_REVISION)
        if meta.birth_revision <= rev:
            self.sset(S_LAST, self.sget(S_LAST) + 1)
            meta.address = self.sget(S_LAST)
            meta.birth_revision = rev + 1
        self.store.write_block(meta.address, self.data[meta.data:meta.data + self.bs])
        self.dirty.pop(meta, None)
        if meta.post_commit is not None:
            f, meta.post_commit = meta.post_commit, None
            f()
        meta.n_commits = 0

    def fetch_block(self, address: int, birth: int, n: int, expected: int) -> Meta:
        """cache.go:139-167 (ReadBlock + VerifyChecksum of a cold block)."""
        if address > self.sget(S_LAST):
            raise KeyError(f"block {address} does not exist")
        meta = self.find_cached_block(address, birth)
        if meta.state == USED_STATE:
            return meta
        raw = self.store.read_block(address, n)
        self.data[meta.data:meta.data + n] = np.frombuffer(raw, np.uint8)
        if o.xxh64(raw) != expected:
            raise ValueError(f"checksum mismatch for block {address}")
        meta.state = USED_STATE
        return meta

    def new_block(self, size: int) -> Meta:
        """cache.go:169-180 + newBlock[T] (cache.go:276-287): zeroed image."""
        self.sset(S_LAST, self.sget(S_LAST) + 1)
        meta = self.find_cached_block(self.sget(S_LAST), self.sget(S_REVISION) + 1)
        meta.state = USED_STATE
        self.dirty[meta] = None
        self.data[meta.data:meta.data + size] = 0
        return meta

    def find_cached_block(self, address: int, birth: int) -> Meta:
        """cache.go:182-241."""
        seed = address % self.n_blocks
        found, sel, invalid_found, unref_found = False, 0, False, False
        for i in range(self.n_blocks):
            idx = int((seed + self.addressing[i]) % self.n_blocks)
            m = self.blocks[idx]
            if m.state == FREE_STATE:
                if not invalid_found:
                    found, sel = True, idx
                break
            if m.state == INVALID_STATE:
                if not invalid_found:
                    invalid_found = unref_found = found = True
                    sel = idx
            else:
                if m.address == address:
                    found, sel = True, idx
                    break
                if not unref_found and m.n_references == 0:
                    unref_found = found = True
                    sel = idx
        if not found:
            raise RuntimeError("there are no free slots in cache")
        meta = self.blocks[sel]
        if meta.state == USED_STATE and meta.address != address:
            if meta in self.dirty:
                self.commit_block(meta)
            meta.state = INVALID_STATE
        if meta.state != USED_STATE:
            meta.n_commits = meta.n_references = 0
            meta.post_commit = None
        meta.address, meta.birth_revision = address, birth
        return meta

    def dirty_block(self, meta: Meta, n_commits: int) -> None:
        meta.n_commits += n_commits
        self.dirty[meta] = None

    # --- trace.go ------------------------------------------------------------------
    def _pointer_post_commit(self, origin: Origin, parent: Optional[Meta], meta: Meta, off: int):
        """newPointerBlockPostCommitFunc (trace.go:261-283). The stormck build also records
        origin, parent, Sizeof(pointer.Block) and the type beside the closure."""
        size = pointer_block_size(self.fanout)
        meta.commit_origin, meta.commit_parent, meta.commit_size, meta.commit_type = origin, parent, size, POINTER_TYPE

        def f():
            self.write_origin(origin, self.checksum(off, size), meta.address, meta.birth_revision, POINTER_TYPE)
            if parent is not None:
                parent.n_references -= meta.n_commits
                self.dirty_block(parent, meta.n_commits)
        return f

    def _leaf_post_commit(self, origin: Origin, parent: Optional[Meta], meta: Meta, off: int):
        """newLeafBlockPostCommitFunc (trace.go:286-308)."""
        size = self.leaf_len
        meta.commit_origin, meta.commit_parent, meta.commit_size, meta.commit_type = origin, parent, size, LEAF_TYPE

        def f():
            self.write_origin(origin, self.checksum(off, size), meta.address, meta.birth_revision, LEAF_TYPE)
            if parent is not None:
                parent.n_references -= meta.n_commits
                self.dirty_block(parent, meta.n_commits)
        return f

    def trace_for_updating(self, origin: Origin, parent_trace: Optional[Trace], tag: int):
        """TraceTagForUpdating (trace.go:48-259) without the split case. Returns
        (leaf meta, Trace, tag reminder)."""
        cur = origin
        parent_meta = parent_trace.meta if parent_trace is not None else None
        ptrace: List[Meta] = []
        rem = tag
        t = parent_trace
        while t is not None:
            t.meta.n_references += 1
            for m in t.pointer_blocks:
                m.n_references += 1
            t = t.parent
        while True:
            cs, addr, birth, btype = self.read_origin(cur)
            if btype == FREE_TYPE:
                meta = self.new_block(self.leaf_len)
                meta.post_commit = self._leaf_post_commit(cur, parent_meta, meta, meta.data)
                meta.n_references = 1
                self.write_origin(cur, 0, meta.address, meta.birth_revision, LEAF_TYPE)
                return meta, Trace(self, meta, ptrace, parent_trace), rem
            if btype == LEAF_TYPE:
                meta = self.fetch_block(addr, birth, self.leaf_len, cs)
                meta.post_commit = self._leaf_post_commit(cur, parent_meta, meta, meta.data)
                meta.n_references += 1
                return meta, Trace(self, meta, ptrace, parent_trace), rem
            meta = self.fetch_block(addr, birth, pointer_block_size(self.fanout), cs)
            meta.n_references += 1
            meta.post_commit = self._pointer_post_commit(cur, parent_meta, meta, meta.data)
            ptrace.append(meta)
            k = rem % self.fanout
            rem //= self.fanout
            parent_meta = meta
            cur = Origin("data", meta.data + 24 * k, meta.data + 24 * self.fanout + k)

    def leaf_child_origin(self, meta: Meta) -> Origin:
        """The nested-tree origin a simulated leaf holds at its start ({Pointer, BlockType})."""
        return Origin("data", meta.data, meta.data + 24)


def build_tree(store: Store, fanout: int, leaf_len: int, tags, revision: int, seed: int) -> None:
    """A committed storm tree of an earlier revision, written straight to the store: the
    singularity -> pointer levels -> one leaf per tag. Tag t sits at child (t // F^k) % F
    of its level-k pointer block (k = 0 at the root), as TraceTagForReading /
    TraceTagForUpdating walk it (trace.go:38-40); the depth is the smallest d with
    F^d > max(tag). Random leaf bytes (the first 25 bytes zero: an empty nested-tree
    origin), every block born in `revision`, addresses 1.. leaves first, then pointer
    blocks bottom-up. The singularity records the root, the revision and the last address."""
    rng = np.random.default_rng(seed)
    tags = sorted(set(int(t) for t in tags))
    depth = 0
    while tags and fanout ** depth <= tags[-1]:
        depth += 1
    addr = 0
    entries = {}  # digit prefix -> (cs, addr, type); full-length prefixes are leaves
    for t in tags:
        addr += 1
        img = rng.integers(0, 256, leaf_len, dtype=np.uint8)
        img[:25] = 0
        store.write_block(addr, img)
        entries[tuple((t // fanout ** k) % fanout for k in range(depth))] = (o.xxh64(img), addr, LEAF_TYPE)
    for k in range(depth, 0, -1):
        parents: Dict[tuple, list] = {}
        for prefix, e in sorted(entries.items()):
            parents.setdefault(prefix[:k - 1], []).append((prefix[k - 1], e))
        entries = {}
        for pp, kids in sorted(parents.items()):
            img = bytearray(pointer_block_size(fanout))
            for i, (cs, a, bt) in kids:
                struct.pack_into("<QQQ", img, 24 * i, cs, a, revision)
                img[24 * fanout + i] = bt
            addr += 1
            store.write_block(addr, img)
            entries[pp] = (o.xxh64(bytes(img)), addr, POINTER_TYPE)
    s = bytearray(store.read_block(0, SING_SIZE))
    if entries:
        cs, a, bt = entries[()]
        struct.pack_into("<QQQ", s, S_SPACE_PTR, cs, a, revision)
        s[S_SPACE_TYPE] = bt
    struct.pack_into("<Q", s, S_REVISION, revision)
    struct.pack_into("<Q", s, S_LAST, addr)
    struct.pack_into("<Q", s, S_CHECKSUM, 0)
    struct.pack_into("<Q", s, S_CHECKSUM, o.xxh64(bytes(s)))
    store.write_block(0, s)


def snapshot(c: Cache) -> dict:
    """Everything Commit leaves behind, for comparing two builds."""
    return {"store": dict(c.store.dev), "sing": bytes(c.sing), "data": c.data.tobytes(),
            "metas": [(m.data, m.address, m.birth_revision, m.n_commits, m.n_references, m.state,
                       m.post_commit is None) for m in c.blocks],
            "dirty": len(c.dirty)}
