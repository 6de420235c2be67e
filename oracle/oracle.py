"""ORACLE — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the CPU baseline — never as the thing
measured or shipped. The product (storm_amd/, libstormck.so) does not import it.

Two restatements of storm's checksum path:

* ``liboracle.so`` (oracle/xxh64_oracle.c): XXH64 seed 0 = blocks.Checksum
  (/root/reference/blocks/checksum.go:15-17) via github.com/cespare/xxhash/v2
  v2.2.0 (go.mod:6), the synthetic generator, pointer-block packing
  (blocks/pointer/block.go:10-13) and the shard Merkle tree.
* pure-Python ``xxh64_py`` / ``pack_pointer_block_py`` for small cases, written
  independently of the C file (cross-check of the C restatement).

Pinned by tests/test_oracle.py against the public XXH64 known answers and the
libxxhash 0.8.2 fixtures in tests/golden/ (oracle/gen_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
from ctypes import c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p, POINTER
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

SYNTH_SEED = 0x53544F524D  # "STORM", SURVEY.md §8d
M64 = (1 << 64) - 1
P1, P2, P3, P4, P5 = (0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9,
                      0x85EBCA77C2B2AE63, 0x27D4EB2F165667C5)


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    lib = ctypes.CDLL(LIB_PATH)
    lib.oracle_xxh64.restype = c_uint64
    lib.oracle_xxh64.argtypes = [c_void_p, c_size_t]
    lib.oracle_checksum_batch.restype = None
    lib.oracle_checksum_batch.argtypes = [c_void_p, c_size_t, c_void_p, c_uint32, c_size_t, c_void_p]
    lib.oracle_checksum_batch_mt.restype = None
    lib.oracle_checksum_batch_mt.argtypes = [c_void_p, c_size_t, c_void_p, c_uint32, c_size_t, c_void_p, c_int]
    lib.oracle_checksum_gather_mt.restype = None
    lib.oracle_checksum_gather_mt.argtypes = [c_void_p, c_void_p, c_void_p, c_uint32, c_size_t, c_void_p, c_int]
    lib.oracle_synth_word.restype = c_uint64
    lib.oracle_synth_word.argtypes = [c_uint64, c_uint64, c_uint64]
    lib.oracle_fill_synthetic.restype = None
    lib.oracle_fill_synthetic.argtypes = [c_void_p, c_size_t, c_size_t, c_uint64, c_uint64]
    lib.oracle_pointer_block_size.restype = c_size_t
    lib.oracle_pointer_block_size.argtypes = [c_uint32]
    lib.oracle_merkle_root.restype = c_size_t
    lib.oracle_merkle_root.argtypes = [c_void_p, c_size_t, c_uint64, c_uint64, c_uint64, c_uint32,
                                       POINTER(c_uint64), POINTER(c_uint8)]
    lib.oracle_commit.restype = c_int
    lib.oracle_commit.argtypes = [c_void_p, c_void_p, c_size_t, c_uint64, POINTER(c_uint64), c_void_p]
    return lib


lib = _load()


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    return np.frombuffer(b, dtype=np.uint8)


def xxh64(b) -> int:
    a = _u8(b)
    return int(lib.oracle_xxh64(a.ctypes.data if a.size else None, a.size))


def checksum_batch(buf, n: int, stride: int, length: int = 0, lens: Optional[Sequence[int]] = None,
                   threads: int = 1) -> np.ndarray:
    a = _u8(buf)
    out = np.zeros(n, dtype=np.uint64)
    la = None if lens is None else np.ascontiguousarray(np.asarray(lens, dtype=np.uint32))
    lp = None if la is None else la.ctypes.data
    if threads > 1:
        lib.oracle_checksum_batch_mt(a.ctypes.data, stride, lp, length, n, out.ctypes.data, threads)
    else:
        lib.oracle_checksum_batch(a.ctypes.data, stride, lp, length, n, out.ctypes.data)
    return out


def checksum_gather(buf, offs, length: int = 0, lens: Optional[Sequence[int]] = None,
                    threads: int = 8) -> np.ndarray:
    """Block i = buf[offs[i] : offs[i] + (lens[i] if lens else length)]."""
    a = _u8(buf)
    oa = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    n = oa.size
    out = np.zeros(n, dtype=np.uint64)
    la = None if lens is None else np.ascontiguousarray(np.asarray(lens, dtype=np.uint32))
    lib.oracle_checksum_gather_mt(a.ctypes.data, oa.ctypes.data, None if la is None else la.ctypes.data, length, n,
                                  out.ctypes.data, threads)
    return out


def fill_synthetic(n: int, stride: int, first: int = 0, seed: int = SYNTH_SEED) -> np.ndarray:
    """n synthetic blocks of `stride` bytes for logical indices first..first+n-1."""
    out = np.empty(n * stride, dtype=np.uint8)
    lib.oracle_fill_synthetic(out.ctypes.data, stride, n, first, seed)
    return out


def pointer_block_size(fanout: int) -> int:
    return int(lib.oracle_pointer_block_size(fanout))


def merkle_root(leaf_cs, leaf_addr_base: int, node_addr_base: int, rev: int,
                fanout: int = 1200) -> Tuple[int, int, int, int]:
    """(Checksum, Address, BirthRevision, BlockType) of the shard tree root."""
    cs = np.ascontiguousarray(np.asarray(leaf_cs, dtype=np.uint64))
    root = (c_uint64 * 3)()
    rt = c_uint8(0)
    lib.oracle_merkle_root(cs.ctypes.data if cs.size else None, cs.size, leaf_addr_base, node_addr_base, rev, fanout,
                           root, ctypes.byref(rt))
    return int(root[0]), int(root[1]), int(root[2]), int(rt.value)


# ---------------------------------------------------------------------------
# pure-Python second restatement (small inputs only)
# ---------------------------------------------------------------------------

def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (64 - r))) & M64


def _round(acc: int, w: int) -> int:
    acc = (acc + w * P2) & M64
    return (_rotl(acc, 31) * P1) & M64


def xxh64_py(data: bytes) -> int:
    n = len(data)
    i = 0
    if n >= 32:
        v = [(P1 + P2) & M64, P2, 0, (-P1) & M64]
        while i + 32 <= n:
            for k in range(4):
                v[k] = _round(v[k], int.from_bytes(data[i + 8 * k:i + 8 * k + 8], "little"))
            i += 32
        h = (_rotl(v[0], 1) + _rotl(v[1], 7) + _rotl(v[2], 12) + _rotl(v[3], 18)) & M64
        for k in range(4):
            h ^= _round(0, v[k])
            h = (h * P1 + P4) & M64
    else:
        h = P5
    h = (h + n) & M64
    while i + 8 <= n:
        h ^= _round(0, int.from_bytes(data[i:i + 8], "little"))
        h = (_rotl(h, 27) * P1 + P4) & M64
        i += 8
    if i + 4 <= n:
        h ^= (int.from_bytes(data[i:i + 4], "little") * P1) & M64
        h = (_rotl(h, 23) * P2 + P3) & M64
        i += 4
    while i < n:
        h ^= (data[i] * P5) & M64
        h = (_rotl(h, 11) * P1) & M64
        i += 1
    h ^= h >> 33
    h = (h * P2) & M64
    h ^= h >> 29
    h = (h * P3) & M64
    h ^= h >> 32
    return h


def pack_pointer_block_py(entries: Iterable[Tuple[int, int, int, int]], fanout: int) -> bytes:
    """storm pointer.Block bytes from (cs, addr, rev, type) entries."""
    entries = list(entries)
    assert len(entries) <= fanout
    size = (25 * fanout + 7) & ~7
    buf = bytearray(size)
    for k, (cs, addr, rev, typ) in enumerate(entries):
        struct.pack_into("<QQQ", buf, 24 * k, cs & M64, addr & M64, rev & M64)
        buf[24 * fanout + k] = typ
    return bytes(buf)


def combine_roots(table: Sequence[Tuple[int, int, int, int]], rev: int, root_addr: int,
                  fanout: int = 1200) -> Tuple[int, int, int, int]:
    """Global root over shard roots (storm_amd.dist.global_root semantics)."""
    return xxh64(pack_pointer_block_py(table, fanout)), root_addr, rev, 1


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def synth_leaf_checksums(n: int, seed: int = SYNTH_SEED) -> np.ndarray:
    """Cheap synthetic leaf checksums for Merkle-only fixtures: splitmix64(seed ^ i)."""
    x = (np.arange(n, dtype=np.uint64) ^ np.uint64(seed)) + np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def commit(arena: np.ndarray, blocks: np.ndarray, revision: int, last_allocated: int):
    """storm's serial commit loop (oracle_commit) over a host arena copy; `blocks` is a
    storm_amd.commit.DIRTY_DTYPE array (updated in place). Returns (checksums, last)."""
    assert blocks.dtype.itemsize == 56 and blocks.flags["C_CONTIGUOUS"]
    assert arena.dtype == np.uint8 and arena.flags["C_CONTIGUOUS"]
    out = np.zeros(blocks.shape[0], dtype=np.uint64)
    la = c_uint64(last_allocated)
    rc = lib.oracle_commit(arena.ctypes.data, blocks.ctypes.data, blocks.shape[0], revision, ctypes.byref(la),
                           out.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_commit: cyclic or unreachable dirty set")
    return out, la.value


def commit_py(arena: bytearray, blocks, revision: int, last_allocated: int):
    """Pure-Python restatement of the same loop for small forests (cross-checks the C
    oracle). `blocks` is a list of dicts with the stormck_dirty_block fields."""
    n = len(blocks)
    height = [0] * n
    for i in range(n):  # walk each leaf-to-root chain
        h, p = 0, blocks[i]["parent"]
        while p >= 0:
            h += 1
            height[p] = max(height[p], h)
            p = blocks[p]["parent"]
    pending = [0] * n
    for b in blocks:
        if b["parent"] >= 0:
            pending[b["parent"]] += 1
    order = sorted(range(n), key=lambda i: (height[i], i))
    cs = [0] * n
    done = [False] * n
    while not all(done):
        for i in order:
            b = blocks[i]
            if done[i] or pending[i]:
                continue
            if b["birth_revision"] <= revision:
                last_allocated += 1
                b["address"], b["birth_revision"] = last_allocated, revision + 1
            off = b["data_offset"]
            cs[i] = xxh64_py(bytes(arena[off:off + b["length"]]))
            if b["origin_pointer"] != M64:
                struct.pack_into("<QQQ", arena, b["origin_pointer"], cs[i], b["address"], b["birth_revision"])
                arena[b["origin_type"]] = b["type"]
            if b["parent"] >= 0:
                pending[b["parent"]] -= 1
            done[i] = True
    return cs, last_allocated
