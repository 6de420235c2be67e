"""Multi-GPU in one process (storm's case): device-resident shards, their trees, the RCCL
gather of the shard roots and the combining node, through the C-ABI
(stormck_shard_plan / stormck_merkle_root_multi, include/stormck.h).

storm is one Go process, so on an 8-GPU node it drives every GPU from one process; this is
the entry its cgo shim binds (integration/go/blocks/checksum_stormck.go MerkleRootDevices).
The process-per-GPU path (torch.distributed over RCCL, storm_amd/dist.py) computes the same
roots; both follow the shard convention of SURVEY.md §8e (tests/test_multi_root.py).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

from . import _lib
from ._lib import PointerStruct, ShardStruct, check, lib

POINTERS_PER_BLOCK = 1200  # blocks/pointer/params.go:6


def plan(n_total: int, n_shards: int, devices: Sequence[int]) -> Tuple[List[ShardStruct], int]:
    """stormck_shard_plan: n_total leaves in n_shards contiguous shards dealt to `devices` in
    consecutive runs; returns the shards (pointers and streams unset) and the combining
    node's address (2 * n_total). Needs no device."""
    arr = (ShardStruct * n_shards)()
    devs = (ctypes.c_int * len(devices))(*devices)
    root_addr = ctypes.c_uint64(0)
    check(lib.stormck_shard_plan(n_total, n_shards, devs if len(devices) else None, len(devices), arr,
                                 ctypes.byref(root_addr)))
    return list(arr), int(root_addr.value)


def layout(shards: Sequence[ShardStruct]) -> Tuple[List[int], int, List[int]]:
    """stormck_multi_layout: (the shards' distinct devices in order of first appearance, R =
    the most shards on one device, each shard's row of the gathered D x R table). Needs no
    device: the gather layout stormck_merkle_root_multi uses, for the CPU tests."""
    n = len(shards)
    arr = (ShardStruct * n)(*shards)
    devs, tr = (ctypes.c_int32 * 64)(), (ctypes.c_uint32 * max(n, 1))()
    nd, rows = ctypes.c_uint32(0), ctypes.c_uint32(0)
    check(lib.stormck_multi_layout(arr, n, devs, ctypes.byref(nd), ctypes.byref(rows), tr))
    return [int(devs[i]) for i in range(nd.value)], int(rows.value), [int(tr[i]) for i in range(n)]


def _row(p: PointerStruct, t: int) -> Tuple[int, int, int, int]:
    return int(p.Checksum), int(p.Address), int(p.BirthRevision), int(t)


def merkle_root_multi(shards: Sequence[ShardStruct], rev: int, root_addr: int, fanout: int = POINTERS_PER_BLOCK
                      ) -> Tuple[Tuple[int, int, int, int], List[Tuple[int, int, int, int]]]:
    """stormck_merkle_root_multi: (global root row {cs, addr, rev, type}, shard root rows).
    Synchronous; raises StormckError on any failure (RCCL included)."""
    n = len(shards)
    arr = (ShardStruct * n)(*shards)
    root, rtype = PointerStruct(), ctypes.c_uint8(0)
    sroots, stypes = (PointerStruct * n)(), (ctypes.c_uint8 * n)()
    check(lib.stormck_merkle_root_multi(arr, n, rev, root_addr, fanout, ctypes.byref(root), ctypes.byref(rtype),
                                        sroots, stypes))
    return _row(root, rtype.value), [_row(sroots[i], stypes[i]) for i in range(n)]


def shard(device: int, n: int, d_checksums: int, leaf_addr_base: int, node_addr_base: int, d_blocks: int = 0,
          stride: int = 0, length: int = 0, stream: int = 0) -> ShardStruct:
    """One stormck_shard (for callers that do not use plan())."""
    return ShardStruct(d_blocks or None, stride, n, d_checksums or None, leaf_addr_base, node_addr_base,
                       stream or None, device, length)


def set_buffers(sh: ShardStruct, d_checksums: int, d_blocks: int = 0, stride: int = 0, length: int = 0,
                stream: Optional[int] = None) -> ShardStruct:
    """Fill the pointers of a planned shard."""
    sh.d_checksums = d_checksums or None
    sh.d_blocks = d_blocks or None
    sh.stride = stride
    sh.len = length
    if stream is not None:
        sh.stream = stream or None
    return sh


__all__ = ["plan", "layout", "merkle_root_multi", "shard", "set_buffers", "_lib"]
