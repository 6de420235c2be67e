"""Multi-GPU sharding of a checksum batch (one process per GPU).

Blocks are independent, so a batch shards into contiguous index ranges with no
data-path collective. The one exchange is the per-shard Merkle roots: every rank
all-gathers the ``world`` root Pointers (4 x u64 each; RCCL over xGMI on GPUs,
gloo in the CPU tests) and combines them into one storm pointer block whose hash
is the global root. The reference has no multi-device code; the
node format is storm's pointer.Block (blocks/pointer/block.go:10-13).
"""
from __future__ import annotations

from typing import Callable, List, Tuple


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) block range of `rank`: sizes differ by at most one."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard_node_addr_base(n_total: int, lo: int) -> int:
    """Address base of a shard's interior Merkle nodes: n_total + lo. Shard s gets
    [n_total + lo_s, n_total + lo_s + nodes_s); for fanout >= 3, nodes_s < hi_s - lo_s
    for any shard of two or more leaves (tests/test_dist.py checks it), so the ranges
    of different shards never overlap and never collide with leaf addresses
    [0, n_total)."""
    return n_total + lo


def global_root_addr(n_total: int) -> int:
    """Address of the combining node (above every shard-node range)."""
    return 2 * n_total


def gather_shard_roots(local_root, group=None):
    """All-gather each rank's root row (int64 tensor [4] = {cs, addr, rev, type})
    into a [world, 4] table in rank order. Works for nccl (RCCL) and gloo."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    row = local_root.reshape(1, 4).contiguous()
    if local_root.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal on CPU collectives (e.g. several ranks sharing one GPU): gloo
        # gathers host tensors; the production backend is nccl (RCCL over xGMI).
        table = torch.empty((world, 4), dtype=row.dtype)
        dist.all_gather_into_tensor(table, row.cpu(), group=group)
        return table.to(local_root.device)
    table = torch.empty((world, 4), dtype=row.dtype, device=row.device)
    dist.all_gather_into_tensor(table, row, group=group)
    return table


def global_root(local_root, rev: int, n_total: int, combine: Callable, group=None):
    """Gather the shard roots and combine them: ``combine(table, rev, root_addr)``
    hashes the pointer block of the table rows (engine.combine_roots_tensor on GPU).
    Every rank returns the identical global root."""
    table = gather_shard_roots(local_root, group)
    return combine(table, rev, global_root_addr(n_total)), table


def plan(n: int, world: int) -> List[Tuple[int, int]]:
    return [shard_range(n, world, r) for r in range(world)]
