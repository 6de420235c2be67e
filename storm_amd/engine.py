"""Device-resident entry points (HBM in, HBM out) over libstormck.

Raw-pointer functions mirror include/stormck.h one to one; the ``*_tensor``
helpers take torch tensors (torch is plumbing here: device memory and streams)
and launch on torch's current stream of the tensor's device.
"""
from __future__ import annotations

import os

from typing import Optional, Tuple

from . import _lib
from ._lib import check, lib

POINTERS_PER_BLOCK = 1200  # blocks/pointer/params.go:6


# Batches the library may give to a ring-staged kernel (k_xxh64_wide_multi, whose
# bounded waits report a stall in the stream's fault slot rather than in the output):
# more than kWideBatch (128) blocks and at most kMultiBpwRing (8) per CU
# (storm_amd/csrc/stormck.hip multi_bpw).
_RING_MIN_EXCLUSIVE, _RING_PER_CU = 128, 8
_cus = {}


def _cu_count() -> int:
    import torch
    d = torch.cuda.current_device()
    if d not in _cus:
        _cus[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _cus[d]


def may_ring(n: int) -> bool:
    """Whether a batch of n blocks can take a ring-staged kernel on the current device."""
    return _RING_MIN_EXCLUSIVE < n <= _RING_PER_CU * _cu_count()


def _after_launch(n: int, stream: int, check_status) -> None:
    # check_status: True = synchronise `stream` and raise on a ring fault of this stream
    # (stormck_device_status); None (the default) = do so only when the batch could have
    # taken a ring kernel, which makes those mid-size launches synchronous; False = the
    # caller checks (device_status) itself, e.g. once after a series of launches, and the
    # launch stays asynchronous. A stream that is being captured into a graph is not
    # checked here (the library reports that for the stream passed, not torch's current
    # one): a captured launch reports into the slot of the stream it was captured on, so
    # check that stream after a replay.
    if check_status is None:
        check_status = may_ring(n)
        if check_status:
            rc = lib.stormck_device_status(stream or None)
            if rc == _lib.EINVAL and "being captured" in _lib.last_error():
                return
            check(rc)
            return
    if check_status:
        device_status(stream)


def checksum_device(d_base: int, stride: int, n: int, d_out: int, length: int = 0, d_lens: int = 0,
                    stream: int = 0, check_status=None) -> None:
    check(lib.stormck_checksum_device(d_base, stride, d_lens or None, length, n, d_out, stream or None))
    _after_launch(n, stream, check_status)


def checksum_gather_device(d_base: int, d_offsets: int, n: int, d_out: int, length: int = 0, d_lens: int = 0,
                           stream: int = 0, check_status=None) -> None:
    check(lib.stormck_checksum_gather_device(d_base, d_offsets, d_lens or None, length, n, d_out, stream or None))
    _after_launch(n, stream, check_status)


def verify_device(d_base: int, stride: int, n: int, d_expected: int, d_result: int, length: int = 0, d_lens: int = 0,
                  stream: int = 0, check_status=None) -> None:
    """Batched VerifyChecksum into d_result = {first_bad, n_bad}. A stalled ring
    workgroup counts its blocks as mismatches (fails closed); the status check also
    raises on it."""
    check(lib.stormck_verify_device(d_base, stride, d_lens or None, length, n, d_expected, d_result, stream or None))
    _after_launch(n, stream, check_status)


def key_tags_device(d_keys: int, n: int, d_out: int, stride: int = 0, length: int = 0, d_offsets: int = 0,
                    d_lens: int = 0, stream: int = 0) -> None:
    """f4: xxhash.Sum64(key) per key (keystore/keystore.go:33,66), one lane per key."""
    check(lib.stormck_key_tags_device(d_keys, stride, d_offsets or None, d_lens or None, length, n, d_out,
                                      stream or None))


def fill_synthetic_device(d_dst: int, stride: int, n: int, first: int, seed: int, stream: int = 0) -> None:
    check(lib.stormck_fill_synthetic_device(d_dst, stride, n, first, seed, stream or None))


def pointer_level_device(d_child_cs: int, m: int, child_addr_base: int, rev: int, child_type: int, fanout: int,
                         d_parent_cs: int, stream: int = 0) -> None:
    check(lib.stormck_pointer_level_device(d_child_cs, m, child_addr_base, rev, child_type, fanout, d_parent_cs,
                                           stream or None))


def pointer_node_device(d_entries: int, d_types: int, count: int, fanout: int, d_out_cs: int, stream: int = 0) -> None:
    check(lib.stormck_pointer_node_device(d_entries or None, d_types or None, count, fanout, d_out_cs, stream or None))


def pack_pointer_blocks_device(d_child_cs: int, m: int, child_addr_base: int, rev: int, child_type: int, fanout: int,
                               d_blocks: int, dst_stride: int, stream: int = 0) -> None:
    check(lib.stormck_pack_pointer_blocks_device(d_child_cs, m, child_addr_base, rev, child_type, fanout, d_blocks,
                                                 dst_stride, stream or None))


def merkle_workspace_bytes(n: int, fanout: int = POINTERS_PER_BLOCK) -> int:
    return int(lib.stormck_merkle_workspace_bytes(n, fanout))


def merkle_root_device(d_leaf_cs: int, n: int, leaf_addr_base: int, node_addr_base: int, rev: int, fanout: int,
                       d_workspace: int, workspace_bytes: int, d_root: int, d_root_type: int, stream: int = 0) -> None:
    check(lib.stormck_merkle_root_device(d_leaf_cs or None, n, leaf_addr_base, node_addr_base, rev, fanout,
                                         d_workspace or None, workspace_bytes, d_root, d_root_type, stream or None))


def build_id() -> str:
    """The loaded library's provenance, "sha256:<hex>" of the sources it was built from
    (storm_amd.build.sources_sha of a tree that matches it)."""
    return lib.stormck_build_id().decode()


def library_record() -> dict:
    """Which libstormck.so this process runs: its path, build id, and whether that id is
    the hash of the sources in this tree (a prebuilt library that travelled with them)."""
    from storm_amd import _lib, build
    bid = build_id()
    tree = "sha256:" + build.sources_sha()
    return {"path": os.path.relpath(_lib.LIB_PATH, build.ROOT), "build_id": bid, "tree_sources": tree,
            "matches_tree": bid == tree}


def init(device: int) -> None:
    check(lib.stormck_init(device))


def device_status(stream: int = 0) -> None:
    """Synchronise `stream`; raise if a ring kernel on the current device faulted
    (stormck_device_status: a stalled workgroup wrote no checksums)."""
    check(lib.stormck_device_status(stream or None))


def device_alloc(nbytes: int) -> int:
    """hipMalloc through the library (a block arena outside torch's caching allocator)."""
    import ctypes
    p = ctypes.c_void_p()
    check(lib.stormck_device_alloc(nbytes, ctypes.byref(p)))
    return int(p.value)


def device_alloc_placed(nbytes: int, mode: int, chunk_bytes: int = 0) -> Tuple[int, int]:
    """Probe build only (STORMCK_LIBRARY=tools/libstormck_probes.so): a block arena in
    placement `mode` (_lib.ALLOC_PLAIN / ALLOC_CONTIGUOUS), the modes measured and rejected
    in round 4; returns (device pointer, 0). The product library allocates with hipMalloc
    only (device_alloc). The VMM mode was deleted in round 6."""
    import ctypes
    if not hasattr(lib, "stormck_device_alloc_placed"):
        if mode == _lib.ALLOC_PLAIN:
            return device_alloc(nbytes), 0
        raise RuntimeError("arena placement modes are in the probe build only: "
                           "STORMCK_LIBRARY=tools/libstormck_probes.so")
    p, ch = ctypes.c_void_p(), ctypes.c_uint64(0)
    check(lib.stormck_device_alloc_placed(nbytes, mode, chunk_bytes, ctypes.byref(p), ctypes.byref(ch)))
    return int(p.value), int(ch.value)


def stream_forget(stream: int) -> None:
    """Release `stream`'s ring-fault slot before the stream is destroyed (raises if a
    fault was still pending there)."""
    check(lib.stormck_stream_forget(stream or None))


def device_free(d_ptr: int) -> None:
    check(lib.stormck_device_free(d_ptr or None))


def shutdown() -> None:
    lib.stormck_shutdown()


# ---------------------------------------------------------------------------
# torch helpers
# ---------------------------------------------------------------------------

def _torch():
    import torch  # local: the C-ABI itself does not need torch
    return torch


def _stream_of(t) -> int:
    torch = _torch()
    return torch.cuda.current_stream(t.device).cuda_stream


def checksum_tensor(blocks, length: Optional[int] = None, lens=None, out=None, check_status=None):
    """Checksums of a device tensor of blocks, shape [n, stride] uint8 (row i =
    block i; ``length`` bytes of each row, default the full row, or ``lens[i]``).
    Returns an int64 tensor [n] (bit pattern of the uint64 checksums). A batch that
    could take a ring kernel is followed by a status check of the stream unless
    ``check_status`` is False (checksum_device)."""
    torch = _torch()
    if blocks.dim() != 2 or blocks.dtype != torch.uint8 or not blocks.is_cuda:
        raise ValueError("blocks must be a 2-D uint8 CUDA tensor [n, stride]")
    if blocks.stride(1) != 1:
        raise ValueError("rows must be contiguous")
    n, width = blocks.shape
    stride = blocks.stride(0)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=blocks.device)
    d_lens = 0
    if lens is not None:
        if lens.dtype != torch.int32 or lens.device != blocks.device or lens.numel() != n:
            raise ValueError("lens must be an int32 tensor [n] on the blocks' device")
        longest = int(lens.max()) if n else 0
        if longest > width:
            raise ValueError("a length exceeds the row width")
        d_lens = lens.data_ptr()
        length = max(longest, 1)  # with lens: the longest, which the library plans the launch with
    elif length is None:
        length = width
    elif length > width:
        raise ValueError("length exceeds the row width")
    checksum_device(blocks.data_ptr(), stride, n, out.data_ptr(), length, d_lens, _stream_of(blocks),
                    check_status=check_status)
    return out


def merkle_root_tensor(leaf_cs, leaf_addr_base: int, node_addr_base: int, rev: int,
                       fanout: int = POINTERS_PER_BLOCK, workspace=None):
    """Shard Merkle root of device leaf checksums (int64 [n]) as an int64 tensor
    [4] = {Checksum, Address, BirthRevision, BlockType} on the same device."""
    torch = _torch()
    n = leaf_cs.numel()
    need = merkle_workspace_bytes(n, fanout)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(max(need // 8, 1), dtype=torch.int64, device=leaf_cs.device)
    root = torch.zeros(4, dtype=torch.int64, device=leaf_cs.device)
    merkle_root_device(leaf_cs.data_ptr() if n else 0, n, leaf_addr_base, node_addr_base, rev, fanout,
                       workspace.data_ptr(), workspace.numel() * 8, root.data_ptr(), root.data_ptr() + 24,
                       _stream_of(leaf_cs))
    return root


def combine_roots_tensor(roots, rev: int, root_addr: int, fanout: int = POINTERS_PER_BLOCK):
    """Global root from a table of shard roots (int64 [k, 4] rows {cs, addr, rev, type},
    shard order): one pointer block holding the k root Pointers, hashed on device.
    Returns int64 [4] {cs, root_addr, rev, Pointer}."""
    torch = _torch()
    k = roots.shape[0]
    if k == 0 or k > fanout:
        raise ValueError("need 1..fanout shard roots")
    entries = roots[:, :3].contiguous()
    types = roots[:, 3].to(torch.uint8).contiguous()
    out = torch.zeros(4, dtype=torch.int64, device=roots.device)
    pointer_node_device(entries.data_ptr(), types.data_ptr(), k, fanout, out.data_ptr(), _stream_of(roots))
    out[1] = root_addr
    out[2] = rev
    out[3] = 1  # BlockType Pointer
    return out


def u64(t) -> "object":
    """int64 tensor -> numpy uint64 (host)."""
    return t.detach().cpu().numpy().view("uint64")


def as_tuple(root) -> Tuple[int, int, int, int]:
    a = u64(root)
    return int(a[0]), int(a[1]), int(a[2]), int(a[3])
