"""ctypes binding of libstormck (include/stormck.h).

Loads the in-tree build ``storm_amd/lib/libstormck.so``. There is no fallback:
if the library is missing, importing this module raises; if no gfx950 device is
present, every batched / device compute call raises :class:`NoDeviceError`
(single calls hash on the host by design: include/stormck.h).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_uint8, c_uint32, c_uint64, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libstormck.so")
# STORMCK_LIBRARY=<path>: load another build of the same ABI instead, e.g. the probe build
# tools/libstormck_probes.so (storm_amd/build.py), whose design knobs the product lacks
LIB_PATH = os.environ.get("STORMCK_LIBRARY") or LIB_PATH

OK = 0
EINVAL = -1
EHIP = -2
ENODEV = -3
ENOMEM = -4
EMISMATCH = -5

# arena placement modes of stormck_device_alloc_placed: the probe build only (measured and
# rejected in round 4; the product allocates with hipMalloc, stormck_device_alloc)
ALLOC_PLAIN = 0
ALLOC_CONTIGUOUS = 2  # (mode 1, a VMM reservation, was deleted in round 6)
# STORMCK_LEG_* (stormck_commit, stormck_checksum_batch, the route plan)
LEG_NONE, LEG_HOST, LEG_DEVICE, LEG_SPLIT = 0, 1, 2, 3
LEG_NAMES = {LEG_NONE: "none", LEG_HOST: "host", LEG_DEVICE: "device", LEG_SPLIT: "split"}
MEM_PAGEABLE, MEM_PINNED = 0, 1  # STORMCK_MEM_*
RATES_LEARN, RATES_FREEZE = 0, 1  # STORMCK_RATES_*
SPLIT_BALANCED = (1 << 64) - 1    # STORMCK_SPLIT_BALANCED


class StormckError(RuntimeError):
    """A libstormck call failed (code < 0)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"stormck error {code}: {msg}")
        self.code = code


class NoDeviceError(StormckError):
    pass


class RouteRates(ctypes.Structure):
    """stormck_route_rates: the routing model's rates (bytes per microsecond) and the
    devices' start latency in a split (microseconds)."""

    _fields_ = [("host_thread", ctypes.c_double), ("host_memory", ctypes.c_double), ("host_cached", ctypes.c_double),
                ("link_pinned", ctypes.c_double), ("link_pageable", ctypes.c_double),
                ("link_inplace", ctypes.c_double), ("device_latency", ctypes.c_double),
                ("observations", c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class PointerStruct(ctypes.Structure):
    """stormck_pointer == blocks.Pointer (/root/reference/blocks/types.go:35-39)."""

    _fields_ = [("Checksum", c_uint64), ("Address", c_uint64), ("BirthRevision", c_uint64)]


class ShardStruct(ctypes.Structure):
    """stormck_shard: one device-resident shard of stormck_merkle_root_multi."""

    _fields_ = [("d_blocks", c_void_p), ("stride", c_uint64), ("n", c_uint64), ("d_checksums", c_void_p),
                ("leaf_addr_base", c_uint64), ("node_addr_base", c_uint64), ("stream", c_void_p),
                ("device", ctypes.c_int32), ("len", c_uint32)]


# name -> (restype, argtypes); mirrors include/stormck.h one to one.
SIGNATURES = {
    "stormck_abi_version": (c_int, []),
    "stormck_build_id": (c_char_p, []),
    "stormck_last_error": (c_char_p, []),
    "stormck_device_count": (c_int, [POINTER(c_int)]),
    "stormck_init": (c_int, [c_int]),
    "stormck_shutdown": (None, []),
    "stormck_device_status": (c_int, [c_void_p]),
    "stormck_device_alloc": (c_int, [c_uint64, POINTER(c_void_p)]),
    "stormck_stream_forget": (c_int, [c_void_p]),
    "stormck_device_free": (c_int, [c_void_p]),
    "stormck_checksum_device": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p]),
    "stormck_checksum_gather_device": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p]),
    "stormck_verify_device": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p]),
    "stormck_checksum_host": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p]),
    "stormck_verify_host": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p]),
    "stormck_checksum_host_multi": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_int]),
    "stormck_verify_host_multi": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "stormck_checksum_batch": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_uint32, POINTER(c_uint32)]),
    "stormck_verify_batch": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p, c_uint32,
                POINTER(c_uint32)]),
    "stormck_checksum_host_leg": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_uint32]),
    "stormck_verify_host_leg": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p, c_uint32]),
    "stormck_xxh64": (c_uint64, [c_void_p, c_uint64]),
    "stormck_checksum": (c_int, [c_void_p, c_uint64, POINTER(c_uint64)]),
    "stormck_checksum_gpu": (c_int, [c_void_p, c_uint64, POINTER(c_uint64)]),
    "stormck_host_register": (c_int, [c_void_p, c_uint64]),
    "stormck_host_unregister": (c_int, [c_void_p]),
    "stormck_host_device_pointer": (c_int, [c_void_p, c_void_p]),
    "stormck_pointer_level_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint8, c_uint32, c_void_p, c_void_p]),
    "stormck_pointer_node_device": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_void_p, c_void_p]),
    "stormck_pack_pointer_blocks_device": (
        c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint8, c_uint32, c_void_p, c_uint64, c_void_p]),
    "stormck_merkle_workspace_bytes": (c_uint64, [c_uint64, c_uint32]),
    "stormck_merkle_root_device": (
        c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "stormck_shard_plan": (c_int, [c_uint64, c_uint32, c_void_p, c_int, POINTER(ShardStruct), POINTER(c_uint64)]),
    "stormck_merkle_root_multi": (
        c_int, [POINTER(ShardStruct), c_uint32, c_uint64, c_uint64, c_uint32, POINTER(PointerStruct),
                POINTER(c_uint8), POINTER(PointerStruct), POINTER(c_uint8)]),
    "stormck_multi_layout": (
        c_int, [POINTER(ShardStruct), c_uint32, c_void_p, POINTER(c_uint32), POINTER(c_uint32), c_void_p]),
    "stormck_read_verify_fd": (
        c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_uint64, c_void_p, c_uint32, c_void_p, c_void_p]),
    "stormck_key_tags_device": (c_int, [c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p]),
    "stormck_commit_device": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, POINTER(c_uint64), c_void_p, c_void_p]),
    "stormck_commit_host": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, POINTER(c_uint64), c_void_p, c_uint32]),
    "stormck_commit": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint64, POINTER(c_uint64), c_void_p, c_void_p, c_uint32, POINTER(c_uint32)]),
    "stormck_route_get_rates": (c_int, [POINTER(RouteRates)]),
    "stormck_route_set_rates": (c_int, [POINTER(RouteRates), c_uint32]),
    "stormck_route_devices": (c_int, [c_void_p, c_int]),
    "stormck_route_plan_batch": (
        c_int, [c_uint64, c_void_p, c_uint32, c_uint64, c_uint32, c_uint32, c_uint32, POINTER(c_uint32), c_void_p]),
    "stormck_route_plan_commit": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, POINTER(c_uint32), c_void_p]),
    "stormck_checksum_split": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_int, c_uint32, c_uint64,
                POINTER(c_uint64)]),
    "stormck_verify_split": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                c_uint32, c_uint64, POINTER(c_uint64)]),
    "stormck_commit_split": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint64, POINTER(c_uint64), c_void_p, c_void_p, c_int, c_uint32,
                c_uint64, POINTER(c_uint64)]),
    "stormck_fill_synthetic_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_void_p]),
}

# Exported by the probe build only (storm_amd/build.py build_probes_lib), bound when present.
PROBE_SIGNATURES = {
    "stormck_device_alloc_placed": (c_int, [c_uint64, c_uint32, c_uint64, POINTER(c_void_p), POINTER(c_uint64)]),
}


def _load() -> ctypes.CDLL:
    # One HIP runtime per process: torch's libtorch_hip NEEDs the unversioned
    # "libamdhip64.so", so if libstormck (NEEDED "libamdhip64.so.7") were loaded first,
    # torch would map a second copy of the runtime and the two would contend for the
    # device. Loading torch first lets libstormck bind to torch's runtime by soname.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libstormck not built ({LIB_PATH} missing): run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in PROBE_SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.stormck_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> None:
    """Raise on a negative libstormck status."""
    if rc == OK:
        return
    if rc == ENODEV:
        raise NoDeviceError(rc, last_error())
    raise StormckError(rc, last_error())


def device_count() -> int:
    c = c_int(0)
    check(lib.stormck_device_count(ctypes.byref(c)))
    return c.value
