"""The shipped library carries one dispatch; the measured-and-rejected variants and
their environment knobs live only in the probe build (CPU checks).

include/stormck.h documents the operational knobs the product reads:
STORMCK_READ_THREADS, STORMCK_READ_SUPER_BYTES, STORMCK_TRACE and the STORMCK_DEBUG_*
test hooks. Every other STORMCK_* variable (STORMCK_WIDE16, STORMCK_MID_WAVES, ...)
selects a kernel variant DESIGN.md measured and rejected, and is compiled in only with
-DSTORMCK_PROBES (tools/libstormck_probes.so, storm_amd/build.py build_probes_lib)."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

OPERATIONAL = {"STORMCK_READ_THREADS", "STORMCK_READ_SUPER_BYTES", "STORMCK_TRACE", "STORMCK_DEBUG_STALL_CHUNK",
               "STORMCK_DEBUG_STALL_STREAM", "STORMCK_DEBUG_READER_LIMIT"}
PROBE_KNOBS = {"STORMCK_STAGE_PIPE", "STORMCK_WIDE16", "STORMCK_WIDE_MULTI", "STORMCK_GLDS_VAR", "STORMCK_VAR_LO",
               "STORMCK_MID_WAVES", "STORMCK_BIG_W", "STORMCK_QUAD_SPREAD", "STORMCK_GATHER_ORDER",
               "STORMCK_COMMIT_WIDE", "STORMCK_COMMIT_MULTI", "STORMCK_COMMIT_MIDW", "STORMCK_COMMIT_CHUNKS",
               "STORMCK_POINTER_RING", "STORMCK_POINTER_C", "STORMCK_POINTER_SIMD", "STORMCK_SINGLE_GPU_MIN",
               "STORMCK_GATHER_RANK", "STORMCK_GATHER_CONTIG"}


def _env_strings(path):
    data = open(path, "rb").read()
    return set(m.decode() for m in re.findall(rb"STORMCK_[A-Z0-9_]+", data))


def _product():
    from storm_amd import build as sb
    return sb.LIB


def test_product_library_reads_only_operational_knobs():
    names = _env_strings(_product())
    env_like = {n for n in names if n in OPERATIONAL | PROBE_KNOBS}
    assert env_like == OPERATIONAL, sorted(env_like ^ OPERATIONAL)
    assert not (names & PROBE_KNOBS)


def test_probe_build_has_the_knobs_and_the_same_abi():
    from storm_amd import build as sb
    from tests.test_abi import declared_functions
    if not os.path.exists(sb.PROBES_LIB):
        pytest.fail("probe build missing: python -c 'import __graft_entry__ as g; g.build()'")
    names = _env_strings(sb.PROBES_LIB)
    assert PROBE_KNOBS <= names, sorted(PROBE_KNOBS - names)
    lib = ctypes.CDLL(sb.PROBES_LIB)
    for fn in declared_functions():
        assert hasattr(lib, fn), fn
    lib.stormck_build_id.restype = ctypes.c_char_p
    assert lib.stormck_build_id().decode() == "sha256:" + sb.sources_sha() + "+probes"


def test_probe_build_is_the_larger_one():
    """The rejected variants are template instances the product no longer carries."""
    from storm_amd import build as sb
    assert os.path.getsize(sb.PROBES_LIB) > os.path.getsize(_product())


def test_product_library_has_one_allocation_mode():
    """The arena placement modes (contiguous allocations; VMM reservations until round 6) were
    measured no better than hipMalloc in round 4 and live in the probe build only: the product
    neither exports stormck_device_alloc_placed nor imports the HIP VMM API, and the probe
    build no longer carries the VMM mode, which twice read wrong blocks."""
    import ctypes
    from storm_amd import build as sb
    lib = ctypes.CDLL(_product())
    assert not hasattr(lib, "stormck_device_alloc_placed")
    data = open(_product(), "rb").read()
    for sym in (b"hipMemCreate", b"hipMemAddressReserve", b"hipMemMap", b"hipExtMallocWithFlags"):
        assert sym not in data, sym
    probes = open(sb.PROBES_LIB, "rb").read()
    assert b"stormck_device_alloc_placed" in probes and b"hipExtMallocWithFlags" in probes
    for sym in (b"hipMemCreate", b"hipMemAddressReserve", b"hipMemMap"):
        assert sym not in probes, sym
