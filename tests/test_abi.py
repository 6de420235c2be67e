"""The C-ABI library loads and exports exactly what include/stormck.h declares (CPU).

On a machine without a gfx950 device every batched / device entry point must fail
loudly (STORMCK_ENODEV), never fall back to the CPU. The one host computation is the
single-call latency leg (stormck_xxh64 / stormck_checksum), checked here against the
oracle and the known answers.
"""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "stormck.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(stormck_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("stormck_checksum_device", "stormck_checksum_host", "stormck_verify_device",
                 "stormck_checksum", "stormck_merkle_root_device", "stormck_pointer_level_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from storm_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    # and the Python binding covers the whole header
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_abi_version():
    from storm_amd import _lib, ABI_VERSION
    assert _lib.lib.stormck_abi_version() == ABI_VERSION == 7


def test_library_build_id_is_the_tree_sources_hash():
    """stormck_build_id() carries the sha256 of the sources the library was compiled
    from (storm_amd/build.py), so a prebuilt libstormck.so can be matched to its tree:
    the in-tree build must match the sources next to it."""
    from storm_amd import engine
    rec = engine.library_record()
    assert rec["build_id"].startswith("sha256:") and len(rec["build_id"]) == 7 + 64
    assert rec["matches_tree"], rec


def test_pointer_struct_is_24_bytes():
    from storm_amd.blocks import Pointer
    assert ctypes.sizeof(Pointer) == 24
    assert [f[0] for f in Pointer._fields_] == ["Checksum", "Address", "BirthRevision"]


def test_workspace_bytes_is_host_logic():
    from storm_amd import engine
    assert engine.merkle_workspace_bytes(0) == 0
    assert engine.merkle_workspace_bytes(1) == 0
    assert engine.merkle_workspace_bytes(1200) == 8
    assert engine.merkle_workspace_bytes(1201) == 8 * (2 + 1)
    assert engine.merkle_workspace_bytes(16 << 20) == 8 * (13982 + 12 + 1)


def _has_gpu():
    from storm_amd import _lib
    return _lib.device_count() > 0


@pytest.mark.skipif("_has_gpu()")
def test_no_device_fails_loudly():
    from storm_amd import _lib, blocks, engine
    assert _lib.device_count() == 0
    with pytest.raises(_lib.NoDeviceError):
        blocks.ChecksumGPU(b"abc")
    with pytest.raises(_lib.NoDeviceError):
        blocks.ChecksumBatch(bytes(64), 2, 32, 32)
    with pytest.raises(_lib.NoDeviceError):
        blocks.VerifyChecksumBatch(bytes(64), 2, 32, [0, 0], 32)
    with pytest.raises(_lib.NoDeviceError):
        engine.checksum_device(1 << 20, 32, 1, 1 << 21, 32)
    with pytest.raises(_lib.NoDeviceError):
        blocks.ChecksumBatch(bytes(64), 2, 32, 32, devices=[0, 0])
    assert "no HIP device" in _lib.last_error() or "gfx950" in _lib.last_error()


def test_argument_errors_precede_the_device_check():
    """Bad arguments are rejected with STORMCK_EINVAL (and a message) before any device
    work, so these run identically with or without a GPU."""
    import numpy as np
    from storm_amd import _lib, commit as sc
    L = _lib.lib
    out = ctypes.c_uint64()
    cases = [
        ("null out", lambda: L.stormck_checksum(b"abc", 3, None)),
        ("null p", lambda: L.stormck_checksum(None, 3, ctypes.byref(out))),
        ("gpu null out", lambda: L.stormck_checksum_gpu(b"abc", 3, None)),
        ("gpu over 256 MiB", lambda: L.stormck_checksum_gpu(1 << 20, (256 << 20) + 1, ctypes.byref(out))),
        ("read-verify address overflow", lambda: L.stormck_read_verify_fd(
            0, (ctypes.c_uint64 * 1)(1 << 60), (ctypes.c_uint32 * 1)(100), 1, 32768, (ctypes.c_uint8 * 64)(), 64,
            (ctypes.c_uint64 * 1)(0), 0, ctypes.byref(out), ctypes.byref(out))),
        ("overlap", lambda: L.stormck_checksum_device(1 << 20, 16, None, 32, 2, 1 << 21, None)),
        ("null base", lambda: L.stormck_checksum_device(None, 32, None, 32, 2, 1 << 21, None)),
        ("gather null", lambda: L.stormck_checksum_gather_device(1 << 20, None, None, 32, 2, 1 << 21, None)),
        ("verify null result", lambda: L.stormck_verify_device(1 << 20, 32, None, 32, 2, 1 << 21, None, None)),
        ("fanout 0", lambda: L.stormck_pointer_level_device(1 << 20, 5, 0, 1, 2, 0, 1 << 21, None)),
        ("node count > fanout", lambda: L.stormck_pointer_node_device(1 << 20, 1 << 21, 11, 10, 1 << 22, None)),
        ("pack stride", lambda: L.stormck_pack_pointer_blocks_device(1 << 20, 5, 0, 1, 2, 10, 1 << 21, 200, None)),
        ("workspace", lambda: L.stormck_merkle_root_device(1 << 20, 5000, 0, 5000, 1, 10, 1 << 21, 8,
                                                           1 << 22, (1 << 22) + 24, None)),
        ("fill stride", lambda: L.stormck_fill_synthetic_device(1 << 20, 24, 4, 0, 1, None)),
        ("register empty", lambda: L.stormck_host_register(None, 0)),
        ("alloc null", lambda: L.stormck_device_alloc(16, None)),
        ("alloc 0 bytes", lambda: L.stormck_device_alloc(0, ctypes.byref(ctypes.c_void_p()))),
        ("split null base", lambda: L.stormck_checksum_split(None, 32, None, 32, 4, ctypes.addressof(out), None, 0,
                                                             0, 0, None)),
        ("split null out", lambda: L.stormck_checksum_split(1 << 20, 32, None, 32, 4, None, None, 0, 0, 0, None)),
        ("split overlap", lambda: L.stormck_checksum_split(1 << 20, 16, None, 32, 4, ctypes.addressof(out), None, 0,
                                                           0, 0, None)),
        ("verify split null result", lambda: L.stormck_verify_split(1 << 20, 32, None, 32, 4, ctypes.addressof(out),
                                                                    None, None, None, 0, 0, 0, None)),
        ("commit split null", lambda: L.stormck_commit_split(None, None, 3, 1, None, None, None, 0, 0, 0, None)),
        ("route rates null", lambda: L.stormck_route_get_rates(None)),
        ("route set flags", lambda: L.stormck_route_set_rates(None, 6)),
        ("route set zero rate", lambda: L.stormck_route_set_rates(ctypes.byref(_lib.RouteRates()), 0)),
        ("route devices null", lambda: L.stormck_route_devices(None, 2)),
        ("route devices count", lambda: L.stormck_route_devices((ctypes.c_int * 1)(0), -1)),
        ("plan leg null", lambda: L.stormck_route_plan_batch(32, None, 32, 4, 0, 0, 1, None, None)),
        ("plan memory kind", lambda: L.stormck_route_plan_batch(32, None, 32, 4, 5, 0, 1, ctypes.byref(
            ctypes.c_uint32()), None)),
        ("plan overlap", lambda: L.stormck_route_plan_batch(16, None, 32, 4, 0, 0, 1, ctypes.byref(ctypes.c_uint32()),
                                                            None)),
        ("plan commit null", lambda: L.stormck_route_plan_commit(None, 3, 1, 0, 1, ctypes.byref(ctypes.c_uint32()),
                                                                 None)),
        ("routed commit null", lambda: L.stormck_commit(None, None, 3, 1, None, None, None, 0, None)),
        ("host leg null", lambda: L.stormck_commit_host(None, None, 3, 1, None, None, 1)),
        ("device pointer null", lambda: L.stormck_host_device_pointer(None, None)),
        ("key tags null", lambda: L.stormck_key_tags_device(None, 48, None, None, 48, 10, 1 << 20, None)),
        ("host null base", lambda: L.stormck_checksum_host(None, 32, None, 32, 4, ctypes.addressof(out))),
        ("multi no devices", lambda: L.stormck_checksum_host_multi(1 << 20, 32, None, 32, 4, ctypes.addressof(out),
                                                                   None, 0)),
        ("multi null out", lambda: L.stormck_checksum_host_multi(1 << 20, 32, None, 32, 4, None,
                                                                 (ctypes.c_int * 1)(0), 1)),
        ("verify multi null", lambda: L.stormck_verify_host_multi(1 << 20, 32, None, 32, 4, None, None, None,
                                                                  (ctypes.c_int * 1)(0), 1)),
        ("batch null base", lambda: L.stormck_checksum_batch(None, 32, None, 32, 4, ctypes.addressof(out), 0, None)),
        ("batch null out", lambda: L.stormck_checksum_batch(1 << 20, 32, None, 32, 4, None, 0, None)),
        ("batch overlap", lambda: L.stormck_checksum_batch(1 << 20, 16, None, 32, 4, ctypes.addressof(out), 0, None)),
        ("verify batch null result", lambda: L.stormck_verify_batch(1 << 20, 32, None, 32, 4, ctypes.addressof(out),
                                                                    None, None, 0, None)),
        ("verify batch null expected", lambda: L.stormck_verify_batch(1 << 20, 32, None, 32, 4, None,
                                                                      ctypes.byref(out), ctypes.byref(out), 0, None)),
        ("host-leg batch null out", lambda: L.stormck_checksum_host_leg(1 << 20, 32, None, 32, 4, None, 1)),
        ("host-leg batch overlap", lambda: L.stormck_checksum_host_leg(1 << 20, 16, None, 32, 4,
                                                                       ctypes.addressof(out), 1)),
        ("host-leg unreadable base", lambda: L.stormck_checksum_host_leg(1 << 20, 64, None, 64, 4,
                                                                         ctypes.addressof(out), 1)),
        ("host-leg verify null result", lambda: L.stormck_verify_host_leg(1 << 20, 32, None, 32, 4,
                                                                          ctypes.addressof(out), None, None, 1)),
        ("read-verify slot", lambda: L.stormck_read_verify_fd(0, (ctypes.c_uint64 * 1)(0), (ctypes.c_uint32 * 1)(100),
                                                              1, 32768, (ctypes.c_uint8 * 64)(), 64,
                                                              (ctypes.c_uint64 * 1)(0), 1, ctypes.byref(out),
                                                              ctypes.byref(out))),
    ]
    for name, fn in cases:
        assert fn() == _lib.EINVAL, name
        assert _lib.last_error(), name
    # f1 planning errors: parent out of range, misaligned origin, cycles
    b, size, last = sc.pointer_forest(25, 100, 10, slot=1024, revision=1)
    la = ctypes.c_uint64(last)
    cs = np.zeros(len(b), dtype=np.uint64)

    def commit(bb):
        return L.stormck_commit_device(1 << 20, bb.ctypes.data, len(bb), 1, ctypes.byref(la), cs.ctypes.data, None)
    bad = b.copy()
    bad["parent"][3] = 10 ** 6
    assert commit(bad) == _lib.EINVAL and "parent" in _lib.last_error()
    bad = b.copy()
    bad["origin_pointer"][3] += 4
    assert commit(bad) == _lib.EINVAL and "aligned" in _lib.last_error()
    bad = b.copy()
    bad["parent"][28] = 0  # root -> leaf 0 -> ... -> root
    assert commit(bad) == _lib.EINVAL and "cycle" in _lib.last_error()
    assert (b["address"] == np.arange(1, len(b) + 1)).all()  # rejected calls left the records untouched


@pytest.mark.skipif("_has_gpu()")
def test_commit_planning_runs_then_fails_loudly_without_device():
    """The host planning passes (pool threads: heights, histograms, counting sort) run on
    a 200K-record shuffled forest, then the call stops at the device check with
    STORMCK_ENODEV and the caller's records are untouched (no relocation applied)."""
    import numpy as np
    from storm_amd import _lib, commit as sc
    b, size, last = sc.pointer_forest(200_000, 1024, 10, slot=1024, revision=5)
    rng = np.random.default_rng(1)
    perm = rng.permutation(len(b))
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(b))
    bp = b[perm].copy()
    has = bp["parent"] >= 0
    bp["parent"][has] = inv[bp["parent"][has]]
    bp["birth_revision"][::3] = 5  # a third would relocate
    before = bp.copy()
    la = ctypes.c_uint64(last)
    cs = np.zeros(len(bp), dtype=np.uint64)
    rc = _lib.lib.stormck_commit_device(1 << 20, bp.ctypes.data, len(bp), 5, ctypes.byref(la), cs.ctypes.data, None)
    assert rc == _lib.ENODEV
    assert np.array_equal(bp, before) and la.value == last


def test_single_call_host_leg_matches_oracle_and_known_answers():
    """stormck_xxh64 / stormck_checksum (the single-call leg, no device needed): the
    public XXH64 answers, every fixture length on zero and iota data, and random buffers
    of every length 0..300 at every start offset mod 8, against the C oracle."""
    import numpy as np
    from oracle import oracle as o
    from storm_amd import _lib, blocks
    from tests.conftest import hx, load_golden
    kat = load_golden("kat.json")
    for s_, v in kat["public"].items():
        assert blocks.Checksum(s_.encode()) == hx(v)
        assert _lib.lib.stormck_xxh64(s_.encode(), len(s_)) == hx(v)
    for r in kat["rows"]:
        n = r["len"]
        assert blocks.Checksum(bytes(n)) == hx(r["zeros"]), n
        assert blocks.Checksum(bytes(i & 0xFF for i in range(n))) == hx(r["iota"]), n
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, size=400, dtype=np.uint8)
    for n in range(0, 301):
        for off in range(8):
            sl = buf[off:off + n]
            assert blocks.Checksum(sl) == o.xxh64(sl), (n, off)
    big = rng.integers(0, 256, size=(300 << 20) + 13, dtype=np.uint8)  # past the 256 MiB device limit
    assert blocks.Checksum(big) == o.xxh64(big)
    assert _lib.lib.stormck_xxh64(None, 0) == 0xEF46DB3751D8E999
