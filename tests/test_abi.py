"""The C-ABI library loads and exports exactly what include/stormck.h declares (CPU).

No compute happens here: on a machine without a gfx950 device every compute
entry point must fail loudly (STORMCK_ENODEV), never fall back to the CPU.
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
    assert _lib.lib.stormck_abi_version() == ABI_VERSION == 1


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
        blocks.Checksum(b"abc")
    with pytest.raises(_lib.NoDeviceError):
        blocks.ChecksumBatch(bytes(64), 2, 32, 32)
    with pytest.raises(_lib.NoDeviceError):
        engine.checksum_device(1 << 20, 32, 1, 1 << 21, 32)
    assert "no HIP device" in _lib.last_error() or "gfx950" in _lib.last_error()
