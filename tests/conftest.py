import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running (full-size configs)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


def hx(s: str) -> int:
    return int(s, 16)


def pytest_sessionfinish(session, exitstatus):
    """STORMCK_CHECK_PARTIAL_QUADS=1 with STORMCK_LIBRARY = the debug build
    (tools/libstormck_debug.so): fail the run if any quad merge ran with part of its quad
    inactive (kernels.h quad_bcast), i.e. a merge that would have read zeros."""
    if os.environ.get("STORMCK_CHECK_PARTIAL_QUADS") != "1":
        return
    import ctypes
    from storm_amd import _lib
    fn = getattr(_lib.lib, "stormck_debug_partial_quads", None)
    if fn is None:
        print("\nSTORMCK_CHECK_PARTIAL_QUADS: the loaded library is not the debug build")
        session.exitstatus = 1
        return
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    c = ctypes.c_uint64(0)
    rc = fn(ctypes.byref(c), 0)
    print(f"\npartial quad merges in this run: {c.value} (rc {rc})")
    if rc != 0 or c.value != 0:
        session.exitstatus = 1
