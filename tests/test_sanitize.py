"""Sanitizer runs of libstormck's host code: ASan + UBSan and TSan builds
(tests/sanitize/build.sh: -fsanitize only after -Xarch_host, device code untouched)
driven by tests/sanitize/host_paths.cpp. On CPU the driver covers the single-call
host leg, argument validation and the threaded f1 commit planning up to the device
check; on the GPU box (-m gpu) the same executables also run commits to completion,
the host pipeline and the file read-verify reader threads against the oracle."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

SAN = os.path.join(ROOT, "tests", "sanitize")
SOURCES = [os.path.join(ROOT, "storm_amd", "csrc", f) for f in ("stormck.hip", "kernels.h", "multi_root.h", "xxh64_dev.h", "xxh64_host.h")]
SOURCES += [os.path.join(SAN, "host_paths.cpp"), os.path.join(SAN, "build.sh"), os.path.join(ROOT, "include", "stormck.h"),
            os.path.join(ROOT, "oracle", "xxh64_oracle.c")]
ENV = {"asan": {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:abort_on_error=0",
                "LSAN_OPTIONS": "suppressions=" + os.path.join(SAN, "lsan.supp"),
                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"},
       "tsan": {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1:suppressions="
                                + os.path.join(SAN, "tsan.supp")}}


def built(kind):
    exe = os.path.join(SAN, "build", f"host_paths_{kind}")
    if not os.path.exists(exe) or any(os.path.getmtime(s) > os.path.getmtime(exe) for s in SOURCES):
        subprocess.run(["bash", os.path.join(SAN, "build.sh"), kind], check=True, capture_output=True)
    return exe


def run(kind, timeout):
    env = dict(os.environ, **ENV[kind])
    r = subprocess.run([built(kind)], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0 and "ok: 0 failure(s)" in r.stdout, (r.stdout[-3000:], r.stderr[-6000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error:" not in r.stderr, r.stderr[-3000:]
    return r.stdout


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_under_sanitizers_cpu(kind):
    from storm_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("GPU present: the -m gpu variant runs the full driver")
    assert "device: no" in run(kind, 600)


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_under_sanitizers_gpu(kind):
    from storm_amd import _lib
    if _lib.device_count() == 0:
        pytest.skip("no GPU")
    exe = os.path.join(SAN, "build", f"host_paths_{kind}")
    if not os.path.exists(exe):
        pytest.skip("sanitizer build missing (bash tests/sanitize/build.sh asan|tsan in the build container)")
    assert "device: yes" in run(kind, 600)
