"""Build libstormck.so (gfx950) in-tree, and the test-only oracle library.

    python -m storm_amd.build            # product library
    python -m storm_amd.build --all      # + oracle/liboracle.so (tests / CPU baseline)

The built .so files are git-ignored and travel to the GPU box with the snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "storm_amd")
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libstormck.so")
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _newer(target: str, sources) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


# the sources libstormck.so is compiled from (its build id hashes them)
SOURCES = [os.path.join(CSRC, f) for f in ("stormck.hip", "kernels.h", "multi_root.h", "xxh64_dev.h", "xxh64_host.h")] + \
    [os.path.join(ROOT, "include", "stormck.h")]


def sources_sha() -> str:
    """sha256 over SOURCES (path relative to the repo, then content): the build id a
    library built from this tree carries (stormck_build_id)."""
    import hashlib
    h = hashlib.sha256()
    for path in SOURCES:
        h.update(os.path.relpath(path, ROOT).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _compile_lib(out: str, extra, sha: str) -> None:
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           f'-DSTORMCK_SRC_SHA="{sha}"', *extra, "-o", tmp, os.path.join(CSRC, "stormck.hip")]
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)


def build_lib(force: bool = False) -> str:
    if not force and _newer(LIB, SOURCES):
        return LIB
    _compile_lib(LIB, [], sources_sha())
    return LIB


# The probe build: the same sources with -DSTORMCK_PROBES, i.e. with the variants measured
# and rejected in DESIGN.md and the environment knobs that select them (stormck.hip
# STORMCK_KNOB). Design tools and tests/test_probe_build.py load it; the product does not.
PROBES_LIB = os.path.join(ROOT, "tools", "libstormck_probes.so")


# The debug build: the product dispatch with every quad merge checked for a partially
# active quad (kernels.h quad_bcast, -DSTORMCK_DEBUG_QUAD); tests/test_quad_debug.py runs
# the kernel families through it.
DEBUG_LIB = os.path.join(ROOT, "tools", "libstormck_debug.so")


def build_debug_lib(force: bool = False) -> str:
    if not force and _newer(DEBUG_LIB, SOURCES):
        return DEBUG_LIB
    _compile_lib(DEBUG_LIB, ["-DSTORMCK_DEBUG_QUAD"], sources_sha() + "+debug-quad")
    return DEBUG_LIB


def build_probes_lib(force: bool = False) -> str:
    if not force and _newer(PROBES_LIB, SOURCES):
        return PROBES_LIB
    _compile_lib(PROBES_LIB, ["-DSTORMCK_PROBES"], sources_sha() + "+probes")
    return PROBES_LIB


def build_oracle(force: bool = False) -> str:
    out = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "xxh64_oracle.c")
    if force or not _newer(out, [src]):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return out


CALLTIMER = os.path.join(ROOT, "tools", "libcalltimer.so")  # bench.py's C timing loop for us-scale calls


def build_calltimer(force: bool = False) -> str:
    """tools/libcalltimer.so: storm-sized calls timed in a C loop (tools/calltimer.cpp;
    measurement only, links the product library)."""
    src = os.path.join(ROOT, "tools", "calltimer.cpp")
    if force or not _newer(CALLTIMER, [src, LIB]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), src,
                        "-L", LIB_DIR, "-lstormck", "-Wl,-rpath,$ORIGIN/../storm_amd/lib", "-o", CALLTIMER],
                       check=True)
    return CALLTIMER


PROBES = ("probe", "probe_keys", "probe_small", "alloc_probe", "phase_probe", "span_probe", "clock_probe")  # tools/<name>.hip: design probes
SANITIZE = os.path.join(ROOT, "tests", "sanitize")
READPEAK = os.path.join(ROOT, "tools", "libreadpeak.so")  # bench.py's measured read peak (not product)


def build_readpeak(force: bool = False) -> str:
    """tools/libreadpeak.so: the shipped kernel's data movement without the hash, which
    bench.py times on its own arena (measurement only)."""
    srcs = [os.path.join(ROOT, "tools", "readpeak.hip"), os.path.join(CSRC, "kernels.h"),
            os.path.join(CSRC, "xxh64_dev.h")]
    if force or not _newer(READPEAK, srcs):
        subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", READPEAK,
                        srcs[0]], check=True)
    return READPEAK


def build_probe(force: bool = False) -> str:
    """Build the design probes (tools/probe*.hip) next to their sources."""
    built = []
    for name in PROBES:
        out = os.path.join(ROOT, "tools", name)
        srcs = [os.path.join(ROOT, "tools", name + ".hip"), os.path.join(CSRC, "kernels.h"),
                os.path.join(CSRC, "xxh64_dev.h")]
        if force or not _newer(out, srcs):
            subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-o", out, srcs[0]], check=True)
        built.append(out)
    # tools/single_call_probe.cpp: host leg vs device single call, in C (links the library)
    out = os.path.join(ROOT, "tools", "single_call_probe")
    src = os.path.join(ROOT, "tools", "single_call_probe.cpp")
    if force or not _newer(out, [src, LIB]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-L", LIB_DIR,
                        "-lstormck", "-Wl,-rpath,$ORIGIN/../storm_amd/lib", "-o", out], check=True)
    built.append(out)
    # tools/route_overhead.cpp: the routed calls' fixed cost in C (links the library)
    out = os.path.join(ROOT, "tools", "route_overhead")
    src = os.path.join(ROOT, "tools", "route_overhead.cpp")
    if force or not _newer(out, [src, LIB]):
        subprocess.run([hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-L", LIB_DIR,
                        "-lstormck", "-Wl,-rpath,$ORIGIN/../storm_amd/lib", "-pthread", "-o", out], check=True)
    built.append(out)
    return " ".join(built)


def build_sanitizers() -> str:
    """tests/sanitize/build/host_paths_{asan,tsan}: the host code under ASan+UBSan and
    TSan (tests/sanitize/build.sh; device code unchanged, no GPU sanitizer)."""
    for kind in ("asan", "tsan"):
        subprocess.run(["bash", os.path.join(SANITIZE, "build.sh"), kind], check=True, capture_output=True)
    return os.path.join(SANITIZE, "build")


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_lib(force))
    if "--all" in sys.argv:
        print(build_oracle(force))
        print(build_readpeak(force))
        print(build_probe(force))
