"""C++ host mirror of the Go `blocks` API (include/storm_blocks.hpp) over the C-ABI.

CPU: the mirror compiles against include/stormck.h and links libstormck.so (the
static_asserts pin the Go struct sizes). GPU: the C++ port of the reference's
blocks tests runs and its values match the libxxhash fixtures.
"""
import json
import os
import subprocess

import pytest

from tests.conftest import ROOT, hx, load_golden

SRC = os.path.join(ROOT, "tests", "cpp", "blocks_test.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "build", "blocks_test")


def build():
    from storm_amd import build as b
    b.build_lib()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    libdir = os.path.dirname(b.LIB)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", OUT, "-L", libdir, "-lstormck", f"-Wl,-rpath,{libdir}"], check=True)
    return OUT


def test_cpp_mirror_compiles_and_links():
    assert os.path.exists(build())


@pytest.mark.gpu
def test_cpp_mirror_runs_reference_tests():
    exe = build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    g = load_golden("layouts.json")
    assert got["failures"] == 0
    assert [hx(v) for v in got["pointer_block_test_sequence"]] == [hx(v) for v in g["pointer_block_test_sequence"]]
    assert hx(got["blob_test_block"]) == hx(g["blob_test_block"]["checksum"])
    assert hx(got["singularity"]) == hx(g["singularity_example"]["checksum"])
    for tag, names in got["zero"].items():
        for name, v in names.items():
            assert hx(v) == hx(g["zero_block_checksums"][tag][name]), (tag, name)
    # the one-process multi-GPU root (PlanShards / MerkleRootDevices) against the oracle
    import numpy as np
    from oracle import oracle as o
    from storm_amd import dist as sdist
    n_total, stride, world = 20000, 4096, 4
    cs = o.checksum_batch(o.fill_synthetic(n_total, stride, 0), n_total, stride, stride, threads=8)
    rows = [o.merkle_root(cs[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), 1)
            for lo, hi in sdist.plan(n_total, world)]
    assert [[hx(r[0]), r[1], r[2]] for r in got["multi"]["shard_roots"]] == [[r[0], r[1], r[3]] for r in rows]
    assert hx(got["multi"]["root"]) == o.combine_roots(rows, 1, sdist.global_root_addr(n_total))[0]
