"""N > 1 path on CPU with gloo: shard planning, the root all-gather, and the
combined global root (oracle as the per-shard hasher; on GPUs the same code runs
with RCCL and the device kernels — bench.py)."""
import os
import socket

import numpy as np
import pytest

from storm_amd import dist as sdist
from tests.conftest import hx, load_golden


def test_shard_ranges_partition():
    for n in (0, 1, 7, 1000, 16 << 20):
        for world in (1, 2, 3, 4, 8):
            ranges = sdist.plan(n, world)
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def _nodes(n, f):
    t, m = 0, n
    while m > 1:
        m = (m + f - 1) // f
        t += m
    return t


@pytest.mark.parametrize("fanout", [3, 10, 1200])
def test_node_address_ranges_disjoint(fanout):
    for n_total in (2, 17, 12345, 1_000_003):
        for world in (1, 2, 8):
            spans = []
            for lo, hi in sdist.plan(n_total, world):
                if hi - lo == 0:
                    continue
                base = sdist.shard_node_addr_base(n_total, lo)
                spans.append((base, base + _nodes(hi - lo, fanout)))
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b <= c
            assert all(a >= n_total for a, _ in spans)
            assert all(b <= sdist.global_root_addr(n_total) for _, b in spans)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, fanout, rev, q):
    import torch
    import torch.distributed as dist
    from oracle import oracle as o

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        leaf = o.synth_leaf_checksums(n_total)
        lo, hi = sdist.shard_range(n_total, world, rank)
        r = o.merkle_root(leaf[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), rev, fanout)
        local = torch.tensor(np.array(r, dtype=np.uint64).view(np.int64))

        def combine(table, rev_, addr):
            rows = [tuple(int(v) for v in row) for row in table.numpy().view(np.uint64)]
            return o.combine_roots(rows, rev_, addr, fanout)

        groot, table = sdist.global_root(local, rev, n_total, combine)
        q.put((rank, groot, [tuple(int(v) for v in row) for row in table.numpy().view(np.uint64)]))
    finally:
        dist.destroy_process_group()


def _run(world, n_total, fanout, rev):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, fanout, rev, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


def test_gloo_world2_global_root_matches_direct():
    from oracle import oracle as o
    n_total, fanout, rev = 30011, 10, 4
    res = _run(2, n_total, fanout, rev)
    leaf = o.synth_leaf_checksums(n_total)
    table = []
    for lo, hi in sdist.plan(n_total, 2):
        table.append(o.merkle_root(leaf[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), rev, fanout))
    want = o.combine_roots(table, rev, sdist.global_root_addr(n_total), fanout)
    for rank, groot, tab in res:
        assert tab == table           # rank order preserved by the all-gather
        assert groot == want          # identical global root on every rank


def test_gloo_world8_matches_fixture():
    g = load_golden("merkle.json")["combine"]
    res = _run(g["world"], g["n_total"], g["fanout"], g["rev"])
    want = [hx(v) for v in g["global_root"][:3]] + [g["global_root"][3]]
    for rank, groot, tab in res:
        assert list(groot) == want
        assert [list(t[:3]) for t in tab] == [[hx(v) for v in row[:3]] for row in g["shard_roots"]]


def _settle_worker(rank, world, port, q):
    import time

    import torch
    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        count = [0]

        def step():  # like bench.py's c3 step: local work of rank-dependent length, then a collective
            time.sleep(0.01 * (1 + 4 * rank))
            t = torch.zeros(1)
            out = [torch.zeros(1) for _ in range(world)]
            dist.all_gather(out, t)
            count[0] += 1

        time.sleep(0.25 * rank)  # uneven setup before the loop, as arena fills and inits are
        bench.settle(step, 0.3, torch.device("cpu"))
        dist.barrier()  # a rank left inside a collective would never reach this
        q.put((rank, count[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(150)
def test_bench_settle_runs_the_same_step_count_on_every_rank():
    """bench.py's clock-settle loop holds a collective per step: a count taken from each
    rank's own clock deadlocks the faster rank in a collective the slower one never
    enters. The ranks must agree on the count."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_settle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=60) for _ in range(2))
    finally:
        for p in procs:
            if p.is_alive():
                p.join(timeout=5)
            if p.is_alive():
                p.kill()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and res[0] >= 1
