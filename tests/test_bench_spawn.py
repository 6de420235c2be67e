"""bench.py --gpus N without a launcher: the parent spawns the N rank processes itself
(before touching any GPU), each with the environment torch.distributed.run would give
it. Rehearsed on CPU with gloo: every rank computes its c4-style shard root (the
oracle as the per-shard hasher), the roots are all-gathered and combined, and every
rank must hold the same global root as the libxxhash combine fixture."""
import json
import os
import time

import numpy as np
import pytest

import bench
from storm_amd import dist as sdist
from tests.conftest import hx, load_golden


def _rank_worker():
    """Spawned by bench.spawn_ranks as "tests.test_bench_spawn:_rank_worker"."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as o

    a = bench.parse()  # argv handed over by the parent
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    assert a.gpus == world and os.environ["MASTER_ADDR"] == "127.0.0.1"
    assert int(os.environ["LOCAL_RANK"]) == rank
    dist.init_process_group("gloo")
    try:
        g = load_golden("merkle.json")["combine"]
        n_total, rev, fanout = g["n_total"], g["rev"], g["fanout"]
        leaf = o.synth_leaf_checksums(n_total)
        lo, hi = sdist.shard_range(n_total, world, rank)
        r = o.merkle_root(leaf[lo:hi], lo, sdist.shard_node_addr_base(n_total, lo), rev, fanout)
        local = torch.tensor(np.array(r, dtype=np.uint64).view(np.int64))

        def combine(table, rev_, addr):
            rows = [tuple(int(v) for v in row) for row in table.numpy().view(np.uint64)]
            return o.combine_roots(rows, rev_, addr, fanout)

        t0 = time.perf_counter()
        groot, _ = sdist.global_root(local, rev, n_total, combine)
        # the N > 1 line's rank summary and scaling fields, through bench.py's own helpers
        # (per-rank stats all-gathered over gloo here, RCCL on GPUs); the "kernel" times are
        # this rank's shard-root time
        el = time.perf_counter() - t0 + 1e-3 * (rank + 1)
        rows = bench.gather_rank_rows(el, el + 1e-3, [el * 1e3, el * 5e2], rank, hi - lo, "cpu")
        line = None
        if rank == 0:
            elapsed, wall, ranks = bench.summarize_ranks(rows, 1)
            value = n_total * bench.BLOCK / elapsed / 2**30
            line = {"value": value, "ranks": ranks, **bench.scaling_reference(world, n_total, ranks, value, "strong")}
        with open(os.path.join(os.environ["SPAWN_TEST_OUT"], f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "world": world, "root": [int(v) for v in groot], "line": line}, f)
    finally:
        dist.destroy_process_group()


def _failing_worker():
    """Rank 1 fails before the collective; rank 0 would wait in it for ever."""
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    if int(os.environ["RANK"]) == 1:
        os._exit(7)
    out = [torch.zeros(1) for _ in range(int(os.environ["WORLD_SIZE"]))]
    dist.all_gather(out, torch.zeros(1))


@pytest.mark.timeout(240)
def test_spawned_ranks_agree_on_the_combine_fixture(tmp_path, monkeypatch):
    world = load_golden("merkle.json")["combine"]["world"]  # 8 shard roots
    monkeypatch.setenv("SPAWN_TEST_OUT", str(tmp_path))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    rc = bench.spawn_ranks(world, ["bench.py", "--gpus", str(world)], entry="tests.test_bench_spawn:_rank_worker",
                           timeout=200)
    assert rc == 0
    g = load_golden("merkle.json")["combine"]
    want = [hx(v) for v in g["global_root"][:3]] + [g["global_root"][3]]
    for r in range(world):
        with open(tmp_path / f"rank{r}.json") as f:
            got = json.load(f)
        assert got["world"] == world and got["root"] == want
        if r == 0:
            line = got["line"]
    # the N > 1 line says which N = 1 number it reads against (verdict r05 item 3)
    n_total = g["n_total"]
    per = line["ranks"]["per_rank"]
    assert [p["rank"] for p in per] == list(range(world))
    assert sum(p["blocks"] for p in per) == n_total
    slow = per[line["ranks"]["slowest_rank"]]
    assert slow["ms_per_step"] == max(p["ms_per_step"] for p in per)
    assert line["per_gpu_GiB_s"] == round(line["value"] / world, 2)
    ref = line["scaling_reference"]
    assert "per_gpu_GiB_s" in ref["read_against"] and "c3" in ref["driver_n1_line"]
    assert ref["strong_scaling_n1_ms_per_step_estimate"] == round(slow["ms_per_step"] / slow["blocks"] * n_total, 3)


@pytest.mark.timeout(120)
def test_a_failing_rank_ends_the_job_with_its_exit_code():
    t0 = time.time()
    rc = bench.spawn_ranks(2, ["bench.py", "--gpus", "2"], entry="tests.test_bench_spawn:_failing_worker", timeout=90)
    assert rc == 7
    assert time.time() - t0 < 60


def test_parent_does_not_touch_the_gpu_before_spawning():
    """main() must reach spawn_ranks before any torch.cuda call: a process that has
    initialised the GPU may not be the parent of the rank processes on the GPU box."""
    import inspect
    src = inspect.getsource(bench.main)
    assert src.index("spawn_ranks") < min(i for i in (src.find("torch"), len(src)) if i >= 0)
    assert "cuda" not in inspect.getsource(bench.spawn_ranks)


def test_root_fixture_names_the_workloads():
    path = os.path.join(bench.ROOT, "tests", "golden", "c3c4_roots.json")
    if not os.path.exists(path):
        pytest.skip("c3c4_roots.json not generated")
    want, name = bench.root_fixture(bench.C3_BLOCKS, 1, False)
    assert name == "c3" and want[1] >= bench.C3_BLOCKS and want[2] == 1 and want[3] == 1
    for world in (2, 4, 8):
        want, name = bench.root_fixture(bench.C4_BLOCKS, world, True)
        assert name == f"c4 world {world}"
        assert want[1] == sdist.global_root_addr(bench.C4_BLOCKS) and want[3] == 1
    assert bench.root_fixture(12345, 1, False) == (None, None)


@pytest.mark.parametrize("n", [2, 8, 12, 13])
def test_e2e_leg_orders_are_balanced(n):
    """The E2E workloads' leg orders (bench.balanced_orders): every leg once per order,
    and each leg right after every other leg equally often (a leg's time depends on what
    ran before it: DESIGN.md §4.2)."""
    from collections import Counter
    names = [f"leg{i}" for i in range(n)]
    orders = bench.balanced_orders(names)
    assert len(orders) == (n if n % 2 == 0 else 2 * n)
    assert all(sorted(o) == sorted(names) for o in orders)
    pairs = Counter((o[i - 1], o[i]) for o in orders for i in range(1, n))
    assert len(pairs) == n * (n - 1) and len(set(pairs.values())) == 1
