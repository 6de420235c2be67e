"""bench.py's multi-rank path on the GPU, as the driver's N > 1 runs take it, at a size
the oracle checks in seconds:

* RCCL: `bench.py --force-dist` at world size 1 under the environment torch.distributed.run
  gives a rank (RANK / WORLD_SIZE / MASTER_*): nccl process group, the shard's passes
  through a small arena (the last one partial), the shard Merkle tree, the RCCL
  all-gather of the root and the device combine.
* Self-spawn: `bench.py --gpus 2` with no launcher; the parent starts both ranks, which
  share cuda:0 and gather over gloo (RCCL will not put two ranks on one GPU).

Each printed global root must equal the oracle's for the same workload (fill seed,
shard ranges, node addresses: storm_amd/dist.py; node format
blocks/pointer/block.go:10-13). The 8-GPU RCCL run itself is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

from oracle import oracle as o
from storm_amd import dist as sdist

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCK, FANOUT, REV = 32768, 1200, 1
N_TOTAL = 40001   # 3 arena passes per rank at world 1 (16384, 16384, 7233); odd split at world 2
ARENA = 16384


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _want(world):
    host = o.fill_synthetic(N_TOTAL, BLOCK, 0)
    leaf = o.checksum_batch(host, N_TOTAL, BLOCK, BLOCK, threads=8)
    table = [o.merkle_root(leaf[lo:hi], lo, sdist.shard_node_addr_base(N_TOTAL, lo), REV, FANOUT)
             for lo, hi in sdist.plan(N_TOTAL, world)]
    return tuple(int(v) for v in o.combine_roots(table, REV, sdist.global_root_addr(N_TOTAL), FANOUT))


def _run_bench(args, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--total-blocks", str(N_TOTAL), "--arena", str(ARENA),
           "--steps", "2", "--warmup", "1", "--settle", "0", "--no-cpu"] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 alone prints the line
    return json.loads(lines[0])


def _root(res):
    rp = res["root_pointer"]
    return tuple(int(v, 16) for v in rp[:3]) + (int(rp[3]),)


@pytest.mark.timeout(300)
def test_bench_rccl_world1_root_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_bench(["--force-dist", "--dist-backend", "nccl"],
                     {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                      "MASTER_PORT": str(_free_port())})
    assert "RCCL all-gather" in res["config"]["workload"]
    assert res["config"]["passes_per_step"] == 3 and res["n_gpus"] == 1
    _check_group(res, 1, "nccl")
    assert _root(res) == _want(1)


def _check_group(res, world, backend):
    """The N > 1 line shows the process group that formed and every rank's timing."""
    g = res["config"]["process_group"]
    assert g["world_size"] == world and g["backend"] == backend and g["device_count"] >= 1
    per = res["ranks"]["per_rank"]
    assert [r["rank"] for r in per] == list(range(world))
    assert 0 <= res["ranks"]["slowest_rank"] < world
    for r in per:
        assert 0 < r["kernel_min_ms"] <= r["kernel_avg_ms"] <= r["kernel_max_ms"]
    slow = per[res["ranks"]["slowest_rank"]]
    assert slow["ms_per_step"] == max(r["ms_per_step"] for r in per) == res["ms_per_step"]
    arena = res["config"]["arena"]
    assert int(arena["va"], 16) % arena["va_alignment"] == 0 and arena["va_alignment"] >= 4096


@pytest.mark.timeout(300)
def test_bench_self_spawned_two_ranks_root_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_bench(["--gpus", "2", "--dist-backend", "gloo"], {})
    assert res["n_gpus"] == 2 and res["config"]["total_blocks"] == N_TOTAL
    assert res["config"]["blocks_per_gpu"] == sdist.shard_range(N_TOTAL, 2, 0)[1]
    _check_group(res, 2, "gloo")
    assert _root(res) == _want(2)
