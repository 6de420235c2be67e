"""N > 1 on the GPU: bench.py's shard path (device fill, checksums, shard Merkle tree,
root all-gather, device combine) in two ranks that share cuda:0 over gloo. Every
rank's global root must equal the oracle's. RCCL itself runs in
`bench.py --force-dist` (world size 1); the 8-GPU run is the driver's."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

N_TOTAL, STRIDE, FANOUT, REV = 20011, 1024, 10, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from oracle import oracle as o
    from storm_amd import dist as sdist
    from storm_amd import engine

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        lo, hi = sdist.shard_range(N_TOTAL, world, rank)
        arena = torch.empty((hi - lo, STRIDE), dtype=torch.uint8, device=dev)
        engine.fill_synthetic_device(arena.data_ptr(), STRIDE, hi - lo, lo, o.SYNTH_SEED,
                                     torch.cuda.current_stream(dev).cuda_stream)
        cs = engine.checksum_tensor(arena)
        root = engine.merkle_root_tensor(cs, lo, sdist.shard_node_addr_base(N_TOTAL, lo), REV, FANOUT)
        groot, table = sdist.global_root(root, REV, N_TOTAL,
                                         lambda t, r, a: engine.combine_roots_tensor(t, r, a, FANOUT))
        torch.cuda.synchronize()
        q.put((rank, engine.as_tuple(groot), [tuple(int(v) for v in row) for row in engine.u64(table)]))
    except Exception as e:  # report, then fail the process
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_global_root():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    from oracle import oracle as o
    from storm_amd import dist as sdist

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    host = o.fill_synthetic(N_TOTAL, STRIDE, 0)
    leaf = o.checksum_batch(host, N_TOTAL, STRIDE, STRIDE, threads=8)
    table = [o.merkle_root(leaf[lo:hi], lo, sdist.shard_node_addr_base(N_TOTAL, lo), REV, FANOUT)
             for lo, hi in sdist.plan(N_TOTAL, 2)]
    want = o.combine_roots(table, REV, sdist.global_root_addr(N_TOTAL), FANOUT)
    for rank, groot, tab in res:
        assert tab == [tuple(r) for r in table], (rank, groot)
        assert tuple(groot) == tuple(want), rank
