"""Benchmark: device-resident block checksums on MI355X (BASELINE.json metric).

One step = checksum every block of the per-GPU workload (XXH64 seed 0 =
storm's blocks.Checksum, /root/reference/blocks/checksum.go:15-17), build the
shard's Merkle pointer tree over the checksums, and (N > 1) all-gather the shard
roots over RCCL and hash the combining pointer block.

Workloads:
  N = 1: BASELINE.json configs[2] (c3) — 16M x 32 KiB blocks (512 GiB).
  N > 1: BASELINE.json configs[3] (c4) — 64M blocks over the N GPUs in contiguous
         shards (strong scaling; 8M per GPU at N = 8), RCCL all-gather of the
         shard roots.
A shard exceeds one MI355X's 288 GB of HBM, so its blocks stream through a
resident 2M-block (64 GiB) arena; before each pass the on-device generator
writes that pass's own logical blocks. The regeneration has its
own HIP events and is taken out of the step time, so `value` covers the hash
launches, the Merkle tree and the gather. Every block hashed is distinct, and the
printed root is checked against the libxxhash fixture of the same workload
(tests/golden/c3c4_roots.json): a mismatch exits non-zero.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)
    python bench.py --gpus N ...   (no launcher: bench.py spawns the N ranks itself)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident block checksum; % of MI355X HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (chip-level parameters)
BLOCK = 32768          # blocks.BlockSize, /root/reference/blocks/types.go:4
FANOUT = 1200          # pointer.PointersPerBlock, /root/reference/blocks/pointer/params.go:6
REV = 1
C3_BLOCKS = 16 << 20  # BASELINE.json configs[2]
C4_BLOCKS = 64 << 20  # BASELINE.json configs[3]
SYNTH_SEED = 0x53544F524D  # synthetic block generator seed ("STORM")
# --alloc: (placement mode, physical chunk bytes); modes other than plain need the probe
# build (STORMCK_LIBRARY=tools/libstormck_probes.so: stormck_device_alloc_placed)
ALLOC_MODES = {"plain": (0, 0), "contig": (2, 0)}
KERNEL = "k_xxh64_glds_skew<16,nt,8w,4KiB>"  # dominant kernel (storm_amd/csrc/kernels.h), as named in profiles/traffic.json


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=0,
                   help="blocks per GPU per step (weak scaling); default: c3 (16M) at N = 1, c4 (64M total) at N > 1")
    p.add_argument("--total-blocks", type=int, default=0, help="blocks over all GPUs per step (strong scaling)")
    # 2M blocks (64 GiB, 8 passes for c3): 0.868-0.896 of peak over 24 fresh processes,
    # median 0.893; a 4M-block (128 GiB) arena ran 0.838-0.902, median 0.876, by where it
    # landed in HBM
    p.add_argument("--arena", type=int, default=2 << 20, help="resident arena (blocks)")
    p.add_argument("--alloc", default="plain", choices=sorted(ALLOC_MODES),
                   help="arena placement: plain = hipMalloc (stormck_device_alloc); with the probe build "
                        "(STORMCK_LIBRARY=tools/libstormck_probes.so) also contig = hipDeviceMallocContiguous")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (rank 0, N=1)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--settle", type=float, default=1.0,
                   help="before the W warmup steps, run untimed steps for at least this many seconds so the "
                        "GPU clocks settle (short workloads otherwise time a ramping clock)")
    p.add_argument("--c5-mix", default="keystore", choices=["keystore", "storm"],
                   help="c5 batch: BenchmarkKeyStore's commit (objectlist leaves) or BenchmarkStorm's (blob leaves "
                        "and a spacelist block)")
    p.add_argument("--gather-blocks", type=int, default=4 << 20, help="gather workload: blocks per step")
    p.add_argument("--gather-order", default="shuffled", choices=["shuffled", "sequential", "strided"],
                   help="gather workload: slot order (storm's cache slots are spread by addressingOffsets); "
                        "strided = no offsets, the blocks at base + i * 32 KiB with per-block lengths "
                        "(stormck_checksum_device with lens: the same kernel without the gather, A/B)")
    p.add_argument("--gather-lens", type=int, default=0, help="gather workload: one length for every block (A/B)")
    p.add_argument("--gather-slot", type=int, default=BLOCK, help="gather workload: slot bytes (a multiple of 16)")
    p.add_argument("--gather-lens-set", default="",
                   help="gather workload: comma-separated lengths drawn per block instead of storm's leaf sizes "
                        "(e.g. 256,536,728: the `-tags test` sizes, storm_test.go:131-138)")
    p.add_argument("--workload", default="c3", choices=["c3", "commit", "keytags", "c5", "gather", "commit_e2e", "batch_e2e"],
                   help="c3 = BASELINE metric (default); commit = f1 level-synchronous Cache.Commit of a dirty "
                        "forest; keytags = f4 xxhash.Sum64 of 48-byte keys")
    p.add_argument("--commit-leaves", type=int, default=1 << 20)
    p.add_argument("--keys", type=int, default=64 << 20, help="f4: keys per step (a multiple of 1024)")
    p.add_argument("--force-dist", action="store_true",
                   help="take the multi-rank path (process group, root all-gather, combine) even at N=1")
    p.add_argument("--in-process", action="store_true",
                   help="c3 / c4 on --gpus N devices from ONE process (storm's case: one Go process), through the "
                        "C-ABI: per-device arena passes, then stormck_merkle_root_multi (shard trees, in-process "
                        "RCCL all-gather of the shard roots, combine on every device)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL (production); gloo only to rehearse N>1 with ranks sharing a GPU")
    return p.parse_args()


def settle(step, seconds: float, group_dev=None):
    """Untimed steps until `seconds` of wall time have passed (GPU clock ramp).

    With a process group (`group_dev` = the tensor device for it) every rank runs the
    same number of steps: a step holds a collective (the root all-gather), so a count
    taken from each rank's own clock would leave one rank waiting in a collective the
    others never enter. The ranks continue while any of them is still short of
    `seconds` (MAX all-reduce of a flag)."""
    import torch
    t0 = time.perf_counter()
    while True:
        more = time.perf_counter() - t0 < seconds
        if group_dev is not None:
            import torch.distributed as dist
            f = torch.tensor([1 if more else 0], dtype=torch.int32, device=group_dev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            more = bool(f.item())
        if not more:
            return
        step()
        if torch.cuda.is_available():  # (the CPU gloo test of this loop has no device)
            torch.cuda.synchronize()


def va_alignment(ptr: int) -> int:
    """Largest power of two (up to 2^40) that divides a virtual address."""
    return min(ptr & -ptr, 1 << 40) if ptr else 0


def measured_read_peak(arena_ptr: int, arena_n: int, stream, achieved: float):
    """The shipped kernel's data movement with the hash replaced by xor
    (tools/libreadpeak.so), 3 launches on the bench's own arena, timed with HIP events
    on the launch stream. None if the measurement library is not built."""
    import ctypes
    import torch
    from storm_amd import build as sb

    if not os.path.exists(sb.READPEAK):
        return None
    lib = ctypes.CDLL(sb.READPEAK)
    fn = lib.readpeak_xor_skew
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.empty(arena_n, dtype=torch.int64, device=stream.device)
    ms = []
    for r in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if fn(arena_ptr, BLOCK, BLOCK, arena_n, sink.data_ptr(), stream.cuda_stream) != 0:
            return None
        e1.record(stream)
        torch.cuda.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
    gbs = arena_n * (BLOCK + 8) / (sum(ms) / len(ms) * 1e-3) / 1e9
    return {"GB/s": round(gbs, 1), "frac": round(achieved / gbs, 4),
            "kernel": KERNEL + " data movement with the hash replaced by xor "
                      "(tools/readpeak.hip), 3 launches on the same arena after the timed region"}


def cpu_baseline(seconds: float):
    """Oracle C restatement (port of XXH64 = xxhash.Sum64) on the host, 1 thread,
    over a bounded sample of the same synthetic 32 KiB blocks. Also timed on all
    threads of this process's CPU share (reported as an extra field)."""
    import numpy as np
    from oracle import oracle as o

    n = 32768  # 1 GiB sample (larger than the host LLC), the GPU arena's first blocks
    buf = o.fill_synthetic(n, BLOCK, 0)
    out = o.checksum_batch(buf, n, BLOCK, BLOCK)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        out = o.checksum_batch(buf, n, BLOCK, BLOCK)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds * 0.75:
            break
    one = reps * n * BLOCK / el / 2**30
    host = host_cpu_info()
    threads = host["usable_cpus"]  # every CPU this process may use (affinity, cgroup quota)
    reps_mt, t0 = 0, time.perf_counter()
    while True:
        o.checksum_batch(buf, n, BLOCK, BLOCK, threads=threads)
        reps_mt += 1
        el_mt = time.perf_counter() - t0
        if el_mt >= seconds * 0.25:
            break
    multi = reps_mt * n * BLOCK / el_mt / 2**30
    assert int(out[0]) == int(o.checksum_batch(buf[:BLOCK], 1, BLOCK, BLOCK)[0])
    # the library's own host leg (stormck_checksum_host_leg: four blocks per thread with
    # AVX-512, the leg routed host-memory batches take), the same sample on the same threads
    from storm_amd import blocks
    got = blocks.ChecksumBatchHost(buf, n, BLOCK, BLOCK, threads=threads)
    assert np.array_equal(got, out)
    reps_h, t0 = 0, time.perf_counter()
    while True:
        blocks.ChecksumBatchHost(buf, n, BLOCK, BLOCK, threads=threads)
        reps_h += 1
        el_h = time.perf_counter() - t0
        if el_h >= max(1.0, seconds * 0.1):
            break
    leg = reps_h * n * BLOCK / el_h / 2**30
    return {"value": round(one, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{n} x 32 KiB synthetic blocks (1 GiB) hashed {reps}x in {el:.1f} s by oracle/xxh64_oracle.c "
                      f"(-O3, 1 thread); Go reference unbuildable here (no Go toolchain)",
            "all_threads": {"value": round(multi, 3), "threads": threads},
            "library_host_leg": {"value": round(leg, 3), "threads": threads,
                                 "what": "stormck_checksum_host_leg (AVX-512, 4 blocks per thread) on the same sample"},
            "host": host}


def cpu_commit_baseline(seconds: float):
    """storm's serial commit loop (oracle_commit: relocation, XXH64 per block, origin
    writes, cache/cache.go:87-137) on the host, 1 thread, over a bounded forest of the
    same shape as the GPU run (32 KiB leaves, fan-out 1200)."""
    import numpy as np
    from oracle import oracle as o
    from storm_amd import commit as sc

    n = 16384  # 512 MiB of leaves
    b0, size, last = sc.pointer_forest(n, BLOCK, FANOUT, slot=BLOCK, revision=REV)
    arena = np.zeros(size, dtype=np.uint8)
    arena[BLOCK:BLOCK + n * BLOCK] = o.fill_synthetic(n, BLOCK, 0)
    reps, t0 = 0, time.perf_counter()
    while True:
        b = b0.copy()
        o.commit(arena, b, REV, last)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(reps * n * BLOCK / el / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"commit of {n} x 32 KiB dirty leaves + {len(b0) - n} pointer blocks, {reps}x in {el:.1f} s, "
                      f"oracle/xxh64_oracle.c oracle_commit (serial Cache.Commit loop, 1 thread)"}


def golden(name: str):
    """A committed libxxhash fixture (tests/golden/, oracle/gen_golden.py), or None."""
    path = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def check_against(got: int, want_hex, what: str):
    """(root_check text, exit code) for a printed result against its fixture value."""
    if want_hex is None:
        return "no fixture for this workload", 0
    if got == int(want_hex, 16):
        return f"match ({what})", 0
    return f"MISMATCH vs {what} {want_hex}", 3


def commit_workload(a):
    """f1: one step = commit of a dirty forest of `commit_leaves` 32 KiB leaves under
    fan-out-1200 pointer blocks held in HBM (level-synchronous, stormck_commit_device:
    children-first planning + relocation on the host, one fused hash+scatter launch per
    level; the kernels read the dirty records from pinned host memory and write the
    checksums back there, all inside the timed call)."""
    import numpy as np
    import torch
    from storm_amd import commit as sc
    from storm_amd import engine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = a.commit_leaves
    b0, size, last = sc.pointer_forest(n, BLOCK, FANOUT, slot=BLOCK, revision=REV)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + BLOCK, BLOCK, n, 0, 0x53544F524D)
    torch.cuda.synchronize()
    # every block is new in this revision (birth = REV + 1), so commit relocates nothing
    # and the metadata array is reusable across steps unchanged
    # (the checksum array is reused across commits, as storm's metadata would be)
    out = np.zeros(len(b0), dtype=np.uint64)
    settle(lambda: sc.commit_device(arena.data_ptr(), b0, REV, last, out=out), a.settle)
    for _ in range(a.warmup):
        sc.commit_device(arena.data_ptr(), b0, REV, last, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        cs, _ = sc.commit_device(arena.data_ptr(), b0, REV, last, out=out)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    blocks_bytes = int(b0["length"].sum())
    value = blocks_bytes * a.steps / el / 2**30
    res = {"metric": "GiB/s level-synchronous commit (f1) of a dirty block forest", "value": round(value, 2),
           "unit": "GiB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"f1 commit: {n} dirty 32 KiB leaves + {len(b0) - n} pointer blocks (fan-out 1200), "
                                  "rooted at the singularity", "dirty_blocks": int(len(b0)),
                      "hashed_bytes": blocks_bytes},
           "roofline": {"bound": "hbm", "achieved": round(blocks_bytes / (el / a.steps) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(blocks_bytes / (el / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None, "kernel": "k_commit_level_glds<16,nt,8w> (whole call: host planning, record and checksum transfers included)"},
           "root": "0x%016x" % int(cs[-1])}
    fx = golden("c3c4_roots.json")
    want = fx["f1_commit_1m"]["root"][0] if fx and "f1_commit_1m" in fx and n == fx["f1_commit_1m"]["leaves"] else None
    res["root_check"], rc = check_against(int(cs[-1]), want, "f1_commit_1m, tests/golden/c3c4_roots.json")
    if not a.no_cpu:
        res["cpu_baseline"] = cpu_commit_baseline(a.cpu_seconds)
    print(json.dumps(res), flush=True)
    return rc


def c5_workload(a):
    """c5: the mixed batch of one storm commit in keystore/benchmark_test.go (SURVEY §8a
    a6: ~1200 objectlist leaves of 31808 B + 1 pointer block of 30000 B + the 72 B
    singularity), device-resident. One step = the batch checksum (per-block lengths)
    AND the same batch committed as a forest through stormck_commit_device (host
    planning, 2 level launches reading the records from pinned host memory, checksums
    back to the caller). Latency-bound by nature: one
    32 KiB block is ~1000 serial XXH64 rounds per accumulator."""
    import numpy as np
    import torch
    from storm_amd import commit as sc
    from storm_amd import engine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_ol = 1200
    storm_mix = a.c5_mix == "storm"
    leaf_len = 32768 if storm_mix else 31808  # blob leaves (BenchmarkStorm) or objectlist leaves (BenchmarkKeyStore)
    lens = np.array([leaf_len] * n_ol + ([28808] if storm_mix else []) + [30000, 72], dtype=np.uint32)
    n = len(lens)
    buf = torch.empty((n, BLOCK), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), BLOCK, n, 0, 0x53544F524D)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    # the commit form: 1200 objectlist leaves under one pointer block (fan-out 1200), rooted at the singularity
    b0, size, last = sc.pointer_forest(n_ol, leaf_len, FANOUT, slot=BLOCK, revision=REV)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + BLOCK, BLOCK, n_ol, 0, 0x53544F524D)

    def batch():  # ring-fault status checked once per series below, not per launch
        engine.checksum_device(buf.data_ptr(), BLOCK, n, out.data_ptr(), 0, d_lens.data_ptr(), st, check_status=False)

    settle(batch, a.settle)
    for _ in range(a.warmup):
        batch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        batch()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    engine.device_status(st)  # raises if a ring launch of the series stalled
    cs = np.zeros(len(b0), dtype=np.uint64)
    settle(lambda: sc.commit_device(arena.data_ptr(), b0, REV, last, out=cs), a.settle)
    tc = time.perf_counter()
    for _ in range(a.steps):
        sc.commit_device(arena.data_ptr(), b0, REV, last, out=cs)
    commit_us = (time.perf_counter() - tc) / a.steps * 1e6
    hashed = int(lens.sum())
    res = {"metric": "GiB/s mixed storm commit batch (c5), device-resident", "value": round(hashed * a.steps / el / 2**30, 2),
           "unit": "GiB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(el / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": ("c5 (storm mix): 1200 x 32768 B blob + 1 x 28808 B spacelist + 1 x 30000 B pointer "
                                   "+ 1 x 72 B singularity (benchmark_test.go BenchmarkStorm commit), per-block lengths"
                                   if storm_mix else
                                   "c5: 1200 x 31808 B objectlist + 1 x 30000 B pointer + 1 x 72 B singularity "
                                   "(keystore/benchmark_test.go commit), per-block lengths"), "blocks": n,
                      "hashed_bytes": hashed},
           "batch_us": round(el / a.steps * 1e6, 1),
           "commit_forest_us": round(commit_us, 1),
           "commit_root": "0x%016x" % int(cs[-1])}
    # the batch's checksums and the commit root against tests/golden/c5.json; the digest
    # is XXH64 of the checksum array, taken with the library's single-call host leg
    from storm_amd import blocks
    fx = golden("c5.json")
    if fx and storm_mix:
        fx = fx.get("storm")
    digest = blocks.Checksum(out.cpu().numpy().view(np.uint64).astype("<u8"))
    c1, rc1 = check_against(digest, fx and fx["batch_digest"], "c5 batch digest, tests/golden/c5.json")
    c2, rc2 = check_against(int(cs[-1]), fx and fx["commit_root"], "c5 commit root, tests/golden/c5.json")
    res["root_check"] = f"batch: {c1}; commit: {c2}"
    rc = rc1 or rc2
    if not a.no_cpu:
        from oracle import oracle as o
        host = buf.cpu().numpy()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(a.cpu_seconds, 5.0):
            o.checksum_batch(host, n, BLOCK, 0, lens=lens)
            reps += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(reps * hashed / el / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": f"the same {n}-block batch hashed {reps}x in {el:.1f} s by oracle/xxh64_oracle.c",
                               "batch_us": round(el / reps * 1e6, 1)}
    print(json.dumps(res), flush=True)
    return rc


def calltimer():
    """tools/libcalltimer.so (storm_amd/build.py build_calltimer): the E2E tables time calls
    of under 1 MiB in a C loop, so a leg's column is what the call costs and not what
    Python's ctypes adds per argument (cgo, storm's binding, costs the same per call
    whatever the argument count). None if not built (then Python's loop is used)."""
    import ctypes
    from storm_amd import build as sb
    if not os.path.exists(sb.CALLTIMER):
        return None
    lib = ctypes.CDLL(sb.CALLTIMER)
    P, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.calltimer_commit.restype = ctypes.c_double
    lib.calltimer_commit.argtypes = [I, P, P, U64, U64, U64, P, U32, I, P, P, P, P]
    lib.calltimer_batch.restype = ctypes.c_double
    lib.calltimer_batch.argtypes = [I, P, U64, P, U32, U64, P, U32, I, P, P, P]
    return lib


def balanced_orders(names):
    """Orders of the legs in which each leg follows every other leg equally often (a Williams
    design: len(names) orders for an even count, twice that for an odd one, each leg once
    per order)."""
    n = len(names)
    first, lo, hi = [0], 1, n - 1
    while len(first) < n:
        first.append(lo)
        lo += 1
        if len(first) < n:
            first.append(hi)
            hi -= 1
    rows = [[(x + i) % n for x in first] for i in range(n)]
    if n % 2:
        rows += [list(reversed(r)) for r in rows]
    return [[names[k] for k in r] for r in rows]


def commit_e2e_workload(a):
    """f1 end to end from host memory, in the Go binding's configuration: storm's
    cache.data as page-aligned registered host memory (integration/go/cache/
    commit_stormck.go newArena), each dirty forest committed by
      dev_inplace  stormck_commit_device on the arena in place (the kernels read the
                   blocks and write the parents' Pointers over PCIe),
      host_1       stormck_commit_host on 1 thread (storm's serial loop: one XXH64 per
                   block, children first),
      host_all     stormck_commit_host on every usable thread,
      split        stormck_commit_split, balanced: the leaves on the pool (from the front)
                   and the device in place (from the back) at once, upper heights on the
                   host (split_dev_share = the leaves the device hashed / all leaves),
      split_1      the same with one host thread,
      routed       stormck_commit (the library's choice of the three),
      routed_1     the same with one host thread allowed (host cores kept for storm),
    and, for reference, dev_hbm: the same forest with cache.data in HBM (device-resident,
    the north-star configuration). Forests: storm's c5 commits (BenchmarkKeyStore's
    1,200 objectlist leaves, BenchmarkStorm's 1,200 blob leaves, each under one pointer
    block, keystore/benchmark_test.go:58-62, benchmark_test.go), the smallest real
    commit (2 leaves + their pointer block), a `-tags test` forest (100 leaves of 536 /
    728 B under fan-out-10 pointer blocks of 256 B, storm_test.go:131-138), and larger
    forests of 16K and 128K leaves. Every leg's checksums must agree. One line per run
    with a table: median us per commit, every leg once per round in balanced orders (each
    leg follows every other equally often; a whole cycle of orders for forests of at most
    64 MiB, --steps rounds up to 1 GiB, 3 above), calls under 1 MiB as the mean of 200."""
    import ctypes
    import numpy as np
    import torch
    from storm_amd import _lib, blocks
    from storm_amd import commit as sc
    from storm_amd import engine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    engine.init(0)
    L = _lib.lib
    shapes = [
        ("c5_keystore", 1200, 31808, FANOUT),
        ("c5_storm", 1200, 32768, FANOUT),
        ("three_blocks", 2, 31808, FANOUT),
        ("test_tag", 100, np.array([536, 728] * 50, dtype=np.uint32), 10),
        ("leaves_16k", 16384, 32768, FANOUT),
        ("leaves_128k", 131072, 32768, FANOUT),
    ]
    threads = host_cpu_info()["usable_cpus"]
    reps = max(3, a.steps)
    rows = []
    ct = calltimer()
    for name, nl, lens, fan in shapes:
        b0, size, last = sc.pointer_forest(nl, lens, fan, slot=BLOCK, revision=REV)
        pages = (size + 4095) // 4096 * 4096
        raw = np.zeros(pages + 4096, dtype=np.uint8)
        off = (-raw.ctypes.data) % 4096
        arena = raw[off:off + pages]
        arena[BLOCK:BLOCK + nl * BLOCK] = engine_fill_host(nl, BLOCK)
        _lib.check(L.stormck_host_register(arena.ctypes.data, arena.nbytes))
        d_host = ctypes.c_void_p()
        _lib.check(L.stormck_host_device_pointer(arena.ctypes.data, ctypes.byref(d_host)))
        hbm = torch.from_numpy(arena).to(dev)
        torch.cuda.synchronize()
        bytes_hashed = int(b0["length"].sum())
        outs = {}

        # calls of a few microseconds are timed as the mean of `inner` back-to-back calls on
        # the same records (relocation happens in the first; the hashing and the stores repeat
        # in every one); the pointers are taken outside the clock
        inner = 200 if bytes_hashed < (1 << 20) else 1
        arena_p = arena.ctypes.data

        def run(leg):
            b = b0.copy()
            out = np.zeros(len(b), dtype=np.uint64)
            la = ctypes.c_uint64(last)
            bp, op, nb = b.ctypes.data, out.ctypes.data, len(b)
            done, used = ctypes.c_uint64(0), ctypes.c_uint32(9)
            if inner > 1 and ct is not None:  # a few microseconds: the C loop
                code = {"dev_inplace": 0, "dev_hbm": 0, "host_1": 1, "host_all": 1, "split": 2, "split_1": 2}.get(leg, 3)
                ap = d_host.value if leg == "dev_inplace" else (hbm.data_ptr() if leg == "dev_hbm" else arena_p)
                nt = threads if leg == "host_all" else (1 if leg.endswith("_1") else 0)
                rc_ = ctypes.c_int(0)
                dt = ct.calltimer_commit(code, ap, bp, nb, REV, last, op, nt, inner, ctypes.byref(rc_),
                                         ctypes.byref(used), ctypes.byref(done), ctypes.byref(la)) * 1e-6
                _lib.check(rc_.value)
                if leg in ("split", "split_1"):
                    shares.setdefault(leg, []).append(done.value / nl)
                elif leg.startswith("routed"):
                    outs[leg + "_leg"] = int(used.value)
                return dt, out
            # every pointer argument is converted outside the clock, so the Python columns
            # differ by the calls' own costs (and ctypes' per-argument cost), not by byref()s
            pla, pdone, pused = ctypes.byref(la), ctypes.byref(done), ctypes.byref(used)
            if leg in ("dev_inplace", "dev_hbm"):
                ap = d_host.value if leg == "dev_inplace" else hbm.data_ptr()

                def f():
                    return L.stormck_commit_device(ap, bp, nb, REV, pla, op, None)
            elif leg in ("host_1", "host_all"):
                nt = 1 if leg == "host_1" else threads

                def f():
                    return L.stormck_commit_host(arena_p, bp, nb, REV, pla, op, nt)
            elif leg in ("split", "split_1"):
                nt = 1 if leg == "split_1" else 0

                def f():
                    return L.stormck_commit_split(arena_p, bp, nb, REV, pla, op, None, 0, nt, _lib.SPLIT_BALANCED, pdone)
            else:  # routed: the library's pool (0) or one host thread ("routed_1")
                nt = 1 if leg == "routed_1" else 0

                def f():
                    return L.stormck_commit(arena_p, bp, nb, REV, pla, op, None, nt, pused)
            t0 = time.perf_counter()
            for _ in range(inner):
                rc = f()
            dt = (time.perf_counter() - t0) / inner
            _lib.check(rc)
            if leg in ("split", "split_1"):
                shares.setdefault(leg, []).append(done.value / nl)
            elif leg.startswith("routed"):
                outs[leg + "_leg"] = int(used.value)
            return dt, out

        row = {"forest": name, "blocks": int(len(b0)), "leaves": nl, "hashed_bytes": bytes_hashed,
               "timed_in": "C loop (tools/libcalltimer.so)" if inner > 1 and ct is not None else "Python"}
        shares = {}
        names = ("dev_inplace", "dev_hbm", "host_1", "host_all", "split", "split_1", "routed", "routed_1")
        ts = {leg: [] for leg in names}
        # 2 warm-up rounds, then timed ones, the legs interleaved in balanced orders (each leg
        # follows every other leg equally often: a leg's time depends on its predecessor,
        # e.g. a device left idle by a long host leg starts slower); calls of at most 64 MiB
        # run a whole cycle of the orders
        rounds = len(names) if bytes_hashed <= (64 << 20) else (reps if bytes_hashed < (1 << 30) else 3)
        orders = balanced_orders(names)
        for r in range(2 + rounds):
            for leg in orders[r % len(orders)]:
                dt, out = run(leg)
                if r >= 2:
                    ts[leg].append(dt)
                outs[leg] = out
        for leg in names:
            med = sorted(ts[leg])[len(ts[leg]) // 2]
            row[leg + "_us"] = round(med * 1e6, 3 if med < 1e-4 else 1)  # ns for calls of a few us
            row[leg + "_GiBps"] = round(bytes_hashed / med / 2**30, 2)
        for k in ("routed_leg", "routed_1_leg"):
            row[k] = _lib.LEG_NAMES.get(outs.get(k), outs.get(k))
        for k, v in shares.items():
            row[k + "_dev_share"] = round(sum(v) / len(v), 3)
        row["routed_over_best"] = round(row["routed_us"] / min(row[k + "_us"] for k in ("host_all", "dev_inplace",
                                                                                          "split")), 3)
        row["routed_1_over_best"] = round(row["routed_1_us"] / min(row[k + "_us"] for k in ("host_1", "dev_inplace",
                                                                                              "split_1")), 3)
        row["split_gain"] = round(min(row["host_all_us"], row["dev_inplace_us"]) / row["split_us"], 3)
        row["rates"] = {k: round(v, 1) for k, v in blocks.RouteRates().items()}
        row["agree"] = all(np.array_equal(outs["host_1"], outs[k]) for k in
                           ("dev_inplace", "dev_hbm", "host_all", "split", "split_1", "routed", "routed_1"))
        rows.append(row)
        print(json.dumps(row), flush=True)
        del hbm
        _lib.check(L.stormck_host_unregister(arena.ctypes.data))
        del raw, arena
    res = {"metric": "us per storm Cache.Commit data phase from host memory (f1 E2E), by leg",
           "value": rows[0]["routed_us"], "unit": "us", "n_gpus": 1, "steps": reps, "warmup": 2,
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": "f1 commit E2E, cache.data registered host memory; value = routed c5_keystore",
                      "host_threads": threads, "host": host_cpu_info()},
           "table": rows}
    print(json.dumps(res), flush=True)
    return 0 if all(r["agree"] for r in rows) else 3


def batch_e2e_workload(a):
    """Host-memory batches end to end (the Go shim's ChecksumBatch / VerifyChecksumBatch),
    by leg, on pageable memory first:
      dev          stormck_checksum_host (staged through pinned buffers, H2D / kernel / D2H
                   pipelined),
      host_1       stormck_checksum_host_leg on 1 thread (storm's serial xxhash.Sum64 loop
                   costs about twice this: one scalar chain per block),
      host_all     stormck_checksum_host_leg on every usable thread,
      routed       stormck_checksum_batch (the library's choice), pool threads,
      routed_1     the same with one host thread allowed (host cores kept for storm);
    then on the same memory registered with stormck_host_register (as the Go binding's
    cache.data):
      dev_reg      the device pipeline, DMA in place,
      host_1_reg / host_all_reg   the host leg on the registered copy (the legs the routed
                   and split calls on registered memory are compared with),
      split        stormck_checksum_split, balanced: the pool from the front and the device
                   from the back at once (split_dev_share = the device's blocks / n),
      split_1      the same with one host thread,
      routed_reg / routed_reg_1   the routed call on registered memory (it may split),
      routed_x2    two callers at once, each routed on its own half of the batch (wall
                   time of both; ADVICE r04: a caller that finds the pool busy plans on its
                   own thread). Batches of 512 MB and more only: below, starting and joining
                   two Python threads costs more than the call (c5-size pairs are timed in C
                   by tools/route_overhead.cpp).
    The routed calls use the rates the library measured so far in this process (every leg
    above updates them): `rates` is the model after the row. Batches: storm's c5 commit
    batch (1,200 objectlist leaves + a pointer block + the singularity,
    keystore/benchmark_test.go:58-62), the c1 batch (1K x 32 KiB), 3 blocks, a `-tags test`
    batch (100 blocks of 536 / 728 B, storm_test.go:131-138), 16K and 256K blocks of 32 KiB
    (512 MiB, 8 GiB). Every leg's checksums must agree. One line per batch with the table:
    median us per call, every leg once per round in balanced orders (each leg follows every
    other equally often; a whole cycle of orders for batches of at most 64 MiB, --steps
    rounds up to 4 GiB, 3 above), calls under 1 MiB as the mean of 200; routed_over_best =
    routed / the best of host_all and dev (pageable memory); routed_reg_over_best = routed_reg
    / the best of host_all_reg, dev_reg and split (registered; 1 thread: the _1 legs)."""
    import ctypes
    import numpy as np
    import torch
    from storm_amd import _lib
    from storm_amd import engine

    import threading
    from storm_amd import blocks

    torch.cuda.set_device(0)
    engine.init(0)
    L = _lib.lib
    c5 = np.array([31808] * 1200 + [30000, 72], dtype=np.uint32)
    shapes = [
        ("c5_keystore", 1202, c5),
        ("c1_1k", 1024, 32768),
        ("three_blocks", 3, np.array([31808, 31808, 30000], dtype=np.uint32)),
        ("test_tag", 100, np.array([536, 728] * 50, dtype=np.uint32)),
        ("blocks_16k", 16384, 32768),
        ("blocks_256k", 262144, 32768),
    ]
    threads = host_cpu_info()["usable_cpus"]
    reps = max(3, a.steps)
    rows = []
    ct = calltimer()
    for name, n, lens in shapes:
        stride = BLOCK
        # the same blocks twice: pageable (the pageable legs) and registered (the rest), so
        # every leg runs in every round, interleaved (each sees the others' cache effects)
        raw = np.zeros(n * stride + 4096, dtype=np.uint8)
        off = (-raw.ctypes.data) % 4096
        reg = raw[off:off + n * stride]
        for lo in range(0, n, 16384):  # synthetic blocks, generated on the device in slices
            hi = min(n, lo + 16384)
            reg[lo * stride:hi * stride] = engine_fill_host(hi - lo, stride)
        pg = reg.copy()
        _lib.check(L.stormck_host_register(reg.ctypes.data, reg.nbytes))
        la = lens if isinstance(lens, np.ndarray) else None
        ln = 0 if la is not None else int(lens)
        lp = la.ctypes.data if la is not None else None
        hashed = int(la.sum()) if la is not None else n * ln
        outs, legs = {}, {}

        # calls of a few microseconds are timed as the mean of `inner` back-to-back calls
        # (one call is within perf_counter's noise); the pointers are taken outside the clock
        inner = 200 if hashed < (1 << 20) else 1
        pg_p, reg_p = pg.ctypes.data, reg.ctypes.data

        def run(leg):
            out = np.zeros(n, dtype=np.uint64)
            op = out.ctypes.data
            bp = pg_p if leg in ("dev", "host_1", "host_all", "routed", "routed_1") else reg_p
            done, used = ctypes.c_uint64(0), ctypes.c_uint32(9)
            pdone, pused = ctypes.byref(done), ctypes.byref(used)  # converted outside the clock
            if inner > 1 and ct is not None and leg != "routed_x2":  # a few microseconds: the C loop
                code = 0 if leg.startswith("dev") else 1 if leg.startswith("host") else 2 if leg.startswith("split") else 3
                nt = threads if leg.startswith("host_all") else (1 if leg.endswith("_1") or leg.startswith("host_1") else 0)
                rc_ = ctypes.c_int(0)
                dt = ct.calltimer_batch(code, bp, stride, lp, ln, n, op, nt, inner, ctypes.byref(rc_), pused,
                                        pdone) * 1e-6
                _lib.check(rc_.value)
                if leg in ("split", "split_1"):
                    shares.setdefault(leg, []).append(done.value / n)
                elif leg.startswith("routed"):
                    legs[leg] = _lib.LEG_NAMES.get(int(used.value), int(used.value))
                return dt, out
            if leg in ("dev", "dev_reg"):
                def f():
                    return L.stormck_checksum_host(bp, stride, lp, ln, n, op)
            elif leg in ("host_1", "host_all", "host_1_reg", "host_all_reg"):
                nt = 1 if leg.startswith("host_1") else threads

                def f():
                    return L.stormck_checksum_host_leg(bp, stride, lp, ln, n, op, nt)
            elif leg in ("split", "split_1"):
                nt = 1 if leg == "split_1" else 0

                def f():
                    return L.stormck_checksum_split(bp, stride, lp, ln, n, op, None, 0, nt, _lib.SPLIT_BALANCED,
                                                    pdone)
            elif leg == "routed_x2":
                h = n // 2
                outs2, rcs = [out[:h], out[h:]], [0, 0]

                def half(k):
                    lo = 0 if k == 0 else h
                    u = ctypes.c_uint32(9)
                    rcs[k] = L.stormck_checksum_batch(reg_p + lo * stride, stride,
                                                      (la[lo:].ctypes.data if la is not None else None), ln,
                                                      (h if k == 0 else n - h), outs2[k].ctypes.data, 0,
                                                      ctypes.byref(u))
                    legs.setdefault("routed_x2", set()).add(_lib.LEG_NAMES.get(int(u.value), int(u.value)))

                def f():
                    ths = [threading.Thread(target=half, args=(k,)) for k in range(2)]
                    for t in ths:
                        t.start()
                    for t in ths:
                        t.join()
                    return rcs[0] or rcs[1]
            else:
                nt = 1 if leg.endswith("_1") else 0

                def f():
                    return L.stormck_checksum_batch(bp, stride, lp, ln, n, op, nt, pused)
            reps_in = 1 if leg == "routed_x2" else inner
            t0 = time.perf_counter()
            for _ in range(reps_in):
                rc = f()
            dt = (time.perf_counter() - t0) / reps_in
            _lib.check(rc)
            if leg in ("split", "split_1"):
                shares.setdefault(leg, []).append(done.value / n)
            elif leg != "routed_x2" and leg.startswith("routed"):
                legs[leg] = _lib.LEG_NAMES.get(int(used.value), int(used.value))
            return dt, out

        row = {"batch": name, "blocks": n, "hashed_bytes": hashed,
               "timed_in": "C loop (tools/libcalltimer.so)" if inner > 1 and ct is not None else "Python"}
        shares = {}
        names = ["dev", "host_1", "host_all", "routed", "routed_1", "dev_reg", "host_1_reg", "host_all_reg", "split",
                 "split_1", "routed_reg",
                 "routed_reg_1"] + (["routed_x2"] if hashed >= (512 << 20) else [])
        ts = {leg: [] for leg in names}
        # 2 warm-up rounds, then timed ones in balanced orders, as in commit_e2e
        rounds = len(names) if hashed <= (64 << 20) else (reps if hashed < (4 << 30) else 3)
        orders = balanced_orders(names)
        for r in range(2 + rounds):
            for leg in orders[r % len(orders)]:
                dt, out = run(leg)
                if r >= 2:
                    ts[leg].append(dt)
                outs[leg] = out
        for leg in names:
            med = sorted(ts[leg])[len(ts[leg]) // 2]
            row[leg + "_us"] = round(med * 1e6, 3 if med < 1e-4 else 1)  # ns for calls of a few us
            row[leg + "_GiBps"] = round(hashed / med / 2**30, 2)
        _lib.check(L.stormck_host_unregister(reg.ctypes.data))
        for k in ("routed", "routed_1", "routed_reg", "routed_reg_1"):
            row[k + "_leg"] = legs.get(k)
        row["routed_x2_legs"] = sorted(legs.get("routed_x2", []))
        for k, v in shares.items():
            row[k + "_dev_share"] = round(sum(v) / len(v), 3)

        def best(*ks):
            return min(row[k + "_us"] for k in ks)
        row["routed_over_best"] = round(row["routed_us"] / best("host_all", "dev"), 3)
        row["routed_1_over_best"] = round(row["routed_1_us"] / best("host_1", "dev"), 3)
        row["routed_reg_over_best"] = round(row["routed_reg_us"] / best("host_all_reg", "dev_reg", "split"), 3)
        row["routed_reg_1_over_best"] = round(row["routed_reg_1_us"] / best("host_1_reg", "dev_reg", "split_1"), 3)
        row["split_gain"] = round(best("host_all_reg", "dev_reg") / row["split_us"], 3)
        row["rates"] = {k: round(v, 1) for k, v in blocks.RouteRates().items()}
        row["agree"] = all(np.array_equal(outs["host_1"], outs[k]) for k in outs)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del raw, reg, pg
    res = {"metric": "us per host-memory batch checksum (ChecksumBatch E2E), by leg",
           "value": rows[0]["routed_us"], "unit": "us", "n_gpus": 1, "steps": reps, "warmup": 2,
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": "host-memory batches, pageable, then registered (dev_reg, split*, routed_reg*); "
                                  "value = routed c5_keystore",
                      "host_threads": threads, "host": host_cpu_info()},
           "table": rows}
    print(json.dumps(res), flush=True)
    return 0 if all(r["agree"] for r in rows) else 3


def engine_fill_host(n: int, stride: int):
    """n synthetic blocks (SURVEY §8d generator) as host bytes: the library's device
    generator, copied back."""
    import torch
    from storm_amd import engine
    t = torch.empty((n, stride), dtype=torch.uint8, device="cuda")
    engine.fill_synthetic_device(t.data_ptr(), stride, n, 0, SYNTH_SEED)
    return t.cpu().numpy().reshape(-1)


def gather_workload(a):
    """storm's batch shape on the LDS-DMA ring: 4M dirty blocks gathered from a 4M-slot
    arena of 32 KiB slots (cache.data, cache/cache.go:36-40) in a shuffled slot order,
    lengths drawn from storm's leaf and node sizes 31,808 / 30,000 / 32,768 / 28,808 B
    (blocks/objectlist, pointer, blob, spacelist), per-block lengths (k_xxh64_glds_var,
    persistent and 4 KiB-skewed). One step = one stormck_checksum_gather_device call."""
    import numpy as np
    import torch
    from storm_amd import engine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    engine.init(0)
    n, slot = a.gather_blocks, a.gather_slot
    rng = np.random.default_rng(3)
    perm = rng.permutation(n).astype(np.uint64) if a.gather_order == "shuffled" else np.arange(n, dtype=np.uint64)
    lset = [int(x) for x in a.gather_lens_set.split(",")] if a.gather_lens_set else [31808, 30000, 32768, 28808]
    if slot % 16 or max(lset + [a.gather_lens]) > slot:
        raise SystemExit("--gather-slot must be a multiple of 16 and hold every length")
    lens = np.array(lset, dtype=np.uint32)[rng.integers(0, len(lset), size=n)]
    if a.gather_lens:
        lens[:] = a.gather_lens
    arena_ptr = engine.device_alloc(n * slot)
    engine.fill_synthetic_device(arena_ptr, slot, n, 0, SYNTH_SEED)
    d_offs = torch.from_numpy((perm * np.uint64(slot)).view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream

    longest = int(lens.max())  # the caller knows its lengths: the bound the library plans with

    def step():
        if a.gather_order == "strided":
            engine.checksum_device(arena_ptr, slot, n, out.data_ptr(), longest, d_lens.data_ptr(), st)
        else:
            engine.checksum_gather_device(arena_ptr, d_offs.data_ptr(), n, out.data_ptr(), longest, d_lens.data_ptr(), st)

    settle(step, a.settle)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        e[0].record(stream)
        step()
        e[1].record(stream)
        evs.append(e)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)
    avg_ms = sum(kms) / len(kms)
    hashed = int(lens.sum())
    alg = hashed + n * (8 + (0 if a.gather_order == "strided" else 8) + 4)  # blocks + checksum + offset, length
    res = {"metric": "GiB/s gathered per-block-length checksum (storm's dirty-slot batch shape), device-resident",
           "value": round(hashed * a.steps / el / 2**30, 2), "unit": "GiB/s", "n_gpus": 1, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"gather: {n} blocks from {n} {a.gather_order} {slot}-byte slots, lengths of "
                                  + (f"{a.gather_lens} B" if a.gather_lens else "/".join(map(str, lset)) + " B")
                                  + ", per-block lengths (stormck_checksum_gather_device)",
                      "blocks": n, "hashed_bytes": hashed,
                      "arena": {"va": "0x%x" % arena_ptr, "va_alignment": va_alignment(arena_ptr)}},
           "roofline": {"bound": "hbm", "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "kernel": "k_xxh64_glds_var<16,nt,8w,4KiB,lens,offs>", "avg_launch_ms": round(avg_ms, 4),
                        "launch_ms": {"n": len(kms), "min": round(kms[0], 4), "max": round(kms[-1], 4)},
                        "algorithmic_bytes_per_launch": alg}}
    res["G_blocks_per_s"] = round(n / (avg_ms * 1e-3) / 1e9, 3)  # the rate that matters for small blocks
    # the same arena through the uniform-length path (k_xxh64_glds_skew: every block 32 KiB,
    # in slot order), 3 launches after the timed region: the rate this placement gives the
    # uniform kernel, beside which the gather's frac reads
    ref = torch.empty(n, dtype=torch.int64, device=dev)
    rms = []
    for r in range(4):
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        e[0].record(stream)
        engine.checksum_device(arena_ptr, slot, n, ref.data_ptr(), slot, 0, st)
        e[1].record(stream)
        torch.cuda.synchronize()
        if r:
            rms.append(e[0].elapsed_time(e[1]))
    ref_gbs = n * (slot + 8) / (sum(rms) / len(rms) * 1e-3) / 1e9
    res["roofline"]["uniform_same_arena"] = {"kernel": KERNEL, "GB/s": round(ref_gbs, 1),
                                             "frac": round(ref_gbs / HBM_PEAK_GBS, 4)}
    del ref
    from storm_amd import blocks
    digest = blocks.Checksum(out.cpu().numpy().view(np.uint64).astype("<u8"))
    res["digest"] = "0x%016x" % digest
    print(json.dumps(res), flush=True)
    del out
    torch.cuda.synchronize()
    engine.device_free(arena_ptr)
    return 0


def keytags_workload(a):
    """f4: one step = xxhash.Sum64 of 64M 48-byte keys resident in HBM (the key shape of
    keystore/benchmark_test.go:27-32), one lane per key (stormck_key_tags_device)."""
    import numpy as np
    import torch
    from storm_amd import engine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, klen = a.keys, 48
    keys = torch.empty(n * klen, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(keys.data_ptr(), 48 * 1024, n * klen // (48 * 1024), 0, 0x53544F524D)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    settle(lambda: engine.key_tags_device(keys.data_ptr(), n, out.data_ptr(), stride=klen, length=klen, stream=st),
           a.settle)
    for _ in range(a.warmup):
        engine.key_tags_device(keys.data_ptr(), n, out.data_ptr(), stride=klen, length=klen, stream=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        engine.key_tags_device(keys.data_ptr(), n, out.data_ptr(), stride=klen, length=klen, stream=st)
    e1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms = e0.elapsed_time(e1) / a.steps
    res = {"metric": "G keys/s key-tag hashing (f4, xxhash.Sum64 of 48-byte keys)",
           "value": round(n * a.steps / el / 1e9, 3), "unit": "Gkeys/s", "n_gpus": 1, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"f4: {n / 2**20:g}M x 48-byte keys in HBM, one tag per key", "keys": n,
                      "key_bytes": klen},
           "roofline": {"bound": "hbm", "achieved": round(n * (klen + 8) / (kms * 1e-3) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(n * (klen + 8) / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "kernel": "k_key_tags_ring<nt,3,4,8> (per-wave 4-slot LDS-DMA ring)", "avg_launch_ms": round(kms, 4)}}
    # all 64M tags against tests/golden/keytags.json (digest by the library's host leg)
    from storm_amd import blocks
    fx = golden("keytags.json")
    digest = blocks.Checksum(out.cpu().numpy().view(np.uint64).astype("<u8"))
    want = fx["digest"] if fx and fx["keys"] == n else None
    res["root_check"], rc = check_against(digest, want, "f4 tag digest, tests/golden/keytags.json")
    if not a.no_cpu:
        from oracle import oracle as o
        m = 1 << 20
        host = keys[:m * klen].cpu().numpy()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < a.cpu_seconds:
            o.checksum_batch(host, m, klen, klen)
            reps += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(reps * m / el / 1e9, 4), "unit": "Gkeys/s", "cores": 1, "kind": "port",
                               "sample": f"{m} 48-byte keys hashed {reps}x in {el:.1f} s by oracle/xxh64_oracle.c"}
    print(json.dumps(res), flush=True)
    return rc


def host_cpu_info():
    """The host the CPU baseline runs on: CPU model, logical CPUs, this process's
    affinity and its cgroup CPU quota (a GPU box shares a large host between GPUs)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return {"model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "usable_cpus": usable}


def _rank_entry(env, argv, entry):
    """Body of one spawned rank: the launcher's environment, then bench main() (or
    `entry` = "module:function", which the CPU tests use to rehearse the launcher)."""
    os.environ.update(env)
    sys.argv = list(argv)
    if entry:
        import importlib
        mod, fn = entry.split(":")
        getattr(importlib.import_module(mod), fn)()
    else:
        main()


def spawn_ranks(n: int, argv, entry=None, timeout: float = 0.0) -> int:
    """`bench.py --gpus N` without torchrun: start N rank processes (spawn context) with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, exactly as
    torch.distributed.run would. The parent never touches the GPU. A rank that fails
    would leave the others blocked inside a collective, so the parent ends them
    (their exact PIDs) and returns the failing exit code."""
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = []
    for r in range(n):
        env = {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
               "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}
        p = ctx.Process(target=_rank_entry, args=(env, list(argv), entry))
        p.start()
        procs.append(p)
    rc, t0 = 0, time.time()
    while any(p.is_alive() for p in procs):
        failed = [p for p in procs if p.exitcode not in (None, 0)]
        late = timeout > 0 and time.time() - t0 > timeout
        if failed or late:
            rc = failed[0].exitcode if failed else 124
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(10)
                if p.is_alive():
                    p.kill()
            break
        time.sleep(0.1)
    for p in procs:
        p.join()
    if rc == 0:
        rc = next((p.exitcode for p in procs if p.exitcode), 0)
    return rc if rc >= 0 else 128 - rc


def gather_rank_rows(elapsed: float, wall: float, kms, rank: int, blocks: int, tdev):
    """All-gather every rank's (elapsed, wall, kernel avg / min / max ms, rank, blocks) over the
    process group (RCCL on GPUs, gloo in the CPU rehearsal) as a list of rows in rank order."""
    import torch
    import torch.distributed as dist
    kms = sorted(kms)
    mine = torch.tensor([elapsed, wall, sum(kms) / len(kms), kms[0], kms[-1], float(rank), float(blocks)],
                        dtype=torch.float64, device=tdev)
    allr = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(allr, mine)
    return [[float(x) for x in r.cpu().tolist()] for r in allr]


def summarize_ranks(rows, steps: int):
    """(the slowest rank's elapsed time, the longest wall time, the per-rank record): the MAX
    over ranks sets `value`."""
    slow = max(range(len(rows)), key=lambda r: rows[r][0])
    ranks = {"slowest_rank": slow,
             "per_rank": [{"rank": int(r[5]), "blocks": int(r[6]), "ms_per_step": round(r[0] / steps * 1e3, 3),
                           "kernel_avg_ms": round(r[2], 4), "kernel_min_ms": round(r[3], 4),
                           "kernel_max_ms": round(r[4], 4)} for r in rows]}
    return rows[slow][0], max(r[1] for r in rows), ranks


C4_WORLD1 = os.path.join(ROOT, "profiles", "c4_world1.json")  # measured c4 N = 1 point (bench.py --in-process)


def scaling_reference(world: int, n_total: int, ranks, value: float, scaling: str) -> dict:
    """Fields of an N > 1 line that say which N = 1 number its scaling reads against (verdict
    r05 item 3): the driver's N = 1 line is c3 (16M blocks on one GPU), while N > 1 runs c4
    (64M blocks split over N GPUs, strong scaling), so per-GPU GiB/s is the comparable figure.
    The strong-scaling N = 1 time of THIS workload is given two ways: estimated from this run
    (the slowest rank's time per block x all n_total blocks) and, when committed, measured
    (c4 world 1 in one process on one GPU: profiles/c4_world1.json)."""
    per = ranks["per_rank"]
    slow = per[ranks["slowest_rank"]]
    est_ms = slow["ms_per_step"] / max(slow["blocks"], 1) * n_total
    ref = {"per_gpu_GiB_s": round(value / world, 2),
           "scaling_reference": {
               "read_against": "per_gpu_GiB_s vs the N = 1 line's value (both are GiB/s of distinct 32 KiB blocks "
                               "per GPU); ms_per_step vs strong_scaling_n1_ms_per_step",
               "driver_n1_line": "bench.py --gpus 1 = c3: 16M blocks on one GPU (weak); not this workload",
               "this_workload": f"{scaling} scaling: {n_total} blocks over {world} GPUs",
               "strong_scaling_n1_ms_per_step_estimate": round(est_ms, 3),
               "estimate_from": f"rank {slow['rank']}: {slow['ms_per_step']} ms per step for {slow['blocks']} "
                                f"blocks, x {n_total} blocks"}}
    if os.path.exists(C4_WORLD1):
        with open(C4_WORLD1) as f:
            m = json.load(f)
        if m.get("total_blocks") == n_total:
            ref["scaling_reference"]["strong_scaling_n1_ms_per_step"] = m["ms_per_step"]
            ref["scaling_reference"]["strong_scaling_n1_value_GiB_s"] = m["value"]
            ref["scaling_reference"]["strong_scaling_n1_source"] = m["source"]
    return ref


def root_fixture(n_total: int, world: int, distributed: bool):
    """The libxxhash root of this workload from tests/golden/c3c4_roots.json
    (oracle/gen_golden.py --c4), as (cs, addr, rev, type), or None if the workload has
    none (a non-default --blocks / --total-blocks)."""
    path = os.path.join(ROOT, "tests", "golden", "c3c4_roots.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        fx = json.load(f)
    row = None
    worlds = fx["c4"]["worlds"]
    if world == 1 and not distributed and n_total == fx["c3"]["n"]:
        row, name = fx["c3"]["root"], "c3"
    elif world == 1 and not distributed and n_total == fx["c4"]["n_total"] and "1" in worlds:
        # the strong-scaling series' N = 1 point: all 64M blocks in one shard tree
        row, name = worlds["1"]["shard_roots"][0], "c4 world 1 (shard root)"
    elif n_total == fx["c4"]["n_total"] and str(world) in worlds and (world > 1 or distributed):
        row, name = worlds[str(world)]["global_root"], f"c4 world {world}"
    if row is None:
        return None, None
    return (int(row[0], 16), int(row[1], 16), int(row[2], 16), int(row[3])), name


def main():
    a = parse()
    if a.in_process:
        sys.exit(block_checksum_inprocess(a))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: one rank process per GPU, started before this process touches a GPU
        sys.exit(spawn_ranks(a.gpus, sys.argv))
    if a.workload == "commit":
        rc = commit_workload(a)
    elif a.workload == "keytags":
        rc = keytags_workload(a)
    elif a.workload == "c5":
        rc = c5_workload(a)
    elif a.workload == "gather":
        rc = gather_workload(a)
    elif a.workload == "commit_e2e":
        rc = commit_e2e_workload(a)
    elif a.workload == "batch_e2e":
        rc = batch_e2e_workload(a)
    else:
        rc = block_checksum_workload(a)
    if rc:
        sys.exit(rc)


def block_checksum_workload(a) -> int:
    """c3 (N = 1) / c4 (N > 1): the BASELINE metric. Returns a non-zero exit code when
    the printed root differs from the libxxhash fixture of the same workload."""
    import torch

    from storm_amd import dist as sdist
    from storm_amd import engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    gpu = local % torch.cuda.device_count()  # == local on a node with one GPU per rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    distributed = world > 1 or a.force_dist
    if distributed:
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    engine.init(gpu)
    if distributed:
        # what the process group actually formed (the driver's N > 1 line must show it)
        group = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                 "device_count": torch.cuda.device_count(), "device": gpu}

    # c3 at N = 1 (16M blocks); c4 at N > 1 (64M blocks in contiguous shards, strong
    # scaling: 8M per GPU at N = 8). --blocks B: B per GPU instead (weak scaling).
    if a.blocks:
        n_total, scaling = a.blocks * world, "weak"
    else:
        n_total = a.total_blocks or (C3_BLOCKS if world == 1 else C4_BLOCKS)
        scaling = "weak" if world == 1 else "strong"
    lo, hi = sdist.shard_range(n_total, world, rank)
    n_gpu = hi - lo
    arena_n = min(a.arena, n_gpu)
    passes = (n_gpu + arena_n - 1) // arena_n
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream

    # The arena is the process's first device allocation (at N > 1, after RCCL's own
    # buffers), taken by plain hipMalloc through the library rather than torch's caching
    # allocator, so a profiled and a plain process place it the same way (DESIGN_LOG.md §5).
    mode, chunk = ALLOC_MODES[a.alloc]
    arena_ptr, mapped_chunk = engine.device_alloc_placed(arena_n * BLOCK, mode, chunk)
    cs = torch.empty(n_gpu, dtype=torch.int64, device=dev)
    ws = torch.empty(max(engine.merkle_workspace_bytes(n_gpu, FANOUT) // 8, 1), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    hash_ev, fill_ev = [], []  # (start, end[, blocks]) events of the timed steps, on `stream`

    def ev_pair():
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(record: bool):
        # The shard's blocks do not fit in HBM (c3: 512 GiB per GPU), so each arena pass
        # is regenerated with its own logical blocks lo + first .. (the on-device
        # generator stands in for the data arriving). The regeneration is timed by its
        # own events and taken out of the step time; the hash launches are timed too.
        for p in range(passes):
            first = p * arena_n
            cnt = min(arena_n, n_gpu - first)
            f = ev_pair() if record else None
            if f:
                f[0].record(stream)
            engine.fill_synthetic_device(arena_ptr, BLOCK, cnt, lo + first, SYNTH_SEED, st)
            e = ev_pair() if record else None
            if f:
                f[1].record(stream)
                fill_ev.append(f)
                e[0].record(stream)
            engine.checksum_device(arena_ptr, BLOCK, cnt, cs[first:].data_ptr(), BLOCK, 0, st)
            if e:
                e[1].record(stream)
                hash_ev.append((e[0], e[1], cnt))
        root = engine.merkle_root_tensor(cs, lo, sdist.shard_node_addr_base(n_total, lo), REV, FANOUT, ws)
        if distributed:
            root, _ = sdist.global_root(root, REV, n_total, lambda t, r, ad: engine.combine_roots_tensor(t, r, ad, FANOUT))
        return root

    settle(lambda: step(False), a.settle, dev if distributed else None)
    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        root = step(True)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    fill_s = sum(f0.elapsed_time(f1) for f0, f1 in fill_ev) * 1e-3
    elapsed = wall - fill_s  # the K steps without the arena regeneration
    # dominant kernel: per-launch durations from HIP events on its stream
    kms = sorted(e0.elapsed_time(e1) for (e0, e1, _) in hash_ev)
    kblocks = [c for (_, _, c) in hash_ev]
    avg_ms = sum(kms) / len(kms)
    ranks = None
    if distributed:
        # every rank's step time and kernel launches; the MAX step time sets `value`
        tdev = dev if a.dist_backend == "nccl" else "cpu"  # gloo all-gathers host tensors
        rows = gather_rank_rows(elapsed, wall, kms, rank, n_gpu, tdev)
        elapsed, wall, ranks = summarize_ranks(rows, a.steps)
    avg_blocks = sum(kblocks) / len(kblocks)
    alg_bytes = avg_blocks * (BLOCK + 8)          # L bytes read + 8 bytes written per block
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9  # GB/s (decimal, like the spec peak)

    total_bytes = n_total * BLOCK * a.steps
    value = total_bytes / elapsed / 2**30
    traffic, prof = None, None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("arena_blocks") == arena_n and tj.get("kernel") == KERNEL:
            traffic = tj.get("hbm_bytes_per_launch")
            # the committed rocprofv3 session this line's frac can be recomputed from
            # (tools/collect_profile.py): its kernel-trace average and the frac it implies
            prof = {k: tj.get(k) for k in ("source", "pmc_source", "profile_calls", "profile_avg_launch_ms",
                                           "profile_frac", "profile_timed_launches", "bench_under_rocprof",
                                           "traffic_over_algorithmic", "placement_spread")}

    # The frac depends on where the arena lands in HBM (0.84-0.89 across fresh processes;
    # neither VMM placement collapses the spread, DESIGN_LOG.md §10.1): report this line's frac
    # beside the committed session's placement spread, the spread widened to include it.
    placement = None
    if prof and prof.get("placement_spread"):
        import statistics
        fr = list(prof["placement_spread"]["fracs"])
        line = round(achieved / HBM_PEAK_GBS, 4)
        placement = {"line_frac": line, "session": prof.get("source"),
                     "session_median": round(statistics.median(fr), 4),
                     "spread_with_line": [min(fr + [line]), max(fr + [line])],
                     "median_with_line": round(statistics.median(fr + [line]), 4),
                     "session_processes_below_line": sum(1 for f in fr if f < line), "session_processes": len(fr)}

    # also report against a measured stream-read peak. Measured here, after
    # the timed region, on the same arena: the rate depends on where the arena lands in
    # HBM (DESIGN_LOG.md §5), so a peak from another process or box would not compare.
    read_peak = measured_read_peak(arena_ptr, arena_n, stream, achieved)

    gather = ""
    if distributed:
        gather = " + RCCL all-gather of shard roots" if a.dist_backend == "nccl" else " + gloo all-gather of shard roots (rehearsal)"
    rc = 0
    if rank == 0:
        root_t = engine.as_tuple(root)
        want, fx_name = root_fixture(n_total, world, distributed)
        if want is None:
            check = "no fixture for this workload"
        elif want == root_t:
            check = f"match ({fx_name}, tests/golden/c3c4_roots.json)"
        else:
            check = f"MISMATCH vs {fx_name} fixture root 0x{want[0]:016x}"
            rc = 3
        cfg = "c3" if (world == 1 and n_total == C3_BLOCKS) else ("c4" if n_total == C4_BLOCKS else "custom")
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": f"{cfg}: {n_total / 2**20:g}M x 32 KiB blocks over {world} GPU(s) "
                                   f"({n_gpu / 2**20:g}M on rank 0), XXH64 seed 0 (blocks.Checksum) "
                                   "+ shard Merkle pointer tree" + gather,
                       "total_blocks": n_total, "blocks_per_gpu": n_gpu, "block_bytes": BLOCK,
                       "arena_blocks": arena_n, "passes_per_step": passes,
                       "parallelism": f"dp{world} (contiguous block ranges)",
                       "library": engine.library_record(),
                       "arena": {"va": "0x%x" % arena_ptr, "va_alignment": va_alignment(arena_ptr),
                                 "bytes": arena_n * BLOCK,
                                 "alloc": {"plain": "hipMalloc",
                                           "contig": "hipExtMallocWithFlags(hipDeviceMallocContiguous)"}[a.alloc]
                                          + (" (stormck_device_alloc)" if a.alloc == "plain" else
                                             " (stormck_device_alloc_placed, probe build)")
                                          + ", the process's first device allocation"
                                          + (" after the process group's" if distributed else ""),
                                 "mode": a.alloc, "mapped_chunk": mapped_chunk},
                       "timed": "K steps between barrier + synchronize, minus the on-device regeneration of "
                                "each arena pass (its own HIP events)",
                       "ms_per_step_with_regeneration": round(wall / a.steps * 1e3, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": KERNEL, "avg_launch_ms": round(avg_ms, 4),
                         "launch_ms": {"n": len(kms), "min": round(kms[0], 4),
                                       "median": round(kms[len(kms) // 2], 4), "max": round(kms[-1], 4),
                                       "in_order": [round(e0.elapsed_time(e1), 3) for (e0, e1, _) in hash_ev]},
                         "algorithmic_bytes_per_launch": int(alg_bytes), "profile_source": prof,
                         "placement": placement,
                         "measured_read_peak": read_peak},
            "root": "0x%016x" % root_t[0],
            "root_pointer": ["0x%016x" % v for v in root_t[:3]] + [root_t[3]],
            "root_check": check,
        }
        if distributed:
            res["config"]["process_group"] = group
            res["ranks"] = ranks
            res.update(scaling_reference(world, n_total, ranks, value, scaling))
        if world == 1 and not a.no_cpu:
            res["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()
    torch.cuda.synchronize()
    engine.device_free(arena_ptr)
    return rc


def block_checksum_inprocess(a) -> int:
    """--in-process: the BASELINE metric on --gpus N devices driven from one process, as storm
    (one Go process) would through its cgo shim. Each device streams its planned shard
    (stormck_shard_plan) through its own arena on its own stream, exactly like a rank of the
    process-per-GPU path; the step's root then comes from ONE C-ABI call,
    stormck_merkle_root_multi: the shard trees on their devices, an in-process RCCL
    ncclAllGather of the shard roots, the combining node hashed on every device. The line has
    the shape of the process-per-GPU line; `ranks` are devices here."""
    import torch

    from storm_amd import engine, multi

    world = a.gpus
    n_dev = torch.cuda.device_count()
    if world > n_dev:
        raise SystemExit(f"--in-process --gpus {world}: only {n_dev} visible device(s)")
    if a.blocks:
        n_total, scaling = a.blocks * world, "weak"
    else:
        n_total = a.total_blocks or (C3_BLOCKS if world == 1 else C4_BLOCKS)
        scaling = "weak" if world == 1 and n_total == C3_BLOCKS else "strong"
    devices = list(range(world))
    shards, root_addr = multi.plan(n_total, world, devices)
    per = []
    for sh in shards:
        d = sh.device
        torch.cuda.set_device(d)
        engine.init(d)
        dev = torch.device("cuda", d)
        arena_n = min(a.arena, max(sh.n, 1))
        stream = torch.cuda.Stream(device=dev)
        P = {"dev": dev, "arena": engine.device_alloc(arena_n * BLOCK), "arena_n": arena_n,
             "cs": torch.empty(max(sh.n, 1), dtype=torch.int64, device=dev), "stream": stream,
             "passes": (sh.n + arena_n - 1) // arena_n, "fill": [], "hash": []}
        # the trees run on the shard's stream, after the passes that produced its checksums
        multi.set_buffers(sh, P["cs"].data_ptr(), stream=stream.cuda_stream)
        per.append(P)
    torch.cuda.set_device(0)

    def sync_all():
        for d in devices:
            torch.cuda.synchronize(d)

    sync_all()

    def ev_pair():
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(record: bool):
        for p in range(max(P["passes"] for P in per)):
            for sh, P in zip(shards, per):  # pass p on every device before pass p + 1 anywhere
                first = p * P["arena_n"]
                if first >= sh.n:
                    continue
                cnt = min(P["arena_n"], sh.n - first)
                st = P["stream"]
                with torch.cuda.device(P["dev"]):
                    f, e = (ev_pair(), ev_pair()) if record else (None, None)
                    if f:
                        f[0].record(st)
                    engine.fill_synthetic_device(P["arena"], BLOCK, cnt, sh.leaf_addr_base + first, SYNTH_SEED,
                                                 st.cuda_stream)
                    if f:
                        f[1].record(st)
                        e[0].record(st)
                    engine.checksum_device(P["arena"], BLOCK, cnt, P["cs"][first:].data_ptr(), BLOCK, 0,
                                           st.cuda_stream)
                    if e:
                        e[1].record(st)
                        P["fill"].append(f)
                        P["hash"].append((e[0], e[1], cnt))
        return multi.merkle_root_multi(shards, REV, root_addr, FANOUT)  # synchronous

    settle(lambda: step(False), a.settle)
    for _ in range(a.warmup):
        step(False)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        root, rows = step(True)
    sync_all()
    wall = time.perf_counter() - t0
    # each device's elapsed time is the wall time less its own regeneration; the MAX over
    # devices (the least regeneration taken out) sets `value`, as the MAX over ranks does
    dev_rows = []
    for k, (sh, P) in enumerate(zip(shards, per)):
        fill_s = sum(f0.elapsed_time(f1) for f0, f1 in P["fill"]) * 1e-3
        kms = sorted(e0.elapsed_time(e1) for (e0, e1, _) in P["hash"])
        dev_rows.append([wall - fill_s, wall, sum(kms) / len(kms), kms[0], kms[-1], float(k), float(sh.n)])
    elapsed, wall, ranks = summarize_ranks(dev_rows, a.steps)
    for r, sh in zip(ranks["per_rank"], shards):
        r["device"] = sh.device
    launches = [(e0.elapsed_time(e1), c) for P in per for (e0, e1, c) in P["hash"]]
    avg_ms = sum(t for t, _ in launches) / len(launches)
    avg_blocks = sum(c for _, c in launches) / len(launches)
    achieved = avg_blocks * (BLOCK + 8) / (avg_ms * 1e-3) / 1e9
    value = n_total * BLOCK * a.steps / elapsed / 2**30

    fx = golden("c3c4_roots.json")
    fmt = lambda r: ["0x%016x" % v for v in r[:3]] + [r[3]]  # noqa: E731
    check, rc = "no fixture for this workload", 0
    if fx and world == 1 and n_total == fx["c3"]["n"]:
        ok = fmt(rows[0]) == fx["c3"]["root"]
        check = "shard root " + ("match (c3" if ok else "MISMATCH vs c3") + ", tests/golden/c3c4_roots.json)"
        rc = 0 if ok else 3
    elif fx and n_total == fx["c4"]["n_total"] and str(world) in fx["c4"]["worlds"]:
        want = fx["c4"]["worlds"][str(world)]
        ok = fmt(root) == want["global_root"] and [fmt(r) for r in rows] == want["shard_roots"]
        check = ("match" if ok else "MISMATCH vs") + f" c4 world {world} (global and shard roots, " \
                                                     "tests/golden/c3c4_roots.json)"
        rc = 0 if ok else 3
    cfg = "c3" if (world == 1 and n_total == C3_BLOCKS) else ("c4" if n_total == C4_BLOCKS else "custom")
    res = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": f"{cfg}: {n_total / 2**20:g}M x 32 KiB blocks over {world} GPU(s) from one process, "
                               "XXH64 seed 0 (blocks.Checksum) + shard Merkle pointer trees + in-process RCCL "
                               "all-gather of the shard roots (stormck_merkle_root_multi)",
                   "total_blocks": n_total, "blocks_per_gpu": [sh.n for sh in shards], "block_bytes": BLOCK,
                   "arena_blocks": per[0]["arena_n"], "passes_per_step": per[0]["passes"],
                   "parallelism": f"dp{world} (one process, contiguous block ranges, a device each)",
                   "library": engine.library_record(),
                   "process_group": {"mode": "in-process", "world_size": world, "device_count": n_dev,
                                     "backend": "rccl: ncclCommInitAll + ncclAllGather inside stormck_merkle_root_multi"},
                   "timed": "K steps between synchronize of every device, minus each device's on-device "
                            "regeneration (its own HIP events); the slowest device sets the time",
                   "ms_per_step_with_regeneration": round(wall / a.steps * 1e3, 3)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": KERNEL,
                     "avg_launch_ms": round(avg_ms, 4), "launch_ms": {"n": len(launches)},
                     "algorithmic_bytes_per_launch": int(avg_blocks * (BLOCK + 8))},
        "root": "0x%016x" % root[0], "root_pointer": fmt(root), "shard_roots": [fmt(r) for r in rows],
        "root_check": check, "ranks": ranks,
    }
    if world > 1:
        res.update(scaling_reference(world, n_total, ranks, value, scaling))
    if world == 1 and not a.no_cpu:
        res["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
    print(json.dumps(res), flush=True)
    sync_all()
    for P in per:
        with torch.cuda.device(P["dev"]):
            engine.device_free(P["arena"])
    return rc


if __name__ == "__main__":
    main()
