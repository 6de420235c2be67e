"""The split leg on the GPU: host threads and the device hash one host-memory call at once.

storm's cache.data is host memory (/root/reference/cache/cache.go:36-40), registered in the
stormck build, so a commit or batch from it can run on the host threads and the device at
the same time: the host threads take blocks from the front, the device chunks from the
back (include/stormck.h, "routing of host-memory work"). Bit-exact against the C oracle
(blocks.Checksum = XXH64 seed 0, /root/reference/blocks/checksum.go:15-17; storm's serial
commit loop, cache/cache.go:87-137 + trace.go:274-320):
  * fixed boundaries, from all-host to all-device, on strided, per-block-length and short
    (`-tags test`) batches, with mismatches planted on each side of the boundary;
  * edge shapes (1-3 blocks, empty and sub-stripe blocks, unaligned rows) and seeded
    fuzzes: split batches (counts, strides, lengths, offsets, threads, shares, planted
    mismatches), split commits (forests, fan-outs, shares), routed calls under rates that
    force each leg;
  * the balanced split and the routed call taking it;
  * the split commit (leaves on both sides, in place) against the oracle's commit, with
    relocations, and the routed commit taking it;
  * the routed commit on a registered arena waits for device writes queued on its stream;
  * concurrent routed callers; stream_forget.
"""
import ctypes
import threading

import numpy as np
import pytest

from oracle import oracle as o
from storm_amd import _lib, blocks, engine
from storm_amd import commit as sc

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

STORM_LENS = [72, 28808, 30000, 31808, 32768]
# rates that make the split the model's clear choice for large calls (a host slower than
# the link), frozen so that the routed calls below are deterministic
SLOW_HOST = dict(host_thread=2000.0, host_memory=8000.0, host_cached=8000.0, link_pinned=55000.0,
                 link_pageable=50000.0, link_inplace=50000.0)
SLOW_LINK = dict(host_thread=40000.0, host_memory=300000.0, host_cached=300000.0, link_pinned=100.0,
                 link_pageable=100.0, link_inplace=100.0)


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()
    engine.init(0)
    yield
    blocks.SetRouteRates(None)
    blocks.RouteDevices(None)


class Registered:
    """A page-aligned host buffer registered with the library (as the Go binding's
    NewHostArena makes cache.data)."""

    def __init__(self, nbytes):
        self.raw = np.zeros(nbytes + 4096, dtype=np.uint8)
        off = (-self.raw.ctypes.data) % 4096
        self.a = self.raw[off:off + nbytes]
        blocks.RegisterHostMemory(self.a)

    def close(self):
        blocks.UnregisterHostMemory(self.a)


def _filled(n, stride, seed, lens=None):
    reg = Registered(n * stride)
    rng = np.random.default_rng(seed)
    reg.a[:] = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    return reg


def test_split_fixed_boundaries_storm_lengths():
    n, stride = 4099, 32768
    lens = np.random.default_rng(1).choice(STORM_LENS, size=n).astype(np.uint32)
    reg = _filled(n, stride, 1)
    try:
        want = o.checksum_batch(reg.a, n, stride, lens=lens, threads=8)
        for d in (0, 1, 7, 2050, n - 1, n):
            got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, lens=lens, devices=[0], device_blocks=d)
            assert done == d and np.array_equal(got, want), d
    finally:
        reg.close()


def test_split_chunks_beyond_one_staging_buffer():
    """Device shares larger than the 256 MiB staging chunk, with lengths below the stride:
    every chunk the copy engine takes fits its staging buffer (rows are stride apart)."""
    n, stride = 12000, 32768  # 393 MB of rows
    lens = np.full(n, 31808, dtype=np.uint32)
    lens[::7] = 30000
    reg = _filled(n, stride, 12)
    try:
        want = o.checksum_batch(reg.a, n, stride, lens=lens, threads=8)
        for d in (n, n - 1, 9000):
            got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, lens=lens, device_blocks=d)
            assert done == d and np.array_equal(got, want), d
        bad = want.copy()
        bad[[5, n - 5]] ^= 9
        assert blocks.VerifyChecksumBatchSplit(reg.a, n, stride, bad, lens=lens, device_blocks=n) == (5, 2, n)
    finally:
        reg.close()


@pytest.mark.parametrize("stride,length", [(32768, 32768), (1024, 1000), (4096, 4096)])
def test_split_uniform_lengths(stride, length):
    n = 3001
    reg = _filled(n, stride, stride)
    try:
        want = o.checksum_batch(reg.a, n, stride, length)
        for d in (1, n // 3, n):
            got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, length, device_blocks=d)
            assert done == d and np.array_equal(got, want), (stride, d)
    finally:
        reg.close()


def test_split_short_test_tag_blocks():
    n, stride = 5000, 1024
    lens = np.random.default_rng(3).choice([256, 536, 728], size=n).astype(np.uint32)
    reg = _filled(n, stride, 3)
    try:
        want = o.checksum_batch(reg.a, n, stride, lens=lens)
        got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, lens=lens, device_blocks=2500)
        assert done == 2500 and np.array_equal(got, want)
    finally:
        reg.close()


@pytest.mark.parametrize("n", [1, 2, 3, 37])
def test_split_edge_shapes(n):
    """Ragged edges of a split: 1-3 blocks with every boundary, empty and sub-stripe blocks
    (0, 1, 7, 31 and 33 bytes beside storm's lengths), a base 8 bytes past a page (rows
    not 16-byte aligned), the device reading in place. Exact against the oracle."""
    stride = 4096
    reg = Registered(n * stride + 4096)
    try:
        reg.a[:] = np.random.default_rng(n).integers(0, 256, size=reg.a.size, dtype=np.uint8)
        view = reg.a[8:8 + n * stride]
        lens = np.array([[0, 1, 7, 31, 33, 4088, 2048][i % 7] for i in range(n)], dtype=np.uint32)
        want = o.checksum_batch(view, n, stride, lens=lens)
        assert int(want[0]) == 0xEF46DB3751D8E999  # XXH64 of no bytes
        for d in sorted({0, 1, n // 2, n - 1, n}):
            got, done = blocks.ChecksumBatchSplit(view, n, stride, lens=lens, device_blocks=d)
            assert done == d and np.array_equal(got, want), (n, d)
            bad = want.copy()
            bad[n - 1] ^= 1
            fb, nb, done = blocks.VerifyChecksumBatchSplit(view, n, stride, bad, lens=lens, device_blocks=d)
            assert (fb, nb, done) == (n - 1, 1, d), (n, d)
    finally:
        reg.close()


@pytest.mark.parametrize("seed", range(16))
def test_split_fuzz(seed):
    """Random splits against the oracle: block count, stride, per-block or uniform lengths
    (storm's and `-tags test` sizes, empty and sub-stripe ones), base offset, host threads,
    a fixed or balanced device share, and planted mismatches anywhere (verify: the lowest
    index and the count over both sides)."""
    rng = np.random.default_rng(1000 + seed)
    stride = int(rng.choice([1024, 4096, 32768]))
    n = int(rng.integers(1, 3000 if stride == 32768 else 9000))
    shift = int(rng.choice([0, 8, 16, 64]))
    reg = Registered(n * stride + 4096)
    try:
        reg.a[:] = rng.integers(0, 256, size=reg.a.size, dtype=np.uint8)
        view = reg.a[shift:shift + n * stride]
        pool = [x for x in STORM_LENS + [0, 1, 31, 256, 536, 728] if x <= stride]
        lens = rng.choice(pool, size=n).astype(np.uint32) if rng.random() < 0.7 else None
        length = None if lens is not None else int(rng.choice([x for x in pool if x > 0]))
        want = o.checksum_batch(view, n, stride, length or 0, lens=lens)
        d = None if rng.random() < 0.4 else int(rng.integers(0, n + 1))
        threads = int(rng.choice([0, 1, 3]))
        got, done = blocks.ChecksumBatchSplit(view, n, stride, length, lens=lens, host_threads=threads,
                                              device_blocks=d)
        assert np.array_equal(got, want) and (d is None or done == d) and done <= n, (seed, n, d)
        bad = want.copy()
        planted = sorted(set(int(i) for i in rng.integers(0, n, size=int(rng.integers(0, 5)))))
        for i in planted:
            bad[i] ^= 1 << int(rng.integers(0, 64))
        fb, nb, done = blocks.VerifyChecksumBatchSplit(view, n, stride, bad, length, lens=lens,
                                                       host_threads=threads, device_blocks=d)
        assert (fb, nb) == ((planted[0], len(planted)) if planted else (n, 0)), (seed, planted, fb, nb)
    finally:
        reg.close()


def test_split_verify_mismatches_on_each_side_of_the_boundary():
    n, stride, d = 3000, 32768, 1000
    edge = n - d  # host: [0, edge), device: [edge, n)
    lens = np.random.default_rng(4).choice(STORM_LENS, size=n).astype(np.uint32)
    reg = _filled(n, stride, 4)
    try:
        want = o.checksum_batch(reg.a, n, stride, lens=lens, threads=8)
        for planted, expect in (([], (n, 0)), ([edge - 1, edge], (edge - 1, 2)), ([edge, n - 1], (edge, 2)),
                                ([5], (5, 1)), ([n - 1], (n - 1, 1)), ([0, edge - 1, edge, n - 1], (0, 4))):
            bad = want.copy()
            for i in planted:
                bad[i] ^= 1 << 17
            fb, nb, done = blocks.VerifyChecksumBatchSplit(reg.a, n, stride, bad, lens=lens, device_blocks=d)
            assert (fb, nb) == expect and done == d, planted
    finally:
        reg.close()


def test_split_balanced_and_listed_twice():
    n, stride = 16384, 32768  # 512 MiB
    reg = Registered(n * stride)
    try:
        reg.a[:] = engine_fill(n, stride)
        want = o.checksum_batch(reg.a, n, stride, stride, threads=8)
        blocks.SetRouteRates(SLOW_HOST, freeze=True)  # the devices' share is then most of the batch
        got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, stride)
        assert np.array_equal(got, want) and 0 < done <= n, done
        got, done2 = blocks.ChecksumBatchSplit(reg.a, n, stride, stride, devices=[0, 0])
        assert np.array_equal(got, want) and 0 < done2 <= n
        blocks.SetRouteRates(None)  # learning, from the priors: any share, always exact
        for _ in range(3):
            got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, stride)
            assert np.array_equal(got, want) and done <= n
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def engine_fill(n, stride):
    t = torch.empty((n, stride), dtype=torch.uint8, device="cuda")
    engine.fill_synthetic_device(t.data_ptr(), stride, n, 0, o.SYNTH_SEED)
    return t.cpu().numpy().reshape(-1)


def test_routed_batch_takes_the_split_when_the_model_says_so():
    n, stride = 8192, 32768
    lens = np.random.default_rng(6).choice(STORM_LENS, size=n).astype(np.uint32)
    reg = _filled(n, stride, 6)
    pageable = reg.a.copy()
    try:
        want = o.checksum_batch(reg.a, n, stride, lens=lens, threads=8)
        blocks.SetRouteRates(SLOW_HOST, freeze=True)
        got, leg = blocks.ChecksumBatchLeg(reg.a, n, stride, lens=lens)
        assert leg == _lib.LEG_SPLIT and np.array_equal(got, want)
        bad = want.copy()
        bad[[10, n - 10]] ^= 3
        assert blocks.VerifyChecksumBatchLeg(reg.a, n, stride, bad, lens=lens) == (10, 2, _lib.LEG_SPLIT)
        # pageable memory never splits (the device would need host copies): the device leg here
        got, leg = blocks.ChecksumBatchLeg(pageable, n, stride, lens=lens)
        assert leg == _lib.LEG_DEVICE and np.array_equal(got, want)
        blocks.SetRouteRates(SLOW_LINK, freeze=True)
        got, leg = blocks.ChecksumBatchLeg(reg.a, n, stride, lens=lens)
        assert leg == _lib.LEG_HOST and np.array_equal(got, want)
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_split_refuses_pageable_and_device_memory():
    buf = np.zeros(4 * 64, dtype=np.uint8)
    out = np.zeros(4, dtype=np.uint64)
    rc = _lib.lib.stormck_checksum_split(buf.ctypes.data, 64, None, 64, 4, out.ctypes.data, None, 0, 0,
                                         _lib.SPLIT_BALANCED, None)
    assert rc == _lib.EINVAL and "pinned or registered" in _lib.last_error()
    t = torch.zeros((4, 64), dtype=torch.uint8, device="cuda")
    rc = _lib.lib.stormck_checksum_split(t.data_ptr(), 64, None, 64, 4, out.ctypes.data, None, 0, 0,
                                         _lib.SPLIT_BALANCED, None)
    assert rc == _lib.EINVAL and "device memory" in _lib.last_error()


def _commit_case(n_leaves, seed, fanout=1200, slot=32768):
    rng = np.random.default_rng(seed)
    lens = rng.choice(STORM_LENS[1:], size=n_leaves)
    b, size, last = sc.pointer_forest(n_leaves, lens, fanout, slot=slot, revision=9, first_address=100)
    b["birth_revision"][rng.random(len(b)) < 0.4] = 3  # relocations
    perm = rng.permutation(len(b))  # the caller's record order is arbitrary
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(b))
    bp = b[perm].copy()
    has = bp["parent"] >= 0
    bp["parent"][has] = inv[bp["parent"][has]]
    reg = Registered(size)
    reg.a[slot:slot + n_leaves * slot] = rng.integers(0, 256, size=n_leaves * slot, dtype=np.uint8)
    ref_arena = reg.a.copy()
    ref_b = bp.copy()
    ref_cs, ref_last = o.commit(ref_arena, ref_b, 9, last)
    return bp, reg, last, (ref_cs, ref_b, ref_last, ref_arena)


@pytest.mark.parametrize("device_leaves", [0, 1, 1500, 2999, 3000])
def test_commit_split_fixed_matches_storm_loop(device_leaves):
    b, reg, last, (ref_cs, ref_b, ref_last, ref_arena) = _commit_case(3000, device_leaves + 1)
    try:
        cs, last2, done = sc.commit_split(reg.a, b, 9, last, devices=[0], device_leaves=device_leaves)
        assert done == device_leaves
        assert np.array_equal(cs, ref_cs) and last2 == ref_last and np.array_equal(b, ref_b)
        assert np.array_equal(reg.a, ref_arena)  # every Pointer and type stored into its parent
    finally:
        reg.close()


@pytest.mark.parametrize("n_leaves,device_leaves", [(1, 0), (1, 1), (2, 1), (2, 2), (1201, 1201)])
def test_commit_split_tiny_and_two_node_forests(n_leaves, device_leaves):
    """The smallest forests (one leaf alone; two leaves under a pointer block) with the
    boundary at each place, and 1,201 leaves (two pointer blocks and their root) all on the
    device."""
    b, reg, last, (ref_cs, ref_b, ref_last, ref_arena) = _commit_case(n_leaves, 100 + n_leaves + device_leaves)
    try:
        cs, last2, done = sc.commit_split(reg.a, b, 9, last, devices=[0], device_leaves=device_leaves)
        assert done == device_leaves
        assert np.array_equal(cs, ref_cs) and last2 == ref_last and np.array_equal(b, ref_b)
        assert np.array_equal(reg.a, ref_arena)
    finally:
        reg.close()


@pytest.mark.parametrize("seed", range(8))
def test_commit_split_fuzz(seed):
    """Random forests through the split commit against storm's loop (the oracle): leaf
    count, fan-out (deeper trees at small fan-outs), relocations, record order, host
    threads, and a fixed or balanced leaf share."""
    rng = np.random.default_rng(2000 + seed)
    n_leaves = int(rng.integers(1, 5000))
    fanout = int(rng.choice([10, 100, 1200]))
    b, reg, last, (ref_cs, ref_b, ref_last, ref_arena) = _commit_case(n_leaves, 3000 + seed, fanout=fanout)
    try:
        d = None if rng.random() < 0.4 else int(rng.integers(0, n_leaves + 1))
        threads = int(rng.choice([0, 1, 3]))
        cs, last2, done = sc.commit_split(reg.a, b, 9, last, host_threads=threads, device_leaves=d)
        assert d is None or done == d
        assert np.array_equal(cs, ref_cs) and last2 == ref_last and np.array_equal(b, ref_b), (seed, n_leaves, d)
        assert np.array_equal(reg.a, ref_arena)
    finally:
        reg.close()


@pytest.mark.parametrize("seed", range(8))
def test_routed_fuzz(seed):
    """The routed batch, verify and commit on random shapes under rates that force each
    leg (a slow host: device or split; a slow link: host; the measured priors: any):
    always exact, whichever leg runs."""
    rng = np.random.default_rng(4000 + seed)
    rates = [SLOW_HOST, SLOW_LINK, None][seed % 3]
    n, stride = int(rng.integers(1, 6000)), 32768
    lens = rng.choice(STORM_LENS, size=n).astype(np.uint32)
    reg = _filled(n, stride, 5000 + seed)
    try:
        blocks.SetRouteRates(rates, freeze=rates is not None)
        want = o.checksum_batch(reg.a, n, stride, lens=lens, threads=8)
        got, leg = blocks.ChecksumBatchLeg(reg.a, n, stride, lens=lens, host_threads=int(rng.choice([0, 1])))
        assert np.array_equal(got, want) and leg in (_lib.LEG_HOST, _lib.LEG_DEVICE, _lib.LEG_SPLIT)
        if rates is SLOW_LINK:
            assert leg == _lib.LEG_HOST
        bad = want.copy()
        k = int(rng.integers(0, n))
        bad[k] ^= 2
        fb, nb, leg = blocks.VerifyChecksumBatchLeg(reg.a, n, stride, bad, lens=lens)
        assert (fb, nb) == (k, 1), (seed, k, fb, nb, leg)
    finally:
        blocks.SetRouteRates(None)
        reg.close()
    b, reg, last, (ref_cs, ref_b, ref_last, ref_arena) = _commit_case(int(rng.integers(1, 4000)), 6000 + seed)
    try:
        blocks.SetRouteRates(rates, freeze=rates is not None)
        cs, last2, leg = sc.commit(reg.a.ctypes.data, b, 9, last, host_threads=int(rng.choice([0, 1])))
        assert leg in (_lib.LEG_HOST, _lib.LEG_DEVICE, _lib.LEG_SPLIT)
        assert np.array_equal(cs, ref_cs) and last2 == ref_last and np.array_equal(b, ref_b), (seed, leg)
        assert np.array_equal(reg.a, ref_arena)
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_routed_commit_takes_the_split_and_matches():
    b, reg, last, (ref_cs, ref_b, ref_last, ref_arena) = _commit_case(6000, 77)
    try:
        blocks.SetRouteRates(SLOW_HOST, freeze=True)
        cs, last2, leg = sc.commit(reg.a.ctypes.data, b, 9, last)
        assert leg == _lib.LEG_SPLIT
        assert np.array_equal(cs, ref_cs) and last2 == ref_last and np.array_equal(b, ref_b)
        assert np.array_equal(reg.a, ref_arena)
        cs2, _, done = sc.commit_split(reg.a, ref_b.copy(), 9, ref_last)  # a second, balanced run
        assert done > 0
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_routed_commit_waits_for_device_writes_on_its_stream():
    """the host leg must not read a registered arena before device work the
    caller queued on `stream` lands. A kernel on a side stream writes every leaf of the
    arena in place over PCIe, and the routed commit (host leg: frozen rates with a slow
    link) is called right behind it on that stream."""
    n_leaves, slot = 4096, 32768
    b, size, last = sc.pointer_forest(n_leaves, 32768, 1200, slot=slot, revision=1)
    reg = Registered(size)
    try:
        d_arena = blocks.HostDevicePointer(reg.a)
        s = torch.cuda.Stream()
        blocks.SetRouteRates(SLOW_LINK, freeze=True)
        engine.fill_synthetic_device(d_arena + slot, slot, n_leaves, 0, o.SYNTH_SEED, s.cuda_stream)
        cs, last2, leg = sc.commit(reg.a.ctypes.data, b, 1, last, stream=s.cuda_stream)
        assert leg == _lib.LEG_HOST
        ref = np.zeros(size, dtype=np.uint8)
        ref[slot:slot + n_leaves * slot] = o.fill_synthetic(n_leaves, slot).reshape(-1)
        b_ref, _, _ = sc.pointer_forest(n_leaves, 32768, 1200, slot=slot, revision=1)
        ref_cs, _ = o.commit(ref, b_ref, 1, last)
        assert np.array_equal(cs, ref_cs)
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_concurrent_routed_batches():
    """Two callers at once (Go goroutines calling ChecksumBatch): each gets its own exact
    result whichever legs they take; a caller that finds the pool busy plans on its own
    thread."""
    n, stride = 8192, 32768
    regs = [_filled(n, stride, 40 + k) for k in range(2)]
    try:
        wants = [o.checksum_batch(r.a, n, stride, stride, threads=8) for r in regs]
        results = [None, None]

        def call(k):
            outs = []
            for _ in range(3):
                outs.append(blocks.ChecksumBatchLeg(regs[k].a, n, stride, stride))
            results[k] = outs

        ts = [threading.Thread(target=call, args=(k,)) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for k in range(2):
            for got, leg in results[k]:
                assert leg in (_lib.LEG_HOST, _lib.LEG_DEVICE, _lib.LEG_SPLIT)
                assert np.array_equal(got, wants[k]), k
    finally:
        for r in regs:
            r.close()


def test_route_devices_and_rates_learned_on_the_gpu():
    blocks.RouteDevices([0, 0])  # listed twice: once
    blocks.RouteDevices(None)
    with pytest.raises(_lib.StormckError):
        blocks.RouteDevices([99])
    # a device leg of >= 64 MiB measures the link
    n, stride = 4096, 32768  # 128 MiB
    reg = _filled(n, stride, 9)
    try:
        # the device leg is the model's choice (a 1-byte/us host), the link prior far too low
        blocks.SetRouteRates(dict(SLOW_HOST, link_pinned=1000.0, link_inplace=1000.0, host_thread=1.0,
                                  host_memory=1.0, host_cached=1.0))
        got, leg = blocks.ChecksumBatchLeg(reg.a, n, stride, stride, host_threads=1)
        assert leg == _lib.LEG_DEVICE
        r = blocks.RouteRates()
        assert r["observations"] >= 1 and r["link_pinned"] > 5000.0, r
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_split_latency_learning_is_bounded():
    """A split's device part measures the devices' start latency, and one observation moves
    it up by at most a quarter of (itself + 100 us): a one-off spike (the process's first
    kernel launches loading their code) must not price the device out of every later
    split, since a device that gets no chunk is never measured again."""
    n, stride = 512, 32768  # 16 MiB: first chunks within the latency probe's size
    reg = _filled(n, stride, 11)
    want = o.checksum_batch(reg.a, n, stride, stride)
    try:
        blocks.SetRouteRates(dict(SLOW_HOST, device_latency=10.0))  # learning
        lat = 10.0
        for _ in range(3):
            got, done = blocks.ChecksumBatchSplit(reg.a, n, stride, stride)
            assert np.array_equal(got, want)
            assert done > 0
            r = blocks.RouteRates()
            assert 1.0 <= r["device_latency"] <= lat + 0.25 * (lat + 100.0) + 1e-6, (lat, r)
            lat = r["device_latency"]
    finally:
        blocks.SetRouteRates(None)
        reg.close()


def test_stream_forget():
    s = torch.cuda.Stream()
    n, stride = 1024, 32768  # a ring-eligible batch (k_xxh64_wide_multi)
    t = torch.zeros((n, stride), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    engine.checksum_device(t.data_ptr(), stride, n, out.data_ptr(), stride, stream=s.cuda_stream, check_status=False)
    engine.stream_forget(s.cuda_stream)
    engine.stream_forget(s.cuda_stream)  # a stream with no slot: nothing to do
    torch.cuda.synchronize()
    assert int(out[0]) & ((1 << 64) - 1) == o.xxh64(bytes(stride))


def test_routed_batch_on_managed_memory():
    """hipMallocManaged memory has no hipHostGetDevicePointer mapping, so it is
    classified as DMA-able host memory (the copy engine), not as registered memory the
    kernels read in place. The routed batch forced onto the split (a slow host, frozen) and
    the split leg with a fixed share hash it exactly."""
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch and the library share
    n, stride = 2048, 32768
    p = ctypes.c_void_p()
    if hip.hipMallocManaged(ctypes.byref(p), ctypes.c_size_t(n * stride), ctypes.c_uint(1)) != 0 or not p.value:
        pytest.skip("hipMallocManaged not available on this device")
    try:
        a = np.ctypeslib.as_array((ctypes.c_uint8 * (n * stride)).from_address(p.value))
        a[:] = np.random.default_rng(77).integers(0, 256, size=n * stride, dtype=np.uint8)
        want = o.checksum_batch(a, n, stride, stride, threads=8)
        blocks.SetRouteRates(SLOW_HOST, freeze=True)
        got, leg = blocks.ChecksumBatchLeg(a, n, stride, stride)
        assert leg in (_lib.LEG_SPLIT, _lib.LEG_DEVICE) and np.array_equal(got, want), leg
        got, done = blocks.ChecksumBatchSplit(a, n, stride, stride, devices=[0], device_blocks=n // 2)
        assert done == n // 2 and np.array_equal(got, want)
    finally:
        blocks.SetRouteRates(None)
        hip.hipFree(p)


def test_fixed_splits_over_reversed_device_lists_finish():
    """two fixed-mode splits at once over the same two devices listed in
    opposite orders take the device workers in one global order, so neither waits for a
    worker the other holds. Skipped on a one-GPU box (a device listed twice is listed once)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("one visible device")
    n, stride = 4096, 32768
    regs = [_filled(n, stride, 90 + k) for k in range(2)]
    try:
        wants = [o.checksum_batch(r.a, n, stride, stride, threads=8) for r in regs]
        errors = []

        def call(k):
            try:
                for _ in range(10):
                    got, done = blocks.ChecksumBatchSplit(regs[k].a, n, stride, stride, devices=[k, 1 - k],
                                                          device_blocks=n - 100)
                    assert done == n - 100 and np.array_equal(got, wants[k])
            except Exception as e:  # reported below
                errors.append(e)

        ts = [threading.Thread(target=call, args=(k,), daemon=True) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not any(t.is_alive() for t in ts), "fixed splits over reversed device lists did not finish"
        assert not errors, errors
    finally:
        for r in regs:
            r.close()
