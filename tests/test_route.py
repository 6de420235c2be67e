"""The routing model (CPU, no device): which leg a host-memory call takes, and how the
rates it decides with are measured at run time.

The routed entry points (stormck_checksum_batch / _verify_batch, stormck_commit: the Go
shim's ChecksumBatch, VerifyChecksumBatch and CommitBatch, which storm's Cache.Commit data
phase drives, /root/reference/cache/cache.go:87-137) run on the host threads, the
device(s) over PCIe, or both at once (the split leg). stormck_route_plan_batch /
_plan_commit expose the decision without a device, so these tests inject rates and check
the choice and the predicted times against the model's formulas (include/stormck.h,
"routing of host-memory work"). The learning tests run the host leg itself,
which needs no device, and watch the rates move.
"""
import math

import numpy as np
import pytest

from storm_amd import _lib, blocks
from storm_amd import commit as sc

RATES = dict(host_thread=40000.0, host_memory=180000.0, host_cached=180000.0, link_pinned=55000.0,
             link_pageable=50000.0, link_inplace=52000.0, device_latency=120.0)
LEVEL_US, CALL_US, CHAIN = 10.0, 16.0, 1600.0  # stormck.hip kHostLevelUs, kDevBatchCallUs, kDevChainBytesPerUs
POOL = 16
GIB8 = 262144  # 8 GiB of 32 KiB blocks


@pytest.fixture
def rates():
    """Freeze the model at RATES (overridable per test); restore the priors after."""
    def set_(**kw):
        r = dict(RATES)
        r.update(kw)
        blocks.SetRouteRates(r, freeze=True)
        return r
    set_()
    yield set_
    blocks.SetRouteRates(None)


def _cpus():
    # the CPUs the library counts (stormck.hip ForkJoin::usable_cpus): the affinity mask,
    # capped by a cgroup v2 CPU quota
    import os
    cpus = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cpus = min(cpus, max(1, int(int(q) / int(per) + 0.5)))
    except (OSError, ValueError):
        pass
    return cpus


def _pool():
    # the library pool: min(16, usable CPUs)
    return min(16, _cpus())


def _split_threads(k):
    # host threads beside k device workers (stormck.hip split_threads)
    pool, cpus = _pool(), _cpus()
    return pool if pool + k <= cpus else max(1, cpus - k if cpus > k else 1)


def test_rates_set_get_and_priors(rates):
    got = blocks.RouteRates()
    for k, v in RATES.items():
        assert got[k] == v, k
    assert got["observations"] == 0
    blocks.SetRouteRates(None)
    pri = blocks.RouteRates()
    assert pri["host_memory"] == 180000.0 and pri["host_cached"] == 180000.0
    assert pri["link_pinned"] == 55000.0 and pri["link_inplace"] == 50000.0
    assert pri["device_latency"] == 150.0
    assert pri["host_thread"] in (24000.0, 48000.0)  # scalar / AVX-512 four-block prior


def test_small_batches_stay_on_the_host(rates):
    for n, length in ((3, 31808), (100, 536), (1, 72)):
        leg, us = blocks.PlanBatch(n, 32768, length, pinned=True)
        assert leg == _lib.LEG_HOST, (n, length, us)
        assert us[0] < us[1]


def test_host_time_formula(rates):
    """bytes / min(threads x per-thread rate, the pool's cap) + fork/join; the cap of a
    pass of at most 64 MiB (cache-resident) is learned apart from larger passes'."""
    rates(host_cached=90000.0)
    n, L = 16384, 32768  # 512 MiB: the DRAM cap
    leg, us = blocks.PlanBatch(n, L, L, pinned=False, host_threads=4)
    assert us[0] == pytest.approx(n * L / min(4 * RATES["host_thread"], RATES["host_memory"]) + LEVEL_US)
    leg, us = blocks.PlanBatch(1024, L, L, pinned=False, host_threads=4)  # 32 MiB: the cache-sized cap
    assert us[0] == pytest.approx(1024 * L / min(4 * RATES["host_thread"], 90000.0) + LEVEL_US)
    leg, us = blocks.PlanBatch(n, L, L, pinned=False, host_threads=1)
    assert us[0] == pytest.approx(n * L / RATES["host_thread"])


def test_device_time_formula_pageable_and_pinned(rates):
    n, L = 16384, 32768
    B = n * L
    _, us = blocks.PlanBatch(n, L, L, pinned=False, host_threads=1)
    fill = min(B, 256 << 20) / 55000.0
    assert us[1] == pytest.approx(CALL_US + L / CHAIN + B / RATES["link_pageable"] + fill)
    assert math.isinf(us[2])  # pageable memory: no split (the devices would need host copies)
    _, us = blocks.PlanBatch(n, L, L, pinned=True, host_threads=1)
    assert us[1] == pytest.approx(CALL_US + L / CHAIN + B / RATES["link_pinned"])


def test_split_formula_and_choice(rates):
    """The split: (B + k r_d L) / (r_h + k r_d) + fork/join, with r_d the in-place link rate,
    L the devices' measured start latency and r_h the rate of the host threads the split
    leaves beside k device workers (one CPU each where the pool would take them all),
    taken when 5% faster than both single legs; more devices, more links."""
    L = 32768
    B = GIB8 * L
    lat = RATES["device_latency"]
    prev = None
    for k in (1, 2, 8):
        leg, us = blocks.PlanBatch(GIB8, L, L, pinned=True, n_devices=k)
        pl = _split_threads(k)  # the host threads a split leaves beside k device workers
        r_h = min(pl * RATES["host_thread"], RATES["host_memory"]) if pl > 1 else RATES["host_thread"]
        r_d = k * RATES["link_inplace"]
        want = (B + r_d * lat) / (r_h + r_d) + (LEVEL_US if pl > 1 else 0)
        assert us[2] == pytest.approx(want), k
        best = min(us[0], us[1])
        expect = _lib.LEG_SPLIT if us[2] < 0.95 * best and us[2] < best - 30 else \
            (_lib.LEG_DEVICE if us[1] < us[0] else _lib.LEG_HOST)
        assert leg == expect, (k, us)
        if k == 1:
            assert leg == _lib.LEG_SPLIT, us
        if prev is not None:
            assert us[2] < prev
        prev = us[2]


def test_no_device_means_host(rates):
    leg, us = blocks.PlanBatch(GIB8, 32768, 32768, pinned=True, n_devices=0)
    assert leg == _lib.LEG_HOST and math.isinf(us[1]) and math.isinf(us[2])


def test_one_host_thread_large_pageable_goes_to_the_device(rates):
    leg, us = blocks.PlanBatch(GIB8, 32768, 32768, pinned=False, host_threads=1)
    assert leg == _lib.LEG_DEVICE, us


def test_a_slow_link_keeps_everything_on_the_host(rates):
    rates(link_pinned=500.0, link_pageable=500.0, link_inplace=500.0)
    for pinned in (False, True):
        leg, us = blocks.PlanBatch(GIB8, 32768, 32768, pinned=pinned)
        assert leg == _lib.LEG_HOST, (pinned, us)


def test_the_split_must_save_a_margin(rates):
    """The split is taken only when predicted to save >= 5% of the best single leg and
    >= 30 us: a 1.5 MB batch whose split would save a few microseconds stays on the host."""
    rates(device_latency=1.0, host_cached=50000.0, host_thread=50000.0)
    leg, us = blocks.PlanBatch(48, 32768, 32768, pinned=True)
    assert math.isfinite(us[2]) and us[2] < 0.95 * us[0] and us[0] - us[2] < 30.0, us
    assert leg == _lib.LEG_HOST


def test_the_start_latency_keeps_short_calls_off_the_split(rates):
    """A split pays the devices' start latency before they return anything: with the pool,
    a c5-size batch (38 MB, ~200 us on the host) does not split when the latency is a large
    part of it, and does when it is small; with one host thread it splits either way."""
    c5 = [31808] * 1200 + [30000, 72]
    rates(device_latency=150.0, host_cached=400000.0)
    leg, us = blocks.PlanBatch(len(c5), 32768, lens=c5, pinned=True)
    if _pool() >= 8:
        assert leg == _lib.LEG_HOST, us
    leg, us = blocks.PlanBatch(len(c5), 32768, lens=c5, pinned=True, host_threads=1)
    assert leg == _lib.LEG_SPLIT, us
    rates(device_latency=1.0, host_cached=100000.0)
    leg, us = blocks.PlanBatch(len(c5), 32768, lens=c5, pinned=True)
    assert leg == _lib.LEG_SPLIT, us


def test_cache_sized_calls_split_only_on_a_wide_margin(rates):
    """A call of at most 64 MiB (storm's c5 commit batch, 38 MB) splits only when predicted
    20% faster than the best single leg: its host leg's rate swings 2x with the host's
    caches. A split predicted 17% faster stays on the pool; with one host thread the split
    is predicted ~2x faster and is taken; the same margin on a 128 MiB batch splits."""
    c5 = [31808] * 1200 + [30000, 72]
    rates(device_latency=40.0)
    leg, us = blocks.PlanBatch(len(c5), 32768, lens=c5, pinned=True)
    if _pool() > 1:
        assert 0.8 <= us[2] / us[0] < 0.95 and us[0] - us[2] >= 30, us
        assert leg == _lib.LEG_HOST, us
    leg, us = blocks.PlanBatch(len(c5), 32768, lens=c5, pinned=True, host_threads=1)
    assert leg == _lib.LEG_SPLIT and us[2] < 0.6 * us[0], us
    leg, us = blocks.PlanBatch(4096, 32768, 32768, pinned=True)
    if _pool() > 1:
        assert us[2] < 0.95 * us[0] and leg == _lib.LEG_SPLIT, us


def test_a_fast_host_makes_the_split_a_tie_and_keeps_the_host(rates):
    """When the link adds under 5% to the host's rate the split is not taken (no flapping
    between two legs of about the same time)."""
    rates(host_thread=400000.0, host_memory=4000000.0, host_cached=4000000.0)
    leg, us = blocks.PlanBatch(GIB8, 32768, 32768, pinned=True)
    if _pool() > 1:
        assert leg == _lib.LEG_HOST, us


def _forest(n_leaves, length=32768):
    b, size, last = sc.pointer_forest(n_leaves, length, 1200, slot=32768, revision=1)
    return b


def test_commit_plan(rates):
    big = _forest(131072)
    leg, us = sc.plan_commit(big, registered=True)
    assert leg == _lib.LEG_SPLIT and us[2] < 0.95 * min(us[0], us[1]), us
    leg, us = sc.plan_commit(big, registered=False)
    assert leg == _lib.LEG_HOST and math.isinf(us[1]) and math.isinf(us[2])
    leg, us = sc.plan_commit(big, registered=True, n_devices=0)
    assert leg == _lib.LEG_HOST
    three = _forest(2, 31808)
    leg, us = sc.plan_commit(three, registered=True)
    assert leg == _lib.LEG_HOST and us[0] < 20, us
    # the split only ever touches the leaves: its time is the host's minus the leaf height's gain
    assert us[2] == math.inf or us[2] < us[0]


def test_commit_plan_rejects_a_malformed_forest(rates):
    b = _forest(25)
    b["parent"][3] = 10 ** 6
    import ctypes
    leg = ctypes.c_uint32()
    assert _lib.lib.stormck_route_plan_commit(b.ctypes.data, len(b), 1, 0, 1, ctypes.byref(leg), None) == _lib.EINVAL


def _rows(n, stride, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n * stride, dtype=np.uint8)


def test_host_leg_measures_the_per_thread_rate():
    """A one-thread host leg of >= 8 MiB moves host_thread toward its observed rate
    (EWMA weight 1/4); a frozen model does not move."""
    n, stride = 512, 32768  # 16 MiB
    buf = _rows(n, stride, 3)
    r = dict(RATES, host_thread=1.0)
    blocks.SetRouteRates(r)  # learning
    try:
        blocks.ChecksumBatchHost(buf, n, stride, stride, threads=1)
        got = blocks.RouteRates()
        assert got["observations"] == 1
        assert got["host_thread"] > 1000.0  # 1 + (observed - 1) / 4, observed in GB/s
        assert got["host_memory"] == RATES["host_memory"] and got["host_cached"] == RATES["host_cached"]
        blocks.SetRouteRates(r, freeze=True)
        blocks.ChecksumBatchHost(buf, n, stride, stride, threads=1)
        assert blocks.RouteRates()["host_thread"] == 1.0
        # below 8 MiB nothing is learned
        blocks.SetRouteRates(r)
        blocks.ChecksumBatchHost(buf, 64, stride, stride, threads=1)
        assert blocks.RouteRates()["observations"] == 0
    finally:
        blocks.SetRouteRates(None)


def test_pool_pass_below_the_threads_rate_measures_the_pool_cap():
    if _pool() < 2:
        pytest.skip("one hardware thread")
    n, stride = 1024, 32768  # 32 MiB
    buf = _rows(n, stride, 4)
    blocks.SetRouteRates(dict(RATES, host_thread=1e9, host_memory=1.0, host_cached=1.0))
    try:
        blocks.ChecksumBatchHost(buf, n, stride, stride, threads=2)  # 32 MiB: the cache-sized cap
        got = blocks.RouteRates()
        assert got["observations"] == 1 and got["host_cached"] > 1000.0 and got["host_thread"] == 1e9
        assert got["host_memory"] == 1.0
    finally:
        blocks.SetRouteRates(None)


def test_tiny_calls_are_not_planned(rates):
    """A call one host thread finishes in under 10 us (kHostOnlyUs) takes the host leg on the
    caller's thread without planning (storm commits at least the singularity every revision,
    /root/reference/cache/cache.go:64-85): the plan entries report exactly that decision, the
    host time bytes / host_thread and no device or split time. Slow the host thread down and
    the same calls are planned again."""
    three = _forest(2, 31808)                       # 2 objectlist leaves + their pointer block
    tag = sc.pointer_forest(100, np.array([536, 728] * 50, dtype=np.uint32), 10, slot=32768, revision=1)[0]
    for forest in (three, tag):
        total = float(forest["length"].sum())
        assert total / RATES["host_thread"] < 10.0
        leg, us = sc.plan_commit(forest, registered=True)
        assert leg == _lib.LEG_HOST and us[0] == pytest.approx(total / RATES["host_thread"]), us
        assert math.isinf(us[1]) and math.isinf(us[2])
        leg, us = blocks.PlanBatch(len(forest), 32768, lens=list(forest["length"]), pinned=True)
        assert leg == _lib.LEG_HOST and us[0] == pytest.approx(total / RATES["host_thread"]) and math.isinf(us[1])
        rates(host_thread=total / 50.0)             # 50 us on one thread: planned
        leg, us = sc.plan_commit(forest, registered=True)
        assert math.isfinite(us[1]), us
        leg, us = blocks.PlanBatch(len(forest), 32768, lens=list(forest["length"]), pinned=True)
        assert math.isfinite(us[1]), us
        rates(host_thread=total / 10.0)             # exactly 10 us: planned (the bound is strict)
        leg, us = sc.plan_commit(forest, registered=True)
        assert math.isfinite(us[1]), us
        rates()
