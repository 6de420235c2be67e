"""storm's Cache.Commit through the stormck binding, against storm's own commit loop.

A simulated storm cache (oracle/storm_cache.py: cache/cache.go, cache/trace.go restated)
holds a committed tree of an earlier revision; a revision of updates then traces tags
through it (TraceTagForUpdating: existing leaves, new leaves under existing pointer
blocks, a released trace, a tree nested under a leaf). Two identical caches commit:

* A: storm's sequential commitData (cache.go:87-137: NReferences sweep, relocation,
  WriteBlock, PostCommitFunc, Data swap), visiting the dirty set in the library's order;
* B: the binding (storm_amd/commit.py commit_cache, the mirror of
  integration/go/cache/commit_stormck.go): the dirty forest as records, one
  level-synchronous commit, then relocations, the root pointer, writes and swaps.

B runs the records through the C oracle's commit here and through
stormck_commit_device on the GPU (tests/test_cache_commit.py -m gpu, arena in HBM and
in registered host memory). Every byte of the store, the singularity, cache.data and
every block's metadata must match A."""
import numpy as np
import pytest

from oracle import oracle as o
from oracle import storm_cache as sc
from storm_amd import commit as cm


def _workload(block_size, fanout, leaf_len, n_tree, n_slots, n_updates, seed):
    """A store holding a committed tree (revision 1) and a cache after one revision of
    updates (not yet committed)."""
    store = sc.Store(block_size, 1 << 20)
    sc.initialize(store)
    sc.build_tree(store, fanout, leaf_len, range(n_tree), 1, seed)
    c = sc.Cache(store, n_slots, fanout, leaf_len, seed=seed)
    rng = np.random.default_rng(seed + 1)
    span = fanout ** max(1, int(np.ceil(np.log(n_tree) / np.log(fanout))))  # tags of the tree's depth
    tags = rng.choice(span, size=n_updates, replace=False)
    for k, t in enumerate(tags):
        meta, trace, _ = c.trace_for_updating(c.space_origin(), None, int(t))
        if k % 17 == 5:
            trace.release()  # traced, not modified
            continue
        c.data[meta.data + 25:meta.data + leaf_len] = rng.integers(0, 256, leaf_len - 25, dtype=np.uint8)
        if k % 23 == 7:
            # a tree nested under this leaf (keystore-style): two new leaves in it
            for sub in (3, 3 + fanout):
                m2, t2, _ = c.trace_for_updating(c.leaf_child_origin(meta), trace, sub)
                c.data[m2.data + 25:m2.data + leaf_len] = rng.integers(0, 256, leaf_len - 25, dtype=np.uint8)
                t2.commit()
        trace.commit()
    return c


def _library_order(c):
    recs, metas, _ = cm.cache_records(c)
    h = cm.commit_heights(recs)
    key = {id(m): (int(h[i]), i) for i, m in enumerate(metas)}
    return lambda m: key[id(m)]


def _storm(c):
    c.commit(order_key=_library_order(c))
    return sc.snapshot(c)


def _binding(c, run):
    cm.commit_cache(c, run)
    c.finish_commit()
    return sc.snapshot(c)


def _oracle_run(c):
    return lambda recs, rev, last: o.commit(c.data, recs, rev, last)


SMALL = dict(block_size=1024, fanout=10, leaf_len=1000, n_tree=700, n_slots=4096, n_updates=240)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_binding_matches_storm_commit_loop(seed):
    a = _storm(_workload(seed=seed, **SMALL))
    c = _workload(seed=seed, **SMALL)
    b = _binding(c, _oracle_run(c))
    assert a["dirty"] == b["dirty"] == 0
    assert a["sing"] == b["sing"]
    assert a["store"] == b["store"]
    assert a["metas"] == b["metas"]
    assert a["data"] == b["data"]


def test_workload_exercises_relocation_new_blocks_and_nesting():
    c = _workload(seed=4, **SMALL)
    recs, metas, external = cm.cache_records(c)
    rev = c.revision()
    assert (recs["birth_revision"] <= rev).sum() > 0       # existing blocks: relocated on commit
    assert (recs["birth_revision"] > rev).sum() > 0        # new leaves (the Free case)
    assert (recs["type"] == cm.POINTER).sum() > 1           # pointer blocks above them
    assert len(external) == 1                               # the root hangs off the singularity
    h = cm.commit_heights(recs)
    assert h.max() >= 3                                     # nested tree under a leaf adds height
    assert any(m.commit_type == cm.LEAF for m in metas if m.commit_parent is not None
               and m.commit_parent.commit_type == cm.LEAF)  # a leaf whose parent is a leaf


def test_open_trace_is_refused_before_anything_changes():
    """A trace neither committed nor released keeps NReferences > 0: storm's sweep would
    spin forever (cache.go:88-90); the oracle stops, the binding refuses up front."""
    c = _workload(seed=5, **SMALL)
    c.trace_for_updating(c.space_origin(), None, 1)  # left open
    before = sc.snapshot(c)
    with pytest.raises(cm.StillReferenced):
        cm.commit_cache(c, _oracle_run(c))
    assert sc.snapshot(c) == before
    with pytest.raises(RuntimeError):
        c.commit()


# --- the host leg (stormck_commit_host): no device needed ----------------------------

def _host_leg_run(c, threads):
    """storm's cache.data committed where it lives by the library's host leg (the leg the
    routed CommitBatch takes for storm's per-revision commits, DESIGN_LOG §11 f1)."""
    def run(recs, rev, last):
        return cm.commit_host(c.data, recs, rev, last, threads=threads)
    return run


@pytest.mark.parametrize("threads", [1, 0])
def test_binding_host_leg_matches_storm_commit_loop(threads):
    a = _storm(_workload(seed=11, **SMALL))
    c = _workload(seed=11, **SMALL)
    b = _binding(c, _host_leg_run(c, threads))
    assert a["sing"] == b["sing"]
    assert a["store"] == b["store"]
    assert a["metas"] == b["metas"]
    assert a["data"] == b["data"]


# --- GPU: the same through stormck_commit_device -------------------------------------

torch = pytest.importorskip("torch")
PROD = dict(block_size=32768, fanout=1200, leaf_len=31808, n_tree=3000, n_slots=8192, n_updates=1500)


def _device_run(c, dev):
    """The arena in HBM: cache.data copied in, committed, copied back."""
    def run(recs, rev, last):
        arena = torch.from_numpy(c.data).to(dev)
        cs, last2 = cm.commit_device(arena.data_ptr(), recs, rev, last)
        c.data[:] = arena.cpu().numpy()
        return cs, last2
    return run


def _registered_run(c):
    """The arena where storm keeps it, in host memory: registered, the kernels read and
    write it in place over PCIe (blocks.CommitBatch over RegisterHostMemory in Go)."""
    from storm_amd import blocks

    def run(recs, rev, last):
        assert c.data.ctypes.data % 256 == 0  # rows at link rate (blocks.RegisterHostMemory)
        blocks.RegisterHostMemory(c.data)
        try:
            return cm.commit_device(blocks.HostDevicePointer(c.data), recs, rev, last)
        finally:
            blocks.UnregisterHostMemory(c.data)
    return run


@pytest.mark.gpu
@pytest.mark.parametrize("arena", ["hbm", "registered"])
def test_binding_on_gpu_matches_storm_commit_loop(arena):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    a = _storm(_workload(seed=11, **PROD))
    c = _workload(seed=11, **PROD)
    b = _binding(c, _device_run(c, dev) if arena == "hbm" else _registered_run(c))
    assert a["sing"] == b["sing"]
    assert a["store"] == b["store"]
    assert a["metas"] == b["metas"]
    assert a["data"] == b["data"]


def _routed_run(c, legs):
    """blocks.CommitBatch as the Go binding calls it: stormck_commit on the registered
    cache.data, which picks the leg (recorded in `legs`)."""
    from storm_amd import blocks

    def run(recs, rev, last):
        blocks.RegisterHostMemory(c.data)
        try:
            cs, last2, leg = cm.commit(c.data.ctypes.data, recs, rev, last)
        finally:
            blocks.UnregisterHostMemory(c.data)
        legs.append(leg)
        return cs, last2
    return run


@pytest.mark.gpu
def test_binding_routed_matches_storm_commit_loop():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    a = _storm(_workload(seed=11, **PROD))
    c = _workload(seed=11, **PROD)
    legs = []
    b = _binding(c, _routed_run(c, legs))
    assert legs and all(x in (_lib.LEG_HOST, _lib.LEG_DEVICE, _lib.LEG_SPLIT) for x in legs), legs
    assert a["sing"] == b["sing"]
    assert a["store"] == b["store"]
    assert a["metas"] == b["metas"]
    assert a["data"] == b["data"]


def _split_run(c, device_leaves, done):
    """stormck_commit_split on the registered cache.data: the leaves hashed by the host
    threads from the front and the device from the back at once (in place), the host
    threads storing every Pointer into its parent."""
    from storm_amd import blocks

    def run(recs, rev, last):
        blocks.RegisterHostMemory(c.data)
        try:
            cs, last2, d = cm.commit_split(c.data, recs, rev, last, device_leaves=device_leaves)
        finally:
            blocks.UnregisterHostMemory(c.data)
        done.append(d)
        return cs, last2
    return run


@pytest.mark.gpu
@pytest.mark.parametrize("device_leaves", [None, 7, 10 ** 9])
def test_binding_split_matches_storm_commit_loop(device_leaves):
    """The split commit through the binding's steps against the restated storm loop
    (oracle/storm_cache.py): store, singularity, cache.data and every block's metadata
    byte for byte, with the devices taking the rates' share, 7 leaves, or every leaf."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    a = _storm(_workload(seed=13, **PROD))
    c = _workload(seed=13, **PROD)
    done = []
    b = _binding(c, _split_run(c, device_leaves, done))
    assert done
    if device_leaves == 7:  # at most 7 (a commit with fewer leaves gives them all)
        assert all(d <= 7 for d in done) and 7 in done, done
    if device_leaves == 10 ** 9:
        assert all(d > 0 for d in done), done
    assert a["sing"] == b["sing"]
    assert a["store"] == b["store"]
    assert a["metas"] == b["metas"]
    assert a["data"] == b["data"]
