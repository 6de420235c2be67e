"""Full-size GPU checks of the secondary workloads against their libxxhash fixtures
(oracle/gen_golden.py), with the same inputs bench.py uses:

* f1: storm's Cache.Commit of 1M dirty 32 KiB leaves under fan-out-1200 pointer blocks
  (cache/cache.go:87-137) -- the commit's root, which covers every leaf and pointer;
* c5 (BASELINE.json configs[4]): the mixed batch of one keystore commit, and of one
  BenchmarkStorm commit (blob leaves, a spacelist block) -- every checksum (digest)
  and the root of the same leaves committed as a forest;
* f4: xxhash.Sum64 of 64M packed 48-byte keys (keystore/keystore.go:33,66) -- the
  digest of all tags.
"""
import numpy as np
import pytest

from tests.conftest import hx, load_golden

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from storm_amd import _lib
    assert _lib.device_count() > 0, "GPU visible to torch but libstormck finds no gfx950 device"
    return torch.device("cuda:0")


def _digest(t):
    from oracle import oracle as o
    return o.xxh64(t.cpu().numpy().view(np.uint64).astype("<u8"))


def test_f1_commit_1m_leaves_root(dev):
    from oracle import oracle as o
    from storm_amd import commit as sc
    from storm_amd import engine
    fx = load_golden("c3c4_roots.json")["f1_commit_1m"]
    n, slot, rev = fx["leaves"], 32768, 1
    b, size, last = sc.pointer_forest(n, slot, 1200, slot=slot, revision=rev)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + slot, slot, n, 0, o.SYNTH_SEED)
    torch.cuda.synchronize()
    cs, last2 = sc.commit_device(arena.data_ptr(), b, rev, last)
    assert last2 == last  # every block is new in this revision: nothing relocates
    assert int(cs[-1]) == hx(fx["root"][0])
    assert int(b["address"][-1]) == hx(fx["root"][1])


def test_c5_batch_and_commit(dev):
    from storm_amd import commit as sc
    from storm_amd import engine
    from oracle import oracle as o
    fx = load_golden("c5.json")
    lens = np.array([31808] * 1200 + [30000, 72], dtype=np.uint32)
    n = len(lens)
    buf = torch.empty((n, 32768), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), 32768, n, 0, o.SYNTH_SEED)
    out = engine.checksum_tensor(buf, lens=torch.from_numpy(lens.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    assert _digest(out) == hx(fx["batch_digest"])
    b0, size, last = sc.pointer_forest(1200, 31808, 1200, slot=32768, revision=1)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + 32768, 32768, 1200, 0, o.SYNTH_SEED)
    torch.cuda.synchronize()
    cs, _ = sc.commit_device(arena.data_ptr(), b0, 1, last)
    assert int(cs[-1]) == hx(fx["commit_root"])
    assert np.array_equal(cs[:1200], out[:1200].cpu().numpy().view(np.uint64))


def test_c5_storm_mix_batch_and_commit(dev):
    """c5, BenchmarkStorm's mix (/root/reference/benchmark_test.go): 1200 blob leaves of
    32,768 B, a 28,808 B spacelist block, the pointer block and the singularity, as
    bench.py --workload c5 --c5-mix storm runs it."""
    from storm_amd import commit as sc
    from storm_amd import engine
    from oracle import oracle as o
    fx = load_golden("c5.json")["storm"]
    lens = np.array([32768] * 1200 + [28808, 30000, 72], dtype=np.uint32)
    n = len(lens)
    buf = torch.empty((n, 32768), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(buf.data_ptr(), 32768, n, 0, o.SYNTH_SEED)
    out = engine.checksum_tensor(buf, lens=torch.from_numpy(lens.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    assert _digest(out) == hx(fx["batch_digest"])
    b0, size, last = sc.pointer_forest(1200, 32768, 1200, slot=32768, revision=1)
    arena = torch.zeros(size, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr() + 32768, 32768, 1200, 0, o.SYNTH_SEED)
    torch.cuda.synchronize()
    cs, _ = sc.commit_device(arena.data_ptr(), b0, 1, last)
    assert int(cs[-1]) == hx(fx["commit_root"])
    assert np.array_equal(cs[:1200], out[:1200].cpu().numpy().view(np.uint64))


def test_f4_64m_key_tags(dev):
    from storm_amd import engine
    from oracle import oracle as o
    fx = load_golden("keytags.json")
    n, klen = fx["keys"], fx["key_bytes"]
    keys = torch.empty(n * klen, dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(keys.data_ptr(), 48 * 1024, n * klen // (48 * 1024), 0, o.SYNTH_SEED)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    engine.key_tags_device(keys.data_ptr(), n, out.data_ptr(), stride=klen, length=klen)
    torch.cuda.synchronize()
    tags = out.cpu().numpy().view(np.uint64)
    assert [int(v) for v in tags[::1 << 20]] == [hx(v) for v in fx["every_1048576th"]]
    assert o.xxh64(tags.astype("<u8")) == hx(fx["digest"])
