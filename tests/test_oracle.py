"""Pin the oracle (CPU restatements) against the golden fixtures — CPU only.

The fixtures are libxxhash 0.8.2 outputs (oracle/gen_golden.py) plus the public
XXH64 known answers; storm's hash is xxhash.Sum64 = XXH64 seed 0
(/root/reference/blocks/checksum.go:16, go.mod:6).
"""
import numpy as np
import pytest

from oracle import oracle as o
from tests.conftest import hx, load_golden


def test_public_known_answers():
    kat = load_golden("kat.json")
    for s, v in kat["public"].items():
        assert o.xxh64(s.encode()) == hx(v)
        assert o.xxh64_py(s.encode()) == hx(v)


@pytest.mark.parametrize("pattern", ["zeros", "iota"])
def test_kat_lengths(pattern):
    for row in load_golden("kat.json")["rows"]:
        n = row["len"]
        data = bytes(n) if pattern == "zeros" else bytes(i & 0xFF for i in range(n))
        assert o.xxh64(data) == hx(row[pattern]), n
        if n <= 1000:
            assert o.xxh64_py(data) == hx(row[pattern]), n


def test_generator_samples():
    g = load_golden("synth_c1.json")
    for s in g["generator_samples"]:
        assert o.lib.oracle_synth_word(hx(g["seed"]), s["block"], s["word"]) == hx(s["value"])


def test_synth_c1_checksums():
    g = load_golden("synth_c1.json")
    n, stride = g["n"], g["stride"]
    buf = o.fill_synthetic(n, stride, 0, hx(g["seed"]))
    cs = o.checksum_batch(buf, n, stride, g["length"])
    assert [int(v) for v in cs] == [hx(v) for v in g["checksums"]]
    assert o.xxh64(cs.astype("<u8").tobytes()) == hx(g["digest"])
    # multi-threaded baseline path agrees
    assert np.array_equal(o.checksum_batch(buf, n, stride, g["length"], threads=4), cs)


def test_mixed_lengths():
    g = load_golden("mixed.json")
    lens = g["lens"]
    n, stride = len(lens), g["stride"]
    buf = o.fill_synthetic(n, stride, g["first"], hx(g["seed"]))
    cs = o.checksum_batch(buf, n, stride, lens=lens)
    assert [int(v) for v in cs] == [hx(v) for v in g["checksums"]]


def test_merkle_cases():
    g = load_golden("merkle.json")
    for c in g["cases"]:
        leaf = o.synth_leaf_checksums(c["n"], hx(g["seed"]))
        root = o.merkle_root(leaf, c["leaf_addr_base"], c["node_addr_base"], c["rev"], c["fanout"])
        assert root[:3] == tuple(hx(v) for v in c["root"]), c["n"]
        assert root[3] == c["root_type"], c["n"]


def test_merkle_combine():
    from storm_amd import dist
    g = load_golden("merkle.json")["combine"]
    leaf = o.synth_leaf_checksums(g["n_total"])
    table = []
    for r in range(g["world"]):
        lo, hi = dist.shard_range(g["n_total"], g["world"], r)
        table.append(o.merkle_root(leaf[lo:hi], lo, dist.shard_node_addr_base(g["n_total"], lo), g["rev"], g["fanout"]))
    assert [list(t[:3]) for t in table] == [[hx(v) for v in row[:3]] for row in g["shard_roots"]]
    groot = o.combine_roots(table, g["rev"], dist.global_root_addr(g["n_total"]), g["fanout"])
    assert list(groot[:3]) == [hx(v) for v in g["global_root"][:3]]
    assert groot[3] == g["global_root"][3]


def test_pointer_block_pack_matches_python():
    entries = [(i * 3 + 1, 1000 + i, 7, 2) for i in range(10)]
    b = o.pack_pointer_block_py(entries, 10)
    assert len(b) == 256 == o.pointer_block_size(10)
    assert o.pointer_block_size(1200) == 30000
    leaf = np.array([e[0] for e in entries], dtype=np.uint64)
    root = o.merkle_root(leaf, 1000, 5000, 7, 10)
    assert root == (o.xxh64_py(b), 5000, 7, 1)


def test_c5_fixture_against_oracle():
    """tests/golden/c5.json (libxxhash) = the C oracle on the same synthetic batch, and
    the commit root = the oracle's packer + XXH64 over the leaves' pointers."""
    import numpy as np
    from oracle import oracle as o
    g = load_golden("c5.json")
    lens = [31808] * 1200 + [30000, 72]
    buf = o.fill_synthetic(len(lens), 32768, 0)
    cs = o.checksum_batch(buf, len(lens), 32768, lens=lens, threads=8)
    assert o.xxh64(cs.astype("<u8")) == hx(g["batch_digest"])
    leaf = [(int(cs[i]), 1 + i, 2, 2) for i in range(1200)]
    assert o.xxh64(o.pack_pointer_block_py(leaf, 1200)) == hx(g["commit_root"])
    # the BenchmarkStorm mix: blob leaves and a spacelist block join the commit
    gs = g["storm"]
    lens = [32768] * 1200 + [28808, 30000, 72]
    buf = o.fill_synthetic(len(lens), 32768, 0)
    cs = o.checksum_batch(buf, len(lens), 32768, lens=lens, threads=8)
    assert o.xxh64(cs.astype("<u8")) == hx(gs["batch_digest"])
    assert [int(v) for v in cs[-3:]] == [hx(v) for v in gs["last3"]]
    leaf = [(int(cs[i]), 1 + i, 2, 2) for i in range(1200)]
    assert o.xxh64(o.pack_pointer_block_py(leaf, 1200)) == hx(gs["commit_root"])


def test_keytags_fixture_samples_against_oracle():
    """tests/golden/keytags.json samples (every 1,048,576th of 64M packed 48-byte keys)
    = the C oracle on the same synthetic bytes."""
    import numpy as np
    from oracle import oracle as o
    g = load_golden("keytags.json")
    for s, want in enumerate(g["every_1048576th"]):
        key = s << 20  # key index; 1024 keys per 48 KiB synthetic block
        blk = o.fill_synthetic(1, 48 * 1024, key // 1024)
        off = (key % 1024) * 48
        assert o.xxh64(blk[off:off + 48]) == hx(want), s
