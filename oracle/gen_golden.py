"""Generate the golden fixtures under tests/golden/ (run in the build container only).

ORACLE / TEST INFRASTRUCTURE. The checksum values come from python-xxhash 3.8.1
(bundled libxxhash 0.8.2) — the canonical XXH64 implementation, independent of
both the C restatement (oracle/xxh64_oracle.c) and the HIP kernels. storm's own
hash is github.com/cespare/xxhash/v2 v2.2.0 Sum64 (/root/reference/go.mod:6),
which is XXH64 seed 0; the Go reference cannot run here (no Go toolchain, SURVEY
§8c), and no reference test asserts an absolute checksum value, so
these fixtures plus the public XXH64 known answers are what pins parity.

Block contents, layouts and trees are rebuilt here with numpy/struct code of
this file alone (independent of oracle/oracle.py and storm_amd/).

    python oracle/gen_golden.py          # small fixtures (seconds)
    python oracle/gen_golden.py --big    # + 1M / 16M synthetic-block digests (minutes)
"""
from __future__ import annotations

import json
import os
import struct
import sys
import time

import numpy as np
import xxhash

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
SEED = 0x53544F524D
M64 = (1 << 64) - 1
STORM_LENGTHS = [72, 256, 536, 728, 28808, 30000, 31808, 32768]


def h(v: int) -> str:
    return "0x%016x" % v


def xx(b) -> int:
    return xxhash.xxh64_intdigest(bytes(b), seed=0)


def splitmix_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_blocks(first: int, n: int, stride: int, seed: int = SEED) -> np.ndarray:
    """word w of block i = splitmix64(seed ^ ((i << 20) + w))."""
    words = stride // 8
    i = np.arange(first, first + n, dtype=np.uint64)[:, None]
    w = np.arange(words, dtype=np.uint64)[None, :]
    key = np.uint64(seed) ^ ((i << np.uint64(20)) + w)
    return splitmix_np(key).astype("<u8").view(np.uint8).reshape(n, stride)


def write(name: str, obj) -> None:
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", path, os.path.getsize(path), "bytes")


# ---------------------------------------------------------------------------
def gen_kat() -> None:
    public = {"": 0xEF46DB3751D8E999, "a": 0xD24EC4F1A98C6E5B, "abc": 0x44BC2CF5AD770999}
    for s, v in public.items():
        assert xx(s.encode()) == v, s  # published XXH64 answers agree with libxxhash
    lengths = list(range(0, 129)) + STORM_LENGTHS + [1000, 4096, 32767, 32769, 65536]
    rows = []
    for n in lengths:
        zeros = bytes(n)
        iota = bytes(i & 0xFF for i in range(n))
        rows.append({"len": n, "zeros": h(xx(zeros)), "iota": h(xx(iota))})
    write("kat.json", {
        "source": "libxxhash 0.8.2 via python-xxhash 3.8.1, XXH64 seed 0",
        "public": {k: h(v) for k, v in public.items()},
        "patterns": {"zeros": "n zero bytes", "iota": "byte i = i & 0xff"},
        "rows": rows,
    })


def gen_synth_c1() -> None:
    n, stride = 1024, 32768
    blocks = synth_blocks(0, n, stride)
    cs = np.array([xx(blocks[i]) for i in range(n)], dtype=np.uint64)
    samples = []
    for (i, w) in [(0, 0), (0, 1), (1, 0), (7, 4095), (1023, 17), (1023, 4095)]:
        samples.append({"block": i, "word": w, "value": h(int(blocks[i].view("<u8")[w]))})
    write("synth_c1.json", {
        "config": "c1: 1K x 32 KiB synthetic blocks (BASELINE.json configs[0] restated)",
        "rule": "word w of block i = splitmix64(seed ^ ((i << 20) + w)), little-endian",
        "seed": h(SEED), "n": n, "stride": stride, "length": stride,
        "checksums": [h(int(v)) for v in cs],
        "digest": h(xx(cs.astype("<u8").tobytes())),
        "generator_samples": samples,
    })


def mixed_lengths() -> list:
    # config c5: objectlist / pointer / singularity / blob / spacelist lengths plus the
    # test-tag sizes and odd lengths that exercise every tail path.
    mix = [31808] * 24 + [30000, 72, 32768, 28808, 256, 536, 728] + \
          [0, 1, 3, 4, 7, 8, 15, 16, 31, 32, 33, 63, 64, 100, 1000, 4097, 32767]
    rng = np.random.default_rng(5)
    rng.shuffle(mix)
    return [int(x) for x in mix]


def gen_mixed() -> None:
    lens = mixed_lengths()
    n, stride = len(lens), 32768
    blocks = synth_blocks(1 << 30, n, stride)
    cs = [h(xx(blocks[i][:lens[i]])) for i in range(n)]
    write("mixed.json", {
        "config": "c5: mixed storm block lengths (objectlist/pointer/singularity/blob/spacelist + tails)",
        "seed": h(SEED), "first": 1 << 30, "stride": stride, "lens": lens, "checksums": cs,
    })


# ---- storm layouts (Go amd64) ---------------------------------------------
def pack_pointer_block(entries, fanout: int) -> bytes:
    size = (25 * fanout + 7) & ~7
    buf = bytearray(size)
    for k, (cs, addr, rev, typ) in enumerate(entries):
        struct.pack_into("<QQQ", buf, 24 * k, cs, addr, rev)
        buf[24 * fanout + k] = typ
    return bytes(buf)


def tree_root(leaf_cs, leaf_base: int, node_base: int, rev: int, fanout: int):
    n = len(leaf_cs)
    if n == 0:
        return (0, 0, 0, 0)
    entries = [(int(leaf_cs[i]), leaf_base + i, rev) for i in range(n)]
    typ, nxt = 2, node_base
    while len(entries) > 1:
        parents = []
        for j in range(0, len(entries), fanout):
            chunk = entries[j:j + fanout]
            node = pack_pointer_block([(c, a, r, typ) for (c, a, r) in chunk], fanout)
            parents.append((xx(node), nxt + len(parents), rev))
        nxt += len(parents)
        entries, typ = parents, 1
    c, a, r = entries[0]
    return (c, a, r, typ)


def gen_merkle() -> None:
    cases = []
    specs = [(0, 1200), (1, 1200), (2, 1200), (1199, 1200), (1200, 1200), (1201, 1200), (5000, 1200),
             (1, 10), (10, 10), (11, 10), (101, 10), (1000, 10), (12345, 10), (1_000_000, 1200)]
    for n, f in specs:
        leaf = splitmix_np(np.arange(n, dtype=np.uint64) ^ np.uint64(SEED))
        leaf_base, rev = 7 * n + 3, 5
        node_base = leaf_base + n
        t = time.time()
        root = tree_root(leaf, leaf_base, node_base, rev, f)
        cases.append({"n": n, "fanout": f, "leaf_addr_base": leaf_base, "node_addr_base": node_base, "rev": rev,
                      "root": [h(v) for v in root[:3]], "root_type": root[3]})
        print(f"  merkle n={n} F={f} {time.time() - t:.1f}s")
    # combine: 8 shard roots of the 1M-leaf tree split 8 ways (storm_amd.dist semantics)
    n_total, world, rev, f = 1_000_000, 8, 5, 1200
    leaf = splitmix_np(np.arange(n_total, dtype=np.uint64) ^ np.uint64(SEED))
    table = []
    for r in range(world):
        q, rem = divmod(n_total, world)
        lo = r * q + min(r, rem)
        hi = lo + q + (1 if r < rem else 0)
        table.append(tree_root(leaf[lo:hi], lo, n_total + lo, rev, f))
    groot = (xx(pack_pointer_block(table, f)), 2 * n_total, rev, 1)
    write("merkle.json", {
        "leaf_rule": "leaf_cs[i] = splitmix64(i ^ seed)", "seed": h(SEED), "cases": cases,
        "combine": {"n_total": n_total, "world": world, "rev": rev, "fanout": f,
                    "shard_roots": [[h(v) for v in t[:3]] + [t[3]] for t in table],
                    "global_root": [h(v) for v in groot[:3]] + [groot[3]]},
    })


def gen_layouts() -> None:
    # Sizes from Go's layout rules, computed by hand here (cross-checks storm_amd.layouts).
    sizes = {"prod": {"singularity": 72, "pointer": 30000, "spacelist": 28808, "objectlist": 31808, "blob": 32768},
             "test": {"singularity": 72, "pointer": 256, "spacelist": 728, "objectlist": 536, "blob": 32768}}
    zero = {tag: {k: h(xx(bytes(v))) for k, v in d.items()} for tag, d in sizes.items()}
    # singularity block after persistence.Initialize-like fill (fields at 0/8/16/24, Pointer 32..55,
    # type 56, LastAllocatedBlock 64; Checksum hashed as 0: cache/cache.go:71-73)
    sb = bytearray(72)
    struct.pack_into("<QQQQ", sb, 0, 0, 0x73746F726D, 3, 1 << 20)
    struct.pack_into("<QQQ", sb, 32, 0x1122334455667788, 42, 2)
    sb[56] = 2
    struct.pack_into("<Q", sb, 64, 777)
    # pointer-block sequence of /root/reference/blocks/pointer/block_test.go:15-34 (prod fanout)
    seq = []
    f = 1200
    pb = bytearray(30000)
    seq.append(xx(pb))
    struct.pack_into("<Q", pb, 0, 2); seq.append(xx(pb))                 # Pointers[0].Checksum = 2
    pb[24 * f + 0] = 2; seq.append(xx(pb))                               # PointedBlockTypes[0] = Leaf
    pb[24 * f + 1] = 2; seq.append(xx(pb))                               # PointedBlockTypes[1] = Leaf
    struct.pack_into("<Q", pb, 24 + 8, 2); seq.append(xx(pb))            # Pointers[1].Address = 2
    struct.pack_into("<Q", pb, 48, 4); seq.append(xx(pb))                # Pointers[2].Checksum = 4
    # blob block with the 4 objects of /root/reference/blocks/blob/block_test.go:19-37
    blob = bytearray(32768)
    items = [(1, 2, 3, 1), (4, 5, 6, 2), (7, 8, 9, 0), (10, 11, 12, 1)]
    for k, (tag, f1, f2, st) in enumerate(items):
        struct.pack_into("<QQBxxxxxxxB", blob, 32 * k, tag, f1, f2, st)
    write("layouts.json", {
        "sizes": sizes, "zero_block_checksums": zero,
        "singularity_example": {"bytes_hex": bytes(sb).hex(), "checksum": h(xx(sb))},
        "pointer_block_test_sequence": [h(v) for v in seq],
        "blob_test_block": {"first_128_hex": bytes(blob[:128]).hex(), "checksum": h(xx(blob))},
    })


def gen_commit() -> None:
    """f1 fixture: a storm-shaped dirty forest (leaves under fan-out-10 pointer blocks,
    rooted at the singularity's SpacePointer) committed by an independent restatement
    of Cache.Commit's loop (cache/cache.go:87-137, trace.go:274-320), hashed with
    libxxhash. Iteration order (height, index), as libstormck documents."""
    slot, fanout, revision, n_leaves = 1024, 10, 5, 137
    rng = np.random.default_rng(2024)
    lens = [int(x) for x in rng.choice([72, 256, 536, 728, 1000, 1024], size=n_leaves)]
    # layout: slot 0 singularity, slots 1..n leaves, then pointer blocks level by level
    recs = []  # dicts: off, len, type, parent, optr, otyp, addr, birth
    for i in range(n_leaves):
        recs.append({"off": (i + 1) * slot, "len": lens[i], "type": 2})
    start, count = 0, n_leaves
    while count > 1:
        pc = (count + fanout - 1) // fanout
        base = len(recs)
        for j in range(pc):
            recs.append({"off": (base + j + 1) * slot, "len": (25 * fanout + 7) & ~7, "type": 1})
        for c in range(count):
            p = base + c // fanout
            recs[start + c]["parent"] = p
            recs[start + c]["optr"] = recs[p]["off"] + 24 * (c % fanout)
            recs[start + c]["otyp"] = recs[p]["off"] + 24 * fanout + c % fanout
        start, count = base, pc
    recs[start].update(parent=-1, optr=32, otyp=56)
    existing = rng.random(len(recs)) < 0.3
    for i, r in enumerate(recs):
        r["addr"] = 1 + i
        r["birth"] = revision if existing[i] else revision + 1
    last = len(recs)
    arena = bytearray((len(recs) + 1) * slot)
    leaf_bytes = rng.integers(0, 256, size=n_leaves * slot, dtype=np.uint8).tobytes()
    for i in range(n_leaves):
        arena[(i + 1) * slot:(i + 2) * slot] = leaf_bytes[i * slot:(i + 1) * slot]
    initial = bytes(arena)
    # heights by walking up, order by (height, index)
    height = [0] * len(recs)
    for i in range(len(recs)):
        h_, p = 0, recs[i]["parent"]
        while p >= 0:
            h_ += 1
            height[p] = max(height[p], h_)
            p = recs[p]["parent"]
    order = sorted(range(len(recs)), key=lambda i: (height[i], i))
    cs = [0] * len(recs)
    for i in order:  # every child precedes its parent in this order
        r = recs[i]
        if r["birth"] <= revision:
            last += 1
            r["addr"], r["birth"] = last, revision + 1
        cs[i] = xx(arena[r["off"]:r["off"] + r["len"]])
        struct.pack_into("<QQQ", arena, r["optr"], cs[i], r["addr"], r["birth"])
        arena[r["otyp"]] = r["type"]
    # then the singularity step (cache/cache.go:71-73): Revision++, Checksum = 0, hash 72 B
    struct.pack_into("<Q", arena, 16, revision + 1)
    struct.pack_into("<Q", arena, 64, last)
    struct.pack_into("<Q", arena, 0, 0)
    sing = xx(arena[:72])
    write("commit.json", {
        "desc": "dirty forest committed children-first; see oracle/gen_golden.py gen_commit",
        "slot": slot, "fanout": fanout, "revision": revision, "n_leaves": n_leaves, "leaf_lens": lens,
        "existing": [int(x) for x in existing], "initial_arena_xxh64": h(xx(initial)),
        "leaf_bytes_seed": 2024,
        "checksums": [h(v) for v in cs], "addresses": [r["addr"] for r in recs],
        "last_allocated": last, "final_arena_xxh64": h(xx(arena[72:])), "singularity_checksum": h(sing),
    })


def gen_c5() -> None:
    """c5 (BASELINE.json configs[4]) as bench.py --workload c5 runs it: synthetic
    32 KiB-stride blocks 0..1201 hashed at storm's mixed lengths (1200 objectlist leaves
    of 31,808 B, one 30,000 B pointer block, the 72 B singularity), and the same 1200
    leaves committed as a forest under one fan-out-1200 pointer block rooted at the
    singularity (storm_amd.commit.pointer_forest: leaf i has address 1 + i and
    BirthRevision 2, nothing relocates), whose root checksum is the pointer block's."""
    n_ol, rev = 1200, 1
    lens = [31808] * n_ol + [30000, 72]
    blocks = synth_blocks(0, len(lens), 32768)
    cs = np.array([xx(blocks[i][:lens[i]]) for i in range(len(lens))], dtype=np.uint64)
    leaf = [(int(cs[i]), 1 + i, rev + 1, 2) for i in range(n_ol)]
    root = xx(pack_pointer_block(leaf, 1200))
    # the BenchmarkStorm mix (/root/reference/benchmark_test.go): storm.Set
    # adds blob leaves of 32,768 B and a spacelist block of 28,808 B to the same commit
    n_bl = 1200
    lens_s = [32768] * n_bl + [28808, 30000, 72]
    blocks_s = synth_blocks(0, len(lens_s), 32768)
    cs_s = np.array([xx(blocks_s[i][:lens_s[i]]) for i in range(len(lens_s))], dtype=np.uint64)
    root_s = xx(pack_pointer_block([(int(cs_s[i]), 1 + i, rev + 1, 2) for i in range(n_bl)], 1200))
    write("c5.json", {
        "config": "c5: bench.py --workload c5 (keystore/benchmark_test.go commit batch)", "seed": h(SEED),
        "lens": {"31808": n_ol, "30000": 1, "72": 1}, "batch_digest": h(xx(cs.astype("<u8").tobytes())),
        "first4": [h(int(v)) for v in cs[:4]], "last2": [h(int(v)) for v in cs[-2:]],
        "commit_root": h(root), "commit_root_address": 1 + n_ol, "commit_revision": rev,
        "storm": {"config": "bench.py --workload c5 --c5-mix storm (benchmark_test.go BenchmarkStorm commit batch)",
                  "lens": {"32768": n_bl, "28808": 1, "30000": 1, "72": 1},
                  "batch_digest": h(xx(cs_s.astype("<u8").tobytes())),
                  "first4": [h(int(v)) for v in cs_s[:4]], "last3": [h(int(v)) for v in cs_s[-3:]],
                  "commit_root": h(root_s), "commit_root_address": 1 + n_bl},
    })


def _keytags_worker(args):
    first, count, klen = args
    sys.path.insert(0, ROOT)
    from oracle import oracle as o  # generator only; hashing stays libxxhash
    per = 48 * 1024 // klen  # keys per 48 KiB synthetic block
    buf = o.fill_synthetic(count // per, 48 * 1024, first // per)
    mv = memoryview(buf)
    return first, np.array([xxhash.xxh64_intdigest(mv[k * klen:(k + 1) * klen]) for k in range(count)],
                           dtype=np.uint64)


def gen_keytags() -> None:
    """f4 as bench.py --workload keytags runs it: 64M keys of 48 B, packed (key i at byte
    48 i of synthetic 48 KiB blocks 0..65535), each tagged with xxhash.Sum64; the digest
    is XXH64 of the 64M tags (about a minute on every core)."""
    import multiprocessing as mp
    n, klen, chunk = 1 << 26, 48, 1 << 20
    tags = np.empty(n, dtype=np.uint64)
    with mp.get_context("fork").Pool(max(1, (os.cpu_count() or 2) - 1)) as pool:
        for first, t in pool.imap_unordered(_keytags_worker, [(f, chunk, klen) for f in range(0, n, chunk)]):
            tags[first:first + chunk] = t
    write("keytags.json", {
        "config": "f4: bench.py --workload keytags, 64M packed 48-byte keys", "seed": h(SEED), "keys": n,
        "key_bytes": klen, "digest": h(xx(tags.astype("<u8").tobytes())),
        "first4": [h(int(v)) for v in tags[:4]], "every_1048576th": [h(int(v)) for v in tags[::1 << 20]],
    })


def gen_big() -> None:
    """Digests (XXH64 of the little-endian checksum array) of the c2 (1M) and c3 (16M)
    synthetic 32 KiB block sets. Blocks are generated with the C oracle's generator
    (pinned against synth_c1.json's numpy words) and hashed with libxxhash."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as o  # generator only; hashing stays libxxhash
    stride = 32768
    res = {}
    for n in (1 << 20, 1 << 24):
        t = time.time()
        chunk = 1 << 14
        cs = np.empty(n, dtype=np.uint64)
        for first in range(0, n, chunk):
            buf = o.fill_synthetic(chunk, stride, first)
            mv = memoryview(buf)
            cs[first:first + chunk] = [xxhash.xxh64_intdigest(mv[i * stride:(i + 1) * stride]) for i in range(chunk)]
        res[str(n)] = {"digest": h(xx(cs.astype("<u8").tobytes())),
                       "first8": [h(int(v)) for v in cs[:8]], "last": h(int(cs[-1])),
                       "every_65536th": [h(int(v)) for v in cs[::65536]]}
        print(f"  big n={n} {time.time() - t:.0f}s")
    write("synth_digests.json", {"rule": "synth_c1.json rule, first = 0, stride = length = 32768",
                                 "seed": h(SEED), "digests": res})


def pack_level_np(cs: np.ndarray, addr_base: int, rev: int, typ: int, fanout: int) -> np.ndarray:
    """Every parent node of one tree level as storm pointer.Block bytes, [pm, size] uint8
    (vectorised form of pack_pointer_block over children {cs[i], addr_base + i, rev})."""
    m = len(cs)
    pm = (m + fanout - 1) // fanout
    size = (25 * fanout + 7) & ~7
    ptr = np.zeros((pm * fanout, 3), dtype="<u8")
    ptr[:m, 0] = cs
    ptr[:m, 1] = np.arange(addr_base, addr_base + m, dtype=np.uint64)
    ptr[:m, 2] = rev
    typ_b = np.zeros(pm * fanout, dtype=np.uint8)
    typ_b[:m] = typ
    out = np.zeros((pm, size), dtype=np.uint8)
    out[:, :24 * fanout] = ptr.view(np.uint8).reshape(pm, 24 * fanout)
    out[:, 24 * fanout:25 * fanout] = typ_b.reshape(pm, fanout)
    return out


def tree_root_np(leaf_cs: np.ndarray, leaf_base: int, node_base: int, rev: int, fanout: int):
    """tree_root for large n: same rule, levels packed with pack_level_np."""
    n = len(leaf_cs)
    if n <= 1:
        return tree_root([int(x) for x in leaf_cs], leaf_base, node_base, rev, fanout)
    cur, base, typ, nxt = np.asarray(leaf_cs, dtype=np.uint64), leaf_base, 2, node_base
    while len(cur) > 1:
        nodes = pack_level_np(cur, base, rev, typ, fanout)
        cur = np.array([xx(memoryview(nodes[k])) for k in range(nodes.shape[0])], dtype=np.uint64)
        base, nxt, typ = nxt, nxt + len(cur), 1
    return (int(cur[0]), base, rev, typ)


def _c4_worker(args):
    first, count, path, total = args
    sys.path.insert(0, ROOT)
    from oracle import oracle as o  # generator only; hashing stays libxxhash
    stride = 32768
    cs = np.memmap(path, dtype=np.uint64, mode="r+", shape=(total,))
    buf = o.fill_synthetic(count, stride, first)
    mv = memoryview(buf)
    cs[first:first + count] = [xxhash.xxh64_intdigest(mv[i * stride:(i + 1) * stride]) for i in range(count)]
    cs.flush()
    return count


def gen_c4() -> None:
    """c3 / c4 roots (BASELINE.json configs[2], configs[3]) over the synthetic 32 KiB
    blocks 0..64M-1, hashed with libxxhash on every host core (several minutes).

    c3: the 16M-block shard tree bench.py builds at N = 1 (leaves 0..16M-1, leaf
    addresses = block index, interior nodes from 16M, BirthRevision 1, fan-out 1200).
    c4: 64M blocks split into `world` contiguous shards (storm_amd.dist.shard_range
    rule restated here); shard s's tree has leaf addresses lo_s.., interior nodes from
    64M + lo_s; the global root hashes one pointer block of the world shard roots and
    has address 2 * 64M (storm_amd.dist.global_root_addr). Roots for world 1, 2, 4 and 8
    (the bench's strong-scaling series over the c4 set; at world 1 the shard root is
    what `bench.py --total-blocks 67108864` prints, the global root what it prints with
    --force-dist)."""
    import multiprocessing as mp
    n_total, rev, f = 1 << 26, 1, 1200
    # the numpy packer agrees with the per-entry packer on ragged trees
    for n_chk, f_chk in ((12345, 10), (5000, 1200), (1201, 1200)):
        leaf = splitmix_np(np.arange(n_chk, dtype=np.uint64) ^ np.uint64(SEED))
        assert tree_root_np(leaf, 3, n_chk + 3, 5, f_chk) == tree_root(leaf, 3, n_chk + 3, 5, f_chk)
    path = os.environ.get("C4_CS_CACHE", "/tmp/c4_checksums.u64")
    t = time.time()
    if not (os.path.exists(path) and os.path.getsize(path) == 8 * n_total):
        np.memmap(path, dtype=np.uint64, mode="w+", shape=(n_total,)).flush()
        chunk = 1 << 14
        jobs = [(first, chunk, path, n_total) for first in range(0, n_total, chunk)]
        with mp.get_context("fork").Pool(max(1, (os.cpu_count() or 2) - 1)) as pool:
            done = 0
            for c in pool.imap_unordered(_c4_worker, jobs):
                done += c
                if done % (1 << 22) == 0:
                    print(f"  c4 checksums {done >> 20}M / 64M {time.time() - t:.0f}s", flush=True)
    cs = np.memmap(path, dtype=np.uint64, mode="r", shape=(n_total,))
    # pinned against the independent single-process digests of gen_big (16M prefix)
    with open(os.path.join(OUT, "synth_digests.json")) as fh:
        dig = json.load(fh)["digests"][str(1 << 24)]["digest"]
    assert h(xx(np.ascontiguousarray(cs[:1 << 24]).astype("<u8").tobytes())) == dig, "16M prefix digest"
    c3 = tree_root_np(cs[:1 << 24], 0, 1 << 24, rev, f)
    worlds = {}
    for world in (1, 2, 4, 8):
        table = []
        for r in range(world):
            q, rem = divmod(n_total, world)
            lo = r * q + min(r, rem)
            hi = lo + q + (1 if r < rem else 0)
            table.append(tree_root_np(cs[lo:hi], lo, n_total + lo, rev, f))
        groot = (xx(pack_pointer_block(table, f)), 2 * n_total, rev, 1)
        worlds[str(world)] = {"shard_roots": [[h(v) for v in r_[:3]] + [r_[3]] for r_ in table],
                              "global_root": [h(v) for v in groot[:3]] + [groot[3]]}
    # f1: bench.py --workload commit commits the first 1M of these blocks as 32 KiB leaves
    # under fan-out-1200 pointer blocks (storm_amd.commit.pointer_forest: leaves get
    # addresses 1.., pointer blocks the next addresses level by level, BirthRevision 2
    # everywhere, nothing relocates); the commit's root is the top pointer block's
    f1 = tree_root_np(cs[:1 << 20], 1, (1 << 20) + 1, 2, f)
    write("c3c4_roots.json", {
        "rule": "synth_c1.json rule, stride = length = 32768, fan-out 1200, BirthRevision 1; see gen_c4",
        "seed": h(SEED),
        "c3": {"n": 1 << 24, "leaf_addr_base": 0, "node_addr_base": 1 << 24,
               "root": [h(v) for v in c3[:3]] + [c3[3]]},
        "f1_commit_1m": {"leaves": 1 << 20, "root": [h(v) for v in f1[:3]] + [f1[3]]},
        "c4": {"n_total": n_total, "digest": h(xx(np.ascontiguousarray(cs).astype("<u8").tobytes())),
               "every_1048576th": [h(int(v)) for v in cs[::1 << 20]], "worlds": worlds},
    })
    print(f"  c4 done {time.time() - t:.0f}s")


if __name__ == "__main__":
    if "--c4" in sys.argv:  # only the c3/c4 roots (several minutes on every core)
        gen_c4()
        sys.exit(0)
    if "--keytags" in sys.argv:  # only the f4 digest (about a minute on every core)
        gen_keytags()
        sys.exit(0)
    gen_kat()
    gen_synth_c1()
    gen_mixed()
    gen_layouts()
    gen_merkle()
    gen_commit()
    gen_c5()
    if "--big" in sys.argv:
        gen_big()
