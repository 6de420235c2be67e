"""Static checks of the Go cgo shim (integration/go/blocks/checksum_stormck.go)
against include/stormck.h (CPU, no Go toolchain in the image).

The shim cannot be compiled here, so these tests hold it to the header the way
cgo would: every C.stormck_* call names a declared function with the declared
number of arguments, every C.STORMCK_* constant is defined, and the Go mirror of
stormck_dirty_block has the C field order, types and offsets.
"""
import os
import re

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "stormck.h")
SHIM = os.path.join(ROOT, "integration", "go", "blocks", "checksum_stormck.go")


def _strip_c_comments(text):
    return re.sub(r"/\*.*?\*/", "", text, flags=re.S)


def _split_args(s):
    """Top-level comma split of an argument list (parentheses and brackets nest)."""
    depth, cur, out = 0, [], []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    tail = "".join(cur).strip()
    if tail:
        out.append(tail)
    return out


def _balanced(text, start):
    """Contents of the parenthesised group whose '(' is at text[start]."""
    assert text[start] == "("
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "(":
            depth += 1
        elif text[i] == ")":
            depth -= 1
            if depth == 0:
                return text[start + 1:i]
    raise AssertionError("unbalanced parentheses")


def header_prototypes():
    text = _strip_c_comments(open(HEADER).read())
    protos = {}
    for m in re.finditer(r"\b(stormck_[a-z_0-9]+)\s*\(", text):
        name = m.group(1)
        before = text[:m.start()].rstrip()
        if not re.search(r"(int|void|uint64_t|char\s*\*|const char\s*\*)$", before):
            continue  # a use inside a macro or typedef, not a prototype
        args = _split_args(_balanced(text, m.end() - 1))
        protos[name] = 0 if args in ([], ["void"]) else len(args)
    return protos


def shim_calls():
    text = open(SHIM).read()
    calls = []
    for m in re.finditer(r"\bC\.(stormck_[a-z_0-9]+)\s*\(", text):
        calls.append((m.group(1), len(_split_args(_balanced(text, m.end() - 1)))))
    return calls


def test_shim_calls_match_header_prototypes():
    protos = header_prototypes()
    calls = shim_calls()
    assert len(calls) >= 9
    for name, nargs in calls:
        assert name in protos, f"{name} is not declared in include/stormck.h"
        assert nargs == protos[name], f"{name}: shim passes {nargs} args, header declares {protos[name]}"


def test_shim_constants_are_defined():
    header = open(HEADER).read()
    shim = open(SHIM).read()
    for const in set(re.findall(r"\bC\.(STORMCK_[A-Z_0-9]+)", shim)):
        assert re.search(r"(#define\s+%s\b|\b%s\s*=)" % (const, const), header), const


def test_shim_keeps_reference_signatures_and_error_format():
    shim = open(SHIM).read()
    # blocks/checksum.go:10-27 signatures, unchanged
    assert "func BlockChecksum[T Block](b *T) Hash {" in shim
    assert "func Checksum(b []byte) Hash {" in shim
    assert "func VerifyChecksum(address BlockAddress, p []byte, expectedChecksum Hash) error {" in shim
    assert '"checksum mismatch for block %d, computed: %#v, expected: %#v"' in shim


_GO_SIZES = {"uint64": 8, "int64": 8, "BlockAddress": 8, "uint32": 4, "BlockType": 1}


def go_dirty_block_fields():
    text = open(SHIM).read()
    body = re.search(r"type DirtyBlock struct \{(.*?)\n\}", text, flags=re.S).group(1)
    fields = []
    for line in body.strip().splitlines():
        line = line.split("//")[0].strip()
        if not line:
            continue
        name, typ = line.split()[:2]
        m = re.fullmatch(r"\[(\d+)\]byte", typ)
        fields.append((name, int(m.group(1)) if m else _GO_SIZES[typ]))
    return fields


_C_SIZES = {"uint64_t": 8, "int64_t": 8, "uint32_t": 4, "uint8_t": 1}


def header_dirty_block_fields():
    text = _strip_c_comments(open(HEADER).read())
    body = re.search(r"typedef struct stormck_dirty_block \{(.*?)\}", text, flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, name = decl.split()
        m = re.fullmatch(r"(\w+)\[(\d+)\]", name)
        fields.append((m.group(1), _C_SIZES[typ] * int(m.group(2))) if m else (name, _C_SIZES[typ]))
    return fields


def test_go_dirty_block_has_the_c_layout():
    from storm_amd.commit import DIRTY_DTYPE  # the Python binding's mirror
    go = go_dirty_block_fields()
    c = header_dirty_block_fields()
    assert [n for n, _ in c] == list(DIRTY_DTYPE.names)
    assert len(go) == len(c)
    off = 0
    for (gname, gsize), (cname, csize) in zip(go, c):
        assert gsize == csize, (gname, cname)
        assert DIRTY_DTYPE.fields[cname][1] == off, (gname, cname)
        off += gsize
    assert off == DIRTY_DTYPE.itemsize == 56


# --- the storm-side f1 binding (integration/go/cache) ---------------------------------

CACHE_DIR = os.path.join(ROOT, "integration", "go", "cache")


def _go(name):
    return open(os.path.join(CACHE_DIR, name)).read()


def _go_funcs(text):
    """name -> number of parameters of every top-level func / method in a Go file."""
    out = {}
    for m in re.finditer(r"^func\s+(?:\([^)]*\)\s*)?([A-Za-z_]\w*)\s*(?:\[[^\]]*\])?\s*\(", text, flags=re.M):
        args = _split_args(_balanced(text, m.end() - 1))
        n = 0
        for a in args:  # "a, b int" declares two parameters
            n += 1
        out[m.group(1)] = n
    return out


def test_cache_binding_build_tags_and_entry_points():
    stormck, default, record = _go("commit_stormck.go"), _go("commit_default.go"), _go("commit_record.go")
    assert stormck.startswith("//go:build stormck\n")
    assert default.startswith("//go:build !stormck\n")
    assert "//go:build" not in record.split("package")[0]
    for text in (stormck, default):  # both builds provide what the patched cache.go calls
        f = _go_funcs(text)
        assert "commitDirty" in f and "newArena" in f
    assert "recordCommit" in _go_funcs(record)
    assert re.search(r"type commitRecord struct \{\s*origin BlockOrigin\s*parent \*blockMetadata\s*size\s+uint32\s*"
                     r"typ\s+blocks\.BlockType\s*\}", record)
    for field in re.findall(r"\.commit\.(\w+)", stormck):
        assert field in ("origin", "parent", "size", "typ"), field


def test_cache_binding_calls_match_the_blocks_shim():
    stormck = re.sub(r"//[^\n]*", "", _go("commit_stormck.go"))
    shim_funcs = _go_funcs(open(SHIM).read())
    calls = [(m.group(1), len(_split_args(_balanced(stormck, m.end() - 1))))
             for m in re.finditer(r"\bblocks\.([A-Z]\w*)\s*\(", stormck)]
    assert ("CommitBatch", 5) in calls and ("NewHostArena", 1) in calls
    for name, n in calls:
        assert name in shim_funcs, f"blocks.{name} is not defined in the shim"
        assert shim_funcs[name] == n, f"blocks.{name}: {n} args, shim declares {shim_funcs[name]}"
    # DirtyBlock fields the binding sets exist in the shim's mirror of stormck_dirty_block
    fields = {n for n, _ in go_dirty_block_fields()}
    for f in set(re.findall(r"\bd\.(\w+)\s*=", stormck)) | set(re.findall(r"dirty\[i\]\.(\w+)", stormck)):
        assert f in fields, f


def test_storm_patch_applies_to_the_reference(tmp_path):
    """trace_types.patch applies cleanly to storm's cache/ (types.go, trace.go, cache.go)
    and wires exactly what the binding needs. Skipped where /root/reference is absent."""
    import shutil
    import subprocess
    ref = "/root/reference/cache"
    if not os.path.isdir(ref):
        import pytest
        pytest.skip("reference not present")
    dst = tmp_path / "cache"
    dst.mkdir()
    for f in ("types.go", "trace.go", "cache.go"):
        shutil.copy(os.path.join(ref, f), dst / f)
    p = subprocess.run(["patch", "-p1", "-d", str(tmp_path), "-i", os.path.join(CACHE_DIR, "trace_types.patch")],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "offset" not in p.stdout and "fuzz" not in p.stdout, p.stdout
    trace = (dst / "trace.go").read_text()
    assert trace.count(".recordCommit(") == 2
    assert "pointerBlockMeta.recordCommit(origin, parentBlockMeta, unsafe.Sizeof(*pointerBlock), blocks.PointerBlockType)" in trace
    assert "leafBlockMeta.recordCommit(origin, parentBlockMeta, unsafe.Sizeof(*leafBlock), blocks.LeafBlockType)" in trace
    cache = (dst / "cache.go").read_text()
    assert "c.commitDirty()" in cache and "newArena(" in cache and "c.commitData()" not in cache
    assert "commit commitRecord" in (dst / "types.go").read_text()


def test_commit_batch_takes_the_routed_commit():
    """CommitBatch hands storm's registered cache.data (a host pointer) to stormck_commit,
    which picks the device or host leg by the measured crossover (DESIGN_LOG §11 f1); it no
    longer calls stormck_commit_device directly. The host-thread knob and the leg
    constants are exported."""
    text = open(SHIM).read()
    body = text[text.index("func CommitBatch("):]
    body = body[:body.index("\n}\n")]
    assert "C.stormck_commit(bytesPtr(arena)" in body
    assert "stormck_commit_device" not in body and "stormck_host_device_pointer" not in body
    assert "C.uint32_t(CommitHostThreads)" in body
    assert re.search(r"var CommitHostThreads uint32", text)
    for name, c in (("LegNone", "STORMCK_LEG_NONE"), ("LegHost", "STORMCK_LEG_HOST"),
                    ("LegDevice", "STORMCK_LEG_DEVICE")):
        assert re.search(name + r"\s*=\s*uint32\(C\." + c + r"\)", text), name
    stormck = _go("commit_stormck.go")
    assert "_, err = blocks.CommitBatch(c.data, dirty, sb.Revision, &last, out)" in stormck


def _go_func(text, name):
    body = text[text.index("func " + name + "("):]
    return body[:body.index("\n}\n")]


def test_batches_take_the_routed_batch():
    """ChecksumBatch / VerifyChecksumBatch hand host blocks to stormck_checksum_batch /
    stormck_verify_batch, which pick the device or host leg by the measured cost model
    (DESIGN_LOG §5, "Host-memory batches, routed"); ChecksumBatchGPU keeps the device leg alone
    and ChecksumBatchDevices the multi-GPU one. The host-thread knob is exported."""
    text = open(SHIM).read()
    cb = _go_func(text, "ChecksumBatch")
    assert "C.stormck_checksum_batch(bytesPtr(data)" in cb and "C.uint32_t(BatchHostThreads)" in cb
    assert "stormck_checksum_host(" not in cb
    vb = _go_func(text, "VerifyChecksumBatch")
    assert "C.stormck_verify_batch(bytesPtr(data)" in vb and "C.uint32_t(BatchHostThreads)" in vb
    assert "C.STORMCK_EMISMATCH" in vb
    assert "C.stormck_checksum_host(bytesPtr(data)" in _go_func(text, "ChecksumBatchGPU")
    assert "C.stormck_checksum_host_multi(" in _go_func(text, "ChecksumBatchDevices")
    assert re.search(r"var BatchHostThreads uint32", text)


def test_go_shard_has_the_c_layout_and_the_multi_entries_bind_it():
    """The one-process multi-GPU entries (stormck_shard_plan / stormck_merkle_root_multi):
    the Go Shard mirrors stormck_shard field by field (sizes and order; 64 bytes), and the
    shim's PlanShards / MerkleRootDevices pass the shard slice, the root and the shard roots
    through the C types."""
    text = open(SHIM).read()
    body = re.search(r"type Shard struct \{(.*?)\n\}", text, flags=re.S).group(1)
    go_sizes = {"uintptr": 8, "uint64": 8, "BlockAddress": 8, "int32": 4, "uint32": 4}
    go = []
    for line in body.strip().splitlines():
        line = line.split("//")[0].strip()
        if line:
            name, typ = line.split()[:2]
            go.append((name, go_sizes[typ]))
    hdr = _strip_c_comments(open(HEADER).read())
    cbody = re.search(r"typedef struct stormck_shard \{(.*?)\}", hdr, flags=re.S).group(1)
    c = []
    for decl in cbody.split(";"):
        decl = decl.strip()
        if decl:
            name = decl.replace("*", " ").split()[-1]
            c.append((name, 8 if "*" in decl else dict(_C_SIZES, int32_t=4)[decl.split()[0]]))
    assert [s for _, s in go] == [s for _, s in c] and sum(s for _, s in c) == 64
    assert [n.lower() for n, _ in go] == [re.sub(r"^d_", "", n).replace("_", "") for n, _ in c]
    plan = _go_func(text, "PlanShards")
    assert "C.stormck_shard_plan(" in plan and "(*C.stormck_shard)(unsafe.Pointer(&shards[0]))" in plan
    root = _go_func(text, "MerkleRootDevices")
    assert "C.stormck_merkle_root_multi((*C.stormck_shard)(unsafe.Pointer(&shards[0]))" in root
    assert "C.STORMCK_POINTERS_PER_BLOCK" in root and "(*C.stormck_pointer)(unsafe.Pointer(&root))" in root
