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
