"""The evidence stays auditable (verdict r05 item 6): every `profiles/` path the design
documents cite exists, and every session kept under `profiles/` is cited by them."""
import fnmatch
import json
import os
import re

from tests.conftest import ROOT

DOCS = ["DESIGN.md", "DESIGN_LOG.md", "README.md", "INTEGRATION.md", os.path.join("tools", "README.md")]
PROFILES = os.path.join(ROOT, "profiles")


def docs_text():
    parts = []
    for d in DOCS:
        p = os.path.join(ROOT, d)
        if os.path.exists(p):
            with open(p, encoding="utf-8") as f:
                parts.append(f.read())
    return "\n".join(parts)


def cited_paths(text):
    """`profiles/...` citations: the path up to the first character no path holds."""
    return sorted(set(m.rstrip(".,;:)") for m in re.findall(r"profiles/([A-Za-z0-9_.*\-/]+)", text)))


def test_every_cited_profile_exists():
    missing = []
    for c in cited_paths(docs_text()):
        if "*" in c:
            head, pat = os.path.split(c)
            base = os.path.join(PROFILES, head)
            if not (os.path.isdir(base) and fnmatch.filter(os.listdir(base), pat)):
                missing.append(c)
        elif not os.path.exists(os.path.join(PROFILES, c)):
            missing.append(c)
    assert not missing, f"cited under profiles/ but absent: {missing}"


def test_every_profile_session_is_cited():
    text = docs_text()
    globs = [c for c in cited_paths(text) if "*" in c and "/" not in c]
    uncited = []
    for entry in sorted(os.listdir(PROFILES)):
        name = entry.rsplit(".", 1)[0] if os.path.isfile(os.path.join(PROFILES, entry)) else entry
        if re.search(r"(?<![A-Za-z0-9_])" + re.escape(name) + r"(?![A-Za-z0-9])", text):
            continue
        if any(fnmatch.fnmatch(entry, g) for g in globs):
            continue
        uncited.append(entry)
    assert not uncited, f"kept under profiles/ but cited by no design document: {uncited}"


def test_profile_source_of_the_line_exists():
    """bench.py names the rocprofv3 session behind the line's frac (profiles/traffic.json)."""
    with open(os.path.join(PROFILES, "traffic.json")) as f:
        tj = json.load(f)
    assert tj.get("source"), "traffic.json names no session"
    for key in ("source", "pmc_source"):  # the PMC passes may come from another session
        for path in re.findall(r"profiles/[A-Za-z0-9_.\-/]+", tj.get(key) or ""):
            assert os.path.exists(os.path.join(ROOT, path.rstrip(".,;:)"))), (key, path)
