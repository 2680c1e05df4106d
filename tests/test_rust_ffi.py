"""The Rust binding a maintainer drops into the reference crate (include/exacto_hip.rs, the
`extern "C"` block of INTEGRATION.md §2 for EVERY entry point) is generated from the C header
(tools/gen_rust_ffi.py): the committed file is current, declares every function the header declares
with the same parameter count, and the info struct has the header's fields in order."""

import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_rust_ffi as G  # noqa: E402


def test_committed_binding_is_current():
    with open(G.HDR) as f:
        src = f.read()
    with open(G.OUT) as f:
        assert f.read() == G.emit(src), "re-run tools/gen_rust_ffi.py"


def test_binding_covers_every_header_function():
    with open(G.HDR) as f:
        src = f.read()
    protos = {name: args for name, args, _ in G.parse(src)}
    body = G.strip_comments(src)
    declared = set(re.findall(r"\b(exacto_\w+)\s*\(", body))
    assert declared == set(protos), declared ^ set(protos)
    with open(G.OUT) as f:
        rs = f.read()
    for name, args in protos.items():
        m = re.search(r"pub fn " + name + r"\((.*?)\)", rs)
        assert m, name
        n = 0 if not m.group(1).strip() else m.group(1).count(":")
        assert n == len(args), (name, n, len(args))
    assert len(protos) >= 90
