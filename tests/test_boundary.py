"""CPU: the C-ABI library loads, exports every symbol include/exacto_hip.h declares, and
validates parameters with the reference's error variants/messages before touching a GPU."""

import ctypes
import os
import re

import pytest

from exacto_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "exacto_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(exacto_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_ffi.lib_path())
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares the same set
    assert sorted(_ffi.EXPORTED_SYMBOLS) == syms


def test_version():
    assert b"gfx950" in _ffi.load().exacto_version()


@pytest.mark.parametrize("n,moduli,plain,variant,text", [
    (12, [65537], 257, "InvalidRingDegree", "ring degree must be a power of 2, got 12"),
    (16, [], 257, "InvalidParam", "must specify at least one ciphertext modulus"),
    (16, [65537], 1, "InvalidParam", "plaintext modulus must be >= 2"),
    (16, [65539], 257, "InvalidParam", "cannot create NTT plan for n=16, q=65539"),
    (8, [65537], 257, "InvalidParam", "cannot create NTT plan for n=8"),
    (16, [(1 << 62) + 1], 257, "InvalidParam", "cannot create NTT plan"),
])
def test_ctx_create_validation(n, moduli, plain, variant, text):
    with pytest.raises(_ffi.ExactoError) as e:
        _ffi.HipContext(n, moduli, plain_modulus=plain)
    assert e.value.variant == variant
    assert text in str(e.value)


def test_no_silent_fallback(monkeypatch, tmp_path):
    monkeypatch.setattr(_ffi, "_LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_ffi, "_lib", None)
    with pytest.raises(RuntimeError):
        _ffi.load()


def test_required_trace_elements_host_entry():
    """coeffs_to_slots.rs:390-396 (the reference's own vectors) and the oracle restatement."""
    from oracle import bootstrap as ob
    assert _ffi.required_trace_elements(8) == [3, 5, 7, 9, 11, 13, 15]
    assert _ffi.required_trace_elements(64) == [65, 33, 17, 9, 5, 3]
    for n in (16, 32, 48, 64, 1024, 4096, 8192):
        assert _ffi.required_trace_elements(n) == ob.required_trace_elements(n)


def test_digit_extract_host_entries():
    """digit_extract.rs:204-267 (the reference's Lagrange / rounding-polynomial tests) and the
    literal O(n^3) oracle restatement."""
    from oracle import bootstrap as ob
    assert _ffi.lagrange_interpolate([0, 1, 2], 7) == [0, 1, 0]
    assert _ffi.lagrange_interpolate([0, 1, 4, 2], 7) == [0, 0, 1, 0]
    vals = [(i * i + 3 * i + 7) % 29 for i in range(10)]
    coeffs = _ffi.lagrange_interpolate(vals, 29)
    for x, want in enumerate(vals):
        assert sum(c * pow(x, k, 29) for k, c in enumerate(coeffs)) % 29 == want
    assert coeffs == ob.lagrange_interpolate(vals, 29)
    for t, qp, tb in ((5, 25, 29), (16, 64, 257), (3, 10, 11)):
        poly = _ffi.compute_rounding_poly(t, qp, tb)
        assert poly == ob.compute_rounding_poly(t, qp, tb)
        for x in range(tb):
            want = (t * (x % qp) + qp // 2) // qp % t
            assert sum(c * pow(x, k, tb) for k, c in enumerate(poly)) % tb % t == want
    assert _ffi.lagrange_interpolate([], 7) == []
    assert _ffi.lagrange_interpolate([9], 7) == [2]
    with pytest.raises(_ffi.ExactoError) as e:
        _ffi.lagrange_interpolate(list(range(9)), 7)  # 9 points mod 7 are not distinct
    assert e.value.variant == "InvalidParam" and "points must be distinct mod p" in str(e.value)
