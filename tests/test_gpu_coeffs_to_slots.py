"""CoeffsToSlots / SlotsToCoeffs on the GPU: exacto_extract_coefficients,
exacto_slots_to_coeffs, with the keys of exacto_required_trace_elements.

Reference: bootstrap/coeffs_to_slots.rs:21-197.  Bit-exact against oracle/bootstrap.py on uniform
ciphertexts and Galois keys for the naive trace (n = 16, the reference's own test parameters)
and the relative-trace chain (n = 64 over cfg3's 3x60-bit basis); the reference's decrypt-level
tests (coeffs_to_slots.rs:221-318) with device-generated keys; the error cases.
"""
import numpy as np
import pytest

from oracle import bfv as obfv, bootstrap as ob, params as P
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues

pytestmark = pytest.mark.gpu

KEY = [42, 0, 0, 1]


def small_test_params():
    """coeffs_to_slots.rs:208-217: n = 16, t = 97, one 51-bit prime, base 8."""
    return (P.BfvParamsBuilder().ring_degree(16).plain_modulus(97).ct_moduli([1125899906842817])
            .sigma(3.2).gadget_base(8).build())


def _oracle_keys(prm, elements, gks):
    return {k: obfv.GaloisKey(np_to_rlk(gks[e], prm).keys, k, prm) for e, k in enumerate(elements)}


@pytest.mark.parametrize("which,j0,count", [("small16", 0, 16), ("cfg3_n64", 5, 6), ("cfg3_n64", 60, 5)])
def test_extract_coefficients_match_oracle(gpu_available, which, j0, count):
    prm = small_test_params() if which == "small16" else P.cfg3_params(64)
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(41)
    ct = uniform_residues(rng, (2,), q, n)
    elements = ctx.required_trace_elements()
    assert elements == ob.required_trace_elements(n)
    # keys in a shuffled order, plus an unused one: the ABI takes them as a map
    order = list(rng.permutation(len(elements)))
    els = [elements[i] for i in order] + [2 * n - 1 if n > 32 else 1]
    gks = uniform_residues(rng, (len(els), 2, 2), q, n)
    got = ctx.extract_coefficients(ct, j0, count, els, gks)
    keys = _oracle_keys(prm, els, gks)
    oc = np_to_ct(ct, prm)
    for t in range(count):
        want = ct_to_np(ob.extract_coefficient(oc, j0 + t, keys))
        assert np.array_equal(got[t], want), (which, j0 + t)


@pytest.mark.parametrize("which", ["small16", "cfg3_n64"])
def test_batched_after_single_extraction(gpu_available, which):
    """One context extracts J = 1 and then J = n coefficients, three times over: every result is
    bit-exact against the oracle.  Regression for the round-1 fault where results changed from
    call to call once scratch blocks were recycled (the key-switch workspace grows from 1 to n
    items between the two calls, and the scratch comes from the stream-ordered pool)."""
    prm = small_test_params() if which == "small16" else P.cfg3_params(64)
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(47)
    elements = ctx.required_trace_elements()
    gks = uniform_residues(rng, (len(elements), 2, 2), q, n)
    keys = _oracle_keys(prm, elements, gks)
    cts = [uniform_residues(rng, (2,), q, n) for _ in range(2)]
    want = [[ct_to_np(ob.extract_coefficient(np_to_ct(ct, prm), j, keys)) for j in range(n)] for ct in cts]
    for rep in range(3):
        for c, ct in enumerate(cts):
            one = ctx.extract_coefficients(ct, 3, 1, elements, gks)
            assert np.array_equal(one[0], want[c][3]), (which, rep, c, "J=1")
            alln = ctx.extract_coefficients(ct, 0, n, elements, gks)
            for j in range(n):
                assert np.array_equal(alln[j], want[c][j]), (which, rep, c, j)


@pytest.mark.parametrize("which", ["small16", "cfg3_n64"])
def test_slots_to_coeffs_matches_oracle(gpu_available, which):
    prm = small_test_params() if which == "small16" else P.cfg3_params(64)
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(43)
    slots = uniform_residues(rng, (n, 2), q, n)
    got = ctx.slots_to_coeffs(slots)
    want = ob.slots_to_coeffs([np_to_ct(slots[j], prm) for j in range(n)])
    assert np.array_equal(got, ct_to_np(want))


def _encrypt(ctx, prm, coeffs, sk, stream):
    pt = np.zeros((1, prm.ring_degree), dtype=np.uint64)
    pt[0, :len(coeffs)] = coeffs
    return ctx.encrypt_sk(pt, sk, KEY, stream=stream)[0]


def test_reference_extract_and_roundtrip(gpu_available):
    """coeffs_to_slots.rs:221-318: extract 42; extract 5, 10, 15 from 5 + 10X + 15X^2; CoeffsToSlots of
    1 + 2X + ... + 16X^15 decrypts slot j to j + 1, and SlotsToCoeffs brings the polynomial back."""
    prm = small_test_params()
    ctx = HipContext.from_params(prm)
    n, t = prm.ring_degree, prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=1)
    els, gks = ctx.gen_trace_galois_keys(sk, KEY, stream=100)
    assert els == list(range(3, 2 * n, 2))
    ct = _encrypt(ctx, prm, [42], sk, 2)
    dec = ctx.bfv_decrypt(ctx.extract_coefficient(ct, 0, els, gks)[None], sk)
    assert int(dec[0, 0]) == 42
    ct = _encrypt(ctx, prm, [5, 10, 15], sk, 3)
    for j, want in enumerate((5, 10, 15)):
        dec = ctx.bfv_decrypt(ctx.extract_coefficient(ct, j, els, gks)[None], sk)
        assert int(dec[0, 0]) == want, j
    coeffs = [i % t for i in range(1, n + 1)]
    ct = _encrypt(ctx, prm, coeffs, sk, 4)
    slots = ctx.coeffs_to_slots(ct, els, gks)
    assert slots.shape[0] == n
    dec = ctx.bfv_decrypt(slots, sk)
    assert [int(v) for v in dec[:, 0]] == coeffs
    recon = ctx.slots_to_coeffs(slots)
    dec = ctx.bfv_decrypt(recon[None], sk)
    assert [int(v) for v in dec[0]] == coeffs


def test_chain_trace_decrypts(gpu_available):
    """The relative-trace chain (n = 64 > 32): extraction decrypts to the coefficient."""
    prm = P.cfg3_params(64)
    ctx = HipContext.from_params(prm)
    sk = ctx.gen_secret_key(KEY, stream=5)
    els, gks = ctx.gen_trace_galois_keys(sk, KEY, stream=200)
    assert els == [65, 33, 17, 9, 5, 3]
    coeffs = [(7 * i + 3) % prm.plain_modulus for i in range(64)]
    ct = _encrypt(ctx, prm, coeffs, sk, 6)
    out = ctx.extract_coefficients(ct, 0, 64, els, gks)
    dec = ctx.bfv_decrypt(out, sk)
    assert [int(v) for v in dec[:, 0]] == coeffs
    assert not dec[:, 1:].any()


def test_errors(gpu_available):
    prm = small_test_params()
    ctx = HipContext.from_params(prm)
    n = prm.ring_degree
    ct = np.zeros((2, 1, n), dtype=np.uint64)
    els = ctx.required_trace_elements()
    gks = np.zeros((len(els), 2, 2, 1, n), dtype=np.uint64)
    with pytest.raises(ExactoError) as e:
        ctx.extract_coefficient(ct, 1, els[:-1], gks[:-1])
    assert e.value.variant == "InvalidParam" and f"missing Galois key for element {els[-1]}" in str(e.value)
    with pytest.raises(ExactoError) as e:
        ctx.slots_to_coeffs(np.zeros((0, 2, 1, n), dtype=np.uint64))
    assert e.value.variant == "InvalidParam" and "empty slots" in str(e.value)
    with pytest.raises(ExactoError) as e:
        ctx.slots_to_coeffs(np.zeros((3, 2, 1, n), dtype=np.uint64))
    assert e.value.variant == "InvalidParam" and f"expected {n} slots, got 3" in str(e.value)
    even = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(256).ct_moduli([1125899906842817])
            .gadget_base(8).build())
    ctx2 = HipContext.from_params(even)
    with pytest.raises(ExactoError) as e:
        ctx2.extract_coefficient(ct, 0, els, gks)
    assert e.value.variant == "InvalidParam" and "n not invertible mod t" in str(e.value)
