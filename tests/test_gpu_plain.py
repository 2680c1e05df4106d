"""Plaintext-ciphertext operations and the trace on the GPU (the linear
layer under CoeffsToSlots): exacto_bfv_plain_mul / plain_add / inner_product / monomial_mul /
trace.

Reference: bfv/eval.rs:468-503 (plain_mul, plain_add), 572-586 (trace), 588-606 (inner_product),
613-652 (monomial_mul).  Bit-exact against the oracle restatements (oracle/bfv.py) on uniform
ciphertexts, keys and plaintexts for a single prime, two primes with Q < 2^64 (the reference's
own CRT is exact there) and cfg3's 3x60-bit basis under the extension semantics; plus the
reference's decrypt-level test_plain_add (eval.rs:978-994) and decrypt-level checks of the other
operations on device-generated keys.
"""
import numpy as np
import pytest

from oracle import bfv as obfv, params as P
from oracle.ring import CoeffPoly
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues

pytestmark = pytest.mark.gpu

KEY = [5, 6, 7, 8]

PARAMS = {
    "compact": P.compact_bfv,
    "multiprime16": lambda: P.BfvParamsBuilder().ring_degree(16).plain_modulus(257)
    .ct_moduli([65537, 1099509805057]).gadget_base(8).build(),
    "cfg3_n64": lambda: P.cfg3_params(64),
}


def _pt(row, p):
    return CoeffPoly([int(v) for v in row], p)


def _plaintexts(rng, rows, n, p):
    pt = rng.integers(0, p, size=(rows, n), dtype=np.uint64)
    pt[0, :4] = [0, 1, p - 1, 2**64 - 1]  # any u64 is accepted and reduced mod each q_i
    return pt


@pytest.mark.parametrize("which", sorted(PARAMS))
def test_plain_mul_add_match_oracle(gpu_available, which):
    prm = PARAMS[which]()
    n, q, p = prm.ring_degree, prm.ct_basis.moduli, prm.plain_modulus
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(23)
    for polys in (2, 3):
        ct = uniform_residues(rng, (3, polys), q, n)
        pt = _plaintexts(rng, 3, n, p)
        got_mul = ctx.bfv_plain_mul(ct, pt)
        got_add = ctx.bfv_plain_add(ct, pt)
        for b in range(3):
            oc = np_to_ct(ct[b], prm)
            assert np.array_equal(got_mul[b], ct_to_np(obfv.bfv_plain_mul(oc, _pt(pt[b], p)))), (which, polys, b)
            assert np.array_equal(got_add[b], ct_to_np(obfv.bfv_plain_add(oc, _pt(pt[b], p)))), (which, polys, b)


@pytest.mark.parametrize("which", sorted(PARAMS))
def test_inner_product_matches_oracle(gpu_available, which):
    prm = PARAMS[which]()
    n, q, p = prm.ring_degree, prm.ct_basis.moduli, prm.plain_modulus
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(29)
    for K in (1, 4):
        cts = uniform_residues(rng, (K, 2), q, n)
        pts = _plaintexts(rng, K, n, p)
        got = ctx.bfv_inner_product(cts, pts)
        acc = obfv.bfv_plain_mul(np_to_ct(cts[0], prm), _pt(pts[0], p))
        for k in range(1, K):
            acc = obfv.bfv_add(acc, obfv.bfv_plain_mul(np_to_ct(cts[k], prm), _pt(pts[k], p)))
        assert np.array_equal(got, ct_to_np(acc)), (which, K)
    with pytest.raises(ExactoError) as e:
        ctx.bfv_inner_product(np.zeros((0, 2, len(q), n), dtype=np.uint64), np.zeros((0, n), dtype=np.uint64))
    assert e.value.variant == "InvalidParam" and "mismatched ct/pt lengths" in str(e.value)


@pytest.mark.parametrize("which", sorted(PARAMS))
def test_monomial_mul_matches_oracle(gpu_available, which):
    prm = PARAMS[which]()
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(31)
    ct = uniform_residues(rng, (2, 2), q, n)
    for j in (0, 1, 7, n - 1, n, n + 3, 2 * n - 1, 2 * n, 5 * n + 2):
        got = ctx.bfv_monomial_mul(ct, j)
        for b in range(2):
            want = ct_to_np(obfv.bfv_monomial_mul(np_to_ct(ct[b], prm), j))
            assert np.array_equal(got[b], want), (which, j, b)


@pytest.mark.parametrize("which", sorted(PARAMS))
def test_trace_matches_oracle(gpu_available, which):
    prm = PARAMS[which]()
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(37)
    ct = uniform_residues(rng, (2, 2), q, n)
    elements = [n + 1, 3, 2 * n - 1]
    nk = prm.gadget_digits
    gks = uniform_residues(rng, (len(elements), nk, 2), q, n)
    got = ctx.bfv_trace(ct, elements, gks)
    keys = {k: obfv.GaloisKey(np_to_rlk(gks[e], prm).keys, k, prm) for e, k in enumerate(elements)}
    for b in range(2):
        want = ct_to_np(obfv.bfv_trace(np_to_ct(ct[b], prm), elements, keys))
        assert np.array_equal(got[b], want), (which, b)
    # no elements: a clone
    assert np.array_equal(ctx.bfv_trace(ct, [], gks[:0]), ct)


def test_reference_plain_add_and_decrypt_level(gpu_available):
    """eval.rs:978-994 (10 + 5 = 15), then plain_mul, monomial_mul, inner_product and the trace
    checked through decryption with device-generated keys."""
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    n, p = prm.ring_degree, prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=1)
    pt = np.zeros((2, n), dtype=np.uint64)
    pt[0, 0] = 10
    pt[1, 0], pt[1, 1], pt[1, 2] = 1, 2, 3           # 1 + 2X + 3X^2
    ct = ctx.encrypt_sk(pt, sk, KEY, stream=2)
    add = np.zeros((2, n), dtype=np.uint64)
    add[:, 0] = 5
    dec = ctx.bfv_decrypt(ctx.bfv_plain_add(ct, add), sk)
    assert int(dec[0, 0]) == 15 and not dec[0, 1:].any()
    assert [int(v) for v in dec[1, :3]] == [6, 2, 3]
    mul = np.zeros((2, n), dtype=np.uint64)
    mul[:, 0] = 7
    dec = ctx.bfv_decrypt(ctx.bfv_plain_mul(ct, mul), sk)
    assert int(dec[0, 0]) == 70 % p and [int(v) for v in dec[1, :3]] == [7, 14, 21]
    # X^(n-1) (1 + 2X + 3X^2) = X^(n-1) - 2 - 3X
    dec = ctx.bfv_decrypt(ctx.bfv_monomial_mul(ct, n - 1), sk)
    assert [int(dec[1, 0]), int(dec[1, 1]), int(dec[1, n - 1])] == [p - 2, p - 3, 1]
    ip = ctx.bfv_inner_product(ct, mul)                # 10*7 + (1 + 2X + 3X^2)*7
    dec = ctx.bfv_decrypt(ip[None], sk)
    assert [int(v) for v in dec[0, :3]] == [(70 + 7) % p, 14, 21]
    # sigma_{n+1}: X^i -> (-1)^i X^i, so m + sigma(m) doubles the even coefficients, clears the odd
    gk = ctx.gen_galois_key(sk, n + 1, KEY, stream=3)
    dec = ctx.bfv_decrypt(ctx.bfv_trace(ct, [n + 1], gk[None]), sk)
    assert [int(v) for v in dec[1, :3]] == [2, 0, 6] and int(dec[0, 0]) == 20


def test_trace_requires_degree_one(gpu_available):
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    n = prm.ring_degree
    ct3 = np.zeros((1, 3, 1, n), dtype=np.uint64)
    gks = np.zeros((1, prm.gadget_digits, 2, 1, n), dtype=np.uint64)
    with pytest.raises(ExactoError) as e:
        ctx.bfv_trace(ct3, [3], gks)
    assert e.value.variant == "InvalidParam" and "automorphism requires degree-1 ciphertext" in str(e.value)
