"""Batched decryption on the GPU: exacto_bfv_decrypt / exacto_dbfv_decrypt[_poly].

Reference: bfv/encrypt.rs:111-178 (exact BigUint CRT and rounding, so parity is pinned for every
Q), dbfv/decrypt.rs:20-79 and dbfv/decomposition.rs:45-68, 112-127.  Bit-exact against the oracle
on uniform ciphertexts (degree 1 and 2) and on genuine encryptions.
"""
import random

import numpy as np
import pytest

from oracle import bfv as obfv, dbfv as odbfv, params as P
from oracle.ring import CoeffPoly
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, rns_to_np, uniform_residues

pytestmark = pytest.mark.gpu


def _setup(prm, seed):
    r = random.Random(seed)
    sk = obfv.gen_secret_key(prm, r)
    ctx = HipContext.from_params(prm)
    return ctx, sk, rns_to_np(sk.poly), r


@pytest.mark.parametrize("which", ["compact", "small", "cfg3_n1024", "cfg3"])
def test_bfv_decrypt_uniform_matches_oracle(gpu_available, which):
    prm = {"compact": P.compact_bfv, "small": P.small_bfv, "cfg3_n1024": lambda: P.cfg3_params(1024),
           "cfg3": P.cfg3_params}[which]()
    ctx, sk, sk_np, _ = _setup(prm, 3)
    rng = np.random.default_rng(5)
    n, moduli = prm.ring_degree, prm.ct_basis.moduli
    for polys in (2, 3):
        ct = uniform_residues(rng, (3, polys), moduli, n)
        got = ctx.bfv_decrypt(ct, sk_np)
        for b in range(3):
            want = obfv.decrypt(np_to_ct(ct[b], prm), sk).coeffs
            assert [int(v) for v in got[b]] == want, (which, polys, b)


@pytest.mark.parametrize("which", ["compact", "cfg3"])
def test_bfv_decrypt_genuine_and_products(gpu_available, which):
    prm = {"compact": P.compact_bfv, "cfg3": P.cfg3_params}[which]()
    ctx, sk, sk_np, r = _setup(prm, 9)
    rlk = obfv.gen_relin_key(sk, r)
    from bridge import rlk_to_np
    ctx.load_relin_key(rlk_to_np(rlk))
    msgs = [(3, 7), (0, 5), (prm.plain_modulus - 1, 2), (12, 12)]
    c1 = np.stack([ct_to_np(obfv.encrypt_sk(obfv.encode_scalar(a, prm), sk, r)) for a, _ in msgs])
    c2 = np.stack([ct_to_np(obfv.encrypt_sk(obfv.encode_scalar(b, prm), sk, r)) for _, b in msgs])
    dec = ctx.bfv_decrypt(c1, sk_np)
    assert [int(d[0]) for d in dec] == [a for a, _ in msgs]
    assert not dec[:, 1:].any()
    prod = ctx.bfv_mul_and_relin(c1, c2)
    dec = ctx.bfv_decrypt(prod, sk_np)
    assert [int(d[0]) for d in dec] == [(a * b) % prm.plain_modulus for a, b in msgs]


def test_dbfv_decrypt_matches_oracle(gpu_available):
    dp = P.compact_dbfv()
    prm = dp.bfv_params
    ctx, sk, sk_np, r = _setup(prm, 21)
    d = dp.num_digits
    xs = [0, 1, 3, 200, 255]
    cts = [odbfv.dbfv_encrypt_scalar_sk(x, sk, dp, r) for x in xs]
    arr = np.stack([np.stack([ct_to_np(l) for l in c.limbs]) for c in cts])
    got = ctx.dbfv_decrypt(d, dp.base, dp.plain_modulus, arr, sk_np)
    assert [int(v) for v in got] == xs
    poly = ctx.dbfv_decrypt_poly(d, dp.base, dp.plain_modulus, arr, sk_np)
    for k, c in enumerate(cts):
        assert [int(v) for v in poly[k]] == odbfv.dbfv_decrypt_poly(c, sk)
    # uniform limbs: centring and recomposition of arbitrary digit values
    rng = np.random.default_rng(8)
    u = uniform_residues(rng, (2, d, 2), prm.ct_basis.moduli, prm.ring_degree)
    poly = ctx.dbfv_decrypt_poly(d, dp.base, dp.plain_modulus, u, sk_np)
    sc = ctx.dbfv_decrypt(d, dp.base, dp.plain_modulus, u, sk_np)
    for k in range(2):
        c = odbfv.DbfvCiphertext([np_to_ct(u[k, i], prm) for i in range(d)], d, 0, dp)
        want = odbfv.dbfv_decrypt_poly(c, sk)
        assert [int(v) for v in poly[k]] == want
        assert int(sc[k]) == want[0] == odbfv.dbfv_decrypt_scalar(c, sk)


def test_dbfv_decrypt_u64_profile_scalar_and_error(gpu_available):
    # plain modulus 0 (= 2^64): scalar recomposition wraps; the poly form is rejected
    dp = P.u64_dbfv()
    prm = dp.bfv_params
    ctx, sk, sk_np, r = _setup(prm, 4)
    d = dp.num_digits
    x = (1 << 63) + 12345
    c = odbfv.dbfv_encrypt_scalar_sk(x, sk, dp, r)
    arr = np.stack([ct_to_np(l) for l in c.limbs])[None]
    assert int(ctx.dbfv_decrypt(d, dp.base, 0, arr, sk_np)[0]) == x == odbfv.dbfv_decrypt_scalar(c, sk)
    with pytest.raises(ExactoError, match="scalar-only"):
        ctx.dbfv_decrypt_poly(d, dp.base, 0, arr, sk_np)
