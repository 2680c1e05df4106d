"""Device-resident dBFV chain: exacto_dbfv_mul_chain[_dev].

Semantics: paper_repro.rs:203-236 (acc <- dbfv_mul(acc, y) with both mul_depth reset to 0
before every step).  Checked bit-exactly against repeated single dbfv_mul calls and against the
oracle's guard-bypassed chain, and at decrypt level (5 * 3^k mod p) while noise allows.
"""
import random

import numpy as np
import pytest

from oracle import bfv as obfv, dbfv as odbfv, params as P
from exacto_amd._ffi import HipContext
from bridge import ct_to_np, np_to_ct, rlk_to_np, uniform_residues

pytestmark = pytest.mark.gpu


def test_chain_equals_repeated_mul(gpu_available):
    dp = P.compact_dbfv()
    prm = dp.bfv_params
    rng = np.random.default_rng(11)
    ctx = HipContext.from_params(prm)
    G = ctx.G
    rlk = uniform_residues(rng, (G, 2), prm.ct_basis.moduli, prm.ring_degree)
    ctx.load_relin_key(rlk)
    d = dp.num_digits
    x = uniform_residues(rng, (3, d, 2), prm.ct_basis.moduli, prm.ring_degree)
    y = uniform_residues(rng, (3, d, 2), prm.ct_basis.moduli, prm.ring_degree)
    acc = x
    for depth in range(4):
        got = ctx.dbfv_mul_chain(d, dp.base, dp.plain_modulus, x, y, depth)
        assert np.array_equal(got, acc), depth
        acc, _ = ctx.dbfv_mul(d, dp.base, dp.plain_modulus, acc, y)


def test_chain_matches_oracle_and_decrypts(gpu_available):
    dp = P.compact_dbfv()
    prm = dp.bfv_params
    r = random.Random(7)
    sk = obfv.gen_secret_key(prm, r)
    rlk = obfv.gen_relin_key(sk, r)
    ctx = HipContext.from_params(prm)
    ctx.load_relin_key(rlk_to_np(rlk))
    ca = odbfv.dbfv_encrypt_scalar_sk(5, sk, dp, r)
    cf = odbfv.dbfv_encrypt_scalar_sk(3, sk, dp, r)
    X = np.stack([ct_to_np(l) for l in ca.limbs])[None]
    Y = np.stack([ct_to_np(l) for l in cf.limbs])[None]
    d = dp.num_digits
    want = ca
    for depth in (1, 2):
        want = odbfv.dbfv_mul(want, cf, rlk, bypass_depth_guard=True)
        got = ctx.dbfv_mul_chain(d, dp.base, dp.plain_modulus, X, Y, depth)
        exp = np.stack([ct_to_np(l) for l in want.limbs])
        assert np.array_equal(got[0], exp), depth
        if depth == 1:  # fresh inputs: within the noise budget
            dec = odbfv.dbfv_decrypt_scalar(
                odbfv.DbfvCiphertext([np_to_ct(got[0, k], prm) for k in range(d)], d, 1, dp), sk)
            assert dec == 15 % dp.plain_modulus
