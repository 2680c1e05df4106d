"""Galois automorphisms on the GPU: exacto_gen_galois_key,
exacto_bfv_apply_automorphism.

Reference: bfv/eval.rs:512-561 (bfv_apply_automorphism), bfv/keygen.rs:171-262 (gen_galois_key,
apply_automorphism).  Bit-exact against the oracle restatement on uniform ciphertexts and keys
(single prime with HPS, multi-prime Q < 2^64 where the reference's own CRT is exact, and cfg3's
3x60-bit basis under the extension semantics), for odd and even elements; key structure checked
exactly; the reference's decrypt-level tests (eval.rs:930-976) on device-generated keys.
"""
import numpy as np
import pytest

from oracle import bfv as obfv, params as P
from oracle.ring import CoeffPoly
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, np_to_rns, np_to_rlk, uniform_residues

pytestmark = pytest.mark.gpu

KEY = [11, 22, 33, 44]

PARAMS = {
    "compact": P.compact_bfv,
    "multiprime16": lambda: P.BfvParamsBuilder().ring_degree(16).plain_modulus(257)
    .ct_moduli([65537, 1099509805057]).gadget_base(8).build(),
    "cfg3_n64": lambda: P.cfg3_params(64),
}


def oracle_auto(prm, ct, element, gk):
    keys = np_to_rlk(gk, prm).keys
    return ct_to_np(obfv.bfv_apply_automorphism(np_to_ct(ct, prm), obfv.GaloisKey(keys, element, prm)))


@pytest.mark.parametrize("which", sorted(PARAMS))
def test_automorphism_matches_oracle(gpu_available, which):
    prm = PARAMS[which]()
    n, q = prm.ring_degree, prm.ct_basis.moduli
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(17)
    ct = uniform_residues(rng, (3, 2), q, n)
    for element in (3, 5, 2 * n - 1, 2, 4 * n + 3):
        for nk in (prm.gadget_digits, 2):
            gk = uniform_residues(rng, (nk, 2), q, n)
            got = ctx.bfv_apply_automorphism(ct, element, gk)
            for b in (0, 2):
                assert np.array_equal(got[b], oracle_auto(prm, ct[b], element, gk)), (which, element, nk, b)


@pytest.mark.parametrize("which", ["compact", "cfg3_n64"])
def test_galois_key_structure(gpu_available, which):
    prm = PARAMS[which]()
    ctx = HipContext.from_params(prm)
    q = prm.ct_basis.moduli
    sk = ctx.gen_secret_key(KEY, stream=1)
    skp = np_to_rns(sk, prm.ct_basis)
    element = 5
    gk = ctx.gen_galois_key(sk, element, KEY, stream=2)
    s_auto = obfv.galois_s_auto(skp, element, prm.ct_basis)
    for g in range(prm.gadget_digits):
        neg_e = np_to_rns(gk[g, 0], prm.ct_basis).add(np_to_rns(gk[g, 1], prm.ct_basis).mul(skp)) \
            .sub(s_auto.scalar_mul(pow(prm.gadget_base, g)))
        e = [[(-x) % qi for x in limb] for limb, qi in zip(neg_e.limb_coeffs(), q)]
        v0 = e[0]
        for i in range(1, len(q)):  # reference sampling semantics: limb i = (value mod q0) mod q_i
            assert e[i] == [x % q[i] for x in v0]
        assert all(min(x, q[0] - x) <= 20 for x in v0)


@pytest.mark.parametrize("which", ["compact", "cfg3_n64"])
def test_reference_decrypt_level_cases(gpu_available, which):
    prm = PARAMS[which]()
    ctx = HipContext.from_params(prm)
    n, p = prm.ring_degree, prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=3)
    gk3 = ctx.gen_galois_key(sk, 3, KEY, stream=4)
    pt = np.zeros((2, n), dtype=np.uint64)
    pt[0, 0] = 10                     # eval.rs:930-951: a scalar survives sigma_3
    pt[1, 0], pt[1, 1] = 1, 2         # eval.rs:954-976: 1 + 2X -> 1 + 2X^3
    ct = ctx.encrypt_sk(pt, sk, KEY, stream=5)
    dec = ctx.bfv_decrypt(ctx.bfv_apply_automorphism(ct, 3, gk3), sk)
    assert int(dec[0, 0]) == 10 and not dec[0, 1:].any()
    assert [int(v) for v in dec[1, :4]] == [1, 0, 0, 2] and not dec[1, 4:].any()
    # sigma_{2n-1}: X -> X^-1 = -X^(n-1)
    gkc = ctx.gen_galois_key(sk, 2 * n - 1, KEY, stream=6)
    dec = ctx.bfv_decrypt(ctx.bfv_apply_automorphism(ct, 2 * n - 1, gkc), sk)
    assert int(dec[1, 0]) == 1 and int(dec[1, n - 1]) == (p - 2) % p


def test_errors(gpu_available):
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    ct3 = np.zeros((1, 3, 1, prm.ring_degree), dtype=np.uint64)
    gk = np.zeros((3, 2, 1, prm.ring_degree), dtype=np.uint64)
    with pytest.raises(ExactoError) as e:
        ctx.bfv_apply_automorphism(ct3, 3, gk)
    assert e.value.variant == "InvalidParam" and "automorphism requires degree-1 ciphertext" in str(e.value)
    with pytest.raises(ExactoError):
        ctx.bfv_apply_automorphism(ct3[:, :2], 3, gk[:0])
