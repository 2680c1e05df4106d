"""The relinearisation key switch over the integers in an auxiliary basis of 31-bit primes
(exacto_amd/csrc/ks32.hip) against the limb-wise 60-bit MAC it replaces (EXACTO_KS32=0) and
against the oracle.

Reference: relinearize (src/bfv/keyswitch.rs:59-101), the MAC loop keyswitch.rs:86-95, inside
bfv_mul_and_relin (src/bfv/eval.rs:73-82) and dbfv_mul (src/dbfv/eval.rs:82-149).  Bit-exact:
integer work.  Sizes cover every transform length the basis is used at (n = 1024 .. 8192), the
BASELINE bases (3 and 4 limbs of ~60 bits, gadget bases 2^16 and 256, G = 12 and 30), keys with
fewer digits than G, and batches that span several pipeline chunks on both lanes.
"""

import os

import numpy as np
import pytest

from oracle import bfv as obfv, params as P
from exacto_amd._ffi import HipContext
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues

pytestmark = pytest.mark.gpu


def _ctx(prm, ks32: bool, chunk=0):
    old = os.environ.get("EXACTO_KS32")
    os.environ["EXACTO_KS32"] = "1" if ks32 else "0"
    try:
        ctx = HipContext.from_params(prm, device=0)
    finally:
        if old is None:
            del os.environ["EXACTO_KS32"]
        else:
            os.environ["EXACTO_KS32"] = old
    if chunk:
        ctx.set_chunk(chunk)
    return ctx


def _params(which, n):
    if which == "cfg3":
        return P.cfg3_params(n)
    if which == "q2":
        return P.BfvParamsBuilder().ring_degree(n).plain_modulus(65537).ct_moduli(P.Q3[1:]).build()
    if which == "q4b16":   # four limbs at base 2^16: a four-prime 31-bit basis (ks32_crt's S = 4 kernels)
        return P.BfvParamsBuilder().ring_degree(n).plain_modulus(65537).ct_moduli(P.Q4).build()
    return P.cfg5_params(n).bfv_params


@pytest.mark.parametrize("n,which,B,keys,chunk", [
    (1024, "cfg3", 5, None, 0),
    (4096, "cfg3", 7, None, 3),        # 3 chunks: both pipeline lanes
    (4096, "cfg3", 2, 7, 0),           # a key with fewer digits than G (keyswitch.rs:87-89)
    (8192, "cfg5", 2, None, 0),
    (2048, "cfg3", 3, None, 0),        # the remaining transform lengths of the 31-bit basis
    (16384, "q2", 1, None, 0),         # n = 16384: cfg3's last two primes (== 1 mod 2^15)
    (8192, "q4b16", 2, None, 0),
])
def test_ks32_matches_limbwise_mac(gpu_available, n, which, B, keys, chunk):
    prm = _params(which, n)
    q = prm.ct_basis.moduli
    rng = np.random.default_rng(n + B)
    ct1 = uniform_residues(rng, (B, 2), q, n)
    ct2 = uniform_residues(rng, (B, 2), q, n)
    ct1[0, 1] = np.array(q, dtype=np.uint64)[:, None] - 1     # extreme c1 -> large third component
    rlk = uniform_residues(rng, (keys or prm.gadget_digits, 2), q, n)
    outs = []
    for ks in (True, False):
        ctx = _ctx(prm, ks, chunk)
        assert (ctx.ks32_primes > 0) == ks       # the 31-bit basis is in use exactly when asked
        if ks and which == "q4b16":
            assert ctx.ks32_primes == 4
        ctx.load_relin_key(rlk)
        outs.append(ctx.bfv_mul_and_relin(ct1, ct2))
    assert np.array_equal(outs[0], outs[1])
    if n <= 1024:
        want = ct_to_np(obfv.bfv_mul_and_relin(np_to_ct(ct1[0], prm), np_to_ct(ct2[0], prm), np_to_rlk(rlk, prm)))
        assert np.array_equal(outs[0][0], want)


def test_ks32_key_reload(gpu_available):
    """A second key load replaces the auxiliary-basis key (no stale conversion)."""
    prm = P.cfg3_params(1024)
    q = prm.ct_basis.moduli
    rng = np.random.default_rng(5)
    ct1 = uniform_residues(rng, (2, 2), q, 1024)
    ct2 = uniform_residues(rng, (2, 2), q, 1024)
    k1 = uniform_residues(rng, (prm.gadget_digits, 2), q, 1024)
    k2 = uniform_residues(rng, (prm.gadget_digits, 2), q, 1024)
    ctx, ref = _ctx(prm, True), _ctx(prm, False)
    for k in (k1, k2, k1):
        ctx.load_relin_key(k)
        ref.load_relin_key(k)
        assert np.array_equal(ctx.bfv_mul_and_relin(ct1, ct2), ref.bfv_mul_and_relin(ct1, ct2))


@pytest.mark.parametrize("n,which,B,keys,chunk", [
    (1024, "cfg3", 3, None, 0),
    (4096, "cfg3", 5, None, 2),        # 3 chunks
    (4096, "cfg3", 2, 5, 0),           # fewer Galois key digits than G (eval.rs:540-548)
    (8192, "cfg5", 2, None, 0),
    (8192, "q4b16", 2, None, 0),
])
def test_ks32_automorphism_matches_limbwise(gpu_available, n, which, B, keys, chunk):
    """bfv_apply_automorphism (eval.rs:512-561) with the ks32 key switch against the limb-wise
    60-bit MAC, for an odd and the conjugation element, and a new key in every call."""
    prm = _params(which, n)
    q = prm.ct_basis.moduli
    rng = np.random.default_rng(3 * n + B)
    ct = uniform_residues(rng, (B, 2), q, n)
    ct[0, 1] = np.array(q, dtype=np.uint64)[:, None] - 1
    ctxs = [_ctx(prm, True, chunk), _ctx(prm, False, chunk)]
    assert ctxs[0].ks32_primes > 0 and ctxs[1].ks32_primes == 0
    for element in (5, 2 * n - 1):
        gk = uniform_residues(rng, (keys or prm.gadget_digits, 2), q, n)
        got, want = (c.bfv_apply_automorphism(ct, element, gk) for c in ctxs)
        assert np.array_equal(got, want), (n, element)
        if n <= 1024:
            keyset = obfv.GaloisKey(np_to_rlk(gk, prm).keys, element, prm)
            assert np.array_equal(got[0], ct_to_np(obfv.bfv_apply_automorphism(np_to_ct(ct[0], prm), keyset)))
