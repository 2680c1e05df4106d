"""Digit extraction on the GPU: exacto_trivial_encrypt, exacto_eval_poly
(Paterson-Stockmeyer over the device's bfv_mul_and_relin), with the host-side rounding polynomial.

Reference: bootstrap/digit_extract.rs:19-197.  Bit-exact against oracle/bootstrap.py on uniform
ciphertexts and relinearisation keys (the schoolbook path at the reference's bootstrap
parameters n = 16, t_boot = 29, and the exact-RNS path over cfg3's basis at n = 64); the reference's
test_trivial_encrypt_decrypt (digit_extract.rs:270-288); the rounding polynomial evaluated on
encryptions decrypts to round(t x / q') mod t.
"""
import numpy as np
import pytest

from oracle import bootstrap as ob, params as P
from oracle.ring import CoeffPoly
from exacto_amd import _ffi
from exacto_amd._ffi import HipContext, ExactoError
from bridge import ct_to_np, np_to_ct, np_to_rlk, uniform_residues

pytestmark = pytest.mark.gpu

KEY = [3, 1, 4, 1]


def boot_params(t_boot=29):
    """bfv_host.rs:383-399: n = 16, Q_boot = 1125899906842817, base 8."""
    return (P.BfvParamsBuilder().ring_degree(16).plain_modulus(t_boot).ct_moduli([1125899906842817])
            .sigma(3.2).gadget_base(8).build())


@pytest.mark.parametrize("which", ["boot16", "cfg3_n64"])
def test_trivial_encrypt_matches_oracle(gpu_available, which):
    prm = boot_params() if which == "boot16" else P.cfg3_params(64)
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(51)
    pt = rng.integers(0, 2**63, size=(3, prm.ring_degree), dtype=np.uint64)
    got = ctx.trivial_encrypt_poly(pt)
    for b in range(3):
        want = ob.trivial_encrypt_poly(CoeffPoly([int(v) for v in pt[b]], prm.plain_modulus), prm)
        assert np.array_equal(got[b], ct_to_np(want))
    got = ctx.trivial_encrypt([5, prm.plain_modulus + 2])
    for b, m in enumerate((5, prm.plain_modulus + 2)):
        assert np.array_equal(got[b], ct_to_np(ob.trivial_encrypt(m, prm)))


def test_reference_trivial_encrypt_decrypt(gpu_available):
    """digit_extract.rs:270-288 on compact_bfv."""
    prm = P.compact_bfv()
    ctx = HipContext.from_params(prm)
    sk = ctx.gen_secret_key(KEY, stream=1)
    ms = [0, 1, 42, 100, 256]
    dec = ctx.bfv_decrypt(ctx.trivial_encrypt(ms), sk)
    assert [int(v) for v in dec[:, 0]] == ms and not dec[:, 1:].any()


@pytest.mark.parametrize("which,coeffs", [
    ("boot16", [7]),
    ("boot16", [3, 1]),
    ("boot16", [1, 2, 3, 4]),
    ("boot16", [0, 5, 0, 0, 9, 28, 1, 0, 2]),
    ("boot16", "rounding"),
    ("cfg3_n64", [11, 0, 7, 65536, 3, 2]),
])
def test_eval_poly_matches_oracle(gpu_available, which, coeffs):
    prm = boot_params() if which == "boot16" else P.cfg3_params(64)
    n, q = prm.ring_degree, prm.ct_basis.moduli
    if coeffs == "rounding":
        coeffs = ob.compute_rounding_poly(5, 25, 29)
    ctx = HipContext.from_params(prm)
    rng = np.random.default_rng(53 + len(coeffs))
    ct = uniform_residues(rng, (2, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    ctx.load_relin_key(rlk)
    got = ctx.eval_poly(ct, coeffs)
    orlk = np_to_rlk(rlk, prm)
    for b in range(2):
        want = ob.eval_poly_homomorphic(np_to_ct(ct[b], prm), list(coeffs), orlk)
        assert np.array_equal(got[b], ct_to_np(want)), (which, len(coeffs), b)


def test_rounding_poly_decrypts(gpu_available):
    """The bootstrap's digit-extraction step (bfv_host.rs:176-184): g(x) on trivial encryptions of every
    x in [0, t_boot) decrypts to round(t x / q') mod t (t = 5, q' = 25, t_boot = 29)."""
    prm = boot_params()
    ctx = HipContext.from_params(prm)
    sk = ctx.gen_secret_key(KEY, stream=2)
    ctx.gen_relin_key(sk, KEY, stream=3, resident=True)
    g = _ffi.compute_rounding_poly(5, 25, 29)
    xs = list(range(29))
    out = ctx.eval_poly(ctx.trivial_encrypt(xs), g)
    dec = ctx.bfv_decrypt(out, sk)
    assert [int(v) % 5 for v in dec[:, 0]] == [(5 * (x % 25) + 12) // 25 % 5 for x in xs]


def test_eval_poly_on_fresh_encryptions(gpu_available):
    """x^3 + 2x + 1 on fresh encryptions decrypts to the value mod t (device keys, cfg3 at n = 64)."""
    prm = P.cfg3_params(64)
    ctx = HipContext.from_params(prm)
    t = prm.plain_modulus
    sk = ctx.gen_secret_key(KEY, stream=4)
    ctx.gen_relin_key(sk, KEY, stream=5, resident=True)
    xs = [0, 1, 2, 7, 1000, t - 1]
    pt = np.zeros((len(xs), prm.ring_degree), dtype=np.uint64)
    pt[:, 0] = xs
    ct = ctx.encrypt_sk(pt, sk, KEY, stream=6)
    dec = ctx.bfv_decrypt(ctx.eval_poly(ct, [1, 2, 0, 1]), sk)
    assert [int(v) for v in dec[:, 0]] == [(x**3 + 2 * x + 1) % t for x in xs]


def test_errors(gpu_available):
    prm = boot_params()
    ctx = HipContext.from_params(prm)
    ct = np.zeros((1, 2, 1, prm.ring_degree), dtype=np.uint64)
    with pytest.raises(ExactoError) as e:
        ctx.eval_poly(ct, [1, 2])
    assert e.value.variant == "MissingKey"
    with pytest.raises(ExactoError) as e:
        ctx.eval_poly(ct, [])
    assert e.value.variant == "InvalidParam"
    # degree 0 needs no key: trivial_encrypt(a_0)
    assert np.array_equal(ctx.eval_poly(ct, [30])[0], ct_to_np(ob.trivial_encrypt(30, prm)))
