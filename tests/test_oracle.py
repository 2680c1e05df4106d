"""CPU: pin the oracle against the reference's own known-answer tests and functional tests.

tests/golden/kats.json transcribes every KAT the reference holds for this path (each entry
cites the reference test line).  The C restatement (oracle/c) is cross-checked against the
Python restatement on every dispatch branch, and both against the committed vectors.
"""

import json
import os
import random

import numpy as np
import pytest

from oracle import bfv as obfv, dbfv as odbfv, modular as om, params as P, cref
from oracle.ring import CoeffPoly, ExactoError, NttPlan, NttPoly, RnsBasis, RnsPoly, make_plan
from bridge import ct_to_np, np_to_ct, np_to_rlk, rlk_to_np, uniform_residues

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_kats():
    with open(os.path.join(GOLD, "kats.json")) as f:
        return json.load(f)


def _eval_kat(k):
    fn, a = k["fn"], k["args"]
    if fn == "barrett_reduce":
        return om.barrett_reduce(a[0], a[1], om.barrett_constant(a[1]))
    if fn in ("mod_mul",):
        return om.mod_mul(a[0], a[1], a[2])
    if fn == "mod_add":
        return om.mod_add(*a)
    if fn == "mod_sub":
        return om.mod_sub(*a)
    if fn == "mod_neg":
        return om.mod_neg(*a)
    if fn == "mod_pow":
        return om.mod_pow(*a)
    if fn == "mod_inv_times_a":
        return om.mod_mul(a[0], om.mod_inv(a[0], a[1]), a[1])
    if fn == "montgomery_check":
        return (a[0] * om.montgomery_inv_neg(a[0]) + 1) % (1 << 64)
    if fn == "montgomery_reduce_am":
        return om.montgomery_reduce(a[0] * a[1], a[1], om.montgomery_inv_neg(a[1]))
    if fn == "poly_add":
        return CoeffPoly.from_coeffs(a[0], a[2]).add(CoeffPoly.from_coeffs(a[1], a[2])).coeffs
    if fn == "poly_sub":
        return CoeffPoly.from_coeffs(a[0], a[2]).sub(CoeffPoly.from_coeffs(a[1], a[2])).coeffs
    if fn == "poly_neg_add_is_zero":
        p = CoeffPoly.from_coeffs(a[0], a[1])
        return p.add(p.neg()).coeffs
    if fn == "mul_naive":
        return CoeffPoly.from_coeffs(a[0], a[2]).mul_naive(CoeffPoly.from_coeffs(a[1], a[2])).coeffs
    if fn == "scalar_mul":
        return CoeffPoly.from_coeffs(a[0], a[2]).scalar_mul(a[1]).coeffs
    if fn == "centered_coeffs":
        return CoeffPoly.from_coeffs(a[0], a[1]).centered_coeffs()
    if fn in ("ntt_roundtrip", "ntt_mul", "ntt_add"):
        n, q = (a[1], a[2]) if fn == "ntt_roundtrip" else (a[2], a[3])
        plan = make_plan(n, q)
        pad = lambda v: CoeffPoly.from_coeffs(v + [0] * (n - len(v)), q)
        x = NttPoly.from_coeff_poly(pad(a[0]), plan)
        if fn == "ntt_roundtrip":
            return x.to_coeff_poly().coeffs[:len(a[0])]
        y = NttPoly.from_coeff_poly(pad(a[1]), plan)
        return (x.mul(y) if fn == "ntt_mul" else x.add(y)).to_coeff_poly().coeffs
    if fn in ("rns_roundtrip", "rns_add", "rns_mul"):
        n, qs = (a[1], a[2]) if fn == "rns_roundtrip" else (a[2], a[3])
        basis = RnsBasis(qs, n)
        pad = lambda v: CoeffPoly.from_coeffs(v + [0] * (n - len(v)), qs[0])
        x = RnsPoly.from_coeff_poly(pad(a[0]), basis)
        if fn == "rns_roundtrip":
            return x.to_coeff_poly(basis).coeffs
        y = RnsPoly.from_coeff_poly(pad(a[1]), basis)
        return (x.add(y) if fn == "rns_add" else x.mul(y)).to_coeff_poly(basis).coeffs
    if fn == "gadget_decompose":
        return [d.coeffs for d in obfv.gadget_decompose(CoeffPoly.from_coeffs(a[0], a[1]), a[2], a[3])]
    if fn == "gadget_reconstruct":
        q, base, nd = a[1], a[2], a[3]
        digits = obfv.gadget_decompose(CoeffPoly.from_coeffs(a[0], q), base, nd)
        return [sum(digits[d].coeffs[i] * pow(base, d, q) for d in range(nd)) % q for i in range(len(a[0]))]
    if fn == "gadget_decompose_digit0":
        return obfv.gadget_decompose(CoeffPoly.from_coeffs(a[0], a[1]), a[2], a[3])[0].coeffs[0]
    if fn == "delta_residues":
        prm = P.BfvParamsBuilder().ring_degree(16).plain_modulus(a[1]).ct_moduli(a[0]).build()
        return obfv.delta_residues(prm)
    return None  # functional entries are exercised by dedicated tests below


@pytest.mark.parametrize("kat", load_kats(), ids=lambda k: f"{k['fn']}@{k['source']}")
def test_reference_kat(kat):
    got = _eval_kat(kat)
    if got is None:
        pytest.skip("functional KAT: covered by a dedicated decrypt-level test")
    assert got == kat["expected"], kat["source"]


@pytest.mark.parametrize("n,q", [(16, 65537), (64, 65537), (256, 65537)])
def test_ntt_convention_is_negacyclic_evaluation(n, q):
    """Position (k mod 16) n/16 + k // 16 holds a(psi^(2*brv(k)+1)) — the documented convention
    (the identity order at n = 16)."""
    plan = NttPlan(n, q)
    rng = random.Random(3)
    a = [rng.randrange(q) for _ in range(n)]
    ev = list(a)
    plan.fwd(ev)
    from oracle.ring import bit_reverse
    logn = n.bit_length() - 1
    for k in range(n):
        x = pow(plan.psi, 2 * bit_reverse(k, logn) + 1, q)
        assert ev[(k % 16) * (n // 16) + k // 16] == sum(c * pow(x, i, q) for i, c in enumerate(a)) % q
    assert pow(plan.psi, n, q) == q - 1
    back = list(ev)
    plan.inv(back)
    plan.normalize(back)
    assert back == a


def test_make_plan_errors():
    with pytest.raises(ExactoError) as e:
        make_plan(12, 65537)
    assert e.value.variant == "InvalidRingDegree"
    with pytest.raises(ExactoError) as e:
        make_plan(16, 65539)  # 65539 - 1 not divisible by 32
    assert "cannot create NTT plan" in str(e.value)


def test_kronecker_equals_schoolbook():
    rng = random.Random(11)
    for n in (128, 256):
        a = [rng.randrange(-2 ** 200, 2 ** 200) for _ in range(n)]
        b = [rng.randrange(-2 ** 200, 2 ** 200) for _ in range(n)]
        assert obfv.poly_mul_schoolbook(a, b) == obfv.poly_mul_exact(a, b)


def test_gadget_edge_cases():
    # balanced digits of boundary values, odd base (Rust truncating %), final carry dropped
    q = 65537
    for base in (2, 3, 5, 16, 256):
        nd = P.compute_gadget_digits([q], base)
        for c in range(0, q, 997):
            digs = obfv.gadget_decompose_coeff(c, q, base, nd)
            signed = [d - q if d > q // 2 else d for d in digs]
            assert all(-base <= s < base for s in signed)
            # reconstruction holds unless the final carry was dropped
            val = sum(s * base ** i for i, s in enumerate(signed))
            cc = c - q if c > q // 2 else c
            assert (val - cc) % (base ** nd) == 0


def test_gadget_digits_counts():
    assert P.compact_bfv().gadget_digits == 3
    assert P.u64_dbfv().bfv_params.gadget_digits == 8
    assert P.cfg3_params(16).gadget_digits == 12
    assert P.cfg5_params(16).bfv_params.gadget_digits == 30


def test_small_reps_all_zero_for_baseline_configs():
    assert all(v == 0 for r in odbfv.small_reps(256, 8, 0) for v in r)
    assert all(v == 0 for r in odbfv.small_reps(16, 2, 256) for v in r)
    assert all(v == 0 for r in odbfv.small_reps(256, 2, 65536) for v in r)
    # a non power: p = 1000, b = 7, d = 4 -> nonzero representatives
    assert any(v for r in odbfv.small_reps(7, 4, 1000) for v in r)


def test_baseline_primes():
    for q in P.Q4 + [18014398509998081, 36028797018972161, 1099509805057, 562949953443841]:
        assert om.is_prime(q)
    for q in P.Q4:
        assert (q - 1) % 16384 == 0


# ---------------------------------------------------------------- functional (decrypt-level)

def test_bfv_mul_decrypt_compact():
    """eval.rs:883-900: compact_bfv 3 * 7 = 21."""
    prm = P.compact_bfv()
    rng = random.Random(42)
    sk = obfv.gen_secret_key(prm, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    c1 = obfv.encrypt_sk(obfv.encode_scalar(3, prm), sk, rng)
    c2 = obfv.encrypt_sk(obfv.encode_scalar(7, prm), sk, rng)
    assert obfv.decode_scalar(obfv.decrypt(obfv.bfv_mul_and_relin(c1, c2, rlk), sk)) == 21


def test_bfv_mul_decrypt_multiprime():
    """eval.rs:903-927: Q = 65537 * 1099509805057, base 8."""
    prm = (P.BfvParamsBuilder().ring_degree(16).plain_modulus(257).ct_moduli([65537, 1099509805057])
           .sigma(3.2).gadget_base(8).build())
    rng = random.Random(1234)
    sk = obfv.gen_secret_key(prm, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    for a, b, e in [(3, 7, 21), (10, 20, 200), (0, 5, 0)]:
        c1 = obfv.encrypt_sk(obfv.encode_scalar(a, prm), sk, rng)
        c2 = obfv.encrypt_sk(obfv.encode_scalar(b, prm), sk, rng)
        assert obfv.decode_scalar(obfv.decrypt(obfv.bfv_mul_and_relin(c1, c2, rlk), sk)) == e


def test_dbfv_mul_decrypt_compact():
    """dbfv/eval.rs:223-237 and 272-290."""
    dp = P.compact_dbfv()
    rng = random.Random(42)
    sk = obfv.gen_secret_key(dp.bfv_params, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    for a, b in [(3, 7), (15, 15), (10, 20), (12, 12)]:
        ca = odbfv.dbfv_encrypt_scalar_sk(a, sk, dp, rng)
        cb = odbfv.dbfv_encrypt_scalar_sk(b, sk, dp, rng)
        r = odbfv.dbfv_mul(ca, cb, rlk)
        assert r.mul_depth == 1 and r.degree == 2
        assert odbfv.dbfv_decrypt_scalar(r, sk) == (a * b) % 256


def test_dbfv_depth_guard():
    """dbfv/eval.rs:292-313."""
    dp = P.compact_dbfv()
    rng = random.Random(777)
    sk = obfv.gen_secret_key(dp.bfv_params, rng)
    rlk = obfv.gen_relin_key(sk, rng)
    c1 = odbfv.dbfv_encrypt_scalar_sk(3, sk, dp, rng)
    c2 = odbfv.dbfv_encrypt_scalar_sk(7, sk, dp, rng)
    c12 = odbfv.dbfv_mul(c1, c2, rlk)
    with pytest.raises(ExactoError) as e:
        odbfv.dbfv_mul(c12, c1, rlk)
    assert "chained dBFV multiplication requires ciphertext-level lattice reduction" in str(e.value)


def test_hps_and_schoolbook_guards():
    """dbfv/eval.rs:385-453 parameters."""
    hps = (P.BfvParamsBuilder().ring_degree(4096).plain_modulus(1040407).ct_moduli([18014398509506561])
           .aux_moduli([36028797018972161]).gadget_base(256).build())
    with pytest.raises(ExactoError) as e:
        obfv.hps_check(hps)
    assert "single aux prime too small" in str(e.value)
    assert obfv.schoolbook_overflow_risk(1040407, 18014398509506561, 4096)


# ---------------------------------------------------------------- vectors / C restatement

def _meta():
    with open(os.path.join(GOLD, "vectors_meta.json")) as f:
        return json.load(f)


def _params(m):
    b = (P.BfvParamsBuilder().ring_degree(m["n"]).plain_modulus(m["plain"])
         .ct_moduli([int(x) for x in m["ct_moduli"]]).gadget_base(m["gadget_base"]))
    if m["aux_moduli"]:
        b = b.aux_moduli([int(x) for x in m["aux_moduli"]])
    return b.build()


@pytest.mark.parametrize("name", [k for k, v in _meta().items() if "d" not in v])
def test_python_oracle_reproduces_vectors(name):
    m = _meta()[name]
    prm = _params(m)
    z = np.load(os.path.join(GOLD, "vectors.npz"))
    ct1, ct2, rlk = z[f"{name}__ct1"], z[f"{name}__ct2"], z[f"{name}__rlk"]
    rk = np_to_rlk(rlk, prm)
    for b in range(ct1.shape[0]):
        got = obfv.bfv_mul_and_relin(np_to_ct(ct1[b], prm), np_to_ct(ct2[b], prm), rk)
        assert np.array_equal(ct_to_np(got), z[f"{name}__out"][b])


@pytest.mark.skipif(not cref.available(), reason="oracle/c not built")
@pytest.mark.parametrize("name", [k for k, v in _meta().items() if "d" not in v])
def test_c_oracle_reproduces_vectors(name):
    m = _meta()[name]
    prm = _params(m)
    z = np.load(os.path.join(GOLD, "vectors.npz"))
    ct1, ct2, rlk = z[f"{name}__ct1"], z[f"{name}__ct2"], z[f"{name}__rlk"]
    assert np.array_equal(cref.bfv_mul_and_relin(prm, ct1, ct2, rlk), z[f"{name}__out"])
    assert np.array_equal(cref.bfv_mul(prm, ct1, ct2, relin=False), z[f"{name}__out3"])


@pytest.mark.skipif(not cref.available(), reason="oracle/c not built")
def test_c_oracle_ntt_matches_python():
    n, q = 256, 1152921504606830593
    rng = np.random.default_rng(4)
    a = rng.integers(0, q, size=(2, n), dtype=np.uint64)
    got = cref.ntt(n, q, a)
    plan = make_plan(n, q)
    for r in range(2):
        v = [int(x) for x in a[r]]
        plan.fwd(v)
        assert [int(x) for x in got[r]] == v
    assert np.array_equal(cref.ntt(n, q, got, inverse=True), a)


@pytest.mark.parametrize("name", [k for k, v in _meta().items() if "d" in v])
def test_dbfv_vectors(name):
    m = _meta()[name]
    prm = _params(m)
    dp = P.DbfvParams(prm, m["base"], m["d"], m["dbfv_plain"])
    z = np.load(os.path.join(GOLD, "vectors.npz"))
    a, b, rlk = z[f"{name}__a"], z[f"{name}__b"], z[f"{name}__rlk"]
    rk = np_to_rlk(rlk, prm)
    d = m["d"]
    for i in range(a.shape[0]):
        A = odbfv.DbfvCiphertext([np_to_ct(a[i, k], prm) for k in range(d)], d, 0, dp)
        B = odbfv.DbfvCiphertext([np_to_ct(b[i, k], prm) for k in range(d)], d, 0, dp)
        r = odbfv.dbfv_mul(A, B, rk)
        assert np.array_equal(np.stack([ct_to_np(l) for l in r.limbs]), z[f"{name}__out"][i])


def test_apply_automorphism_kat():
    """keygen.rs:264-279: X -> X^3 on 1 + X + X^2 + X^3 in Z_17[X]/(X^4 + 1) = [1, 1, 16, 1]."""
    from oracle import bfv as obfv
    from oracle.ring import CoeffPoly
    assert obfv.apply_automorphism(CoeffPoly([1, 1, 1, 1], 17), 3).coeffs == [1, 1, 16, 1]
    # sigma_k then sigma_k^-1 is the identity (odd k)
    p = CoeffPoly([5, 0, 7, 1, 0, 0, 3, 2], 97)
    assert obfv.apply_automorphism(obfv.apply_automorphism(p, 3), 11).coeffs == p.coeffs  # 3 * 11 = 33 = 1 mod 16


def test_monomial_mul_poly_kat():
    """eval.rs:634-652: X^3 (1 + 2X + 3X^2) in Z_17[X]/(X^4 + 1) = -2 - 3X + X^3; X^(2n) is 1."""
    from oracle import bfv as obfv
    from oracle.ring import CoeffPoly
    assert obfv.monomial_mul_poly(CoeffPoly([1, 2, 3, 0], 17), 3, 4).coeffs == [15, 14, 0, 1]
    assert obfv.monomial_mul_poly(CoeffPoly([1, 2, 3, 0], 17), 4, 4).coeffs == [16, 15, 14, 0]
    assert obfv.monomial_mul_poly(CoeffPoly([1, 2, 3, 0], 17), 8, 4).coeffs == [1, 2, 3, 0]


@pytest.mark.parametrize("base,d,p", [(256, 2, 65536), (7, 4, 1000)])
def test_c_dbfv_mul_matches_python(base, d, p):
    """oracle/c oracle_dbfv_mul (all d^2 products, per-limb sums, reduce with reps) == the Python
    restatement (dbfv/eval.rs:82-149, reduction.rs:15-93); (7, 4, 1000) has non-zero reps."""
    if not cref.available():
        pytest.skip("oracle/c not built")
    from bridge import np_to_ct, ct_to_np, np_to_rlk, uniform_residues
    n = 16
    prm = P.BfvParamsBuilder().ring_degree(n).plain_modulus(1009).ct_moduli(P.Q3).build()
    dp = P.DbfvParams(prm, base, d, p)
    rng = np.random.default_rng(5)
    q = prm.ct_basis.moduli
    a = uniform_residues(rng, (2, d, 2), q, n)
    b = uniform_residues(rng, (2, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    got = cref.dbfv_mul(dp, a, b, rlk, threads=2)
    rk = np_to_rlk(rlk, prm)
    for it in range(2):
        ca = odbfv.DbfvCiphertext([np_to_ct(a[it, i], prm) for i in range(d)], d, 0, dp)
        cb = odbfv.DbfvCiphertext([np_to_ct(b[it, i], prm) for i in range(d)], d, 0, dp)
        want = np.stack([ct_to_np(l) for l in odbfv.dbfv_mul(ca, cb, rk).limbs])
        assert np.array_equal(got[it], want)


def test_c_dbfv_mul_hps_matches_python():
    """oracle/c oracle_dbfv_mul over the literal HPS multiplier (L = 1 with two aux primes, the
    u64_dbfv preset's basis, presets.rs:61-75, at n = 16) == the Python restatement: every one of the
    d^2 products dispatches to bfv_mul_hps (eval.rs:99-107, 157-413)."""
    if not cref.available():
        pytest.skip("oracle/c not built")
    from bridge import np_to_ct, ct_to_np, np_to_rlk, uniform_residues
    ref = P.u64_dbfv()
    b0 = ref.bfv_params
    n, d = 16, 8
    prm = (P.BfvParamsBuilder().ring_degree(n).plain_modulus(b0.plain_modulus).ct_moduli(b0.ct_basis.moduli)
           .aux_moduli(b0.aux_basis.moduli).gadget_base(b0.gadget_base).build())
    dp = P.DbfvParams(prm, 256, d, 0)
    rng = np.random.default_rng(9)
    q = prm.ct_basis.moduli
    a = uniform_residues(rng, (2, d, 2), q, n)
    b = uniform_residues(rng, (2, d, 2), q, n)
    rlk = uniform_residues(rng, (prm.gadget_digits, 2), q, n)
    got = cref.dbfv_mul(dp, a, b, rlk, threads=2)
    rk = np_to_rlk(rlk, prm)
    for it in range(2):
        ca = odbfv.DbfvCiphertext([np_to_ct(a[it, i], prm) for i in range(d)], d, 0, dp)
        cb = odbfv.DbfvCiphertext([np_to_ct(b[it, i], prm) for i in range(d)], d, 0, dp)
        want = np.stack([ct_to_np(l) for l in odbfv.dbfv_mul(ca, cb, rk).limbs])
        assert np.array_equal(got[it], want)


def test_c_polymul_matches_naive():
    """oracle_polymul (the cfg2 CPU baseline: NTT, pointwise, INTT, ntt.rs:181-195) == mul_naive."""
    if not cref.available():
        pytest.skip("oracle/c not built")
    n, q = 64, 1152921504606830593
    rng = np.random.default_rng(3)
    a = rng.integers(0, q, size=(3, n), dtype=np.uint64)
    b = rng.integers(0, q, size=(3, n), dtype=np.uint64)
    got = cref.polymul(n, q, a, b, threads=2)
    for k in range(3):
        want = CoeffPoly.from_coeffs([int(x) for x in a[k]], q).mul_naive(CoeffPoly.from_coeffs([int(x) for x in b[k]], q))
        assert [int(x) for x in got[k]] == want.coeffs
