"""L3 BFV scheme on the multiply path — restates reference src/bfv/{eval,keyswitch}.rs.

TEST ORACLE ONLY.  Exact Python integers stand in for Rust u128/i128/BigInt.
Key generation / encryption / decryption are *not* on the hot path; they are
included (mathematically, with this build's own sampler — the ChaCha20 stream
need not match because the hot path is deterministic given (ct1, ct2, rlk))
so that decrypt-level sanity tests mirroring the reference's can be written.
"""

from __future__ import annotations

import functools
import random

from .modular import barrett_constant, mod_inv, mod_mul, rust_div, rust_rem
from .ring import CoeffPoly, ExactoError, NttPoly, RnsPoly, crt_exact

_mod_inv = functools.lru_cache(maxsize=None)(mod_inv)


class BfvCiphertext:
    """bfv/mod.rs:19-24."""

    def __init__(self, c: list[RnsPoly], params):
        self.c = c
        self.params = params

    def degree(self):
        return len(self.c) - 1

    def clone(self):
        return BfvCiphertext([p.clone() for p in self.c], self.params)


class RelinKey:
    """bfv/keygen.rs:39-45: keys[i] = (rlk0_i, rlk1_i), NTT form."""

    def __init__(self, keys, params):
        self.keys = keys
        self.params = params


class SecretKey:
    def __init__(self, poly: RnsPoly, params, signed_coeffs):
        self.poly = poly
        self.params = params
        self.signed = signed_coeffs


# ------------------------------------------------------------------ add / sub / neg

def bfv_add(ct1, ct2):
    """eval.rs:14-31."""
    out = []
    for i in range(max(len(ct1.c), len(ct2.c))):
        a = ct1.c[i] if i < len(ct1.c) else None
        b = ct2.c[i] if i < len(ct2.c) else None
        out.append(a.add(b) if a is not None and b is not None else (a or b).clone())
    return BfvCiphertext(out, ct1.params)


def bfv_sub(ct1, ct2):
    """eval.rs:34-51."""
    out = []
    for i in range(max(len(ct1.c), len(ct2.c))):
        a = ct1.c[i] if i < len(ct1.c) else None
        b = ct2.c[i] if i < len(ct2.c) else None
        if a is not None and b is not None:
            out.append(a.sub(b))
        elif a is not None:
            out.append(a.clone())
        else:
            out.append(b.neg())
    return BfvCiphertext(out, ct1.params)


def bfv_neg(ct):
    """eval.rs:54-60."""
    return BfvCiphertext([c.neg() for c in ct.c], ct.params)


# ------------------------------------------------------------------ multiplication

def bfv_mul_and_relin(ct1, ct2, rlk):
    """eval.rs:73-82."""
    return relinearize(bfv_mul_no_relin(ct1, ct2), rlk)


def bfv_mul_no_relin(ct1, ct2):
    """eval.rs:89-108: dispatch multi-limb -> exact generic; aux -> HPS; else schoolbook."""
    if len(ct1.c) != 2 or len(ct2.c) != 2:
        raise ExactoError.invalid_param("multiplication requires degree-1 ciphertexts")
    params = ct1.params
    if params.ct_basis.num_moduli() > 1:
        return bfv_mul_generic_rns(ct1, ct2)
    if params.aux_basis is not None:
        return bfv_mul_hps(ct1, ct2)
    return bfv_mul_schoolbook(ct1, ct2)


# --- exact integer negacyclic product (eval.rs:669-686 i128 / 794-810 BigInt) ---

def poly_mul_schoolbook(a: list[int], b: list[int]) -> list[int]:
    """Literal O(n^2) negacyclic product over Z (eval.rs:794-810)."""
    n = len(a)
    res = [0] * n
    for i in range(n):
        ai = a[i]
        if ai == 0:
            continue
        for j in range(n):
            bj = b[j]
            if bj == 0:
                continue
            idx = i + j
            if idx < n:
                res[idx] += ai * bj
            else:
                res[idx - n] -= ai * bj
    return res


def _pack(vals, kb):
    return int.from_bytes(b"".join(v.to_bytes(kb, "little") for v in vals), "little")


def _unpack(x, kb, count):
    raw = x.to_bytes(kb * count, "little")
    return [int.from_bytes(raw[i * kb:(i + 1) * kb], "little") for i in range(count)]


def poly_mul_exact(a: list[int], b: list[int]) -> list[int]:
    """Same function as ``poly_mul_schoolbook`` (exact product over Z[X]/(X^n+1)), computed by
    Kronecker substitution so the oracle finishes n=4096 in seconds.  Cross-checked against the
    literal schoolbook in tests/test_oracle.py."""
    n = len(a)
    if n <= 64:
        return poly_mul_schoolbook(a, b)
    ma = max((abs(x) for x in a), default=0)
    mb = max((abs(x) for x in b), default=0)
    bound = 2 * n * ma * mb + 1
    kb = (bound.bit_length() + 8) // 8 + 1
    ap = _pack([x if x > 0 else 0 for x in a], kb)
    an = _pack([-x if x < 0 else 0 for x in a], kb)
    bp = _pack([x if x > 0 else 0 for x in b], kb)
    bn = _pack([-x if x < 0 else 0 for x in b], kb)
    pos = _unpack(ap * bp + an * bn, kb, 2 * n)
    neg = _unpack(ap * bn + an * bp, kb, 2 * n)
    lin = [p - q for p, q in zip(pos, neg)]
    return [lin[i] - lin[i + n] for i in range(n)]


def centered(vals: list[int], q: int) -> list[int]:
    """eval.rs:657-666 / 755: c > floor(q/2) -> c - q."""
    h = q // 2
    return [v - q if v > h else v for v in vals]


def reconstruct_centered_bigint(poly: RnsPoly, basis) -> list[int]:
    """eval.rs:719-762: INTT each limb, exact CRT, centre (> floor(Q/2) -> -Q)."""
    coeffs = crt_exact(poly.limb_coeffs(), basis)
    return centered(coeffs, basis.product())


def scale_round(x: int, p: int, q_big: int, half_q: int) -> int:
    """eval.rs:816-831 (and 695-709): sign * floor((|p*x| + floor(Q/2)) / Q)."""
    num = p * x
    if num < 0:
        return -((-num + half_q) // q_big)
    return (num + half_q) // q_big


def centered_bigint_to_rns(coeffs: list[int], basis) -> RnsPoly:
    """eval.rs:764-792: Euclidean residue per limb, then forward NTT."""
    return RnsPoly.from_limb_coeffs([[c % q for c in coeffs] for q in basis.moduli], basis)


def tensor_exact(ct1, ct2, basis):
    """Centered lifts and the exact tensor (t0, t1, t2) over Z (eval.rs:126-133)."""
    c0 = reconstruct_centered_bigint(ct1.c[0], basis)
    c1 = reconstruct_centered_bigint(ct1.c[1], basis)
    d0 = reconstruct_centered_bigint(ct2.c[0], basis)
    d1 = reconstruct_centered_bigint(ct2.c[1], basis)
    t0 = poly_mul_exact(c0, d0)
    t1 = [x + y for x, y in zip(poly_mul_exact(c0, d1), poly_mul_exact(c1, d0))]
    t2 = poly_mul_exact(c1, d1)
    return t0, t1, t2


def bfv_mul_generic_rns(ct1, ct2):
    """eval.rs:113-147: exact CRT + exact tensor + BigInt scale-and-round."""
    params = ct1.params
    basis = params.ct_basis
    p = params.plain_modulus
    q_big = basis.product()
    half_q = q_big >> 1
    ts = tensor_exact(ct1, ct2, basis)
    rs = [[scale_round(x, p, q_big, half_q) for x in t] for t in ts]
    return BfvCiphertext([centered_bigint_to_rns(r, basis) for r in rs], params)


def schoolbook_overflow_risk(p: int, q: int, n: int) -> bool:
    """eval.rs:457-464 (u128 saturating arithmetic)."""
    sat = (1 << 128) - 1
    i128max = (1 << 127) - 1
    max_coeff = q // 2
    max_tensor = min(min(n * max_coeff, sat) * max_coeff, sat)
    max_scaled = min(max_tensor * p, sat)
    return max_tensor > i128max or max_scaled > i128max


def bfv_mul_schoolbook(ct1, ct2):
    """eval.rs:416-454: single q, no aux basis, exact i128 (guarded)."""
    params = ct1.params
    basis = params.ct_basis
    p, q, n = params.plain_modulus, basis.moduli[0], params.ring_degree
    if schoolbook_overflow_risk(p, q, n):
        raise ExactoError.not_implemented(
            "schoolbook BFV multiplication can overflow i128 for these parameters; "
            "use HPS auxiliary basis")
    ts = tensor_exact(ct1, ct2, basis)
    out = []
    for t in ts:
        r = [scale_round(x, p, q, q // 2) % q for x in t]  # scale_tensor_component eval.rs:695-709
        out.append(RnsPoly.from_coeff_poly(CoeffPoly.from_coeffs(r, q), basis))
    return BfvCiphertext(out, params)


# --- HPS (single q, 1 or 2 aux primes), restated literally ---

def _ext_centered(c: int, q: int, pj: int) -> int:
    """eval.rs:232-239 (and 307-313, 355-372)."""
    if c > q // 2:
        rem = (q - c) % pj
        return 0 if rem == 0 else pj - rem
    return c % pj


def base_extend_centered(poly: RnsPoly, q: int, basis_p) -> RnsPoly:
    """eval.rs:217-247."""
    cq = poly.components[0].to_coeff_poly().coeffs
    comps = []
    for pj, plan in zip(basis_p.moduli, basis_p.plans):
        comps.append(NttPoly.from_coeff_poly(CoeffPoly([_ext_centered(c, q, pj) for c in cq], pj), plan))
    return RnsPoly(comps, poly.ring_degree)


def hps_scale_coeff(a: int, bs: list[int], p: int, q: int, aux: list[int]) -> int:
    """One coefficient of eval.rs:hps_scale (lines 301-332 for K=1, 349-404 for K=2)."""
    half_q = q // 2
    a_centered = a - q if a > half_q else a
    pa = p * a_centered
    round_pa_q = (pa + q // 2) // q if pa >= 0 else -((-pa + q // 2) // q)
    if len(aux) == 1:
        big_p = aux[0]
        q_inv = _mod_inv(q % big_p, big_p)
        a_ext = _ext_centered(a, q, big_p)
        b = bs[0]
        diff = b - a_ext if b >= a_ext else big_p - a_ext + b
        m_raw = mod_mul(diff, q_inv, big_p)
        m_centered = m_raw - big_p if m_raw > big_p // 2 else m_raw
        scaled = round_pa_q + p * m_centered
        return ((rust_rem(scaled, q)) + q) % q
    p0, p1 = aux
    q_inv0 = _mod_inv(q % p0, p0)
    q_inv1 = _mod_inv(q % p1, p1)
    p1_inv_p0 = _mod_inv(p1 % p0, p0)
    p0_inv_p1 = _mod_inv(p0 % p1, p1)
    big_p = p0 * p1
    half_big_p = big_p // 2
    a0 = _ext_centered(a, q, p0)
    diff0 = bs[0] - a0 if bs[0] >= a0 else p0 - a0 + bs[0]
    m0 = mod_mul(diff0, q_inv0, p0)
    a1 = _ext_centered(a, q, p1)
    diff1 = bs[1] - a1 if bs[1] >= a1 else p1 - a1 + bs[1]
    m1 = mod_mul(diff1, q_inv1, p1)
    t0 = mod_mul(m0, p1_inv_p0, p0)
    t1 = mod_mul(m1, p0_inv_p1, p1)
    m_crt = (t0 * p1 + t1 * p0) % big_p
    m_centered = m_crt - big_p if m_crt > half_big_p else m_crt
    m_mod_q = (rust_rem(m_centered, q) + q) % q
    round_mod_q = (rust_rem(round_pa_q, q) + q) % q
    pm_mod_q = mod_mul(p, m_mod_q, q, barrett_constant(q))
    return (round_mod_q + pm_mod_q) % q


def hps_scale_coeffs(t_q: RnsPoly, t_p: RnsPoly, p: int, q: int, aux_basis) -> list[int]:
    """eval.rs:257-410 (coefficient-domain output, before the final forward NTT)."""
    k = len(aux_basis.moduli)
    if k not in (1, 2):
        raise ExactoError.invalid_param(f"HPS scaling supports 1 or 2 aux primes, got {k}")
    a_poly = t_q.components[0].to_coeff_poly().coeffs
    b_polys = [c.to_coeff_poly().coeffs for c in t_p.components]
    return [hps_scale_coeff(a_poly[i], [bp[i] for bp in b_polys], p, q, aux_basis.moduli)
            for i in range(len(a_poly))]


def hps_check(params):
    """eval.rs:170-178 guard (+ the K>2 error raised later by hps_scale, eval.rs:405-408)."""
    q = params.ct_basis.moduli[0]
    aux = params.aux_basis
    if len(aux.moduli) == 1:
        big_p = aux.moduli[0]
        min_required = (params.ring_degree * q) // 2
        if big_p <= min_required:
            raise ExactoError.invalid_param(
                f"single aux prime too small for HPS centering: P={big_p} <= n*Q/2={min_required}")


def bfv_mul_hps(ct1, ct2):
    """eval.rs:157-209."""
    params = ct1.params
    aux = params.aux_basis
    p = params.plain_modulus
    q = params.ct_basis.moduli[0]
    hps_check(params)
    c0p = base_extend_centered(ct1.c[0], q, aux)
    c1p = base_extend_centered(ct1.c[1], q, aux)
    d0p = base_extend_centered(ct2.c[0], q, aux)
    d1p = base_extend_centered(ct2.c[1], q, aux)
    t0q = ct1.c[0].mul(ct2.c[0])
    t1q = ct1.c[0].mul(ct2.c[1]).add(ct1.c[1].mul(ct2.c[0]))
    t2q = ct1.c[1].mul(ct2.c[1])
    t0p = c0p.mul(d0p)
    t1p = c0p.mul(d1p).add(c1p.mul(d0p))
    t2p = c1p.mul(d1p)
    out = []
    for tq, tp in ((t0q, t0p), (t1q, t1p), (t2q, t2p)):
        r = hps_scale_coeffs(tq, tp, p, q, aux)
        out.append(RnsPoly.from_coeff_poly(CoeffPoly(r, q), params.ct_basis))
    return BfvCiphertext(out, params)


# ------------------------------------------------------------------ key switching

def gadget_decompose_coeff(c_mod_q: int, q: int, base: int, num_digits: int) -> list[int]:
    """keyswitch.rs:24-44 for one coefficient (balanced digits, final carry dropped)."""
    half_base = base // 2
    remaining = c_mod_q - q if c_mod_q > q // 2 else c_mod_q
    out = []
    for _ in range(num_digits):
        rem = rust_rem(remaining, base)
        if rem < -half_base:
            rem += base
        elif rem >= half_base:
            rem -= base
        out.append((rust_rem(rem, q) + q) % q)
        remaining = rust_div(remaining - rem, base)
    return out


def gadget_decompose(poly: CoeffPoly, base: int, num_digits: int) -> list[CoeffPoly]:
    """keyswitch.rs:11-52."""
    q = poly.modulus
    cols = [gadget_decompose_coeff(c, q, base, num_digits) for c in poly.coeffs]
    return [CoeffPoly([col[d] for col in cols], q) for d in range(num_digits)]


def relinearize(ct, rlk):
    """keyswitch.rs:59-101 (to_coeff_poly under extension semantics for Q >= 2^64)."""
    if len(ct.c) < 3:
        return ct.clone()
    if len(ct.c) > 3:
        raise ExactoError.invalid_param("relinearization only supports degree-2 ciphertexts")
    params = ct.params
    basis = params.ct_basis
    c2 = ct.c[2].to_coeff_poly(basis)
    digits = gadget_decompose(c2, params.gadget_base, params.gadget_digits)
    c0 = ct.c[0].clone()
    c1 = ct.c[1].clone()
    for i, digit in enumerate(digits):
        if i >= len(rlk.keys):
            break
        d = RnsPoly.from_coeff_poly(digit, basis)
        c0 = c0.add(d.mul(rlk.keys[i][0]))
        c1 = c1.add(d.mul(rlk.keys[i][1]))
    return BfvCiphertext([c0, c1], params)


# ------------------------------------------------------------------ Galois automorphisms

class GaloisKey:
    """keygen.rs:49-56: key-switch key from s(X^element) to s(X)."""

    def __init__(self, keys, element, params):
        self.keys = keys
        self.element = element
        self.params = params


def apply_automorphism(poly: CoeffPoly, k: int) -> CoeffPoly:
    """keygen.rs:239-262: X^i -> X^(ik) mod X^n + 1, accumulated with mod_add / mod_sub."""
    n, q = len(poly.coeffs), poly.modulus
    res = [0] * n
    for i, c in enumerate(poly.coeffs):
        if c == 0:
            continue
        e = (i * k) % (2 * n)
        if e < n:
            res[e] = (res[e] + c) % q
        else:
            res[e - n] = (res[e - n] - c) % q
    return CoeffPoly(res, q)


def bfv_apply_automorphism(ct, gk):
    """eval.rs:512-561 (to_coeff_poly under extension semantics for Q >= 2^64, as relinearize)."""
    if len(ct.c) != 2:
        raise ExactoError.invalid_param("automorphism requires degree-1 ciphertext")
    params = ct.params
    basis = params.ct_basis
    k = gk.element
    c0 = apply_automorphism(ct.c[0].to_coeff_poly(basis), k)
    c1 = apply_automorphism(ct.c[1].to_coeff_poly(basis), k)
    c0f = RnsPoly.from_coeff_poly(c0, basis)
    digits = gadget_decompose(c1, params.gadget_base, params.gadget_digits)
    c1f = None
    for i, digit in enumerate(digits):
        if i >= len(gk.keys):
            break
        d = RnsPoly.from_coeff_poly(digit, basis)
        c0f = c0f.add(d.mul(gk.keys[i][0]))
        p1 = d.mul(gk.keys[i][1])
        c1f = p1 if c1f is None else c1f.add(p1)
    if c1f is None:
        raise ExactoError.invalid_param("galois key is empty")  # the reference unwraps None (panic)
    return BfvCiphertext([c0f, c1f], params)


def bfv_trace(ct, elements, galois_keys):
    """eval.rs:572-586: result <- result + sigma_k(result) for each element k, in order."""
    result = ct.clone()
    for k in elements:
        if k not in galois_keys:
            raise ExactoError.invalid_param(f"missing Galois key for element {k}")
        rot = bfv_apply_automorphism(result, galois_keys[k])
        result = bfv_add(result, rot)
    return result


def monomial_mul_poly(poly: CoeffPoly, j: int, n: int) -> CoeffPoly:
    """eval.rs:634-652."""
    q = poly.modulus
    res = [0] * n
    for i, c in enumerate(poly.coeffs):
        if c == 0:
            continue
        e = (i + j) % (2 * n)
        if e < n:
            res[e] = (res[e] + c) % q
        else:
            res[e - n] = (res[e - n] - c) % q
    return CoeffPoly(res, q)


def bfv_monomial_mul(ct, j: int):
    """eval.rs:613-632 (to_coeff_poly under extension semantics for Q >= 2^64)."""
    params = ct.params
    basis = params.ct_basis
    n = params.ring_degree
    j %= 2 * n
    if j == 0:
        return ct.clone()
    return BfvCiphertext([RnsPoly.from_coeff_poly(monomial_mul_poly(c.to_coeff_poly(basis), j, n), basis)
                          for c in ct.c], params)


def bfv_plain_mul(ct, pt: CoeffPoly):
    """eval.rs:468-486: every component times the raw plaintext (no Delta)."""
    ptr = RnsPoly.from_coeff_poly(pt, ct.params.ct_basis)
    return BfvCiphertext([c.mul(ptr) for c in ct.c], ct.params)


def bfv_plain_add(ct, pt: CoeffPoly):
    """eval.rs:489-503: c0 + Delta m."""
    params = ct.params
    basis = params.ct_basis
    dr = delta_residues(params)
    dm = RnsPoly.from_limb_coeffs([[(m % q) * d % q for m in pt.coeffs] for q, d in zip(basis.moduli, dr)], basis)
    c = [x.clone() for x in ct.c]
    c[0] = c[0].add(dm)
    return BfvCiphertext(c, params)


def galois_s_auto(sk_poly: RnsPoly, k: int, basis) -> RnsPoly:
    """keygen.rs:179-182: limb 0 of s in the coefficient domain (mod q0), permuted, lifted to every limb."""
    s0 = sk_poly.components[0].to_coeff_poly()
    return RnsPoly.from_coeff_poly(apply_automorphism(s0, k), basis)


# ------------------------------------------------------------------ keygen / encrypt / decrypt
# Not on the hot path: mathematically equivalent restatement of bfv/keygen.rs:64-162 and
# bfv/encrypt.rs:79-178 with this build's own sampler (signed small values reduced per limb).

def _signed_to_rns(vals: list[int], basis) -> RnsPoly:
    return RnsPoly.from_limb_coeffs([[v % q for v in vals] for q in basis.moduli], basis)


def _uniform_rns(rng: random.Random, basis) -> RnsPoly:
    n = basis.ring_degree
    return RnsPoly.from_limb_coeffs([[rng.randrange(q) for _ in range(n)] for q in basis.moduli],
                                    basis)


def _gaussian(rng: random.Random, n: int, sigma: float) -> list[int]:
    return [int(round(rng.gauss(0.0, sigma))) for _ in range(n)]


def gen_secret_key(params, rng: random.Random) -> SecretKey:
    """keygen.rs:64-79 (ternary s)."""
    s = [rng.choice((-1, 0, 1)) for _ in range(params.ring_degree)]
    return SecretKey(_signed_to_rns(s, params.ct_basis), params, s)


def gen_relin_key(sk: SecretKey, rng: random.Random, num_keys=None) -> RelinKey:
    """keygen.rs:123-162: rlk_i = (-(a_i s + e_i) + base^i s^2, a_i)."""
    params = sk.params
    basis = params.ct_basis
    s_sq = sk.poly.mul(sk.poly)
    g = s_sq.clone()
    keys = []
    count = params.gadget_digits if num_keys is None else num_keys
    for i in range(count):
        a = _uniform_rns(rng, basis)
        e = _signed_to_rns(_gaussian(rng, params.ring_degree, params.sigma), basis)
        rlk0 = a.mul(sk.poly).add(e).neg().add(g)
        keys.append((rlk0, a))
        if i + 1 < count:
            g = g.scalar_mul(params.gadget_base)
    return RelinKey(keys, params)


def delta_residues(params) -> list[int]:
    """encrypt.rs:205-229: Delta = floor(Q/p) mod q_i."""
    q_big = params.ct_basis.product()
    delta = q_big // params.plain_modulus
    if delta == 0:
        raise ExactoError.invalid_param("ciphertext modulus product Q must be >= plaintext modulus p")
    return [delta % q for q in params.ct_basis.moduli]


def encrypt_sk(pt: CoeffPoly, sk: SecretKey, rng: random.Random) -> BfvCiphertext:
    """encrypt.rs:79-106: (-a s + e + Delta m, a)."""
    params = sk.params
    basis = params.ct_basis
    dr = delta_residues(params)
    dm = RnsPoly.from_limb_coeffs([[(m % q) * d % q for m in pt.coeffs] for q, d in zip(basis.moduli, dr)],
                                  basis)
    a = _uniform_rns(rng, basis)
    e = _signed_to_rns(_gaussian(rng, params.ring_degree, params.sigma), basis)
    c0 = a.mul(sk.poly).neg().add(e).add(dm)
    return BfvCiphertext([c0, a], params)


def decrypt(ct: BfvCiphertext, sk: SecretKey) -> CoeffPoly:
    """encrypt.rs:111-178: m = floor((x p + floor(Q/2)) / Q) mod p, x = CRT(phase) in [0, Q)."""
    params = ct.params
    basis = params.ct_basis
    phase = ct.c[0].clone()
    s_pow = sk.poly.clone()
    for i in range(1, len(ct.c)):
        phase = phase.add(ct.c[i].mul(s_pow))
        if i < len(ct.c) - 1:
            s_pow = s_pow.mul(sk.poly)
    q_big = basis.product()
    half_q = q_big >> 1
    p = params.plain_modulus
    xs = crt_exact(phase.limb_coeffs(), basis)
    return CoeffPoly([((x * p + half_q) // q_big) % p for x in xs], p)


def encode_scalar(m: int, params) -> CoeffPoly:
    """encoding.rs:7-20."""
    if m >= params.plain_modulus:
        raise ExactoError.invalid_param(f"plaintext {m} >= plain_modulus {params.plain_modulus}")
    c = [0] * params.ring_degree
    c[0] = m
    return CoeffPoly(c, params.plain_modulus)


def decode_scalar(poly: CoeffPoly) -> int:
    """encoding.rs:23-25."""
    return poly.coeffs[0]
