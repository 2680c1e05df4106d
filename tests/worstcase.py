"""Worst-case inputs for the two exactness bounds of the GPU path (test helper).

1. The key switch over the integers (ks32): relinearize adds sum_g d_g * r_{g,c,l}
   (keyswitch.rs:86-95), d_g the balanced gadget digits of c2 (|d| <= B/2) and r the key in the
   coefficient domain, balanced (|r| <= q/2).  The library lifts that integer from a basis of 31-bit
   primes p_s, exact while prod p_s > 2 m G n (B/2) (q/2) for m products whose digits are summed
   first (dBFV).  `digit_inputs` makes EVERY coefficient of every product's c2 decompose into -B/2
   in each of the low G' digits (all the digits a |value| < Q/2 can hold), and `aligned_key` makes
   r = [-h, h, ..., h] (h = floor(q_l / 2)), so coefficient 0 of the key switch is
   u_0 = m G' n (B/2) h: the bound with G' for G.
2. psum (dBFV): an output limb's c0 / c1 are scaled once from the sum of its m products' tensors,
   exact while m (p n Q + 2) < P.  `tensor_inputs` makes every product's c1 tensor reach
   2 n floor(Q/2)^2 at coefficient 0 (a = (h, h, ..., h), b = (h, -h, ..., -h), h = floor(Q/2)),
   so the scaled sum approaches m p n Q / 2.

Ciphertext components are given in the coefficient domain as centred integers and moved to the NTT
domain with the C restatement's transform (oracle/c, the convention of this build).
"""

from __future__ import annotations

import math

import numpy as np

from oracle import cref
from oracle.bfv import gadget_decompose_coeff, scale_round


def to_ntt(coeffs, moduli, n):
    """Centred integer coefficient vector -> [L][n] u64 NTT-domain residues."""
    out = np.empty((len(moduli), n), dtype=np.uint64)
    for l, q in enumerate(moduli):
        out[l] = np.array([c % q for c in coeffs], dtype=np.uint64)
        out[l] = cref.ntt(n, q, out[l][None, :])[0]
    return out


def digit_target(Q: int, base: int, G: int) -> tuple[int, int]:
    """(x, G'): x = -(B/2) (1 + B + ... + B^(G'-1)) with the most digits G' <= G such that |x| <= Q/2;
    its balanced gadget digits (keyswitch.rs:24-44) are -B/2 in positions < G'."""
    half = base // 2
    gp = G
    while gp > 0 and half * (base ** gp - 1) // (base - 1) > Q // 2:
        gp -= 1
    return -half * (base ** gp - 1) // (base - 1), gp


def digit_inputs(moduli, plain, base, G, n):
    """(a1, b1) coefficient-domain centred ints with round(p (a1 * b1) / Q) = x at every coefficient
    (x from digit_target): b1 = c X^0 with c = floor(Q / p), a1 = (v, ..., v), c v within the
    rounding interval of Q x / p."""
    Q = math.prod(moduli)
    x, gp = digit_target(Q, base, G)
    c = Q // plain
    num, den = Q * x, plain * c
    v = (2 * num + den) // (2 * den)          # nearest integer to Q x / (p c), exactly
    for dv in (0, -1, 1, -2, 2):
        if scale_round(c * (v + dv), plain, Q, Q >> 1) == x:
            v += dv
            break
    else:
        raise AssertionError("no coefficient rounds to the target")
    assert abs(v) <= Q // 2 and abs(c) <= Q // 2
    digits = gadget_decompose_coeff(x % Q, Q, base, G)
    assert all(d == Q - base // 2 for d in digits[:gp]), "target digits are not -B/2"
    return [v] * n, [c] + [0] * (n - 1), x, gp


def aligned_key(moduli, G, n):
    """rlk [G][2][L][n] (NTT domain) whose every row is r = [-h_l, h_l, ..., h_l] mod q_l."""
    rows = np.empty((G, 2, len(moduli), n), dtype=np.uint64)
    for l, q in enumerate(moduli):
        h = q // 2
        r = np.full((1, n), h, dtype=np.uint64)
        r[0, 0] = q - h
        r = cref.ntt(n, q, r)[0]
        rows[:, :, l, :] = r
    return rows


def random_c0(rng, moduli, n, count):
    out = np.empty((count, len(moduli), n), dtype=np.uint64)
    for l, q in enumerate(moduli):
        out[:, l] = rng.integers(0, q, size=(count, n), dtype=np.uint64)
    return out


def digit_case_bfv(moduli, plain, base, G, n, seed=11):
    """cfg3-style bfv_mul_and_relin inputs: ct1 = (random, a1), ct2 = (random, b1), aligned key."""
    rng = np.random.default_rng(seed)
    a1, b1, x, gp = digit_inputs(moduli, plain, base, G, n)
    ct1 = np.stack([random_c0(rng, moduli, n, 1)[0], to_ntt(a1, moduli, n)])[None]
    ct2 = np.stack([random_c0(rng, moduli, n, 1)[0], to_ntt(b1, moduli, n)])[None]
    return ct1, ct2, aligned_key(moduli, G, n), gp


def digit_case_dbfv(moduli, plain, base, G, n, d, seed=12):
    """dbfv_mul inputs [1][d][2][L][n]: every limb of a is (random, a1), of b (random, b1), so every
    product's c2 has digits -B/2 and a limb's m summed digits are -m B/2."""
    rng = np.random.default_rng(seed)
    a1, b1, x, gp = digit_inputs(moduli, plain, base, G, n)
    A1, B1 = to_ntt(a1, moduli, n), to_ntt(b1, moduli, n)
    a = np.stack([np.stack([random_c0(rng, moduli, n, 1)[0], A1]) for _ in range(d)])[None]
    b = np.stack([np.stack([random_c0(rng, moduli, n, 1)[0], B1]) for _ in range(d)])[None]
    return a, b, aligned_key(moduli, G, n), gp


def tensor_case_dbfv(moduli, n, d, G, seed=13):
    """dbfv_mul inputs whose every product reaches |T1_0| = 2 n floor(Q/2)^2 (psum's bound)."""
    rng = np.random.default_rng(seed)
    Q = math.prod(moduli)
    h = Q // 2
    A = to_ntt([h] * n, moduli, n)
    Bp = to_ntt([h] + [-h] * (n - 1), moduli, n)
    a = np.stack([np.stack([A, A]) for _ in range(d)])[None]
    b = np.stack([np.stack([Bp, Bp]) for _ in range(d)])[None]
    key = random_c0(rng, moduli, n, 2 * G).reshape(G, 2, len(moduli), n)
    return a, b, key


# ---------------------------------------------------------------- the bounds themselves, restated

def ks32_basis(n, q_max, base, G, pmax, sums=1, maxs=4):
    """The library's 31-bit basis rule (context.hip build_ks32_basis): primes p == 1 mod 2n below
    pmax and above 2^30, largest first, the fewest with prod p > 2 sums G n floor(B/2) floor(q/2)."""
    from oracle.modular import is_prime
    bound = 2 * sums * G * n * (base // 2) * (q_max // 2) + 1
    ps, P = [], 1
    p = (pmax - 1) // (2 * n) * (2 * n) + 1
    while p > (1 << 30) and len(ps) < maxs:
        if is_prime(p):
            ps.append(p)
            P *= p
            if P > bound:
                return ps
        p -= 2 * n
    return None


def lift_centred(u: int, primes) -> int:
    """ks32_crt's lift restated: residues of u mod each p_s, mixed-radix (Garner) digits, centred
    against floor(P/2) -> the integer the library adds (exact iff |u| < P/2)."""
    res = [u % p for p in primes]
    v = []
    for i, p in enumerate(primes):
        t = res[i]
        for k in range(i):
            t = (t - v[k]) * pow(primes[k], -1, p) % p
        v.append(t)
    x, w = 0, 1
    for i, p in enumerate(primes):
        x += v[i] * w
        w *= p
    return x - w if x > w // 2 else x
