"""CPU check of the rounded-float CRT over P (kernels.hip fpc_lift, the FPC form of exact_scale_sp_kernel
and exact_psum_sp_kernel): with y_a = r (P / p_a)^-1 mod p_a, alpha = round(sum_a fl(y_a) * fl(1 / p_a))
(fp64, fused multiply-adds in the kernel's order) equals round(X / P) for X = sum_a y_a (P / p_a), so
r = X - alpha P exactly, for every |r| < P / 4 -- at the auxiliary bases the context builds for cfg3, cfg4
and cfg5 (primes == 1 mod 2n just below 2^60, P > 4 p n Q), extremes included.  Also the two bounds that
make |r| < P / 4 hold: the scale's |r| <= p n Q / 2 + 1 < P / 8, and psum_fp_max's m (2 p n Q + 4) <= P.

A Python restatement of the device arithmetic (each fp64 operation correctly rounded, as gfx950's
v_cvt_f64_u32 / v_add_f64 / v_fma_f64 are), not the kernel."""
import math
import random
from fractions import Fraction

import pytest

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]
CONFIGS = {"cfg3": (4096, 65537, Q3), "cfg4": (4096, 260111, Q3), "cfg5": (8192, 1040407, Q4)}


def is_prime(n):
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d, s = d // 2, s + 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def aux_basis(n, p, qs):
    """exacto_ctx_create's exact-path auxiliary basis: primes == 1 mod 2n below 2^60, largest first,
    not ciphertext primes, until P > 4 p n Q."""
    need = 4 * p * n * math.prod(qs)
    step, cand, ps = 2 * n, ((1 << 60) - 1) // (2 * n) * (2 * n) + 1, []
    while math.prod(ps) <= need:
        cand -= step
        while cand in qs or not is_prime(cand):
            cand -= step
        ps.append(cand)
    return ps


def fma(x, y, z):
    return float(Fraction(x) * Fraction(y) + Fraction(z))


def fpc_alpha(r, ps):
    P = math.prod(ps)
    y = [r % P * pow(P // pa, -1, pa) % pa for pa in ps]
    f = 0.0
    for ya, pa in zip(y, ps):
        f = fma(float(ya), 1.0 / pa, f)
    X = sum(ya * (P // pa) for ya, pa in zip(y, ps))
    return round(f), y, X


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_fpc_alpha_exact_below_quarter_P(cfg):
    n, p, qs = CONFIGS[cfg]
    ps = aux_basis(n, p, qs)
    P = math.prod(ps)
    rng = random.Random(len(ps))
    lim = P // 4 - 1
    rs = [0, 1, -1, lim, -lim, lim - 1, -(lim - 1), P // 8, -(P // 8)]
    rs += [rng.randrange(-lim, lim + 1) for _ in range(3000)]
    rs += [rng.choice((1, -1)) * (lim - rng.randrange(1 << 40)) for _ in range(500)]   # near the bound
    for r in rs:
        alpha, y, X = fpc_alpha(r, ps)
        assert 0 <= alpha <= len(ps)
        assert X - alpha * P == r, (cfg, r)
        # res_i as the kernel forms it: sum_a y_a ((P / p_a) mod q_i) + alpha (q_i - P mod q_i)
        for q in qs:
            res = (sum(ya * ((P // pa) % q) for ya, pa in zip(y, ps)) + alpha * ((q - P % q) % q)) % q
            assert res == r % q


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_fpc_bounds(cfg):
    n, p, qs = CONFIGS[cfg]
    ps = aux_basis(n, p, qs)
    P, Q = math.prod(ps), math.prod(qs)
    assert 8 * (p * n * Q // 2 + 1) < P                 # the scale: |r| < P / 8
    fp_max = max(m for m in range(1, 65) if 2 * m * (p * n * Q + 2) < P) if 2 * (p * n * Q + 2) < P else 0
    # the BASELINE dBFV configs sum at most d products per limb (cfg4: 2, cfg5: 8)
    assert fp_max >= {"cfg3": 1, "cfg4": 2, "cfg5": 8}[cfg]
    for m in range(1, fp_max + 1):
        assert 4 * m * (p * n * Q // 2 + 1) <= P         # |R| <= P / 4
