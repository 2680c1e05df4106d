"""CPU check of ks32_crt's rounded-float CRT lift (ks32_dev.hpp ks32_fpc_one, context.hip sums_lifted):
with y_s = u (P / p_s)^-1 mod p_s taken anywhere in [0, 2 p_s) (the inverse transforms' FOLD + OUT2P
outputs), alpha = round(sum_s fl(y_s) fl(1 / p_s)) (fp64, the kernel's multiply then fused multiply-adds)
gives u = sum_s y_s (P / p_s) - alpha P exactly for every |u| <= m `one` that the host's margin
(P 2^20 > (2 m one + 1)(2^20 + 1)) admits, and the kernel's 30-bit-split evaluation mod q = 2^60 - d
stays below 2^64 and equals u + r mod q.  At the three 31-bit bases the context builds (narrow primes
below 2^32 / 3, wide below 2^31, lazy below 2^30) for the cfg3 / cfg4 / cfg5 parameters, with `one`
pushed to the margin's limit; and four narrow / lazy primes (cfg5's ring at base 2^16).

A Python restatement of the device arithmetic (each fp64 operation correctly rounded, as gfx950's
v_cvt_f64_u32 / v_mul_f64 / v_fma_f64 are), not the kernel."""
import math
import random
from fractions import Fraction

import pytest

from test_fpc_crt import Q3, Q4, is_prime

M64 = (1 << 64) - 1
# (n, G, gadget base, ciphertext primes): cfg3 / cfg4 (the same ring), cfg5 (base 256, oracle/params.py
# cfg5_params), and a four-prime case (cfg5's ring at base 2^16: the S = 4 kernels)
CONFIGS = {"cfg3": (4096, 12, 1 << 16, Q3), "cfg5": (8192, 30, 256, Q4), "s4": (8192, 15, 1 << 16, Q4)}


def basis(n, pmax, bound, fixed_s=0):
    """context.hip build_ks32_basis_impl: primes == 1 mod 2n below pmax, largest first, above 2^30 (the
    lazy basis: exactly fixed_s primes above 7/8 pmax), until their product exceeds `bound`."""
    step = 2 * n
    pmin = pmax - pmax // 8 if fixed_s else 1 << 30
    ps, p = [], (pmax - 1) // step * step + 1
    while p > pmin and len(ps) < 4:
        if is_prime(p):
            ps.append(p)
            if (len(ps) == fixed_s) if fixed_s else math.prod(ps) > bound:
                break
        p -= step
    return ps


def sums_lifted(P, one, fpc):
    r = 0
    for m in range(1, 65):
        bm = 2 * m * one + 1
        if (P << 20 if fpc else P) <= (bm * ((1 << 20) + 1) if fpc else bm):
            break
        r = m
    return r


def fma(x, y, z):
    return float(Fraction(x) * Fraction(y) + Fraction(z))


def fpc_one(y, r, ps, q):
    """ks32_fpc_one, step by step with its 64-bit bounds asserted."""
    S, P, dq = len(ps), math.prod(ps), (1 << 60) - q
    f = float(y[0]) * (1.0 / ps[0])
    for s in range(1, S):
        f = fma(float(y[s]), 1.0 / ps[s], f)
    al = round(f)                      # v_rndne_f64: ties to even, never a tie here
    assert 0 <= al <= 2 * S
    negp = (q - P % q) % q
    cs = [(P // p) % q for p in ps]
    n0, n1 = negp & ((1 << 30) - 1), negp >> 30
    a0, a1 = al * n0, al * n1
    for s in range(S):
        a0 += y[s] * (cs[s] & ((1 << 30) - 1))
        a1 += y[s] * (cs[s] >> 30)
    assert a0 <= M64 and a1 <= M64
    h, l30 = a1 >> 30, (a1 & ((1 << 30) - 1)) << 30
    t = a0 + l30 + (h & 0xFFFFFFFF) * dq + (((h >> 32) * dq & 0xFFFFFFFF) << 32)
    assert t + r <= M64
    x = t + r
    x = (x & ((1 << 60) - 1)) + (x >> 60) * dq        # reduce_near60
    return x - q if x >= q else x, al


def bases(cfg):
    n, G, B, qs = CONFIGS[cfg]
    one = G * n * (B // 2) * (max(qs) // 2)
    bound = 2 * one + 1
    out = {"narrow": basis(n, (1 << 32) // 3, bound), "wide": basis(n, 1 << 31, bound)}
    out["lazy"] = basis(n, 1 << 30, bound, fixed_s=len(out["narrow"]))
    return n, qs, one, out


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("kind", ["narrow", "wide", "lazy"])
def test_ks32_fpc_lift_exact_at_the_margin(cfg, kind):
    n, qs, _, bs = bases(cfg)
    ps = bs[kind]
    if len(ps) > 3 and kind == "wide":
        pytest.skip("four wide primes: ks32_crt keeps the Garner lift (the 64-bit sums could overflow)")
    P = math.prod(ps)
    assert all(p % (2 * n) == 1 for p in ps)
    # the largest per-term bound the margin admits for m = 1 .. 3: every |u| <= m one must lift exactly
    rng = random.Random(len(ps) * 7 + n)
    for m in (1, 2, 3):
        lo, hi = 0, P
        while lo < hi:      # largest `one` with sums_lifted(P, one, True) >= m
            mid = (lo + hi + 1) // 2
            if sums_lifted(P, mid, True) >= m:
                lo = mid
            else:
                hi = mid - 1
        lim = m * lo
        assert 2 * lim < P
        us = [0, 1, -1, lim, -lim, lim - 1, -(lim - 1)]
        us += [rng.randrange(-lim, lim + 1) for _ in range(300)]
        us += [rng.choice((1, -1)) * (lim - rng.randrange(1 << 30)) for _ in range(200)]
        for u in us:
            # the inverse transform's residues: either representative below 2 p_s
            y = [u * pow(P // p, -1, p) % p for p in ps]
            y = [v + p if rng.random() < 0.5 and v + p < 2 * p else v for v, p in zip(y, ps)]
            assert all(v < 2 * p < (1 << 32) for v, p in zip(y, ps))
            X = sum(v * (P // p) for v, p in zip(y, ps))
            for q in qs:
                r = rng.randrange(q)
                got, al = fpc_one(y, r, ps, q)
                assert X - al * P == u, (cfg, kind, m, u)
                assert got == (u + r) % q


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_ks32_fpc_max_against_sum_max(cfg):
    """The margin costs no sums at the BASELINE parameters: fpc_max == sum_max for every basis at the
    analytic bound, and at cfg4's key-norm bound (2^90.6 for the two-product sums) on the narrow basis."""
    _, _, one, bs = bases(cfg)
    for kind in ("narrow", "wide"):
        ps = bs[kind]
        if len(ps) > 3 and kind == "wide":
            continue
        P = math.prod(ps)
        assert sums_lifted(P, one, True) == sums_lifted(P, one, False) >= 1
    if cfg == "cfg3":
        P = math.prod(bs["narrow"])
        worst = int(2 ** 90.6) // 4          # (B/2) sum_g ||r||_1 of a uniform key, cfg4's m = 2
        assert sums_lifted(P, worst, False) >= 2
        assert sums_lifted(P, worst, True) == sums_lifted(P, worst, False)
