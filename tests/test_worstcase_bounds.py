"""The two exactness bounds of the GPU path at their extremes, on CPU (the GPU side of the same inputs
is tests/test_gpu_worstcase.py):

* ks32 (the key switch over the integers): coefficient 0 of the key switch of
  tests/worstcase.py's inputs is m G' n (B/2) floor(q/2) -- every digit -B/2, the key sign-aligned.
  Lifted from the library's 31-bit basis (its selection rule restated) it is exact; from the same
  basis with one prime fewer it is not.  cfg3 (m = 1, primary basis), cfg4 (m = 2, the wide basis),
  cfg5 (m = 8, primary basis, base 256).
* psum: m products whose c1 tensors reach 2 n floor(Q/2)^2 sum (after scaling) to m round(p T / Q);
  the library's condition m (p n Q + 2) < P holds at the BASELINE dBFV configs and the sum lifts
  from P, but not from P with one auxiliary prime fewer.
"""

import math

import numpy as np
import pytest

from oracle.modular import is_prime
from oracle.bfv import scale_round, gadget_decompose_coeff
from worstcase import digit_target, ks32_basis, lift_centred

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]

# (name, n, moduli, plain, base, G, m = products per output limb whose digits are summed, pmax)
KS_CASES = [
    ("cfg3", 4096, Q3, 65537, 1 << 16, 12, 1, (1 << 32) // 3),
    ("cfg4", 4096, Q3, 260111, 1 << 16, 12, 2, 1 << 31),
    ("cfg5", 8192, Q4, 1040407, 256, 30, 8, (1 << 32) // 3),
]


def negacyclic(a, b):
    n = len(a)
    out = [0] * n
    for i in range(n):
        for j in range(n):
            k = i + j
            if k < n:
                out[k] += a[i] * b[j]
            else:
                out[k - n] -= a[i] * b[j]
    return out


def test_aligned_key_switch_reaches_the_bound_small_n():
    # the worst-case coefficient is u_0 = G' n (B/2) h: checked by the full convolution at n = 16
    n, B, h, gp = 16, 1 << 16, (1 << 59) - 7, 3
    d = [-(B // 2)] * n
    r = [-h] + [h] * (n - 1)
    u = [0] * n
    for _ in range(gp):
        u = [x + y for x, y in zip(u, negacyclic(d, r))]
    assert u[0] == gp * n * (B // 2) * h
    assert max(abs(x) for x in u) == u[0]


@pytest.mark.parametrize("name,n,q,plain,base,G,m,pmax", KS_CASES)
def test_ks32_lift_exact_at_worst_case_and_not_with_a_prime_fewer(name, n, q, plain, base, G, m, pmax):
    Q = math.prod(q)
    x, gp = digit_target(Q, base, G)
    digits = gadget_decompose_coeff(x % Q, Q, base, G)
    assert digits[:gp] == [Q - base // 2] * gp and gp >= G - 1
    qmax = max(q)
    primary = ks32_basis(n, qmax, base, G, (1 << 32) // 3)
    basis = primary if pmax == (1 << 32) // 3 else ks32_basis(n, qmax, base, G, pmax)
    assert basis is not None and len(basis) == 3
    # the library takes a basis for m summed products when its prod p > 2 m G n (B/2) (q/2)
    assert math.prod(basis) > 2 * m * G * n * (base // 2) * (qmax // 2) + 1
    for ql in q:
        u0 = m * gp * n * (base // 2) * (ql // 2)      # coefficient 0 of the summed key switch
        assert lift_centred(u0, basis) == u0
        assert lift_centred(-u0, basis) == -u0
        assert lift_centred(u0, basis[:-1]) != u0       # one prime fewer: the lift wraps
    if name == "cfg4":   # two summed products do not fit the primary basis: the wide one is needed
        u0 = m * gp * n * (base // 2) * (qmax // 2)
        assert lift_centred(u0, primary) != u0


def aux_basis(n, q, plain):
    """The library's auxiliary primes (context.hip exacto_ctx_create): p == 1 mod 2n below 2^60,
    largest first, not a ciphertext prime, the fewest with P > 4 p n Q."""
    need = 4 * plain * n * math.prod(q)
    ps, P = [], 1
    c = ((1 << 60) - 1) // (2 * n) * (2 * n) + 1
    while P <= need:
        c -= 2 * n
        while c in q or not is_prime(c):
            c -= 2 * n
        ps.append(c)
        P *= c
    return ps


@pytest.mark.parametrize("n,q,plain,m", [(4096, Q3, 260111, 2), (8192, Q4, 1040407, 8)])
def test_psum_sum_liftable_at_worst_case_and_not_with_a_prime_fewer(n, q, plain, m):
    Q = math.prod(q)
    h = Q // 2
    T = 2 * n * h * h                                   # c1 = a0 b1 + a1 b0 at coefficient 0
    r = scale_round(T, plain, Q, Q >> 1)
    assert r > 0 and abs(r) <= plain * n * Q // 2 + 1
    R = m * r                                           # a limb's m identical products, summed
    P = aux_basis(n, q, plain)
    assert len(P) == len(q) + 1
    Pp = math.prod(P)
    assert m * (plain * n * Q + 2) < Pp                 # the library's psum condition
    assert lift_centred(R, P) == R
    assert lift_centred(R, P[:-1]) != R
