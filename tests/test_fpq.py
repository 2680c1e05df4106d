"""CPU check of the scale kernels' centred s = [p T]_Q by a rounded float sum (kernels.hip fpq_y, the FPQ
form of exact_scale_sp_kernel / exact_psum_sp_kernel; context.hip's FPQ constants): with
z_i = T_i p (Q / q_i)^-1 mod q_i split in 30-bit halves, f = the kernel's fused multiply-adds
z0_i fl(1 / q_i) + z1_i fl(2^30 / q_i) in order, beta = rint(f): wherever |f - beta| <= 1/2 - 2^-40 the
fast path is taken and sum_i z_i (Q / q_i) - beta Q equals the centred s the Garner path computes
(s > floor(Q/2) -> s - Q); and y_a = T_a pq Pi_a + sum_i z_i fpq_c[i][a] + beta Pi_a equals the Garner
path's T_a pq Pi_a + sum_k v_k fpc_qpq[k][a] + negs Pi_a mod every p_a.  Random residues, zeros, and s
driven to within a few units (and within 2^-45 Q) of +-Q/2, where the band must send the lane to Garner.

A Python restatement of the device arithmetic (each fp64 operation correctly rounded), not the kernel."""
import math
import random
from fractions import Fraction

import pytest

from test_fpc_crt import Q3, Q4, aux_basis

# (n, plaintext modulus, ciphertext primes) as CONFIGS in test_fpc_crt.py
CONFIGS = {"cfg3": (4096, 65537, Q3), "cfg4": (4096, 260111, Q3), "cfg5": (8192, 1040407, Q4)}
LIM = 0.5 - 2.0 ** -40
M30 = (1 << 30) - 1


def fma(x, y, z):
    return float(Fraction(x) * Fraction(y) + Fraction(z))


def rint(x):
    return float(round(x))   # Python rounds half to even, as v_rndne_f64


def consts(n, p, qs):
    ps = aux_basis(n, p, qs)
    Q, P = math.prod(qs), math.prod(ps)
    pi = [pow((P // pa) % pa, -1, pa) for pa in ps]
    pz = [p % q * pow((Q // q) % q, -1, q) % q for q in qs]
    fq = [[(pa - pow(q % pa, -1, pa)) % pa * pi[a] % pa for a, pa in enumerate(ps)] for q in qs]
    pq = [p * pow(Q % pa, -1, pa) % pa * pi[a] % pa for a, pa in enumerate(ps)]
    # the Garner path's constants: qpq[k][a] = (q_0 .. q_{k-1}) Q^-1 mod p_a, fpc_qpq = (p_a - qpq) Pi_a
    qpq = [[math.prod(qs[:k]) % pa * pow(Q % pa, -1, pa) % pa for pa in ps] for k in range(len(qs))]
    fqpq = [[(pa - qpq[k][a]) % pa * pi[a] % pa for a, pa in enumerate(ps)] for k in range(len(qs))]
    return ps, Q, pi, pz, fq, pq, fqpq


def fpq(T, qs, pz):
    z = [t * w % q for t, w, q in zip(T, pz, qs)]
    f = 0.0
    for zi, q in zip(z, qs):
        f = fma(float(zi & M30), 1.0 / q, f)
        f = fma(float(zi >> 30), float(1 << 30) / float(q), f)
    return z, f, rint(f)


def garner_s(T, p, qs):
    """The Garner path's s: [p T]_Q, centred with s > floor(Q/2) negative; its mixed-radix digits."""
    Q = math.prod(qs)
    x = sum(t * (Q // q) * pow((Q // q) % q, -1, q) for t, q in zip(T, qs)) % Q
    st = p * x % Q
    v, rest = [], st
    for q in qs:
        v.append(rest % q)
        rest //= q
    negs = st > Q // 2
    return st - Q if negs else st, v, negs


def check(T, Ta, p, qs, c):
    ps, Q, pi, pz, fq, pq, fqpq = c
    s, v, negs = garner_s(T, p, qs)
    z, f, b = fpq(T, qs, pz)
    if abs(f - b) > LIM:
        return False            # the lane takes Garner
    beta = int(b)
    assert 0 <= beta <= len(qs)
    assert sum(zi * (Q // q) for zi, q in zip(z, qs)) - beta * Q == s
    for a, pa in enumerate(ps):
        fast = (Ta[a] * pq[a] + sum(zi * fq[i][a] for i, zi in enumerate(z)) + beta * pi[a]) % pa
        slow = (Ta[a] * pq[a] + sum(vk * fqpq[k][a] for k, vk in enumerate(v)) + (pi[a] if negs else 0)) % pa
        assert fast == slow
    return True


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_fpq_matches_garner(cfg):
    n, p, qs = CONFIGS[cfg]
    c = consts(n, p, qs)
    ps, Q = c[0], c[1]
    rng = random.Random(17 + len(qs))
    pinv = pow(p, -1, Q)
    taken = 0
    cases = [[0] * len(qs), [q - 1 for q in qs]]
    cases += [[rng.randrange(q) for q in qs] for _ in range(2000)]
    # s driven to the centring boundary: p T == s (mod Q) for s next to floor(Q/2) and 2^-45 Q away
    for s in [Q // 2 - k for k in range(4)] + [Q // 2 + 1 + k for k in range(4)] + \
             [Q // 2 + sg * (Q >> 45) for sg in (-1, 1)] + [Q // 2 + sg * (Q >> 38) for sg in (-1, 1)]:
        x = s * pinv % Q
        cases.append([x % q for q in qs])
    for T in cases:
        Ta = [rng.randrange(2 * pa) for pa in ps]       # the tensor's [0, 2p) aux residues
        taken += check(T, Ta, p, qs, c)
    # every uniform case (and the zeros) takes the fast path, of the boundary ones only the two 2^-38 Q
    # away from Q/2 do
    assert taken == 2002 + 2, taken


def test_fpq_boundary_goes_to_garner():
    n, p, qs = CONFIGS["cfg3"]
    c = consts(n, p, qs)
    Q = c[1]
    pinv = pow(p, -1, Q)
    for s in (Q // 2, Q // 2 + 1, Q // 2 - (Q >> 45), Q // 2 + (Q >> 45)):
        x = s * pinv % Q
        _, f, b = fpq([x % q for q in qs], qs, c[3])
        assert abs(f - b) > LIM


@pytest.mark.parametrize("cfg", ["cfg4", "cfg5"])
def test_fpq_psum_deferred_dot(cfg):
    """exact_psum_sp_kernel's FPQ form: the products' z_i summed as integers (up to 15, then flushed) and
    their betas summed; fpq_flush reduces Z_i = r_i + k_i q_i and takes -k_i Pi_a with the betas.  Equal mod
    every p_a to adding each product's own y_a contribution (the per-product dot it replaces)."""
    n, p, qs = CONFIGS[cfg]
    c = consts(n, p, qs)
    ps, Q, pi, pz, fq = c[:5]
    rng = random.Random(5)
    for nprod in (0, 1, 2, 8, 15, 16, 31):
        carry = [rng.randrange(pa) for pa in ps]
        want = list(carry)
        Z, bs, cnt = [0] * len(qs), 0, 0

        def flush():
            nonlocal Z, bs, carry
            ks = 0
            rr = []
            for i, q in enumerate(qs):
                kq = Z[i] >> 60
                r = (Z[i] & ((1 << 60) - 1)) + kq * ((1 << 60) - q)
                assert r < 2 * q
                if r >= q:
                    r, kq = r - q, kq + 1
                assert Z[i] == r + kq * q
                ks += kq
                rr.append(r)
            carry = [(carry[a] + bs * pi[a] + ks * (pa - pi[a]) + sum(r * fq[i][a] for i, r in enumerate(rr))) % pa
                     for a, pa in enumerate(ps)]
            Z, bs = [0] * len(qs), 0

        for _ in range(nprod):
            z, f, b = fpq([rng.randrange(q) for q in qs], qs, pz)
            assert abs(f - b) <= LIM
            for a, pa in enumerate(ps):
                want[a] = (want[a] + sum(zi * fq[i][a] for i, zi in enumerate(z)) + int(b) * pi[a]) % pa
            Z = [Zi + zi for Zi, zi in zip(Z, z)]
            assert max(Z) < 1 << 64
            bs += int(b)
            cnt += 1
            if cnt == 15:
                flush()
                cnt = 0
        flush()
        assert carry == want, (cfg, nprod)
