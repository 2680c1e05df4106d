"""CPU check of the narrow-prime 32-bit forward butterfly of exacto_amd/csrc/ks32_dev.hpp
(fwd32_round<..., NARROW = true>), step by step in 32-bit arithmetic as the kernel issues it:

    X  = red32(min(x0, x0 - 2p))                      x0 in [0, 3p]  ->  X in [0, p)
    qh = mulhi(x1, ws)                                ws = floor(w 2^32 / p)
    o0 = lo32(qh (2^32 - p) + (x1 w + X))             two v_mad_u64_u32, low words only
    o1 = 2X + 2p - o0

For every prime with 3p < 2^32 (the primary ks32 basis): o0 == x0 + x1 w, o1 == x0 - x1 w (mod p),
o0 < 3p and o1 <= 3p, i.e. the values stay in the [0, 3p] the next stage assumes.  The forward NTT
of the digits (keyswitch.rs:86-89 moved into the 31-bit basis) is a sequence of these butterflies;
the GPU parity of the whole key switch is tests/test_gpu_ks32.py."""

import numpy as np

M32 = (1 << 32) - 1


def _narrow(x0, x1, w, p):
    ws = (w << 32) // p
    t = (x0 - 2 * p) & M32
    a = min(x0, t)
    X = min(a, (a - p) & M32)
    qh = (x1 * ws) >> 32
    np_ = (-p) & M32
    o0 = (qh * np_ + x1 * w + X) & M32
    o1 = (2 * X + 2 * p - o0) & M32
    return X, o0, o1


def _primes():
    # primes of the primary basis shape: p = 1 mod 2n in (2^30, 2^32 / 3); the last one is the
    # largest p with 3p < 2^32 that is 1 mod 8192 and prime
    out = []
    p = (0x55555555 // 8192) * 8192 + 1
    while len(out) < 3:
        if p <= 0x55555555 and all(p % d for d in range(3, int(p ** 0.5) + 1, 2)):
            out.append(p)
        p -= 8192
    return out + [1073750017]   # a prime just above 2^30


def test_narrow_butterfly_bounds_and_congruence():
    rng = np.random.default_rng(32)
    for p in _primes():
        assert 3 * p <= M32
        cases = [(3 * p, M32, p - 1), (0, 0, 0), (2 * p, 3 * p, 1), (p, 2 * p - 1, p - 1), (3 * p, 3 * p, p - 1)]
        cases += [(int(rng.integers(0, 3 * p + 1)), int(rng.integers(0, 3 * p + 1)), int(rng.integers(0, p)))
                  for _ in range(4000)]
        for x0, x1, w in cases:
            X, o0, o1 = _narrow(x0, x1, w, p)
            assert X < p and X % p == x0 % p
            assert o0 < 3 * p and 0 < o1 <= 3 * p, (p, x0, x1, w, o0, o1)
            assert o0 % p == (x0 + x1 * w) % p
            assert o1 % p == (x0 - x1 * w) % p
