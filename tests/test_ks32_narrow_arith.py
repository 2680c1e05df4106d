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


# ---- the lazy basis (every prime below 2^30, 4p < 2^32: F32_LAZY in ks32_dev.hpp) ----

def _lazy_primes():
    """The three largest primes p = 1 mod 2n below 2^30 for n = 1024 / 4096 / 8192 (the lazy bases
    build_ks32_basis picks), and the smallest it may pick (just above 7/8 2^30)."""
    out = []
    for step in (2048, 8192, 16384):
        p, got = (1 << 30) - step + 1, 0
        while got < 3:
            if all(p % d for d in range(3, int(p ** 0.5) + 1, 2)):
                out.append(p)
                got += 1
            p -= step
    p = (7 << 27) // 8192 * 8192 + 8192 + 1
    while not all(p % d for d in range(3, int(p ** 0.5) + 1, 2)):
        p += 8192
    return out + [p]


def _shoup(x, w, p):
    ws = (w << 32) // p
    return (x * w - ((x * ws) >> 32) * p) & M32


def _lazy_fwd(x0, x1, w, p, canon=False):
    X = x0 if canon else min(x0, (x0 - 2 * p) & M32)
    qh = (x1 * ((w << 32) // p)) >> 32
    o0 = (qh * ((-p) & M32) + x1 * w + X) & M32
    o1 = (2 * X + 2 * p - o0) & M32
    return X, o0, o1


def _lazy_inv(u, v, w, p):
    s = (u + v) & M32
    return min(s, (s - 2 * p) & M32), _shoup((u + 2 * p - v) & M32, w, p)


def _red_s64_lz(x, p):
    """ks32.hip red_s64_lz: signed 64-bit x -> [0, 2p), x mod p."""
    c32 = (1 << 32) % p
    k63 = (-(1 << 63)) % p
    xu = x & ((1 << 64) - 1)
    hu = (xu >> 32) ^ 0x80000000
    a = _shoup(hu, c32, p)
    a = min(a, (a - p) & M32)
    lo = xu & M32
    b = (lo - (lo >> 30) * p) & M32
    s = (a + b + k63) & M32
    return min(s, (s - 2 * p) & M32)


def test_lazy_butterflies_bounds_and_congruence():
    rng = np.random.default_rng(30)
    for p in _lazy_primes():
        assert 4 * p <= M32
        cases = [(4 * p - 1, M32, p - 1), (0, 0, 0), (2 * p, 4 * p - 1, 1), (2 * p - 1, 2 * p - 1, p - 1)]
        cases += [(int(rng.integers(0, 4 * p)), int(rng.integers(0, 4 * p)), int(rng.integers(0, p)))
                  for _ in range(3000)]
        for x0, x1, w in cases:                      # forward: values in [0, 4p) between stages
            X, o0, o1 = _lazy_fwd(x0, x1, w, p)
            assert X < 2 * p and X % p == x0 % p
            assert o0 < 4 * p and 0 < o1 < 4 * p, (p, x0, x1, w, o0, o1)
            assert o0 % p == (x0 + x1 * w) % p and o1 % p == (x0 - x1 * w) % p
        for x0, x1, w in cases[:1000]:               # first stage of round 0: canonical X
            X, o0, o1 = _lazy_fwd(x0 % p, x1, w, p, canon=True)
            assert o0 < 4 * p and 0 < o1 < 4 * p
        for _, _, w in cases:                        # inverse: values in [0, 2p) between stages
            u, v = int(rng.integers(0, 2 * p)), int(rng.integers(0, 2 * p))
            o0, o1 = _lazy_inv(u, v, w, p)
            assert o0 < 2 * p and o1 < 2 * p
            assert o0 % p == (u + v) % p and o1 % p == ((u - v) * w) % p
        for u, v in [(2 * p - 1, 0), (0, 2 * p - 1), (2 * p - 1, 2 * p - 1)]:
            o0, o1 = _lazy_inv(u, v, p - 1, p)
            assert o0 < 2 * p and o1 < 2 * p


def _signed_first_stage(x0, x1, w, p):
    """fwd32_round SIN: int16 x0, x1 as int32 bits, one twiddle w; returns (o0, o1) as u32."""
    c = _shoup(1 << 15, w, p)
    c = min(c, (c - p) & M32)
    k1 = 2 * p - c if (p - c) < (1 << 15) else p - c
    k2 = c + 3 * p if c < (1 << 15) else c + 2 * p
    kd = (k2 - k1) & M32
    XK = (x0 + k1) & M32
    Y = (x1 + (1 << 15)) & M32
    qh = (Y * ((w << 32) // p)) >> 32
    o0 = (qh * ((-p) & M32) + Y * w + XK) & M32
    o1 = (2 * XK + kd - o0) & M32
    return o0, o1


def test_signed_first_stage_bounds_and_congruence():
    """The digit transform's first stage over raw int16 digits (ks32_dev.hpp fwd32_round SIN): both
    outputs in [0, 4p) and congruent to x0 +- x1 w, at the int16 extremes and for twiddles whose
    2^15 w mod p lands near 0 and p (the K1 / K2 adjustments)."""
    rng = np.random.default_rng(15)
    for p in _lazy_primes():
        ws = [int(v) for v in rng.integers(0, p, size=300)] + [0, 1, p - 1]
        inv = pow(1 << 15, -1, p)
        ws += [(c * inv) % p for c in (0, 1, (1 << 15) - 1, 1 << 15, p - 1, p - (1 << 15), p - (1 << 15) + 1)]
        edge = [-(1 << 15), -1, 0, 1, (1 << 15) - 1]
        for w in ws:
            xs = [(a, b) for a in edge for b in edge]
            xs += [(int(a), int(b)) for a, b in rng.integers(-(1 << 15), 1 << 15, size=(20, 2))]
            for a, b in xs:
                o0, o1 = _signed_first_stage(a & M32, b & M32, w, p)
                assert o0 < 4 * p and o1 < 4 * p, (p, w, a, b, o0, o1)
                assert o0 % p == (a + b * w) % p and o1 % p == (a - b * w) % p, (p, w, a, b)


def test_lazy_mac_reduction():
    """The MAC's lazy reduction of a signed 64-bit accumulator: [0, 2p), congruent (ks32.hip)."""
    rng = np.random.default_rng(64)
    for p in _lazy_primes():
        xs = [0, 1, -1, (1 << 63) - 1, -(1 << 63), (1 << 62) + 12345, -(1 << 62) - 777]
        xs += [int(v) for v in rng.integers(-(1 << 63), (1 << 63) - 1, size=2000, dtype=np.int64)]
        for x in xs:
            r = _red_s64_lz(x, p)
            assert r < 2 * p and r % p == x % p, (p, x, r)
