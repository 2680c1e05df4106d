"""CPU checks of the integer identities behind the SP scale/lift kernels (kernels.hip):

- dot30_fold: a sum of up to 7 products of 60-bit operands, kept as three 30-bit-limb columns and
  folded through 2^60 == d for q = 2^60 - d, equals the exact sum mod q, including at the column
  bounds the kernel comment states;
- gadget_digits16_sp: balanced base-2^sh digits read from the magnitude's fields with a 1-bit
  carry equal the digits of the multiword-increment form (gadget_digits, keyswitch.rs:24-44).

Python restatements of the device arithmetic (64-bit wrap modelled explicitly), not the kernels.
"""
import random

import pytest

M64 = (1 << 64) - 1
M30 = (1 << 30) - 1
SPECIAL = [1152921504606830593, 1152921504606748673, 1152921504606683137, 1152921504606601217]


def dot30(xs, cs, add0=0):
    a0, a1, a2 = add0, 0, 0
    for x, c in zip(xs, cs):
        x0, x1, c0, c1 = x & M30, x >> 30, c & M30, c >> 30
        a0 += x0 * c0
        a1 += x0 * c1 + x1 * c0
        a2 += x1 * c1
    assert max(a0, a1, a2) < 1 << 64        # no column carries out of its 64-bit register
    return a0, a1, a2


def fold(a0, a1, a2, q):
    d = (1 << 60) - q
    H = (a2 + (a1 >> 30)) & M64
    F = (H >> 32) * d
    x = a0 + (H & 0xFFFFFFFF) * d
    x += (a1 & M30) << 30
    x += (F & ((1 << 28) - 1)) << 32
    x += (F >> 28) * d
    assert x < 1 << 64
    r = (x & ((1 << 60) - 1)) + (x >> 60) * d
    return r - q if r >= q else r


@pytest.mark.parametrize("m", [1, 3, 4, 5, 7])
def test_dot30_fold_exact(m):
    rng = random.Random(m)
    for q in SPECIAL:
        for trial in range(400):
            if trial < 4:   # extremes: every operand at its maximum
                xs = [q - 1] * m
                cs = [q - 1 if trial & 1 else (1 << 60) - 1 - (trial >> 1)] * m
                add0 = q - 1 if trial & 2 else 0
            else:
                xs = [rng.randrange(q) for _ in range(m)]
                cs = [rng.randrange(1, q + 1) for _ in range(m)]   # complements reach q itself
                add0 = rng.choice([0, 1, rng.randrange(q + 1)])
            want = (sum(x * c for x, c in zip(xs, cs)) + add0) % q
            assert fold(*dot30(xs, cs, add0), q) == want


def digits_multiword(v, Q, sh, G):
    """gadget_digits: magnitude, truncating remainder, balance, carry added back to the magnitude."""
    B, half = 1 << sh, 1 << (sh - 1)
    neg = v > Q // 2
    M = Q - v if neg else v
    out = []
    for _ in range(G):
        r = M & (B - 1)
        M >>= sh
        if not neg:
            if r >= half:
                out.append(-(B - r)); M += 1
            else:
                out.append(r)
        else:
            if r > half:
                out.append(B - r); M += 1
            else:
                out.append(-r)
    return out


def digits_fields(v, Q, sh, G, words):
    """gadget_digits16_sp: fields of the 32-bit words of the magnitude plus a 1-bit carry."""
    B = 1 << sh
    neg = v > Q // 2
    M = Q - v if neg else v
    thr = (B >> 1) - (0 if neg else 1)
    out, c, g = [], 0, 0
    for w in range(words):
        word = (M >> (32 * w)) & 0xFFFFFFFF
        for o in range(0, 32, sh):
            if g >= G:
                break
            r = ((word >> o) & (B - 1)) + c
            c = 1 if r > thr else 0
            dv = r - (c << sh)
            out.append(-dv if neg else dv)
            g += 1
    while g < G:
        r = c
        c = 1 if r > thr else 0
        dv = r - (c << sh)
        out.append(-dv if neg else dv)
        g += 1
    return out


@pytest.mark.parametrize("L,sh", [(1, 16), (2, 16), (3, 16), (3, 8), (4, 8), (2, 4)])
def test_gadget_digit_fields_match_multiword(L, sh):
    rng = random.Random(L * 100 + sh)
    Q = 1
    for q in SPECIAL[:L]:
        Q *= q
    G = 1
    while (1 << (sh * G)) < Q:
        G += 1
    specials = [0, 1, Q - 1, Q // 2, Q // 2 + 1, Q // 2 - 1]
    # runs of ones in the magnitude make the carry ripple through whole fields
    for k in range(1, 8):
        specials += [(1 << (sh * k)) - 1, Q - ((1 << (sh * k)) - 1), (1 << (sh * k - 1))]
    vals = [x % Q for x in specials] + [rng.randrange(Q) for _ in range(3000)]
    for v in vals:
        want = digits_multiword(v, Q, sh, G)
        assert digits_fields(v, Q, sh, G, 2 * L) == want
        assert all(-(1 << (sh - 1)) <= d <= (1 << (sh - 1)) for d in want)
