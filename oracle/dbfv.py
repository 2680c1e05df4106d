"""L4 dBFV on the multiply path — restates reference src/dbfv/{eval,reduction}.rs (TEST ORACLE ONLY)."""

from __future__ import annotations

from . import bfv
from .ring import ExactoError


class DbfvCiphertext:
    """dbfv/ciphertext.rs:10-22."""

    def __init__(self, limbs, degree, mul_depth, params):
        self.limbs = limbs
        self.degree = degree
        self.mul_depth = mul_depth
        self.params = params

    def num_limbs(self):
        return len(self.limbs)


def digit_decompose(value: int, base: int, num_digits: int) -> list[int]:
    """dbfv/decomposition.rs:8-16 (unsigned digits, excess dropped)."""
    out = []
    rem = value
    for _ in range(num_digits):
        out.append(rem % base)
        rem //= base
    return out


def digit_recompose_signed(digits, base, modulus, bfv_plain_mod) -> int:
    """dbfv/decomposition.rs:46-69."""
    half_t = bfv_plain_mod // 2
    result, power = 0, 1
    for d in digits:
        c = d - bfv_plain_mod if d > half_t else d
        result += c * power
        power *= base
    if modulus == 0:
        return result % (1 << 64)
    return result % modulus


def small_reps(base: int, d: int, p: int) -> list[list[int]]:
    """lattice.rs:104-122 SmallReps::compute_simple (p = 0 means 2^64, wrapping_pow)."""
    reps = []
    for j in range(d, 2 * d - 1):
        val = pow(base, j, 1 << 64) if p == 0 else pow(base, j, p)
        reps.append(digit_decompose(val, base, d))
    return reps


def reduce(ct: DbfvCiphertext, rlk=None) -> DbfvCiphertext:
    """reduction.rs:15-60: fold limbs j >= d into limbs i < d with the small reps."""
    params = ct.params
    d = params.num_digits
    if ct.degree <= d:
        return ct
    reps = small_reps(params.base, d, params.plain_modulus)
    res = list(ct.limbs[:d])
    for j in range(d, len(ct.limbs)):
        ri = j - d
        if ri >= len(reps):
            continue
        rep = reps[ri]
        for i in range(d):
            coeff = rep[i]
            if coeff == 0:
                continue
            res[i] = bfv.bfv_add(res[i], _scale_ct(ct.limbs[j], coeff))
    return DbfvCiphertext(res, d, ct.mul_depth, params)


def _scale_ct(ct, scalar: int):
    """reduction.rs:65-93."""
    scaled = bfv.BfvCiphertext([c.scalar_mul(abs(scalar)) for c in ct.c], ct.params)
    return bfv.bfv_neg(scaled) if scalar < 0 else scaled


def dbfv_mul(ct1: DbfvCiphertext, ct2: DbfvCiphertext, rlk, bypass_depth_guard=False):
    """dbfv/eval.rs:82-149.

    ``bypass_depth_guard`` reproduces paper_repro's chain semantics (mul_depth reset to 0 before
    each step, src/bin/paper_repro.rs:155-158, 217-220)."""
    params = ct1.params
    d = params.num_digits
    if ct1.num_limbs() != d or ct2.num_limbs() != d:
        raise ExactoError.invalid_param("multiplication requires d-limb ciphertexts")
    depth1 = 0 if bypass_depth_guard else ct1.mul_depth
    depth2 = 0 if bypass_depth_guard else ct2.mul_depth
    next_depth = max(depth1, depth2) + 1
    if next_depth > 1:
        raise ExactoError.not_implemented(
            "chained dBFV multiplication requires ciphertext-level lattice reduction (paper §4.6.2)")
    result_len = 2 * d - 1
    limbs = [None] * result_len
    for i in range(d):
        for j in range(d):
            prod = bfv.bfv_mul_and_relin(ct1.limbs[i], ct2.limbs[j], rlk)
            k = i + j
            limbs[k] = prod if limbs[k] is None else bfv.bfv_add(limbs[k], prod)
    out = DbfvCiphertext(limbs, result_len, next_depth, params)
    return reduce(out, rlk)


def needed_pairs(params):
    """(i, j) products whose output survives ``reduce`` (all pairs with i+j < d, plus those
    feeding a limb j >= d whose small representative has a nonzero digit)."""
    d = params.num_digits
    reps = small_reps(params.base, d, params.plain_modulus)
    keep = []
    for i in range(d):
        for j in range(d):
            k = i + j
            if k < d or any(reps[k - d]):
                keep.append((i, j))
    return keep


def dbfv_encrypt_scalar_sk(value: int, sk, params, rng) -> DbfvCiphertext:
    """dbfv/encrypt.rs (scalar): base-b digits, each encoded as a BFV scalar."""
    digits = digit_decompose(value, params.base, params.num_digits)
    limbs = [bfv.encrypt_sk(bfv.encode_scalar(dg, params.bfv_params), sk, rng) for dg in digits]
    return DbfvCiphertext(limbs, params.num_digits, 0, params)


def dbfv_decrypt_scalar(ct: DbfvCiphertext, sk) -> int:
    """dbfv/decrypt.rs:20-43 (coefficient 0 of each limb, signed recomposition)."""
    params = ct.params
    t = params.bfv_params.plain_modulus
    digits = [bfv.decode_scalar(bfv.decrypt(l, sk)) for l in ct.limbs]
    use = min(params.num_digits, len(digits))
    return digit_recompose_signed(digits[:use], params.base, params.plain_modulus, t)


def dbfv_decrypt_poly(ct: DbfvCiphertext, sk):
    """dbfv/decrypt.rs:48-79: per-limb BFV decrypt, signed recomposition of every coefficient."""
    params = ct.params
    if params.plain_modulus == 0:
        raise ExactoError.invalid_param(
            "polynomial dBFV decrypt requires finite plain_modulus (plain_modulus=0 is scalar-only)")
    t = params.bfv_params.plain_modulus
    use = min(params.num_digits, len(ct.limbs))
    polys = [bfv.decrypt(l, sk).coeffs for l in ct.limbs[:use]]
    n = min(len(p) for p in polys)
    return [digit_recompose_signed([p[i] for p in polys], params.base, params.plain_modulus, t)
            for i in range(n)]
