"""CoeffsToSlots / SlotsToCoeffs — restates reference src/bootstrap/coeffs_to_slots.rs.

TEST ORACLE ONLY: the checker for exacto_{extract_coefficients,slots_to_coeffs}[_dev] and
exacto_required_trace_elements.  Galois keys are passed as a dict element -> GaloisKey, like the
reference's HashMap.
"""

from __future__ import annotations

from .bfv import BfvCiphertext, bfv_add, bfv_apply_automorphism, bfv_monomial_mul, bfv_plain_mul
from .modular import mod_inv
from .ring import CoeffPoly, ExactoError


def required_trace_elements(n: int) -> list[int]:
    """coeffs_to_slots.rs:168-183."""
    if n <= 32 or n & (n - 1):
        return list(range(3, 2 * n, 2))
    elems, step = [], n
    while step >= 2:
        elems.append(step + 1)
        step >>= 1
    return elems


def _key(galois_keys, k):
    if k not in galois_keys:
        raise ExactoError.invalid_param(f"missing Galois key for element {k}")
    return galois_keys[k]


def naive_trace(ct: BfvCiphertext, n: int, galois_keys) -> BfvCiphertext:
    """coeffs_to_slots.rs:79-95: ct + sum_{k odd, 3 <= k < 2n} sigma_k(ct) (every sigma of ct)."""
    result = ct.clone()
    for k in range(3, 2 * n, 2):
        result = bfv_add(result, bfv_apply_automorphism(ct, _key(galois_keys, k)))
    return result


def shifted_trace(ct: BfvCiphertext, n: int, galois_keys) -> BfvCiphertext:
    """coeffs_to_slots.rs:55-76: the relative-trace chain prod (1 + sigma_{s+1}) for n = 2^l > 32."""
    if n <= 32 or n & (n - 1):
        return naive_trace(ct, n, galois_keys)
    result = ct.clone()
    for k in required_trace_elements(n):
        result = bfv_add(result, bfv_apply_automorphism(result, _key(galois_keys, k)))
    return result


def extract_coefficient(ct: BfvCiphertext, j: int, galois_keys) -> BfvCiphertext:
    """coeffs_to_slots.rs:21-49: X^(2n-j) shift, trace, times n^-1 mod t."""
    params = ct.params
    n, t = params.ring_degree, params.plain_modulus
    shifted = ct.clone() if j == 0 else bfv_monomial_mul(ct, 2 * n - j)
    result = shifted_trace(shifted, n, galois_keys)
    n_inv = mod_inv(n % t, t)
    if n_inv is None:
        raise ExactoError.invalid_param("n not invertible mod t")
    scale = [0] * n
    scale[0] = n_inv
    return bfv_plain_mul(result, CoeffPoly(scale, t))


def coeffs_to_slots(ct: BfvCiphertext, galois_keys) -> list[BfvCiphertext]:
    """coeffs_to_slots.rs:103-115."""
    return [extract_coefficient(ct, j, galois_keys) for j in range(ct.params.ring_degree)]


def slots_to_coeffs(slots: list[BfvCiphertext]) -> BfvCiphertext:
    """coeffs_to_slots.rs:121-145: sum_j X^j ct_j."""
    if not slots:
        raise ExactoError.invalid_param("empty slots")
    n = slots[0].params.ring_degree
    if len(slots) != n:
        raise ExactoError.invalid_param(f"expected {n} slots, got {len(slots)}")
    result = slots[0].clone()
    for j in range(1, n):
        result = bfv_add(result, bfv_monomial_mul(slots[j], j))
    return result


# ---- digit extraction (bootstrap/digit_extract.rs) ----

def lagrange_interpolate(values: list[int], p: int) -> list[int]:
    """digit_extract.rs:37-90, literally (O(n^3)); small n only."""
    n = len(values)
    if n == 0:
        return []
    if n == 1:
        return [values[0] % p]
    result = [0] * n
    for j in range(n):
        if values[j] % p == 0:
            continue
        num, deg = [0] * n, 0
        num[0] = 1
        for k in range(n):
            if k == j:
                continue
            neg_k = (-(k % p)) % p
            new = [0] * n
            for d in range(deg + 1):
                if d + 1 < n:
                    new[d + 1] = (new[d + 1] + num[d]) % p
                new[d] = (new[d] + num[d] * neg_k) % p
            num, deg = new, deg + 1
        denom = 1
        for k in range(n):
            if k != j:
                denom = denom * ((j - k) % p) % p
        inv = mod_inv(denom, p)
        if inv is None:
            raise ExactoError.invalid_param("points must be distinct mod p")
        scale = values[j] % p * inv % p
        for d in range(n):
            result[d] = (result[d] + num[d] * scale) % p
    return result


def rounding_values(t_orig: int, q_prime: int, t_boot: int) -> list[int]:
    """digit_extract.rs:20-27."""
    return [(t_orig * (x % q_prime) + q_prime // 2) // q_prime % t_orig for x in range(t_boot)]


def compute_rounding_poly(t_orig: int, q_prime: int, t_boot: int) -> list[int]:
    """digit_extract.rs:19-30."""
    return lagrange_interpolate(rounding_values(t_orig, q_prime, t_boot), t_boot)


def trivial_encrypt_poly(pt: CoeffPoly, params) -> BfvCiphertext:
    """digit_extract.rs:179-189: (Delta m, 0)."""
    from .bfv import delta_residues
    from .ring import RnsPoly
    basis = params.ct_basis
    dr = delta_residues(params)
    c0 = RnsPoly.from_limb_coeffs([[(m % q) * d % q for m in pt.coeffs] for q, d in zip(basis.moduli, dr)], basis)
    c1 = RnsPoly.from_limb_coeffs([[0] * params.ring_degree for _ in basis.moduli], basis)
    return BfvCiphertext([c0, c1], params)


def trivial_encrypt(m: int, params) -> BfvCiphertext:
    """digit_extract.rs:160-176."""
    coeffs = [0] * params.ring_degree
    coeffs[0] = m % params.plain_modulus
    return trivial_encrypt_poly(CoeffPoly(coeffs, params.plain_modulus), params)


def bfv_scalar_mul(ct: BfvCiphertext, scalar: int) -> BfvCiphertext:
    """digit_extract.rs:192-197."""
    params = ct.params
    coeffs = [0] * params.ring_degree
    coeffs[0] = scalar % params.plain_modulus
    return bfv_plain_mul(ct, CoeffPoly(coeffs, params.plain_modulus))


def eval_poly_homomorphic(ct_x: BfvCiphertext, coeffs: list[int], rlk) -> BfvCiphertext:
    """digit_extract.rs:101-157 (Paterson-Stockmeyer with the reference's schedule)."""
    import math
    from .bfv import bfv_mul_and_relin
    params = ct_x.params
    d = max(len(coeffs) - 1, 0)
    if d == 0:
        return trivial_encrypt(coeffs[0], params)
    k = max(math.ceil(math.sqrt(d + 1.0)), 2)
    baby = [trivial_encrypt(1, params), ct_x.clone()]
    for i in range(2, k + 1):
        half = i // 2
        baby.append(bfv_mul_and_relin(baby[half], baby[i - half], rlk))
    groups = []
    for gi in range((d + k) // k):
        g = trivial_encrypt(0, params)
        for j in range(k):
            idx = gi * k + j
            if idx >= len(coeffs):
                break
            if coeffs[idx] == 0:
                continue
            g = bfv_add(g, bfv_scalar_mul(baby[j], coeffs[idx]))
        groups.append(g)
    result = groups.pop()
    while groups:
        result = bfv_add(bfv_mul_and_relin(result, baby[k], rlk), groups.pop())
    return result


# ---- bootstrap composition (bootstrap/bfv_host.rs) ----

def boot_key_images(s_coeffs: list[int], q_orig: int, q_boot: int, t_boot: int):
    """bfv_host.rs:68-86 (the plaintext bsk encrypts) and 296-315 (create_boot_sk's coefficients)."""
    s_pt, boot = [], []
    for c in s_coeffs:
        if c == 0:
            s_pt.append(0)
        elif c == 1:
            s_pt.append(1)
        elif c == q_orig - 1:
            s_pt.append(t_boot - 1)
        elif c > q_orig // 2:
            s_pt.append(t_boot - (q_orig - c) % t_boot)
        else:
            s_pt.append(c % t_boot)
        if c == 0:
            boot.append(0)
        elif c <= q_orig // 2:
            boot.append(c % q_boot)
        else:
            boot.append(q_boot - (q_orig - c) % q_boot)
    return s_pt, boot


def bfv_bootstrap(ct: BfvCiphertext, bsk_ct: BfvCiphertext, boot_rlk, galois_keys, rounding_poly, q_prime):
    """bfv_host.rs:131-205."""
    q = ct.params.ct_basis.moduli[0]
    boot_params = bsk_ct.params
    n = ct.params.ring_degree
    if len(ct.c) != 2:
        raise ExactoError.invalid_param("bootstrap requires degree-1 ciphertext")
    c0 = ct.c[0].to_coeff_poly(ct.params.ct_basis).coeffs
    c1 = ct.c[1].to_coeff_poly(ct.params.ct_basis).coeffs
    tb = boot_params.plain_modulus
    c0p = [(q_prime * c + q // 2) // q % q_prime for c in c0]
    c1p = [(q_prime * c + q // 2) // q % q_prime for c in c1]
    ct_c0 = trivial_encrypt_poly(CoeffPoly([c % tb for c in c0p], tb), boot_params)
    ct_c1s = bfv_plain_mul(bsk_ct, CoeffPoly([c % tb for c in c1p], tb))
    phase = bfv_add(ct_c0, ct_c1s)
    if all(c == 0 for c in c1):
        return eval_poly_homomorphic(phase, rounding_poly, boot_rlk)
    slots = coeffs_to_slots(phase, galois_keys)
    rounded = [eval_poly_homomorphic(s, rounding_poly, boot_rlk) for s in slots]
    result = rounded[0].clone()
    for j in range(1, n):
        result = bfv_add(result, bfv_monomial_mul(rounded[j], j))
    return result
