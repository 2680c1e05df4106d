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
