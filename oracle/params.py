"""L2 parameters — restates reference src/params/{mod,presets}.rs (TEST ORACLE ONLY).

Also defines the five BASELINE.json configurations.
"""

from __future__ import annotations

from .ring import ExactoError, RnsBasis, is_power_of_two


class BfvParams:
    """params/mod.rs:12-27."""

    def __init__(self, ring_degree, plain_modulus, ct_basis, aux_basis, sigma, gadget_base,
                 gadget_digits):
        self.ring_degree = ring_degree
        self.plain_modulus = plain_modulus
        self.ct_basis = ct_basis
        self.aux_basis = aux_basis
        self.sigma = sigma
        self.gadget_base = gadget_base
        self.gadget_digits = gadget_digits


def compute_gadget_digits(ct_moduli, base) -> int:
    """params/mod.rs:126-140: smallest G with base^G >= Q (at least 1)."""
    q_big = 1
    for q in ct_moduli:
        q_big *= q
    pow_, digits = 1, 0
    while pow_ < q_big:
        pow_ *= base
        digits += 1
    return max(digits, 1)


class BfvParamsBuilder:
    """params/mod.rs:30-124."""

    def __init__(self):
        self._n = 4096
        self._p = 65537
        self._ct = []
        self._aux = []
        self._sigma = 3.2
        self._base = 0

    def ring_degree(self, n):
        self._n = n
        return self

    def plain_modulus(self, p):
        self._p = p
        return self

    def ct_moduli(self, m):
        self._ct = list(m)
        return self

    def aux_moduli(self, m):
        self._aux = list(m)
        return self

    def sigma(self, s):
        self._sigma = s
        return self

    def gadget_base(self, b):
        self._base = b
        return self

    def build(self) -> BfvParams:
        if not is_power_of_two(self._n) or self._n < 2:
            raise ExactoError.invalid_ring_degree(self._n)
        if not self._ct:
            raise ExactoError.invalid_param("must specify at least one ciphertext modulus")
        if self._p < 2:
            raise ExactoError.invalid_param("plaintext modulus must be >= 2")
        ct_basis = RnsBasis(self._ct, self._n)
        aux_basis = RnsBasis(self._aux, self._n) if self._aux else None
        base = (1 << 16) if self._base == 0 else self._base
        digits = max(compute_gadget_digits(self._ct, base), 1)
        return BfvParams(self._n, self._p, ct_basis, aux_basis, self._sigma, base, digits)


class DbfvParams:
    """params/mod.rs:144-193 (plain_modulus 0 == 2^64)."""

    def __init__(self, bfv_params, base, num_digits, plain_modulus):
        if base < 2:
            raise ExactoError.invalid_param("base must be >= 2")
        if num_digits < 1:
            raise ExactoError.invalid_param("num_digits must be >= 1")
        bd = 1
        for _ in range(num_digits):
            bd = min(bd * base, (1 << 128) - 1)  # saturating_mul
        p128 = (1 << 64) if plain_modulus == 0 else plain_modulus
        if bd < p128:
            raise ExactoError.invalid_param(f"base^digits = {bd} < plain_modulus = {p128}")
        self.bfv_params = bfv_params
        self.base = base
        self.num_digits = num_digits
        self.plain_modulus = plain_modulus


# ------------------------------------------------------------------ presets (presets.rs)

def compact_bfv():
    """presets.rs:24-35."""
    return (BfvParamsBuilder().ring_degree(1024).plain_modulus(257)
            .ct_moduli([1099509805057]).aux_moduli([562949953443841]).sigma(3.2).build())


def small_bfv():
    """presets.rs:39-51."""
    return (BfvParamsBuilder().ring_degree(4096).plain_modulus(65537)
            .ct_moduli([576460752308273153]).sigma(3.2).build())


def u64_dbfv():
    """presets.rs:61-75."""
    bfv = (BfvParamsBuilder().ring_degree(4096).plain_modulus(1040407)
           .ct_moduli([1152921504606830593])
           .aux_moduli([18014398509998081, 36028797018972161])
           .gadget_base(256).sigma(3.2).build())
    return DbfvParams(bfv, 256, 8, 0)


def compact_dbfv():
    """presets.rs:86-98."""
    bfv = (BfvParamsBuilder().ring_degree(1024).plain_modulus(929)
           .ct_moduli([1099509805057]).aux_moduli([562949953443841]).sigma(3.2).build())
    return DbfvParams(bfv, 16, 2, 256)


# ------------------------------------------------------------------ BASELINE configs

Q3 = [1152921504606830593, 1152921504606748673, 1152921504606683137]
Q4 = Q3 + [1152921504606601217]


def cfg1_params():
    """BASELINE configs[0]: compact_bfv."""
    return compact_bfv()


def cfg2_modulus():
    """BASELINE configs[1]: n=4096, 1x60-bit q (u64_dbfv's prime, presets.rs:66)."""
    return 4096, 1152921504606830593


def cfg3_params(n=4096):
    """BASELINE configs[2]: n=4096, 3x60-bit limbs, p=65537 (builder default), base 2^16."""
    return BfvParamsBuilder().ring_degree(n).plain_modulus(65537).ct_moduli(Q3).build()


def cfg4_params(n=4096):
    """BASELINE configs[3]: dBFV p=2^16, b=256, d=2 over cfg3's basis; t=260111."""
    bfv = BfvParamsBuilder().ring_degree(n).plain_modulus(260111).ct_moduli(Q3).build()
    return DbfvParams(bfv, 256, 2, 65536)


def cfg5_params(n=8192):
    """BASELINE configs[4]: u64 profile p=2^64, b=256, d=8, t=1040407, gadget 256, 4x60-bit."""
    bfv = (BfvParamsBuilder().ring_degree(n).plain_modulus(1040407).ct_moduli(Q4)
           .gadget_base(256).build())
    return DbfvParams(bfv, 256, 8, 0)
