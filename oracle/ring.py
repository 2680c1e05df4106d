"""L1 polynomial rings — restates reference src/ring/{poly,ntt,rns}.rs (TEST ORACLE ONLY).

The NTT engine of the reference is the third-party crate concrete-ntt 0.2.0
(``prime64::Plan``; call sites src/ring/ntt.rs:24,43,49,60,62 and
src/ring/rns.rs:36-38).  Its source is not in the container, so ``NttPlan``
below states THIS BUILD's convention, which the HIP kernels implement
bit-for-bit:

* psi = x^((q-1)/2n) for the smallest x = 2, 3, ... with psi^n == -1 (mod q);
* forward = Cooley-Tukey negacyclic NTT, natural-order input, bit-reversed
  evaluation order: evaluation k = a(psi^(2*brv(k)+1)) (Longa-Naehrig 2016,
  Alg. 1), stored at position (k mod 16) n/16 + k // 16 (``storage_order``;
  round 5: the order in which the device threads hold their values, so the
  device loads and stores of NTT-domain data are contiguous);
* inverse = Gentleman-Sande from that storage, natural output, unscaled;
  ``normalize`` multiplies by n^-1 (concrete-ntt's inv/normalize split,
  pinned by the roundtrip KAT ntt.rs:170-178).

Everything observable after ``to_coeff_poly`` is convention-independent, which
is exactly what the reference's own NTT tests pin (ntt.rs:170-212).
"""

from __future__ import annotations

from .modular import (barrett_constant, mod_add, mod_inv, mod_mul, mod_neg, mod_sub,
                      is_prime, U64)


class ExactoError(Exception):
    """Mirror of reference src/error.rs:4-31 (variant name + Display text)."""

    VARIANTS = ("InvalidParam", "DimensionMismatch", "ModulusMismatch", "InvalidRingDegree",
                "DecryptionError", "DecompositionError", "LatticeError", "MissingKey",
                "NotImplemented")

    def __init__(self, variant: str, message: str):
        assert variant in self.VARIANTS
        super().__init__(message)
        self.variant = variant
        self.code = self.VARIANTS.index(variant) + 1

    # constructors mirroring the #[error(...)] strings
    @classmethod
    def invalid_param(cls, s):
        return cls("InvalidParam", f"invalid parameter: {s}")

    @classmethod
    def dimension_mismatch(cls, expected, got):
        return cls("DimensionMismatch", f"dimension mismatch: expected {expected}, got {got}")

    @classmethod
    def modulus_mismatch(cls):
        return cls("ModulusMismatch", "modulus mismatch")

    @classmethod
    def invalid_ring_degree(cls, n):
        return cls("InvalidRingDegree", f"ring degree must be a power of 2, got {n}")

    @classmethod
    def not_implemented(cls, s):
        return cls("NotImplemented", f"not yet implemented: {s}")


def is_power_of_two(n: int) -> bool:
    return n > 0 and (n & (n - 1)) == 0


def bit_reverse(x: int, bits: int) -> int:
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def find_psi(n: int, q: int) -> int:
    """Primitive 2n-th root of unity: smallest x >= 2 whose x^((q-1)/2n) has order 2n."""
    e = (q - 1) // (2 * n)
    x = 2
    while True:
        psi = pow(x, e, q)
        if pow(psi, n, q) == q - 1:
            return psi
        x += 1


class NttPlan:
    """Replacement for concrete_ntt::prime64::Plan (ntt.rs:19-29 make_plan)."""

    def __init__(self, n: int, q: int):
        self.n = n
        self.q = q
        self.logn = n.bit_length() - 1
        self.psi = find_psi(n, q)
        psi_inv = pow(self.psi, q - 2, q)
        self.psi_rev = [pow(self.psi, bit_reverse(i, self.logn), q) for i in range(n)]
        self.psi_inv_rev = [pow(psi_inv, bit_reverse(i, self.logn), q) for i in range(n)]
        self.n_inv = pow(n, q - 2, q)

    @staticmethod
    def try_new(n: int, q: int):
        # concrete-ntt: power-of-two size >= 16, prime modulus == 1 mod 2n.
        if n < 16 or not is_power_of_two(n):
            return None
        if q <= 1 or q >= (1 << 64) or (q - 1) % (2 * n) != 0 or not is_prime(q):
            return None
        return NttPlan(n, q)

    def modulus(self) -> int:
        return self.q

    def storage_order(self) -> list[int]:
        """position -> evaluation index of this build's NTT-domain storage: position
        (k mod 16) (n/16) + k // 16 holds evaluation k = a(psi^(2 brv(k) + 1)) (the order in which
        the device transforms' threads hold their 16 values; the identity at n = 16)."""
        T = self.n // 16
        return [((p % T) << 4) | (p // T) for p in range(self.n)]

    def fwd(self, a: list[int]) -> None:
        """In-place forward negacyclic NTT (Cooley-Tukey, bit-reversed evaluation order), stored in
        storage_order()."""
        n, q, tw = self.n, self.q, self.psi_rev
        t = n
        m = 1
        while m < n:
            t >>= 1
            for i in range(m):
                j1 = 2 * i * t
                s = tw[m + i]
                for j in range(j1, j1 + t):
                    u = a[j]
                    v = a[j + t] * s % q
                    a[j] = (u + v) % q
                    a[j + t] = (u - v) % q
            m <<= 1
        std = list(a)
        for p, k in enumerate(self.storage_order()):
            a[p] = std[k]

    def inv(self, a: list[int]) -> None:
        """In-place inverse (Gentleman-Sande, input in storage_order()), NOT scaled by n^-1."""
        n, q, tw = self.n, self.q, self.psi_inv_rev
        stored = list(a)
        for p, k in enumerate(self.storage_order()):
            a[k] = stored[p]
        t = 1
        m = n
        while m > 1:
            h = m >> 1
            j1 = 0
            for i in range(h):
                s = tw[h + i]
                for j in range(j1, j1 + t):
                    u = a[j]
                    v = a[j + t]
                    a[j] = (u + v) % q
                    a[j + t] = (u - v) * s % q
                j1 += 2 * t
            t <<= 1
            m = h

    def normalize(self, a: list[int]) -> None:
        ni, q = self.n_inv, self.q
        for i in range(len(a)):
            a[i] = a[i] * ni % q


def make_plan(n: int, modulus: int) -> NttPlan:
    """ntt.rs:19-29."""
    if not is_power_of_two(n) or n < 2:
        raise ExactoError.invalid_ring_degree(n)
    plan = NttPlan.try_new(n, modulus)
    if plan is None:
        raise ExactoError.invalid_param(
            f"cannot create NTT plan for n={n}, q={modulus} (need prime q ≡ 1 mod {2 * n}")
    return plan


# ------------------------------------------------------------------ CoeffPoly (poly.rs)

class CoeffPoly:
    """poly.rs:6-9."""

    def __init__(self, coeffs: list[int], modulus: int):
        self.coeffs = list(coeffs)
        self.modulus = modulus

    @classmethod
    def zero(cls, n, modulus):
        return cls([0] * n, modulus)

    @classmethod
    def from_coeffs(cls, coeffs, modulus):
        """poly.rs:21-25 (reduces mod q)."""
        return cls([c % modulus for c in coeffs], modulus)

    def __len__(self):
        return len(self.coeffs)

    def __eq__(self, other):
        return self.modulus == other.modulus and self.coeffs == other.coeffs

    def _check(self, other):
        if len(self) != len(other):
            raise ExactoError.dimension_mismatch(len(self), len(other))
        if self.modulus != other.modulus:
            raise ExactoError.modulus_mismatch()

    def add(self, other):
        """poly.rs:40-55."""
        self._check(other)
        return CoeffPoly([mod_add(a, b, self.modulus) for a, b in zip(self.coeffs, other.coeffs)],
                         self.modulus)

    def sub(self, other):
        """poly.rs:58-73."""
        self._check(other)
        return CoeffPoly([mod_sub(a, b, self.modulus) for a, b in zip(self.coeffs, other.coeffs)],
                         self.modulus)

    def neg(self):
        """poly.rs:76-81."""
        return CoeffPoly([mod_neg(a, self.modulus) for a in self.coeffs], self.modulus)

    def mul_naive(self, other):
        """poly.rs:85-120: O(n^2) negacyclic schoolbook (the reference's test oracle)."""
        self._check(other)
        n, q = len(self), self.modulus
        bk = barrett_constant(q)
        res = [0] * n
        for i in range(n):
            ai = self.coeffs[i]
            if ai == 0:
                continue
            for j in range(n):
                bj = other.coeffs[j]
                if bj == 0:
                    continue
                prod = mod_mul(ai, bj, q, bk)
                idx = i + j
                if idx < n:
                    res[idx] = mod_add(res[idx], prod, q)
                else:
                    res[idx - n] = mod_sub(res[idx - n], prod, q)
        return CoeffPoly(res, q)

    def scalar_mul(self, scalar):
        """poly.rs:123-131."""
        q = self.modulus
        bk = barrett_constant(q)
        s = scalar % q
        return CoeffPoly([mod_mul(c, s, q, bk) for c in self.coeffs], q)

    def is_zero(self):
        return all(c == 0 for c in self.coeffs)

    def centered_coeffs(self):
        """poly.rs:138-147."""
        half = self.modulus // 2
        return [c - self.modulus if c > half else c for c in self.coeffs]


# ------------------------------------------------------------------ NttPoly (ntt.rs)

class NttPoly:
    """ntt.rs:11-15: evaluation-domain polynomial (the at-rest ciphertext form)."""

    def __init__(self, evals: list[int], modulus: int, plan: NttPlan):
        self.evals = evals
        self.modulus = modulus
        self.plan = plan

    @classmethod
    def zero(cls, n, modulus, plan):
        return cls([0] * n, modulus, plan)

    @classmethod
    def from_coeff_poly(cls, poly: CoeffPoly, plan: NttPlan):
        """ntt.rs:42-55."""
        if poly.modulus != plan.modulus():
            raise ExactoError.modulus_mismatch()
        evals = list(poly.coeffs)
        plan.fwd(evals)
        return cls(evals, poly.modulus, plan)

    def to_coeff_poly(self) -> CoeffPoly:
        """ntt.rs:58-67: inv + normalize."""
        c = list(self.evals)
        self.plan.inv(c)
        self.plan.normalize(c)
        return CoeffPoly(c, self.modulus)

    def __len__(self):
        return len(self.evals)

    def __eq__(self, other):
        return self.modulus == other.modulus and self.evals == other.evals

    def _check(self, other):
        if len(self) != len(other) or self.modulus != other.modulus:
            raise ExactoError.modulus_mismatch()

    def add(self, other):
        """ntt.rs:75-89."""
        self._check(other)
        q = self.modulus
        return NttPoly([a + b - q if a + b >= q else a + b for a, b in zip(self.evals, other.evals)],
                       q, self.plan)

    def sub(self, other):
        """ntt.rs:92-105."""
        self._check(other)
        q = self.modulus
        return NttPoly([a - b if a >= b else q - b + a for a, b in zip(self.evals, other.evals)],
                       q, self.plan)

    def neg(self):
        """ntt.rs:108-113."""
        q = self.modulus
        return NttPoly([0 if a == 0 else q - a for a in self.evals], q, self.plan)

    def mul(self, other):
        """ntt.rs:119-129 (pointwise, u128 % for q > 2^32)."""
        self._check(other)
        q = self.modulus
        bk = barrett_constant(q)
        return NttPoly([mod_mul(a, b, q, bk) for a, b in zip(self.evals, other.evals)], q, self.plan)

    def scalar_mul(self, scalar):
        """ntt.rs:132-139."""
        q = self.modulus
        s = scalar % q
        bk = barrett_constant(q)
        return NttPoly([mod_mul(a, s, q, bk) for a in self.evals], q, self.plan)

    def is_zero(self):
        return all(e == 0 for e in self.evals)


# ------------------------------------------------------------------ RNS (rns.rs)

class RnsBasis:
    """rns.rs:21-63."""

    def __init__(self, moduli: list[int], ring_degree: int):
        self.plans = [make_plan(ring_degree, q) for q in moduli]
        self.moduli = list(moduli)
        self.ring_degree = ring_degree
        self.barrett_ks = [barrett_constant(q) for q in moduli]
        self.q_star_inv = []
        for i, qi in enumerate(moduli):
            prod = 1
            for j, qj in enumerate(moduli):
                if i != j:
                    prod = mod_mul(prod, qj % qi, qi, self.barrett_ks[i])
            inv = mod_inv(prod, qi)
            if inv is None:
                raise AssertionError("RNS moduli must be coprime")
            self.q_star_inv.append(inv)

    def num_moduli(self):
        return len(self.moduli)

    def product(self) -> int:
        p = 1
        for q in self.moduli:
            p *= q
        return p


class RnsPoly:
    """rns.rs:14-17: L NttPoly limbs."""

    def __init__(self, components: list[NttPoly], ring_degree: int):
        self.components = components
        self.ring_degree = ring_degree

    @classmethod
    def zero(cls, basis: RnsBasis):
        return cls([NttPoly.zero(basis.ring_degree, q, p) for q, p in zip(basis.moduli, basis.plans)],
                   basis.ring_degree)

    @classmethod
    def from_coeff_poly(cls, poly: CoeffPoly, basis: RnsBasis):
        """rns.rs:84-105: reduce each coefficient mod q_i, then forward NTT."""
        if len(poly) != basis.ring_degree:
            raise ExactoError.dimension_mismatch(basis.ring_degree, len(poly))
        comps = []
        for q, plan in zip(basis.moduli, basis.plans):
            reduced = CoeffPoly.from_coeffs([c % q for c in poly.coeffs], q)
            comps.append(NttPoly.from_coeff_poly(reduced, plan))
        return cls(comps, basis.ring_degree)

    @classmethod
    def from_limb_coeffs(cls, limbs: list[list[int]], basis: RnsBasis):
        """Build from per-limb coefficient vectors (already reduced mod q_i)."""
        comps = [NttPoly.from_coeff_poly(CoeffPoly(c, q), plan)
                 for c, q, plan in zip(limbs, basis.moduli, basis.plans)]
        return cls(comps, basis.ring_degree)

    def to_coeff_poly(self, basis: RnsBasis) -> CoeffPoly:
        """rns.rs:114-151 under extension semantics.

        L = 1: limb 0 (rns.rs:130-132).  L > 1: exact CRT into [0, Q) with
        ``modulus = Q``.  For Q < 2^64 this is bit-identical to the reference's
        u128 computation; for Q >= 2^64 the reference truncates/overflows
        (rns.rs:135,147,150) and this is the documented extension.
        """
        coeff_components = [c.to_coeff_poly() for c in self.components]
        if len(basis.moduli) == 1:
            return coeff_components[0]
        return CoeffPoly(crt_exact([cc.coeffs for cc in coeff_components], basis), basis.product())

    def limb_coeffs(self) -> list[list[int]]:
        return [c.to_coeff_poly().coeffs for c in self.components]

    def num_components(self):
        return len(self.components)

    def _check(self, other):
        if len(self.components) != len(other.components):
            raise ExactoError.dimension_mismatch(len(self.components), len(other.components))

    def add(self, other):
        self._check(other)
        return RnsPoly([a.add(b) for a, b in zip(self.components, other.components)], self.ring_degree)

    def sub(self, other):
        self._check(other)
        return RnsPoly([a.sub(b) for a, b in zip(self.components, other.components)], self.ring_degree)

    def neg(self):
        return RnsPoly([a.neg() for a in self.components], self.ring_degree)

    def mul(self, other):
        self._check(other)
        return RnsPoly([a.mul(b) for a, b in zip(self.components, other.components)], self.ring_degree)

    def scalar_mul(self, scalar):
        return RnsPoly([a.scalar_mul(scalar) for a in self.components], self.ring_degree)

    def clone(self):
        return RnsPoly([NttPoly(list(c.evals), c.modulus, c.plan) for c in self.components],
                       self.ring_degree)


def crt_exact(limb_coeffs: list[list[int]], basis: RnsBasis) -> list[int]:
    """x_j = sum_i (c_ij * q*_inv_i mod q_i) * (Q/q_i) mod Q, exactly (rns.rs:138-148)."""
    Q = basis.product()
    terms = []
    for i, qi in enumerate(basis.moduli):
        terms.append((qi, basis.q_star_inv[i], Q // qi))
    n = len(limb_coeffs[0])
    out = [0] * n
    for j in range(n):
        v = 0
        for i, (qi, inv, qs) in enumerate(terms):
            v += (limb_coeffs[i][j] * inv % qi) * qs
        out[j] = v % Q
    return out
