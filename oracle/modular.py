"""L0 modular arithmetic — restates reference src/ring/modular.rs (TEST ORACLE ONLY).

Python ints are unbounded, so Rust's u64/u128 wrapping is reproduced with
explicit masks where the reference relies on it.
"""

U64 = (1 << 64) - 1
U128 = (1 << 128) - 1


def barrett_constant(m: int) -> int:
    """floor(2^64 / m) — modular.rs:23-27."""
    assert m > 1, "modulus must be > 1"
    return ((1 << 64) // m) & U64


def barrett_reduce(a: int, m: int, barrett_k: int) -> int:
    """modular.rs:7-19: exact u128 % for m > 2^32, one-correction Barrett otherwise."""
    if m > (1 << 32):
        return (a % m) & U64
    q_hat = (((a & U128) * barrett_k) & U128) >> 64
    q_hat &= U64
    r = ((a & U64) - ((q_hat * m) & U64)) & U64
    return (r - m) & U64 if r >= m else r


def montgomery_reduce(t: int, m: int, m_inv_neg: int) -> int:
    """modular.rs:34-40 (exported, unused on the path; KAT only)."""
    t_lo = t & U64
    k = (t_lo * m_inv_neg) & U64
    km = k * m
    r = (((t + km) & U128) >> 64) & U64
    return (r - m) & U64 if r >= m else r


def montgomery_inv_neg(m: int) -> int:
    """modular.rs:43-53."""
    assert m & 1 == 1, "Montgomery requires odd modulus"
    inv = m
    for _ in range(6):
        inv = (inv * ((2 - m * inv) & U64)) & U64
    return (-inv) & U64


def mod_add(a: int, b: int, m: int) -> int:
    """modular.rs:57-62."""
    s = a + b
    return (s - m) & U64 if s >= m else s & U64


def mod_sub(a: int, b: int, m: int) -> int:
    """modular.rs:65-71."""
    return a - b if a >= b else m - b + a


def mod_neg(a: int, m: int) -> int:
    """modular.rs:75-77."""
    return 0 if a == 0 else m - a


def mod_mul(a: int, b: int, m: int, barrett_k: int | None = None) -> int:
    """modular.rs:81-84."""
    if barrett_k is None:
        barrett_k = barrett_constant(m)
    return barrett_reduce(a * b, m, barrett_k)


def mod_pow(base: int, exp: int, m: int) -> int:
    """modular.rs:87-99."""
    bk = barrett_constant(m)
    result = 1
    base %= m
    while exp > 0:
        if exp & 1:
            result = mod_mul(result, base, m, bk)
        exp >>= 1
        base = mod_mul(base, base, m, bk)
    return result


def mod_inv(a: int, m: int) -> int | None:
    """modular.rs:102-121 (extended Euclid; None if not coprime)."""
    old_r, r = a, m
    old_s, s = 1, 0
    while r != 0:
        q = int(old_r / r) if (old_r < 0) != (r < 0) else old_r // r  # Rust truncating /
        old_r, r = r, old_r - q * r
        old_s, s = s, old_s - q * s
    if old_r != 1:
        return None
    return ((rust_rem(old_s, m)) + m) % m


def rust_rem(a: int, b: int) -> int:
    """Rust's truncating integer remainder (sign follows the dividend)."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def rust_div(a: int, b: int) -> int:
    """Rust's truncating integer division."""
    q = abs(a) // abs(b)
    return -q if (a < 0) != (b < 0) else q


# --- primality (host-side parameter validation; concrete-ntt's Plan::try_new checks primality) ---

def is_prime(n: int) -> bool:
    if n < 2:
        return False
    small = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)
    for p in small:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in small:  # deterministic for n < 3.3e24
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True
