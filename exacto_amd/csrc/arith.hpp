// Device-side modular arithmetic for 64-bit RNS primes on CDNA4 (gfx950).
//
// Replaces reference src/ring/modular.rs (exact u128 %, modular.rs:7-19, 81-84)
// with division-free forms:
//   * Shoup multiplication by a precomputed constant (NTT twiddles, CRT/Garner
//     constants): one __umul64hi + two 64-bit mul-lo, result in [0, 2q).
//   * Barrett (Menezes/HAC 14.42 with mu = floor(2^(2s)/q), s = bitlen(q)) for
//     the product of two variable residues (pointwise tensor, relin MAC).
//   * reduce64: x mod q for any 64-bit x via mu64 = floor(2^64/q).
// gfx950 has no 64x64->128 multiply; hipcc lowers these to v_mad_u64_u32 /
// v_mul_hi_u32 / v_mul_lo_u32 sequences (NTT roofline).
// Every prime handled here satisfies q < 2^62 so 4q fits in 64 bits (Harvey
// lazy butterflies keep values in [0, 4q)).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef int64_t i64;
typedef unsigned __int128 u128;
typedef __int128 i128;

#define EXACTO_MAX_L 8        // ciphertext RNS limbs
#define EXACTO_MAX_K 10       // auxiliary primes (exact path: about L + 2)
#define EXACTO_MAX_PRIMES (EXACTO_MAX_L + EXACTO_MAX_K)
#define EXACTO_MAX_G 64       // gadget digits

struct __attribute__((aligned(16))) TwPair {
    u64 w;   // twiddle
    u64 ws;  // floor(w * 2^64 / q)
};

// Per-prime constants, device-resident (one array per context).
struct PrimeConst {
    u64 q, two_q;
    u64 mu64;          // floor(2^64 / q)
    u64 bar_mu;        // floor(2^(2s) / q)
    int bar_s;         // s = bitlen(q)
    int pad_;
    u64 n_inv, n_inv_s;        // n^-1 mod q and its Shoup companion
    u64 last_w, last_ws;       // psi_inv_rev[1] * n^-1 (fused last inverse stage)
    const TwPair* tw_fwd;      // [n] psi^brv(i)
    const TwPair* tw_inv;      // [n] psi^-brv(i)
    // Montgomery products (R = 2^64) in the generic-prime tensor: -q^-1 mod 2^64, and the last
    // inverse stage's two constants times R mod q (they cancel the products' R^-1)
    u64 qinv_neg;
    u64 n_inv_r, n_inv_rs, last_wr, last_wrs;
};

// a b R^-1 mod q in [0, 2q) (R = 2^64) for a b < q 2^64 (a, b < q): Montgomery's REDC with
// m = lo(a b) (-q^-1) mod 2^64; (a b + m q) / 2^64 = hi(a b) + hi(m q) + (lo(a b) != 0), since the
// low words sum to 0 or 2^64 exactly.
__device__ __forceinline__ u64 mont_mul_lazy(u64 a, u64 b, u64 q, u64 qinv_neg) {
    const u64 lo = a * b, hi = __umul64hi(a, b);
    const u64 m = lo * qinv_neg;
    return hi + __umul64hi(m, q) + (lo != 0 ? 1 : 0);
}

// hi64(y * s) from 32-bit halves.  u = y1*s0 + hi(y0*s0) fits 64 bits; v = y0*s1 + u is
// a 65-bit sum, and y*s = lo(y0*s0) + 2^32*v + 2^64*y1*s1, so hi64 = y1*s1 + (v >> 32).
// Written this way hipcc keeps every v_mad_u64_u32 addend a natural 64-bit value
// (no zero-extension moves) and the carry in v_addc.
__device__ __forceinline__ u64 mulhi64(u64 y, u64 s) {
    const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
    const uint32_t s0 = (uint32_t)s, s1 = (uint32_t)(s >> 32);
    const u64 u = (u64)y1 * s0 + __umulhi(y0, s0);
    const u128 v = (u128)((u64)y0 * s1) + u;
    return (u64)y1 * s1 + (u64)(v >> 32);
}

// Shoup: x < 2^64, w < q, ws = floor(w * 2^64 / q), nq = 2^64 - q.  Returns x*w mod q in
// [0, 2q) as lo64(x*w + qhat*nq): -q is folded into a chained mad instead of a 64-bit sub.
__device__ __forceinline__ u64 shoup_mul_nq(u64 x, u64 w, u64 ws, u64 nq) {
    const u64 qh = mulhi64(x, ws);
    const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
    const uint32_t w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    const uint32_t h0 = (uint32_t)qh, h1 = (uint32_t)(qh >> 32);
    const uint32_t n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
    const u64 t = (u64)h0 * n0 + (u64)x0 * w0;
    const uint32_t cross = x0 * w1 + x1 * w0 + h0 * n1 + h1 * n0;
    return t + ((u64)cross << 32);
}

__device__ __forceinline__ u64 shoup_mul(u64 x, u64 w, u64 ws, u64 q) {
    return shoup_mul_nq(x, w, ws, (u64)0 - q);
}

__device__ __forceinline__ u64 shoup_mul_red(u64 x, u64 w, u64 ws, u64 q) {
    u64 r = shoup_mul(x, w, ws, q);
    return r >= q ? r - q : r;
}

__device__ __forceinline__ u64 reduce64(u64 x, u64 q, u64 mu64) {
    // any x < 2^64 -> x mod q
    u64 qh = __umul64hi(x, mu64);
    u64 r = x - qh * q;
    if (r >= q) r -= q;
    if (r >= q) r -= q;
    return r;
}

// x mod q for any x < 2^64 and q = 2^60 - d, d < 2^24: (x mod 2^60) + floor(x / 2^60) d < 2q,
// then one conditional subtraction (reduce64's quotient estimate costs a 64x64 high product).
__device__ __forceinline__ u64 reduce_near60(u64 x, u64 q) {
    const uint32_t d = (uint32_t)((1ull << 60) - q);
    const u64 r = (x & ((1ull << 60) - 1)) + (u64)(uint32_t)(x >> 60) * d;
    return r >= q ? r - q : r;
}

__device__ __forceinline__ u64 barrett128(u64 hi, u64 lo, u64 q, u64 mu, int s) {
    // x = hi:lo < 2^(2s) -> x mod q
    u64 xs = (lo >> (s - 1)) | (hi << (65 - s));
    u64 plo = xs * mu;
    u64 phi = __umul64hi(xs, mu);
    u64 qhat = (plo >> (s + 1)) | (phi << (63 - s));
    u64 r = lo - qhat * q;
    if (r >= q) r -= q;
    if (r >= q) r -= q;
    return r;
}

__device__ __forceinline__ u64 mul_mod(u64 a, u64 b, const PrimeConst& P) {
    return barrett128(__umul64hi(a, b), a * b, P.q, P.bar_mu, P.bar_s);
}

__device__ __forceinline__ u64 add_mod(u64 a, u64 b, u64 q) {
    u64 s = a + b;
    return s >= q ? s - q : s;
}

__device__ __forceinline__ u64 sub_mod(u64 a, u64 b, u64 q) {
    return a >= b ? a - b : a + q - b;
}

__device__ __forceinline__ u64 neg_mod(u64 a, u64 q) { return a == 0 ? 0 : q - a; }

// Literal restatement of reference mod_mul (modular.rs:7-19, 81-84) for the HPS
// per-coefficient formulas, where operands are not always canonical.
__device__ __forceinline__ u64 ref_mod_mul(u64 a, u64 b, u64 m) {
    u128 prod = (u128)a * b;
    if (m > (1ull << 32)) return (u64)(prod % m);
    u64 k = (u64)(((u128)1 << 64) / m);
    u64 q_hat = (u64)((prod * (u128)k) >> 64);
    u64 r = (u64)prod - q_hat * m;
    return r >= m ? r - m : r;
}

// Signed value (|v| < 2^63) mod q, Euclidean.
__device__ __forceinline__ u64 signed_mod(i64 v, u64 q, u64 mu64) {
    if (v >= 0) return reduce64((u64)v, q, mu64);
    u64 r = reduce64((u64)(-(v + 1)) + 1u, q, mu64);  // |v| mod q without overflow at INT64_MIN
    return r == 0 ? 0 : q - r;
}
