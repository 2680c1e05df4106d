// Device CRT helpers shared by the coefficient-wise kernels (kernels.hip) and the fused
// transform + lift kernel (ntt.hip): mixed-radix comparison, Garner over Q for near primes below
// 2^60, and the 30-bit-limb dot products for special primes.
#pragma once
#include "exacto_internal.hpp"

namespace exacto {

template <int MAXN>
__device__ __forceinline__ bool mr_greater(const u64 (&v)[MAXN], const u64* h, int cnt) {
    // lexicographic compare, most significant digit first
    int res = 0;  // 0 undecided, 1 greater, -1 smaller
#pragma unroll
    for (int k = MAXN - 1; k >= 0; --k) {
        if (k < cnt && res == 0) {
            if (v[k] > h[k]) res = 1;
            else if (v[k] < h[k]) res = -1;
        }
    }
    return res == 1;
}

// Garner over Q; x[i] < 2 q_i.
template <int LT>
__device__ __forceinline__ void garner_q_fast(u64 (&v)[EXACTO_MAX_L], const u64 (&x)[EXACTO_MAX_L], int L_arg,
                                              const CrtTables* __restrict__ C,
                                              const PrimeConst* __restrict__ primes) {
    const int L = LT ? LT : L_arg;
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i) {
        if (i < L) {
            const u64 qi = primes[i].q, nq = (u64)0 - qi;
            u64 t = x[i];
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_L; ++k)
                if (k < i) t = shoup_mul_nq(t + 2 * qi - v[k], C->gq_w[i][k], C->gq_ws[i][k], nq);
            v[i] = t >= qi ? t - qi : t;
        }
    }
}

// ---- 30-bit-limb dot products (SP: every prime 2^60 - d, d < 2^24) ----
// sum_k x_k c_k with x_k, c_k < 2^60, kept exactly as a0 + a1 2^30 + a2 2^60: each operand is
// split into 30-bit limbs, so every limb product is below 2^60 and one v_mad_u64_u32 adds it to
// its column without a carry (up to 7 terms plus an additive constant below 2^60 in a0).  One
// fold through 2^60 == d at the end replaces a Shoup product (about 16 VALU) per term with 4
// multiply-adds per term.  The constants are wave-uniform: their limbs are split on the SALU.
struct Dot30 {
    u64 a0, a1, a2;
};

constexpr uint32_t M30 = (1u << 30) - 1;

__device__ __forceinline__ void dot30_mac(Dot30& A, uint32_t x0, uint32_t x1, u64 c) {
    const uint32_t c0 = (uint32_t)c & M30, c1 = (uint32_t)(c >> 30);
    A.a0 += (u64)x0 * c0;
    A.a1 += (u64)x0 * c1;
    A.a1 += (u64)x1 * c0;
    A.a2 += (u64)x1 * c1;
}

// (a0 + a1 2^30 + a2 2^60) mod q, canonical.  With m <= 7 terms: a0 < (m + 1) 2^60,
// a1 < 2 m 2^60, a2 < m 2^60.  2^60 == d gives
//   X == a0 + (a1 mod 2^30) 2^30 + H d,   H = a2 + floor(a1 / 2^30) < 2^63,
//   H d = Hl d + F 2^32 (Hl = H mod 2^32, F = floor(H / 2^32) d < 2^55),
//   F 2^32 == (F mod 2^28) 2^32 + floor(F / 2^28) d,
// and the five terms sum below (m + 3.1) 2^60 < 2^64; reduce_near60 makes it canonical.
__device__ __forceinline__ u64 dot30_fold(const Dot30& A, u64 q) {
    const uint32_t d = (uint32_t)((1ull << 60) - q);
    const u64 H = A.a2 + (A.a1 >> 30);
    const u64 F = (u64)(uint32_t)(H >> 32) * d;
    u64 x = A.a0 + (u64)(uint32_t)H * d;
    x += (A.a1 & M30) << 30;
    x += (F & ((1ull << 28) - 1)) << 32;
    x += (u64)(uint32_t)(F >> 28) * d;
    return reduce_near60(x, q);
}

}  // namespace exacto
