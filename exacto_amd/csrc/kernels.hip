// Coefficient-wise kernels of the BFV multiplication path (gfx950).
//
//   exact_lift   : centred exact Q -> P base extension        (eval.rs:719-762 reconstruct_centered_bigint)
//   hps_extend   : literal single-q centred extension         (eval.rs:217-247 base_extend_centered)
//   tensor       : (c0d0, c0d1 + c1d0, c1d1) in every prime   (eval.rs:131-133, 186-198)
//   exact_scale  : r = round(p*T/Q) exactly, r mod q_i        (eval.rs:816-831, 764-792)
//   hps_scale    : literal HPS m-recovery, 1 or 2 aux primes  (eval.rs:257-413)
//   gadget digits: balanced base-B digits of [c2]_Q           (keyswitch.rs:11-52, rns.rs:114-151)
//   relin_mac    : c_k + sum_g d_g (.) rlk_k,g                (keyswitch.rs:86-95)
//   dbfv_combine : per-k limb sums + degree reduction         (dbfv/eval.rs:124-132, reduction.rs:34-52)
//
// Every kernel is a flat 1-D grid of 256-thread blocks, one coefficient per
// thread; the "row" (item x polynomial) is blockIdx.x / blocks_per_row so
// consecutive lanes touch consecutive 8-byte words of one residue polynomial.
#include "exacto_internal.hpp"
#include "crt_dev.hpp"

#include <cstdlib>

namespace exacto {

static constexpr int TPB = 256;

static inline int blocks_per_row(int n) { return (n + TPB - 1) / TPB; }

// n is a power of two: blocks per row too (1 below TPB), so row and column are a shift and a
// mask of the block index (SALU), not a division
#define ROW_SETUP(n)                                                   \
    const int nblk = (n + TPB - 1) / TPB;                              \
    const int nsh = __builtin_ctz((unsigned)nblk);                     \
    const long row = (long)(blockIdx.x >> nsh);                        \
    const int j = (int)(blockIdx.x & (unsigned)(nblk - 1)) * TPB + threadIdx.x; \
    if (j >= (n)) return;

// ---------------------------------------------------------------- mixed radix helpers

// A residue of one prime moved to another: with NEAR (max prime < 2 * min prime) a value
// below any prime needs one conditional subtraction, otherwise a full reduce64.
template <bool NEAR>
__device__ __forceinline__ u64 xfer(u64 v, u64 q, u64 mu) {
    if (NEAR) return v >= q ? v - q : v;
    return reduce64(v, q, mu);
}

// Garner: residues x[i] mod q_i (i < L) -> mixed-radix digits v (x = v0 + v1 q0 + v2 q0 q1 + ...).
template <bool NEAR>
__device__ __forceinline__ void garner_q(u64 (&v)[EXACTO_MAX_L], const u64 (&x)[EXACTO_MAX_L], int L,
                                         const CrtTables* __restrict__ C,
                                         const PrimeConst* __restrict__ primes) {
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i) {
        if (i < L) {
            const u64 qi = primes[i].q, mui = primes[i].mu64;
            u64 t = x[i];
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_L; ++k) {
                if (k < i) {
                    t = sub_mod(t, xfer<NEAR>(v[k], qi, mui), qi);
                    t = shoup_mul_red(t, C->gq_w[i][k], C->gq_ws[i][k], qi);
                }
            }
            v[i] = t;
        }
    }
}


// sum_k (v_k mod prime_t) * pref[k][t]  -  neg * pref[cnt][t]   (mod prime_t)
template <int MAXN, int STRIDE, bool NEAR>
__device__ __forceinline__ u64 mr_eval(const u64 (&v)[MAXN], int cnt, bool neg, const u64* pw,
                                       const u64* pws, int t, const PrimeConst& P) {
    const u64 q = P.q, mu = P.mu64;
    u64 acc = 0;
#pragma unroll
    for (int k = 0; k < MAXN; ++k) {
        if (k < cnt) {
            const u64 vk = xfer<NEAR>(v[k], q, mu);
            acc = add_mod(acc, shoup_mul_red(vk, pw[k * STRIDE + t], pws[k * STRIDE + t], q), q);
        }
    }
    if (neg) acc = sub_mod(acc, pw[cnt * STRIDE + t], q);
    return acc;
}

// ---- lazy CRT helpers (FAST: primes near each other and all < 2^60) ----
// A Shoup product accepts any 64-bit input and returns [0, 2q), so differences are formed as
// t + 2q - v (v < 2q by nearness) and fed to it unreduced; sums of Shoup outputs are reduced
// once with reduce64.  Only the mixed-radix digits themselves are made canonical.


// sum_k v_k * pref[k][t] - neg * pref[cnt][t]  (mod prime_t), canonical; 14q < 2^64 bounds
// the unreduced run to 7 terms.
// SP: every prime is 2^60 - d, d < 2^24 (reduce_near60).
template <bool SP>
__device__ __forceinline__ u64 reduce_any(u64 x, const PrimeConst& P) {
    return SP ? reduce_near60(x, P.q) : reduce64(x, P.q, P.mu64);
}

template <int MAXN, int STRIDE, bool SP = false>
__device__ __forceinline__ u64 mr_eval_fast(const u64 (&v)[MAXN], int cnt, bool neg, const u64* pw,
                                            const u64* pws, int t, const PrimeConst& P) {
    const u64 q = P.q, nq = (u64)0 - q;
    u64 acc = 0;
#pragma unroll
    for (int k = 0; k < MAXN; ++k) {
        if (k < cnt) {
            acc += shoup_mul_nq(v[k], pw[k * STRIDE + t], pws[k * STRIDE + t], nq);
            if (k % 7 == 6) acc = reduce_any<SP>(acc, P);
        }
    }
    acc = reduce_any<SP>(acc, P);
    if (neg) acc = sub_mod(acc, pw[cnt * STRIDE + t], q);
    return acc;
}


// Balanced gadget digits of the centred CRT value of residues res[0..L) (mod Q).
// keyswitch.rs:24-44 literally (truncating %, [-B/2, B/2) adjustment, final carry dropped),
// on the exact value (extension semantics for Q >= 2^64; identical to rns.rs:114-151 below).
// Writes digit g, limb i at D[g * L * n + i * n] (D already offset by the coefficient j), or, with
// D16 (gadget base <= 2^16: every balanced digit lies in [-2^15, 2^15)), the signed digit once
// at D16[g * n] for all limbs: 2 bytes per digit instead of 8 L.
template <bool NEAR, int LT = 0, typename DT = int16_t>
__device__ __forceinline__ void gadget_digits(const u64 (&res)[EXACTO_MAX_L], int L_arg,
                                              const CrtTables* __restrict__ C,
                                              const PrimeConst* __restrict__ primes, u64* D, int n, int guse,
                                              DT* D16 = nullptr) {
    const int L = LT ? LT : L_arg;  // LT > 0: limb count known at compile time
    u64 z[EXACTO_MAX_L];
    garner_q<NEAR>(z, res, L, C, primes);
    const bool neg = mr_greater<EXACTO_MAX_L>(z, C->halfQ_mr, L);
    // multiword value via Horner on the mixed-radix digits
    u64 M[EXACTO_MAX_L];
#pragma unroll
    for (int w = 0; w < EXACTO_MAX_L; ++w) M[w] = 0;
#pragma unroll
    for (int k = 0; k < EXACTO_MAX_L; ++k)
        if (k == L - 1) M[0] = z[k];
#pragma unroll
    for (int k = EXACTO_MAX_L - 2; k >= 0; --k) {
        if (k <= L - 2) {
            const u64 qk = primes[k].q;
            u64 carry = z[k];
#pragma unroll
            for (int w = 0; w < EXACTO_MAX_L; ++w) {
                if (w < L) {
                    const u128 t = (u128)M[w] * qk + carry;
                    M[w] = (u64)t;
                    carry = (u64)(t >> 64);
                }
            }
        }
    }
    if (neg) {  // magnitude Q - x
        u64 borrow = 0;
#pragma unroll
        for (int w = 0; w < EXACTO_MAX_L; ++w) {
            if (w < L) {
                const u64 a = C->Qwords[w], b = M[w];
                const u64 d1 = a - b;
                const u64 b1 = a < b;
                const u64 d2 = d1 - borrow;
                const u64 b2 = d1 < borrow;
                M[w] = d2;
                borrow = b1 | b2;
            }
        }
    }
    const u64 B = C->gbase;
    const u64 half = B >> 1;
    const int sh = C->gshift;
    for (int g = 0; g < guse; ++g) {
        u64 r;
        if (sh >= 0) {
            r = M[0] & (B - 1);
#pragma unroll
            for (int w = 0; w < EXACTO_MAX_L; ++w) {
                if (w < L) {
                    const u64 hi = (w + 1 < L) ? M[w + 1] : 0;
                    M[w] = (M[w] >> sh) | (sh ? (hi << (64 - sh)) : 0);
                }
            }
        } else {
            u64 rem = 0;
#pragma unroll
            for (int w = EXACTO_MAX_L - 1; w >= 0; --w) {
                if (w < L) {
                    const u128 cur = ((u128)rem << 64) | M[w];
                    M[w] = (u64)(cur / B);
                    rem = (u64)(cur % B);
                }
            }
            r = rem;
        }
        // signed remainder: value = +/- M_old; Rust truncating % then balance
        u64 mag;
        bool dneg;
        bool carry;
        if (!neg) {
            if (r >= half) { mag = B - r; dneg = true; carry = true; }
            else { mag = r; dneg = false; carry = false; }
        } else {
            if (r > half) { mag = B - r; dneg = false; carry = true; }
            else { mag = r; dneg = (r != 0); carry = false; }
        }
        if (carry) {
            u64 c = 1;
#pragma unroll
            for (int w = 0; w < EXACTO_MAX_L; ++w) {
                if (w < L) {
                    const u64 s = M[w] + c;
                    c = (s < c);
                    M[w] = s;
                }
            }
        }
        if (D16) {   // int16 (base <= 2^16) or int8 (base <= 2^8) signed digit
            D16[(long)g * n] = (DT)(dneg ? -(i64)mag : (i64)mag);
            continue;
        }
        // digit residue (rem mod Q) mod q_i == rem mod q_i; |rem| < B <= q_i when digit_small
        const bool small = C->digit_small != 0;
#pragma unroll
        for (int i = 0; i < EXACTO_MAX_L; ++i) {
            if (i < L) {
                const u64 qi = primes[i].q;
                u64 m = small ? mag : reduce64(mag, qi, primes[i].mu64);
                if (dneg && m != 0) m = qi - m;
                D[((long)g * L + i) * n] = m;
            }
        }
    }
}

// int16 gadget digits (base 2^sh, sh | 32) of the centred CRT value of canonical residues res,
// the same digits as gadget_digits (keyswitch.rs:24-44: truncating %, [-B/2, B/2) adjustment,
// final carry dropped).  gadget_digits adds each balancing carry back into the multiword
// magnitude; here it is a 1-bit carry c added to the next raw field instead: r = field + c lies in
// [0, B], and r == B (the carry rippling through a field of ones) gives digit 0 with carry 1 under
// the same rule, exactly as the multiword increment does.  The fields are read from the 32-bit
// words of the magnitude in place: no multiword shift or add per digit.  Digit g goes to
// D16[g * n].
template <int LT, typename DT = int16_t>
__device__ __forceinline__ void gadget_digits16_sp(const u64 (&res)[EXACTO_MAX_L], const CrtTables* __restrict__ C,
                                                   const PrimeConst* __restrict__ primes, int n, int guse,
                                                   DT* D16) {
    constexpr int L = LT;
    u64 z[EXACTO_MAX_L];
    garner_q_fast<LT>(z, res, L, C, primes);
    const bool neg = mr_greater<EXACTO_MAX_L>(z, C->halfQ_mr, L);
    u64 M[L];
    M[0] = z[L - 1];
#pragma unroll
    for (int w = 1; w < L; ++w) M[w] = 0;
#pragma unroll
    for (int k = L - 2; k >= 0; --k) {
        const u64 qk = primes[k].q;
        u64 carry = z[k];
#pragma unroll
        for (int w = 0; w < L; ++w) {
            const u128 t = (u128)M[w] * qk + carry;
            M[w] = (u64)t;
            carry = (u64)(t >> 64);
        }
    }
    if (neg) {  // magnitude Q - x
        u64 borrow = 0;
#pragma unroll
        for (int w = 0; w < L; ++w) {
            const u64 a = C->Qwords[w], b = M[w];
            const u64 d1 = a - b;
            const u64 b1 = a < b;
            const u64 d2 = d1 - borrow;
            const u64 b2 = d1 < borrow;
            M[w] = d2;
            borrow = b1 | b2;
        }
    }
    const int sh = C->gshift;
    const uint32_t B = 1u << sh, mask = B - 1;
    // !neg: r >= B/2 balances down; neg: r > B/2 does (the digit then takes the other sign)
    const uint32_t thr = (B >> 1) - (neg ? 0u : 1u);
    const int sgn = neg ? -1 : 0;
    uint32_t c = 0;
    int g = 0;
#pragma unroll
    for (int w = 0; w < 2 * L; ++w) {
        const uint32_t word = (w & 1) ? (uint32_t)(M[w >> 1] >> 32) : (uint32_t)M[w >> 1];
        for (int o = 0; o < 32 && g < guse; o += sh, ++g) {
            const uint32_t r = ((word >> o) & mask) + c;
            c = r > thr ? 1u : 0u;
            const int dv = (int)r - (int)(c << sh);
            D16[(long)g * n] = (DT)((dv ^ sgn) - sgn);
        }
    }
    for (; g < guse; ++g) {   // past the magnitude's words: only the carry remains
        const uint32_t r = c;
        c = r > thr ? 1u : 0u;
        const int dv = (int)r - (int)(c << sh);
        D16[(long)g * n] = (DT)((dv ^ sgn) - sgn);
    }
}

// ---------------------------------------------------------------- exact lift Q -> P

template <bool NEAR, bool FAST, int LT, int KT, bool SP = false>
__global__ void __launch_bounds__(TPB)
exact_lift_kernel(const u64* __restrict__ coefQ, u64* __restrict__ extP, int n, int L_arg, int K_arg,
                  const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const int L = LT ? LT : L_arg;  // LT/KT > 0: limb counts known at compile time
    const int K = KT ? KT : K_arg;
    u64 x[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i)
        if (i < L) x[i] = coefQ[(row * L + i) * n + j];
    if (FAST) garner_q_fast<LT>(v, x, L, C, primes);
    else garner_q<NEAR>(v, x, L, C, primes);
    const bool neg = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
    for (int a = 0; a < K; ++a) {
        const int t = L + a;
        extP[(row * K + a) * n + j] =
            FAST ? mr_eval_fast<EXACTO_MAX_L, EXACTO_MAX_PRIMES, SP>(v, L, neg, &C->qpref_w[0][0],
                                                                   &C->qpref_ws[0][0], t, primes[t])
                 : mr_eval<EXACTO_MAX_L, EXACTO_MAX_PRIMES, NEAR>(v, L, neg, &C->qpref_w[0][0],
                                                                 &C->qpref_ws[0][0], t, primes[t]);
    }
}

// SP, K = L + 1: extP_a = sum_k v_k (q_0 .. q_{k-1}) - neg Q  mod p_a as one 30-bit-limb dot
// product per auxiliary prime (the constant -Q folded into the accumulator).
template <int LT>
__global__ void __launch_bounds__(TPB)
exact_lift_sp_kernel(const u64* __restrict__ coefQ, u64* __restrict__ extP, int n,
                     const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    constexpr int L = LT, K = LT + 1;
    u64 x[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < L; ++i) x[i] = coefQ[(row * L + i) * n + j];
    garner_q_fast<LT>(v, x, L, C, primes);
    const bool neg = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
    uint32_t v0[L], v1[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        v0[k] = (uint32_t)v[k] & M30;
        v1[k] = (uint32_t)(v[k] >> 30);
    }
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const int t = L + a;
        const u64 pa = primes[t].q;
        Dot30 A{neg ? pa - C->qpref_w[L][t] : 0, 0, 0};
#pragma unroll
        for (int k = 0; k < L; ++k) dot30_mac(A, v0[k], v1[k], C->qpref_w[k][t]);
        extP[(row * K + a) * n + j] = dot30_fold(A, pa);
    }
}

// EXACTO_DOT30=0 keeps the Shoup-per-term SP kernels (A/B switch)
static bool use_dot30() {
    static const bool on = [] {
        const char* e = std::getenv("EXACTO_DOT30");
        return !(e && e[0] == '0');
    }();
    return on;
}

void launch_exact_lift(const u64* coefQ, u64* extP, long rows, int n, const CrtTables* ct,
                       const PrimeConst* primes, int L, int K, int mode, hipStream_t s) {
    const long blocks = rows * blocks_per_row(n);
    if (blocks == 0) return;
    if (mode == 3 && K == L + 1 && L >= 1 && L <= 6 && use_dot30()) {
#define LIFT30(LT) EXACTO_LAUNCH((exact_lift_sp_kernel<LT>), dim3(blocks), dim3(TPB), 0, s, coefQ, extP, n, ct, primes)
        switch (L) {
            case 1: LIFT30(1); break;
            case 2: LIFT30(2); break;
            case 3: LIFT30(3); break;
            case 4: LIFT30(4); break;
            case 5: LIFT30(5); break;
            default: LIFT30(6); break;
        }
#undef LIFT30
        return;
    }
#define LIFT(NR, FS, LT, KT)                                                                                     \
    EXACTO_LAUNCH((exact_lift_kernel<NR, FS, LT, KT>), dim3(blocks), dim3(TPB), 0, s, coefQ, extP, n, L, K, ct, \
                       primes)
#define LIFT_SP(LT)                                                                                              \
    EXACTO_LAUNCH((exact_lift_kernel<true, true, LT, LT + 1, true>), dim3(blocks), dim3(TPB), 0, s, coefQ,  \
                       extP, n, L, K, ct, primes)
    if (mode == 3 && K == L + 1 && L >= 1 && L <= 6) {
        switch (L) {
            case 1: LIFT_SP(1); break;
            case 2: LIFT_SP(2); break;
            case 3: LIFT_SP(3); break;
            case 4: LIFT_SP(4); break;
            case 5: LIFT_SP(5); break;
            default: LIFT_SP(6); break;
        }
    } else if (mode >= 2) {
        switch (L) {
            case 1: if (K == 2) LIFT(true, true, 1, 2); else LIFT(true, true, 1, 0); break;
            case 2: if (K == 3) LIFT(true, true, 2, 3); else LIFT(true, true, 2, 0); break;
            case 3: if (K == 4) LIFT(true, true, 3, 4); else LIFT(true, true, 3, 0); break;
            case 4: if (K == 5) LIFT(true, true, 4, 5); else LIFT(true, true, 4, 0); break;
            case 5: if (K == 6) LIFT(true, true, 5, 6); else LIFT(true, true, 5, 0); break;
            case 6: if (K == 7) LIFT(true, true, 6, 7); else LIFT(true, true, 6, 0); break;
            default: LIFT(true, true, 0, 0); break;
        }
    } else if (mode == 1) {
        LIFT(true, false, 0, 0);
    } else {
        LIFT(false, false, 0, 0);
    }
#undef LIFT
#undef LIFT_SP
}

// ---------------------------------------------------------------- HPS extension

__global__ void __launch_bounds__(TPB)
hps_extend_kernel(const u64* __restrict__ coefQ, u64* __restrict__ extP, int n, int K,
                  const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const u64 q = primes[0].q;
    const u64 c = coefQ[row * n + j];
    // centred once, branch-free: |c_c| mod p_a, negated for negative c_c; no reduction at all where
    // q <= p_a (block-uniform: compact_bfv's 40-bit q under its 49-bit p)
    const bool neg = c > q / 2;
    const u64 mag = neg ? q - c : c;
    for (int a = 0; a < K; ++a) {
        const PrimeConst& P = primes[1 + a];
        const u64 rem = q <= P.q ? mag : reduce64(mag, P.q, P.mu64);
        extP[(row * K + a) * n + j] = (neg && rem) ? P.q - rem : rem;
    }
}

void launch_hps_extend(const u64* coefQ, u64* extP, long rows, int n, const PrimeConst* primes,
                       int K, hipStream_t s) {
    const long blocks = rows * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(hps_extend_kernel, dim3(blocks), dim3(TPB), 0, s, coefQ, extP, n, K, primes);
}

// ---------------------------------------------------------------- exact scale-and-round

template <bool NEAR, bool FAST, int LT, int KT, bool SP = false>
__global__ void __launch_bounds__(TPB)
exact_scale_kernel(const u64* __restrict__ T, u64* __restrict__ R, long r_stride, int ncomp_r,
                   u64* __restrict__ D, int16_t* __restrict__ D16, int guse, int n, int L_arg, int K_arg,
                   const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const int L = LT ? LT : L_arg;  // LT/KT > 0: limb counts known at compile time
    const int K = KT ? KT : K_arg;
    const int NP = L + K;
    const long item = row / 3;
    const int comp = (int)(row - item * 3);
    const u64* Tin = T + row * NP * n + j;
    // u = p * T mod q_i; s = [u]_Q centred, as mixed-radix digits v + sign
    u64 u[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i)
        if (i < L)
            u[i] = FAST ? shoup_mul(Tin[(long)i * n], C->pmod_w[i], C->pmod_ws[i], primes[i].q)
                        : shoup_mul_red(Tin[(long)i * n], C->pmod_w[i], C->pmod_ws[i], primes[i].q);
    if (FAST) garner_q_fast<LT>(v, u, L, C, primes);
    else garner_q<NEAR>(v, u, L, C, primes);
    const bool negs = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
    // r = (p*T - s) / Q in every auxiliary prime, with Q^-1 folded into the constants:
    // r = T*(p Q^-1) - sum_k v_k*(qpref_k Q^-1) + negs   (Q * Q^-1 == 1)
    u64 w[EXACTO_MAX_K];
#pragma unroll
    for (int a = 0; a < EXACTO_MAX_K; ++a) {
        if (a < K && FAST) {
            const PrimeConst& P = primes[L + a];
            const u64 pa = P.q, np = (u64)0 - pa;
            // terms in (0, 2p]: 2p - x*c instead of a modular subtraction; <= 7 before a reduce
            u64 acc = shoup_mul_nq(Tin[(long)(L + a) * n], C->pq_w[a], C->pq_ws[a], np) + (negs ? 1 : 0);
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_L; ++k) {
                if (k < L) {
                    acc += 2 * pa - shoup_mul_nq(v[k], C->qpq_w[k][a], C->qpq_ws[k][a], np);
                    if (k % 6 == 5) acc = reduce_any<SP>(acc, P);
                }
            }
            acc = reduce_any<SP>(acc, P);
            // Garner over P on the fly; w_k < p_k < 2 p_a
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_K; ++k)
                if (k < a) acc = shoup_mul_nq(acc + 2 * pa - w[k], C->gp_w[a][k], C->gp_ws[a][k], np);
            w[a] = acc >= pa ? acc - pa : acc;
        } else if (a < K) {
            const PrimeConst& P = primes[L + a];
            const u64 pa = P.q;
            u64 acc = shoup_mul_red(Tin[(long)(L + a) * n], C->pq_w[a], C->pq_ws[a], pa);
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_L; ++k)
                if (k < L)
                    acc = sub_mod(acc, shoup_mul_red(xfer<NEAR>(v[k], pa, P.mu64), C->qpq_w[k][a], C->qpq_ws[k][a], pa), pa);
            if (negs) acc = add_mod(acc, 1, pa);
            // Garner over P on the fly (w_a depends on w_0..w_{a-1})
#pragma unroll
            for (int k = 0; k < EXACTO_MAX_K; ++k) {
                if (k < a) {
                    acc = sub_mod(acc, xfer<NEAR>(w[k], pa, P.mu64), pa);
                    acc = shoup_mul_red(acc, C->gp_w[a][k], C->gp_ws[a][k], pa);
                }
            }
            w[a] = acc;
        }
    }
    const bool negr = mr_greater<EXACTO_MAX_K>(w, C->halfP_mr, K);
    u64 res[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i)
        if (i < L)
            res[i] = FAST ? mr_eval_fast<EXACTO_MAX_K, EXACTO_MAX_L, SP>(w, K, negr, &C->ppref_w[0][0],
                                                                          &C->ppref_ws[0][0], i, primes[i])
                          : mr_eval<EXACTO_MAX_K, EXACTO_MAX_L, NEAR>(w, K, negr, &C->ppref_w[0][0],
                                                                      &C->ppref_ws[0][0], i, primes[i]);
    if (comp < ncomp_r) {
        u64* out = R + item * r_stride + (long)comp * L * n + j;
#pragma unroll
        for (int i = 0; i < EXACTO_MAX_L; ++i)
            if (i < L) out[(long)i * n] = res[i];
    }
    if (comp == 2 && D16 != nullptr)
        gadget_digits<NEAR, LT>(res, L, C, primes, nullptr, n, guse, D16 + item * (long)guse * n + j);
    else if (comp == 2 && D != nullptr)
        gadget_digits<NEAR, LT>(res, L, C, primes, D + item * (long)guse * L * n + j, n, guse);
}

// FPC: the centred lift of r from P by a rounded float sum instead of Garner over P.  y_a = r Pi_a mod
// p_a (Pi_a = (P / p_a)^-1 mod p_a, folded into the dot products' constants, so y_a costs what r_a
// did), X = sum_a y_a (P / p_a) == r (mod P) with X / P = sum_a y_a / p_a, and the centred r is
// X - round(X / P) P.  Exact whenever |r| < P / 4: X / P is then within 1/4 of an integer, and the
// fp64 sum of K <= 7 terms y_a * fl(1 / p_a) (each < 1, y_a rounded to 53 bits) is off by < 2^-48.
// The scale's |r| <= p n Q / 2 + 1 < P / 8 (P > 4 p n Q); a psum of m terms needs m (2 p n Q + 4) <= P
// (context psum_fp_max).  res_i = sum_a y_a ((P / p_a) mod q_i) + alpha (q_i - P mod q_i), alpha <= K.
// Replaces K (K - 1) / 2 Shoup products, the digits' comparison with floor(P/2) and their splits.
template <int LT>
__device__ __forceinline__ void fpc_lift(const u64 (&y)[LT + 1], u64 (&res)[EXACTO_MAX_L], const CrtTables* __restrict__ C,
                                         const PrimeConst* __restrict__ primes) {
    constexpr int L = LT, K = LT + 1;
    double f = 0.0;
    uint32_t y0[K], y1[K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        f = fma((double)y[a], C->fpc_inv[a], f);
        y0[a] = (uint32_t)y[a] & M30;
        y1[a] = (uint32_t)(y[a] >> 30);
    }
    const uint32_t alpha = (uint32_t)__double2int_rn(f);   // 0 .. K
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const u64 q = primes[i].q;
        Dot30 A{0, 0, 0};
        dot30_mac(A, alpha, 0, C->fpc_negP[i]);
#pragma unroll
        for (int a = 0; a < K; ++a) dot30_mac(A, y0[a], y1[a], C->fpc_pm[a][i]);
        res[i] = dot30_fold(A, q);
    }
}

// FPC's y_a from the ciphertext-prime residues T_i (i < L) and T_a: s = [p T]_Q centred by Garner over Q
// (mixed-radix digits v, their comparison with floor(Q/2)), then
//   y_a = T_a fpc_pq[a] + sum_k v_k fpc_qpq[k][a] + negs Pi_a   (mod p_a, in [0, p_a)).
// `carry` (psum: the products' running sum, < p_a) is added to each y_a; T_a's term only when ta is set.
template <int LT, bool TA>
__device__ __forceinline__ void fpc_y_garner(const u64* __restrict__ Tin, int n, u64 (&y)[LT + 1],
                                             const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    constexpr int L = LT, K = LT + 1;
    u64 u[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < L; ++i) u[i] = shoup_mul(Tin[(long)i * n], C->pmod_w[i], C->pmod_ws[i], primes[i].q);
    garner_q_fast<LT>(v, u, L, C, primes);
    const bool negs = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
    uint32_t v0[L], v1[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        v0[k] = (uint32_t)v[k] & M30;
        v1[k] = (uint32_t)(v[k] >> 30);
    }
#pragma unroll
    for (int a = 0; a < K; ++a) {
        // y[a] (TA: unused on entry; else the carry < p_a): a0's constant < 2^61, inside dot30_fold's budget
        Dot30 A{(TA ? 0ull : y[a]) + (negs ? C->fpc_neg[a] : 0ull), 0, 0};
        if constexpr (TA) {
            const u64 ta = Tin[(long)(L + a) * n];   // [0, 2q) (the tensor's lazy last stage)
            dot30_mac(A, (uint32_t)ta & M30, (uint32_t)(ta >> 30), C->fpc_pq[a]);
        }
#pragma unroll
        for (int k = 0; k < L; ++k) dot30_mac(A, v0[k], v1[k], C->fpc_qpq[k][a]);
        y[a] = dot30_fold(A, primes[L + a].q);
    }
}

// FPQ: the same y_a with s centred by a rounded float sum.  z_i = T_i p (Q / q_i)^-1 mod q_i (one Shoup
// product, as u_i was), f = sum_i z_i fl(1 / q_i) (z_i in 30-bit halves: exact doubles), beta = round(f):
// sum_i z_i (Q / q_i) = s + beta Q with s the centred residue, |s| / Q = |f - beta| up to the float
// error (< 2^-47 for L <= 6).  So beta is exact wherever |f - beta| <= 1/2 - 2^-40 (`lim`), and then
//   y_a = T_a fpc_pq[a] + sum_i z_i fpq_c[i][a] + beta Pi_a,   fpq_c[i][a] = (-q_i^-1 mod p_a) Pi_a
// (s Q^-1 = sum_i z_i q_i^-1 - beta).  Elsewhere (s within 2^-40 Q of +-Q/2; about 2^-39 of uniform
// coefficients) the lane takes fpc_y_garner.  Replaces Garner over Q's L (L - 1) / 2 Shoup products and
// the mixed-radix comparison with 2 L conversions and fused multiply-adds.
template <int LT, bool TA>
__device__ __forceinline__ void fpq_y(const u64* __restrict__ Tin, int n, u64 (&y)[LT + 1], const CrtTables* __restrict__ C,
                                      const PrimeConst* __restrict__ primes, double lim) {
    constexpr int L = LT, K = LT + 1;
    uint32_t z0[L], z1[L];
    double f = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const u64 z = shoup_mul_red(Tin[(long)i * n], C->fpq_pz_w[i], C->fpq_pz_ws[i], primes[i].q);
        z0[i] = (uint32_t)z & M30;
        z1[i] = (uint32_t)(z >> 30);
        f = fma((double)z0[i], C->fpq_inv0[i], f);
        f = fma((double)z1[i], C->fpq_inv1[i], f);
    }
    const double b = __builtin_rint(f);
    if (__builtin_fabs(f - b) <= lim) {
        const uint32_t beta = (uint32_t)b;   // 0 .. L
#pragma unroll
        for (int a = 0; a < K; ++a) {
            Dot30 A{TA ? 0ull : y[a], 0, 0};
            dot30_mac(A, beta, 0, C->fpc_neg[a]);     // < 2^33 in a0 and a1: not a full term
            if constexpr (TA) {
                const u64 ta = Tin[(long)(L + a) * n];
                dot30_mac(A, (uint32_t)ta & M30, (uint32_t)(ta >> 30), C->fpc_pq[a]);
            }
#pragma unroll
            for (int i = 0; i < L; ++i) dot30_mac(A, z0[i], z1[i], C->fpq_c[i][a]);
            y[a] = dot30_fold(A, primes[L + a].q);
        }
    } else {
        fpc_y_garner<LT, TA>(Tin, n, y, C, primes);
    }
}

// psum (FPQ): one product's z_i (< q_i) added to the row's integer sums Z_i and its beta to bs; the dot over
// the z_i is linear, so fpq_flush runs it once for every product summed.  A lane in the band adds its
// product by Garner to carry instead.
template <int LT>
__device__ __forceinline__ void fpq_acc(const u64* __restrict__ Tin, int n, u64 (&Z)[LT], uint32_t& bs, u64 (&carry)[LT + 1],
                                        const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes,
                                        double lim) {
    constexpr int L = LT;
    u64 z[L];
    double f = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        z[i] = shoup_mul_red(Tin[(long)i * n], C->fpq_pz_w[i], C->fpq_pz_ws[i], primes[i].q);
        f = fma((double)((uint32_t)z[i] & M30), C->fpq_inv0[i], f);
        f = fma((double)(uint32_t)(z[i] >> 30), C->fpq_inv1[i], f);
    }
    const double b = __builtin_rint(f);
    if (__builtin_fabs(f - b) <= lim) {
#pragma unroll
        for (int i = 0; i < L; ++i) Z[i] += z[i];
        bs += (uint32_t)b;
    } else {
        fpc_y_garner<LT, false>(Tin, n, carry, C, primes);
    }
}

// carry[a] += sum_i Z_i fpq_c[i][a] + bs Pi_a (mod p_a), then Z = 0, bs = 0.  Z_i (at most 15 products:
// < 15 q_i < 2^64) = r_i + k_i q_i with r_i < q_i, and q_i fpq_c[i][a] == -Pi_a, so the dot takes the
// r_i and the k_i join beta with the opposite sign.
template <int LT>
__device__ __forceinline__ void fpq_flush(u64 (&Z)[LT], uint32_t& bs, u64 (&carry)[LT + 1], const CrtTables* __restrict__ C,
                                          const PrimeConst* __restrict__ primes) {
    constexpr int L = LT, K = LT + 1;
    constexpr u64 M60 = (1ull << 60) - 1;
    uint32_t z0[L], z1[L], ks = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const u64 q = primes[i].q;
        uint32_t kq = (uint32_t)(Z[i] >> 60);
        u64 r = (Z[i] & M60) + (u64)kq * (uint32_t)((1ull << 60) - q);   // Z - kq q < 2^60 + 2^28 < 2q
        if (r >= q) {
            r -= q;
            ++kq;
        }
        ks += kq;
        z0[i] = (uint32_t)r & M30;
        z1[i] = (uint32_t)(r >> 30);
        Z[i] = 0;
    }
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const u64 pa = primes[L + a].q;
        Dot30 A{carry[a], 0, 0};
        dot30_mac(A, bs, 0, C->fpc_neg[a]);          // bs, ks < 2^7: not full terms
        dot30_mac(A, ks, 0, pa - C->fpc_neg[a]);
#pragma unroll
        for (int i = 0; i < L; ++i) dot30_mac(A, z0[i], z1[i], C->fpq_c[i][a]);
        carry[a] = dot30_fold(A, pa);
    }
    bs = 0;
}

// SP, K = L + 1: exact_scale_kernel with every modular dot product as a 30-bit-limb dot:
//   r_a = T_a (p Q^-1) + sum_k v_k (p_a - qpq_k,a) + negs        mod p_a   (then Garner over P)
//   res_i = sum_a w_a (p_0 .. p_{a-1}) + negr (q_i - P mod q_i)    mod q_i
// (FPC: y_a = r_a Pi_a by the same dots with folded constants, then fpc_lift), and int16 gadget
// digits by gadget_digits16_sp.
template <int LT, int DIG, bool FPC, bool FPQ = false>
__global__ void __launch_bounds__(TPB)
exact_scale_sp_kernel(const u64* __restrict__ T, u64* __restrict__ R, long r_stride, int ncomp_r,
                      u64* __restrict__ D, int16_t* __restrict__ D16, int guse, int n,
                      const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes, int c2only,
                      double fpq_lim = 0.0) {
    ROW_SETUP(n)
    constexpr int L = LT, K = LT + 1, NP = L + K;
    const long item = c2only ? row : row / 3;
    const int comp = c2only ? 2 : (int)(row - item * 3);
    const u64* Tin = T + (item * 3 + comp) * NP * n + j;
    u64 res[EXACTO_MAX_L];
    if constexpr (FPQ) {
        static_assert(FPC, "FPQ feeds the float lift from P");
        u64 y[K];
        fpq_y<LT, true>(Tin, n, y, C, primes, fpq_lim);
        fpc_lift<LT>(y, res, C, primes);
    } else {
    u64 u[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < L; ++i) u[i] = shoup_mul(Tin[(long)i * n], C->pmod_w[i], C->pmod_ws[i], primes[i].q);
    garner_q_fast<LT>(v, u, L, C, primes);
    const bool negs = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
    uint32_t v0[L], v1[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        v0[k] = (uint32_t)v[k] & M30;
        v1[k] = (uint32_t)(v[k] >> 30);
    }
    if constexpr (FPC) {
        u64 y[K];
#pragma unroll
        for (int a = 0; a < K; ++a) {
            const u64 ta = Tin[(long)(L + a) * n];   // [0, 2q): as below
            Dot30 A{negs ? C->fpc_neg[a] : 0ull, 0, 0};
            dot30_mac(A, (uint32_t)ta & M30, (uint32_t)(ta >> 30), C->fpc_pq[a]);
#pragma unroll
            for (int k = 0; k < L; ++k) dot30_mac(A, v0[k], v1[k], C->fpc_qpq[k][a]);
            y[a] = dot30_fold(A, primes[L + a].q);
        }
        fpc_lift<LT>(y, res, C, primes);
    } else {
    u64 w[EXACTO_MAX_K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const u64 pa = primes[L + a].q, np = (u64)0 - pa;
        // [0, 2q) (the tensor's lazy last stage): ta >> 30 < 2^31 doubles one term of a1 and a2,
        // still far inside dot30_fold's budget (< (m + 4.1) 2^60 with m = L + 1 <= 7 terms)
        const u64 ta = Tin[(long)(L + a) * n];
        Dot30 A{negs ? 1ull : 0ull, 0, 0};
        dot30_mac(A, (uint32_t)ta & M30, (uint32_t)(ta >> 30), C->pq_w[a]);
#pragma unroll
        for (int k = 0; k < L; ++k) dot30_mac(A, v0[k], v1[k], pa - C->qpq_w[k][a]);
        u64 acc = dot30_fold(A, pa);
        // Garner over P on the fly; w_k < p_k < 2 p_a
#pragma unroll
        for (int k = 0; k < a; ++k) acc = shoup_mul_nq(acc + 2 * pa - w[k], C->gp_w[a][k], C->gp_ws[a][k], np);
        w[a] = (a > 0 && acc >= pa) ? acc - pa : acc;
    }
    const bool negr = mr_greater<EXACTO_MAX_K>(w, C->halfP_mr, K);
    uint32_t w0[K], w1[K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        w0[a] = (uint32_t)w[a] & M30;
        w1[a] = (uint32_t)(w[a] >> 30);
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const u64 q = primes[i].q;
        Dot30 A{negr ? q - C->ppref_w[K][i] : 0, 0, 0};
#pragma unroll
        for (int a = 0; a < K; ++a) dot30_mac(A, w0[a], w1[a], C->ppref_w[a][i]);
        res[i] = dot30_fold(A, q);
    }
    }
    }   // FPQ
    if (comp < ncomp_r) {
        u64* out = R + item * r_stride + (long)comp * L * n + j;
#pragma unroll
        for (int i = 0; i < L; ++i) out[(long)i * n] = res[i];
    }
    if (comp != 2) return;
    if constexpr (DIG == 1) {
        gadget_digits16_sp<LT>(res, C, primes, n, guse, D16 + item * (long)guse * n + j);
    } else if constexpr (DIG == 3) {   // int8: base <= 2^8, every balanced digit in [-128, 127]
        gadget_digits16_sp<LT, int8_t>(res, C, primes, n, guse,
                                       reinterpret_cast<int8_t*>(D16) + item * (long)guse * n + j);
    } else if constexpr (DIG == 2) {
        if (D16 != nullptr)
            gadget_digits<true, LT>(res, L, C, primes, nullptr, n, guse, D16 + item * (long)guse * n + j);
        else
            gadget_digits<true, LT>(res, L, C, primes, D + item * (long)guse * L * n + j, n, guse);
    }
}

// dBFV psum: one output limb k's component c (0 or 1) = sum over its products of their scaled
// components, computed as one scale.  Per product, r = (p T - s) / Q with s = [p T]_Q centred;
// in an auxiliary prime p_a that is r = T_a (p Q^-1) + sum_k v_k (p_a - qpq_k,a) + negs (the v_k and
// negs from the product's ciphertext-prime residues).  The first term is linear in T, so its sum
// over the products is the summed auxiliary residue (dbfv_pairsum_kernel + inverse NTT); the others are
// added product by product.  R = sum r is then lifted from P exactly as exact_scale_sp_kernel
// lifts one r: the context checks m (p n Q + 2) < P (|R| < P / 2, psum_max).  Bit-identical to
// summing the per-product results mod q_i (dbfv_combine_kernel), which is what it replaces.
// row = (ib d + k) 2 + c; T as the tensor kernels leave it, Tsum [ib][k][c][a][n] (launch_dbfv_pairsum).
template <int LT, bool FPC, bool FPQ = false>
__global__ void __launch_bounds__(TPB)
exact_psum_sp_kernel(const u64* __restrict__ T, const u64* __restrict__ Tsum, u64* __restrict__ out, int d, int npairs,
                     const int* __restrict__ term_start, const CombineTerm* __restrict__ terms, int n,
                     const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes, double fpq_lim = 0.0) {
    ROW_SETUP(n)
    constexpr int L = LT, K = LT + 1, NP = L + K;
    const int c = (int)(row & 1);
    const long r2 = row >> 1;
    const int k = (int)(r2 % d);
    const long ib = r2 / d;
    u64 carry[K];
    {
        const u64* Ts = Tsum + row * K * (long)n + j;  // [ib][k][c][a][n]
#pragma unroll
        for (int a = 0; a < K; ++a) {
            const u64 ta = Ts[(long)a * n];   // canonical (inverse transform output)
            Dot30 A{0, 0, 0};
            dot30_mac(A, (uint32_t)ta & M30, (uint32_t)(ta >> 30), FPC ? C->fpc_pq[a] : C->pq_w[a]);
            carry[a] = dot30_fold(A, primes[L + a].q);
        }
    }
    if constexpr (FPQ) {   // the products' s parts by the float sum (Garner near +-Q/2), one dot per row
        static_assert(FPC, "FPQ feeds the float lift from P");
        u64 Z[L];
#pragma unroll
        for (int i = 0; i < L; ++i) Z[i] = 0;
        uint32_t bs = 0;
        int cnt = 0;
        for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
            fpq_acc<LT>(T + ((ib * npairs + terms[t].pair) * 3 + c) * (long)NP * n + j, n, Z, bs, carry, C, primes,
                        fpq_lim);
            if (++cnt == 15) {   // Z_i < 15 q_i < 2^64
                fpq_flush<LT>(Z, bs, carry, C, primes);
                cnt = 0;
            }
        }
        fpq_flush<LT>(Z, bs, carry, C, primes);
        u64 res[EXACTO_MAX_L];
        fpc_lift<LT>(carry, res, C, primes);
        u64* o = out + row * L * (long)n + j;
#pragma unroll
        for (int i = 0; i < L; ++i) o[(long)i * n] = res[i];
        return;
    }
    for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
        const u64* Tin = T + ((ib * npairs + terms[t].pair) * 3 + c) * (long)NP * n + j;
        u64 u[EXACTO_MAX_L], v[EXACTO_MAX_L];
#pragma unroll
        for (int i = 0; i < L; ++i) u[i] = shoup_mul(Tin[(long)i * n], C->pmod_w[i], C->pmod_ws[i], primes[i].q);
        garner_q_fast<LT>(v, u, L, C, primes);
        const bool negs = mr_greater<EXACTO_MAX_L>(v, C->halfQ_mr, L);
        uint32_t v0[L], v1[L];
#pragma unroll
        for (int kk = 0; kk < L; ++kk) {
            v0[kk] = (uint32_t)v[kk] & M30;
            v1[kk] = (uint32_t)(v[kk] >> 30);
        }
#pragma unroll
        for (int a = 0; a < K; ++a) {
            const u64 pa = primes[L + a].q;
            // carry < p_a: a0's constant stays < 2^60 (FPC: < 2^61, inside dot30_fold's budget)
            Dot30 A{carry[a] + (negs ? (FPC ? C->fpc_neg[a] : 1ull) : 0ull), 0, 0};
#pragma unroll
            for (int kk = 0; kk < L; ++kk) dot30_mac(A, v0[kk], v1[kk], FPC ? C->fpc_qpq[kk][a] : pa - C->qpq_w[kk][a]);
            carry[a] = dot30_fold(A, pa);
        }
    }
    u64* o = out + row * L * (long)n + j;
    if constexpr (FPC) {   // carry[a] = R Pi_a mod p_a
        u64 res[EXACTO_MAX_L];
        fpc_lift<LT>(carry, res, C, primes);
#pragma unroll
        for (int i = 0; i < L; ++i) o[(long)i * n] = res[i];
        return;
    }
    u64 w[EXACTO_MAX_K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const u64 pa = primes[L + a].q, np = (u64)0 - pa;
        u64 acc = carry[a];
#pragma unroll
        for (int kk = 0; kk < a; ++kk) acc = shoup_mul_nq(acc + 2 * pa - w[kk], C->gp_w[a][kk], C->gp_ws[a][kk], np);
        w[a] = (a > 0 && acc >= pa) ? acc - pa : acc;
    }
    const bool negr = mr_greater<EXACTO_MAX_K>(w, C->halfP_mr, K);
    uint32_t w0[K], w1[K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        w0[a] = (uint32_t)w[a] & M30;
        w1[a] = (uint32_t)(w[a] >> 30);
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const u64 q = primes[i].q;
        Dot30 A{negr ? q - C->ppref_w[K][i] : 0, 0, 0};
#pragma unroll
        for (int a = 0; a < K; ++a) dot30_mac(A, w0[a], w1[a], C->ppref_w[a][i]);
        o[(long)i * n] = dot30_fold(A, q);
    }
}

bool launch_psum_scale(const u64* T, const u64* Tsum, u64* out, int items_b, int d, int npairs, const int* term_start,
                       const CombineTerm* terms, int n, const CrtTables* ct, const PrimeConst* primes, int L,
                       hipStream_t s, bool fpc, double fpq_lim) {
    const long blocks = (long)items_b * d * 2 * blocks_per_row(n);
    if (blocks == 0) return true;
#define PSUM_(LT)                                                                                                   \
    do {                                                                                                            \
        if (fpc && fpq_lim > 0.0)                                                                                   \
            EXACTO_LAUNCH((exact_psum_sp_kernel<LT, true, true>), dim3(blocks), dim3(TPB), 0, s, T, Tsum, out, d,   \
                          npairs, term_start, terms, n, ct, primes, fpq_lim);                                      \
        else if (fpc) EXACTO_LAUNCH((exact_psum_sp_kernel<LT, true>), dim3(blocks), dim3(TPB), 0, s, T, Tsum, out,  \
                                    d, npairs, term_start, terms, n, ct, primes, 0.0);                             \
        else EXACTO_LAUNCH((exact_psum_sp_kernel<LT, false>), dim3(blocks), dim3(TPB), 0, s, T, Tsum, out, d,       \
                           npairs, term_start, terms, n, ct, primes, 0.0);                                         \
    } while (0)
    switch (L) {
        case 1: PSUM_(1); break;
        case 2: PSUM_(2); break;
        case 3: PSUM_(3); break;
        case 4: PSUM_(4); break;
        case 5: PSUM_(5); break;
        case 6: PSUM_(6); break;
        default: return false;
    }
#undef PSUM_
    return true;
}

bool exact_scale_sp_ok(int L, int K, int mode) { return mode == 3 && K == L + 1 && L >= 1 && L <= 6 && use_dot30(); }

void launch_exact_scale(const u64* T, u64* R, long r_stride, int ncomp_r, u64* D, int16_t* D16, int guse,
                        int items, int n, const CrtTables* ct, const PrimeConst* primes, int L,
                        int K, int mode, hipStream_t s, int gshift, bool c2only, bool digits8, bool fpc,
                        double fpq_lim) {
    const long blocks = (long)items * (c2only ? 1 : 3) * blocks_per_row(n);
    if (blocks == 0) return;
    if (mode == 3 && K == L + 1 && L >= 1 && L <= 6 && use_dot30()) {
        // digit code: 0 none, 1 int16 fields of the magnitude (base 2^sh, sh | 32), 2 gadget_digits
        const int dig = (D16 == nullptr && D == nullptr) || guse <= 0 ? 0
                        : (D16 != nullptr && gshift > 0 && 32 % gshift == 0) ? (digits8 && gshift <= 8 ? 3 : 1) : 2;
#define SCALE30_(LT, DG)                                                                                        \
    do {                                                                                                        \
        if (fpc && fpq_lim > 0.0)                                                                               \
            EXACTO_LAUNCH((exact_scale_sp_kernel<LT, DG, true, true>), dim3(blocks), dim3(TPB), 0, s, T, R,     \
                          r_stride, ncomp_r, D, D16, guse, n, ct, primes, c2only ? 1 : 0, fpq_lim);             \
        else if (fpc) EXACTO_LAUNCH((exact_scale_sp_kernel<LT, DG, true>), dim3(blocks), dim3(TPB), 0, s, T, R, \
                               r_stride, ncomp_r, D, D16, guse, n, ct, primes, c2only ? 1 : 0, 0.0);            \
        else EXACTO_LAUNCH((exact_scale_sp_kernel<LT, DG, false>), dim3(blocks), dim3(TPB), 0, s, T, R,         \
                           r_stride, ncomp_r, D, D16, guse, n, ct, primes, c2only ? 1 : 0, 0.0);                \
    } while (0)
#define SCALE30(LT)                         \
    do {                                    \
        if (dig == 1) SCALE30_(LT, 1);      \
        else if (dig == 3) SCALE30_(LT, 3); \
        else if (dig == 2) SCALE30_(LT, 2); \
        else SCALE30_(LT, 0);               \
    } while (0)
        switch (L) {
            case 1: SCALE30(1); break;
            case 2: SCALE30(2); break;
            case 3: SCALE30(3); break;
            case 4: SCALE30(4); break;
            case 5: SCALE30(5); break;
            default: SCALE30(6); break;
        }
#undef SCALE30
#undef SCALE30_
        return;
    }
#define SCALE(NR, FS, LT, KT)                                                                                    \
    EXACTO_LAUNCH((exact_scale_kernel<NR, FS, LT, KT>), dim3(blocks), dim3(TPB), 0, s, T, R, r_stride, ncomp_r, \
                       D, D16, guse, n, L, K, ct, primes)
#define SCALE_SP(LT)                                                                                             \
    EXACTO_LAUNCH((exact_scale_kernel<true, true, LT, LT + 1, true>), dim3(blocks), dim3(TPB), 0, s, T, R,   \
                       r_stride, ncomp_r, D, D16, guse, n, L, K, ct, primes)
    if (mode == 3 && K == L + 1 && L >= 1 && L <= 6) {
        switch (L) {
            case 1: SCALE_SP(1); break;
            case 2: SCALE_SP(2); break;
            case 3: SCALE_SP(3); break;
            case 4: SCALE_SP(4); break;
            case 5: SCALE_SP(5); break;
            default: SCALE_SP(6); break;
        }
    } else if (mode >= 2) {
        switch (L) {
            case 1: if (K == 2) SCALE(true, true, 1, 2); else SCALE(true, true, 1, 0); break;
            case 2: if (K == 3) SCALE(true, true, 2, 3); else SCALE(true, true, 2, 0); break;
            case 3: if (K == 4) SCALE(true, true, 3, 4); else SCALE(true, true, 3, 0); break;
            case 4: if (K == 5) SCALE(true, true, 4, 5); else SCALE(true, true, 4, 0); break;
            case 5: if (K == 6) SCALE(true, true, 5, 6); else SCALE(true, true, 5, 0); break;
            case 6: if (K == 7) SCALE(true, true, 6, 7); else SCALE(true, true, 6, 0); break;
            default: SCALE(true, true, 0, 0); break;
        }
    } else if (mode == 1) {
        SCALE(true, false, 0, 0);
    } else {
        SCALE(false, false, 0, 0);
    }
#undef SCALE
#undef SCALE_SP
}

// ---------------------------------------------------------------- decryption

// phase = sum_k c_k * s^k (encrypt.rs:115-123), NTT domain, one thread per (item, limb, coeff).
__global__ void __launch_bounds__(TPB)
phase_kernel(const u64* __restrict__ ct, int polys, long ct_stride, const u64* __restrict__ sk,
             u64* __restrict__ out, int n, int L, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const long item = row / L;
    const int i = (int)(row - item * L);
    const PrimeConst& P = primes[i];
    const long Ln = (long)L * n;
    const u64* c = ct + item * ct_stride + (long)i * n + j;
    const u64 s = sk[(long)i * n + j];
    u64 acc = c[0], sp = s;
    for (int k = 1; k < polys; ++k) {
        acc = add_mod(acc, mul_mod(c[k * Ln], sp, P), P.q);
        if (k + 1 < polys) sp = mul_mod(sp, s, P);
    }
    out[row * n + j] = acc;
}

void launch_phase(const u64* ct, int polys, long ct_stride, const u64* sk, u64* out, int items, int n, int L,
                  const PrimeConst* primes, hipStream_t s) {
    const long blocks = (long)items * L * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(phase_kernel, dim3(blocks), dim3(TPB), 0, s, ct, polys, ct_stride, sk, out, n, L, primes);
}

// m = floor((x p + floor(Q/2)) / Q) mod p for x = CRT(phase) in [0, Q) (encrypt.rs:145-171),
// one thread per (item, coefficient).  L = 1: one 128-by-64 division.  L >= 2: in RNS, with
// s = (p x + floor(Q/2)) mod Q from its Garner digits and r = (p x + floor(Q/2) - s) / Q
// evaluated in the first auxiliary prime P0 > p, where it is exact because 0 <= r <= p.
__global__ void __launch_bounds__(TPB)
decrypt_round_kernel(const u64* __restrict__ X, u64* __restrict__ out, int n, int L,
                     const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes, u64 plain) {
    ROW_SETUP(n)
    u64 r;
    if (L == 1) {
        const u64 q = primes[0].q;
        const u128 y = (u128)X[row * n + j] * plain + (q >> 1);
        r = (u64)(y / q);
    } else {
        u64 x[EXACTO_MAX_L], s[EXACTO_MAX_L], vx[EXACTO_MAX_L], vs[EXACTO_MAX_L];
#pragma unroll
        for (int i = 0; i < EXACTO_MAX_L; ++i) {
            if (i < L) {
                const u64 qi = primes[i].q;
                x[i] = X[(row * L + i) * n + j];
                s[i] = add_mod(shoup_mul_red(x[i], C->pmod_w[i], C->pmod_ws[i], qi), C->hq[i], qi);
            }
        }
        garner_q<false>(vx, x, L, C, primes);
        garner_q<false>(vs, s, L, C, primes);
        const int t = L;
        const PrimeConst& P0 = primes[t];
        const u64 p0 = P0.q;
        const u64 xP = mr_eval<EXACTO_MAX_L, EXACTO_MAX_PRIMES, false>(vx, L, false, &C->qpref_w[0][0],
                                                                       &C->qpref_ws[0][0], t, P0);
        const u64 sP = mr_eval<EXACTO_MAX_L, EXACTO_MAX_PRIMES, false>(vs, L, false, &C->qpref_w[0][0],
                                                                       &C->qpref_ws[0][0], t, P0);
        const u64 a = shoup_mul_red(xP, C->pq_w[0], C->pq_ws[0], p0);
        const u64 b = shoup_mul_red(sub_mod(C->hq[t], sP, p0), C->qinvp_w[0], C->qinvp_ws[0], p0);
        r = add_mod(a, b, p0);
    }
    out[row * n + j] = r >= plain ? r - plain : r;  // r <= p
}

void launch_decrypt_round(const u64* X, u64* out, int items, int n, int L, const CrtTables* ct,
                          const PrimeConst* primes, u64 plain, hipStream_t s) {
    const long blocks = (long)items * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(decrypt_round_kernel, dim3(blocks), dim3(TPB), 0, s, X, out, n, L, ct, primes, plain);
}

// Signed digit recomposition (dbfv/decomposition.rs:45-68, 112-127): sum centred(mu_k) b^k in
// i128 with Rust's release-mode wrapping, then mod p (p = 0: truncation to 64 bits).
__global__ void __launch_bounds__(TPB)
dbfv_recompose_kernel(const u64* __restrict__ digits, u64* __restrict__ out, int items, int n, int d, u64 base,
                      u64 plain, u64 t, int scalar) {
    const long idx = (long)blockIdx.x * TPB + threadIdx.x;
    const int ncoef = scalar ? 1 : n;
    if (idx >= (long)items * ncoef) return;
    const long item = idx / ncoef;
    const int j = (int)(idx - item * ncoef);
    const u64 half_t = t / 2;
    u128 result = 0, power = 1;  // two's-complement i128, wrapping
    for (int k = 0; k < d; ++k) {
        const u64 dk = digits[(item * d + k) * n + j];
        const u128 centred = dk > half_t ? (u128)dk - (u128)t : (u128)dk;  // wraps to a negative i128
        result += centred * power;
        power *= (u128)base;
    }
    u64 r;
    if (plain == 0) {
        r = (u64)result;
    } else if ((i128)result >= 0) {
        r = (u64)(result % plain);
    } else {
        const u64 m = (u64)((~result + 1) % plain);  // |result| mod p
        r = m == 0 ? 0 : plain - m;
    }
    out[idx] = r;
}

void launch_dbfv_recompose(const u64* digits, u64* out, int items, int n, int d, u64 base, u64 plain, u64 t,
                           bool scalar, hipStream_t s) {
    const long total = (long)items * (scalar ? 1 : n);
    if (total == 0) return;
    EXACTO_LAUNCH(dbfv_recompose_kernel, dim3((unsigned)((total + TPB - 1) / TPB)), dim3(TPB), 0, s, digits,
                       out, items, n, d, base, plain, t, scalar ? 1 : 0);
}

// ---------------------------------------------------------------- HPS scale (eval.rs:257-413)

// HPS round(p a_c / q) + p m (mod q) without any division (FAST: q > 2^32 and p < min(q, 2^32)).
// Every step is exact integer arithmetic, so the result equals the literal form below bit for bit:
//   * est = floor((p |a_c| + floor(q/2)) / q) < p/2 + 1 < 2^31: with pc = floor(p 2^64 / q),
//     hi64(|a_c| pc) is floor(p |a_c| / q) or one less (|a_c| < 2^61), so est is that plus 0, 1 or 2,
//     decided on the remainder x - e q, which lies in [0, 3q) and so is exact in 64-bit wrapping
//     arithmetic (q < 2^62);
//   * every product by a constant is a Shoup product (the unique residue, as ref_mod_mul's u128 %);
//   * (a + b) mod q for the integer sum round + p m is formed from each part mod q (a ring map).
__device__ __forceinline__ u64 hps_round_mod(u64 a, u64 q, u64 p, u64 pc) {
    const bool neg = a > q / 2;
    const u64 mag = neg ? q - a : a;                      // |a_c|
    u64 e = mulhi64(mag, pc);
    u64 r = p * mag + (q >> 1) - e * q;                   // exact: the true value is in [0, 3q)
    if (r >= q) { ++e; r -= q; }
    if (r >= q) ++e;
    // round_pa_q = +/- e; mod q (e < 2^31 < q)
    return (neg && e) ? q - e : e;
}

// gadget_digits for one ciphertext prime (HPS) and a power-of-two base 2^sh (1 <= sh <= 16), signed
// digits only: the same digits (keyswitch.rs:24-44: truncating %, [-B/2, B/2) adjustment, final
// carry dropped) from one word, branch-free.
template <typename DT>
__device__ __forceinline__ void gadget_digits_l1(u64 v, u64 q, int sh, int guse, DT* D16, int n) {
    const bool neg = v > (q >> 1);
    u64 M = neg ? q - v : v;                      // |centred value|
    const u64 B = 1ull << sh, mask = B - 1, half = B >> 1;
    for (int g = 0; g < guse; ++g) {
        const u64 r = M & mask;
        M >>= sh;
        // value +M: r >= B/2 -> digit r - B and a carry; value -M: r > B/2 -> digit B - r and a carry
        const bool carry = neg ? (r > half) : (r >= half);
        const i64 mag = carry ? (i64)(B - r) : (i64)r;
        const bool dneg = neg ? !carry : carry;
        M += carry ? 1 : 0;
        D16[(long)g * n] = (DT)(dneg ? -mag : mag);
    }
}

// hps_round_mod on a value already centred: |a_c| and its sign
__device__ __forceinline__ u64 hps_round_mag(u64 mag, bool neg, u64 q, u64 p, u64 pc) {
    u64 e = mulhi64(mag, pc);
    u64 r = p * mag + (q >> 1) - e * q;                   // exact: the true value is in [0, 3q)
    if (r >= q) { ++e; r -= q; }
    if (r >= q) ++e;
    return (neg && e) ? q - e : e;
}

__device__ __forceinline__ u64 hps_ext_fast(u64 a, u64 q, const PrimeConst& P) {
    // eval.rs:307-313 with reduce64 instead of the % of a runtime divisor
    if (a > q / 2) {
        const u64 rem = reduce64(q - a, P.q, P.mu64);
        return rem == 0 ? 0 : P.q - rem;
    }
    return reduce64(a, P.q, P.mu64);
}

__device__ __forceinline__ u64 hps_ext(u64 a, u64 q, u64 pj) {
    // eval.rs:307-313
    if (a > q / 2) {
        const u64 rem = (q - a) % pj;
        return rem == 0 ? 0 : pj - rem;
    }
    return a % pj;
}

// Scaled component c of one item, coefficient j (eval.rs:257-413).  The third component's balanced
// gadget digits go to D as residues mod q ([item][g][n]) or, with DT = int16_t / int8_t, to D16 as
// signed digits (gadget base <= 2^16 / 2^8; dBFV sums them per output limb before one key switch).
// KK (FAST only): the number of auxiliary primes, 1 or 2, as a compile-time constant (0: K at run
// time, the literal path).
template <bool FAST, typename DT, int KK = 0>
__global__ void __launch_bounds__(TPB)
hps_scale_kernel(const u64* __restrict__ T, u64* __restrict__ R, long r_stride, int ncomp_r,
                 u64* __restrict__ D, DT* __restrict__ D16, int guse, int n, int K_,
                 const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    const int K = KK ? KK : K_;
    ROW_SETUP(n)
    const long item = row / 3;
    const int comp = (int)(row - item * 3);
    if (comp >= ncomp_r && (comp != 2 || (D == nullptr && D16 == nullptr))) return;
    const u64* Tin = T + row * (1 + K) * n + j;
    const u64 q = primes[0].q;
    const u64 p = C->plain;
    const u64 a = Tin[0];
    u64 result;
    if (FAST) {
        const PrimeConst& Pq = primes[0];
        // a centred once: |a_c| feeds the rounding and the extension to every auxiliary prime
        const bool aneg = a > (q >> 1);
        const u64 amag = aneg ? q - a : a;
        const u64 rq = hps_round_mag(amag, aneg, q, p, C->hps_pc);
        // a_c mod p_j (eval.rs:307-313): |a_c| < q/2 needs no reduction when q <= p_j (block-uniform)
        auto ext = [&](const PrimeConst& P) {
            const u64 m = q <= P.q ? amag : reduce64(amag, P.q, P.mu64);
            return (aneg && m) ? P.q - m : m;
        };
        u64 mq;   // m mod q, Euclidean
        if (K == 1) {
            // eval.rs:301-332
            const PrimeConst& P1 = primes[1];
            const u64 bp = P1.q;
            const u64 diff = sub_mod(Tin[n], ext(P1), bp);
            const u64 m_raw = shoup_mul_red(diff, C->hps_qinv[0], C->hps_qinv_s[0], bp);
            const bool mneg = m_raw > bp / 2;
            const u64 mag = mneg ? bp - m_raw : m_raw;
            const u64 r = reduce64(mag, q, Pq.mu64);
            mq = (mneg && r) ? q - r : r;
        } else {
            // eval.rs:349-404: m from its residues mod p0, p1 by CRT, centred mod P = p0 p1.
            // t_j = (T_j - a mod p_j) q^-1 p_{1-j}^-1 mod p_j (one folded constant each); the CRT sum
            // t0 p1 + t1 p0 < 2P decides how many P to subtract (k = 0, 1, 2: the Euclidean residue,
            // then the centring), and m mod q = t0 (p1 mod q) + t1 (p0 mod q) - k (P mod q).
            const u64 p0 = primes[1].q, p1 = primes[2].q;
            const u64 t0 = shoup_mul_red(sub_mod(Tin[n], ext(primes[1]), p0), C->hps_t_w[0], C->hps_t_ws[0], p0);
            const u64 t1 = shoup_mul_red(sub_mod(Tin[2L * n], ext(primes[2]), p1), C->hps_t_w[1], C->hps_t_ws[1], p1);
            const u128 bigp = ((u128)C->hps_P[1] << 64) | C->hps_P[0];
            const u128 halfp = ((u128)C->hps_halfP[1] << 64) | C->hps_halfP[0];
            u128 mc = (u128)t0 * p1 + (u128)t1 * p0;           // < 2 P
            int k = 0;
            if (mc >= bigp) { mc -= bigp; k = 1; }
            if (mc > halfp) ++k;
            const u64 s = add_mod(shoup_mul_red(t0, C->hps_pq_w[0], C->hps_pq_ws[0], q),
                                  shoup_mul_red(t1, C->hps_pq_w[1], C->hps_pq_ws[1], q), q);
            mq = sub_mod(s, C->hps_kPq[k], q);
        }
        // p < q: pc = floor(p 2^64 / q) is p's Shoup companion mod q
        result = add_mod(rq, shoup_mul_red(mq, p, C->hps_pc, q), q);
    } else {
        const i128 q128 = (i128)q;
        const u64 half_q = q / 2;
        const i128 a_centered = a > half_q ? (i128)a - q128 : (i128)a;
        const i128 pa = (i128)p * a_centered;
        const i128 round_pa_q = pa >= 0 ? (pa + q128 / 2) / q128 : -((-pa + q128 / 2) / q128);
        if (K == 1) {
            // eval.rs:301-332
            const u64 big_p = primes[1].q;
            const u64 b = Tin[n];
            const u64 a_ext = hps_ext(a, q, big_p);
            const u64 diff = b >= a_ext ? b - a_ext : big_p - a_ext + b;
            const u64 m_raw = ref_mod_mul(diff, C->hps_qinv[0], big_p);
            const i128 m_centered = m_raw > big_p / 2 ? (i128)m_raw - (i128)big_p : (i128)m_raw;
            const i128 scaled = round_pa_q + (i128)p * m_centered;
            result = (u64)(((scaled % q128) + q128) % q128);
        } else {
            // eval.rs:349-404
            const u64 p0 = primes[1].q, p1 = primes[2].q;
            const u64 b0 = Tin[n], b1 = Tin[2L * n];
            const u64 a_ext0 = hps_ext(a, q, p0);
            const u64 diff0 = b0 >= a_ext0 ? b0 - a_ext0 : p0 - a_ext0 + b0;
            const u64 m0 = ref_mod_mul(diff0, C->hps_qinv[0], p0);
            const u64 a_ext1 = hps_ext(a, q, p1);
            const u64 diff1 = b1 >= a_ext1 ? b1 - a_ext1 : p1 - a_ext1 + b1;
            const u64 m1 = ref_mod_mul(diff1, C->hps_qinv[1], p1);
            const i128 t0 = (i128)ref_mod_mul(m0, C->hps_p1_inv_p0, p0);
            const i128 t1 = (i128)ref_mod_mul(m1, C->hps_p0_inv_p1, p1);
            const i128 big_p = (i128)p0 * (i128)p1;
            const i128 half_big_p = big_p / 2;
            const i128 crt_sum = t0 * (i128)p1 + t1 * (i128)p0;
            const i128 m_crt = crt_sum % big_p;
            const i128 m_centered = m_crt > half_big_p ? m_crt - big_p : m_crt;
            const i128 m_mod_q = ((m_centered % q128) + q128) % q128;
            const u64 round_mod_q = (u64)(((round_pa_q % q128) + q128) % q128);
            const u64 pm_mod_q = ref_mod_mul(p, (u64)m_mod_q, q);
            result = (u64)(((u128)round_mod_q + pm_mod_q) % q);
        }
    }
    if (comp < ncomp_r) R[item * r_stride + (long)comp * n + j] = result;
    if (comp == 2) {
        u64 res[EXACTO_MAX_L];
        res[0] = result;
        if (D16 && C->gshift >= 1 && C->gshift <= 16)   // every HPS config: base 2^8 or 2^16
            gadget_digits_l1<DT>(result, q, C->gshift, guse, D16 + item * (long)guse * n + j, n);
        else if (D16) gadget_digits<false, 1, DT>(res, 1, C, primes, nullptr, n, guse, D16 + item * (long)guse * n + j);
        else if (D) gadget_digits<false, 1>(res, 1, C, primes, D + item * (long)guse * n + j, n, guse);
    }
}

void launch_hps_scale(const u64* T, u64* R, long r_stride, int ncomp_r, u64* D, void* D16, bool d8, int guse,
                      int items, int n, const CrtTables* ct, const PrimeConst* primes, int K, bool fast,
                      hipStream_t s) {
    const long blocks = (long)items * 3 * blocks_per_row(n);
    if (blocks == 0) return;
#define HPS_(F, DT, KK) EXACTO_LAUNCH((hps_scale_kernel<F, DT, KK>), dim3(blocks), dim3(TPB), 0, s, T, R, \
                                           r_stride, ncomp_r, D, (DT*)D16, guse, n, K, ct, primes)
    if (fast && K == 1) {
        if (d8) HPS_(true, int8_t, 1); else HPS_(true, int16_t, 1);
    } else if (fast && K == 2) {
        if (d8) HPS_(true, int8_t, 2); else HPS_(true, int16_t, 2);
    } else {
        if (d8) HPS_(false, int8_t, 0); else HPS_(false, int16_t, 0);
    }
#undef HPS_
}

// ---------------------------------------------------------------- standalone decomposition

__global__ void __launch_bounds__(TPB)
decompose_kernel(const u64* __restrict__ C2, long c2_stride, u64* __restrict__ D, int16_t* __restrict__ D16,
                 int guse, int n, int L, const CrtTables* __restrict__ C, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    u64 res[EXACTO_MAX_L];
#pragma unroll
    for (int i = 0; i < EXACTO_MAX_L; ++i)
        if (i < L) res[i] = C2[row * c2_stride + (long)i * n + j];
    if (D16)
        gadget_digits<false>(res, L, C, primes, nullptr, n, guse, D16 + row * (long)guse * n + j);
    else
        gadget_digits<false>(res, L, C, primes, D + row * (long)guse * L * n + j, n, guse);
}

void launch_decompose(const u64* C2, long c2_stride, u64* D, int guse, int items, int n,
                      const CrtTables* ct, const PrimeConst* primes, int L, hipStream_t s, int16_t* D16) {
    const long blocks = (long)items * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(decompose_kernel, dim3(blocks), dim3(TPB), 0, s, C2, c2_stride, D, D16, guse, n, L,
                       ct, primes);
}

// ---------------------------------------------------------------- relinearisation MAC

// out_c = base_c + sum_g D_g (.) rlk_g,c  (keyswitch.rs:86-95), NTT domain.  One thread per
// (item, limb i, coefficient j).  Blocks are numbered item-fastest, so the blocks resident at
// any time share a few 256-coefficient key slices: the key and its Shoup companions
// (G*2*L*n words each, more than one XCD's L2 at cfg3) come from HBM about once per XCD
// instead of once per item.  Accumulators stay in [0, 2q); D is canonical.
__global__ void __launch_bounds__(TPB)
relin_mac_kernel(const u64* __restrict__ base, long base_stride, const u64* __restrict__ D,
                 const u64* __restrict__ rlk, const u64* __restrict__ rlk_s, int guse, u64* out,
                 long out_stride, int items, int n, int L, const PrimeConst* __restrict__ primes) {
    // two consecutive coefficients per thread: 16-byte loads/stores (n is even)
    const long Ln = (long)L * n;
    const int it = (int)(blockIdx.x % (unsigned)items);
    const long coef = ((long)(blockIdx.x / (unsigned)items) * TPB + threadIdx.x) * 2;
    if (coef >= Ln) return;
    const int i = (int)(coef / n);
    const PrimeConst& P = primes[i];
    const u64 q = P.q, q2 = P.two_q, nq = (u64)0 - q;
    typedef ulonglong2 V2;
    const u64* bp = base + it * base_stride;
    const V2 b0 = *(const V2*)(bp + coef), b1 = *(const V2*)(bp + Ln + coef);
    u64 a0x = b0.x, a0y = b0.y, a1x = b1.x, a1y = b1.y;
    const u64* dp = D + (long)it * guse * Ln + coef;
    constexpr int U = 4;
    for (int g0 = 0; g0 < guse; g0 += U) {
        V2 d[U], w0[U], s0[U], w1[U], s1[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int g = min(g0 + t, guse - 1);  // clamped (re-read) tail, masked below
            const long k0 = 2L * g * Ln + coef;
            d[t] = *(const V2*)(dp + (long)g * Ln);
            w0[t] = *(const V2*)(rlk + k0);
            s0[t] = *(const V2*)(rlk_s + k0);
            w1[t] = *(const V2*)(rlk + k0 + Ln);
            s1[t] = *(const V2*)(rlk_s + k0 + Ln);
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
            if (g0 + t < guse) {
                u64 v = a0x + shoup_mul_nq(d[t].x, w0[t].x, s0[t].x, nq);
                a0x = v >= q2 ? v - q2 : v;
                v = a0y + shoup_mul_nq(d[t].y, w0[t].y, s0[t].y, nq);
                a0y = v >= q2 ? v - q2 : v;
                v = a1x + shoup_mul_nq(d[t].x, w1[t].x, s1[t].x, nq);
                a1x = v >= q2 ? v - q2 : v;
                v = a1y + shoup_mul_nq(d[t].y, w1[t].y, s1[t].y, nq);
                a1y = v >= q2 ? v - q2 : v;
            }
        }
    }
    u64* op = out + it * out_stride;
    *(V2*)(op + coef) = make_ulonglong2(a0x >= q ? a0x - q : a0x, a0y >= q ? a0y - q : a0y);
    *(V2*)(op + Ln + coef) = make_ulonglong2(a1x >= q ? a1x - q : a1x, a1y >= q ? a1y - q : a1y);
}

// Same MAC with the key slice staged in LDS: a block owns 64 consecutive coefficients of one
// limb and MAC_IG items; its key words and Shoup companions for every digit (guse * 2 KiB) are
// read from HBM once and then served from LDS, so global traffic is D + base + out only.
// Wave w of the block handles items it0 + w, it0 + w + 4, ...; lane = coefficient.
constexpr int MAC_LS = 64;   // coefficients per block
constexpr int MAC_IG = 64;   // items per block
constexpr int MAC_GMAX = 32; // digits staged (LDS = 2 KiB per digit)

__global__ void __launch_bounds__(TPB)
relin_mac_lds_kernel(const u64* __restrict__ base, long base_stride, const u64* __restrict__ D,
                     const u64* __restrict__ rlk, const u64* __restrict__ rlk_s, int guse, u64* out,
                     long out_stride, int items, int n, int L, const PrimeConst* __restrict__ primes) {
    extern __shared__ u64 ks[];  // [guse][4][MAC_LS]: w0, ws0, w1, ws1
    const long Ln = (long)L * n;
    const long c0 = (long)blockIdx.x * MAC_LS;  // first coefficient (flat limb*n + j)
    const int lane = threadIdx.x & (MAC_LS - 1), wave = threadIdx.x / MAC_LS;
    for (int r = threadIdx.x; r < guse * 4 * MAC_LS; r += TPB) {
        const int g = r / (4 * MAC_LS), w = (r / MAC_LS) & 3, l = r & (MAC_LS - 1);
        const long kk = (2L * g + (w >> 1)) * Ln + c0 + l;
        ks[r] = (w & 1) ? rlk_s[kk] : rlk[kk];
    }
    __syncthreads();
    const long coef = c0 + lane;
    const int i = (int)(coef / n);
    const PrimeConst& P = primes[i];
    const u64 q = P.q, q2 = P.two_q, nq = (u64)0 - q;
    const int it_end = min(items, (int)(blockIdx.y + 1) * MAC_IG);
    for (int it = blockIdx.y * MAC_IG + wave; it < it_end; it += TPB / MAC_LS) {
        const u64* bp = base + it * base_stride;
        u64 a0 = bp[coef], a1 = bp[Ln + coef];
        const u64* dp = D + (long)it * guse * Ln + coef;
        constexpr int U = 4;
        for (int g0 = 0; g0 < guse; g0 += U) {
            u64 d[U];
#pragma unroll
            for (int t = 0; t < U; ++t) d[t] = dp[(long)min(g0 + t, guse - 1) * Ln];
#pragma unroll
            for (int t = 0; t < U; ++t) {
                if (g0 + t < guse) {
                    const u64* kg = ks + (g0 + t) * 4 * MAC_LS + lane;
                    u64 v = a0 + shoup_mul_nq(d[t], kg[0], kg[MAC_LS], nq);
                    a0 = v >= q2 ? v - q2 : v;
                    v = a1 + shoup_mul_nq(d[t], kg[2 * MAC_LS], kg[3 * MAC_LS], nq);
                    a1 = v >= q2 ? v - q2 : v;
                }
            }
        }
        u64* op = out + it * out_stride;
        op[coef] = a0 >= q ? a0 - q : a0;
        op[Ln + coef] = a1 >= q ? a1 - q : a1;
    }
}

// Strided row copy / zero fill: dst[r * dst_stride + k] = src ? src[r * src_stride + k] : 0 for
// k < len, r < rows: the strided ciphertext-component fills and copies as one ordinary kernel on
// the context stream (no 2D memset/memcpy engine path).
// EXACTO_DEBUG_BOOT: a watched byte range [lo, hi) (lo >= hi: off), passed to the
// library's generic writers (rows, copy, fill) as kernel arguments; a write inside it sets
// hit[kind] (a vector store): 0 rows copy, 1 rows zero fill, 2 copy_u64, 3 fill_u32 of 0, 4 fill_u32
// of another value.  Arguments rather than a device symbol: setting a symbol needs a copy and a
// synchronisation on the stream, and with those the round-5 failing runs no longer failed.
struct DbgWatch {
    u64 lo = 0, hi = 0;
    uint32_t* hit = nullptr;
    hipStream_t stream = nullptr;   // only launches on this stream get the watch
};
// host side, read by the launchers below: per host thread, and applied only to launches on the stream
// the bootstrap call registered (another context, thread or device never receives its hit pointer)
static thread_local DbgWatch g_watch;
static DbgWatch watch_for(hipStream_t s) { return (g_watch.hit && s == g_watch.stream) ? g_watch : DbgWatch{}; }
__device__ __forceinline__ void dbg_watch(const void* a, int kind, u64 lo, u64 hi, uint32_t* hit) {
    const u64 x = (u64)a;
    if (x >= lo && x < hi) hit[kind] = 1;
}

void debug_watch_set(const void* lo, const void* hi, uint32_t* hit, hipStream_t s) {
    g_watch.lo = (u64)lo;
    g_watch.hi = (u64)hi;
    g_watch.hit = hit;
    g_watch.stream = s;
}

__global__ void __launch_bounds__(TPB)
rows_kernel(u64* __restrict__ dst, long dst_stride, const u64* __restrict__ src, long src_stride, long len,
            long total, u64 wlo, u64 whi, uint32_t* whit) {
    for (long t = (long)blockIdx.x * TPB + threadIdx.x; t < total; t += (long)gridDim.x * TPB) {
        const long r = t / len, k = t - r * len;
        dbg_watch(&dst[r * dst_stride + k], src ? 0 : 1, wlo, whi, whit);
        dst[r * dst_stride + k] = src ? src[r * src_stride + k] : 0;
    }
}

// Diagnostic (EXACTO_DEBUG_BOOT): every block copies the same `words` words into its
// own slot of dst and records the XCD it ran on, so a stale per-XCD L2 line shows as one slot
// differing from the others.
__global__ void __launch_bounds__(64) xcd_probe_kernel(const u64* src, u64* dst, long words, uint32_t* xcc) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    for (long i = threadIdx.x; i < words; i += 64) dst[blockIdx.x * words + i] = src[i];
    if (threadIdx.x == 0) xcc[blockIdx.x] = x;
}

void launch_xcd_probe(const u64* src, u64* dst, long words, uint32_t* xcc, int blocks, hipStream_t s) {
    EXACTO_LAUNCH(xcd_probe_kernel, dim3(blocks), dim3(64), 0, s, src, dst, words, xcc);
}

void launch_rows(u64* dst, long dst_stride, const u64* src, long src_stride, long len, long rows, hipStream_t s) {
    const long total = len * rows;
    if (total <= 0) return;
    const long blocks = std::min<long>((total + TPB - 1) / TPB, 65536);
    const DbgWatch w = watch_for(s);
    EXACTO_LAUNCH(rows_kernel, dim3((unsigned)blocks), dim3(TPB), 0, s, dst, dst_stride, src, src_stride, len,
                       total, w.lo, w.hi, w.hit);
}

void launch_relin_mac(const u64* base, long base_stride, const u64* D, const u64* rlk, const u64* rlk_s,
                      int guse, u64* out, long out_stride, int items, int n, int L, const PrimeConst* primes,
                      hipStream_t s) {
    if (items <= 0) return;
    const long Ln = (long)L * n;
    static const int use_lds = [] {
        const char* e = getenv("EXACTO_MAC_LDS");
        return e ? atoi(e) : 1;
    }();
    if (use_lds && guse <= MAC_GMAX && Ln % MAC_LS == 0) {
        const dim3 grid((unsigned)(Ln / MAC_LS), (unsigned)((items + MAC_IG - 1) / MAC_IG));
        EXACTO_LAUNCH(relin_mac_lds_kernel, grid, dim3(TPB), (size_t)guse * 4 * MAC_LS * sizeof(u64), s, base,
                           base_stride, D, rlk, rlk_s, guse, out, out_stride, items, n, L, primes);
        return;
    }
    const long blocks = (long)items * ((Ln / 2 + TPB - 1) / TPB);
    EXACTO_LAUNCH(relin_mac_kernel, dim3((unsigned)blocks), dim3(TPB), 0, s, base, base_stride, D, rlk, rlk_s,
                       guse, out, out_stride, items, n, L, primes);
}

// ---------------------------------------------------------------- pointwise RNS ops

__global__ void __launch_bounds__(TPB)
pointwise_kernel(int op, const u64* __restrict__ a, const u64* __restrict__ b, u64* __restrict__ out,
                 int n, int L, const u64* __restrict__ scal, const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const int limb = (int)(row % L);
    const PrimeConst& P = primes[limb];
    const long idx = row * n + j;
    const u64 x = a[idx];
    u64 r;
    switch (op) {
        case 0: r = add_mod(x, b[idx], P.q); break;
        case 1: r = sub_mod(x, b[idx], P.q); break;
        case 2: r = neg_mod(x, P.q); break;
        case 3: r = mul_mod(x, b[idx], P); break;
        case 4: r = mul_mod(x, scal[limb], P); break;
        default: r = x; break;
    }
    out[idx] = r;
}

void launch_pointwise(PwOp op, const u64* a, const u64* b, u64* out, long polys, int n, int L,
                      const u64* scalar_mod, const PrimeConst* primes, hipStream_t s) {
    const long blocks = polys * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(pointwise_kernel, dim3(blocks), dim3(TPB), 0, s, (int)op, a, b, out, n, L,
                       scalar_mod, primes);
}

// bfv_add / bfv_sub of ciphertexts with p1 and p2 components (eval.rs:14-51): component i <
// min(p1, p2) is a +/- b; beyond it the longer operand's component passes through, negated when
// it is ct2's under subtraction.  ct1 [B][p1][L][n], ct2 [B][p2][L][n], out [B][max][L][n]; row =
// (item * max + comp) * L + limb.  out may alias ct1 or ct2 only when its component count equals
// that operand's (same strides): each thread reads its element before writing it, so a, b and out
// are not __restrict__ (the host rejects any other overlap).
__global__ void __launch_bounds__(TPB)
bfv_addsub_kernel(int sub, const u64* a, int p1, const u64* b, int p2, u64* out, int n, int L,
                  const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    const int pm = p1 > p2 ? p1 : p2;
    const int limb = (int)(row % L);
    const long r1 = row / L;
    const int comp = (int)(r1 % pm);
    const long item = r1 / pm;
    const u64 q = primes[limb].q;
    const long ia = ((item * p1 + comp) * L + limb) * (long)n + j;
    const long ib = ((item * p2 + comp) * L + limb) * (long)n + j;
    u64 r;
    if (comp < p1 && comp < p2) r = sub ? sub_mod(a[ia], b[ib], q) : add_mod(a[ia], b[ib], q);
    else if (comp < p1) r = a[ia];
    else r = sub ? neg_mod(b[ib], q) : b[ib];
    out[row * n + j] = r;
}

void launch_bfv_addsub(bool sub, const u64* a, int p1, const u64* b, int p2, u64* out, long items, int n, int L,
                       const PrimeConst* primes, hipStream_t s) {
    const long blocks = items * (p1 > p2 ? p1 : p2) * L * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(bfv_addsub_kernel, dim3(blocks), dim3(TPB), 0, s, sub ? 1 : 0, a, p1, b, p2, out, n, L, primes);
}

// ---------------------------------------------------------------- dBFV combine

__global__ void __launch_bounds__(TPB)
dbfv_combine_kernel(const u64* __restrict__ prod, int npairs, const int* __restrict__ term_start,
                    const CombineTerm* __restrict__ terms, u64* __restrict__ out, int d, int n, int L,
                    const PrimeConst* __restrict__ primes) {
    ROW_SETUP(n)
    // row = ((item * d + k) * 2 + poly) * L + limb
    const int limb = (int)(row % L);
    const long r1 = row / L;
    const int poly = (int)(r1 % 2);
    const long r2 = r1 / 2;
    const int k = (int)(r2 % d);
    const long item = r2 / d;
    const PrimeConst& P = primes[limb];
    u64 acc = 0;
    for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
        const CombineTerm tm = terms[t];
        const u64 x = prod[(((item * npairs + tm.pair) * 2 + poly) * L + limb) * n + j];
        if (tm.coef == 1) acc = add_mod(acc, x, P.q);
        else acc = add_mod(acc, mul_mod(x, signed_mod(tm.coef, P.q, P.mu64), P), P.q);
    }
    out[row * n + j] = acc;
}

void launch_dbfv_combine(const u64* prod, int npairs, const int* term_start,
                         const CombineTerm* terms, u64* out, int items, int d, int n, int L,
                         const PrimeConst* primes, hipStream_t s) {
    const long blocks = (long)items * d * 2 * L * blocks_per_row(n);
    if (blocks == 0) return;
    EXACTO_LAUNCH(dbfv_combine_kernel, dim3(blocks), dim3(TPB), 0, s, prod, npairs, term_start,
                       terms, out, d, n, L, primes);
}


// ---------------------------------------------------------------- device-to-device copy

// dst <- src, u64 words, as a kernel (context.hip dev_copy: the library's device copies)
__global__ void __launch_bounds__(256)
copy_u64_kernel(u64* __restrict__ dst, const u64* __restrict__ src, long words, u64 wlo, u64 whi, uint32_t* whit) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
        dbg_watch(&dst[i], 2, wlo, whi, whit);
        dst[i] = src[i];
    }
}

void launch_copy_u64(u64* dst, const u64* src, long words, hipStream_t s) {
    if (words <= 0) return;
    long blocks = (words + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    const DbgWatch w = watch_for(s);
    EXACTO_LAUNCH(copy_u64_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, words, w.lo, w.hi, w.hit);
}


__global__ void __launch_bounds__(256)
fill_u32_kernel(uint32_t* __restrict__ dst, uint32_t v, long words, u64 wlo, u64 whi, uint32_t* whit) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
        dbg_watch(&dst[i], v == 0 ? 3 : 4, wlo, whi, whit);
        dst[i] = v;
    }
}

void launch_fill_u32(uint32_t* dst, uint32_t v, long words, hipStream_t s) {
    if (words <= 0) return;
    long blocks = (words + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    const DbgWatch w = watch_for(s);
    EXACTO_LAUNCH(fill_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, v, words, w.lo, w.hi, w.hit);
}

}  // namespace exacto
