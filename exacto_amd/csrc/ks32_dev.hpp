// Device pieces of the 31-bit key switch shared by ks32.hip and the fused CRT + forward NTT kernel
// in ntt.hip: 32-bit Shoup arithmetic, the 32-bit forward / inverse transform rounds (one residue
// polynomial per workgroup, n/16 threads x 16 coefficients, the round/LDS structure of ntt.hip) and
// the centred CRT lift of the key-switched sums.
#pragma once
#include "exacto_internal.hpp"
#include "bufmem.hpp"

namespace exacto {

// Twiddles through the global address space: the generic pointers of Prime32 gave flat loads,
// which count against lgkmcnt, so every LDS barrier of a round also waited for the next twiddles
// (the same fix as ntt.hip's TwTab)
typedef const uint2 __attribute__((address_space(1)))* Tw32;
__device__ __forceinline__ Tw32 tw32(const uint2* p) { return (Tw32)p; }

// x * w mod p in [0, 2p) for any x < 2^32 (ws = floor(w 2^32 / p), p < 2^31)
__device__ __forceinline__ uint32_t shoup32(uint32_t x, uint32_t w, uint32_t ws, uint32_t p) {
    return x * w - __umulhi(x, ws) * p;
}

// [0, 2p) -> [0, p): x - p wraps above x when x < p
__device__ __forceinline__ uint32_t red32(uint32_t x, uint32_t p) { return min(x, x - p); }

__device__ __forceinline__ int swz32(int j) { return j ^ ((j >> 4) & 15) ^ (((j >> 8) & 1) << 4); }

template <int LO>
__device__ __forceinline__ int eidx(int tid, int k) {
    return ((tid >> LO) << (LO + 4)) | (k << LO) | (tid & ((1 << LO) - 1));
}

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The swizzle is linear over GF(2) and eidx<LO>(tid, k) = A(tid) ^ (k << LO) with disjoint bits, so
// every exchange address is one per-thread base XOR a compile-time constant (as ntt.hip's
// lds_store_x): one VALU per access instead of recomputing the swizzle of each index.
template <int LO>
__device__ __forceinline__ void lds32_store(uint32_t* lds, const uint32_t (&x)[16], int tid) {
    char* lb = reinterpret_cast<char*>(lds);
    const int b = swz32(eidx<LO>(tid, 0)) << 2;
#pragma unroll
    for (int k = 0; k < 16; ++k) *reinterpret_cast<uint32_t*>(lb + (b ^ (swz32(k << LO) << 2))) = x[k];
}

template <int LO>
__device__ __forceinline__ void lds32_load(const uint32_t* lds, uint32_t (&x)[16], int tid) {
    const char* lb = reinterpret_cast<const char*>(lds);
    const int b = swz32(eidx<LO>(tid, 0)) << 2;
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = *reinterpret_cast<const uint32_t*>(lb + (b ^ (swz32(k << LO) << 2)));
}

// ---------------------------------------------------------------- forward (Cooley-Tukey)

// 64-bit a * b + c by one v_mad_u64_u32 (callers use the low word: c's high word and the carry-out
// never reach it, so c may be a register pair whose high half is anything)
__device__ __forceinline__ u64 mad64(uint32_t a, uint32_t b, u64 c) {
    u64 r, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(c));
    return r;
}

// x as the low half of a 64-bit operand whose high half is left undefined (no zero-extension move)
__device__ __forceinline__ u64 lo_only(uint32_t x) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 v = __builtin_nondeterministic_value(v);
    v.x = x;
    return __builtin_bit_cast(u64, v);
}

// Prime ranges of a 31-bit basis, and the butterfly form each takes (a template parameter of the
// kernels, chosen on the host from the basis: Ks32Basis::mac_form uses the same numbering):
//   F32_LAZY   p < 2^30 (4p < 2^32): Harvey's lazy butterflies, values in [0, 4p) forward and
//              [0, 2p) inverse between stages, one conditional subtraction per butterfly;
//   F32_NARROW p < 2^32 / 3: values in [0, 3p] forward, both inverse inputs reduced to [0, p);
//   F32_WIDE   p < 2^31: values below 2p, every operand reduced to [0, p).
enum { F32_WIDE = 0, F32_NARROW = 1, F32_LAZY = 2 };

// One round: stage bits BHI..LO of the 4-bit window at LO.
// Narrow primes (3p < 2^32): values in [0, 3p] between stages.  X is brought to [0, p) (two
// min-subtractions), and X + T comes straight out of the Shoup chain: qh = hi(Y ws), then
// lo32(qh (2^32 - p) + (Y w + X)) by two v_mad_u64_u32 = X + T with T = Y w - qh p in [0, 2p), and
// the second output 2X + 2p - (X + T) = X + 2p - T: 3 multiplies and 7 simple ops per butterfly
// instead of 3 + 9 (the ~12 % cut of the digit transforms' VALU).
// Lazy primes (4p < 2^32): the same chain with values in [0, 4p) between stages, X brought to
// [0, 2p) by ONE min-subtraction (X + T < 4p, X + 2p - T < 4p): 3 multiplies and 5 simple ops.
// Wide primes (up to 2^31): values < 2p between stages, X and T reduced to [0, p) separately.
// CANON: the round's inputs are canonical (round 0: the caller's values are in [0, p)), so the first
// stage's X needs no reduction (8 butterflies x 4 VALU per thread less in the digit transforms).
// SIN (lazy primes, round 0 only): the inputs are int16 values x in [-2^15, 2^15) as int32 bits, not
// residues.  The first stage (one twiddle w, b = LOGN - 1) takes them as they are: Y + 2^15 >= 0 goes
// through the Shoup chain (T' = (Y + 2^15) w mod p, in [0, 2p)), and the constants K1 == -c, K2 == c
// with c = 2^15 w mod p, K1 in [2^15, p + 2^15), K2 in [2p + 2^15, 3p + 2^15), bring
//   X + T' + K1 == X + Y w  and  X - T' + K2 == X - Y w  into [0, 4p)
// (4 VALU per butterfly less than converting both inputs to canonical residues first).
template <int LOGN, int LO, int BHI, int FORM, bool CANON = false, bool SIN = false>
__device__ __forceinline__ void fwd32_round(uint32_t (&x)[16], int tid, Tw32 tw, uint32_t p) {
    constexpr int N = 1 << LOGN;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
    const uint32_t p2 = 2 * p, np = 0u - p;
    static_assert(!SIN || (FORM == F32_LAZY && CANON && BHI == LOGN - 1), "signed inputs: lazy round 0 only");
    if constexpr (SIN) {
        const uint2 t = make_uint2(tw[1].x, tw[1].y);
        const uint32_t c = red32(shoup32(1u << 15, t.x, t.y, p), p);
        const uint32_t k1 = (p - c) < (1u << 15) ? 2 * p - c : p - c;
        const uint32_t k2 = c < (1u << 15) ? c + 3 * p : c + p2;
        const uint32_t kd = k2 - k1;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t XK = x[m] + k1, Y = x[m + 8] + (1u << 15);
            const uint32_t qh = __umulhi(Y, t.y);
            const uint32_t o0 = (uint32_t)mad64(qh, np, mad64(Y, t.x, lo_only(XK)));
            // 2 XK + kd in one instruction (as C++, hipcc reassociates it into three)
            uint32_t x2;
            asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(x2) : "v"(XK), "v"(kd));
            x[m] = o0;                       // X + T' + K1
            x[m + 8] = x2 - o0;              // X - T' + K2
        }
    }
#pragma unroll
    for (int b = SIN ? BHI - 1 : BHI; b >= LO; --b) {
        const int lb = b - LO, half = 1 << lb;
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            const uint2 t = make_uint2(tw[base + g].x, tw[base + g].y);
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m, k1 = k0 + half;
                if constexpr (FORM != F32_WIDE) {
                    // narrow: [0, 3p] -> [0, p); lazy: [0, 4p) -> [0, 2p); canonical already in the
                    // first stage of a CANON round
                    const uint32_t X = (CANON && b == BHI) ? x[k0]
                                       : FORM == F32_LAZY ? min(x[k0], x[k0] - p2)
                                                          : red32(min(x[k0], x[k0] - p2), p);
                    const uint32_t qh = __umulhi(x[k1], t.y);
                    const uint32_t o0 = (uint32_t)mad64(qh, np, mad64(x[k1], t.x, lo_only(X)));
                    x[k0] = o0;                      // X + T (< 3p narrow, < 4p lazy)
                    x[k1] = 2 * X + p2 - o0;         // X + 2p - T (in (0, 3p] narrow, (0, 4p) lazy)
                } else {
                    const uint32_t X = red32(x[k0], p);
                    const uint32_t T = red32(shoup32(x[k1], t.x, t.y, p), p);
                    x[k0] = X + T;
                    x[k1] = X + p - T;
                }
            }
        }
    }
}

template <int LOGN, int R, int FORM, bool SIN = false>
__device__ __forceinline__ void fwd32_rounds(uint32_t (&x)[16], uint32_t* lds, int tid, Tw32 tw, uint32_t p) {
    constexpr int LO = (LOGN - 4 * (R + 1)) > 0 ? (LOGN - 4 * (R + 1)) : 0;
    constexpr int BHI = LOGN - 1 - 4 * R;
    if constexpr (R > 0) {
        constexpr int PLO = (LOGN - 4 * R) > 0 ? (LOGN - 4 * R) : 0;
        lds_sync();
        lds32_store<PLO>(lds, x, tid);
        lds_sync();
        lds32_load<LO>(lds, x, tid);
    }
    // round 0: canonical inputs (fwd32_store), or int16 values (SIN)
    fwd32_round<LOGN, LO, BHI, FORM, R == 0, SIN && R == 0>(x, tid, tw, p);
    if constexpr (LO > 0) fwd32_rounds<LOGN, R + 1, FORM>(x, lds, tid, tw, p);
}

// x (element tid + k T, canonical: round 0 relies on it) -> NTT, stored in ntt.hip's evaluation
// order (evaluation 16 tid + k at position tid + k T: coalesced, no LDS transpose), as balanced
// residues in (-p/2, p/2] (int32 bits): the only consumer, ks32_mac_kernel, multiplies balanced
// values position by position, and ks32_crt_values reads its sums in the same order
// BAL = false (the digit transforms under the lazy form): canonical [0, p) instead of balanced; with
// p < 2^30 and the key balanced (|r| <= p/2), a product stays below 2^59 and the MAC's runs of 12
// below 2^63 all the same (3 VALU per value less)
template <int LOGN, int FORM, bool SIN = false, bool BAL = true>
__device__ __forceinline__ void fwd32_store(uint32_t (&x)[16], uint32_t* lds, int tid, const Prime32& P,
                                            uint32_t* __restrict__ dst) {
    constexpr int T = (1 << LOGN) / 16;
    const uint32_t p = P.p, half = p >> 1;
    static_assert(BAL || FORM == F32_LAZY, "canonical digit residues: lazy primes only (MAC bound)");
    fwd32_rounds<LOGN, 0, FORM, SIN>(x, lds, tid, tw32(P.tw_fwd), p);
#pragma unroll
    for (int k = 0; k < 16; ++k)   // lazy [0, 4p) / narrow [0, 3p] / wide [0, 2p) -> [0, p)
        x[k] = FORM == F32_WIDE ? red32(x[k], p) : red32(min(x[k], x[k] - 2 * p), p);
    if constexpr (BAL) {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = x[k] > half ? x[k] - p : x[k];
    }
    const __amdgpu_buffer_rsrc_t rd = poly_rsrc(dst, T * 16 * 4);
#pragma unroll
    for (int k = 0; k < 16; ++k) buf_st32(rd, x[k], tid * 4, k * T * 4);   // evaluation 16 tid + k (ntt.hip store_evals)
}

// ---------------------------------------------------------------- inverse (Gentleman-Sande)

// Inputs below 2p.  Lazy primes (4p < 2^32): U + V < 4p is brought back below 2p by one
// min-subtraction and U + 2p - V < 4p goes to the Shoup product as is (9 VALU per butterfly);
// otherwise both inputs are first reduced to [0, p) (11 VALU).  Outputs below 2p, the last stage's
// canonical.
// OUT2P: the last stage's outputs stay in [0, 2p) (the Garner terms of ks32_lift_one for s >= 1 take
// them unreduced, the float-CRT lift all of them).  FOLD: the last stage multiplies by n^-1 pi
// instead of n^-1 (Prime32::fn_inv, the float-CRT lift's CRT factor).
template <int LOGN, int LO, int BLO, int BHI, bool LAZY, bool OUT2P = false, bool FOLD = false>
__device__ __forceinline__ void inv32_round(uint32_t (&x)[16], int tid, const Prime32& P) {
    constexpr int N = 1 << LOGN;
    const uint32_t p = P.p, p2 = 2 * p;
    const uint32_t ni = FOLD ? P.fn_inv : P.n_inv, nis = FOLD ? P.fn_inv_s : P.n_inv_s;
    const uint32_t lw = FOLD ? P.flast_w : P.last_w, lws = FOLD ? P.flast_ws : P.last_ws;
    const Tw32 twi = tw32(P.tw_inv);
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
#pragma unroll
    for (int b = BLO; b <= BHI; ++b) {
        const int lb = b - LO, half = 1 << lb;
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            uint2 t = make_uint2(0, 0);
            if (b != LOGN - 1) t = make_uint2(twi[base + g].x, twi[base + g].y);
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m, k1 = k0 + half;
                if constexpr (LAZY) {
                    const uint32_t U = x[k0], V = x[k1];
                    if (b == LOGN - 1) {  // n^-1 folded in, canonical (OUT2P: below 2p)
                        x[k0] = shoup32(U + V, ni, nis, p);
                        x[k1] = shoup32(U + p2 - V, lw, lws, p);
                        if constexpr (!OUT2P) {
                            x[k0] = red32(x[k0], p);
                            x[k1] = red32(x[k1], p);
                        }
                    } else {
                        const uint32_t sum = U + V;
                        x[k0] = min(sum, sum - p2);
                        x[k1] = shoup32(U + p2 - V, t.x, t.y, p);
                    }
                } else {
                    const uint32_t U = red32(x[k0], p), V = red32(x[k1], p);
                    if (b == LOGN - 1) {  // n^-1 folded in, canonical (OUT2P: below 2p)
                        x[k0] = shoup32(U + V, ni, nis, p);
                        x[k1] = shoup32(U + p - V, lw, lws, p);
                        if constexpr (!OUT2P) {
                            x[k0] = red32(x[k0], p);
                            x[k1] = red32(x[k1], p);
                        }
                    } else {
                        x[k0] = U + V;
                        x[k1] = shoup32(U + p - V, t.x, t.y, p);
                    }
                }
            }
        }
    }
}

template <int LOGN, int R, bool LAZY, bool OUT2P = false, bool FOLD = false>
__device__ __forceinline__ void inv32_rounds(uint32_t (&x)[16], uint32_t* lds, int tid, const Prime32& P) {
    constexpr int LO = (4 * R) < (LOGN - 4) ? 4 * R : LOGN - 4;
    constexpr int BLO = 4 * R;
    constexpr int BHI = (4 * R + 3) < (LOGN - 1) ? 4 * R + 3 : LOGN - 1;
    if constexpr (R > 0) {
        constexpr int PLO = (4 * (R - 1)) < (LOGN - 4) ? 4 * (R - 1) : LOGN - 4;
        lds_sync();
        lds32_store<PLO>(lds, x, tid);
        lds_sync();
        lds32_load<LO>(lds, x, tid);
    }
    inv32_round<LOGN, LO, BLO, BHI, LAZY, OUT2P, FOLD>(x, tid, P);
    if constexpr (BHI < LOGN - 1) inv32_rounds<LOGN, R + 1, LAZY, OUT2P, FOLD>(x, lds, tid, P);
}

// One coefficient's centred Garner lift of its S residues v[s] (canonical mod p_s) evaluated mod
// q_l = 2^60 - dq, plus r (canonical mod q_l): the result canonical.  The lift mod q is a Horner
// evaluation x = a_0 + p_0 (a_1 + p_1 (a_2 + ...)) whose every step folds the 92-bit product through
// 2^60 == d (5 instructions); the centring (x > floor(P/2)) is decided on the mixed-radix digits and
// adds q - (P mod q).
// LAZY (every p_s below 2^30): a_kk < p_kk < 2 p_s enters t + 2 p_s - a_kk < 4 p_s < 2^32 unreduced
// (the Shoup product takes any 32-bit input): one min-subtraction less per Garner term; v[s] for
// s >= 1 may then be anywhere in [0, 2 p_s) (the inverse transforms' OUT2P form).
template <int S, bool LAZY = false>
__device__ __forceinline__ u64 ks32_lift_one(const uint32_t (&v)[S], u64 r, const uint32_t (&pr)[S],
                                             const uint32_t (&hp)[S], const Ks32Tables* __restrict__ KT, u64 q,
                                             uint32_t dq, u64 negP) {
    uint32_t a[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const uint32_t ps = pr[s];
        uint32_t t = v[s];
#pragma unroll
        for (int kk = 0; kk < s; ++kk) {   // a_kk < p_kk < 2 p_s
            t = LAZY ? t + 2 * ps - a[kk]                        // (0, 4 p_s)
                     : t + ps - red32(a[kk], ps);                // (0, 2 p_s)
            t = red32(shoup32(t, KT->ginv[s][kk], KT->ginv_s[s][kk], ps), ps);
        }
        a[s] = t;
    }
    bool gt = false, eq = true;
#pragma unroll
    for (int s = S - 1; s >= 0; --s) {
        gt = gt || (eq && a[s] > hp[s]);
        eq = eq && a[s] == hp[s];
    }
    u64 t = a[S - 1];
#pragma unroll
    for (int s = S - 2; s >= 0; --s) {
        const u64 lo = (u64)(uint32_t)t * pr[s] + a[s];                      // < 2^63
        const u64 hi = (u64)(uint32_t)(t >> 32) * pr[s] + (lo >> 32);         // x = hi 2^32 + lo.lo
        const u64 l60 = ((hi & 0x0FFFFFFFull) << 32) | (uint32_t)lo;
        t = l60 + (hi >> 28) * dq;                                         // < 2^60 + 2^56
    }
    if (gt) t += negP;
    return reduce_near60(t + r, q);                                        // t + r < 2^62
}

// The same lift by a rounded float sum (S <= 3, or S = 4 below 2^32 / 3).  y_s = u pi_s mod p_s, below 2 p_s (the inverse
// transforms' FOLD + OUT2P form, pi_s = (P / p_s)^-1 mod p_s), so sum_s y_s (P / p_s) = u_c + alpha P
// with u_c the centred residue and alpha = round(sum_s y_s / p_s) in [0, 2S]: the float sum of the
// y_s fl(1 / p_s) is within 2^-48 of the exact one and |u_c| / P < 1/2 - 2^-21 (the host's margin:
// the basis' fpc_max), so the rounding is exact.  Mod q = 2^60 - d:
//   sum_s y_s C_s + alpha negP, C_s = (P / p_s) mod q, negP = q - P mod q,
// with C_s and negP in 30-bit halves: A0 = sum y_s C_s,lo + alpha negP_lo < S 2 p_max 2^30 + 2^33
// (< 3 2^62 at S = 3, p < 2^31; < 2^63.42 at S = 4, p < 2^32 / 3), A1 likewise, value = A0 + A1 2^30,
// A1 2^30 = (A1 mod 2^30) 2^30 + (A1 >> 30) 2^60 and 2^60 == d.
// 8 multiply-adds for the products against the Garner form's 3 Shoup products, mixed-radix compare
// and 2 Horner folds.
template <int S>
__device__ __forceinline__ u64 ks32_fpc_one(const uint32_t (&y)[S], u64 r, const double (&ip)[S],
                                            const uint32_t (&c0)[S], const uint32_t (&c1)[S], uint32_t n0,
                                            uint32_t n1, u64 q, uint32_t dq) {
    static_assert(S <= 4, "A0, A1 < 2^64: S <= 3, or S = 4 with p < 2^32 / 3 (ks32_crt)");
    double f = (double)y[0] * ip[0];
#pragma unroll
    for (int s = 1; s < S; ++s) f = __builtin_fma((double)y[s], ip[s], f);
    const uint32_t al = (uint32_t)__builtin_rint(f);
    u64 a0 = (u64)al * n0, a1 = (u64)al * n1;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        a0 += (u64)y[s] * c0[s];
        a1 += (u64)y[s] * c1[s];
    }
    const u64 h = a1 >> 30;                                               // < 2^34
    const u64 l30 = (a1 & ((1ull << 30) - 1)) << 30;                      // < 2^60
    const u64 t = a0 + l30 + (u64)(uint32_t)h * dq + ((u64)((uint32_t)(h >> 32) * dq) << 32);  // < 2^63.72
    return reduce_near60(t + r, q);                                       // t + r < 2^63.83 (S = 4: 2^63.55)
}

// Per (item, c, l) = block b: the S accumulated rows -> inverse NTT mod p_s -> centred Garner lift ->
// R[item][c][l] + lift mod q_l, returned in x (element k T + tid in x[k], canonical; R canonical,
// coefficient domain).  The lift mod q = 2^60 - d is a Horner evaluation x = a_0 + p_0 (a_1 + p_1
// (a_2 + ...)) whose every step folds the 92-bit product through 2^60 == d (5 instructions); the
// centring (x > floor(P/2)) is decided on the mixed-radix digits and adds q - (P mod q).
// FPC: ks32_fpc_one instead.
template <int LOGN, int S, bool LAZY, bool FPC = false>
__device__ __forceinline__ void ks32_crt_values(u64 (&x)[16], const uint32_t* __restrict__ U, const u64* __restrict__ R,
                                                long r_stride, int L, uint32_t b, uint32_t* lds, int tid,
                                                const Ks32Tables* __restrict__ KT, const Prime32* __restrict__ primes,
                                                const PrimeConst* __restrict__ qprimes) {
    constexpr int N = 1 << LOGN, T = N / 16;
    const uint32_t CL = 2 * L;
    const long item = b / CL;
    const int cl = (int)(b - (uint32_t)item * CL);
    const int l = cl % L;
    uint32_t v[S][16];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        // evaluation 16 tid + k at tid + k T
        const __amdgpu_buffer_rsrc_t rs = poly_rsrc(U + ((long)b * S + s) * N, N * 4);
#pragma unroll
        for (int k = 0; k < 16; ++k) v[s][k] = buf_ld32(rs, tid * 4, k * T * 4);
        // s >= 1 (lazy): residues in [0, 2p), which the Garner terms take as they are; the float-CRT
        // lift takes every residue below 2p, its CRT factor folded into the last stage
        if constexpr (FPC) inv32_rounds<LOGN, 0, LAZY, true, true>(v[s], lds, tid, primes[s]);
        else if (s == 0) inv32_rounds<LOGN, 0, LAZY>(v[s], lds, tid, primes[s]);
        else inv32_rounds<LOGN, 0, LAZY, LAZY>(v[s], lds, tid, primes[s]);
    }
    // element k*T + tid of every row is in v[s][k]
    const u64 q = qprimes[l].q;
    const uint32_t dq = (uint32_t)((1ull << 60) - q);
    const __amdgpu_buffer_rsrc_t rr = poly_rsrc(R + item * r_stride + (long)cl * N, N * 8);
    if constexpr (FPC) {
        // the residues pass through an empty asm here, so the float sum's conversions are not hoisted
        // into the later primes' transforms (16 doubles live per prime: 151 VGPRs, 3 waves per SIMD)
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(v[s][k]));
        double ip[S];
        uint32_t c0[S], c1[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            ip[s] = primes[s].inv_p;
            c0[s] = KT->fpc_c[l][s][0];
            c1[s] = KT->fpc_c[l][s][1];
        }
        const uint32_t n0 = KT->fpc_n[l][0], n1 = KT->fpc_n[l][1];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t vk[S];
#pragma unroll
            for (int s = 0; s < S; ++s) vk[s] = v[s][k];
            x[k] = ks32_fpc_one<S>(vk, buf_ld64(rr, tid * 8, k * T * 8), ip, c0, c1, n0, n1, q, dq);
        }
        return;
    }
    uint32_t pr[S], hp[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        pr[s] = primes[s].p;
        hp[s] = KT->halfP[s];
    }
    const u64 negP = KT->negP[l];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        uint32_t vk[S];
#pragma unroll
        for (int s = 0; s < S; ++s) vk[s] = v[s][k];
        x[k] = ks32_lift_one<S, LAZY>(vk, buf_ld64(rr, tid * 8, k * T * 8), pr, hp, KT, q, dq, negP);
    }
}

}  // namespace exacto
