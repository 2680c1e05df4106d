// Device pieces of the 31-bit key switch shared by ks32.hip and the fused CRT + forward NTT kernel
// in ntt.hip: 32-bit Shoup arithmetic, the 32-bit forward / inverse transform rounds (one residue
// polynomial per workgroup, n/16 threads x 16 coefficients, the round/LDS structure of ntt.hip) and
// the centred CRT lift of the key-switched sums.
#pragma once
#include "exacto_internal.hpp"

namespace exacto {

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

// One round: stage bits BHI..LO of the 4-bit window at LO.  Values < 2p between stages.
template <int LOGN, int LO, int BHI>
__device__ __forceinline__ void fwd32_round(uint32_t (&x)[16], int tid, const uint2* __restrict__ tw, uint32_t p) {
    constexpr int N = 1 << LOGN;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
#pragma unroll
    for (int b = BHI; b >= LO; --b) {
        const int lb = b - LO, half = 1 << lb;
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            const uint2 t = tw[base + g];
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m, k1 = k0 + half;
                const uint32_t X = red32(x[k0], p);
                const uint32_t T = red32(shoup32(x[k1], t.x, t.y, p), p);
                x[k0] = X + T;
                x[k1] = X + p - T;
            }
        }
    }
}

template <int LOGN, int R>
__device__ __forceinline__ void fwd32_rounds(uint32_t (&x)[16], uint32_t* lds, int tid, const uint2* tw, uint32_t p) {
    constexpr int LO = (LOGN - 4 * (R + 1)) > 0 ? (LOGN - 4 * (R + 1)) : 0;
    constexpr int BHI = LOGN - 1 - 4 * R;
    if constexpr (R > 0) {
        constexpr int PLO = (LOGN - 4 * R) > 0 ? (LOGN - 4 * R) : 0;
        lds_sync();
        lds32_store<PLO>(lds, x, tid);
        lds_sync();
        lds32_load<LO>(lds, x, tid);
    }
    fwd32_round<LOGN, LO, BHI>(x, tid, tw, p);
    if constexpr (LO > 0) fwd32_rounds<LOGN, R + 1>(x, lds, tid, tw, p);
}

// x (element tid + k T) -> NTT, stored coalesced at dst (element tid + k T of the
// bit-reversed-order evaluation array), as balanced residues in (-p/2, p/2] (int32 bits): the
// only consumer, ks32_mac_kernel, multiplies balanced values
template <int LOGN>
__device__ __forceinline__ void fwd32_store(uint32_t (&x)[16], uint32_t* lds, int tid, const Prime32& P,
                                            uint32_t* __restrict__ dst) {
    constexpr int T = (1 << LOGN) / 16;
    fwd32_rounds<LOGN, 0>(x, lds, tid, P.tw_fwd, P.p);
    const uint32_t half = P.p >> 1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = red32(x[k], P.p);
        x[k] = v > half ? v - P.p : v;
    }
    lds_sync();
    lds32_store<0>(lds, x, tid);
    lds_sync();
    lds32_load<LOGN - 4>(lds, x, tid);
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[tid + k * T] = x[k];
}

// ---------------------------------------------------------------- inverse (Gentleman-Sande)

template <int LOGN, int LO, int BLO, int BHI>
__device__ __forceinline__ void inv32_round(uint32_t (&x)[16], int tid, const Prime32& P) {
    constexpr int N = 1 << LOGN;
    const uint32_t p = P.p;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
#pragma unroll
    for (int b = BLO; b <= BHI; ++b) {
        const int lb = b - LO, half = 1 << lb;
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            uint2 t = make_uint2(0, 0);
            if (b != LOGN - 1) t = P.tw_inv[base + g];
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m, k1 = k0 + half;
                const uint32_t U = red32(x[k0], p), V = red32(x[k1], p);
                if (b == LOGN - 1) {  // n^-1 folded in, canonical
                    x[k0] = red32(shoup32(U + V, P.n_inv, P.n_inv_s, p), p);
                    x[k1] = red32(shoup32(U + p - V, P.last_w, P.last_ws, p), p);
                } else {
                    x[k0] = U + V;
                    x[k1] = shoup32(U + p - V, t.x, t.y, p);
                }
            }
        }
    }
}

template <int LOGN, int R>
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
    inv32_round<LOGN, LO, BLO, BHI>(x, tid, P);
    if constexpr (BHI < LOGN - 1) inv32_rounds<LOGN, R + 1>(x, lds, tid, P);
}

// Per (item, c, l) = block b: the S accumulated rows -> inverse NTT mod p_s -> centred Garner lift ->
// R[item][c][l] + lift mod q_l, returned in x (element k T + tid in x[k], canonical; R canonical,
// coefficient domain).  The lift mod q = 2^60 - d is a Horner evaluation x = a_0 + p_0 (a_1 + p_1
// (a_2 + ...)) whose every step folds the 92-bit product through 2^60 == d (5 instructions); the
// centring (x > floor(P/2)) is decided on the mixed-radix digits and adds q - (P mod q).
template <int LOGN, int S>
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
        const uint4* src = reinterpret_cast<const uint4*>(U + ((long)b * S + s) * N + 16 * tid);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint4 w = src[h];
            v[s][4 * h] = w.x; v[s][4 * h + 1] = w.y; v[s][4 * h + 2] = w.z; v[s][4 * h + 3] = w.w;
        }
        inv32_rounds<LOGN, 0>(v[s], lds, tid, primes[s]);
    }
    uint32_t pr[S], hp[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        pr[s] = primes[s].p;
        hp[s] = KT->halfP[s];
    }
    // element k*T + tid of every row is in v[s][k]
    const u64 q = qprimes[l].q;
    const uint32_t dq = (uint32_t)((1ull << 60) - q);
    const u64 negP = KT->negP[l];
    const u64* src = R + item * r_stride + (long)cl * N;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        // Garner over the p_s: a_s = (v_s - a_0 - a_1 p_0 - ...) / (p_0 ... p_{s-1}) mod p_s
        uint32_t a[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t ps = pr[s];
            uint32_t t = v[s][k];
#pragma unroll
            for (int kk = 0; kk < s; ++kk) {   // a_kk < p_kk < 2 p_s
                t = t + ps - red32(a[kk], ps);                       // (0, 2 p_s)
                t = red32(shoup32(t, KT->ginv[s][kk], KT->ginv_s[s][kk], ps), ps);
            }
            a[s] = t;
        }
        // centred: x > floor(P/2), on the mixed-radix digits, most significant first
        bool gt = false, eq = true;
#pragma unroll
        for (int s = S - 1; s >= 0; --s) {
            gt = gt || (eq && a[s] > hp[s]);
            eq = eq && a[s] == hp[s];
        }
        const bool neg = gt;
        // Horner mod q from the most significant digit; t < 2q between steps
        u64 t = a[S - 1];
#pragma unroll
        for (int s = S - 2; s >= 0; --s) {
            const u64 lo = (u64)(uint32_t)t * pr[s] + a[s];                      // < 2^63
            const u64 hi = (u64)(uint32_t)(t >> 32) * pr[s] + (lo >> 32);         // x = hi 2^32 + lo.lo
            const u64 l60 = ((hi & 0x0FFFFFFFull) << 32) | (uint32_t)lo;
            t = l60 + (hi >> 28) * dq;                                         // < 2^60 + 2^56
        }
        if (neg) t += negP;
        t += src[k * T + tid];
        x[k] = reduce_near60(t, q);                                                // t < 2^62
    }
}

}  // namespace exacto
