// Relinearisation key switching over the integers in an auxiliary basis of 31-bit primes.
//
// relinearize (reference src/bfv/keyswitch.rs:86-95) adds sum_g NTT_l(d_g) (.) rlk_{g,c,l} to the
// scaled components, limb by limb.  By the negacyclic convolution theorem that is
// NTT_l(sum_g d_g * r_{g,c,l} mod q_l) with r = INTT_l(rlk) the key in the coefficient domain.  The
// digits d_g are small integers (|d| <= B/2) and the same for every limb, so the integer
// polynomial u_{c,l} = sum_g d_g * r_{g,c,l} (r balanced, |r| < q_l / 2) has coefficients below
// G n (B/2) (q/2) in magnitude: for cfg3 below 2^90, for cfg5 below 2^84.  It is computed exactly
// modulo S 31-bit primes p_s with prod p_s > 2 |u|max (S = 3 for every BASELINE config), then
// lifted (Garner, centred) and reduced mod q_l.  Bit-identical with the limb-wise MAC by
// construction; the work moves from G L 60-bit digit NTTs to G S 32-bit ones (no carry chains:
// a 32-bit butterfly is three multiplies) plus 2 L S 32-bit inverse transforms.
//
// Kernels (all one residue polynomial per workgroup, n/16 threads x 16 coefficients, the same
// round/LDS structure as ntt.hip):
//   ks32_digit_ntt_kernel : int16 digits [item][g][n] -> DS [item][g][s][n], forward NTT mod p_s
//   ks32_key_kernel        : coefficient-domain key rows (canonical mod q_l) -> balanced -> mod p_s,
//                            forward NTT -> RS [g][c][l][s][n] (once per key)
//   ks32_mac_kernel        : U [item][c][l][s] = sum_g DS [item][g][s] (.) RS [g][c][l][s] mod p_s,
//                            key slice staged in LDS, 64-bit lazy accumulation
//   ks32_crt_kernel        : per (item, c, l): S inverse NTTs, centred Garner or float-CRT lift, + R[item][c][l]
//                            mod q_l, written back into R (coefficient domain)
#include "exacto_internal.hpp"
#include "ks32_dev.hpp"

#include <algorithm>

namespace exacto {

// ---------------------------------------------------------------- kernels

// digits [item][g][n] (int16, or int32 for dBFV digit sums beyond int16) -> DS [item][g][s][n]
template <int LOGN, typename DT, int FORM>
__global__ void __launch_bounds__((1 << LOGN) / 16)
ks32_digit_ntt_kernel(const DT* __restrict__ D16, uint32_t* __restrict__ DS, int G, int S,
                      const Prime32* __restrict__ primes) {
    constexpr int N = 1 << LOGN, T = N / 16;
    __shared__ uint32_t lds[N];
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;             // (item, g, s)
    const int s = (int)(b % (uint32_t)S);
    const long ig = b / (uint32_t)S;           // item * G + g
    const Prime32& P = primes[s];
    const DT* src = D16 + ig * N;
    uint32_t x[16];
    // int16 digits under the lazy form: the transform's first stage takes the signed values as they
    // are (fwd32_round SIN); otherwise they become canonical residues first
    constexpr bool SIN = FORM == F32_LAZY && sizeof(DT) == 2;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int d = src[tid + k * T];
        x[k] = SIN ? (uint32_t)d : d < 0 ? P.p + (uint32_t)d : (uint32_t)d;
    }
    fwd32_store<LOGN, FORM, SIN, FORM != F32_LAZY>(x, lds, tid, P, DS + (long)b * N);
}

// key rows [rows][n] canonical mod q_{row's limb} (u64) -> RS [rows][S][n]: balanced, mod p_s, NTT
template <int LOGN, int FORM>
__global__ void __launch_bounds__((1 << LOGN) / 16)
ks32_key_kernel(const u64* __restrict__ K, uint32_t* __restrict__ RS, int L, int S,
                const Prime32* __restrict__ primes, const PrimeConst* __restrict__ qprimes) {
    constexpr int N = 1 << LOGN, T = N / 16;
    __shared__ uint32_t lds[N];
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;             // (row, s), row = (g * 2 + c) * L + l
    const int s = (int)(b % (uint32_t)S);
    const uint32_t row = b / (uint32_t)S;
    const int l = (int)(row % (uint32_t)L);
    const Prime32& P = primes[s];
    const u64 q = qprimes[l].q, half = q >> 1;
    const u64* src = K + (long)row * N;
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const u64 r = src[tid + k * T];
        // balanced representative r - q (r > q/2) as a residue mod p
        if (r > half) {
            const uint32_t m = (uint32_t)((q - r) % P.p);
            x[k] = m == 0 ? 0 : P.p - m;
        } else {
            x[k] = (uint32_t)(r % P.p);
        }
    }
    fwd32_store<LOGN, FORM>(x, lds, tid, P, RS + (long)b * N);
}

// Per key row [rows][n] (coefficient domain, canonical mod q_{row's limb}): sum_j floor(|r_j| / 2^20)
// of its balanced coefficients, so that (sum + n) 2^20 bounds the row's L1 norm (each term < 2^39,
// the sum < 2^53: exact in u64).  One block per row; the lazy basis is chosen from these (ensure_rs).
__global__ void __launch_bounds__(256)
ks32_key_norm_kernel(const u64* __restrict__ K, u64* __restrict__ out, int L, int n,
                     const PrimeConst* __restrict__ qprimes) {
    __shared__ u64 part[256];
    const uint32_t row = blockIdx.x;
    const u64 q = qprimes[row % (uint32_t)L].q, half = q >> 1;
    const u64* src = K + (long)row * n;
    u64 acc = 0;
    for (int j = threadIdx.x; j < n; j += 256) {
        const u64 r = src[j];
        acc += (r > half ? q - r : r) >> 20;
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[row] = part[0];
}

// Signed 64-bit x -> x mod p, canonical (p in (2^30, 2^31)): x = hi 2^32 + lo with hi signed;
// (hi + 2^31) 2^32 by Shoup with 2^32 mod p, lo by two halvings, -2^63 by the constant k63.
__device__ __forceinline__ uint32_t red_s64(long long x, const Prime32& P) {
    const uint32_t p = P.p;
    const uint32_t hu = (uint32_t)((unsigned long long)x >> 32) ^ 0x80000000u;
    const uint32_t a = red32(shoup32(hu, P.c32, P.c32s, p), p);
    const uint32_t b = red32(red32((uint32_t)x, 2 * p), p);
    return red32(red32(a + b, p) + P.k63, p);        // every partial sum < 2p < 2^32
}

// Signed 64-bit x (|x| < 2^63) -> a small non-negative value == x mod p, below 3p + 2^32 < 2^33.6:
// (hi + 2^31) 2^32 by Shoup with 2^32 mod p, plus lo, plus (-2^63) mod p.  Carried between runs
// of signed products (7 VALU instead of red_s64's full reduction).
// Lazy basis (7/8 2^30 < p < 2^30): x mod p in [0, 2p), the lazy inverse transform's input range.
// The low word goes below 2p by lo - floor(lo / 2^30) p (< 2^30 + 3 (2^30 - p) < 2p for p > 0.8 2^30),
// so a + b + k63 < 4p < 2^32 needs one min-subtraction (13 VALU instead of red_s64's 17).
__device__ __forceinline__ uint32_t red_s64_lz(long long x, const Prime32& P) {
    const uint32_t p = P.p;
    const uint32_t hu = (uint32_t)((unsigned long long)x >> 32) ^ 0x80000000u;
    const uint32_t a = red32(shoup32(hu, P.c32, P.c32s, p), p);
    const uint32_t lo = (uint32_t)x;
    const uint32_t b = lo - (lo >> 30) * p;
    const uint32_t s = a + b + P.k63;
    return min(s, s - 2 * p);
}

__device__ __forceinline__ long long red_s64_lazy(long long x, const Prime32& P) {
    const uint32_t hu = (uint32_t)((unsigned long long)x >> 32) ^ 0x80000000u;
    const uint32_t a = shoup32(hu, P.c32, P.c32s, P.p);
    return (long long)((unsigned long long)a + (uint32_t)x + P.k63);
}

// U[item][cl][s][j] = sum_g DS[item][g][s][j] * RS[g][cl][s][j] mod p_s   (cl = c * L + l)
// Block: 64 coefficients j of one prime s, CLB consecutive (c, l) pairs starting at cl0, and up to
// 4 NW items; its key words (G * CLB * 64, balanced) are staged in LDS once.  Lane = coefficient,
// wave w handles items it0 + w, it0 + w + NW, ...  The key is stored balanced by its transform, the
// digit residues balanced too except under the lazy form (canonical, < p < 2^30: |product| <
// 2^30 2^29 = 2^59 still), so the run's signed products plus the carried value (< 2^33.6) stay
// below 2^63 (one v_mad_i64_i32 each) before a lazy reduction.
constexpr int KS_LS = 64;
// RUN: signed products summed between reductions: 12 for primes below 2^32 / 3 (balanced products
// below 2^58.9; lazy basis: below 2^59), 7 for primes up to 2^31 (products below 2^60;
// 7 * 2^60 + 2^33.6 < 2^63)
// LZ: lazy basis (p < 2^30), sums written in [0, 2p) (red_s64_lz) for the lazy inverse transforms
template <int CLB, int NW, int RUN, bool LZ = false>
__global__ void __launch_bounds__(NW * 64)
ks32_mac_kernel(const int* __restrict__ DS, const int* __restrict__ RS, uint32_t* __restrict__ U,
                int G, int CL, int S, int items, int n, const Prime32* __restrict__ primes) {
    extern __shared__ int kl[];                // [g][cl - cl0][lane]
    constexpr int IG = 4 * NW;                 // items per block
    const int lane = threadIdx.x & (KS_LS - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / KS_LS);   // uniform: item math on the SALU
    const int nb = n / KS_LS;
    const int jb = blockIdx.x % nb;
    const int s = (blockIdx.x / nb) % S;
    const int cl0 = (blockIdx.x / (nb * S)) * CLB;
    const int j = jb * KS_LS + lane;
    const Prime32& P = primes[s];
    // key slice rows rr = g CLB + c, one per wave at a time (rr wave-uniform: the row index math runs
    // on the SALU; a flat index r / (CLB 64) per element cost ~20 VALU per word staged)
    for (int rr = wave; rr < G * CLB; rr += NW) {
        const int g = rr / CLB, c = rr - g * CLB;
        kl[rr * KS_LS + lane] = RS[(((long)g * CL + cl0 + c) * S + s) * n + jb * KS_LS + lane];
    }
    __syncthreads();
    const int it_end = min(items, (int)(blockIdx.y + 1) * IG);
    for (int it = blockIdx.y * IG + wave; it < it_end; it += NW) {
        const int* dp = DS + ((long)it * G * S + s) * n + j;
        long long acc[CLB];
#pragma unroll
        for (int c = 0; c < CLB; ++c) acc[c] = 0;
        for (int g0 = 0; g0 < G; g0 += RUN) {
            // unconditional (clamped) loads, all in flight together; digits past G are zeroed after
            int d[RUN];
#pragma unroll
            for (int e = 0; e < RUN; ++e) d[e] = dp[(long)min(g0 + e, G - 1) * S * n];
#pragma unroll
            for (int e = 0; e < RUN; ++e) d[e] = g0 + e < G ? d[e] : 0;
#pragma unroll
            for (int e = 0; e < RUN; ++e) {
                const int* kg = kl + (min(g0 + e, G - 1) * CLB) * KS_LS + lane;
#pragma unroll
                for (int c = 0; c < CLB; ++c) acc[c] += (long long)d[e] * kg[c * KS_LS];
            }
            if (g0 + RUN < G) {
#pragma unroll
                for (int c = 0; c < CLB; ++c) acc[c] = red_s64_lazy(acc[c], P);
            }
        }
#pragma unroll
        for (int c = 0; c < CLB; ++c)
            U[(((long)it * CL + cl0 + c) * S + s) * n + j] = LZ ? red_s64_lz(acc[c], P) : red_s64(acc[c], P);
    }
}

template <int LOGN, int S, bool LAZY, bool FPC>
__global__ void __launch_bounds__((1 << LOGN) / 16)
ks32_crt_kernel(const uint32_t* __restrict__ U, u64* __restrict__ R, long r_stride, int L,
                const Ks32Tables* __restrict__ KT, const Prime32* __restrict__ primes,
                const PrimeConst* __restrict__ qprimes) {
    constexpr int N = 1 << LOGN, T = N / 16;
    __shared__ uint32_t lds[N];
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;             // (item, cl)
    u64 x[16];
    ks32_crt_values<LOGN, S, LAZY, FPC>(x, U, R, r_stride, L, b, lds, tid, KT, primes, qprimes);
    const uint32_t CL = 2 * L;
    const long item = b / CL;
    const __amdgpu_buffer_rsrc_t rd = poly_rsrc(R + item * r_stride + (long)(b - (uint32_t)item * CL) * N, N * 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) buf_st64(rd, x[k], tid * 8, k * T * 8);
}

// dBFV: the gadget digits of the products of one output limb k summed before their transforms.
// Every step after the digits (NTT mod p_s, MAC with the key, lift) is linear in them, so the sum
// of the products' key switches is the key switch of the summed digits (an integer identity; the
// basis bound covers the sum, see setup_ks32).  D [item][pair][g][n] -> out [item][k][g][n].
template <typename OT, typename IT>
__global__ void __launch_bounds__(256)
ks32_digit_sum_kernel(const IT* __restrict__ D, int npairs, const int* __restrict__ term_start,
                      const CombineTerm* __restrict__ terms, OT* __restrict__ out, int d, int gu, int n,
                      int nsh) {
    // eight consecutive digits per thread (one 16-byte load per term), 2048 per block
    const uint32_t row = blockIdx.x >> nsh;              // (item * d + k) * gu + g
    const int j = (int)(blockIdx.x & ((1u << nsh) - 1)) * 2048 + 8 * threadIdx.x;
    const uint32_t g = row % (uint32_t)gu;
    const uint32_t ik = row / (uint32_t)gu;
    const int k = (int)(ik % (uint32_t)d);
    const long item = ik / (uint32_t)d;
    int acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
        const IT* src = D + ((item * npairs + terms[t].pair) * gu + g) * (long)n + j;
        if constexpr (sizeof(IT) == 2) {   // one 16-byte load
            const uint4 w = *reinterpret_cast<const uint4*>(src);
            const uint32_t v[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                acc[2 * h] += (int)(int16_t)(v[h] & 0xFFFF);
                acc[2 * h + 1] += (int)(int16_t)(v[h] >> 16);
            }
        } else {                           // int8: one 8-byte load
            const uint2 w = *reinterpret_cast<const uint2*>(src);
            const uint32_t v[2] = {w.x, w.y};
#pragma unroll
            for (int h = 0; h < 8; ++h) acc[h] += (int)(int8_t)(v[h >> 2] >> (8 * (h & 3)));
        }
    }
    if constexpr (sizeof(OT) == 2) {
        uint4 o;
        uint32_t* op = &o.x;
#pragma unroll
        for (int h = 0; h < 4; ++h) op[h] = ((uint32_t)acc[2 * h] & 0xFFFF) | ((uint32_t)acc[2 * h + 1] << 16);
        *reinterpret_cast<uint4*>(out + (long)row * n + j) = o;
    } else {
        int4* o4 = reinterpret_cast<int4*>(out + (long)row * n + j);
        o4[0] = make_int4(acc[0], acc[1], acc[2], acc[3]);
        o4[1] = make_int4(acc[4], acc[5], acc[6], acc[7]);
    }
}

// ---------------------------------------------------------------- launchers

// form: the basis' butterfly form (F32_WIDE / F32_NARROW / F32_LAZY = Ks32Basis::mac_form), a
// template parameter of every kernel (a runtime branch kept the union of both forms' registers)
#define FORM_SWITCH(form, CALL)                          \
    switch (form) {                                      \
        case F32_LAZY: CALL(F32_LAZY); break;            \
        case F32_NARROW: CALL(F32_NARROW); break;        \
        default: CALL(F32_WIDE); break;                  \
    }

template <int LOGN>
static void ks32_launch_digits(const void* D, bool wide, uint32_t* DS, int items, int G, int S, const Prime32* primes,
                               int form, hipStream_t st) {
    const dim3 grid((unsigned)((long)items * G * S)), block((1 << LOGN) / 16);
#define DIG_(F_)                                                                                                \
    do {                                                                                                        \
        if (wide)                                                                                               \
            EXACTO_LAUNCH((ks32_digit_ntt_kernel<LOGN, int32_t, F_>), grid, block, 0, st, (const int32_t*)D, \
                               DS, G, S, primes);                                                               \
        else                                                                                                    \
            EXACTO_LAUNCH((ks32_digit_ntt_kernel<LOGN, int16_t, F_>), grid, block, 0, st, (const int16_t*)D, \
                               DS, G, S, primes);                                                               \
    } while (0)
    FORM_SWITCH(form, DIG_)
#undef DIG_
}

template <int LOGN>
static void ks32_launch_key(const u64* K, uint32_t* RS, long rows, int L, int S, const Prime32* primes,
                            const PrimeConst* qprimes, int form, hipStream_t st) {
#define KEY_(F_) EXACTO_LAUNCH((ks32_key_kernel<LOGN, F_>), dim3((unsigned)(rows * S)), dim3((1 << LOGN) / 16), 0, \
                                    st, K, RS, L, S, primes, qprimes)
    FORM_SWITCH(form, KEY_)
#undef KEY_
}

template <int LOGN, bool LAZY>
static void ks32_launch_crt(const uint32_t* U, u64* R, long r_stride, int items, int L, int S, const Ks32Tables* KT,
                            const Prime32* primes, const PrimeConst* qprimes, hipStream_t st, bool fpc) {
    const dim3 grid((unsigned)((long)items * 2 * L)), block((1 << LOGN) / 16);
#define CRT_(S_, F_) EXACTO_LAUNCH((ks32_crt_kernel<LOGN, S_, LAZY, F_>), grid, block, 0, st, U, R, r_stride, L, KT, \
                                   primes, qprimes)
    if (S == 2) {
        if (fpc) CRT_(2, true); else CRT_(2, false);
    } else if (S == 3) {
        if (fpc) CRT_(3, true); else CRT_(3, false);
    } else {
        if (fpc) CRT_(4, true); else CRT_(4, false);
    }
#undef CRT_
}

#define KS32_SWITCH(logn, CALL)                  \
    switch (logn) {                              \
        case 10: CALL(10); break;                \
        case 11: CALL(11); break;                \
        case 12: CALL(12); break;                \
        case 13: CALL(13); break;                \
        case 14: CALL(14); break;                \
        default: break;                          \
    }

void ks32_digits(const int16_t* D16, uint32_t* DS, int items, int G, int S, int logn, const Prime32* primes, int form,
                 hipStream_t st) {
    if (items <= 0) return;
#define CALL(L_) ks32_launch_digits<L_>(D16, false, DS, items, G, S, primes, form, st)
    KS32_SWITCH(logn, CALL)
#undef CALL
}

void ks32_digits32(const int32_t* D, uint32_t* DS, int items, int G, int S, int logn, const Prime32* primes, int form,
                   hipStream_t st) {
    if (items <= 0) return;
#define CALL(L_) ks32_launch_digits<L_>(D, true, DS, items, G, S, primes, form, st)
    KS32_SWITCH(logn, CALL)
#undef CALL
}

void ks32_key(const u64* K, uint32_t* RS, long rows, int L, int S, int logn, const Prime32* primes,
              const PrimeConst* qprimes, int form, hipStream_t st) {
    if (rows <= 0) return;
#define CALL(L_) ks32_launch_key<L_>(K, RS, rows, L, S, primes, qprimes, form, st)
    KS32_SWITCH(logn, CALL)
#undef CALL
}

void ks32_key_norms(const u64* K, u64* out, long rows, int L, int n, const PrimeConst* qprimes, hipStream_t st) {
    if (rows <= 0) return;
    EXACTO_LAUNCH(ks32_key_norm_kernel, dim3((unsigned)rows), dim3(256), 0, st, K, out, L, n, qprimes);
}

void ks32_mac(const uint32_t* DS, const uint32_t* RS, uint32_t* U, int items, int G, int L, int S, int n,
              const Prime32* primes, int mac_form, hipStream_t st) {
    if (items <= 0) return;
    const int CL = 2 * L;
    // (c, l) pairs per block: the largest divisor of 2L whose key slice (G * CLB * 64 words) fits
    // 64 KiB of LDS, so the digits are read once per pair group (once at every BASELINE config);
    // a slice above 32 KiB leaves room for 2 blocks per CU, which then get 8 waves each
    int CLB = CL;
    while (CLB > 1 && (CL % CLB != 0 || (size_t)G * CLB * KS_LS * sizeof(int) > 65536)) --CLB;
    const size_t lds = (size_t)G * CLB * KS_LS * sizeof(int);
    const int NW = lds > 32768 ? 8 : 4;
    const dim3 grid((unsigned)((n / KS_LS) * S * (CL / CLB)), (unsigned)((items + 4 * NW - 1) / (4 * NW)));
    const int* ds = reinterpret_cast<const int*>(DS);
    const int* rs = reinterpret_cast<const int*>(RS);
// mac_form: 0 primes up to 2^31 (7 products per reduction), 1 below 2^32 / 3 (12), 2 below 2^30
// (12, lazy output)
#define MAC_(C_, W_, R_, Z_) EXACTO_LAUNCH((ks32_mac_kernel<C_, W_, R_, Z_>), grid, dim3(W_ * 64), lds, st, ds, rs, U, G, CL, S, items, n, primes)
#define MAC(C_)                                                  \
    do {                                                         \
        if (mac_form == 2) { if (NW == 8) MAC_(C_, 8, 12, true); else MAC_(C_, 4, 12, true); } \
        else if (mac_form == 1) { if (NW == 8) MAC_(C_, 8, 12, false); else MAC_(C_, 4, 12, false); } \
        else { if (NW == 8) MAC_(C_, 8, 7, false); else MAC_(C_, 4, 7, false); }          \
    } while (0)
    switch (CLB) {
        case 8: MAC(8); break;
        case 6: MAC(6); break;
        case 4: MAC(4); break;
        case 3: MAC(3); break;
        case 2: MAC(2); break;
        default: MAC(1); break;
    }
#undef MAC
#undef MAC_
}

void ks32_digit_sum(const void* D, bool in8, int npairs, const int* term_start, const CombineTerm* terms, void* out,
                    bool wide, int items, int d, int gu, int n, hipStream_t st) {
    const long rows = (long)items * d * gu;
    if (rows <= 0) return;
    const int nb = n >= 2048 ? n / 2048 : 1;   // n >= 1024, a power of two; 2048 digits per block
    const dim3 grid((unsigned)(rows * nb)), block(n >= 2048 ? 256 : n / 8);
    const int nsh = __builtin_ctz((unsigned)nb);
#define DSUM_(OT, IT) EXACTO_LAUNCH((ks32_digit_sum_kernel<OT, IT>), grid, block, 0, st, (const IT*)D, npairs, \
                                         term_start, terms, (OT*)out, d, gu, n, nsh)
    if (wide) {
        if (in8) DSUM_(int32_t, int8_t); else DSUM_(int32_t, int16_t);
    } else {
        if (in8) DSUM_(int16_t, int8_t); else DSUM_(int16_t, int16_t);
    }
#undef DSUM_
}

void ks32_crt(const uint32_t* U, u64* R, long r_stride, int items, int L, int S, int logn, const Ks32Tables* KT,
              const Prime32* primes, const PrimeConst* qprimes, int form, hipStream_t st, bool fpc) {
    if (items <= 0) return;
    fpc = fpc && (S <= 3 || form != F32_WIDE);   // ks32_fpc_one's 64-bit sums
#define CALL(L_)                                                                                                \
    do {                                                                                                        \
        if (form == F32_LAZY) ks32_launch_crt<L_, true>(U, R, r_stride, items, L, S, KT, primes, qprimes, st, fpc); \
        else ks32_launch_crt<L_, false>(U, R, r_stride, items, L, S, KT, primes, qprimes, st, fpc);                \
    } while (0)
    KS32_SWITCH(logn, CALL)
#undef CALL
}

}  // namespace exacto
