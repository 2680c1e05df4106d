// Batched negacyclic NTT / INTT for gfx950 — replaces concrete-ntt's
// prime64::Plan::{fwd, inv, normalize} (reference call sites src/ring/ntt.rs:24,43,49,60,62).
//
// One residue polynomial per workgroup, n/16 threads, 16 coefficients per
// thread held in VGPRs.  The log2(n) radix-2 stages are grouped into rounds of
// four: inside a round every butterfly is thread-local (no LDS, no barrier);
// between rounds the 16 values are exchanged through one n*8-byte LDS image
// under an XOR swizzle that keeps every ds_write_b64 / ds_read_b64 of the
// three access patterns conflict-free.  Harvey lazy butterflies (values in
// [0, 4q) forward, [0, 2q) inverse) with Shoup twiddles; n^-1 is folded into
// the last inverse stage.  Convention (documented in DESIGN.md, restated by
// oracle/ring.py NttPlan): Cooley-Tukey forward, natural in / bit-reversed out;
// Gentleman-Sande inverse, bit-reversed in / natural out.
#include "exacto_internal.hpp"
#include "ks32_dev.hpp"
#include "bufmem.hpp"
#include "crt_dev.hpp"

namespace exacto {

// Twiddle tables are read-only for a kernel's lifetime: addressing them through the
// constant address space turns block-uniform loads into s_load and the rest into
// global_load (a generic pointer read from PrimeConst would give flat_load, which
// counts against lgkmcnt, so every LDS barrier would also wait on the twiddle preload).
#ifndef EXACTO_TW_AS
#define EXACTO_TW_AS 1
#endif
#if EXACTO_TW_AS == 0
typedef const TwPair* TwTab;
#else
typedef const TwPair __attribute__((address_space(EXACTO_TW_AS)))* TwTab;
#endif

__device__ __forceinline__ TwTab tw_table(const TwPair* p) { return (TwTab)p; }

__device__ __forceinline__ TwPair ld_tw(TwTab tab, int i) {
    TwPair t;
    t.w = tab[i].w;
    t.ws = tab[i].ws;
    return t;
}

__device__ __forceinline__ int swz(int j) {
    return j ^ ((j >> 4) & 15) ^ (((j >> 8) & 1) << 4);
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic only (__syncthreads() would
// also add vmcnt(0), serialising the tail of the output stores of the previous round).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int LO>
__device__ __forceinline__ int elem_index(int tid, int k) {
    return ((tid >> LO) << (LO + 4)) | (k << LO) | (tid & ((1 << LO) - 1));
}

template <int LO>
__device__ __forceinline__ void lds_store(u64* lds, const u64 (&x)[16], int tid) {
#pragma unroll
    for (int k = 0; k < 16; ++k) lds[swz(elem_index<LO>(tid, k))] = x[k];
}

template <int LO>
__device__ __forceinline__ void lds_load(const u64* lds, u64 (&x)[16], int tid) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = lds[swz(elem_index<LO>(tid, k))];
}

// Thread index that hipcc cannot prove wave-uniform (used when T < 64).  At n = 16 a polynomial has one thread
// (T = 1): after `if (tid >= T) return` every address in the kernel is uniform and hipcc loaded the
// polynomial with s_load_dwordx16, i.e. through the scalar data cache.  When a buffer was reused
// (the stream-ordered pool hands the same block to the next call), those scalar loads returned the
// block's previous contents instead of what the preceding kernel had just stored with vector
// stores: wrong results at n = 16 only, changing from run to run (round-1 ADVICE item).  Keeping
// the index in a VGPR makes every polynomial access a vector load.
__device__ __forceinline__ int vtid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// ---------------------------------------------------------------- forward

// Twiddles of one round: stage bit b uses (8 >> (b - LO)) groups; at most 1+2+4+8 = 15 pairs.
// Index of group g at bit b: (N >> (b+1)) + (thigh << (LO+3-b)) + g.
template <int LOGN, int LO, int BHI, int BLO>
__device__ __forceinline__ void load_round_tw(TwPair (&tw)[15], int tid, TwTab tab) {
    constexpr int N = 1 << LOGN;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
    int slot = 0;
#pragma unroll
    for (int b = BHI; b >= BLO; --b) {
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> (b - LO)); ++g) tw[slot++] = ld_tw(tab, base + g);
    }
}

// Butterflies for stage bits BHI..BLO (descending) inside window [LO, LO+4).
template <int LOGN, int LO, int BHI, int BLO, bool LAZY>
__device__ __forceinline__ void fwd_round(u64 (&x)[16], const TwPair (&tw)[15], u64 nq, u64 q2) {
    int slot = 0;
#pragma unroll
    for (int b = BHI; b >= BLO; --b) {
        const int lb = b - LO;
        const int half = 1 << lb;
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            const TwPair t = tw[slot++];
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m;
                const int k1 = k0 + half;
                u64 X = x[k0];
                if (!LAZY) X = X >= q2 ? X - q2 : X;
                const u64 T = shoup_mul_nq(x[k1], t.w, t.ws, nq);
                x[k0] = X + T;
                x[k1] = X - T + q2;
            }
        }
    }
}

// LAZY (all q < 2^60, so 16q <= 2^64): no per-butterfly reduction.  A round of <= 4 stages
// adds < 2q per stage to the bound, so values < 8q at a round start stay < 16q; one
// conditional subtraction of 8q per value at each round start restores the invariant.
// Butterflies of one round with each twiddle loaded right before its group (low register
// pressure; used where the accumulators of the fused key switch need the VGPRs).
template <int LOGN, int LO, int BHI, int BLO, bool LAZY>
__device__ __forceinline__ void fwd_round_direct(u64 (&x)[16], int tid, TwTab tab,
                                                 u64 nq, u64 q2) {
    constexpr int N = 1 << LOGN;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
#pragma unroll
    for (int b = BHI; b >= BLO; --b) {
        const int lb = b - LO;
        const int half = 1 << lb;
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            // generic (flat) load: the scheduler keeps it next to its use instead of clustering
            // a whole round's twiddles (the fused key switch has no VGPRs to spare)
            const TwPair t = ((const TwPair*)tab)[base + g];
#pragma unroll
            for (int m = 0; m < half; ++m) {
                const int k0 = g * 2 * half + m;
                const int k1 = k0 + half;
                u64 X = x[k0];
                if (!LAZY) X = X >= q2 ? X - q2 : X;
                const u64 T = shoup_mul_nq(x[k1], t.w, t.ws, nq);
                x[k0] = X + T;
                x[k1] = X - T + q2;
            }
        }
    }
}

template <int LOGN, int R, bool LAZY, bool PRELOAD = true>
__device__ __forceinline__ void fwd_rounds(u64 (&x)[16], u64* lds, int tid, TwTab tab, u64 nq,
                                           u64 q2, u64 q8) {
    constexpr int LO = (LOGN - 4 * (R + 1)) > 0 ? (LOGN - 4 * (R + 1)) : 0;
    constexpr int BHI = LOGN - 1 - 4 * R;
    TwPair tw[15];
    if constexpr (PRELOAD) load_round_tw<LOGN, LO, BHI, LO>(tw, tid, tab);  // in flight across the exchange
    int t2 = tid;
    // direct-twiddle (fused key switch) callers run this inside a loop: stop the exchange and
    // twiddle addresses derived from tid being hoisted out of it and spilled
    if constexpr (!PRELOAD) asm volatile("" : "+v"(t2));
    if constexpr (R > 0) {
        constexpr int PLO = (LOGN - 4 * R) > 0 ? (LOGN - 4 * R) : 0;
        lds_barrier();
        lds_store<PLO>(lds, x, t2);
        lds_barrier();
        lds_load<LO>(lds, x, t2);
        if constexpr (LAZY) {
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = x[k] >= q8 ? x[k] - q8 : x[k];
        }
    }
    if constexpr (PRELOAD) fwd_round<LOGN, LO, BHI, LO, LAZY>(x, tw, nq, q2);
    else fwd_round_direct<LOGN, LO, BHI, LO, LAZY>(x, t2, tab, nq, q2);
    if constexpr (LO > 0) fwd_rounds<LOGN, R + 1, LAZY, PRELOAD>(x, lds, tid, tab, nq, q2, q8);
}

// Build-time tuning knobs (tools/build_variants.sh measures them).
#ifndef EXACTO_NTT_PRELOAD
#define EXACTO_NTT_PRELOAD 1
#endif

// NTT-domain storage order: evaluation k = a(psi^(2 brv(k) + 1)) is stored at
// position (k mod 16) (n/16) + floor(k / 16).  The forward's last round leaves evaluations
// 16 tid .. 16 tid + 15 in thread tid and the inverse's first round wants exactly those, so both
// move them as x[k] <-> position tid + k n/16: every load / store instruction of a wave covers
// contiguous memory, and the forward needs no LDS transpose before its stores.  (Round 5: with
// the standard order the inverse-side loads ran at a 128-byte lane stride; the cfg3 tensor kernel
// 308 -> 265 us.)
// (Also the order of the inverse's output, elem_index<LOGN - 4>(tid, k) = tid + k n/16, and of the
// forward's coefficient input.)  Buffer accesses (bufmem.hpp): no VALU for the addresses.
#ifndef EXACTO_BUF_LD
#define EXACTO_BUF_LD 1
#endif
#ifndef EXACTO_BUF_ST
#define EXACTO_BUF_ST 1
#endif
typedef PolyIO<EXACTO_BUF_LD != 0> PolyRd;
typedef PolyIO<EXACTO_BUF_ST != 0> PolyWr;

template <int N>
__device__ __forceinline__ void store_evals(u64* dst, const u64 (&x)[16], int tid) {
    const PolyWr w(dst, N * 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) w.st64(x[k], tid * 8, k * (N / 16) * 8);
}

template <int N>
__device__ __forceinline__ void load_evals(u64 (&x)[16], const u64* src, int tid) {
    const PolyRd r(src, N * 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = r.ld64(tid * 8, k * (N / 16) * 8);
}
#ifdef EXACTO_NTT_WAVES
#define NTT_OCC __attribute__((amdgpu_waves_per_eu(EXACTO_NTT_WAVES)))
#else
#define NTT_OCC
#endif

// Coefficient-domain input of a forward transform: element tid + k*T of the polynomial, from
// the u64 source or, for int16 gadget digits, the signed digit as a residue mod q.
template <int N>
__device__ __forceinline__ void load_coeffs(u64 (&x)[16], const NttBatch& nb, const u64* src, int item, int sub,
                                            u64 q, int tid) {
    constexpr int T = N / 16;
    if (nb.src16) {
        const int16_t* s16 = nb.src16 + (long)item * nb.src16_item_stride + (long)(sub / nb.period) * N;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const i64 d = s16[tid + k * T];
            x[k] = d < 0 ? q + (u64)d : (u64)d;
        }
    } else {
        load_evals<N>(x, src, tid);
    }
}

template <int LOGN, bool LAZY>
__global__ void __launch_bounds__((1 << LOGN) / 16 < 64 ? 64 : (1 << LOGN) / 16) NTT_OCC
ntt_fwd_kernel(NttBatch nb, const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    constexpr int T = N / 16;
    __shared__ u64 lds[N];
    const int tid = T < 64 ? vtid() : (int)threadIdx.x;
    if (tid >= T) return;
    const int p = blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64 q = P.q, q2 = P.two_q;
    const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                     (long)sub * N;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;

    u64 x[16];
    load_coeffs<N>(x, nb, src, item, sub, q, tid);

    const u64 q8 = 8 * q;
    fwd_rounds<LOGN, 0, LAZY, EXACTO_NTT_PRELOAD>(x, lds, tid, tw_table(P.tw_fwd), (u64)0 - q, q2, q8);

    // final layout: element 16*tid + k; reduce [0,16q) (LAZY) or [0,4q) -> [0,q)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        u64 v = x[k];
        if (LAZY) {
            v = v >= q8 ? v - q8 : v;
            v = v >= 4 * q ? v - 4 * q : v;
        }
        v = v >= q2 ? v - q2 : v;
        x[k] = v >= q ? v - q : v;
    }
    store_evals<N>(dst, x, tid);
}

// ---------------------------------------------------------------- forward, hand-scheduled rounds

// n = 4096 / 8192 with every prime of the batch in (2^60 - 2^32, 2^60): the butterfly rounds are
// the generated inline-asm statements of ntt_asm.inc (tools/gen_ntt_asm.py): two butterflies
// interleaved so that the SGPR carry chains of the 64-bit arithmetic need no s_nop padding.
// Same convention, same LDS exchanges and same output layout as ntt_fwd_kernel.
#include "ntt_asm.inc"

// The swizzle is linear over GF(2) and elem_index<LO>(tid, k) = A(tid) ^ (k << LO) with disjoint
// bits, so every exchange address is one per-thread base XOR a compile-time constant: one VALU
// per access instead of recomputing the swizzle of each index.
template <int LO>
__device__ __forceinline__ int lds_base_bytes(int tid) {
    return swz(((tid >> LO) << (LO + 4)) | (tid & ((1 << LO) - 1))) << 3;
}

template <int LO>
__device__ __forceinline__ void lds_store_x(u64* lds, const u64 (&x)[16], int tid) {
    char* lb = reinterpret_cast<char*>(lds);
    const int b = lds_base_bytes<LO>(tid);
#pragma unroll
    for (int k = 0; k < 16; ++k) *reinterpret_cast<u64*>(lb + (b ^ (swz(k << LO) << 3))) = x[k];
}

template <int LO>
__device__ __forceinline__ void lds_load_x(const u64* lds, u64 (&x)[16], int tid) {
    const char* lb = reinterpret_cast<const char*>(lds);
    const int b = lds_base_bytes<LO>(tid);
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = *reinterpret_cast<const u64*>(lb + (b ^ (swz(k << LO) << 3)));
}

// GEN: the generic-prime statements (FwdRoundGenAsm: any prime below 2^QB; the HPS primes).
template <int LOGN, int R, bool GEN = false, int QB = 60>
__device__ __forceinline__ void fwd_rounds_asm(u64 (&x)[16], u64* lds, int tid, TwTab tab, const AsmK& K) {
    constexpr int LO = (LOGN - 4 * (R + 1)) > 0 ? (LOGN - 4 * (R + 1)) : 0;
    constexpr int BHI = LOGN - 1 - 4 * R;
    TwPair tw[15];
    load_round_tw<LOGN, LO, BHI, LO>(tw, tid, tab);  // in flight across the exchange
    if constexpr (R > 0) {
        constexpr int PLO = (LOGN - 4 * R) > 0 ? (LOGN - 4 * R) : 0;
        // recompute the exchange addresses per round instead of keeping 32 of them live
        int t2 = tid;
        asm volatile("" : "+v"(t2));
        lds_barrier();
        lds_store_x<PLO>(lds, x, t2);
        lds_barrier();
        lds_load_x<LO>(lds, x, t2);
    }
    if constexpr (GEN) FwdRoundGenAsm<LOGN, R, QB>::run(x, tw, K);
    else FwdRoundAsm<LOGN, R>::run(x, tw, K);
    if constexpr (LO > 0) fwd_rounds_asm<LOGN, R + 1, GEN, QB>(x, lds, tid, tab, K);
}

// ---------------------------------------------------------------- inverse

template <int LOGN, int LO, int BLO, int BHI>
__device__ __forceinline__ void load_round_tw_inv(TwPair (&tw)[15], int tid, TwTab tab) {
    constexpr int N = 1 << LOGN;
    const int thigh = (LO + 4 >= LOGN) ? 0 : (tid >> LO);
    int slot = 0;
#pragma unroll
    for (int b = BLO; b <= BHI; ++b) {
        if (b == LOGN - 1) continue;  // last stage uses the n^-1-folded constants
        const int base = (N >> (b + 1)) + (thigh << (LO + 3 - b));
#pragma unroll
        for (int g = 0; g < (8 >> (b - LO)); ++g) tw[slot++] = ld_tw(tab, base + g);
    }
}

// Gentleman-Sande stages with per-register bound tracking.  m[k] is a compile-time bound
// (x[k] < m[k]*q; the array folds away after unrolling).  Sums are left unreduced while
// the pair's sum stays < 16q (< 2^64 since q < 2^60); otherwise the larger operand is
// halved with one conditional subtraction.  Differences enter Shoup as U - V + m[V]*q
// (any value < 2^64 is a valid Shoup input) and leave in [0, 2q).  Rounds start and end
// with every value < 4q: 12 conditional subtractions per 4-stage round instead of 32.
__device__ __forceinline__ void halve(u64& v, int& m, u64 q) {
    const u64 t = q * (u64)(m / 2);
    v = v >= t ? v - t : v;
    m = (m + 1) / 2;   // v < m q -> v < ceil(m / 2) q (every m the rounds halve is even)
}

template <int LOGN, int LO, int BLO, int BHI, bool LAZY>
__device__ __forceinline__ void inv_round(u64 (&x)[16], const TwPair (&tw)[15], const PrimeConst& P) {
    // LAZY: all q < 2^60, sums may reach 16q; otherwise (q < 2^62) only 4q, round invariant 2q
    constexpr int CAP = LAZY ? 16 : 4, INV = LAZY ? 4 : 2;
    const u64 q = P.q, nq = (u64)0 - q;
    int m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = INV;
    int slot = 0;
#pragma unroll
    for (int b = BLO; b <= BHI; ++b) {
        const int lb = b - LO;
        const int half = 1 << lb;
#pragma unroll
        for (int g = 0; g < (8 >> lb); ++g) {
            TwPair t{0, 0};
            if (b != LOGN - 1) t = tw[slot++];
#pragma unroll
            for (int mm = 0; mm < half; ++mm) {
                const int k0 = g * 2 * half + mm, k1 = k0 + half;
#pragma unroll
                for (int r = 0; r < 3; ++r)
                    if (m[k0] + m[k1] > CAP) {
                        if (m[k0] >= m[k1]) halve(x[k0], m[k0], q);
                        else halve(x[k1], m[k1], q);
                    }
                const u64 U = x[k0], V = x[k1];
                const u64 D = U - V + q * (u64)m[k1];
                if (b == LOGN - 1) {
                    // last stage: (U+V) * n^-1, (U-V) * psi_inv_rev[1] * n^-1, fully reduced
                    const u64 a = shoup_mul_nq(U + V, P.n_inv, P.n_inv_s, nq);
                    const u64 c = shoup_mul_nq(D, P.last_w, P.last_ws, nq);
                    x[k0] = a >= q ? a - q : a;
                    x[k1] = c >= q ? c - q : c;
                    m[k0] = m[k1] = 1;
                } else {
                    x[k0] = U + V;
                    x[k1] = shoup_mul_nq(D, t.w, t.ws, nq);
                    m[k0] += m[k1];
                    m[k1] = 2;
                }
            }
        }
    }
    if (BHI < LOGN - 1) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int r = 0; r < 3; ++r)
                if (m[k] > INV) halve(x[k], m[k], q);
    }
}

template <int LOGN, int R, bool LAZY>
__device__ __forceinline__ void inv_rounds(u64 (&x)[16], u64* lds, int tid, TwTab tab,
                                           const PrimeConst& P) {
    constexpr int LO = (4 * R) < (LOGN - 4) ? 4 * R : LOGN - 4;
    constexpr int BLO = 4 * R;
    constexpr int BHI = (4 * R + 3) < (LOGN - 1) ? 4 * R + 3 : LOGN - 1;
    TwPair tw[15];
    load_round_tw_inv<LOGN, LO, BLO, BHI>(tw, tid, tab);
    if constexpr (R > 0) {
        constexpr int PLO = (4 * (R - 1)) < (LOGN - 4) ? 4 * (R - 1) : LOGN - 4;
        lds_barrier();
        lds_store<PLO>(lds, x, tid);
        lds_barrier();
        lds_load<LO>(lds, x, tid);
    }
    inv_round<LOGN, LO, BLO, BHI, LAZY>(x, tw, P);
    if constexpr (BHI < LOGN - 1) inv_rounds<LOGN, R + 1, LAZY>(x, lds, tid, tab, P);
}

template <int LOGN, bool LAZY>
__global__ void __launch_bounds__((1 << LOGN) / 16 < 64 ? 64 : (1 << LOGN) / 16) NTT_OCC
ntt_inv_kernel(NttBatch nb, const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    constexpr int T = N / 16;
    __shared__ u64 lds[N];
    const int tid = T < 64 ? vtid() : (int)threadIdx.x;
    if (tid >= T) return;
    const int p = blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                     (long)sub * N;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;

    u64 x[16];
    load_evals<N>(x, src, tid);   // evaluation 16 tid + k

    inv_rounds<LOGN, 0, LAZY>(x, lds, tid, tw_table(P.tw_inv), P);

    store_evals<N>(dst, x, tid);
}

// ---------------------------------------------------------------- inverse, hand-scheduled rounds

// n = 4096 / 8192 with every prime of the batch in (2^60 - 2^32, 2^60): the Gentleman-Sande rounds
// are the generated statements of ntt_asm.inc (InvRoundAsm): bounds tracked per value at
// generation time (inputs < 4q), special-prime reductions, n^-1 folded into the last stage.  Same
// convention, twiddle layout and LDS exchanges as inv_rounds.
// GEN: the generic-prime statements (InvRoundGenAsm: any prime below 2^60, conditional-subtraction
// reductions; the HPS auxiliary primes), same layout and bounds contract.
// LZ (special primes only): the last round leaves its outputs in [0, 2q) (InvRoundAsm<.., true>;
// the tensor kernels' consumers take them)
template <int LOGN, int R, bool GEN = false, int QB = 60, bool LZ = false>
__device__ __forceinline__ void inv_rounds_asm(u64 (&x)[16], u64* lds, int tid, TwTab tab, const AsmK& K) {
    constexpr int LO = (4 * R) < (LOGN - 4) ? 4 * R : LOGN - 4;
    constexpr int BLO = 4 * R;
    constexpr int BHI = (4 * R + 3) < (LOGN - 1) ? 4 * R + 3 : LOGN - 1;
    TwPair tw[15];
    load_round_tw_inv<LOGN, LO, BLO, BHI>(tw, tid, tab);  // in flight across the exchange
    if constexpr (R > 0) {
        constexpr int PLO = (4 * (R - 1)) < (LOGN - 4) ? 4 * (R - 1) : LOGN - 4;
        int t2 = tid;
        asm volatile("" : "+v"(t2));
        lds_barrier();
        lds_store_x<PLO>(lds, x, t2);
        lds_barrier();
        lds_load_x<LO>(lds, x, t2);
    }
    if constexpr (GEN) InvRoundGenAsm<LOGN, R, QB>::run(x, tw, K);
    else InvRoundAsm<LOGN, R, LZ && BHI == LOGN - 1>::run(x, tw, K);
    if constexpr (BHI < LOGN - 1) inv_rounds_asm<LOGN, R + 1, GEN, QB, LZ>(x, lds, tid, tab, K);
}

// The smaller-prime forms of the generic rounds (tools/gen_ntt_asm.py GEN_QBITS): a batch whose
// primes are all below 2^gen_qb<LOGN>() takes rounds with fewer reductions (the values' headroom
// below 2^64 is larger); the host picks the kernel instance (launch_ntt / launch_inv_tensor: qbits).
template <int LOGN>
constexpr int gen_qb() { return LOGN == 10 ? 50 : LOGN == 12 ? 56 : 60; }

// ---------------------------------------------------------------- pinned-home rounds

// The generated statements above keep the 16 values of a round in the tied u64 operands x[k] and,
// because inline asm cannot address the halves of a compiler-allocated 64-bit operand, copy them
// into a second set of fixed VGPR pairs for the round (32 VGPRs twice over).  The pinned form
// binds the values to fixed pairs for the whole kernel instead (EXACTO_PIN_DECL: register
// variables xl_k / xh_k = v[PIN_BASE + 2k], v[PIN_BASE + 2k + 1]; hipcc keeps them there at every
// statement, and its loads, LDS exchanges and stores use the pairs in place), and the statements
// (EXACTO_FWD_PIN_*, EXACTO_INV_PIN_*) work on the homes directly: one set of value registers,
// ~124 VGPRs in all, so four waves per SIMD (n = 8192: two 8-wave workgroups per CU instead of one).
#define PIN_X16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)
#define PIN_GET(k) (((u64)xh##k << 32) | xl##k)
#define PIN_SET(k, val)                      \
    {                                        \
        const u64 pv_ = (val);               \
        xl##k = (uint32_t)pv_;               \
        xh##k = (uint32_t)(pv_ >> 32);       \
    }
// LDS exchange of the pinned values: element index of value k is base(tid) ^ (k << LO) (lds_store_x)
#define PIN_ST1(k) *reinterpret_cast<u64*>(pin_lb + (pin_b ^ (swz((k) << PIN_LO_ST) << 3))) = PIN_GET(k);
#define PIN_LD1(k) PIN_SET(k, *reinterpret_cast<const u64*>(pin_lbc + (pin_bl ^ (swz((k) << PIN_LO_LD) << 3))))
#define PIN_EXCHANGE(lds_, tid_, LOST, LOLD)                                           \
    {                                                                                  \
        constexpr int PIN_LO_ST = (LOST), PIN_LO_LD = (LOLD);                          \
        int pin_t2 = (tid_);                                                           \
        asm volatile("" : "+v"(pin_t2));                                               \
        lds_barrier();                                                                 \
        char* pin_lb = reinterpret_cast<char*>(lds_);                                  \
        const int pin_b = lds_base_bytes<PIN_LO_ST>(pin_t2);                           \
        PIN_X16(PIN_ST1)                                                               \
        lds_barrier();                                                                 \
        const char* pin_lbc = reinterpret_cast<const char*>(lds_);                     \
        const int pin_bl = lds_base_bytes<PIN_LO_LD>(pin_t2);                          \
        PIN_X16(PIN_LD1)                                                               \
    }

// The inverse rounds over the pinned homes (inputs < 4q; output element LAST_LO-layout, canonical):
// inv_rounds_asm's twiddles and exchanges.  A macro because the homes are the enclosing
// kernel's register variables.
// SFX_: empty, or _LZ for the tensor kernels' last round with outputs in [0, 2q)
#define PIN_INV_ROUNDS(LOGN_, lds_, tid_, tab_, K_, SFX_)                                        \
    {                                                                                            \
        const AsmK pin_K = (K_);                                                                 \
        const TwTab pin_tab = (tab_);                                                            \
        {                                                                                        \
            TwPair tw[15];                                                                       \
            load_round_tw_inv<LOGN_, 0, 0, 3>(tw, tid_, pin_tab);                                \
            if constexpr (LOGN_ == 12) EXACTO_INV_PIN_12_0(tw, pin_K); else EXACTO_INV_PIN_13_0(tw, pin_K); \
        }                                                                                        \
        {                                                                                        \
            TwPair tw[15];                                                                       \
            load_round_tw_inv<LOGN_, 4, 4, 7>(tw, tid_, pin_tab); /* in flight across the exchange */ \
            PIN_EXCHANGE(lds_, tid_, 0, 4)                                                       \
            if constexpr (LOGN_ == 12) EXACTO_INV_PIN_12_1(tw, pin_K); else EXACTO_INV_PIN_13_1(tw, pin_K); \
        }                                                                                        \
        {                                                                                        \
            TwPair tw[15];                                                                       \
            load_round_tw_inv<LOGN_, 8, 8, 11>(tw, tid_, pin_tab);                               \
            PIN_EXCHANGE(lds_, tid_, 4, 8)                                                       \
            if constexpr (LOGN_ == 12) EXACTO_INV_PIN_12_2##SFX_(tw, pin_K); else EXACTO_INV_PIN_13_2(tw, pin_K); \
        }                                                                                        \
        if constexpr (LOGN_ == 13) {                                                             \
            TwPair tw[15];                                                                       \
            load_round_tw_inv<13, 9, 12, 12>(tw, tid_, pin_tab);                                 \
            PIN_EXCHANGE(lds_, tid_, 8, 9)                                                       \
            EXACTO_INV_PIN_13_3##SFX_(tw, pin_K);                                                \
        }                                                                                        \
    }

// n = 8192: the last exchange (element layout LO = 1 -> LO = 0, a swap of 8 values within each lane
// pair) by DPP instead of LDS (EXACTO_XCHG_PIN_LP, tools/gen_ntt_asm.py LanePairXchg); the values of
// the last round then sit in the homes PERM_LP (value 2j in home j, 2j + 1 in home 8 + j).
#ifndef EXACTO_FWD13_LP
#define EXACTO_FWD13_LP 1
#endif
// position of the value in home h after the last forward round (the stores' order)
template <int LOGN>
__device__ constexpr int fwd_pin_value_of_home(int h) {
    return (LOGN == 13 && EXACTO_FWD13_LP) ? (h < 8 ? 2 * h : 2 * (h - 8) + 1) : h;
}

// The forward rounds over the pinned homes (canonical inputs, element tid + k T; canonical outputs,
// element 16 tid + k): fwd_rounds_asm's twiddles and exchanges.
// SFX_: empty, or _LZ for the last round with outputs in [0, 2q) (NttBatch::lazy_out)
#define PIN_FWD_ROUNDS(LOGN_, lds_, tid_, tab_, K_, SFX_)                                        \
    {                                                                                            \
        const AsmK pin_K = (K_);                                                                 \
        const TwTab pin_tab = (tab_);                                                            \
        {                                                                                        \
            TwPair tw[15];                                                                       \
            load_round_tw<LOGN_, LOGN_ - 4, LOGN_ - 1, LOGN_ - 4>(tw, tid_, pin_tab);            \
            if constexpr (LOGN_ == 12) EXACTO_FWD_PIN_12_0(tw, pin_K); else EXACTO_FWD_PIN_13_0(tw, pin_K); \
        }                                                                                        \
        {                                                                                        \
            TwPair tw[15];                                                                       \
            load_round_tw<LOGN_, LOGN_ - 8, LOGN_ - 5, LOGN_ - 8>(tw, tid_, pin_tab);            \
            PIN_EXCHANGE(lds_, tid_, LOGN_ - 4, LOGN_ - 8)                                       \
            if constexpr (LOGN_ == 12) EXACTO_FWD_PIN_12_1(tw, pin_K); else EXACTO_FWD_PIN_13_1(tw, pin_K); \
        }                                                                                        \
        {                                                                                        \
            constexpr int pin_lo = LOGN_ == 12 ? 0 : 1;                                          \
            TwPair tw[15];                                                                       \
            load_round_tw<LOGN_, pin_lo, LOGN_ - 9, pin_lo>(tw, tid_, pin_tab);                  \
            PIN_EXCHANGE(lds_, tid_, LOGN_ - 8, pin_lo)                                          \
            if constexpr (LOGN_ == 12) EXACTO_FWD_PIN_12_2##SFX_(tw, pin_K); else EXACTO_FWD_PIN_13_2(tw, pin_K); \
        }                                                                                        \
        if constexpr (LOGN_ == 13) {                                                             \
            TwPair tw[15];                                                                       \
            load_round_tw<13, 0, 0, 0>(tw, tid_, pin_tab);                                       \
            if constexpr (EXACTO_FWD13_LP) { /* the exchange within lane pairs, no LDS */        \
                EXACTO_XCHG_PIN_LP(tid_);                                                        \
                EXACTO_FWD_PIN_13_3_LP##SFX_(tw, pin_K);                                         \
            } else {                                                                             \
                PIN_EXCHANGE(lds_, tid_, 1, 0)                                                   \
                EXACTO_FWD_PIN_13_3##SFX_(tw, pin_K);                                            \
            }                                                                                    \
        }                                                                                        \
    }

// Inverse NTT, n = 4096 / 8192, pinned homes: the generated inverse rounds (inv_rounds_asm's twiddles,
// exchanges, bounds and output layout) on values bound to fixed VGPR pairs for the whole kernel.
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(4)))
ntt_inv_pin_kernel(NttBatch nb, const PrimeConst* __restrict__ primes) {
    static_assert(LOGN == 12 || LOGN == 13, "pinned rounds exist for n = 4096 and 8192");
    constexpr int N = 1 << LOGN;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const int p = blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                     (long)sub * N;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;
    EXACTO_PIN_DECL
    {   // evaluation 16 tid + k from position tid + k T (store_evals' order)
        constexpr int T = N / 16;
        const PolyRd rs(src, N * 8);
#define PIN_INP(k) PIN_SET(k, rs.ld64(tid * 8, (k) * T * 8))
        PIN_X16(PIN_INP)
#undef PIN_INP
    }
    PIN_INV_ROUNDS(LOGN, lds, tid, tw_table(P.tw_inv), make_asmk_inv(P), )
    {
        const PolyWr rd(dst, N * 8);
#define PIN_OUT(k) rd.st64(PIN_GET(k), tid * 8, (k) * (N / 16) * 8);
        PIN_X16(PIN_OUT)
#undef PIN_OUT
    }
}

// Probe mode 3 (tools/ntt_probe.hip): the first generation of resident blocks (`slots`, one per CU
// per step of blockIdx / 256) start staggered by `ph` of PHASES block lifetimes, so that loads and
// arithmetic of co-resident blocks stop running in phase; later blocks inherit their slot's offset.
// exacto_probe_sleeps >= 0 (set by the probe tool) overrides the compiled sleeps per phase.
__device__ int exacto_probe_sleeps = -1;
template <int PHASES>
__device__ __forceinline__ void probe_stagger(int slots, int sleeps_per_phase) {
    if ((int)blockIdx.x >= slots) return;
    const int ph = (int)(blockIdx.x / 256) % PHASES;
    const int sp = exacto_probe_sleeps >= 0 ? exacto_probe_sleeps : sleeps_per_phase;
    for (int i = 0; i < ph * sp; ++i) __builtin_amdgcn_s_sleep(16);   // ~1024 cycles each
}
#ifndef EXACTO_PROBE_SLEEPS_FWD
#define EXACTO_PROBE_SLEEPS_FWD 11      // a quarter of a 4096-point forward block's ~21 us lifetime
#endif
#ifndef EXACTO_PROBE_SLEEPS_TENSOR
#define EXACTO_PROBE_SLEEPS_TENSOR 14   // a third of a cfg3 tensor block's ~21 us lifetime
#endif

// Forward NTT, n = 1024 / 4096 / 8192, every prime of the batch below 2^60 but not all of the
// 2^60 - d form (the HPS primes): ntt_fwd_kernel's loads, the generated generic-prime rounds
// (FwdRoundGenAsm, canonical outputs) and store_evals' output order.
template <int LOGN, int QB = 60>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(3)))
ntt_fwd_gen_kernel(NttBatch nb, const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const int p = blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                     (long)sub * N;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;
    u64 x[16];
    load_coeffs<N>(x, nb, src, item, sub, P.q, tid);
    fwd_rounds_asm<LOGN, 0, true, QB>(x, lds, tid, tw_table(P.tw_fwd), make_asmk(P.q));
    store_evals<N>(dst, x, tid);
}

// Inverse NTT, n = 1024 / 4096 / 8192, every prime of the batch below 2^60 but not of the 2^60 - d form
// (HPS auxiliary primes): ntt_inv_kernel with the generated generic-prime rounds (InvRoundGenAsm).
template <int LOGN, int QB = 60>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(3)))
ntt_inv_gen_kernel(NttBatch nb, const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const int p = blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                     (long)sub * N;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;
    u64 x[16];
    load_evals<N>(x, src, tid);
    inv_rounds_asm<LOGN, 0, true, QB>(x, lds, tid, tw_table(P.tw_inv), make_asmk_inv(P));
    store_evals<N>(dst, x, tid);
}

// Forward NTT, n = 4096 / 8192, pinned homes: fwd_rounds_asm's rounds and exchanges, output in
// store_evals' order, with the u64 or int16-digit input of load_coeffs.
// PROBE (tools/ntt_probe.hip only; the library instantiates 0): 1 = compute only (synthetic
// canonical inputs, no global loads, stores skipped at run time), 2 = memory only (loads, the
// same LDS exchanges and stores, no butterflies and no twiddle loads), 3 = the product kernel with
// its first generation staggered (probe_stagger).
// nb2 / split: blocks from `split` on transform a second batch (nb2, block - split): one launch for
// two batches of the same transform size (a dBFV chain step's output limbs and the next step's
// extension)
template <int LOGN, int PROBE = 0, bool LZO = false>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(4)))
ntt_fwd_pin_kernel(NttBatch nb1, const PrimeConst* __restrict__ primes, NttBatch nb2 = NttBatch{},
                   int split = 0x7fffffff) {
    static_assert(LOGN == 12 || LOGN == 13, "pinned rounds exist for n = 4096 and 8192");
    constexpr int N = 1 << LOGN;
    constexpr int T = N / 16;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const bool second = (int)blockIdx.x >= split;
    const NttBatch& nb = second ? nb2 : nb1;
    const int p = second ? (int)blockIdx.x - split : (int)blockIdx.x;
    const int item = p / nb.ppi, sub = p - item * nb.ppi;
    const PrimeConst& P = primes[nb.prime_base + sub % nb.period];
    const u64 q = P.q;
    u64* dst = nb.dst + (long)item * nb.dst_item_stride + (long)sub * N;
    if constexpr (PROBE == 3) {
        if constexpr (LOGN == 12) probe_stagger<4>(1024, EXACTO_PROBE_SLEEPS_FWD);
        else probe_stagger<2>(512, EXACTO_PROBE_SLEEPS_FWD);   // n = 8192: two blocks per CU
    }
    EXACTO_PIN_DECL
    if constexpr (PROBE == 1) {
        const u64 h = ((u64)p << 20) ^ (u64)tid;
#define PIN_SYN(k) PIN_SET(k, ((h + (k)) * 0x9E3779B97F4A7C15ull) & ((1ull << 59) - 1))
        PIN_X16(PIN_SYN)
#undef PIN_SYN
    } else if (nb.src16) {
        const int16_t* s16 = nb.src16 + (long)item * nb.src16_item_stride + (long)(sub / nb.period) * N + tid;
#define PIN_IN16(k) { const i64 d_ = s16[(k) * T]; PIN_SET(k, d_ < 0 ? q + (u64)d_ : (u64)d_) }
        PIN_X16(PIN_IN16)
#undef PIN_IN16
    } else {
        const u64* src = nb.src + (nb.src_off ? (long)nb.src_off[item] : (long)item * nb.src_item_stride) +
                         (long)sub * N;
        const PolyRd rs(src, N * 8);
#define PIN_IN64(k) PIN_SET(k, rs.ld64(tid * 8, (k) * T * 8))
        PIN_X16(PIN_IN64)
#undef PIN_IN64
    }
    if constexpr (PROBE == 2) {   // the exchanges of PIN_FWD_ROUNDS without its butterflies
        PIN_EXCHANGE(lds, tid, LOGN - 4, LOGN - 8)
        PIN_EXCHANGE(lds, tid, LOGN - 8, LOGN == 12 ? 0 : 1)
        if constexpr (LOGN == 13) {
            if constexpr (EXACTO_FWD13_LP) EXACTO_XCHG_PIN_LP(tid);
            else PIN_EXCHANGE(lds, tid, 1, 0)
        }
    } else if constexpr (LZO) {
        PIN_FWD_ROUNDS(LOGN, lds, tid, tw_table(P.tw_fwd), make_asmk(q), _LZ)
    } else {
        PIN_FWD_ROUNDS(LOGN, lds, tid, tw_table(P.tw_fwd), make_asmk(q), )
    }
    // canonical, evaluation 16 tid + k -> position tid + k T (store_evals' order)
    if constexpr (PROBE == 1) {
        if (nb.dst_item_stride != -7) return;   // never stored; the compiler cannot drop the work
    }
    const PolyWr rd(dst, N * 8);
#define PIN_OUT(k) rd.st64(PIN_GET(k), tid * 8, fwd_pin_value_of_home<LOGN>(k) * T * 8);
    PIN_X16(PIN_OUT)
#undef PIN_OUT
}

// ---------------------------------------------------------------- tensor product + inverse

// Degree-2 tensor of two degree-1 ciphertexts fused into the inverse transform of its
// components (eval.rs:186-198 for HPS, the exact tensor of A22 for the generic path):
// block = (item, component c, prime t), laid out like T[item][c][t][n].
//   c0 = a0*b0,  c1 = a0*b1 + a1*b0,  c2 = a1*b1   (pointwise, NTT domain)
// Operands of prime t < L come from the ciphertexts, of the auxiliary primes from extP
// ([item][a0,a1,b0,b1][K][n], already forward-transformed).  LAZY products skip Barrett's
// final corrections (< 3q) and c1 is brought under 4q: the inverse rounds' input bound.
__device__ __forceinline__ u64 barrett_mul_lazy(u64 a, u64 b, const PrimeConst& P) {
    const u64 hi = __umul64hi(a, b), lo = a * b;
    const int s = P.bar_s;
    const u64 xs = (lo >> (s - 1)) | (hi << (65 - s));
    const u64 qhat = ((xs * P.bar_mu) >> (s + 1)) | (__umul64hi(xs, P.bar_mu) << (63 - s));
    return lo - qhat * P.q;  // < 3q
}

// ASM (n = 4096 / 8192, every prime in (2^60 - 2^32, 2^60)): the inverse rounds are the generated
// InvRoundAsm statements (inputs < 4q: products < 3q, c1 < 4q).
// a * b mod q for q = 2^60 - d, d < 2^24, a, b < q: P = H 2^60 + L == L + H d (mod q), folded
// twice (H d < 2^84, then H2 d < 2^49): result < 2^60 + 2^49 < 2q.  No quotient estimate and no
// runtime shift counts (barrett_mul_lazy needs both).
__device__ __forceinline__ u64 mulmod_near60(u64 a, u64 b, uint32_t d) {
    constexpr u64 M60 = (1ull << 60) - 1;
    const u64 lo = a * b, hi = __umul64hi(a, b);
    const u64 H = (hi << 4) | (lo >> 60);
    const u64 xl = (lo & M60) + (u64)(uint32_t)H * d;               // < 2^60 + 2^56
    const u64 xh = (u64)(uint32_t)(H >> 32) * d + (xl >> 32);       // X = xh 2^32 + (uint32)xl
    const u64 H2 = xh >> 28;                                         // X >> 60
    const u64 L2 = ((xh & 0x0FFFFFFFull) << 32) | (uint32_t)xl;
    return L2 + H2 * d;
}

// Products of the tensor kernels by the generated MulNear60Asm statements (ntt_asm.inc,
// tools/gen_ntt_asm.py MulPair): 9 slow + 6 fast instructions per product, the same result (< 2q) as
// mulmod_near60, which hipcc compiles to ~26 (EXACTO_MUL_ASM=0 keeps the C++ for A/B builds).
// The statements clobber fixed VGPRs (v104 up), so the register allocator must keep everything
// live across them elsewhere: in kernels that hold many operands that costs spills.  Measured
// same-box A/B (ROUND 3): ntt_inv_tensor_kernel<12> 323 -> 305 us per launch with the asm (no
// spills either way), but dbfv_pairsum 51 -> 95 us, ntt_inv_tensor3_kernel<13> 258 -> 277 us and
// ntt_inv_tensor_c2_kernel<13> 130 -> 156 us (12 / 28 VGPRs spilled): those take the C++ form
// (ASM = false at their call sites).
#ifndef EXACTO_MUL_ASM
#define EXACTO_MUL_ASM 1
#endif
template <bool ASM = (EXACTO_MUL_ASM != 0)>
__device__ __forceinline__ void mul2_near60(u64& r0, u64 a0, u64 b0, u64& r1, u64 a1, u64 b1, uint32_t d) {
    if constexpr (ASM) {
        MulNear60Asm<2>::run(r0, r1, a0, b0, a1, b1, d, 16 * d);
    } else {
        r0 = mulmod_near60(a0, b0, d);
        r1 = mulmod_near60(a1, b1, d);
    }
}

template <bool ASM = (EXACTO_MUL_ASM != 0)>
__device__ __forceinline__ u64 mul1_near60(u64 a, u64 b, uint32_t d) {
    if constexpr (ASM) {
        u64 r;
        MulNear60Asm<1>::run(r, a, b, d, 16 * d);
        return r;
    } else {
        return mulmod_near60(a, b, d);
    }
}

// x[k] = a[k] b[k] mod q (< 2q), k < 16
template <bool ASM = (EXACTO_MUL_ASM != 0)>
__device__ __forceinline__ void mul16_near60(u64 (&x)[16], const u64 (&a)[16], const u64 (&b)[16], uint32_t d) {
#pragma unroll
    for (int k = 0; k < 16; k += 2) mul2_near60<ASM>(x[k], a[k], b[k], x[k + 1], a[k + 1], b[k + 1], d);
}

// Block b -> logical index, so that each group of G consecutive logical indices runs on one XCD
// in consecutive dispatch slots (workgroups go to XCDs round robin, b % 8: a placement used for
// speed only, never for correctness).  Bijective on [0, total); a tail that does not fill 8
// groups keeps the identity.
__device__ __forceinline__ long xcd_group_remap(long b, long total, int G) {
    const long span = 8L * G;
    const long full = total / span * span;
    if (b >= full) return b;
    const long x = b & 7, slot = b >> 3;
    return ((slot / G) * 8 + x) * G + slot % G;
}

// Block -> (prime t, component c) within one item's blocks (`rem`): the ciphertext primes' three
// components back to back (c1 re-reads c0's and c2's operands: adjacent blocks of one XCD group load
// them at the same time, so the L2 serves the repeats), then p2only's auxiliary-prime c2 blocks.
// (Round 4: placing the c1 blocks after all c0 / c2 blocks of the item instead raised the cfg5
// tensor's reads from 1.30x to 1.62x algorithmic: by then the operands had left the 4 MB L2.)
__device__ __forceinline__ void tensor_unit(int rem, int L, int p2only, int& t, int& c) {
    if (!p2only || rem < 3 * L) {
        t = rem / 3;
        c = rem - 3 * t;
    } else {
        t = L + (rem - 3 * L);
        c = 2;
    }
}

// Block -> (product, unit rem in tensor_unit's order).  share_np = 0: product-major (the units of
// one product together; xcd_group_remap keeps each (product, prime)'s three components, or with
// p2only a whole product, on one XCD).  share_np > 0 (dBFV with shared extensions; the launch holds
// whole items of share_np products that read the same 2d ciphertexts): prime-major within an item,
// so the products of one (item, prime) run back to back on one XCD and read the item's operands in
// that prime (2d ciphertexts x 2 components, 1 MiB at n = 4096 / 2 MiB at n = 8192) once from HBM,
// the repeats from its L2.  Region 1: the primes with three components, order (item, prime,
// component, product), XCD groups of 3 share_np blocks = one (item, prime); region 2 (p2only): the
// auxiliary primes' c2, order (item, prime, product), groups of share_np.
__device__ __forceinline__ void tensor_block(long b, long total, int per, int L, int K, int p2only, int np,
                                             int remap, long& prod, int& rem) {
    if (np <= 0) {
        const long p = remap ? xcd_group_remap(b, total, p2only ? per : 3) : b;
        prod = p / per;
        rem = (int)(p - prod * per);
        return;
    }
    const long items = total / ((long)per * np);
    const int LQ = p2only ? L : L + K;
    const long nQ = items * LQ * 3 * np;
    if (b < nQ) {
        const long G = 3L * np;
        const long p = remap ? xcd_group_remap(b, nQ, (int)G) : b;
        const long g = p / G;
        const int w = (int)(p - g * G);
        const long ib = g / LQ;
        const int t = (int)(g - ib * LQ), c = w / np, pi = w - c * np;
        prod = ib * np + pi;
        rem = 3 * t + c;
    } else {
        const long bb = b - nQ;
        const long p = remap ? xcd_group_remap(bb, total - nQ, np) : bb;
        const long g = p / np;
        const int pi = (int)(p - g * np);
        const long ib = g / K;
        prod = ib * np + pi;
        rem = 3 * L + (int)(g - ib * K);
    }
}

// PROBE (tools/ntt_probe.hip only; the library instantiates 0): 1 = compute only (synthetic operands
// instead of the loads, stores skipped at run time), 2 = no transform (the loads, the pointwise
// products and the stores), 3 = the product kernel with its first generation staggered.  (Round 4
// also measured the next generation's operands prefetched into the L2 by scalar loads before or
// after the transform: 296 -> 357 us, removed.)
// GEN (n = 4096 / 8192, every prime below 2^60 but not all 2^60 - d: HPS): lazy Barrett products,
// then the generated generic-prime inverse rounds (InvRoundGenAsm) instead of the C++ ones.
// LZO (ASM only): outputs in [0, 2q), as ntt_inv_tensor_pin_kernel
template <int LOGN, bool LAZY, bool ASM = false, int PROBE = 0, bool GEN = false, int QB = 60, bool LZO = false>
__global__ void __launch_bounds__((1 << LOGN) / 16 < 64 ? 64 : (1 << LOGN) / 16)
__attribute__((amdgpu_waves_per_eu(3)))  // the ASM form otherwise takes 184 VGPRs (2 waves/SIMD)
ntt_inv_tensor_kernel(Operands op, const u64* __restrict__ extP, u64* __restrict__ Tout, int L, int K,
                      const PrimeConst* __restrict__ primes, int remap, int p2only = 0, int share_np = 0) {
    constexpr int N = 1 << LOGN;
    constexpr int T = N / 16;
    __shared__ u64 lds[N];
    const int tid = T < 64 ? vtid() : (int)threadIdx.x;
    if (tid >= T) return;
    if constexpr (PROBE == 3) probe_stagger<3>(768, EXACTO_PROBE_SLEEPS_TENSOR);
    const int NP = L + K;
    // the three components of one (item, prime) read overlapping inputs (c1 reads c0's and c2's):
    // with xcd_group_remap they run back to back on one XCD, so the second reads hit its L2
    // p2only (dBFV psum: the P residues of c0 / c1 summed by launch_dbfv_pairsum): 3L + K blocks per item, every
    // component of the ciphertext primes, the third only of the auxiliary primes
    const int per = p2only ? 3 * L + K : 3 * NP;
    // groups of 3 keep each (item, prime)'s components together only while every item's blocks are a
    // multiple of 3; p2only's 3L + K is not (cfg5: 17), so there a whole item is one group
    long item;
    int rem;
    tensor_block(blockIdx.x, gridDim.x, per, L, K, p2only, share_np, remap, item, rem);
    int t, c;
    tensor_unit(rem, L, p2only, t, c);
    const PrimeConst& P = primes[t];
    // the four operand polynomials of (item, prime t)
    auto operands = [&](long it, int tt, const u64*& A0, const u64*& A1, const u64*& B0, const u64*& B1) {
        if (tt < L) {
            const u64* A = op.a + (op.a_off ? (long)op.a_off[it] : it * op.a_stride);
            const u64* B = op.b + (op.b_off ? (long)op.b_off[it] : it * op.b_stride);
            A0 = A + (long)tt * N; A1 = A + (long)(L + tt) * N;
            B0 = B + (long)tt * N; B1 = B + (long)(L + tt) * N;
        } else if (op.ea) {  // shared per-ciphertext extensions (dBFV)
            const u64* EA = op.ea + (long)op.ea_off[it] + (long)(tt - L) * N;
            const u64* EB = op.eb + (long)op.eb_off[it] + (long)(tt - L) * N;
            A0 = EA; A1 = EA + (long)K * N; B0 = EB; B1 = EB + (long)K * N;
        } else {
            const u64* E = extP + it * 4 * K * N + (long)(tt - L) * N;
            A0 = E; A1 = E + (long)K * N; B0 = E + 2L * K * N; B1 = E + 3L * K * N;
        }
    };
    const u64 *A0, *A1, *B0, *B1;
    operands(item, t, A0, A1, B0, B1);
    // ASM: every prime is 2^60 - d with d < 2^24 (launch_inv_tensor's caller checks)
    const uint32_t dq = (uint32_t)((1ull << 60) - P.q);
    // GEN: Montgomery products a b R^-1 (< 2q, fewer instructions than Barrett's quotient); the
    // generated inverse's last stage multiplies by R with its constants (make_asmk_inv_mont)
    auto mulr = [&](u64 a, u64 b) {
        return ASM ? mulmod_near60(a, b, dq)
                   : GEN ? mont_mul_lazy(a, b, P.q, P.qinv_neg) : LAZY ? barrett_mul_lazy(a, b, P) : mul_mod(a, b, P);
    };
    auto load = [&](const u64* src, u64 (&v)[16]) {
        if constexpr (PROBE == 1) {
            const u64 h = (u64)(src - op.a) ^ ((u64)tid << 40);
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = ((h + k) * 0x9E3779B97F4A7C15ull) & ((1ull << 59) - 1);
        } else {
            load_evals<N>(v, src, tid);
        }
    };
    u64 x[16], y[16];
    if (c != 1) {
        load(c == 0 ? A0 : A1, x);
        load(c == 0 ? B0 : B1, y);
        if constexpr (ASM) {
            mul16_near60(x, x, y, dq);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = mulr(x[k], y[k]);
        }
    } else {
        u64 z[16];
        load(A0, x);
        load(B1, y);
        if constexpr (ASM) {
            mul16_near60(z, x, y, dq);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) z[k] = mulr(x[k], y[k]);
        }
        load(A1, x);
        load(B0, y);
        const u64 q = P.q, q2 = P.two_q;
        if constexpr (ASM) {
            mul16_near60(x, x, y, dq);
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] += z[k];   // < 4q
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const u64 v = z[k] + mulr(x[k], y[k]);
                // GEN: two Montgomery products < 2q each, already under the inverse's 4q
                x[k] = GEN ? v : LAZY ? (v >= q2 ? v - q2 : v) : (v >= q ? v - q : v);
            }
        }
    }
    if constexpr (PROBE == 2) {
        // no transform: the products are stored as they are
    } else if constexpr (ASM || GEN) {
        const AsmK AK = GEN ? make_asmk_inv_mont(P) : make_asmk_inv(P);
        inv_rounds_asm<LOGN, 0, GEN, QB, LZO && ASM && !GEN>(x, lds, tid, tw_table(P.tw_inv), AK);
    } else {
        inv_rounds<LOGN, 0, LAZY>(x, lds, tid, tw_table(P.tw_inv), P);
    }
    if constexpr (PROBE == 1) {
        if (remap != -7) return;   // never stored; the compiler cannot drop the work
    }
    u64* dst = Tout + ((item * 3 + c) * NP + t) * N;   // [item][c][prime][n]
    store_evals<N>(dst, x, tid);
}

// The tensor kernel over pinned homes (n = 4096 / 8192, special primes): the products
// (MulNear60PinAsm: temps v44-v71, below the homes; < 2q, c1 < 4q) go straight into the homes, and the inverse rounds are
// PIN_INV_ROUNDS -- one set of value registers, four waves per SIMD (n = 8192: two 8-wave
// workgroups per CU).  Same blocks, remap and p2only as ntt_inv_tensor_kernel.
// LZO: outputs in [0, 2q) (the exact path's scale kernels take them; never for HPS, whose scale
// subtracts residues as canonical)
template <int LOGN, bool LZO = false>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(4)))
ntt_inv_tensor_pin_kernel(Operands op, const u64* __restrict__ extP, u64* __restrict__ Tout, int L, int K,
                          const PrimeConst* __restrict__ primes, int remap, int p2only, int share_np) {
    static_assert(LOGN == 12 || LOGN == 13, "pinned rounds exist for n = 4096 and 8192");
    constexpr int N = 1 << LOGN;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const int NP = L + K;
    const int per = p2only ? 3 * L + K : 3 * NP;
    // p2only: a whole item per group (see ntt_inv_tensor_kernel)
    long item;
    int rem;
    tensor_block(blockIdx.x, gridDim.x, per, L, K, p2only, share_np, remap, item, rem);
    int t, c;
    tensor_unit(rem, L, p2only, t, c);
    const PrimeConst& P = primes[t];
    const u64 *A0, *A1, *B0, *B1;
    if (t < L) {
        const u64* A = op.a + (op.a_off ? (long)op.a_off[item] : item * op.a_stride);
        const u64* B = op.b + (op.b_off ? (long)op.b_off[item] : item * op.b_stride);
        A0 = A + (long)t * N; A1 = A + (long)(L + t) * N;
        B0 = B + (long)t * N; B1 = B + (long)(L + t) * N;
    } else if (op.ea) {
        const u64* EA = op.ea + (long)op.ea_off[item] + (long)(t - L) * N;
        const u64* EB = op.eb + (long)op.eb_off[item] + (long)(t - L) * N;
        A0 = EA; A1 = EA + (long)K * N; B0 = EB; B1 = EB + (long)K * N;
    } else {
        const u64* E = extP + item * 4 * K * N + (long)(t - L) * N;
        A0 = E; A1 = E + (long)K * N; B0 = E + 2L * K * N; B1 = E + 3L * K * N;
    }
    const uint32_t dq = (uint32_t)((1ull << 60) - P.q), e16 = 16 * dq;
    EXACTO_PIN_DECL
    // operands in store_evals' order: evaluation 16 tid + k at position tid + k T
    constexpr int T = N / 16;
    const int vo = tid * 8;
#define LDE(r_, k_) r_.ld64(vo, (k_) * T * 8)
    if (c != 1) {
        const PolyRd sa(c == 0 ? A0 : A1, N * 8), sb(c == 0 ? B0 : B1, N * 8);
#define PIN_T1(k0, k1)                                                   \
        {                                                          \
            u64 r0_, r1_;                                          \
            MulNear60PinAsm<2>::run(r0_, r1_, LDE(sa, k0), LDE(sb, k0), LDE(sa, k1), LDE(sb, k1), dq, e16); \
            PIN_SET(k0, r0_) PIN_SET(k1, r1_)                      \
        }
        PIN_T1(0, 1) PIN_T1(2, 3) PIN_T1(4, 5) PIN_T1(6, 7)
        PIN_T1(8, 9) PIN_T1(10, 11) PIN_T1(12, 13) PIN_T1(14, 15)
#undef PIN_T1
    } else {
        const PolyRd sa0(A0, N * 8), sa1(A1, N * 8), sb0(B0, N * 8), sb1(B1, N * 8);
#define PIN_T2(k0, k1)                                                   \
        {                                                          \
            u64 r0_, r1_, s0_, s1_;                                \
            MulNear60PinAsm<2>::run(r0_, r1_, LDE(sa0, k0), LDE(sb1, k0), LDE(sa0, k1), LDE(sb1, k1), dq, e16); \
            MulNear60PinAsm<2>::run(s0_, s1_, LDE(sa1, k0), LDE(sb0, k0), LDE(sa1, k1), LDE(sb0, k1), dq, e16); \
            PIN_SET(k0, r0_ + s0_) PIN_SET(k1, r1_ + s1_)          \
        }
        // two halves of 16 loads each: hoisting all 32 (128 VGPRs) past the products would spill
        PIN_T2(0, 1) PIN_T2(2, 3) PIN_T2(4, 5) PIN_T2(6, 7)
        __builtin_amdgcn_sched_barrier(0);
        PIN_T2(8, 9) PIN_T2(10, 11) PIN_T2(12, 13) PIN_T2(14, 15)
#undef PIN_T2
    }
#undef LDE
    if constexpr (LZO) {
        PIN_INV_ROUNDS(LOGN, lds, tid, tw_table(P.tw_inv), make_asmk_inv(P), _LZ)
    } else {
        PIN_INV_ROUNDS(LOGN, lds, tid, tw_table(P.tw_inv), make_asmk_inv(P), )
    }
    u64* dst = Tout + ((item * 3 + c) * NP + t) * N;   // [item][c][prime][n]
    {
        const PolyWr rd(dst, N * 8);
#define PIN_OUT(k) rd.st64(PIN_GET(k), tid * 8, (k) * (N / 16) * 8);
        PIN_X16(PIN_OUT)
#undef PIN_OUT
    }
}

// ---------------------------------------------------------------- fused product + inverse

// out = INTT(a (.) b) per residue polynomial: NttPoly::mul then to_coeff_poly (ntt.rs:58-67,
// 119-129) in one pass, the product formed on load as the tensor kernel does (the pointwise pass
// and its HBM round trip disappear).  Rows [rows][n], row r mod prime r % period.
template <int LOGN, bool LAZY, bool ASM = false>
__global__ void __launch_bounds__((1 << LOGN) / 16 < 64 ? 64 : (1 << LOGN) / 16)
__attribute__((amdgpu_waves_per_eu(3)))
ntt_mulinv_kernel(const u64* A, const u64* B, u64* out, int period,
                  const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    constexpr int T = N / 16;
    __shared__ u64 lds[N];
    const int tid = T < 64 ? vtid() : (int)threadIdx.x;
    if (tid >= T) return;
    const long p = blockIdx.x;
    const PrimeConst& P = primes[(int)(blockIdx.x % (unsigned)period)];
    const uint32_t dq = (uint32_t)((1ull << 60) - P.q);
    u64 x[16], y[16];
    load_evals<N>(x, A + p * N, tid);
    load_evals<N>(y, B + p * N, tid);
    if constexpr (ASM) {
        mul16_near60<false>(x, x, y, dq);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = LAZY ? barrett_mul_lazy(x[k], y[k], P) : mul_mod(x[k], y[k], P);
    }
    if constexpr (ASM) {
        const AsmK AK = make_asmk_inv(P);
        inv_rounds_asm<LOGN, 0>(x, lds, tid, tw_table(P.tw_inv), AK);
    } else {
        inv_rounds<LOGN, 0, LAZY>(x, lds, tid, tw_table(P.tw_inv), P);
    }
    u64* dst = out + p * N;
    store_evals<N>(dst, x, tid);
}

template <int LOGN>
static void launch_mi(const u64* A, const u64* B, u64* out, long rows, int period, bool lazy, bool asm_inv,
                      const PrimeConst* primes, hipStream_t s) {
    constexpr int threads = (1 << LOGN) / 16 < 64 ? 64 : (1 << LOGN) / 16;
    if constexpr (LOGN == 12 || LOGN == 13) {
        if (asm_inv) {
            EXACTO_LAUNCH((ntt_mulinv_kernel<LOGN, true, true>), dim3(rows), dim3(threads), 0, s, A, B, out, period,
                               primes);
            return;
        }
    }
    if (lazy)
        EXACTO_LAUNCH((ntt_mulinv_kernel<LOGN, true>), dim3(rows), dim3(threads), 0, s, A, B, out, period, primes);
    else
        EXACTO_LAUNCH((ntt_mulinv_kernel<LOGN, false>), dim3(rows), dim3(threads), 0, s, A, B, out, period,
                           primes);
}

void launch_mul_inv(const u64* A, const u64* B, u64* out, long rows, int period, int logn, bool lazy, bool asm_inv,
                    const PrimeConst* primes, hipStream_t s) {
    if (rows <= 0) return;
    switch (logn) {
        case 4: launch_mi<4>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 5: launch_mi<5>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 6: launch_mi<6>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 7: launch_mi<7>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 8: launch_mi<8>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 9: launch_mi<9>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 10: launch_mi<10>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 11: launch_mi<11>(A, B, out, rows, period, lazy, false, primes, s); break;
        case 12: launch_mi<12>(A, B, out, rows, period, lazy, asm_inv, primes, s); break;
        case 13: launch_mi<13>(A, B, out, rows, period, lazy, asm_inv, primes, s); break;
        case 14: launch_mi<14>(A, B, out, rows, period, lazy, false, primes, s); break;
        default: break;
    }
}

// ---------------------------------------------------------------- fused negacyclic product

// out = INTT(NTT(a) (.) NTT(b)) per residue polynomial (coefficient domain in and out): the
// reference's NTT multiplication (ntt.rs:181-195: from_coeff_poly twice, mul, to_coeff_poly) in
// one workgroup.  The forward transform leaves element 16 tid + k in x[k], which is the layout
// the inverse's first round takes, so neither operand's evaluations nor the product ever leave
// the chip: 3 HBM passes per product instead of 7, and no output transposes of the forward
// transforms.  n = 4096 / 8192, every prime 2^60 - d with d < 2^24 (asm rounds, mulmod_near60).
// b's coefficients are loaded at the start and stay in flight across a's transform; x_a is held
// across b's, which needs 2 waves per SIMD (the asm rounds' clobbered VGPRs plus both operands).
template <int LOGN>
__global__ void __launch_bounds__((1 << LOGN) / 16) __attribute__((amdgpu_waves_per_eu(2)))
ntt_polymul_kernel(const u64* A, const u64* B, u64* out, int period, const PrimeConst* __restrict__ primes) {
    constexpr int N = 1 << LOGN;
    __shared__ u64 lds[N];
    const int tid = threadIdx.x;
    const long p = blockIdx.x;
    const PrimeConst& P = primes[(int)(blockIdx.x % (unsigned)period)];
    const u64 q = P.q;
    const u64* a = A + p * N;
    const u64* b = B + p * N;
    u64 xa[16], xb[16];
    load_evals<N>(xa, a, tid);   // coefficients tid + k T
    load_evals<N>(xb, b, tid);
    const AsmK K = make_asmk(q);
    const TwTab tf = tw_table(P.tw_fwd);
    fwd_rounds_asm<LOGN, 0>(xa, lds, tid, tf, K);
    fwd_rounds_asm<LOGN, 0>(xb, lds, tid, tf, K);
    const uint32_t dq = (uint32_t)((1ull << 60) - q);
    mul16_near60(xa, xa, xb, dq);   // < 2q: the inverse's input bound
    const AsmK AK = make_asmk_inv(P);
    inv_rounds_asm<LOGN, 0>(xa, lds, tid, tw_table(P.tw_inv), AK);
    u64* dst = out + p * N;
    store_evals<N>(dst, xa, tid);
}

bool launch_polymul(const u64* A, const u64* B, u64* out, long rows, int period, int logn, const PrimeConst* primes,
                    hipStream_t s) {
    // (a pinned-home form at 4 waves per SIMD, a parked in out's rows, measured 866-876 vs 806 us per
    // cfg2 launch and was removed, round 4)
    if (logn == 12)
        EXACTO_LAUNCH(ntt_polymul_kernel<12>, dim3(rows), dim3(256), 0, s, A, B, out, period, primes);
    else if (logn == 13)
        EXACTO_LAUNCH(ntt_polymul_kernel<13>, dim3(rows), dim3(512), 0, s, A, B, out, period, primes);
    else
        return false;
    return true;
}

// rlk_s = floor(rlk * 2^64 / q_limb) (Shoup companions of the resident key, computed once)
__global__ void shoup_companion_kernel(const u64* __restrict__ w, u64* __restrict__ ws, long count, int n,
                                       int L, const PrimeConst* __restrict__ primes) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= count) return;
    const int limb = (int)((idx / n) % L);
    ws[idx] = (u64)(((u128)w[idx] << 64) / primes[limb].q);
}

// ---------------------------------------------------------------- launchers

template <int LOGN>
static void launch_one(const NttBatch& nb, int count, bool inverse, bool lazy, const PrimeConst* primes,
                       hipStream_t s) {
    constexpr int threads = (1 << LOGN) / 16;
    if (inverse)
        EXACTO_LAUNCH((lazy ? ntt_inv_kernel<LOGN, true> : ntt_inv_kernel<LOGN, false>), dim3(count),
                           dim3(threads), 0, s, nb, primes);
    else if (lazy)
        EXACTO_LAUNCH((ntt_fwd_kernel<LOGN, true>), dim3(count), dim3(threads), 0, s, nb, primes);
    else
        EXACTO_LAUNCH((ntt_fwd_kernel<LOGN, false>), dim3(count), dim3(threads), 0, s, nb, primes);
}

// dBFV, psum (dbfv_mul_core): the auxiliary-prime residues of each output limb's c0 and c1 tensors
// summed over its products in the NTT domain (c0 = sum a0_i b0_j, c1 = sum a0_i b1_j + a1_i b0_j
// over the limb's pairs), one coefficient per thread, out [ib][k][c][a][n] canonical; one batched
// inverse transform per (limb, component, prime) follows instead of one per product.  Every step
// of the scale up to the Garner over P is linear in T (r = T (p Q^-1) + sum_k v_k (...) + negs mod
// p_a), so exact_psum_sp_kernel adds the per-product corrections to these sums.  Block = (ib, a, k)
// x 256 coefficients (consecutive k of one (item, prime) back to back: they re-read the same
// operands, from L2).
#ifndef EXACTO_PAIRSUM_DOT
#define EXACTO_PAIRSUM_DOT 1   // the pair sums as 30-bit-limb dots (A/B build switch; 0: a fold per product)
#endif
__global__ void __launch_bounds__(256)
dbfv_pairsum_kernel(Operands op, u64* __restrict__ out, int d, int npairs, int L, int K, int n,
                    const int* __restrict__ term_start, const CombineTerm* __restrict__ terms,
                    const PrimeConst* __restrict__ primes) {
    const int nb = n >> 8;
    const long row = blockIdx.x / nb;                  // (ib * K + a) * d + k
    const int j = (int)(blockIdx.x - row * nb) * 256 + (int)threadIdx.x;
    const int k = (int)(row % d);
    const long r1 = row / d;
    const int a = (int)(r1 % K);
    const long ib = r1 / K;
    const u64 q = primes[L + a].q;
    const long off_a = (long)a * n + j, off_k = (long)K * n;
#if EXACTO_PAIRSUM_DOT
    // the products as 30-bit-limb dots (crt_dev.hpp): operands canonical, so every limb product is below
    // 2^60; c1 takes two products per pair, so the columns fold every 3 pairs (dot30_fold: at most 7
    // products plus a canonical constant) instead of a 120-bit fold per product
    Dot30 S0{0, 0, 0}, S1{0, 0, 0};
    int cnt = 0;
    for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
        const long pr = ib * npairs + terms[t].pair;
        const u64* EA = op.ea + (long)op.ea_off[pr] + off_a;
        const u64* EB = op.eb + (long)op.eb_off[pr] + off_a;
        u64 a0 = EA[0], a1 = EA[off_k], b0 = EB[0], b1 = EB[off_k];   // < 2q
        a0 = a0 >= q ? a0 - q : a0;
        a1 = a1 >= q ? a1 - q : a1;
        b0 = b0 >= q ? b0 - q : b0;
        b1 = b1 >= q ? b1 - q : b1;
        const uint32_t a00 = (uint32_t)a0 & M30, a01 = (uint32_t)(a0 >> 30);
        const uint32_t a10 = (uint32_t)a1 & M30, a11 = (uint32_t)(a1 >> 30);
        dot30_mac(S0, a00, a01, b0);
        dot30_mac(S1, a00, a01, b1);
        dot30_mac(S1, a10, a11, b0);
        if (++cnt == 3) {
            S0 = Dot30{dot30_fold(S0, q), 0, 0};
            S1 = Dot30{dot30_fold(S1, q), 0, 0};
            cnt = 0;
        }
    }
    u64* o = out + (((ib * d + k) * 2) * K + a) * (long)n + j;
    o[0] = dot30_fold(S0, q);
    o[(long)K * n] = dot30_fold(S1, q);
#else
    const u64 q2 = 2 * q;
    const uint32_t dq = (uint32_t)((1ull << 60) - q);
    u64 s0 = 0, s1 = 0;                                // < 2q between terms (products < 2q)
    for (int t = term_start[k]; t < term_start[k + 1]; ++t) {
        const long pr = ib * npairs + terms[t].pair;
        const u64* EA = op.ea + (long)op.ea_off[pr] + off_a;
        const u64* EB = op.eb + (long)op.eb_off[pr] + off_a;
        const u64 a0 = EA[0], a1 = EA[off_k], b0 = EB[0], b1 = EB[off_k];
        u64 p0, p1;
        mul2_near60<false>(p0, a0, b1, p1, a1, b0, dq);
        u64 v = s1 + p0 + p1;                      // < 6q
        v = v >= 4 * q ? v - 4 * q : v;
        s1 = v >= q2 ? v - q2 : v;
        v = s0 + mul1_near60<false>(a0, b0, dq);
        s0 = v >= q2 ? v - q2 : v;
    }
    u64* o = out + (((ib * d + k) * 2) * K + a) * (long)n + j;
    o[0] = s0 >= q ? s0 - q : s0;
    o[(long)K * n] = s1 >= q ? s1 - q : s1;
#endif
}

void launch_dbfv_pairsum(const Operands& op, u64* out, int items_b, int d, int npairs, const int* term_start,
                         const CombineTerm* terms, int L, int K, int n, const PrimeConst* primes, hipStream_t s) {
    const long blocks = (long)items_b * K * d * (n >> 8);
    if (blocks == 0 || n < 256) return;
    EXACTO_LAUNCH(dbfv_pairsum_kernel, dim3(blocks), dim3(256), 0, s, op, out, d, npairs, L, K, n, term_start,
                       terms, primes);
}

// Pinned-home tensor kernel (runtime A/B switch, read once): ntt_inv_tensor_pin_kernel at n = 8192
// (it replaced the one-block-per-(item, prime) tensor3 + tensor_c2 pair: cfg5 1996 -> 2175 chains/s,
// same box); at n = 4096 the 3-wave ntt_inv_tensor_kernel stays (pinned 297-302 vs 295-296 us per
// cfg3 launch).  EXACTO_TENSOR_PIN=0: never, =1: at both sizes.
static int env_switch(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && e[0] ? (e[0] != '0') : dflt;
}
static bool tensor_pin_at(int logn) {
    static const int on = env_switch("EXACTO_TENSOR_PIN", -1);
    return on < 0 ? logn == 13 : on && (logn == 12 || logn == 13);
}

// EXACTO_NTT_GEN=0: the C++ generic-prime inverse rounds instead of the generated ones (A/B switch).
static bool ntt_gen_on() {
    static const int on = env_switch("EXACTO_NTT_GEN", 1);
    return on != 0;
}

// the smaller-prime generic rounds apply: every prime of the batch below 2^gen_qb<LOGN>().
// EXACTO_NTT_GENQ=0: never (A/B switch)
template <int LOGN>
static bool gen_small(int qbits) {
    static const int on = env_switch("EXACTO_NTT_GENQ", 1);
    return on && gen_qb<LOGN>() < 60 && qbits <= gen_qb<LOGN>();
}

template <int LOGN>
static void launch_it(const Operands& op, const u64* extP, u64* T, long blocks, int L, int K, bool lazy,
                      const PrimeConst* primes, hipStream_t s, bool asm_inv = false, int p2only = 0, int qbits = 64,
                      int np = 0, bool lzo = false) {
    constexpr int threads = (1 << LOGN) / 16;
    // EXACTO_XCD_REMAP=0: plain block order (A/B switch)
    static const int remap = [] { const char* e = std::getenv("EXACTO_XCD_REMAP"); return (e && e[0] == '0') ? 0 : 1; }();
    if constexpr (LOGN == 12 || LOGN == 13) {
        if (asm_inv && tensor_pin_at(LOGN)) {
            const long b2 = p2only ? blocks / (3 * (L + K)) * (3 * L + K) : blocks;
            if (lzo)
                EXACTO_LAUNCH((ntt_inv_tensor_pin_kernel<LOGN, true>), dim3(b2), dim3(threads), 0, s, op, extP, T,
                                   L, K, primes, remap, p2only, np);
            else
                EXACTO_LAUNCH((ntt_inv_tensor_pin_kernel<LOGN>), dim3(b2), dim3(threads), 0, s, op, extP, T, L,
                                   K, primes, remap, p2only, np);
            return;
        }
        if (asm_inv) {
            const long b2 = p2only ? blocks / (3 * (L + K)) * (3 * L + K) : blocks;
            if (lzo)
                EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, true, true, 0, false, 60, true>), dim3(b2),
                                   dim3(threads), 0, s, op, extP, T, L, K, primes, remap, p2only, np);
            else
                EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, true, true>), dim3(b2), dim3(threads), 0, s, op, extP,
                                   T, L, K, primes, remap, p2only, np);
            return;
        }
    }
    if constexpr (LOGN == 10 || LOGN == 12 || LOGN == 13) {
        if (lazy && !p2only && ntt_gen_on()) {   // every prime below 2^60: the generated generic-prime rounds
            if (gen_small<LOGN>(qbits))
                EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, true, false, 0, true, gen_qb<LOGN>()>), dim3(blocks),
                                   dim3(threads), 0, s, op, extP, T, L, K, primes, remap, 0, np);
            else
                EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, true, false, 0, true>), dim3(blocks), dim3(threads), 0,
                                   s, op, extP, T, L, K, primes, remap, 0, np);
            return;
        }
    }
    if (lazy)
        EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, true>), dim3(blocks), dim3(threads), 0, s, op, extP, T, L, K,
                           primes, remap);
    else
        EXACTO_LAUNCH((ntt_inv_tensor_kernel<LOGN, false>), dim3(blocks), dim3(threads), 0, s, op, extP, T, L,
                           K, primes, remap);
}

void launch_inv_tensor(const Operands& op, const u64* extP, u64* T, int items, int logn, int L, int K, bool lazy,
                       const PrimeConst* primes, hipStream_t s, bool asm_inv, bool p2only, int qbits, int share_np,
                       bool lazy_out) {
    // prime-major block order needs whole dBFV items in the launch (tensor_block)
    // (measured: cfg5, 36 products per item, tensor 270 -> 261 us; cfg4's 3 products per item and
    // u64_dbfv within noise: applied from 8 products per item; round 6 again at cfg4:
    // tensor 140 -> 143-147 us, 185.6k vs 185.1k/s)
    if (share_np < 8 || items % share_np != 0) share_np = 0;
    const long blocks = (long)items * 3 * (L + K);
    if (blocks == 0) return;
    if (p2only) {   // the caller checks asm_inv and n = 4096 / 8192
        if (logn == 12) launch_it<12>(op, extP, T, blocks, L, K, lazy, primes, s, true, 1, 64, share_np, lazy_out);
        else if (logn == 13) launch_it<13>(op, extP, T, blocks, L, K, lazy, primes, s, true, 1, 64, share_np, lazy_out);
        return;
    }
    switch (logn) {
        case 4: launch_it<4>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 5: launch_it<5>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 6: launch_it<6>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 7: launch_it<7>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 8: launch_it<8>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 9: launch_it<9>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 10: launch_it<10>(op, extP, T, blocks, L, K, lazy, primes, s, false, 0, qbits, share_np); break;
        case 11: launch_it<11>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        case 12: launch_it<12>(op, extP, T, blocks, L, K, lazy, primes, s, asm_inv, 0, qbits, share_np, lazy_out); break;
        case 13: launch_it<13>(op, extP, T, blocks, L, K, lazy, primes, s, asm_inv, 0, qbits, share_np, lazy_out); break;
        case 14: launch_it<14>(op, extP, T, blocks, L, K, lazy, primes, s); break;
        default: break;
    }
}

bool launch_ntt_fwd2(const NttBatch& nb1, int count1, const NttBatch& nb2, int count2, int logn,
                     const PrimeConst* primes, hipStream_t s) {
    if (count1 <= 0 || count2 <= 0 || (logn != 12 && logn != 13)) return false;
    const dim3 grid((unsigned)(count1 + count2));
    if (logn == 12) EXACTO_LAUNCH((ntt_fwd_pin_kernel<12>), grid, dim3(256), 0, s, nb1, primes, nb2, count1);
    else EXACTO_LAUNCH((ntt_fwd_pin_kernel<13>), grid, dim3(512), 0, s, nb1, primes, nb2, count1);
    return true;
}

void launch_ntt(const NttBatch& nb, int count, int logn, bool inverse, bool lazy, const PrimeConst* primes,
                hipStream_t s, bool asm_fwd, bool asm_inv, int qbits) {
    if (count <= 0) return;
    // n = 4096 / 8192, every prime of the batch in (2^60 - 2^32, 2^60): the pinned-home kernels (the
    // non-pinned asm kernels and the persistent LDS-DMA forward kernel measured slower and were removed,
    // DESIGN.md §6)
    if (asm_fwd && !inverse && (logn == 12 || logn == 13)) {
        if (nb.lazy_out) {
            if (logn == 12) EXACTO_LAUNCH((ntt_fwd_pin_kernel<12, 0, true>), dim3(count), dim3(256), 0, s, nb, primes);
            else EXACTO_LAUNCH((ntt_fwd_pin_kernel<13, 0, true>), dim3(count), dim3(512), 0, s, nb, primes);
        } else {
            if (logn == 12) EXACTO_LAUNCH((ntt_fwd_pin_kernel<12>), dim3(count), dim3(256), 0, s, nb, primes);
            else EXACTO_LAUNCH((ntt_fwd_pin_kernel<13>), dim3(count), dim3(512), 0, s, nb, primes);
        }
        return;
    }
    if (asm_inv && inverse && (logn == 12 || logn == 13)) {
        if (logn == 12) EXACTO_LAUNCH((ntt_inv_pin_kernel<12>), dim3(count), dim3(256), 0, s, nb, primes);
        else EXACTO_LAUNCH((ntt_inv_pin_kernel<13>), dim3(count), dim3(512), 0, s, nb, primes);
        return;
    }
    if (lazy && (logn == 10 || logn == 12 || logn == 13) && ntt_gen_on()) {   // every prime below 2^60: generic asm rounds
        const dim3 th(1u << (logn - 4));
#define GEN_NTT_(K_, LG_, QB_) EXACTO_LAUNCH((K_<LG_, QB_>), dim3(count), th, 0, s, nb, primes)
        if (inverse) {
            if (logn == 10) { if (gen_small<10>(qbits)) GEN_NTT_(ntt_inv_gen_kernel, 10, 50); else GEN_NTT_(ntt_inv_gen_kernel, 10, 60); }
            else if (logn == 12) { if (gen_small<12>(qbits)) GEN_NTT_(ntt_inv_gen_kernel, 12, 56); else GEN_NTT_(ntt_inv_gen_kernel, 12, 60); }
            else GEN_NTT_(ntt_inv_gen_kernel, 13, 60);
        } else {
            if (logn == 10) { if (gen_small<10>(qbits)) GEN_NTT_(ntt_fwd_gen_kernel, 10, 50); else GEN_NTT_(ntt_fwd_gen_kernel, 10, 60); }
            else if (logn == 12) { if (gen_small<12>(qbits)) GEN_NTT_(ntt_fwd_gen_kernel, 12, 56); else GEN_NTT_(ntt_fwd_gen_kernel, 12, 60); }
            else GEN_NTT_(ntt_fwd_gen_kernel, 13, 60);
        }
#undef GEN_NTT_
        return;
    }
    switch (logn) {
        case 4: launch_one<4>(nb, count, inverse, lazy, primes, s); break;
        case 5: launch_one<5>(nb, count, inverse, lazy, primes, s); break;
        case 6: launch_one<6>(nb, count, inverse, lazy, primes, s); break;
        case 7: launch_one<7>(nb, count, inverse, lazy, primes, s); break;
        case 8: launch_one<8>(nb, count, inverse, lazy, primes, s); break;
        case 9: launch_one<9>(nb, count, inverse, lazy, primes, s); break;
        case 10: launch_one<10>(nb, count, inverse, lazy, primes, s); break;
        case 11: launch_one<11>(nb, count, inverse, lazy, primes, s); break;
        case 12: launch_one<12>(nb, count, inverse, lazy, primes, s); break;
        case 13: launch_one<13>(nb, count, inverse, lazy, primes, s); break;
        case 14: launch_one<14>(nb, count, inverse, lazy, primes, s); break;
        default: break;  // rejected at context creation
    }
}

void launch_shoup_companions(const u64* w, u64* ws, long count, int n, int L, const PrimeConst* primes,
                             hipStream_t s) {
    if (count <= 0) return;
    EXACTO_LAUNCH(shoup_companion_kernel, dim3((count + 255) / 256), dim3(256), 0, s, w, ws, count, n, L,
                       primes);
}

}  // namespace exacto
