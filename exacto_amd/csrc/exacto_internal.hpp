// Internal (non-ABI) declarations shared by the HIP kernels and the host runtime.
#pragma once
#include "arith.hpp"

namespace exacto {

// A batch of independent residue polynomials for the NTT kernels.
// Polynomial p (0 <= p < count) belongs to item p / ppi, sub-polynomial p % ppi.
// Source: src + (src_off ? src_off[item] : item * src_item_stride) + sub * n.
// Destination: dst + item * dst_item_stride + sub * n (may alias the source).
// Prime: prime_base + sub % period.
struct NttBatch {
    const u64* src;
    const u64* src_off;
    long src_item_stride;
    u64* dst;
    long dst_item_stride;
    int ppi;
    int prime_base;
    int period;
    // optional int16 source (gadget digits): polynomial (item, sub) reads
    // src16 + item * src16_item_stride + (sub / period) * n, converted to residues mod its prime
    const int16_t* src16;
    long src16_item_stride;
    // forward, pinned kernels only: outputs in [0, 2q) (set only for the exact path's extension
    // transforms, whose sole reader is the asm tensor product: MulPair takes operands below 2^61)
    int lazy_out;
};

enum class MulPath : int { Exact = 0, Hps = 1 };

// Constants for exact CRT / base conversion, HPS and gadget decomposition.
// Mixed-radix (Garner) digits are used everywhere so that centring decisions are exact.
struct CrtTables {
    int L;          // ciphertext primes (prime indices 0..L-1)
    int K;          // auxiliary primes used by the path (prime indices L..L+K-1)
    int G;          // gadget digits  (params/mod.rs:126-140)
    int gshift;     // log2(gadget base) if a power of two, else -1
    u64 gbase;
    u64 plain;      // BFV plaintext modulus p
    // Garner over Q: gq[i][k] = q_k^-1 mod q_i (k < i)
    u64 gq_w[EXACTO_MAX_L][EXACTO_MAX_L];
    u64 gq_ws[EXACTO_MAX_L][EXACTO_MAX_L];
    u64 halfQ_mr[EXACTO_MAX_L];                 // mixed-radix digits of floor(Q/2)
    // qpref[k][t] = (q_0 ... q_{k-1}) mod prime_t, k = 0..L (k = L: Q mod prime_t)
    u64 qpref_w[EXACTO_MAX_L + 1][EXACTO_MAX_PRIMES];
    u64 qpref_ws[EXACTO_MAX_L + 1][EXACTO_MAX_PRIMES];
    // Garner over P (auxiliary primes, exact path)
    u64 gp_w[EXACTO_MAX_K][EXACTO_MAX_K];
    u64 gp_ws[EXACTO_MAX_K][EXACTO_MAX_K];
    u64 halfP_mr[EXACTO_MAX_K];
    // ppref[k][i] = (p_0 ... p_{k-1}) mod q_i, k = 0..K
    u64 ppref_w[EXACTO_MAX_K + 1][EXACTO_MAX_L];
    u64 ppref_ws[EXACTO_MAX_K + 1][EXACTO_MAX_L];
    u64 qinvp_w[EXACTO_MAX_K], qinvp_ws[EXACTO_MAX_K];   // Q^-1 mod p_j
    // folded scale constants: pq[t] = p * Q^-1 mod p_t (aux t), qpq[k][a] = qpref[k][L+a] * Q^-1 mod p_a
    u64 pq_w[EXACTO_MAX_K], pq_ws[EXACTO_MAX_K];
    u64 qpq_w[EXACTO_MAX_L + 1][EXACTO_MAX_K], qpq_ws[EXACTO_MAX_L + 1][EXACTO_MAX_K];
    // CRT over P by a rounded float sum (the SP scale kernels' FPC form): with Pi_a = (P / p_a)^-1 mod p_a
    // folded into every constant, each dot product gives y_a = r Pi_a mod p_a directly, and
    // r = sum_a y_a (P / p_a) - round(sum_a y_a / p_a) P when |r| < P / 4
    u64 fpc_pq[EXACTO_MAX_K];                    // pq[a] Pi_a
    u64 fpc_qpq[EXACTO_MAX_L][EXACTO_MAX_K];     // (p_a - qpq[k][a]) Pi_a
    u64 fpc_neg[EXACTO_MAX_K];                   // Pi_a (the +1 of a negative s)
    double fpc_inv[EXACTO_MAX_K];                // 1 / p_a
    u64 fpc_pm[EXACTO_MAX_K][EXACTO_MAX_L];      // (P / p_a) mod q_i
    u64 fpc_negP[EXACTO_MAX_L];                  // (q_i - P mod q_i) mod q_i
    // FPQ: the centred s = [p T]_Q by a rounded float sum too (kernels.hip fpq_y): with
    // z_i = T_i p (Q / q_i)^-1 mod q_i, s = sum_i z_i (Q / q_i) - round(sum_i z_i / q_i) Q, and in p_a
    // y_a = T_a fpc_pq[a] + sum_i z_i fpq_c[i][a] + beta fpc_neg[a]
    u64 fpq_pz_w[EXACTO_MAX_L], fpq_pz_ws[EXACTO_MAX_L];  // p (Q / q_i)^-1 mod q_i (Shoup)
    double fpq_inv0[EXACTO_MAX_L], fpq_inv1[EXACTO_MAX_L]; // fl(1 / q_i), fl(2^30 / q_i)
    u64 fpq_c[EXACTO_MAX_L][EXACTO_MAX_K];                 // (p_a - q_i^-1 mod p_a) Pi_a
    int near;       // max prime < 2 * min prime: residues move between primes by one conditional subtraction
    int fast;       // near and every prime < 2^60: lazy CRT kernels (unreduced Shoup sums)
    int special;    // fast and every prime is 2^60 - d, d < 2^24: reduce_near60 instead of reduce64
    int digit_small;  // gadget base <= every ciphertext prime: digit magnitudes are already reduced
    u64 pmod_w[EXACTO_MAX_PRIMES], pmod_ws[EXACTO_MAX_PRIMES];  // plain mod prime_t
    u64 Qwords[EXACTO_MAX_L];                   // Q as little-endian 64-bit words
    u64 hq[EXACTO_MAX_PRIMES];                  // floor(Q/2) mod prime_t (decryption rounding)
    // HPS (single q, 1 or 2 aux primes), eval.rs:257-413
    u64 hps_qinv[2];        // q^-1 mod p_j
    u64 hps_p1_inv_p0, hps_p0_inv_p1;
    // division-free HPS scale (hps_scale_kernel FAST): every product by a constant as a Shoup product
    u64 hps_pc;             // floor(p 2^64 / q): the quotient estimate of round(p a / q), and p's Shoup companion mod q
    u64 hps_qinv_s[2];      // Shoup companions of hps_qinv (mod p_j)
    u64 hps_t_w[2], hps_t_ws[2];   // K = 2: q^-1 p1^-1 mod p0, q^-1 p0^-1 mod p1 (m's CRT coefficients, folded)
    u64 hps_pq_w[2], hps_pq_ws[2]; // K = 2: p1 mod q, p0 mod q
    u64 hps_kPq[3];         // K = 2: k P mod q, k = 0, 1, 2 (P = p0 p1)
    u64 hps_P[2], hps_halfP[2];    // K = 2: P and floor(P / 2) as (lo, hi)
};

// lazy: every prime of the batch is < 2^60 (forward NTT skips per-butterfly reductions)
// asm_fwd / asm_inv: every prime of the batch is in (2^60 - 2^32, 2^60): the forward / inverse
// transforms at n = 4096 / 8192 run the pinned-home kernels over the generated rounds (ntt_asm.inc)
// qbits: bit length of the batch's largest prime (the generic kernels' smaller-prime forms)
// one forward launch over two batches (n = 4096 / 8192, every prime 2^60 - d of the pinned rounds);
// false: not applicable, nothing launched
bool launch_ntt_fwd2(const NttBatch& nb1, int count1, const NttBatch& nb2, int count2, int logn,
                     const PrimeConst* primes, hipStream_t s);
void launch_ntt(const NttBatch& nb, int count, int logn, bool inverse, bool lazy, const PrimeConst* primes,
                hipStream_t s, bool asm_fwd = false, bool asm_inv = false, int qbits = 64);

void launch_shoup_companions(const u64* w, u64* ws, long count, int n, int L, const PrimeConst* primes,
                             hipStream_t s);

// ---- ks32.hip: relinearisation MAC over the integers in an auxiliary basis of 31-bit primes ----
#define EXACTO_KS32_MAXS 4
struct Prime32 {
    uint32_t p;                 // prime in (2^30, 2^31), p == 1 mod 2n
    uint32_t n_inv, n_inv_s;    // n^-1 and its Shoup companion floor(w 2^32 / p)
    uint32_t last_w, last_ws;   // psi_inv_rev[1] n^-1 (fused last inverse stage)
    uint32_t c32, c32s;         // 2^32 mod p
    uint32_t k63;               // (-2^63) mod p
    uint32_t fn_inv, fn_inv_s;  // n^-1 pi and last_w pi, pi = (P / p)^-1 mod p: the float-CRT lift's
    uint32_t flast_w, flast_ws; // inverse transforms fold its CRT factor into the last stage
    double inv_p;               // fl(1 / p)
    const uint2* tw_fwd;        // [n] {psi^brv(i), Shoup}
    const uint2* tw_inv;        // [n] {psi^-brv(i), Shoup}
};
struct Ks32Tables {
    uint32_t ginv[EXACTO_KS32_MAXS][EXACTO_KS32_MAXS];    // p_k^-1 mod p_s (k < s)
    uint32_t ginv_s[EXACTO_KS32_MAXS][EXACTO_KS32_MAXS];
    uint32_t halfP[EXACTO_KS32_MAXS];                     // mixed-radix digits of floor(P / 2)
    u64 pref_w[EXACTO_MAX_L][EXACTO_KS32_MAXS];           // (p_0 ... p_{s-1}) mod q_l
    u64 pref_ws[EXACTO_MAX_L][EXACTO_KS32_MAXS];
    u64 negP[EXACTO_MAX_L];                               // (q_l - P mod q_l) mod q_l
    uint32_t fpc_c[EXACTO_MAX_L][EXACTO_KS32_MAXS][2];     // (P / p_s) mod q_l in two 30-bit halves
    uint32_t fpc_n[EXACTO_MAX_L][2];                       // negP[l] in two 30-bit halves
};
// int16 digits [items][G][n] -> DS [items][G][S][n], NTT mod p_s
// form: the basis' butterfly form, 0 primes up to 2^31, 1 below 2^32 / 3, 2 below 2^30 (lazy)
// (ks32_dev.hpp F32_*; Ks32Basis::mac_form)
void ks32_digits(const int16_t* D16, uint32_t* DS, int items, int G, int S, int logn, const Prime32* primes,
                 int form, hipStream_t st);
void ks32_digits32(const int32_t* D, uint32_t* DS, int items, int G, int S, int logn, const Prime32* primes,
                   int form, hipStream_t st);
// key rows [rows][n] (coefficient domain, canonical mod q_{row % L}) -> RS [rows][S][n]
void ks32_key(const u64* K, uint32_t* RS, long rows, int L, int S, int logn, const Prime32* primes,
              const PrimeConst* qprimes, int form, hipStream_t st);
// per key row: sum_j floor(|balanced r_j| / 2^20) (the lazy basis' key-norm bound)
void ks32_key_norms(const u64* K, u64* out, long rows, int L, int n, const PrimeConst* qprimes, hipStream_t st);
// U [items][2L][S][n] = sum_g DS (.) RS
void ks32_mac(const uint32_t* DS, const uint32_t* RS, uint32_t* U, int items, int G, int L, int S, int n,
              const Prime32* primes, int mac_form, hipStream_t st);
// R[item][c][l] += centred lift of INTT(U[item][c][l][.]) mod q_l (every q_l = 2^60 - d, d < 2^24)
// fpc: the lift by a rounded float sum (ks32_dev.hpp ks32_fpc_one; taken when S <= 3 or the primes are
// below 2^32 / 3, and the caller checked the basis' fpc_max)
void ks32_crt(const uint32_t* U, u64* R, long r_stride, int items, int L, int S, int logn, const Ks32Tables* KT,
              const Prime32* primes, const PrimeConst* qprimes, int form, hipStream_t st, bool fpc = false);

// ---- kernels.hip launchers (all asynchronous on `s`) ----
struct Operands {            // two degree-1 ciphertext sources, [2][L][n] per item
    const u64* a;
    const u64* a_off;        // per-item element offsets (device) or nullptr -> item * a_stride
    long a_stride;
    const u64* b;
    const u64* b_off;
    long b_stride;
    // optional: the operands already extended to the auxiliary primes, forward-transformed,
    // [2][K][n] per ciphertext at ea + ea_off[item] / eb + eb_off[item] (shared by every product
    // that uses the ciphertext, dBFV); when set the pipeline skips steps 1-3
    const u64* ea;
    const u64* ea_off;
    const u64* eb;
    const u64* eb_off;
};

// Tensor product + inverse NTT of its three components, T[item][3][L+K][n] (ntt.hip).
// asm_inv: every prime is 2^60 - d with d < 2^24 and n = 4096 / 8192 (generated inverse rounds,
// special-prime products)
// out = INTT(NTT(A) (.) NTT(B)) row by row, one workgroup per row (n = 4096 / 8192 and primes
// 2^60 - d, d < 2^24 only; false = not launched)
bool launch_polymul(const u64* A, const u64* B, u64* out, long rows, int period, int logn, const PrimeConst* primes,
                    hipStream_t s);
// out = INTT(A (.) B) row by row ([rows][n], row r mod prime r % period); out may alias A or B
void launch_mul_inv(const u64* A, const u64* B, u64* out, long rows, int period, int logn, bool lazy, bool asm_inv,
                    const PrimeConst* primes, hipStream_t s);
// p2only: every component of the ciphertext primes, the third only of the auxiliary primes (dBFV
// psum; asm_inv and n = 4096 / 8192 only)
void launch_inv_tensor(const Operands& op, const u64* extP, u64* T, int items, int logn, int L, int K, bool lazy,
                       const PrimeConst* primes, hipStream_t s, bool asm_inv = false, bool p2only = false,
                       int qbits = 64, int share_np = 0, bool lazy_out = false);
// lazy_out (asm_inv only): T's residues in [0, 2q) instead of canonical -- for the exact path's
// scale kernels (shoup products and 30-bit-limb dot products), never for HPS
// Decryption (bfv/encrypt.rs:111-178, dbfv/decrypt.rs:20-79), kernels.hip.
void launch_phase(const u64* ct, int polys, long ct_stride, const u64* sk, u64* out, int items, int n, int L,
                  const PrimeConst* primes, hipStream_t s);
void launch_decrypt_round(const u64* X, u64* out, int items, int n, int L, const CrtTables* ct,
                          const PrimeConst* primes, u64 plain, hipStream_t s);
void launch_dbfv_recompose(const u64* digits, u64* out, int items, int n, int d, u64 base, u64 plain, u64 t,
                           bool scalar, hipStream_t s);
// rows = polynomials of coefQ ([rows][L][n] -> extP [rows][K][n])
void launch_exact_lift(const u64* coefQ, u64* extP, long rows, int n, const CrtTables* ct,
                       const PrimeConst* primes, int L, int K, int mode, hipStream_t s);
void launch_hps_extend(const u64* coefQ, u64* extP, long rows, int n, const PrimeConst* primes,
                       int K, hipStream_t s);
// D16 (or nullptr): gadget digits of the third component as int16 [item][g][n] instead of D;
// gshift: log2 of the gadget base (-1 if not a power of two), selects the digit code at launch
// the 30-bit-limb scale kernel (exact_scale_sp_kernel) serves these limb counts and CRT mode
bool exact_scale_sp_ok(int L, int K, int mode);
// c2only: the third component's rows alone (its gadget digits; dBFV psum, mode 3 with K = L + 1 only)
void launch_exact_scale(const u64* T, u64* R, long r_stride, int ncomp_r, u64* D, int16_t* D16, int guse,
                        int items, int n, const CrtTables* ct, const PrimeConst* primes, int L,
                        int K, int mode, hipStream_t s, int gshift = -1, bool c2only = false,
                        bool digits8 = false, bool fpc = false, double fpq_lim = 0.0);
// fpq_lim > 0 (with fpc): s = [p T]_Q centred by the float sum (fpq_y) wherever |f - round(f)| <= fpq_lim,
// Garner over Q elsewhere (0.5 - 2^-40: exact; smaller values only send more coefficients to Garner)
// D: digits as residues mod q [item][g][n]; D16 (instead): signed int16 (d8: int8) digits [item][g][n].
// fast: q > 2^32 and p < min(q, 2^32): the division-free form (bit-identical to the literal one)
void launch_hps_scale(const u64* T, u64* R, long r_stride, int ncomp_r, u64* D, void* D16, bool d8, int guse,
                      int items, int n, const CrtTables* ct, const PrimeConst* primes, int K, bool fast,
                      hipStream_t s);
// D16 != nullptr (gadget base <= 2^16): signed int16 digits [item][g][n] instead of residues
void launch_decompose(const u64* C2, long c2_stride, u64* D, int guse, int items, int n,
                      const CrtTables* ct, const PrimeConst* primes, int L, hipStream_t s, int16_t* D16 = nullptr);
// dst[r][k] = src ? src[r][k] : 0 over rows x len with the given row strides (u64 elements)
void launch_rows(u64* dst, long dst_stride, const u64* src, long src_stride, long len, long rows, hipStream_t s);
void launch_copy_u64(u64* dst, const u64* src, long words, hipStream_t s);
void launch_xcd_probe(const u64* src, u64* dst, long words, uint32_t* xcc, int blocks, hipStream_t s);
void launch_fill_u32(uint32_t* dst, uint32_t v, long words, hipStream_t s);
// EXACTO_DEBUG_BOOT: watch a byte range for writes by rows / copy / fill (kernels.hip DbgWatch); hit: a
// device buffer of 8 words, kind k set to 1 on a write inside [lo, hi); only launches on stream s from
// the calling host thread get it
void debug_watch_set(const void* lo, const void* hi, uint32_t* hit, hipStream_t s = nullptr);
void launch_relin_mac(const u64* base, long base_stride, const u64* D, const u64* rlk, const u64* rlk_s,
                      int guse, u64* out, long out_stride, int items, int n, int L, const PrimeConst* primes,
                      hipStream_t s);

enum class PwOp : int { Add = 0, Sub = 1, Neg = 2, Mul = 3, ScalarMul = 4, Copy = 5 };
void launch_pointwise(PwOp op, const u64* a, const u64* b, u64* out, long polys, int n, int L,
                      const u64* scalar_mod /*[L] or null*/, const PrimeConst* primes,
                      hipStream_t s);
void launch_bfv_addsub(bool sub, const u64* a, int p1, const u64* b, int p2, u64* out, long items, int n, int L,
                       const PrimeConst* primes, hipStream_t s);

struct CombineTerm {
    int pair;      // product index inside the item
    int pad_;
    i64 coef;      // signed small integer
};
void launch_dbfv_combine(const u64* prod, int npairs, const int* term_start,
                         const CombineTerm* terms, u64* out, int items, int d, int n, int L,
                         const PrimeConst* primes, hipStream_t s);
// dBFV psum (special primes, K = L + 1, n = 4096 / 8192): the auxiliary-prime residues of each output
// limb's c0 / c1 tensors summed over its products (NTT domain) into out [items_b][d][2][K][n]
// (ntt.hip), then inverse-transformed; exact_psum_sp_kernel: the scale of those sums plus the
// per-product corrections from the ciphertext-prime residues of T, the centred lift to Q, written to
// out [items_b][d][2][L][n] (coefficient domain, kernels.hip)
void launch_dbfv_pairsum(const Operands& op, u64* out, int items_b, int d, int npairs, const int* term_start,
                         const CombineTerm* terms, int L, int K, int n, const PrimeConst* primes, hipStream_t s);
bool launch_psum_scale(const u64* T, const u64* Tsum, u64* out, int items_b, int d, int npairs, const int* term_start,
                       const CombineTerm* terms, int n, const CrtTables* ct, const PrimeConst* primes, int L,
                       hipStream_t s, bool fpc = false, double fpq_lim = 0.0);
// dBFV: int16 gadget digits of the products of one output limb summed (combine terms with
// coefficient 1): D [item][pair][gu][n] -> out [item][k][gu][n], int16 or (wide) int32
// D: int16 digits, or int8 when in8 (base <= 2^8, exact_scale's digits8)
void ks32_digit_sum(const void* D, bool in8, int npairs, const int* term_start, const CombineTerm* terms, void* out,
                    bool wide, int items, int d, int gu, int n, hipStream_t st);

}  // namespace exacto

namespace exacto {
// ---- key generation / encryption (keygen.hip) ----
struct ChaChaKey { u64 w[4]; };
enum { KG_UNIFORM = 0, KG_TERNARY = 1, KG_BINARY = 2, KG_GAUSSIAN = 3 };
enum { KG_RLK = 0, KG_PK = 1, KG_ENC_SK = 2, KG_ENC_PK = 3, KG_GALOIS = 4 };
// sigma_k (keygen.rs:239-262) on coefficient-domain rows [item][poly][limb][n]; prime_fixed >= 0:
// every row is modulo that prime (limb index ignored)
void launch_automorph(const u64* in, long in_stride, u64* out, long out_stride, long items, int polys, int n, int L,
                      u64 k, const PrimeConst* primes, int prime_fixed, hipStream_t s);
void launch_lift_q0(const u64* v, u64* out, long rows, int n, int L, const PrimeConst* primes, hipStream_t s);
void launch_sample(int kind, const ChaChaKey& key, u64 nonce, u64* out, long out_stride, u64 poly_base,
                   u64 poly_step, long polys, int n, int L, const PrimeConst* primes, const double* cdt, int cdt_len,
                   int tail, double total, hipStream_t s);
void launch_scale_plain(const u64* pt, const u64* delta, u64* dm, long items, int n, int L, const PrimeConst* primes,
                        hipStream_t s);
void launch_combine(int op, u64* x, long items, long item_stride, long x1_off, const u64* s, const u64* aux,
                    const u64* aux2, const u64* pk, const u64* gpow, int n, int L, const PrimeConst* primes,
                    hipStream_t st);

// ---- plaintext-ciphertext operations (plain.hip) ----
enum { PLAIN_MUL = 0, PLAIN_ADD = 1 };
void launch_plain_apply(int op, const u64* x, long x_item_stride, u64* out, long items, int polys, const u64* pt,
                        long pt_item_stride, int n, int L, const PrimeConst* primes, hipStream_t s);
void launch_inner_product(const u64* cts, const u64* pts, u64* out, int K, int polys, int n, int L,
                          const PrimeConst* primes, hipStream_t s);
void launch_monomials(u64* out, long J, u64 j0, bool neg, int n, int L, const PrimeConst* primes, hipStream_t s);
void launch_axpy(u64* out, const u64* x, u64 a, long rows, int n, int L, const PrimeConst* primes, hipStream_t s);
void launch_modswitch(const u64* coef, u64* out, int* flags, long items, int n, u64 q, u64 qp, u64 tb, hipStream_t s);
void launch_boot_key_map(const u64* s, u64* boot_coef, u64* s_pt, int n, u64 q, u64 qb, u64 tb, hipStream_t st);
void launch_trivial_const(u64* out, long items, u64 m, const u64* delta, int n, int L, const PrimeConst* primes,
                          hipStream_t s);
}  // namespace exacto

namespace exacto {
// Every kernel launch of the library goes through EXACTO_LAUNCH, which records the launched kernel's
// host handle (thread-local) before the launch.  The profiler (ProfScope, exacto_prof_kernels) names
// what actually ran from it (dladdr + demangling: the rocprofv3 name), so no caller keeps a mirror of
// the library's kernel choices.
extern thread_local const void* g_last_kernel;
}  // namespace exacto
#define EXACTO_LAUNCH(K_, ...)                                                  \
    do {                                                                        \
        ::exacto::g_last_kernel = reinterpret_cast<const void*>(&(K_));         \
        hipLaunchKernelGGL(K_, __VA_ARGS__);                                    \
    } while (0)
