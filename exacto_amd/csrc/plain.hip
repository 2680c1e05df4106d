// Plaintext-ciphertext operations on the device (the linear layer under
// CoeffsToSlots): bfv_plain_mul, bfv_plain_add, bfv_inner_product, bfv_monomial_mul
// (bfv/eval.rs:468-503, 588-652).  All of them are coefficient-wise in the NTT domain once the
// plaintext is lifted into it, so each is one HBM-bound streaming pass over the ciphertexts:
//   plain_mul  : c_p <- c_p * NTT(pt mod q_i)                        (eval.rs:468-486)
//   plain_add  : c_0 <- c_0 + NTT(Delta * pt mod q_i)                 (eval.rs:489-503)
//   inner prod : sum_k c_{k,p} * NTT(pt_k mod q_i)                    (eval.rs:588-606)
//   monomial   : c_p <- c_p * NTT(X^j)  -- the reference's coefficient rotation with sign
//                (eval.rs:613-652) is multiplication by X^j in Z_q[X]/(X^n+1), which the NTT
//                diagonalises; per limb, rotating the CRT representative mod Q and reducing mod
//                q_i equals rotating the residue mod q_i, so this is bit-identical.
#include "exacto_internal.hpp"

namespace exacto {

static constexpr int PL_TPB = 256;

// rows [item][poly][limb][n] (x items x_item_stride apart, 0 = one ciphertext for every item);
// plaintext rows [item (or 0 when pt_item_stride == 0)][limb][n]
//   op PLAIN_MUL: out = x * pt      (every poly)
//   op PLAIN_ADD: out = x + pt on poly 0, x elsewhere
__global__ void __launch_bounds__(PL_TPB)
plain_apply_kernel(int op, const u64* __restrict__ x, long x_item_stride, u64* __restrict__ out, int polys,
                   const u64* __restrict__ pt, long pt_item_stride, int n, int L, const PrimeConst* __restrict__ primes) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;
    const int j = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (j >= n) return;
    const long pl = (long)polys * L;
    const long item = row / pl;
    const long r = row - item * pl;
    const int i = (int)(r % L);
    const int poly = (int)(r / L);
    const PrimeConst& P = primes[i];
    const long idx = row * n + j;
    const u64 v = x[item * x_item_stride + r * n + j];
    const u64 m = pt[item * pt_item_stride + (long)i * n + j];
    u64 res;
    if (op == PLAIN_MUL) res = mul_mod(v, m, P);
    else res = poly == 0 ? add_mod(v, m, P.q) : v;
    out[idx] = res;
}

void launch_plain_apply(int op, const u64* x, long x_item_stride, u64* out, long items, int polys, const u64* pt,
                        long pt_item_stride, int n, int L, const PrimeConst* primes, hipStream_t s) {
    const long blocks = items * polys * L * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(plain_apply_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, op, x, x_item_stride, out, polys,
                       pt, pt_item_stride, n, L, primes);
}

// out[poly][limb][j] = sum_k cts[k][poly][limb][j] * pts[k][limb][j]  (accumulated in the
// reference's order: acc = c_0 pt_0, then acc + c_k pt_k, every step reduced mod q_i)
__global__ void __launch_bounds__(PL_TPB)
inner_product_kernel(const u64* __restrict__ cts, const u64* __restrict__ pts, u64* __restrict__ out, int K,
                     int polys, int n, int L, const PrimeConst* __restrict__ primes) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;  // row = poly * L + limb
    const int j = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (j >= n) return;
    const int i = (int)(row % L);
    const PrimeConst& P = primes[i];
    const long ct_stride = (long)polys * L * n;
    const long Ln = (long)L * n;
    u64 acc = 0;
    for (int k = 0; k < K; ++k)
        acc = add_mod(acc, mul_mod(cts[k * ct_stride + row * n + j], pts[k * Ln + (long)i * n + j], P), P.q);
    out[row * n + j] = acc;
}

void launch_inner_product(const u64* cts, const u64* pts, u64* out, int K, int polys, int n, int L,
                          const PrimeConst* primes, hipStream_t s) {
    const long blocks = (long)polys * L * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0 || K == 0) return;
    EXACTO_LAUNCH(inner_product_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, cts, pts, out, K, polys, n,
                       L, primes);
}

// Monomials X^e mod (X^n + 1) as coefficient rows [J][L][n], item t: e = j mod 2n, or
// e = (2n - j) mod 2n (X^-j) when neg, with j = j0 + t: +1 at e (e < n) or q_i - 1 at e - n.
__global__ void __launch_bounds__(PL_TPB)
monomial_kernel(u64* __restrict__ out, u64 j0, int neg, int n, int L, const PrimeConst* __restrict__ primes) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;  // row = t * L + i
    const int c = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (c >= n) return;
    const u64 two_n = 2 * (u64)n;
    const u64 j = (j0 + (u64)(row / L)) % two_n;
    const u64 e = neg ? (two_n - j) % two_n : j;
    const u64 pos = e < (u64)n ? e : e - n;
    u64 v = 0;
    if ((u64)c == pos) v = e < (u64)n ? 1 : primes[row % L].q - 1;
    out[row * n + c] = v;
}

void launch_monomials(u64* out, long J, u64 j0, bool neg, int n, int L, const PrimeConst* primes, hipStream_t s) {
    const long blocks = J * L * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(monomial_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, out, j0, (int)neg, n, L, primes);
}

}  // namespace exacto

namespace exacto {

// out[row] += (a mod q_i) * x[row] over contiguous rows [rows][n], limb = row % L
// (bfv_scalar_mul + bfv_add, digit_extract.rs:131-140, 191-196)
__global__ void __launch_bounds__(PL_TPB)
axpy_kernel(u64* __restrict__ out, const u64* __restrict__ x, u64 a, int n, int L,
            const PrimeConst* __restrict__ primes) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;
    const int j = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (j >= n) return;
    const PrimeConst& P = primes[row % L];
    const long idx = row * n + j;
    out[idx] = add_mod(out[idx], mul_mod(x[idx], reduce64(a, P.q, P.mu64), P), P.q);
}

void launch_axpy(u64* out, const u64* x, u64 a, long rows, int n, int L, const PrimeConst* primes, hipStream_t s) {
    const long blocks = rows * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(axpy_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, out, x, a, n, L, primes);
}

// trivial encryptions of the constant m (digit_extract.rs:160-176): (Delta m, 0) per item, where the
// NTT of the constant polynomial Delta_i m is that constant in every slot.  out [items][2][L][n].
__global__ void __launch_bounds__(PL_TPB)
trivial_const_kernel(u64* __restrict__ out, u64 m, const u64* __restrict__ delta, int n, int L,
                     const PrimeConst* __restrict__ primes) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;  // row = (item * 2 + poly) * L + limb
    const int j = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (j >= n) return;
    const int i = (int)(row % L);
    const int poly = (int)((row / L) % 2);
    const PrimeConst& P = primes[i];
    out[row * n + j] = poly == 0 ? mul_mod(reduce64(m, P.q, P.mu64), delta[i], P) : 0;
}

void launch_trivial_const(u64* out, long items, u64 m, const u64* delta, int n, int L, const PrimeConst* primes,
                          hipStream_t s) {
    const long blocks = items * 2 * L * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(trivial_const_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, out, m, delta, n, L, primes);
}

}  // namespace exacto

namespace exacto {

// bfv_host.rs:149-170: modulus switch of coefficient rows [items][2][n] (mod q) to
// ((q' c + q/2) / q) mod q' mod t_boot; flags[item] = 1 when c1 has a nonzero coefficient (the
// reference's is_trivial test, bfv_host.rs:180).
__global__ void __launch_bounds__(PL_TPB)
modswitch_kernel(const u64* __restrict__ coef, u64* __restrict__ out, int* __restrict__ flags, int n, u64 q, u64 qp,
                 u64 tb) {
    const int nblk = (n + PL_TPB - 1) / PL_TPB;
    const long row = blockIdx.x / nblk;  // row = item * 2 + poly
    const int j = (blockIdx.x - row * nblk) * PL_TPB + threadIdx.x;
    if (j >= n) return;
    const u64 c = coef[row * n + j];
    const u64 v = (u64)(((u128)qp * c + q / 2) / q);
    out[row * n + j] = v % qp % tb;
    if ((row & 1) && c != 0) atomicOr(&flags[row >> 1], 1);
}

void launch_modswitch(const u64* coef, u64* out, int* flags, long items, int n, u64 q, u64 qp, u64 tb, hipStream_t s) {
    const long blocks = items * 2 * ((n + PL_TPB - 1) / PL_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(modswitch_kernel, dim3((unsigned)blocks), dim3(PL_TPB), 0, s, coef, out, flags, n, q, qp, tb);
}

// gen_bootstrap_key's two images of the ternary secret s (coefficients mod q_orig):
//   boot_coef: create_boot_sk's map into Z_{q_boot}    (bfv_host.rs:296-315)
//   s_pt     : the plaintext encrypted as the key      (bfv_host.rs:68-86)
__global__ void __launch_bounds__(PL_TPB)
boot_key_map_kernel(const u64* __restrict__ s, u64* __restrict__ boot_coef, u64* __restrict__ s_pt, int n, u64 q,
                    u64 qb, u64 tb) {
    const int i = blockIdx.x * PL_TPB + threadIdx.x;
    if (i >= n) return;
    const u64 c = s[i];
    u64 b;
    if (c == 0) b = 0;
    else if (c <= q / 2) b = c % qb;
    else b = qb - (q - c) % qb;
    boot_coef[i] = b;
    u64 p;
    if (c == 0) p = 0;
    else if (c == 1) p = 1;
    else if (c == q - 1) p = tb - 1;
    else if (c > q / 2) p = tb - (q - c) % tb;
    else p = c % tb;
    s_pt[i] = p;
}

void launch_boot_key_map(const u64* s, u64* boot_coef, u64* s_pt, int n, u64 q, u64 qb, u64 tb, hipStream_t st) {
    EXACTO_LAUNCH(boot_key_map_kernel, dim3((unsigned)((n + PL_TPB - 1) / PL_TPB)), dim3(PL_TPB), 0, st, s,
                       boot_coef, s_pt, n, q, qb, tb);
}

}  // namespace exacto
