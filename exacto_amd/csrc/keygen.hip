// Key generation and encryption on the device: samplers and the
// coefficient-wise combinations of bfv/keygen.rs:64-162 and bfv/encrypt.rs:29-106, 181-229.
//
// Sampling semantics follow the reference literally (sampling/uniform.rs, sampling/gaussian.rs):
// every polynomial is sampled as a CoeffPoly modulo the FIRST ciphertext prime q0 and then
// reduced modulo each q_i (RnsPoly::from_coeff_poly), so for L > 1 a "-1" is q0 - 1 in every limb.
//   uniform : v = r & mask (mask = 2^bitlen(q0) - 1), rejected until v < q0   (uniform.rs:8-22)
//   ternary : r = byte & 3, 3 rejected; 0 -> q0 - 1, 1 -> 0, 2 -> 1          (uniform.rs:25-41)
//   binary  : r & 1                                                            (uniform.rs:44-49)
//   gaussian: inverse CDT over [-ceil(6 sigma), ceil(6 sigma)] with unnormalised weights
//             exp(-x^2 / 2 sigma^2), u = f64 in [0,1) * total; x >= 0 -> x mod q0, else
//             (q0 + x % q0) % q0                                               (gaussian.rs:5-46)
// The random words come from ChaCha20 (the reference's ChaCha20Rng primitive) in counter mode:
// key = the caller's 256-bit key, nonce = the caller's stream id, 64-bit block counter =
// (polynomial index << 32) | (coefficient * 4 + retry block).  The stream of words is this
// library's own (the reference's RNG stream is not reproducible here and not needed: the hot path
// is deterministic given its inputs); parity is checked at decryption level and statistically.
#include "exacto_internal.hpp"

namespace exacto {

static constexpr int KG_TPB = 256;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define CHACHA_QR(a, b, c, d)            \
    a += b; d ^= a; d = rotl32(d, 16);   \
    c += d; b ^= c; b = rotl32(b, 12);   \
    a += b; d ^= a; d = rotl32(d, 8);    \
    c += d; b ^= c; b = rotl32(b, 7);

// One ChaCha20 block (DJB layout: 64-bit counter, 64-bit nonce) as 8 little-endian u64 words.
__device__ void chacha20_block(const ChaChaKey& k, u64 nonce, u64 counter, u64 (&out)[8]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s[4 + 2 * i] = (uint32_t)k.w[i];
        s[5 + 2 * i] = (uint32_t)(k.w[i] >> 32);
    }
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32);
    s[14] = (uint32_t)nonce; s[15] = (uint32_t)(nonce >> 32);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        CHACHA_QR(x[0], x[4], x[8], x[12]);
        CHACHA_QR(x[1], x[5], x[9], x[13]);
        CHACHA_QR(x[2], x[6], x[10], x[14]);
        CHACHA_QR(x[3], x[7], x[11], x[15]);
        CHACHA_QR(x[0], x[5], x[10], x[15]);
        CHACHA_QR(x[1], x[6], x[11], x[12]);
        CHACHA_QR(x[2], x[7], x[8], x[13]);
        CHACHA_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = (u64)(x[2 * i] + s[2 * i]) | ((u64)(x[2 * i + 1] + s[2 * i + 1]) << 32);
}

// One sampled coefficient in the reference's CoeffPoly mod q0.  Retry blocks are bounded
// (4 blocks = 32 words / 256 bytes; the chance of exhausting them is < 2^-200 for uniform with
// q0 > 2^(bitlen-1), and 4^-256 for ternary); the last candidate is then kept reduced.
__device__ u64 sample_coeff(int kind, const ChaChaKey& key, u64 nonce, u64 poly, int j, u64 q0, u64 mask,
                            const double* __restrict__ cdt, int cdt_len, int tail, double total) {
    u64 w[8];
    const u64 ctr0 = (poly << 32) | ((u64)j * 4);
    chacha20_block(key, nonce, ctr0, w);
    if (kind == KG_BINARY) return w[0] & 1;
    if (kind == KG_GAUSSIAN) {
        const double u = (double)(w[0] >> 11) * 0x1.0p-53 * total;  // rand's f64: 53 random bits
        int idx = cdt_len - 1;
        for (int i = cdt_len - 1; i >= 0; --i)
            if (u < cdt[i]) idx = i;
        const i64 x = (i64)idx - tail;
        const i64 m = (i64)q0;
        return x >= 0 ? (u64)x % q0 : (u64)((m + (x % m)) % m);
    }
    for (int b = 0; b < 4; ++b) {
        if (b > 0) chacha20_block(key, nonce, ctr0 + b, w);
        if (kind == KG_UNIFORM) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const u64 v = w[i] & mask;
                if (v < q0) return v;
            }
        } else {  // ternary
            for (int i = 0; i < 64; ++i) {
                const uint32_t r = (uint32_t)(w[i >> 3] >> (8 * (i & 7))) & 3u;
                if (r < 3) return r == 0 ? q0 - 1 : (u64)(r - 1);
            }
        }
    }
    return kind == KG_UNIFORM ? (w[7] & mask) % q0 : 0;
}

// out[p][i][j] = sample(poly_base + p * poly_step, j) mod q_i, polynomials p at out + p * out_stride.
__global__ void __launch_bounds__(KG_TPB)
sample_kernel(int kind, ChaChaKey key, u64 nonce, u64* __restrict__ out, long out_stride, u64 poly_base,
              u64 poly_step, int n, int L, const PrimeConst* __restrict__ primes, const double* __restrict__ cdt,
              int cdt_len, int tail, double total) {
    const int nblk = (n + KG_TPB - 1) / KG_TPB;
    const long p = blockIdx.x / nblk;
    const int j = (blockIdx.x - p * nblk) * KG_TPB + threadIdx.x;
    if (j >= n) return;
    const u64 q0 = primes[0].q;
    const u64 mask = q0 >> 63 ? ~0ull : ((u64)1 << (64 - __clzll(q0))) - 1;
    const u64 v = sample_coeff(kind, key, nonce, poly_base + (u64)p * poly_step, j, q0, mask, cdt, cdt_len, tail,
                               total);
    u64* o = out + p * out_stride + j;
    for (int i = 0; i < L; ++i) o[(long)i * n] = (i == 0) ? v : reduce64(v, primes[i].q, primes[i].mu64);
}

void launch_sample(int kind, const ChaChaKey& key, u64 nonce, u64* out, long out_stride, u64 poly_base,
                   u64 poly_step, long polys, int n, int L, const PrimeConst* primes, const double* cdt, int cdt_len,
                   int tail, double total, hipStream_t s) {
    const long blocks = polys * ((n + KG_TPB - 1) / KG_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(sample_kernel, dim3((unsigned)blocks), dim3(KG_TPB), 0, s, kind, key, nonce, out, out_stride,
                       poly_base, poly_step, n, L, primes, cdt, cdt_len, tail, total);
}

// Delta*m (encrypt.rs:181-201): dm[b][i][j] = (pt[b][j] mod q_i) * Delta_i mod q_i, coefficient domain.
__global__ void __launch_bounds__(KG_TPB)
scale_plain_kernel(const u64* __restrict__ pt, const u64* __restrict__ delta, u64* __restrict__ dm, int n, int L,
                   const PrimeConst* __restrict__ primes) {
    const int nblk = (n + KG_TPB - 1) / KG_TPB;
    const long row = blockIdx.x / nblk;  // row = b * L + i
    const int j = (blockIdx.x - row * nblk) * KG_TPB + threadIdx.x;
    if (j >= n) return;
    const long b = row / L;
    const int i = (int)(row - b * L);
    const PrimeConst& P = primes[i];
    const u64 m = reduce64(pt[b * n + j], P.q, P.mu64);
    dm[row * n + j] = delta ? mul_mod(m, delta[i], P) : m;  // delta == nullptr: plain lift
}

void launch_scale_plain(const u64* pt, const u64* delta, u64* dm, long items, int n, int L, const PrimeConst* primes,
                        hipStream_t s) {
    const long blocks = items * L * ((n + KG_TPB - 1) / KG_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(scale_plain_kernel, dim3((unsigned)blocks), dim3(KG_TPB), 0, s, pt, delta, dm, n, L, primes);
}

// NTT-domain combinations, one thread per (item, limb, coefficient); polynomials [L][n] per item.
//   KG_RLK : x0 <- -(x1*s + x0) + s^2 * base^key  (rlk_i = (-(a_i s + e_i) + g_i s^2, a_i): x0 holds e_i,
//            x1 holds a_i; gpow[key * L + i] = base^key mod q_i)                       keygen.rs:137-155
//   KG_PK  : x0 <- -(x1*s + x0)                     (pk = (-(a s + e), a))             keygen.rs:98-110
//   KG_ENC_SK: x0 <- -(x1*s) + x0 + dm              (ct = (-a s + e + Delta m, a))     encrypt.rs:92-105
//   KG_ENC_PK: x0 <- pk0*u + x0 + dm, x1 <- pk1*u + x1  (x0, x1 hold e1, e2)           encrypt.rs:44-69
// u and dm are [item][L][n] (NTT domain): u = aux, dm = aux (ENC_SK) or aux2 (ENC_PK).
__global__ void __launch_bounds__(KG_TPB)
combine_kernel(int op, u64* __restrict__ x, long item_stride, long x1_off, const u64* __restrict__ s,
               const u64* __restrict__ aux, const u64* __restrict__ aux2, const u64* __restrict__ pk,
               const u64* __restrict__ gpow, int n, int L, const PrimeConst* __restrict__ primes) {
    const int nblk = (n + KG_TPB - 1) / KG_TPB;
    const long row = blockIdx.x / nblk;  // row = item * L + i
    const int j = (blockIdx.x - row * nblk) * KG_TPB + threadIdx.x;
    if (j >= n) return;
    const long item = row / L;
    const int i = (int)(row - item * L);
    const PrimeConst& P = primes[i];
    const u64 q = P.q;
    const long li = (long)i * n + j;
    u64* x0 = x + item * item_stride + li;
    u64* x1 = x0 + x1_off;
    const long Ln = (long)L * n;
    if (op == KG_ENC_PK) {
        const u64 u = aux[item * Ln + li];
        const u64 dm = aux2[item * Ln + li];
        *x0 = add_mod(add_mod(mul_mod(pk[li], u, P), *x0, q), dm, q);
        *x1 = add_mod(mul_mod(pk[(long)L * n + li], u, P), *x1, q);
        return;
    }
    const u64 sv = s[li];
    const u64 as = mul_mod(*x1, sv, P);
    if (op == KG_ENC_SK) {
        *x0 = add_mod(add_mod(neg_mod(as, q), *x0, q), aux[item * Ln + li], q);
        return;
    }
    u64 r = neg_mod(add_mod(as, *x0, q), q);
    if (op == KG_RLK) r = add_mod(r, mul_mod(mul_mod(sv, sv, P), gpow[item * L + i], P), q);
    if (op == KG_GALOIS) r = add_mod(r, mul_mod(aux[li], gpow[item * L + i], P), q);  // aux = s(X^k)
    *x0 = r;
}

void launch_combine(int op, u64* x, long items, long item_stride, long x1_off, const u64* s, const u64* aux,
                    const u64* aux2, const u64* pk, const u64* gpow, int n, int L, const PrimeConst* primes,
                    hipStream_t st) {
    const long blocks = items * L * ((n + KG_TPB - 1) / KG_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(combine_kernel, dim3((unsigned)blocks), dim3(KG_TPB), 0, st, op, x, item_stride, x1_off, s, aux,
                       aux2, pk, gpow, n, L, primes);
}

// ---------------------------------------------------------------- Galois automorphisms

// sigma_k on coefficient-domain residues (keygen.rs:239-262), odd k: a signed permutation, as a
// gather: out[j] = +in[t] if t = j * k^-1 mod 2n < n, else -in[t - n].  rows = [item][poly][limb].
__global__ void __launch_bounds__(KG_TPB)
automorph_kernel(const u64* __restrict__ in, long in_stride, u64* __restrict__ out, long out_stride, int polys,
                 int n, int L, u64 kinv, const PrimeConst* __restrict__ primes, int prime_fixed) {
    const int nblk = (n + KG_TPB - 1) / KG_TPB;
    const long row = blockIdx.x / nblk;
    const int j = (blockIdx.x - row * nblk) * KG_TPB + threadIdx.x;
    if (j >= n) return;
    const long pl = (long)polys * L;
    const long item = row / pl;
    const long r = row - item * pl;
    const int i = (int)(r % L);
    const u64 q = primes[prime_fixed >= 0 ? prime_fixed : i].q;
    const u64 t = ((u64)j * kinv) % (2 * (u64)n);
    const u64 v = in[item * in_stride + r * n + (t < (u64)n ? t : t - n)];
    out[item * out_stride + r * n + j] = t < (u64)n ? v : neg_mod(v, q);
}

// even k (not an automorphism of the ring; the reference computes it anyway): the literal
// accumulation, one thread per row.  out must be zeroed.
__global__ void automorph_serial_kernel(const u64* __restrict__ in, long in_stride, u64* __restrict__ out,
                                        long out_stride, int polys, int n, int L, u64 k, long rows,
                                        const PrimeConst* __restrict__ primes, int prime_fixed) {
    const long row = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= rows) return;
    const long pl = (long)polys * L;
    const long item = row / pl;
    const long r = row - item * pl;
    const int i = (int)(r % L);
    const u64 q = primes[prime_fixed >= 0 ? prime_fixed : i].q;
    const u64* a = in + item * in_stride + r * n;
    u64* o = out + item * out_stride + r * n;
    for (int c = 0; c < n; ++c) {
        if (a[c] == 0) continue;
        const u64 e = ((u64)c * k) % (2 * (u64)n);
        if (e < (u64)n) o[e] = add_mod(o[e], a[c], q);
        else o[e - n] = sub_mod(o[e - n], a[c], q);
    }
}

void launch_automorph(const u64* in, long in_stride, u64* out, long out_stride, long items, int polys, int n, int L,
                      u64 k, const PrimeConst* primes, int prime_fixed, hipStream_t s) {
    const u64 two_n = 2 * (u64)n;
    k %= two_n;
    const long rows = items * polys * L;
    if (rows == 0) return;
    if (k & 1) {
        u64 kinv = 1;  // k^-1 mod 2n by Newton iteration (2n is a power of two)
        for (int it = 0; it < 7; ++it) kinv = kinv * (2 - k * kinv);
        kinv &= two_n - 1;
        const long blocks = rows * ((n + KG_TPB - 1) / KG_TPB);
        EXACTO_LAUNCH(automorph_kernel, dim3((unsigned)blocks), dim3(KG_TPB), 0, s, in, in_stride, out,
                           out_stride, polys, n, L, kinv, primes, prime_fixed);
    } else {
        launch_rows(out, out_stride, nullptr, 0, (long)polys * L * n, items, s);
        EXACTO_LAUNCH(automorph_serial_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, s, in,
                           in_stride, out, out_stride, polys, n, L, k, rows, primes, prime_fixed);
    }
}

// v (canonical mod q0, [rows][n]) -> [rows][L][n] residues mod each q_i (RnsPoly::from_coeff_poly)
__global__ void __launch_bounds__(KG_TPB)
lift_q0_kernel(const u64* __restrict__ v, u64* __restrict__ out, int n, int L, const PrimeConst* __restrict__ primes) {
    const int nblk = (n + KG_TPB - 1) / KG_TPB;
    const long row = blockIdx.x / nblk;
    const int j = (blockIdx.x - row * nblk) * KG_TPB + threadIdx.x;
    if (j >= n) return;
    const u64 x = v[row * n + j];
    for (int i = 0; i < L; ++i)
        out[(row * L + i) * n + j] = i == 0 ? x : reduce64(x, primes[i].q, primes[i].mu64);
}

void launch_lift_q0(const u64* v, u64* out, long rows, int n, int L, const PrimeConst* primes, hipStream_t s) {
    const long blocks = rows * ((n + KG_TPB - 1) / KG_TPB);
    if (blocks == 0) return;
    EXACTO_LAUNCH(lift_q0_kernel, dim3((unsigned)blocks), dim3(KG_TPB), 0, s, v, out, n, L, primes);
}

}  // namespace exacto
