/* oracle.c — C restatement of the reference's multiplication path (TEST ORACLE / CPU BASELINE).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and by bench.py's cpu_baseline leg, never by the
 * product path.  It restates, with fixed-width multiword integers in place of num-bigint:
 *   ring/ntt.rs:42-67      forward / inverse+normalize NTT (this build's documented convention,
 *                          identical to oracle/ring.py NttPlan)
 *   bfv/eval.rs:113-147    bfv_mul_generic_rns: exact centred CRT lift, O(n^2) BigInt schoolbook
 *                          negacyclic tensor (eval.rs:794-810), scale-and-round (816-831)
 *   bfv/eval.rs:157-413    bfv_mul_hps literally (1 or 2 aux primes)
 *   bfv/eval.rs:416-454    bfv_mul_schoolbook (exact; overflow guard checked by the caller)
 *   bfv/keyswitch.rs:11-101 gadget_decompose + relinearize (exact CRT; extension semantics for
 *                          Q >= 2^64 as documented in oracle/__init__.py)
 * Layout as include/exacto_hip.h: [B][poly][limb][n] uint64, NTT domain.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef uint64_t u64;
typedef uint32_t u32;
typedef unsigned __int128 u128;
typedef __int128 i128;
typedef int64_t i64;

#define MAXL 8
#define MAXW 20 /* multiword accumulator words */

/* ------------------------------------------------------------------ modular helpers */
static u64 mulmod(u64 a, u64 b, u64 m) { return (u64)((u128)a * b % m); }
static u64 powmod(u64 b, u64 e, u64 m) {
    u64 r = 1 % m;
    b %= m;
    while (e) {
        if (e & 1) r = mulmod(r, b, m);
        b = mulmod(b, b, m);
        e >>= 1;
    }
    return r;
}
static u64 invmod(u64 a, u64 m) { /* extended Euclid (modular.rs:102-121) */
    i128 t = 0, nt = 1, r = m, nr = a % m;
    while (nr) {
        i128 q = r / nr, tmp;
        tmp = t - q * nt; t = nt; nt = tmp;
        tmp = r - q * nr; r = nr; nr = tmp;
    }
    if (r != 1) return 0;
    if (t < 0) t += m;
    return (u64)t;
}
/* reference mod_mul literally (modular.rs:7-19, 81-84) */
static u64 ref_mod_mul(u64 a, u64 b, u64 m) {
    u128 prod = (u128)a * b;
    if (m > (1ull << 32)) return (u64)(prod % m);
    u64 k = (u64)(((u128)1 << 64) / m);
    u64 qh = (u64)((prod * (u128)k) >> 64);
    u64 r = (u64)prod - qh * m;
    return r >= m ? r - m : r;
}

/* ------------------------------------------------------------------ NTT plan */
typedef struct {
    int n, logn;
    u64 q, n_inv;
    u64 *fwd, *inv; /* psi^brv(i), psi^-brv(i) */
} plan_t;

static int brv(int x, int bits) {
    int r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

static void plan_init(plan_t* p, int n, u64 q) {
    p->n = n;
    p->q = q;
    p->logn = 0;
    while ((1 << p->logn) < n) p->logn++;
    u64 e = (q - 1) / (2 * (u64)n), psi = 0;
    for (u64 x = 2;; ++x) {
        psi = powmod(x, e, q);
        if (powmod(psi, n, q) == q - 1) break;
    }
    u64 psi_inv = invmod(psi, q);
    p->fwd = (u64*)malloc(sizeof(u64) * n);
    p->inv = (u64*)malloc(sizeof(u64) * n);
    for (int i = 0; i < n; ++i) {
        p->fwd[i] = powmod(psi, brv(i, p->logn), q);
        p->inv[i] = powmod(psi_inv, brv(i, p->logn), q);
    }
    p->n_inv = invmod((u64)n % q, q);
}
static void plan_free(plan_t* p) { free(p->fwd); free(p->inv); }

/* NTT-domain storage order (oracle/ring.py NttPlan.storage_order): evaluation k
   (bit-reversed order) at position (k mod 16) n/16 + k / 16; the identity at n = 16 */
static void ntt_store_order(u64* a, int n, int to_storage) {
    const int T = n / 16;
    if (T <= 1) return;
    u64* tmp = (u64*)malloc(sizeof(u64) * (size_t)n);
    memcpy(tmp, a, sizeof(u64) * (size_t)n);
    for (int k = 0; k < n; ++k) {
        const int pos = (k & 15) * T + (k >> 4);
        if (to_storage) a[pos] = tmp[k];
        else a[k] = tmp[pos];
    }
    free(tmp);
}

static void ntt_fwd(const plan_t* p, u64* a) {
    const int n = p->n;
    const u64 q = p->q;
    int t = n;
    for (int m = 1; m < n; m <<= 1) {
        t >>= 1;
        for (int i = 0; i < m; ++i) {
            const u64 s = p->fwd[m + i];
            for (int j = 2 * i * t; j < 2 * i * t + t; ++j) {
                u64 u = a[j], v = mulmod(a[j + t], s, q);
                a[j] = u + v >= q ? u + v - q : u + v;
                a[j + t] = u >= v ? u - v : u + q - v;
            }
        }
    }
    ntt_store_order(a, n, 1);
}
static void ntt_inv(const plan_t* p, u64* a) { /* inv + normalize */
    const int n = p->n;
    const u64 q = p->q;
    int t = 1;
    ntt_store_order(a, n, 0);
    for (int m = n; m > 1; m >>= 1) {
        const int h = m >> 1;
        int j1 = 0;
        for (int i = 0; i < h; ++i) {
            const u64 s = p->inv[h + i];
            for (int j = j1; j < j1 + t; ++j) {
                u64 u = a[j], v = a[j + t];
                a[j] = u + v >= q ? u + v - q : u + v;
                a[j + t] = mulmod(u >= v ? u - v : u + q - v, s, q);
            }
            j1 += 2 * t;
        }
        t <<= 1;
    }
    for (int i = 0; i < n; ++i) a[i] = mulmod(a[i], p->n_inv, q);
}

/* ------------------------------------------------------------------ multiword (W words, two's complement) */
typedef struct { u64 w[MAXW]; } mw_t;

static void mw_zero(mw_t* x, int W) { memset(x->w, 0, sizeof(u64) * W); }
static int mw_neg_p(const mw_t* x, int W) { return (int)(x->w[W - 1] >> 63); }
static void mw_negate(mw_t* x, int W) {
    u64 c = 1;
    for (int i = 0; i < W; ++i) { u64 v = ~x->w[i] + c; c = (c && v == 0); x->w[i] = v; }
}
static void mw_add_mag(mw_t* acc, const u64* m, int mw, int W, int subtract) {
    /* acc +=/-= m (m: magnitude of mw words) */
    if (!subtract) {
        u64 c = 0;
        for (int i = 0; i < W; ++i) {
            u128 s = (u128)acc->w[i] + (i < mw ? m[i] : 0) + c;
            acc->w[i] = (u64)s;
            c = (u64)(s >> 64);
        }
    } else {
        u64 b = 0;
        for (int i = 0; i < W; ++i) {
            u64 mi = i < mw ? m[i] : 0;
            u128 d = (u128)acc->w[i] - mi - b;
            acc->w[i] = (u64)d;
            b = (u64)(d >> 64) ? 1 : 0;
        }
    }
}
/* magnitude product of L-word numbers -> 2L words */
static void mag_mul(u64* out, const u64* a, const u64* b, int L) {
    memset(out, 0, sizeof(u64) * 2 * L);
    for (int i = 0; i < L; ++i) {
        u64 c = 0;
        for (int j = 0; j < L; ++j) {
            u128 t = (u128)a[i] * b[j] + out[i + j] + c;
            out[i + j] = (u64)t;
            c = (u64)(t >> 64);
        }
        out[i + L] = c;
    }
}

/* Knuth algorithm D on 32-bit digits: q = u / v, u has m digits, v has nn digits (v[nn-1] != 0) */
static void divmnu(u32* q, const u32* u, int m, const u32* v, int nn) {
    if (nn == 1) {
        u64 k = 0;
        for (int j = m - 1; j >= 0; --j) { u64 cur = (k << 32) | u[j]; q[j] = (u32)(cur / v[0]); k = cur % v[0]; }
        return;
    }
    int s = __builtin_clz(v[nn - 1]);
    u32 vn[2 * MAXW * 2], un[2 * MAXW * 2 + 1];
    for (int i = nn - 1; i > 0; --i) vn[i] = (v[i] << s) | (s ? (u32)((u64)v[i - 1] >> (32 - s)) : 0);
    vn[0] = v[0] << s;
    un[m] = s ? (u32)((u64)u[m - 1] >> (32 - s)) : 0;
    for (int i = m - 1; i > 0; --i) un[i] = (u[i] << s) | (s ? (u32)((u64)u[i - 1] >> (32 - s)) : 0);
    un[0] = u[0] << s;
    for (int j = m - nn; j >= 0; --j) {
        u64 num = ((u64)un[j + nn] << 32) | un[j + nn - 1];
        u64 qhat = num / vn[nn - 1], rhat = num % vn[nn - 1];
        while (qhat >= (1ull << 32) || qhat * vn[nn - 2] > ((rhat << 32) | un[j + nn - 2])) {
            qhat--;
            rhat += vn[nn - 1];
            if (rhat >= (1ull << 32)) break;
        }
        int64_t k = 0, t;
        for (int i = 0; i < nn; ++i) {
            u64 p = qhat * vn[i];
            t = (int64_t)un[i + j] - k - (int64_t)(p & 0xFFFFFFFFull);
            un[i + j] = (u32)t;
            k = (int64_t)(p >> 32) - (t >> 32);
        }
        t = (int64_t)un[j + nn] - k;
        un[j + nn] = (u32)t;
        q[j] = (u32)qhat;
        if (t < 0) {
            q[j]--;
            u64 c = 0;
            for (int i = 0; i < nn; ++i) {
                u64 s2 = (u64)un[i + j] + vn[i] + c;
                un[i + j] = (u32)s2;
                c = s2 >> 32;
            }
            un[j + nn] += (u32)c;
        }
    }
}

/* magnitude (words) mod a u64 */
static u64 mag_mod(const u64* x, int W, u64 m) {
    u128 r = 0;
    for (int i = W - 1; i >= 0; --i) r = ((r << 64) | x[i]) % m;
    return (u64)r;
}

/* ------------------------------------------------------------------ context */
typedef struct {
    int n, L, K;         /* K = HPS aux count (0 for exact / schoolbook) */
    u64 q[MAXL], aux[2];
    u64 plain, gbase;
    int G;
    plan_t plan[MAXL], aplan[2];
    u64 Q[MAXL];         /* Q words (L words) */
    u64 halfQ[MAXL];     /* floor(Q/2) words */
    u64 crt_term[MAXL][MAXL]; /* (Q/q_i) * inv_i as L words */
} octx_t;


/* exact CRT of residues -> value in [0,Q) as L words (rns.rs:138-148 / eval.rs:719-762) */
static void crt(const octx_t* c, const u64* res, u64* out /* L words */) {
    const int L = c->L;
    u64 acc[MAXL + 2];
    memset(acc, 0, sizeof(acc));
    for (int i = 0; i < L; ++i) {
        /* acc += res_i * crt_term_i  (crt_term < Q * q_i -> fits L+1 words) */
        u64 cc = 0;
        for (int w = 0; w < L + 1; ++w) {
            u64 t_w = w < L ? c->crt_term[i][w] : 0;
            u128 t = (u128)res[i] * t_w + acc[w] + cc;
            acc[w] = (u64)t;
            cc = (u64)(t >> 64);
        }
        acc[L + 1] += cc;
    }
    /* acc mod Q: acc < L * q * Q -> subtract via division */
    u32 u[2 * (MAXL + 2)], v[2 * MAXL], qq[2 * (MAXL + 2)];
    int m = 2 * (L + 2), nn = 2 * L;
    for (int w = 0; w < L + 2; ++w) { u[2 * w] = (u32)acc[w]; u[2 * w + 1] = (u32)(acc[w] >> 32); }
    for (int w = 0; w < L; ++w) { v[2 * w] = (u32)c->Q[w]; v[2 * w + 1] = (u32)(c->Q[w] >> 32); }
    while (nn > 1 && v[nn - 1] == 0) nn--;
    divmnu(qq, u, m, v, nn);
    /* r = acc - qq*Q */
    u64 qw[MAXL + 3];
    memset(qw, 0, sizeof(qw));
    for (int i = 0; i <= m - nn; ++i) qw[i / 2] |= (u64)qq[i] << (32 * (i & 1));
    u64 prod[2 * MAXL + 4];
    memset(prod, 0, sizeof(prod));
    for (int i = 0; i < L + 2; ++i) {
        u64 cc = 0;
        for (int j = 0; j < L; ++j) {
            if (i + j >= 2 * MAXL + 4) break;
            u128 t = (u128)qw[i] * c->Q[j] + prod[i + j] + cc;
            prod[i + j] = (u64)t;
            cc = (u64)(t >> 64);
        }
        if (i + L < 2 * MAXL + 4) prod[i + L] += cc;
    }
    u64 b = 0;
    for (int w = 0; w < L; ++w) {
        u128 d = (u128)acc[w] - prod[w] - b;
        out[w] = (u64)d;
        b = (u64)(d >> 64) ? 1 : 0;
    }
}

static int cmp_words(const u64* a, const u64* b, int L) {
    for (int i = L - 1; i >= 0; --i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return 0;
}

/* centred signed value: sign + L-word magnitude */
static void centre(const octx_t* c, const u64* x, u64* mag, int* neg) {
    const int L = c->L;
    if (cmp_words(x, c->halfQ, L) > 0) {
        u64 b = 0;
        for (int w = 0; w < L; ++w) {
            u128 d = (u128)c->Q[w] - x[w] - b;
            mag[w] = (u64)d;
            b = (u64)(d >> 64) ? 1 : 0;
        }
        *neg = 1;
    } else {
        memcpy(mag, x, sizeof(u64) * L);
        *neg = 0;
    }
}

/* balanced digits of a centred value (keyswitch.rs:24-44), digit residues mod each q_i */
static void gadget(const octx_t* c, const u64* mag_in, int neg, int G, u64* dig /* [G][L] */) {
    const int L = c->L;
    u64 M[MAXL + 1];
    memset(M, 0, sizeof(M));
    memcpy(M, mag_in, sizeof(u64) * L);
    const u64 B = c->gbase, half = B / 2;
    for (int g = 0; g < G; ++g) {
        u128 rem = 0;
        for (int w = L - 1; w >= 0; --w) {
            u128 cur = (rem << 64) | M[w];
            M[w] = (u64)(cur / B);
            rem = cur % B;
        }
        u64 r = (u64)rem, mag;
        int dneg, carry;
        if (!neg) {
            if (r >= half) { mag = B - r; dneg = 1; carry = 1; } else { mag = r; dneg = 0; carry = 0; }
        } else {
            if (r > half) { mag = B - r; dneg = 0; carry = 1; } else { mag = r; dneg = r != 0; carry = 0; }
        }
        if (carry) {
            u64 cc = 1;
            for (int w = 0; w < L && cc; ++w) { M[w] += cc; cc = M[w] == 0; }
        }
        for (int i = 0; i < L; ++i) {
            u64 v = mag % c->q[i];
            dig[g * L + i] = (dneg && v) ? c->q[i] - v : v;
        }
    }
}

static void octx_init(octx_t* c, int n, int L, const u64* q, int K, const u64* aux, u64 plain, u64 gbase, int G) {
    memset(c, 0, sizeof(*c));
    c->n = n; c->L = L; c->K = K; c->plain = plain; c->gbase = gbase; c->G = G;
    for (int i = 0; i < L; ++i) { c->q[i] = q[i]; plan_init(&c->plan[i], n, q[i]); }
    for (int a = 0; a < K; ++a) { c->aux[a] = aux[a]; plan_init(&c->aplan[a], n, aux[a]); }
    /* Q words */
    u64 Qw[MAXL + 1];
    memset(Qw, 0, sizeof(Qw));
    Qw[0] = 1;
    for (int i = 0; i < L; ++i) {
        u64 cc = 0;
        for (int w = 0; w < L; ++w) { u128 t = (u128)Qw[w] * q[i] + cc; Qw[w] = (u64)t; cc = (u64)(t >> 64); }
    }
    memcpy(c->Q, Qw, sizeof(u64) * L);
    for (int w = 0; w < L; ++w) c->halfQ[w] = (c->Q[w] >> 1) | (w + 1 < L ? c->Q[w + 1] << 63 : 0);
    /* crt_term_i = (Q/q_i) * ((Q/q_i)^-1 mod q_i) */
    for (int i = 0; i < L; ++i) {
        u64 qs[MAXL + 1];
        memset(qs, 0, sizeof(qs));
        qs[0] = 1;
        u64 qs_mod = 1;
        for (int k = 0; k < L; ++k) {
            if (k == i) continue;
            u64 cc = 0;
            for (int w = 0; w < L; ++w) { u128 t = (u128)qs[w] * q[k] + cc; qs[w] = (u64)t; cc = (u64)(t >> 64); }
            qs_mod = mulmod(qs_mod, q[k] % q[i], q[i]);
        }
        u64 inv = invmod(qs_mod, q[i]);
        u64 cc = 0;
        for (int w = 0; w < L; ++w) { u128 t = (u128)qs[w] * inv + cc; c->crt_term[i][w] = (u64)t; cc = (u64)(t >> 64); }
    }
}
static void octx_free(octx_t* c) {
    for (int i = 0; i < c->L; ++i) plan_free(&c->plan[i]);
    for (int a = 0; a < c->K; ++a) plan_free(&c->aplan[a]);
}

/* ------------------------------------------------------------------ generic exact path (eval.rs:113-147) */
static void mul_generic(const octx_t* c, const u64* ct1, const u64* ct2, u64* r /* [3][L][n] coeff */) {
    const int n = c->n, L = c->L;
    const int W = 2 * L + 2;
    /* 1. centred lifts of c0, c1, d0, d1: sign + L-word magnitude */
    u64* mag = (u64*)malloc(sizeof(u64) * 4 * n * L);
    int* sg = (int*)malloc(sizeof(int) * 4 * n);
    u64* tmp = (u64*)malloc(sizeof(u64) * L * n);
    for (int p = 0; p < 4; ++p) {
        const u64* src = (p < 2 ? ct1 : ct2) + (size_t)(p & 1) * L * n;
        memcpy(tmp, src, sizeof(u64) * L * n);
        for (int i = 0; i < L; ++i) ntt_inv(&c->plan[i], tmp + (size_t)i * n);
        for (int j = 0; j < n; ++j) {
            u64 res[MAXL], x[MAXL];
            for (int i = 0; i < L; ++i) res[i] = tmp[(size_t)i * n + j];
            crt(c, res, x);
            centre(c, x, mag + ((size_t)p * n + j) * L, &sg[p * n + j]);
        }
    }
    /* 2. O(n^2) schoolbook tensor over Z (eval.rs:794-810, 131-133) */
    mw_t* T = (mw_t*)calloc((size_t)3 * n, sizeof(mw_t));
    const int pa[4] = {0, 0, 1, 1}, pb[4] = {2, 3, 2, 3}, dst[4] = {0, 1, 1, 2};
    u64 prod[2 * MAXL];
    for (int t = 0; t < 4; ++t) {
        const u64* A = mag + (size_t)pa[t] * n * L;
        const u64* Bm = mag + (size_t)pb[t] * n * L;
        const int* sa = sg + pa[t] * n;
        const int* sb = sg + pb[t] * n;
        mw_t* out = T + (size_t)dst[t] * n;
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) {
                mag_mul(prod, A + (size_t)i * L, Bm + (size_t)j * L, L);
                int neg = sa[i] ^ sb[j];
                int idx = i + j;
                if (idx >= n) { idx -= n; neg ^= 1; }
                mw_add_mag(&out[idx], prod, 2 * L, W, neg);
            }
        }
    }
    /* 3. r = sign * floor((|p*T| + floor(Q/2)) / Q) (eval.rs:816-831), then r mod q_i */
    for (int k = 0; k < 3; ++k) {
        for (int j = 0; j < n; ++j) {
            mw_t x = T[(size_t)k * n + j];
            int neg = mw_neg_p(&x, W);
            if (neg) mw_negate(&x, W);
            /* x *= p */
            u64 cc = 0;
            for (int w = 0; w < W; ++w) { u128 t = (u128)x.w[w] * c->plain + cc; x.w[w] = (u64)t; cc = (u64)(t >> 64); }
            mw_add_mag(&x, c->halfQ, L, W, 0);
            u32 u[2 * MAXW], v[2 * MAXL], qq[2 * MAXW];
            for (int w = 0; w < W; ++w) { u[2 * w] = (u32)x.w[w]; u[2 * w + 1] = (u32)(x.w[w] >> 32); }
            int nn = 2 * L;
            for (int w = 0; w < L; ++w) { v[2 * w] = (u32)c->Q[w]; v[2 * w + 1] = (u32)(c->Q[w] >> 32); }
            while (nn > 1 && v[nn - 1] == 0) nn--;
            memset(qq, 0, sizeof(qq));
            divmnu(qq, u, 2 * W, v, nn);
            u64 qw[MAXW];
            memset(qw, 0, sizeof(qw));
            for (int i = 0; i <= 2 * W - nn; ++i) qw[i / 2] |= (u64)qq[i] << (32 * (i & 1));
            for (int i = 0; i < L; ++i) {
                u64 m = mag_mod(qw, W, c->q[i]);
                r[((size_t)k * L + i) * n + j] = (neg && m) ? c->q[i] - m : m;
            }
        }
    }
    free(T); free(tmp); free(sg); free(mag);
}

/* ------------------------------------------------------------------ literal HPS (eval.rs:157-413) */
static u64 ext_c(u64 c, u64 q, u64 pj) {
    if (c > q / 2) { u64 rem = (q - c) % pj; return rem ? pj - rem : 0; }
    return c % pj;
}

static void mul_hps(const octx_t* c, const u64* ct1, const u64* ct2, u64* r /* [3][n] */) {
    const int n = c->n, K = c->K;
    const u64 q = c->q[0], p = c->plain;
    u64* cq = (u64*)malloc(sizeof(u64) * 4 * n);
    u64* tq = (u64*)malloc(sizeof(u64) * 3 * n);
    u64* tp = (u64*)malloc(sizeof(u64) * 3 * 2 * n);
    u64* ep = (u64*)malloc(sizeof(u64) * 4 * n);
    for (int s = 0; s < 4; ++s) {
        memcpy(cq + (size_t)s * n, (s < 2 ? ct1 : ct2) + (size_t)(s & 1) * n, sizeof(u64) * n);
    }
    /* Q tensor in NTT domain (ntt.rs:119-129 + add) */
    for (int j = 0; j < n; ++j) {
        u64 a0 = cq[j], a1 = cq[n + j], b0 = cq[2 * n + j], b1 = cq[3 * n + j];
        tq[j] = mulmod(a0, b0, q);
        tq[n + j] = (mulmod(a0, b1, q) + mulmod(a1, b0, q)) % q;
        tq[2 * n + j] = mulmod(a1, b1, q);
    }
    for (int s = 0; s < 4; ++s) ntt_inv(&c->plan[0], cq + (size_t)s * n);
    for (int a = 0; a < K; ++a) {
        const u64 pj = c->aux[a];
        for (int s = 0; s < 4; ++s) {
            for (int j = 0; j < n; ++j) ep[(size_t)s * n + j] = ext_c(cq[(size_t)s * n + j], q, pj);
            ntt_fwd(&c->aplan[a], ep + (size_t)s * n);
        }
        for (int j = 0; j < n; ++j) {
            u64 a0 = ep[j], a1 = ep[n + j], b0 = ep[2 * n + j], b1 = ep[3 * n + j];
            tp[((size_t)0 * 2 + a) * n + j] = mulmod(a0, b0, pj);
            tp[((size_t)1 * 2 + a) * n + j] = (mulmod(a0, b1, pj) + mulmod(a1, b0, pj)) % pj;
            tp[((size_t)2 * 2 + a) * n + j] = mulmod(a1, b1, pj);
        }
        for (int k = 0; k < 3; ++k) ntt_inv(&c->aplan[a], tp + ((size_t)k * 2 + a) * n);
    }
    for (int k = 0; k < 3; ++k) ntt_inv(&c->plan[0], tq + (size_t)k * n);
    const i128 q128 = q;
    for (int k = 0; k < 3; ++k) {
        for (int j = 0; j < n; ++j) {
            const u64 av = tq[(size_t)k * n + j];
            const i128 ac = av > q / 2 ? (i128)av - q128 : (i128)av;
            const i128 pa = (i128)p * ac;
            const i128 rnd = pa >= 0 ? (pa + q128 / 2) / q128 : -((-pa + q128 / 2) / q128);
            u64 res;
            if (K == 1) {
                const u64 P = c->aux[0], b = tp[((size_t)k * 2) * n + j];
                const u64 ae = ext_c(av, q, P);
                const u64 diff = b >= ae ? b - ae : P - ae + b;
                const u64 mr = ref_mod_mul(diff, invmod(q % P, P), P);
                const i128 mc = mr > P / 2 ? (i128)mr - (i128)P : (i128)mr;
                const i128 sc = rnd + (i128)p * mc;
                res = (u64)(((sc % q128) + q128) % q128);
            } else {
                const u64 p0 = c->aux[0], p1 = c->aux[1];
                const u64 b0 = tp[((size_t)k * 2) * n + j], b1 = tp[((size_t)k * 2 + 1) * n + j];
                const u64 e0 = ext_c(av, q, p0), e1 = ext_c(av, q, p1);
                const u64 d0 = b0 >= e0 ? b0 - e0 : p0 - e0 + b0;
                const u64 d1 = b1 >= e1 ? b1 - e1 : p1 - e1 + b1;
                const u64 m0 = ref_mod_mul(d0, invmod(q % p0, p0), p0);
                const u64 m1 = ref_mod_mul(d1, invmod(q % p1, p1), p1);
                const i128 t0 = (i128)ref_mod_mul(m0, invmod(p1 % p0, p0), p0);
                const i128 t1 = (i128)ref_mod_mul(m1, invmod(p0 % p1, p1), p1);
                const i128 P = (i128)p0 * (i128)p1;
                const i128 mcrt = (t0 * (i128)p1 + t1 * (i128)p0) % P;
                const i128 mc = mcrt > P / 2 ? mcrt - P : mcrt;
                const i128 mq = ((mc % q128) + q128) % q128;
                const u64 rq = (u64)(((rnd % q128) + q128) % q128);
                const u64 pm = ref_mod_mul(p, (u64)mq, q);
                res = (u64)(((u128)rq + pm) % q);
            }
            r[(size_t)k * n + j] = res;
        }
    }
    free(cq); free(tq); free(tp); free(ep);
}

/* ------------------------------------------------------------------ public entry points */

/* One product (eval.rs:73-108 + keyswitch.rs:59-101): ct1, ct2 = [2][L][n] -> o = [2][L][n] (relin)
 * or [3][L][n], NTT domain. */
static void bfv_mul_one(const octx_t* c, int hps, const u64* ct1, const u64* ct2, const u64* rlk, int guse,
                        int relin, u64* o) {
    const int n = c->n, L = c->L, G = c->G;
    u64* r = (u64*)malloc(sizeof(u64) * 3 * L * n);
    if (hps) mul_hps(c, ct1, ct2, r);
    else mul_generic(c, ct1, ct2, r);
    if (!relin) {
        memcpy(o, r, sizeof(u64) * 3 * L * n);
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < L; ++i) ntt_fwd(&c->plan[i], o + ((size_t)k * L + i) * n);
    } else {
        memcpy(o, r, sizeof(u64) * 2 * L * n);
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < L; ++i) ntt_fwd(&c->plan[i], o + ((size_t)k * L + i) * n);
        /* relinearize: c2 coefficients -> CRT -> centred -> digits (keyswitch.rs:76-95) */
        u64* dig = (u64*)malloc(sizeof(u64) * (size_t)(G > 0 ? G : 1) * L * n);
        for (int j = 0; j < n; ++j) {
            u64 res[MAXL], x[MAXL], mg[MAXL], dj[64 * MAXL];
            int neg;
            for (int i = 0; i < L; ++i) res[i] = r[((size_t)2 * L + i) * n + j];
            if (L == 1) memcpy(x, res, sizeof(u64));
            else crt(c, res, x);
            centre(c, x, mg, &neg);
            gadget(c, mg, neg, guse, dj);
            for (int g = 0; g < guse; ++g)
                for (int i = 0; i < L; ++i) dig[((size_t)g * L + i) * n + j] = dj[g * L + i];
        }
        for (int g = 0; g < guse; ++g)
            for (int i = 0; i < L; ++i) {
                u64* d = dig + ((size_t)g * L + i) * n;
                ntt_fwd(&c->plan[i], d);
                const u64* k0 = rlk + (((size_t)g * 2 + 0) * L + i) * n;
                const u64* k1 = rlk + (((size_t)g * 2 + 1) * L + i) * n;
                u64* o0 = o + (size_t)i * n;
                u64* o1 = o + ((size_t)L + i) * n;
                for (int j = 0; j < n; ++j) {
                    o0[j] = (o0[j] + mulmod(d[j], k0[j], c->q[i])) % c->q[i];
                    o1[j] = (o1[j] + mulmod(d[j], k1[j], c->q[i])) % c->q[i];
                }
            }
        free(dig);
    }
    free(r);
}

/* ct1, ct2 = [B][2][L][n]; rlk = [nkeys][2][L][n]; out = [B][2][L][n] (relin) or [B][3][L][n] */
int oracle_bfv_mul(int n, int L, const u64* q, int K, const u64* aux, u64 plain, u64 gbase, int G,
                   const u64* ct1, const u64* ct2, const u64* rlk, int nkeys, u64* out, int B, int relin,
                   int threads) {
    if (L > MAXL || L < 1 || (L == 1 && K > 2) || (L > 1 && K != 0 && 0)) return 1;
    octx_t c;
    octx_init(&c, n, L, q, L > 1 ? 0 : K, aux, plain, gbase, G);
    const int hps = (L == 1 && K > 0);
    const size_t ctw = (size_t)2 * L * n;
    const int guse = G < nkeys ? G : nkeys;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int b = 0; b < B; ++b)
        bfv_mul_one(&c, hps, ct1 + b * ctw, ct2 + b * ctw, rlk, guse, relin, out + (size_t)b * (relin ? 2 : 3) * L * n);
    octx_free(&c);
    return 0;
}

/* dbfv_mul (dbfv/eval.rs:82-149) + reduce (reduction.rs:15-93) of B item pairs a, b = [B][d][2][L][n]
 * -> out [B][d][2][L][n], literally: ALL d^2 products bfv_mul_and_relin(a_i, b_j) in parallel over
 * (item, i, j) (the reference's rayon par_iter, eval.rs:117-122), summed per k = i + j in order
 * (eval.rs:124-132), then limbs j >= d folded into limbs i < d with the small representatives of
 * base^j mod p (lattice.rs:104-122; p = 0 is 2^64 by wrapping_pow), scaled by |coef| (NTT-domain
 * scalar_mul) and negated for coef < 0 (reduction.rs:65-93).  Depth guard: the caller's. */
int oracle_dbfv_mul(int n, int L, const u64* q, int K, const u64* aux, u64 plain, u64 gbase, int G, int d,
                    u64 base, u64 dplain, const u64* a, const u64* b, const u64* rlk, int nkeys, u64* out, int B,
                    int threads) {
    if (L > MAXL || L < 1 || d < 1 || (L == 1 && K > 2)) return 1;
    /* the products dispatch as bfv_mul_no_relin does (eval.rs:99-107): L == 1 with an aux basis
     * takes the literal HPS multiplier (u64_dbfv, presets.rs:61-75), otherwise the exact one */
    const int hps = (L == 1 && K > 0);
    octx_t c;
    octx_init(&c, n, L, q, hps ? K : 0, aux, plain, gbase, G);
    const size_t ctw = (size_t)2 * L * n;
    const int guse = G < nkeys ? G : nkeys;
    const int R = 2 * d - 1;
    u64* prod = (u64*)malloc(sizeof(u64) * (size_t)B * d * d * ctw);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (long w = 0; w < (long)B * d * d; ++w) {
        const long item = w / (d * d);
        const int i = (int)(w % (d * d)) / d, j = (int)(w % d);
        bfv_mul_one(&c, hps, a + ((size_t)item * d + i) * ctw, b + ((size_t)item * d + j) * ctw, rlk, guse, 1,
                    prod + (size_t)w * ctw);
    }
    u64* limbs = (u64*)calloc((size_t)R * ctw, sizeof(u64));
    for (int item = 0; item < B; ++item) {
        memset(limbs, 0, sizeof(u64) * (size_t)R * ctw);
        for (int i = 0; i < d; ++i)
            for (int j = 0; j < d; ++j) {
                const u64* p = prod + (((size_t)item * d + i) * d + j) * ctw;
                u64* l = limbs + (size_t)(i + j) * ctw;
                for (int t = 0; t < 2 * L; ++t) {
                    const u64 qm = c.q[t % L];
                    for (int x = 0; x < n; ++x) {
                        const u64 v = l[(size_t)t * n + x] + p[(size_t)t * n + x];
                        l[(size_t)t * n + x] = v >= qm ? v - qm : v;
                    }
                }
            }
        /* reduce: reps_j = base-b digits of (base^j mod p), j = d .. 2d-2 */
        for (int jj = d; jj < R; ++jj) {
            u64 val = 1;
            if (dplain == 0) for (int e = 0; e < jj; ++e) val *= base;
            else val = powmod(base, (u64)jj, dplain);
            for (int i = 0; i < d; ++i) {
                const i64 coef = (i64)(val % base);
                val /= base;
                if (coef == 0) continue;
                const u64 mag = (u64)(coef < 0 ? -coef : coef);
                const u64* src = limbs + (size_t)jj * ctw;
                u64* dst = limbs + (size_t)i * ctw;
                for (int t = 0; t < 2 * L; ++t) {
                    const u64 qm = c.q[t % L];
                    for (int x = 0; x < n; ++x) {
                        u64 s = mulmod(src[(size_t)t * n + x], mag % qm, qm);
                        if (coef < 0 && s) s = qm - s;
                        const u64 v = dst[(size_t)t * n + x] + s;
                        dst[(size_t)t * n + x] = v >= qm ? v - qm : v;
                    }
                }
            }
        }
        memcpy(out + (size_t)item * d * ctw, limbs, sizeof(u64) * (size_t)d * ctw);
    }
    free(limbs);
    free(prod);
    octx_free(&c);
    return 0;
}

/* NTT of [count][n] polys mod q (for the cfg2 CPU baseline and NTT checks) */
int oracle_ntt(int n, u64 q, u64* polys, int count, int inverse, int threads) {
    plan_t p;
    plan_init(&p, n, q);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for
#endif
    for (int b = 0; b < count; ++b) {
        if (inverse) ntt_inv(&p, polys + (size_t)b * n);
        else ntt_fwd(&p, polys + (size_t)b * n);
    }
    plan_free(&p);
    return 0;
}

/* Negacyclic products through the NTT, as the reference's own test composes them (ntt.rs:181-195):
 * out = INTT(NTT(a) (.) NTT(b)) per poly, a, b, out = [count][n] coefficient domain mod q (the cfg2
 * CPU baseline: two forward transforms, the pointwise ref_mod_mul, one inverse + normalize). */
int oracle_polymul(int n, u64 q, const u64* a, const u64* b, u64* out, int count, int threads) {
    plan_t p;
    plan_init(&p, n, q);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        u64* t = (u64*)malloc(sizeof(u64) * (size_t)n);
#ifdef _OPENMP
#pragma omp for
#endif
        for (int k = 0; k < count; ++k) {
            u64* o = out + (size_t)k * n;
            memcpy(o, a + (size_t)k * n, sizeof(u64) * (size_t)n);
            memcpy(t, b + (size_t)k * n, sizeof(u64) * (size_t)n);
            ntt_fwd(&p, o);
            ntt_fwd(&p, t);
            for (int j = 0; j < n; ++j) o[j] = ref_mod_mul(o[j], t[j], q);
            ntt_inv(&p, o);
        }
        free(t);
    }
    plan_free(&p);
    return 0;
}
