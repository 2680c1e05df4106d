/* exacto_hip.h — C ABI of the MI355X (gfx950) ciphertext-multiplication path.
 *
 * Drop-in boundary for the hot path of RajeshRk18/exacto (Rust).  Each entry point
 * names the reference interface it replaces (paths relative to the reference repo).
 * A Rust caller binds these with an `extern "C"` block.
 *
 * Conventions
 *   - Return value: 0 = Ok; 1..9 = ExactoError variants in declaration order
 *     (src/error.rs:4-31): 1 InvalidParam, 2 DimensionMismatch, 3 ModulusMismatch,
 *     4 InvalidRingDegree, 5 DecryptionError, 6 DecompositionError, 7 LatticeError,
 *     8 MissingKey, 9 NotImplemented; 100 = HIP runtime failure.  The Display text
 *     of the error (same wording as the reference's #[error(...)] strings) is
 *     available from exacto_last_error() on the calling thread.
 *   - Layout: little-endian uint64, ciphertext batches are [batch][poly][limb][coeff]
 *     (BfvCiphertext.c: Vec<RnsPoly>, src/bfv/mod.rs:19-24; RnsPoly.components:
 *     Vec<NttPoly>, src/ring/rns.rs:14-17).  dBFV batches are
 *     [batch][digit][poly][limb][coeff] (DbfvCiphertext.limbs, src/dbfv/ciphertext.rs:10-22).
 *     Relinearisation keys are [key][2][limb][coeff] (RelinKey.keys,
 *     src/bfv/keygen.rs:39-45).  Residues are canonical, in [0, q_i).
 *   - NTT domain: ciphertexts are stored as NttPoly evaluations (src/ring/ntt.rs:11-15)
 *     in THIS library's documented convention (DESIGN.md "NTT convention"): negacyclic
 *     Cooley-Tukey, evaluation k = a(psi^(2*brv(k)+1)), psi = smallest-generator
 *     primitive 2n-th root, stored at position (k mod 16)*(n/16) + k/16 (the order
 *     the device threads hold the values in: contiguous loads and stores).
 *     concrete-ntt's own order is not observable from the reference's tests; all
 *     parity is checked after the inverse transform.
 *   - Functions without suffix take HOST pointers and are synchronous.  The `_dev`
 *     variants take DEVICE pointers (hipMalloc'd on the context's device) and are
 *     asynchronous on the context's stream (exacto_ctx_set_stream); call
 *     exacto_synchronize() before reading results.
 *   - Inputs are read-only (the reference borrows &BfvCiphertext); outputs never alias
 *     inputs unless stated.
 *   - A context is not thread-safe; use one context per host thread (the reference's
 *     types are Send+Sync because they are immutable; here the stream is shared state).
 */
#ifndef EXACTO_HIP_H
#define EXACTO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct exacto_ctx exacto_ctx;

enum exacto_status {
    EXACTO_OK = 0,
    EXACTO_ERR_INVALID_PARAM = 1,
    EXACTO_ERR_DIMENSION_MISMATCH = 2,
    EXACTO_ERR_MODULUS_MISMATCH = 3,
    EXACTO_ERR_INVALID_RING_DEGREE = 4,
    EXACTO_ERR_DECRYPTION = 5,
    EXACTO_ERR_DECOMPOSITION = 6,
    EXACTO_ERR_LATTICE = 7,
    EXACTO_ERR_MISSING_KEY = 8,
    EXACTO_ERR_NOT_IMPLEMENTED = 9,
    EXACTO_ERR_HIP = 100
};

/* Multiplication algorithm selected for the context (mirrors the dispatcher
 * bfv_mul_no_relin, src/bfv/eval.rs:89-108). */
enum exacto_mul_path {
    EXACTO_PATH_EXACT_RNS = 0,   /* L > 1: exact CRT + exact rounding (eval.rs:113-147) */
    EXACTO_PATH_HPS = 1,         /* L = 1 with aux basis: literal HPS (eval.rs:157-413)  */
    EXACTO_PATH_SCHOOLBOOK = 2   /* L = 1, no aux: exact i128 semantics (eval.rs:416-454) */
};

typedef struct exacto_ctx_info {
    size_t ring_degree;       /* n */
    size_t num_ct_moduli;     /* L */
    size_t num_aux_moduli;    /* user aux basis size */
    size_t num_internal_aux;  /* primes the exact path adds internally (0 for HPS) */
    size_t gadget_digits;     /* G (params/mod.rs:126-140) */
    uint64_t gadget_base;
    uint64_t plain_modulus;
    int mul_path;             /* enum exacto_mul_path */
    int device;
    int ks32_primes;          /* primes of the 31-bit key-switch basis in use (0: limb-wise MAC) */
    int psum_max;             /* dbfv_mul: products per output limb scaled as one sum (0: per product) */
    int ks32_lazy;            /* 1: the resident relinearisation key runs in the lazy 31-bit basis (primes
                                 below 2^30, chosen from the key's own norms at its first use) */
    int ntt_order;            /* storage order of every NTT-domain buffer (keys, ciphertexts): 1 = evaluation k
                                 at position (k mod 16)*n/16 + floor(k/16) (library 0.5 and later); 0 would be
                                 the plain bit-reversed order of 0.4 and earlier, which this library no longer
                                 reads or writes.  Bindings check it (INTEGRATION.md "Format versions") */
    int dbfv_key_switch;      /* the last dbfv_mul's key switch: 1 = the products' digits summed per output
                                 limb in the primary 31-bit basis, 2 = the same in the wide basis, 0 = one key
                                 switch per product, -1 = no dbfv_mul yet */
} exacto_ctx_info;

#define EXACTO_NTT_ORDER 1

/* ---- context: replaces BfvParamsBuilder::build + RnsBasis::new + make_plan ----
 * params/mod.rs:81-124, ring/rns.rs:35-63, ring/ntt.rs:19-29.
 * gadget_base = 0 selects the reference default 2^16 (params/mod.rs:102-108).
 * aux_moduli may be NULL when num_aux == 0.  Errors as the builder: InvalidRingDegree,
 * InvalidParam ("must specify at least one ciphertext modulus", "plaintext modulus must
 * be >= 2", "cannot create NTT plan for n=.., q=.. ..."). */
int exacto_ctx_create(exacto_ctx** out, size_t ring_degree, const uint64_t* ct_moduli,
                      size_t num_ct_moduli, const uint64_t* aux_moduli, size_t num_aux,
                      uint64_t plain_modulus, uint64_t gadget_base, int device);
void exacto_ctx_destroy(exacto_ctx* ctx);
int exacto_ctx_get_info(const exacto_ctx* ctx, exacto_ctx_info* info);
/* Enqueue on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream), used as
 * given: NULL is the device's default stream.  A new context starts on a stream of its own. */
int exacto_ctx_set_stream(exacto_ctx* ctx, void* hip_stream);
/* Products per pipeline chunk (workspace = chunk * ~3 MB at n=4096, L=3). 0 = default. */
int exacto_ctx_set_chunk(exacto_ctx* ctx, size_t products_per_chunk);
int exacto_synchronize(exacto_ctx* ctx);

/* ---- relinearisation key: RelinKey (bfv/keygen.rs:39-45, made by gen_relin_key_with_rng
 * keygen.rs:123-162).  rlk = [num_keys][2][L][n], NTT domain.  relinearize uses
 * min(G, num_keys) digits (keyswitch.rs:86-89). */
int exacto_ctx_load_relin_key(exacto_ctx* ctx, const uint64_t* rlk, size_t num_keys);
int exacto_ctx_load_relin_key_dev(exacto_ctx* ctx, const uint64_t* rlk_dev, size_t num_keys);
/* Device pointer of the resident key (for an RCCL broadcast into it), or NULL. */
uint64_t* exacto_ctx_relin_key_buffer(exacto_ctx* ctx, size_t num_keys);

/* ---- NTT engine: concrete_ntt::prime64::Plan::{fwd, inv + normalize} ----
 * NttPoly::from_coeff_poly / to_coeff_poly (ntt.rs:42-67).  polys = [count][n], all mod
 * ct prime `limb`, transformed in place. */
int exacto_ntt_fwd(exacto_ctx* ctx, uint64_t* polys, size_t count, size_t limb);
int exacto_ntt_inv(exacto_ctx* ctx, uint64_t* polys, size_t count, size_t limb);
int exacto_ntt_fwd_dev(exacto_ctx* ctx, uint64_t* polys, size_t count, size_t limb);
int exacto_ntt_inv_dev(exacto_ctx* ctx, uint64_t* polys, size_t count, size_t limb);
/* RnsPoly batches [count][L][n]: RnsPoly::from_coeff_poly per limb (rns.rs:84-105,
 * coefficients already reduced mod q_i) and the per-limb inverse. */
int exacto_rns_fwd_dev(exacto_ctx* ctx, uint64_t* polys, size_t count);
int exacto_rns_inv_dev(exacto_ctx* ctx, uint64_t* polys, size_t count);

/* ---- RNS pointwise ops: RnsPoly::{add,sub,neg,mul,scalar_mul} (rns.rs:159-217 ->
 * NttPoly ops ntt.rs:75-139).  a, b, out = [count][L][n]; out may alias a or b. */
int exacto_rns_add_dev(exacto_ctx* ctx, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t count);
int exacto_rns_sub_dev(exacto_ctx* ctx, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t count);
int exacto_rns_neg_dev(exacto_ctx* ctx, const uint64_t* a, uint64_t* out, size_t count);
int exacto_rns_mul_dev(exacto_ctx* ctx, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t count);
int exacto_rns_scalar_mul_dev(exacto_ctx* ctx, const uint64_t* a, uint64_t scalar, uint64_t* out, size_t count);
/* INTT(a (.) b): RnsPoly::mul followed by the per-limb inverse (to_coeff_poly, ntt.rs:58-67,
 * 119-129) fused into one pass, as the reference's own negacyclic-product test composes them
 * (ntt.rs:181-195).  a, b NTT domain, out coefficient domain; out may alias a or b. */
int exacto_rns_mul_inv_dev(exacto_ctx* ctx, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t count);
/* Negacyclic products of coefficient-domain RnsPolys: to_coeff_poly(from_coeff_poly(a) (.)
 * from_coeff_poly(b)) per limb, the reference's NTT multiplication (ntt.rs:181-195), fused into
 * one kernel at n = 4096 / 8192 (neither operand's evaluations are stored).  out may alias a or b. */
int exacto_rns_polymul_dev(exacto_ctx* ctx, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t count);

/* ---- BFV ciphertext ops (bfv/eval.rs).  Degree-1 ct batches [B][2][L][n]. ---- */
/* bfv_add / bfv_sub / bfv_neg (eval.rs:14-60), batched.  ct1 = [B][polys1][L][n], ct2 =
 * [B][polys2][L][n] -> out = [B][max(polys1, polys2)][L][n]: component i < min is the pointwise
 * sum / difference; the longer operand's further components pass through (eval.rs:21-22), negated
 * when they are ct2's under subtraction (eval.rs:41-42).  out may alias an input only when that
 * input has max(polys1, polys2) components. */
int exacto_bfv_add(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2, size_t polys2,
                   uint64_t* out, size_t batch);
int exacto_bfv_add_dev(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2, size_t polys2,
                       uint64_t* out, size_t batch);
int exacto_bfv_sub(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2, size_t polys2,
                   uint64_t* out, size_t batch);
int exacto_bfv_sub_dev(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2, size_t polys2,
                       uint64_t* out, size_t batch);
int exacto_bfv_neg(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t* out, size_t batch);
int exacto_bfv_neg_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t* out, size_t batch);

/* bfv_mul_no_relin (eval.rs:89-108): out = [B][3][L][n].  `polys1`/`polys2` are the
 * input ciphertexts' component counts (must be 2: "multiplication requires degree-1
 * ciphertexts"). */
int exacto_bfv_mul_no_relin(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2,
                            size_t polys2, uint64_t* out, size_t batch);
int exacto_bfv_mul_no_relin_dev(exacto_ctx* ctx, const uint64_t* ct1, size_t polys1, const uint64_t* ct2,
                                size_t polys2, uint64_t* out, size_t batch);

/* relinearize (bfv/keyswitch.rs:59-101): ct = [B][3][L][n] -> out = [B][2][L][n].
 * polys < 3: cloned, out = [B][polys][L][n] (keyswitch.rs:63-65); polys > 3: InvalidParam
 * "relinearization only supports degree-2 ciphertexts". */
int exacto_relinearize(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t* out, size_t batch);
int exacto_relinearize_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t* out, size_t batch);

/* bfv_mul_and_relin (eval.rs:73-82): ct1, ct2 = [B][2][L][n] -> out = [B][2][L][n]. */
int exacto_bfv_mul_and_relin(exacto_ctx* ctx, const uint64_t* ct1, const uint64_t* ct2, uint64_t* out,
                             size_t batch);
int exacto_bfv_mul_and_relin_dev(exacto_ctx* ctx, const uint64_t* ct1, const uint64_t* ct2,
                                 uint64_t* out, size_t batch);

/* gadget_decompose (keyswitch.rs:11-52) of coefficient-domain RNS polynomials [B][L][n]
 * (CRT value mod Q, extension semantics when Q >= 2^64) -> digits [B][G'][L][n] as
 * residues mod q_i, G' = min(G, num_digits). */
int exacto_gadget_decompose_dev(exacto_ctx* ctx, const uint64_t* coeffs, uint64_t* digits,
                                size_t batch, size_t num_digits);

/* ---- dBFV: dbfv_mul (dbfv/eval.rs:82-149) + reduce (dbfv/reduction.rs:15-60) ----
 * a, b, out = [B][d][2][L][n]; base/plain as DbfvParams (params/mod.rs:144-193,
 * plain_modulus 0 == 2^64).  depth_a/depth_b = mul_depth of each input (NULL = 0);
 * depth_out receives mul_depth of each output (NULL allowed).  Errors:
 * "multiplication requires d-limb ciphertexts" is not reachable through fixed shapes;
 * depth > 1 -> NotImplemented "chained dBFV multiplication requires ciphertext-level
 * lattice reduction (paper §4.6.2)". */
int exacto_dbfv_mul(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                    const uint64_t* a, const uint64_t* b, uint64_t* out, size_t batch,
                    const uint32_t* depth_a, const uint32_t* depth_b, uint32_t* depth_out);
int exacto_dbfv_mul_dev(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                        const uint64_t* a, const uint64_t* b, uint64_t* out, size_t batch,
                        const uint32_t* depth_a, const uint32_t* depth_b, uint32_t* depth_out);

/* One GPU's share of a dbfv_mul whose d output limbs are split across GPUs (the d^2 digit-pair
 * products of dbfv/eval.rs:109-122 partitioned by output limb k = i + j, so no cross-GPU sum is
 * needed): only the output limbs limbs[0..nlimbs) (host array, distinct, < d) are computed, out =
 * [B][nlimbs][2][L][n] with slot s holding limb limbs[s] exactly as exacto_dbfv_mul computes it
 * (including the reduce folding of limbs >= d, reduction.rs:34-52).  The caller gathers the slots of
 * all GPUs (exacto_rccl_allgather_u64) into [B][d][2][L][n].  Inputs at mul_depth 0. */
int exacto_dbfv_mul_limbs(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                          const uint64_t* a, const uint64_t* b, uint64_t* out, size_t batch, const uint32_t* limbs,
                          size_t nlimbs);
int exacto_dbfv_mul_limbs_dev(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                              const uint64_t* a, const uint64_t* b, uint64_t* out, size_t batch, const uint32_t* limbs,
                              size_t nlimbs);

/* dBFV multiplication chain, device-resident (paper_repro.rs:203-236 guard-bypass semantics;
 * bfv_host.rs:258-288 without the bootstrap): out = (((x*y)*y)...*y), `depth` dbfv_mul steps,
 * each with both inputs' mul_depth reset to 0, intermediates kept in context-owned HBM buffers.
 * x, y, out = [B][d][2][L][n]; depth 0 copies x.  Errors as exacto_dbfv_mul. */
int exacto_dbfv_mul_chain(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                          const uint64_t* x, const uint64_t* y, uint64_t* out, size_t batch, size_t depth);
int exacto_dbfv_mul_chain_dev(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                              const uint64_t* x, const uint64_t* y, uint64_t* out, size_t batch, size_t depth);

/* ---- decryption ----
 * BFV decrypt (bfv/encrypt.rs:111-178), batched: phase = sum_k c_k * s^k in the NTT domain,
 * INTT, x = CRT(phase) in [0, Q), m = floor((x*p + floor(Q/2)) / Q) mod p, exact for any Q.
 * ct = [B][polys][L][n] (polys >= 1), sk = secret key [L][n] (NTT domain), out = [B][n] mod p.
 * L >= 2 needs p below the first internal auxiliary prime (~2^60), else NotImplemented. */
int exacto_bfv_decrypt(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* sk, uint64_t* out,
                       size_t batch);
int exacto_bfv_decrypt_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* sk,
                           uint64_t* out, size_t batch);
/* dBFV decrypt (dbfv/decrypt.rs:20-43): each limb decrypted mod t (the context's plain modulus),
 * coefficient 0 of every limb centred and recomposed: sum centred(mu_i) * base^i mod p (i128,
 * p = 0 -> mod 2^64).  ct = [B][d][2][L][n], out = [B]. */
int exacto_dbfv_decrypt(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                        const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t batch);
int exacto_dbfv_decrypt_dev(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                            const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t batch);
/* dbfv_decrypt_poly (dbfv/decrypt.rs:48-79): the same recomposition for every coefficient,
 * out = [B][n]; plain modulus 0 -> InvalidParam "polynomial dBFV decrypt requires finite
 * plain_modulus (plain_modulus=0 is scalar-only)". */
int exacto_dbfv_decrypt_poly(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                             const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t batch);
int exacto_dbfv_decrypt_poly_dev(exacto_ctx* ctx, size_t d, uint64_t base, uint64_t dbfv_plain_modulus,
                                 const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t batch);

/* ---- diagnostics ---- */
/* Copies the last error message of this thread (NUL-terminated); returns its length. */
/* ---- key generation and encryption on the device ----
 * keygen.rs:64-162 and encrypt.rs:29-106, 181-229.  Polynomials are sampled exactly as the
 * reference's samplers define them (sampling/uniform.rs, sampling/gaussian.rs: values of a CoeffPoly
 * modulo the FIRST ciphertext prime, then reduced modulo every q_i), from a ChaCha20 stream in
 * counter mode (the reference's ChaCha20Rng primitive; the word stream is this library's own):
 * `key` = 4 words (256 bits, HOST pointer, also for _dev), `stream` = 64-bit nonce.  Equal
 * (key, stream) reproduce the same output.  sigma: Gaussian width (BfvParams.sigma, 3.2 default).
 * sk [L][n], pk [2][L][n], rlk [num_keys][2][L][n], ct [B][2][L][n]: NTT domain.  pt [B][n]:
 * plaintext coefficients (CoeffPoly mod p). */
int exacto_gen_secret_key(exacto_ctx* ctx, const uint64_t* key, uint64_t stream, uint64_t* sk);
int exacto_gen_secret_key_dev(exacto_ctx* ctx, const uint64_t* key, uint64_t stream, uint64_t* sk);
int exacto_gen_public_key(exacto_ctx* ctx, const uint64_t* sk, double sigma, const uint64_t* key,
                          uint64_t stream, uint64_t* pk);
int exacto_gen_public_key_dev(exacto_ctx* ctx, const uint64_t* sk, double sigma, const uint64_t* key,
                              uint64_t stream, uint64_t* pk);
/* rlk == NULL: the key is generated straight into the context's resident relinearisation key
 * (replaces exacto_ctx_load_relin_key: no host build, no upload). */
int exacto_gen_relin_key(exacto_ctx* ctx, const uint64_t* sk, double sigma, const uint64_t* key,
                         uint64_t stream, size_t num_keys, uint64_t* rlk);
int exacto_gen_relin_key_dev(exacto_ctx* ctx, const uint64_t* sk, double sigma, const uint64_t* key,
                             uint64_t stream, size_t num_keys, uint64_t* rlk);
int exacto_encrypt_sk(exacto_ctx* ctx, const uint64_t* pt, const uint64_t* sk, double sigma, const uint64_t* key,
                      uint64_t stream, uint64_t* ct, size_t batch);
int exacto_encrypt_sk_dev(exacto_ctx* ctx, const uint64_t* pt, const uint64_t* sk, double sigma,
                          const uint64_t* key, uint64_t stream, uint64_t* ct, size_t batch);
int exacto_encrypt_pk(exacto_ctx* ctx, const uint64_t* pt, const uint64_t* pk, double sigma, const uint64_t* key,
                      uint64_t stream, uint64_t* ct, size_t batch);
int exacto_encrypt_pk_dev(exacto_ctx* ctx, const uint64_t* pt, const uint64_t* pk, double sigma,
                          const uint64_t* key, uint64_t stream, uint64_t* ct, size_t batch);

/* ---- Galois automorphisms ----
 * gen_galois_key_with_rng (keygen.rs:171-209): key-switch key from s(X^element) to s(X), gk =
 * [num_keys][2][L][n]; s(X^element) is formed from limb 0 of s as the reference does
 * (keygen.rs:179-182).  bfv_apply_automorphism (eval.rs:512-561), batched: ct/out [B][2][L][n],
 * polys must be 2 ("automorphism requires degree-1 ciphertext"); min(G, num_keys) digits are
 * used; an empty key is InvalidParam (the reference panics on it). */
int exacto_gen_galois_key(exacto_ctx* ctx, const uint64_t* sk, uint64_t element, double sigma,
                          const uint64_t* key, uint64_t stream, size_t num_keys, uint64_t* gk);
int exacto_gen_galois_key_dev(exacto_ctx* ctx, const uint64_t* sk, uint64_t element, double sigma,
                              const uint64_t* key, uint64_t stream, size_t num_keys, uint64_t* gk);
int exacto_bfv_apply_automorphism(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t element,
                                  const uint64_t* gk, size_t num_keys, uint64_t* out, size_t batch);
int exacto_bfv_apply_automorphism_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t element,
                                      const uint64_t* gk, size_t num_keys, uint64_t* out, size_t batch);

/* Plaintext-ciphertext operations (CoeffsToSlots' linear layer), all in the NTT domain.
 * ct/out [B][polys][L][n]; pt [B][n] plaintext coefficients (any u64, reduced mod each q_i).
 *   bfv_plain_mul     replaces bfv::eval::bfv_plain_mul      (src/bfv/eval.rs:468-486)
 *   bfv_plain_add     replaces bfv::eval::bfv_plain_add      (src/bfv/eval.rs:489-503), c0 + Delta m
 *   bfv_inner_product replaces bfv::eval::bfv_inner_product  (src/bfv/eval.rs:588-606):
 *                     cts [K][polys][L][n], pts [K][n] -> out [polys][L][n]; K == 0 is InvalidParam
 *   bfv_monomial_mul  replaces bfv::eval::bfv_monomial_mul   (src/bfv/eval.rs:613-652), X^j, j mod 2n
 *   bfv_trace         replaces bfv::eval::bfv_trace          (src/bfv/eval.rs:572-586): elements is a
 *                     HOST array [E]; gks [E][num_keys][2][L][n] holds the key of elements[e] at e. */
int exacto_bfv_plain_mul(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* pt, uint64_t* out,
                         size_t batch);
int exacto_bfv_plain_mul_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* pt, uint64_t* out,
                             size_t batch);
int exacto_bfv_plain_add(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* pt, uint64_t* out,
                         size_t batch);
int exacto_bfv_plain_add_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* pt, uint64_t* out,
                             size_t batch);
int exacto_bfv_inner_product(exacto_ctx* ctx, const uint64_t* cts, const uint64_t* pts, size_t K, size_t polys,
                             uint64_t* out);
int exacto_bfv_inner_product_dev(exacto_ctx* ctx, const uint64_t* cts, const uint64_t* pts, size_t K, size_t polys,
                                 uint64_t* out);
int exacto_bfv_monomial_mul(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t j, uint64_t* out,
                            size_t batch);
int exacto_bfv_monomial_mul_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, uint64_t j, uint64_t* out,
                                size_t batch);
int exacto_bfv_trace(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* elements, size_t E,
                     const uint64_t* gks, size_t num_keys, uint64_t* out, size_t batch);
int exacto_bfv_trace_dev(exacto_ctx* ctx, const uint64_t* ct, size_t polys, const uint64_t* elements, size_t E,
                         const uint64_t* gks, size_t num_keys, uint64_t* out, size_t batch);

/* CoeffsToSlots / SlotsToCoeffs (src/bootstrap/coeffs_to_slots.rs).
 *   exacto_required_trace_elements replaces required_trace_elements (coeffs_to_slots.rs:168-183):
 *     pure host function, writes up to cap elements and returns how many there are.
 *   exacto_extract_coefficients replaces extract_coefficient (coeffs_to_slots.rs:21-49) for the J
 *     indices j0 .. j0+J-1 of one ciphertext ct [2][L][n] -> out [J][2][L][n] (coeffs_to_slots,
 *     coeffs_to_slots.rs:103-115, is j0 = 0, J = n).  (elements [E] host, gks [E][num_keys][2][L][n])
 *     is the reference's HashMap<element, GaloisKey>; a required element missing from it is
 *     InvalidParam "missing Galois key for element k"; n not invertible mod t is InvalidParam.
 *   exacto_slots_to_coeffs replaces slots_to_coeffs (coeffs_to_slots.rs:121-145): slots
 *     [S][polys][L][n] -> out [polys][L][n]; S == 0 "empty slots", S != n "expected n slots, got S". */
size_t exacto_required_trace_elements(size_t n, uint64_t* out, size_t cap);
int exacto_extract_coefficients(exacto_ctx* ctx, const uint64_t* ct, uint64_t j0, size_t J, const uint64_t* elements,
                                size_t E, const uint64_t* gks, size_t num_keys, uint64_t* out);
int exacto_extract_coefficients_dev(exacto_ctx* ctx, const uint64_t* ct, uint64_t j0, size_t J,
                                    const uint64_t* elements, size_t E, const uint64_t* gks, size_t num_keys,
                                    uint64_t* out);
int exacto_slots_to_coeffs(exacto_ctx* ctx, const uint64_t* slots, size_t S, size_t polys, uint64_t* out);
int exacto_slots_to_coeffs_dev(exacto_ctx* ctx, const uint64_t* slots, size_t S, size_t polys, uint64_t* out);

/* Digit extraction (src/bootstrap/digit_extract.rs).
 *   exacto_lagrange_interpolate replaces lagrange_interpolate (digit_extract.rs:37-90): host only,
 *     out [n]; a zero denominator (points not distinct mod p) is InvalidParam (the reference panics).
 *   exacto_compute_rounding_poly replaces compute_rounding_poly (digit_extract.rs:19-30): host only,
 *     out [t_boot].
 *   exacto_trivial_encrypt replaces trivial_encrypt_poly (digit_extract.rs:179-189): pt [B][n] ->
 *     (Delta m, 0) [B][2][L][n]; trivial_encrypt(m) is pt = (m mod t, 0, ..., 0).
 *   exacto_eval_poly replaces eval_poly_homomorphic (digit_extract.rs:101-157) on B ciphertexts at
 *     once with the reference's Paterson-Stockmeyer schedule; coeffs is a HOST array [m], m >= 1;
 *     the relinearisation key is the context's resident one (MissingKey if none). */
int exacto_lagrange_interpolate(const uint64_t* values, size_t n, uint64_t p, uint64_t* out);
int exacto_compute_rounding_poly(uint64_t t_orig, uint64_t q_prime, uint64_t t_boot, uint64_t* out);
int exacto_trivial_encrypt(exacto_ctx* ctx, const uint64_t* pt, uint64_t* out, size_t batch);
int exacto_trivial_encrypt_dev(exacto_ctx* ctx, const uint64_t* pt, uint64_t* out, size_t batch);
int exacto_eval_poly(exacto_ctx* ctx, const uint64_t* ct, const uint64_t* coeffs, size_t m, uint64_t* out,
                     size_t batch);
int exacto_eval_poly_dev(exacto_ctx* ctx, const uint64_t* ct, const uint64_t* coeffs, size_t m, uint64_t* out,
                         size_t batch);

/* Bootstrapping (src/bootstrap/bfv_host.rs), over two contexts on one device: `orig` (the scheme
 * being refreshed; ONE ciphertext prime, because the reference switches from moduli[0] after
 * to_coeff_poly, bfv_host.rs:149-157) and `boot` (same n).
 *   exacto_bootstrap_key_material replaces the key-material half of gen_bootstrap_key and
 *     create_boot_sk (bfv_host.rs:57-100, 289-330): sk [1][n] (NTT) -> boot_sk [Lb][n] (NTT) and the
 *     plaintext s_pt [n] that bsk encrypts.  bsk, boot_rlk and the trace keys are then made with
 *     exacto_encrypt_sk / exacto_gen_relin_key / exacto_gen_galois_key on `boot`.
 *   exacto_bfv_bootstrap replaces bfv_bootstrap (bfv_host.rs:131-205) for B ciphertexts:
 *     ct [B][2][1][n] -> out [B][2][Lb][n]; bsk [2][Lb][n]; rpoly [m] HOST (compute_rounding_poly);
 *     (elements [E] HOST, gks [E][num_keys][2][Lb][n]) the trace keys; boot's resident relin key is
 *     boot_rlk.  Items with c1 = 0 take the trivial path (bfv_host.rs:180-186), the rest the full
 *     ring path (CoeffsToSlots -> rounding polynomial on the n slots at once -> SlotsToCoeffs). */
int exacto_bootstrap_key_material(exacto_ctx* orig, exacto_ctx* boot, const uint64_t* sk, uint64_t* boot_sk,
                                  uint64_t* s_pt);
int exacto_bootstrap_key_material_dev(exacto_ctx* orig, exacto_ctx* boot, const uint64_t* sk, uint64_t* boot_sk,
                                      uint64_t* s_pt);
int exacto_bfv_bootstrap(exacto_ctx* orig, exacto_ctx* boot, const uint64_t* ct, size_t polys, const uint64_t* bsk,
                         const uint64_t* rpoly, size_t m, uint64_t q_prime, const uint64_t* elements, size_t E,
                         const uint64_t* gks, size_t num_keys, uint64_t* out, size_t batch);
int exacto_bfv_bootstrap_dev(exacto_ctx* orig, exacto_ctx* boot, const uint64_t* ct, size_t polys,
                             const uint64_t* bsk, const uint64_t* rpoly, size_t m, uint64_t q_prime,
                             const uint64_t* elements, size_t E, const uint64_t* gks, size_t num_keys, uint64_t* out,
                             size_t batch);

/* ---- RCCL collectives over xGMI ----
 * Replace the host-side key distribution of the reference (keys built once, keygen.rs:123-209, and
 * shared by every rayon worker) with one broadcast per key to every GPU, and gather the output limbs
 * of a split dbfv_mul.  `comm` is an ncclComm_t (RCCL), as void*: made by exacto_rccl_comm_init or by
 * the caller's own RCCL.  RCCL is opened at first use (librccl.so.1, or $EXACTO_RCCL_LIB); failures
 * return EXACTO_ERR_HIP with an "RCCL error: ..." message.  All collectives are enqueued on the
 * context's stream.
 *   exacto_rccl_unique_id      ncclGetUniqueId -> id[128] (rank 0; share it out of band)
 *   exacto_rccl_comm_init      ncclCommInitRank on `device`
 *   exacto_rccl_comm_count     ncclCommCount: the ranks the communicator spans (bench lines record it)
 *   exacto_ctx_broadcast_relin_key   root's resident relinearisation key -> every rank's resident key
 *                              (in place; non-root ranks need no prior load), num_keys = [G] rows.
 *                              Collective agreement first: every rank all-gathers {num_keys, verdict},
 *                              so a root without a key of that size, or ranks passing different
 *                              num_keys, fail with InvalidParam on EVERY rank, keys untouched
 *   exacto_broadcast_galois_key      a device Galois key buffer [num_keys][2][L][n], in place
 *   exacto_rccl_allgather_u64  recv = [nranks][count] u64 (never a reduction: residues are not summable
 *                              by RCCL)
 *   exacto_rccl_sync           waits for the context stream (the collectives enqueued on it) with a deadline
 * Deadlines: communicator init, the agreement all-gather and exacto_rccl_sync wait at most
 * $EXACTO_RCCL_TIMEOUT_S seconds (default 300, 0 = forever) for the other ranks; on expiry they return
 * EXACTO_ERR_HIP "RCCL error: ... timed out" (a collective's communicator is aborted with ncclCommAbort,
 * after which exacto_rccl_comm_destroy on it is a no-op), so a rank that never joins cannot block the
 * others for good. */
int exacto_rccl_unique_id(uint8_t* id);
int exacto_rccl_comm_init(void** comm, int nranks, const uint8_t* id, int rank, int device);
int exacto_rccl_comm_destroy(void* comm);
int exacto_rccl_comm_count(void* comm, int* nranks);
int exacto_ctx_broadcast_relin_key(exacto_ctx* ctx, void* comm, int root, size_t num_keys);
int exacto_broadcast_galois_key(exacto_ctx* ctx, void* comm, int root, uint64_t* gk_dev, size_t num_keys);
int exacto_rccl_allgather_u64(exacto_ctx* ctx, void* comm, const uint64_t* send, uint64_t* recv, size_t count);
int exacto_rccl_sync(exacto_ctx* ctx, void* comm);

size_t exacto_last_error(char* buf, size_t len);
/* Per-kernel-family timing of the last profiled calls: enable, then read
 * (kind 0 = forward NTT, 1 = inverse NTT): launches, summed device ms, summed algorithmic
 * bytes (16*n per polynomial). */
int exacto_prof_enable(exacto_ctx* ctx, int enable);
int exacto_prof_read(exacto_ctx* ctx, int kind, uint64_t* launches, double* total_ms,
                     double* total_bytes, uint64_t* polys);
/* The kernels that ran for one family in the records exacto_prof_read consumed (since the last call for
 * that kind), named as rocprofv3 names them ("exacto::ntt_fwd_pin_kernel<12, 0, false>"), by descending
 * event time: "name (launches, ms); ...".  Returns the full length (snprintf-like); buf may be NULL (a
 * size query, which keeps the list; a call with a buffer clears it). */
size_t exacto_prof_kernels(exacto_ctx* ctx, int kind, char* buf, size_t len);
const char* exacto_version(void);

#ifdef __cplusplus
}
#endif
#endif /* EXACTO_HIP_H */
