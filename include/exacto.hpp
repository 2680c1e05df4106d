// exacto.hpp — C++ host API mirroring the reference's Rust API on the multiplication path,
// layered on the C ABI (exacto_hip.h).  Same names and argument meaning as
//   exacto::params::{BfvParams, BfvParamsBuilder, DbfvParams}   (src/params/mod.rs:12-193)
//   exacto::bfv::{BfvCiphertext, RelinKey}                       (src/bfv/mod.rs:19-24, keygen.rs:39-45)
//   exacto::bfv::eval::{bfv_mul_and_relin, bfv_mul_no_relin, bfv_add, bfv_sub, bfv_neg}
//   exacto::bfv::keyswitch::relinearize
//   exacto::dbfv::{DbfvCiphertext, eval::dbfv_mul}
//   exacto::bfv::keygen / encrypt (device samplers), eval::{bfv_plain_mul, bfv_plain_add,
//     bfv_inner_product, bfv_monomial_mul, bfv_trace, bfv_apply_automorphism}
//   exacto::bootstrap::{coeffs_to_slots, digit_extract, bfv_host}  (src/bootstrap/*.rs)
// Errors: Rust's Result<T, ExactoError> becomes a thrown exacto::ExactoError carrying the
// variant (src/error.rs:4-31) and the reference's Display text.
// Ciphertexts are host-resident here (one H2D/D2H per call); the batched overloads amortise it.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "exacto_hip.h"

namespace exacto {

class ExactoError : public std::runtime_error {
  public:
    ExactoError(int code, const std::string& msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }
    const char* variant() const {
        static const char* names[] = {"InvalidParam", "DimensionMismatch", "ModulusMismatch",
                                      "InvalidRingDegree", "DecryptionError", "DecompositionError",
                                      "LatticeError", "MissingKey", "NotImplemented"};
        return (code_ >= 1 && code_ <= 9) ? names[code_ - 1] : "HipError";
    }

  private:
    int code_;
};

namespace detail {
inline void check(int rc) {
    if (rc == 0) return;
    char buf[1024];
    exacto_last_error(buf, sizeof buf);
    throw ExactoError(rc, buf);
}
}  // namespace detail

// RnsPoly (src/ring/rns.rs:14-17): L limbs of n NTT-domain evaluations, stored [L][n].
struct RnsPoly {
    size_t ring_degree = 0;
    size_t num_limbs = 0;
    std::vector<uint64_t> data;  // [limb][n]
    uint64_t* limb(size_t i) { return data.data() + i * ring_degree; }
    const uint64_t* limb(size_t i) const { return data.data() + i * ring_degree; }
};

class BfvParams {
  public:
    size_t ring_degree;
    uint64_t plain_modulus;
    std::vector<uint64_t> ct_moduli, aux_moduli;
    double sigma;
    uint64_t gadget_base;
    size_t gadget_digits;
    ~BfvParams() { exacto_ctx_destroy(ctx_); }
    exacto_ctx* ctx() const { return ctx_; }
    size_t num_limbs() const { return ct_moduli.size(); }
    // the key last uploaded to the context (identity, not contents)
    mutable const void* loaded_key = nullptr;

  private:
    friend class BfvParamsBuilder;
    exacto_ctx* ctx_ = nullptr;
};
using BfvParamsPtr = std::shared_ptr<const BfvParams>;

// BfvParamsBuilder (src/params/mod.rs:30-124); build() also creates the device context.
class BfvParamsBuilder {
  public:
    BfvParamsBuilder& ring_degree(size_t n) { n_ = n; return *this; }
    BfvParamsBuilder& plain_modulus(uint64_t p) { p_ = p; return *this; }
    BfvParamsBuilder& ct_moduli(std::vector<uint64_t> m) { ct_ = std::move(m); return *this; }
    BfvParamsBuilder& aux_moduli(std::vector<uint64_t> m) { aux_ = std::move(m); return *this; }
    BfvParamsBuilder& sigma(double s) { sigma_ = s; return *this; }
    BfvParamsBuilder& gadget_base(uint64_t b) { base_ = b; return *this; }
    BfvParamsBuilder& device(int d) { device_ = d; return *this; }
    BfvParamsPtr build() const {
        auto p = std::shared_ptr<BfvParams>(new BfvParams());
        detail::check(exacto_ctx_create(&p->ctx_, n_, ct_.data(), ct_.size(),
                                        aux_.empty() ? nullptr : aux_.data(), aux_.size(), p_, base_,
                                        device_));
        exacto_ctx_info info{};
        detail::check(exacto_ctx_get_info(p->ctx_, &info));
        // NTT-domain data (keys, ciphertexts) is laid out in the library's storage order: refuse a
        // library whose order differs from the one this header was written for
        if (info.ntt_order != EXACTO_NTT_ORDER)
            throw ExactoError(EXACTO_ERR_INVALID_PARAM, "libexacto_hip NTT-domain order differs from exacto.hpp's");
        p->ring_degree = n_;
        p->plain_modulus = p_;
        p->ct_moduli = ct_;
        p->aux_moduli = aux_;
        p->sigma = sigma_;
        p->gadget_base = info.gadget_base;
        p->gadget_digits = info.gadget_digits;
        return p;
    }

  private:
    size_t n_ = 4096;        // params/mod.rs:42
    uint64_t p_ = 65537;     // params/mod.rs:43
    std::vector<uint64_t> ct_, aux_;
    double sigma_ = 3.2;
    uint64_t base_ = 0;      // auto: 2^16 (params/mod.rs:102-108)
    int device_ = 0;
};

struct BfvCiphertext {
    std::vector<RnsPoly> c;
    BfvParamsPtr params;
    size_t degree() const { return c.size() - 1; }
};

struct RelinKey {
    std::vector<std::pair<RnsPoly, RnsPoly>> keys;
    BfvParamsPtr params;
};

// SecretKey (src/bfv/keygen.rs): the secret polynomial s in the NTT domain, [L][n].
struct SecretKey {
    RnsPoly poly;
    BfvParamsPtr params;
};

// CoeffPoly (src/ring/poly.rs:6-9): plaintext coefficients mod `modulus`.
struct CoeffPoly {
    std::vector<uint64_t> coeffs;
    uint64_t modulus = 0;
};

namespace detail {
inline std::vector<uint64_t> flatten(const std::vector<BfvCiphertext>& cts, size_t polys) {
    std::vector<uint64_t> out;
    for (auto& ct : cts) {
        if (ct.c.size() != polys) throw ExactoError(1, "invalid parameter: mixed ciphertext degrees in a batch");
        for (auto& p : ct.c) out.insert(out.end(), p.data.begin(), p.data.end());
    }
    return out;
}
inline std::vector<BfvCiphertext> unflatten(const std::vector<uint64_t>& flat, size_t batch, size_t polys,
                                            const BfvParamsPtr& prm) {
    const size_t L = prm->num_limbs(), n = prm->ring_degree;
    std::vector<BfvCiphertext> out(batch);
    for (size_t b = 0; b < batch; ++b) {
        out[b].params = prm;
        out[b].c.resize(polys);
        for (size_t k = 0; k < polys; ++k) {
            RnsPoly& p = out[b].c[k];
            p.ring_degree = n;
            p.num_limbs = L;
            auto it = flat.begin() + (long)((b * polys + k) * L * n);
            p.data.assign(it, it + (long)(L * n));
        }
    }
    return out;
}
inline void load_key(const RelinKey& rlk) {
    const BfvParams& prm = *rlk.params;
    if (prm.loaded_key == &rlk) return;
    std::vector<uint64_t> flat;
    for (auto& kp : rlk.keys) {
        flat.insert(flat.end(), kp.first.data.begin(), kp.first.data.end());
        flat.insert(flat.end(), kp.second.data.begin(), kp.second.data.end());
    }
    check(exacto_ctx_load_relin_key(prm.ctx(), flat.empty() ? nullptr : flat.data(), rlk.keys.size()));
    prm.loaded_key = &rlk;
}
}  // namespace detail

// ---- exacto::bfv::eval (batched forms; the single-ciphertext forms below wrap them)
inline std::vector<BfvCiphertext> bfv_mul_no_relin(const std::vector<BfvCiphertext>& a,
                                                   const std::vector<BfvCiphertext>& b) {
    if (a.empty()) return {};
    const BfvParamsPtr& prm = a[0].params;
    const size_t p1 = a[0].c.size(), p2 = b[0].c.size();
    auto fa = detail::flatten(a, p1), fb = detail::flatten(b, p2);
    std::vector<uint64_t> out(a.size() * 3 * prm->num_limbs() * prm->ring_degree);
    detail::check(exacto_bfv_mul_no_relin(prm->ctx(), fa.data(), p1, fb.data(), p2, out.data(), a.size()));
    return detail::unflatten(out, a.size(), 3, prm);
}

inline std::vector<BfvCiphertext> relinearize(const std::vector<BfvCiphertext>& cts, const RelinKey& rlk) {
    if (cts.empty()) return {};
    const BfvParamsPtr& prm = cts[0].params;
    const size_t polys = cts[0].c.size();
    detail::load_key(rlk);
    auto f = detail::flatten(cts, polys);
    const size_t outp = polys < 3 ? polys : 2;
    std::vector<uint64_t> out(cts.size() * outp * prm->num_limbs() * prm->ring_degree);
    detail::check(exacto_relinearize(prm->ctx(), f.data(), polys, out.data(), cts.size()));
    return detail::unflatten(out, cts.size(), outp, prm);
}

inline std::vector<BfvCiphertext> bfv_mul_and_relin(const std::vector<BfvCiphertext>& a,
                                                    const std::vector<BfvCiphertext>& b, const RelinKey& rlk) {
    if (a.empty()) return {};
    const BfvParamsPtr& prm = a[0].params;
    if (a[0].c.size() != 2 || b[0].c.size() != 2)
        throw ExactoError(1, "invalid parameter: multiplication requires degree-1 ciphertexts");
    detail::load_key(rlk);
    auto fa = detail::flatten(a, 2), fb = detail::flatten(b, 2);
    std::vector<uint64_t> out(fa.size());
    detail::check(exacto_bfv_mul_and_relin(prm->ctx(), fa.data(), fb.data(), out.data(), a.size()));
    return detail::unflatten(out, a.size(), 2, prm);
}

inline BfvCiphertext bfv_mul_no_relin(const BfvCiphertext& a, const BfvCiphertext& b) {
    return bfv_mul_no_relin(std::vector<BfvCiphertext>{a}, std::vector<BfvCiphertext>{b})[0];
}
inline BfvCiphertext relinearize(const BfvCiphertext& ct, const RelinKey& rlk) {
    return relinearize(std::vector<BfvCiphertext>{ct}, rlk)[0];
}
inline BfvCiphertext bfv_mul_and_relin(const BfvCiphertext& a, const BfvCiphertext& b, const RelinKey& rlk) {
    return bfv_mul_and_relin(std::vector<BfvCiphertext>{a}, std::vector<BfvCiphertext>{b}, rlk)[0];
}

// bfv_add / bfv_sub (eval.rs:14-51): each batch has one component count; the two counts may differ
// (the longer operand's extra components pass through, ct2's negated under subtraction)
namespace detail {
inline std::vector<BfvCiphertext> addsub(bool sub, const std::vector<BfvCiphertext>& a,
                                         const std::vector<BfvCiphertext>& b) {
    if (a.empty()) return {};
    if (a.size() != b.size()) throw ExactoError(1, "invalid parameter: batch sizes differ");
    const BfvParamsPtr& prm = a[0].params;
    const size_t p1 = a[0].c.size(), p2 = b[0].c.size(), pm = p1 > p2 ? p1 : p2;
    auto fa = flatten(a, p1), fb = flatten(b, p2);
    std::vector<uint64_t> out(a.size() * pm * prm->num_limbs() * prm->ring_degree);
    check((sub ? exacto_bfv_sub : exacto_bfv_add)(prm->ctx(), fa.data(), p1, fb.data(), p2, out.data(), a.size()));
    return unflatten(out, a.size(), pm, prm);
}
}  // namespace detail
inline std::vector<BfvCiphertext> bfv_add(const std::vector<BfvCiphertext>& a, const std::vector<BfvCiphertext>& b) {
    return detail::addsub(false, a, b);
}
inline std::vector<BfvCiphertext> bfv_sub(const std::vector<BfvCiphertext>& a, const std::vector<BfvCiphertext>& b) {
    return detail::addsub(true, a, b);
}
inline std::vector<BfvCiphertext> bfv_neg(const std::vector<BfvCiphertext>& cts) {
    if (cts.empty()) return {};
    const BfvParamsPtr& prm = cts[0].params;
    const size_t polys = cts[0].c.size();
    auto f = detail::flatten(cts, polys);
    std::vector<uint64_t> out(f.size());
    detail::check(exacto_bfv_neg(prm->ctx(), f.data(), polys, out.data(), cts.size()));
    return detail::unflatten(out, cts.size(), polys, prm);
}
inline BfvCiphertext bfv_add(const BfvCiphertext& a, const BfvCiphertext& b) {
    return bfv_add(std::vector<BfvCiphertext>{a}, std::vector<BfvCiphertext>{b})[0];
}
inline BfvCiphertext bfv_sub(const BfvCiphertext& a, const BfvCiphertext& b) {
    return bfv_sub(std::vector<BfvCiphertext>{a}, std::vector<BfvCiphertext>{b})[0];
}
inline BfvCiphertext bfv_neg(const BfvCiphertext& ct) { return bfv_neg(std::vector<BfvCiphertext>{ct})[0]; }

// decrypt (src/bfv/encrypt.rs:111-178), batched over ciphertexts of one degree.
inline std::vector<CoeffPoly> decrypt(const std::vector<BfvCiphertext>& cts, const SecretKey& sk) {
    if (cts.empty()) return {};
    const BfvParams& prm = *cts[0].params;
    const size_t polys = cts[0].c.size(), n = prm.ring_degree;
    auto flat = detail::flatten(cts, polys);
    std::vector<uint64_t> out(cts.size() * n);
    detail::check(exacto_bfv_decrypt(prm.ctx(), flat.data(), polys, sk.poly.data.data(), out.data(), cts.size()));
    std::vector<CoeffPoly> res(cts.size());
    for (size_t b = 0; b < cts.size(); ++b) {
        res[b].coeffs.assign(out.begin() + (long)(b * n), out.begin() + (long)((b + 1) * n));
        res[b].modulus = prm.plain_modulus;
    }
    return res;
}
inline CoeffPoly decrypt(const BfvCiphertext& ct, const SecretKey& sk) {
    return decrypt(std::vector<BfvCiphertext>{ct}, sk)[0];
}

// ---- key generation / encryption on the device (src/bfv/keygen.rs, src/bfv/encrypt.rs:29-106)
// ChaChaRng stands in for the reference's `R: Rng` argument (ChaCha20Rng): a 256-bit key and a
// stream counter; every call consumes one stream id, as a call consumes words of the reference's
// RNG.  The word stream is this library's own (see include/exacto_hip.h).
struct ChaChaRng {
    uint64_t key[4];
    uint64_t stream = 0;
    explicit ChaChaRng(uint64_t seed) {  // SplitMix64 expansion of a 64-bit seed
        uint64_t z = seed;
        for (auto& k : key) {
            z += 0x9E3779B97F4A7C15ull;
            uint64_t x = z;
            x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
            k = x ^ (x >> 31);
        }
    }
    uint64_t next() { return stream++; }
};

// PublicKey (keygen.rs:28-34): pk0 = -(a s + e), pk1 = a.
struct PublicKey {
    RnsPoly pk0, pk1;
    BfvParamsPtr params;
};

namespace detail {
inline RnsPoly make_poly(const BfvParams& prm, const uint64_t* src) {
    RnsPoly p;
    p.ring_degree = prm.ring_degree;
    p.num_limbs = prm.num_limbs();
    p.data.assign(src, src + p.ring_degree * p.num_limbs);
    return p;
}
}  // namespace detail

// gen_secret_key_with_rng (keygen.rs:64-79)
inline SecretKey gen_secret_key_with_rng(const BfvParamsPtr& prm, ChaChaRng& rng) {
    std::vector<uint64_t> sk(prm->num_limbs() * prm->ring_degree);
    detail::check(exacto_gen_secret_key(prm->ctx(), rng.key, rng.next(), sk.data()));
    return SecretKey{detail::make_poly(*prm, sk.data()), prm};
}

// gen_public_key_with_rng (keygen.rs:87-110)
inline PublicKey gen_public_key_with_rng(const SecretKey& sk, ChaChaRng& rng) {
    const BfvParams& prm = *sk.params;
    const size_t Ln = prm.num_limbs() * prm.ring_degree;
    std::vector<uint64_t> pk(2 * Ln);
    detail::check(exacto_gen_public_key(prm.ctx(), sk.poly.data.data(), prm.sigma, rng.key, rng.next(), pk.data()));
    return PublicKey{detail::make_poly(prm, pk.data()), detail::make_poly(prm, pk.data() + Ln), sk.params};
}

// gen_relin_key_with_rng (keygen.rs:123-162): gadget_digits keys
inline RelinKey gen_relin_key_with_rng(const SecretKey& sk, ChaChaRng& rng) {
    const BfvParams& prm = *sk.params;
    const size_t Ln = prm.num_limbs() * prm.ring_degree, G = prm.gadget_digits;
    std::vector<uint64_t> flat(G * 2 * Ln);
    detail::check(exacto_gen_relin_key(prm.ctx(), sk.poly.data.data(), prm.sigma, rng.key, rng.next(), G,
                                       flat.data()));
    RelinKey rlk;
    rlk.params = sk.params;
    for (size_t g = 0; g < G; ++g)
        rlk.keys.emplace_back(detail::make_poly(prm, flat.data() + 2 * g * Ln),
                              detail::make_poly(prm, flat.data() + (2 * g + 1) * Ln));
    return rlk;
}

// encrypt_sk_with_rng / encrypt_pk_with_rng (encrypt.rs:29-106), batched over plaintexts
inline std::vector<BfvCiphertext> encrypt_batch(const std::vector<CoeffPoly>& pts, const SecretKey* sk,
                                                const PublicKey* pk, const BfvParamsPtr& prm, ChaChaRng& rng) {
    const size_t n = prm->ring_degree, Ln = prm->num_limbs() * n;
    std::vector<uint64_t> pt;
    for (auto& p : pts) {
        if (p.coeffs.size() != n) throw ExactoError(2, "dimension mismatch: expected " + std::to_string(n) +
                                                           ", got " + std::to_string(p.coeffs.size()));
        pt.insert(pt.end(), p.coeffs.begin(), p.coeffs.end());
    }
    std::vector<uint64_t> ct(pts.size() * 2 * Ln);
    if (sk) {
        detail::check(exacto_encrypt_sk(prm->ctx(), pt.data(), sk->poly.data.data(), prm->sigma, rng.key,
                                        rng.next(), ct.data(), pts.size()));
    } else {
        std::vector<uint64_t> pkf(pk->pk0.data);
        pkf.insert(pkf.end(), pk->pk1.data.begin(), pk->pk1.data.end());
        detail::check(exacto_encrypt_pk(prm->ctx(), pt.data(), pkf.data(), prm->sigma, rng.key, rng.next(),
                                        ct.data(), pts.size()));
    }
    return detail::unflatten(ct, pts.size(), 2, prm);
}
inline BfvCiphertext encrypt_sk_with_rng(const CoeffPoly& pt, const SecretKey& sk, const BfvParamsPtr& prm,
                                         ChaChaRng& rng) {
    return encrypt_batch({pt}, &sk, nullptr, prm, rng)[0];
}
inline BfvCiphertext encrypt_pk_with_rng(const CoeffPoly& pt, const PublicKey& pk, const BfvParamsPtr& prm,
                                         ChaChaRng& rng) {
    return encrypt_batch({pt}, nullptr, &pk, prm, rng)[0];
}

// GaloisKey (keygen.rs:49-56) and bfv_apply_automorphism (eval.rs:512-561)
struct GaloisKey {
    std::vector<std::pair<RnsPoly, RnsPoly>> keys;
    size_t element = 0;
    BfvParamsPtr params;
};

inline GaloisKey gen_galois_key_with_rng(const SecretKey& sk, size_t element, ChaChaRng& rng) {
    const BfvParams& prm = *sk.params;
    const size_t Ln = prm.num_limbs() * prm.ring_degree, G = prm.gadget_digits;
    std::vector<uint64_t> flat(G * 2 * Ln);
    detail::check(exacto_gen_galois_key(prm.ctx(), sk.poly.data.data(), element, prm.sigma, rng.key, rng.next(), G,
                                        flat.data()));
    GaloisKey gk;
    gk.element = element;
    gk.params = sk.params;
    for (size_t g = 0; g < G; ++g)
        gk.keys.emplace_back(detail::make_poly(prm, flat.data() + 2 * g * Ln),
                             detail::make_poly(prm, flat.data() + (2 * g + 1) * Ln));
    return gk;
}

inline std::vector<BfvCiphertext> bfv_apply_automorphism(const std::vector<BfvCiphertext>& cts, const GaloisKey& gk) {
    if (cts.empty()) return {};
    const BfvParams& prm = *cts[0].params;
    const size_t polys = cts[0].c.size();
    if (polys != 2) throw ExactoError(1, "invalid parameter: automorphism requires degree-1 ciphertext");
    auto flat = detail::flatten(cts, polys);
    std::vector<uint64_t> key;
    for (auto& k : gk.keys) {
        key.insert(key.end(), k.first.data.begin(), k.first.data.end());
        key.insert(key.end(), k.second.data.begin(), k.second.data.end());
    }
    std::vector<uint64_t> out(flat.size());
    detail::check(exacto_bfv_apply_automorphism(prm.ctx(), flat.data(), polys, gk.element, key.data(),
                                                gk.keys.size(), out.data(), cts.size()));
    return detail::unflatten(out, cts.size(), 2, cts[0].params);
}
inline BfvCiphertext bfv_apply_automorphism(const BfvCiphertext& ct, const GaloisKey& gk) {
    return bfv_apply_automorphism(std::vector<BfvCiphertext>{ct}, gk)[0];
}

// encode_scalar / decode_scalar (src/bfv/encoding.rs:7-20)
inline CoeffPoly encode_scalar(uint64_t m, const BfvParamsPtr& prm) {
    if (m >= prm->plain_modulus)
        throw ExactoError(1, "invalid parameter: plaintext " + std::to_string(m) + " >= plain_modulus " +
                                 std::to_string(prm->plain_modulus));
    CoeffPoly p;
    p.coeffs.assign(prm->ring_degree, 0);
    p.coeffs[0] = m;
    p.modulus = prm->plain_modulus;
    return p;
}
inline uint64_t decode_scalar(const CoeffPoly& p) { return p.coeffs.empty() ? 0 : p.coeffs[0]; }

// ---- plaintext operations and the trace (src/bfv/eval.rs:468-652)
namespace detail {
inline std::vector<uint64_t> flatten_pts(const std::vector<CoeffPoly>& pts, size_t n) {
    std::vector<uint64_t> out;
    for (auto& p : pts) {
        if (p.coeffs.size() != n) throw ExactoError(2, "dimension mismatch: expected " + std::to_string(n) +
                                                           ", got " + std::to_string(p.coeffs.size()));
        out.insert(out.end(), p.coeffs.begin(), p.coeffs.end());
    }
    return out;
}
inline BfvCiphertext one_ct(const std::vector<uint64_t>& flat, size_t polys, const BfvParamsPtr& prm) {
    return unflatten(flat, 1, polys, prm)[0];
}
}  // namespace detail

inline BfvCiphertext bfv_plain_mul(const BfvCiphertext& ct, const CoeffPoly& pt) {
    const BfvParams& prm = *ct.params;
    auto flat = detail::flatten({ct}, ct.c.size());
    auto p = detail::flatten_pts({pt}, prm.ring_degree);
    std::vector<uint64_t> out(flat.size());
    detail::check(exacto_bfv_plain_mul(prm.ctx(), flat.data(), ct.c.size(), p.data(), out.data(), 1));
    return detail::one_ct(out, ct.c.size(), ct.params);
}
inline BfvCiphertext bfv_plain_add(const BfvCiphertext& ct, const CoeffPoly& pt) {
    const BfvParams& prm = *ct.params;
    auto flat = detail::flatten({ct}, ct.c.size());
    auto p = detail::flatten_pts({pt}, prm.ring_degree);
    std::vector<uint64_t> out(flat.size());
    detail::check(exacto_bfv_plain_add(prm.ctx(), flat.data(), ct.c.size(), p.data(), out.data(), 1));
    return detail::one_ct(out, ct.c.size(), ct.params);
}
inline BfvCiphertext bfv_monomial_mul(const BfvCiphertext& ct, size_t j) {
    const BfvParams& prm = *ct.params;
    auto flat = detail::flatten({ct}, ct.c.size());
    std::vector<uint64_t> out(flat.size());
    detail::check(exacto_bfv_monomial_mul(prm.ctx(), flat.data(), ct.c.size(), j, out.data(), 1));
    return detail::one_ct(out, ct.c.size(), ct.params);
}
inline BfvCiphertext bfv_inner_product(const std::vector<BfvCiphertext>& cts, const std::vector<CoeffPoly>& pts) {
    if (cts.empty() || cts.size() != pts.size()) throw ExactoError(1, "invalid parameter: mismatched ct/pt lengths");
    const BfvParams& prm = *cts[0].params;
    const size_t polys = cts[0].c.size();
    auto flat = detail::flatten(cts, polys);
    auto p = detail::flatten_pts(pts, prm.ring_degree);
    std::vector<uint64_t> out(polys * prm.num_limbs() * prm.ring_degree);
    detail::check(exacto_bfv_inner_product(prm.ctx(), flat.data(), p.data(), cts.size(), polys, out.data()));
    return detail::one_ct(out, polys, cts[0].params);
}

// HashMap<usize, GaloisKey> of the reference
using GaloisKeys = std::map<size_t, GaloisKey>;
namespace detail {
// the map as (elements, keys stacked in that order); every key must carry the same digit count
inline size_t pack_keys(const GaloisKeys& keys, std::vector<uint64_t>& els, std::vector<uint64_t>& flat) {
    size_t nk = 0;
    for (auto& kv : keys) {
        if (nk == 0) nk = kv.second.keys.size();
        if (kv.second.keys.size() != nk) throw ExactoError(1, "invalid parameter: Galois keys differ in digit count");
        els.push_back(kv.first);
        for (auto& k : kv.second.keys) {
            flat.insert(flat.end(), k.first.data.begin(), k.first.data.end());
            flat.insert(flat.end(), k.second.data.begin(), k.second.data.end());
        }
    }
    return nk;
}
}  // namespace detail

// bfv_trace (eval.rs:572-586)
inline BfvCiphertext bfv_trace(const BfvCiphertext& ct, const std::vector<size_t>& elements, const GaloisKeys& keys) {
    const BfvParams& prm = *ct.params;
    std::vector<uint64_t> els, flat;
    size_t nk = 0;
    for (size_t k : elements) {
        auto it = keys.find(k);
        if (it == keys.end()) throw ExactoError(1, "invalid parameter: missing Galois key for element " + std::to_string(k));
        if (nk == 0) nk = it->second.keys.size();
        els.push_back(k);
        for (auto& kp : it->second.keys) {
            flat.insert(flat.end(), kp.first.data.begin(), kp.first.data.end());
            flat.insert(flat.end(), kp.second.data.begin(), kp.second.data.end());
        }
    }
    auto c = detail::flatten({ct}, ct.c.size());
    std::vector<uint64_t> out(c.size());
    detail::check(exacto_bfv_trace(prm.ctx(), c.data(), ct.c.size(), els.data(), els.size(),
                                   flat.empty() ? nullptr : flat.data(), nk, out.data(), 1));
    return detail::one_ct(out, ct.c.size(), ct.params);
}

// ---- exacto::bootstrap::coeffs_to_slots (src/bootstrap/coeffs_to_slots.rs)
inline std::vector<size_t> required_trace_elements(size_t n) {
    std::vector<uint64_t> v(exacto_required_trace_elements(n, nullptr, 0));
    exacto_required_trace_elements(n, v.data(), v.size());
    return std::vector<size_t>(v.begin(), v.end());
}
inline GaloisKeys gen_trace_galois_keys(const SecretKey& sk, ChaChaRng& rng) {
    GaloisKeys keys;
    for (size_t k : required_trace_elements(sk.params->ring_degree)) keys[k] = gen_galois_key_with_rng(sk, k, rng);
    return keys;
}
inline GaloisKeys gen_all_galois_keys(const SecretKey& sk, ChaChaRng& rng) {
    GaloisKeys keys;
    for (size_t k = 3; k < 2 * sk.params->ring_degree; k += 2) keys[k] = gen_galois_key_with_rng(sk, k, rng);
    return keys;
}
namespace detail {
inline std::vector<BfvCiphertext> extract_range(const BfvCiphertext& ct, size_t j0, size_t count,
                                                const GaloisKeys& keys) {
    const BfvParams& prm = *ct.params;
    if (ct.c.size() != 2) throw ExactoError(1, "invalid parameter: automorphism requires degree-1 ciphertext");
    std::vector<uint64_t> els, flat;
    const size_t nk = pack_keys(keys, els, flat);
    auto c = flatten({ct}, 2);
    std::vector<uint64_t> out(count * c.size());
    check(exacto_extract_coefficients(prm.ctx(), c.data(), j0, count, els.data(), els.size(),
                                      flat.empty() ? nullptr : flat.data(), nk, out.data()));
    return unflatten(out, count, 2, ct.params);
}
}  // namespace detail
inline BfvCiphertext extract_coefficient(const BfvCiphertext& ct, size_t j, const GaloisKeys& keys) {
    return detail::extract_range(ct, j, 1, keys)[0];
}
inline std::vector<BfvCiphertext> coeffs_to_slots(const BfvCiphertext& ct, const GaloisKeys& keys) {
    return detail::extract_range(ct, 0, ct.params->ring_degree, keys);
}
inline BfvCiphertext slots_to_coeffs(const std::vector<BfvCiphertext>& slots) {
    if (slots.empty()) throw ExactoError(1, "invalid parameter: empty slots");
    const BfvParams& prm = *slots[0].params;
    const size_t polys = slots[0].c.size();
    auto flat = detail::flatten(slots, polys);
    std::vector<uint64_t> out(polys * prm.num_limbs() * prm.ring_degree);
    detail::check(exacto_slots_to_coeffs(prm.ctx(), flat.data(), slots.size(), polys, out.data()));
    return detail::one_ct(out, polys, slots[0].params);
}

// ---- exacto::bootstrap::digit_extract (src/bootstrap/digit_extract.rs)
inline std::vector<uint64_t> lagrange_interpolate(const std::vector<uint64_t>& values, uint64_t p) {
    std::vector<uint64_t> out(values.size());
    if (!values.empty()) detail::check(exacto_lagrange_interpolate(values.data(), values.size(), p, out.data()));
    return out;
}
inline std::vector<uint64_t> compute_rounding_poly(uint64_t t_orig, uint64_t q_prime, uint64_t t_boot) {
    std::vector<uint64_t> out(t_boot);
    detail::check(exacto_compute_rounding_poly(t_orig, q_prime, t_boot, out.data()));
    return out;
}
inline BfvCiphertext trivial_encrypt_poly(const CoeffPoly& pt, const BfvParamsPtr& prm) {
    auto p = detail::flatten_pts({pt}, prm->ring_degree);
    std::vector<uint64_t> out(2 * prm->num_limbs() * prm->ring_degree);
    detail::check(exacto_trivial_encrypt(prm->ctx(), p.data(), out.data(), 1));
    return detail::one_ct(out, 2, prm);
}
inline BfvCiphertext trivial_encrypt(uint64_t m, const BfvParamsPtr& prm) {
    CoeffPoly p;
    p.coeffs.assign(prm->ring_degree, 0);
    p.coeffs[0] = m % prm->plain_modulus;
    p.modulus = prm->plain_modulus;
    return trivial_encrypt_poly(p, prm);
}
inline BfvCiphertext eval_poly_homomorphic(const BfvCiphertext& ct, const std::vector<uint64_t>& coeffs,
                                           const RelinKey& rlk) {
    const BfvParams& prm = *ct.params;
    if (coeffs.size() > 1) detail::load_key(rlk);
    auto c = detail::flatten({ct}, 2);
    std::vector<uint64_t> out(c.size());
    detail::check(exacto_eval_poly(prm.ctx(), c.data(), coeffs.data(), coeffs.size(), out.data(), 1));
    return detail::one_ct(out, 2, ct.params);
}

// ---- exacto::bootstrap::bfv_host (src/bootstrap/bfv_host.rs)
struct BootstrapKey {
    BfvCiphertext bsk;
    BfvParamsPtr boot_params;
    RelinKey boot_rlk;
    GaloisKeys galois_keys;
    std::vector<uint64_t> rounding_poly;
    uint64_t t_orig = 0, q_prime = 0;
    SecretKey boot_sk;  // create_boot_sk's key (the reference recomputes it in its tests)
};

inline BootstrapKey gen_bootstrap_key(const SecretKey& sk, const BfvParamsPtr& boot_params, uint64_t q_prime,
                                      uint64_t t_orig, ChaChaRng& rng) {
    const BfvParams& o = *sk.params;
    const size_t n = o.ring_degree;
    std::vector<uint64_t> boot_sk(boot_params->num_limbs() * n), s_pt(n);
    detail::check(exacto_bootstrap_key_material(o.ctx(), boot_params->ctx(), sk.poly.data.data(), boot_sk.data(),
                                                s_pt.data()));
    BootstrapKey k;
    k.boot_params = boot_params;
    k.boot_sk = SecretKey{detail::make_poly(*boot_params, boot_sk.data()), boot_params};
    CoeffPoly spt{s_pt, boot_params->plain_modulus};
    k.bsk = encrypt_sk_with_rng(spt, k.boot_sk, boot_params, rng);
    k.boot_rlk = gen_relin_key_with_rng(k.boot_sk, rng);
    k.galois_keys = gen_trace_galois_keys(k.boot_sk, rng);
    k.rounding_poly = compute_rounding_poly(t_orig, q_prime, boot_params->plain_modulus);
    k.t_orig = t_orig;
    k.q_prime = q_prime;
    return k;
}

inline std::vector<BfvCiphertext> bfv_bootstrap(const std::vector<BfvCiphertext>& cts, const BootstrapKey& bsk) {
    if (cts.empty()) return {};
    const BfvParams& o = *cts[0].params;
    const BfvParams& b = *bsk.boot_params;
    if (cts[0].c.size() != 2) throw ExactoError(1, "invalid parameter: bootstrap requires degree-1 ciphertext");
    detail::load_key(bsk.boot_rlk);
    auto flat = detail::flatten(cts, 2);
    auto key = detail::flatten({bsk.bsk}, 2);
    std::vector<uint64_t> els, gks;
    const size_t nk = detail::pack_keys(bsk.galois_keys, els, gks);
    std::vector<uint64_t> out(cts.size() * 2 * b.num_limbs() * b.ring_degree);
    detail::check(exacto_bfv_bootstrap(o.ctx(), b.ctx(), flat.data(), 2, key.data(), bsk.rounding_poly.data(),
                                       bsk.rounding_poly.size(), bsk.q_prime, els.data(), els.size(),
                                       gks.empty() ? nullptr : gks.data(), nk, out.data(), cts.size()));
    return detail::unflatten(out, cts.size(), 2, bsk.boot_params);
}
inline BfvCiphertext bfv_bootstrap(const BfvCiphertext& ct, const BootstrapKey& bsk) {
    return bfv_bootstrap(std::vector<BfvCiphertext>{ct}, bsk)[0];
}

// ---- exacto::dbfv
struct DbfvParams {
    BfvParamsPtr bfv_params;
    uint64_t base;
    size_t num_digits;
    uint64_t plain_modulus;  // 0 == 2^64
};

struct DbfvCiphertext {
    std::vector<BfvCiphertext> limbs;
    size_t degree = 0;
    size_t mul_depth = 0;
    std::shared_ptr<const DbfvParams> params;
    size_t num_limbs() const { return limbs.size(); }
};

// dbfv_mul (src/dbfv/eval.rs:82-149), batched over independent products.
inline std::vector<DbfvCiphertext> dbfv_mul(const std::vector<DbfvCiphertext>& a,
                                            const std::vector<DbfvCiphertext>& b, const RelinKey& rlk) {
    if (a.empty()) return {};
    const auto& dp = *a[0].params;
    const size_t d = dp.num_digits;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].num_limbs() != d || b[i].num_limbs() != d)
            throw ExactoError(1, "invalid parameter: multiplication requires d-limb ciphertexts");
    detail::load_key(rlk);
    std::vector<uint64_t> fa, fb;
    std::vector<uint32_t> da, db, dout(a.size());
    for (size_t i = 0; i < a.size(); ++i) {
        auto x = detail::flatten(a[i].limbs, 2), y = detail::flatten(b[i].limbs, 2);
        fa.insert(fa.end(), x.begin(), x.end());
        fb.insert(fb.end(), y.begin(), y.end());
        da.push_back((uint32_t)a[i].mul_depth);
        db.push_back((uint32_t)b[i].mul_depth);
    }
    std::vector<uint64_t> out(fa.size());
    detail::check(exacto_dbfv_mul(dp.bfv_params->ctx(), d, dp.base, dp.plain_modulus, fa.data(), fb.data(),
                                  out.data(), a.size(), da.data(), db.data(), dout.data()));
    std::vector<DbfvCiphertext> res(a.size());
    const size_t per = d * 2 * dp.bfv_params->num_limbs() * dp.bfv_params->ring_degree;
    for (size_t i = 0; i < a.size(); ++i) {
        std::vector<uint64_t> slice(out.begin() + (long)(i * per), out.begin() + (long)((i + 1) * per));
        res[i].limbs = detail::unflatten(slice, d, 2, dp.bfv_params);
        res[i].degree = d;
        res[i].mul_depth = dout[i];
        res[i].params = a[0].params;
    }
    return res;
}

inline DbfvCiphertext dbfv_mul(const DbfvCiphertext& a, const DbfvCiphertext& b, const RelinKey& rlk) {
    return dbfv_mul(std::vector<DbfvCiphertext>{a}, std::vector<DbfvCiphertext>{b}, rlk)[0];
}

namespace detail {
inline std::vector<uint64_t> flatten_dbfv(const DbfvCiphertext& ct) {
    if (ct.num_limbs() != ct.params->num_digits)
        throw ExactoError(1, "invalid parameter: expected d-limb dBFV ciphertext");
    return flatten(ct.limbs, 2);
}
}  // namespace detail

// dbfv_decrypt (src/dbfv/decrypt.rs:20-43): scalar plaintext (coefficient 0).
inline uint64_t dbfv_decrypt(const DbfvCiphertext& ct, const SecretKey& sk) {
    const auto& dp = *ct.params;
    auto flat = detail::flatten_dbfv(ct);
    uint64_t out = 0;
    detail::check(exacto_dbfv_decrypt(dp.bfv_params->ctx(), dp.num_digits, dp.base, dp.plain_modulus, flat.data(),
                                      sk.poly.data.data(), &out, 1));
    return out;
}

// dbfv_decrypt_poly (src/dbfv/decrypt.rs:48-79).
inline CoeffPoly dbfv_decrypt_poly(const DbfvCiphertext& ct, const SecretKey& sk) {
    const auto& dp = *ct.params;
    auto flat = detail::flatten_dbfv(ct);
    CoeffPoly res;
    res.coeffs.resize(dp.bfv_params->ring_degree);
    res.modulus = dp.plain_modulus;
    detail::check(exacto_dbfv_decrypt_poly(dp.bfv_params->ctx(), dp.num_digits, dp.base, dp.plain_modulus,
                                           flat.data(), sk.poly.data.data(), res.coeffs.data(), 1));
    return res;
}

// The benchmark chain of src/bin/paper_repro.rs:203-236: x * y^depth with mul_depth reset before
// every dbfv_mul (guard bypass), run device-resident in one call.
inline DbfvCiphertext dbfv_mul_chain(const DbfvCiphertext& x, const DbfvCiphertext& y, const RelinKey& rlk,
                                     size_t depth) {
    const auto& dp = *x.params;
    detail::load_key(rlk);
    auto fx = detail::flatten_dbfv(x), fy = detail::flatten_dbfv(y);
    std::vector<uint64_t> out(fx.size());
    detail::check(exacto_dbfv_mul_chain(dp.bfv_params->ctx(), dp.num_digits, dp.base, dp.plain_modulus, fx.data(),
                                        fy.data(), out.data(), 1, depth));
    DbfvCiphertext res;
    res.limbs = detail::unflatten(out, dp.num_digits, 2, dp.bfv_params);
    res.degree = dp.num_digits;
    res.mul_depth = depth ? 1 : x.mul_depth;
    res.params = x.params;
    return res;
}


// One GPU's share of a dbfv_mul split by output limb (dbfv/eval.rs:109-132): the limbs `limbs` of each
// product a[i] * b[i] (mul_depth 0 inputs), as BfvCiphertexts [item][slot] (exacto_dbfv_mul_limbs).
inline std::vector<std::vector<BfvCiphertext>> dbfv_mul_limbs(const std::vector<DbfvCiphertext>& a,
                                                             const std::vector<DbfvCiphertext>& b,
                                                             const RelinKey& rlk, const std::vector<uint32_t>& limbs) {
    if (a.empty()) return {};
    const auto& dp = *a[0].params;
    detail::load_key(rlk);
    std::vector<uint64_t> fa, fb;
    for (size_t i = 0; i < a.size(); ++i) {
        auto x = detail::flatten_dbfv(a[i]), y = detail::flatten_dbfv(b[i]);
        fa.insert(fa.end(), x.begin(), x.end());
        fb.insert(fb.end(), y.begin(), y.end());
    }
    const size_t per = 2 * dp.bfv_params->num_limbs() * dp.bfv_params->ring_degree;
    std::vector<uint64_t> out(a.size() * limbs.size() * per);
    detail::check(exacto_dbfv_mul_limbs(dp.bfv_params->ctx(), dp.num_digits, dp.base, dp.plain_modulus, fa.data(),
                                        fb.data(), out.data(), a.size(), limbs.data(), limbs.size()));
    std::vector<std::vector<BfvCiphertext>> res(a.size());
    for (size_t i = 0; i < a.size(); ++i)
        res[i] = detail::unflatten(std::vector<uint64_t>(out.begin() + (long)(i * limbs.size() * per),
                                                         out.begin() + (long)((i + 1) * limbs.size() * per)),
                                   limbs.size(), 2, dp.bfv_params);
    return res;
}

// ---- RCCL over xGMI (exacto_hip.h): one communicator per GPU, keys broadcast from one root
class RcclComm {
  public:
    // ncclGetUniqueId on the root; every rank passes the same 128 bytes
    static std::vector<uint8_t> unique_id() {
        std::vector<uint8_t> id(128);
        detail::check(exacto_rccl_unique_id(id.data()));
        return id;
    }
    RcclComm(int nranks, const std::vector<uint8_t>& id, int rank, int device) {
        detail::check(exacto_rccl_comm_init(&h_, nranks, id.data(), rank, device));
    }
    ~RcclComm() { exacto_rccl_comm_destroy(h_); }
    RcclComm(const RcclComm&) = delete;
    RcclComm& operator=(const RcclComm&) = delete;
    void* handle() const { return h_; }

  private:
    void* h_ = nullptr;
};

// The root's relinearisation key (loaded with load_relin_key / generated on its device) becomes the
// resident key of every rank's context (ncclBroadcast in place): keys are made once, keygen.rs:123-162.
inline void broadcast_relin_key(const BfvParams& prm, const RcclComm& comm, int root, size_t num_keys) {
    detail::check(exacto_ctx_broadcast_relin_key(prm.ctx(), comm.handle(), root, num_keys));
    prm.loaded_key = nullptr;   // resident contents now come from the root
}

}  // namespace exacto
