// C++ host-API tests (include/exacto.hpp), mirroring the reference's Rust tests of the path.
// Usage: test_api <fixture-dir> <case>...   (fixtures written by tests/test_cpp_api.py from
// tests/golden/vectors.npz).  Prints "PASS <name>" per case and "ALL OK" at the end.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "exacto.hpp"

using namespace exacto;

static std::vector<uint64_t> read_u64(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("missing " + path);
    const auto bytes = (size_t)f.tellg();
    std::vector<uint64_t> v(bytes / 8);
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
    return v;
}

struct Meta {
    size_t n, L, K;
    uint64_t plain, gbase;
    std::vector<uint64_t> q, aux;
    size_t d = 0;
    uint64_t base = 0, dplain = 0;
};

static Meta read_meta(const std::string& path) {
    std::ifstream f(path);
    Meta m{};
    f >> m.n >> m.L >> m.K >> m.plain >> m.gbase;
    m.q.resize(m.L);
    for (auto& x : m.q) f >> x;
    m.aux.resize(m.K);
    for (auto& x : m.aux) f >> x;
    f >> m.d >> m.base >> m.dplain;
    return m;
}

static std::vector<BfvCiphertext> to_cts(const std::vector<uint64_t>& flat, size_t batch, size_t polys,
                                         const BfvParamsPtr& prm) {
    return detail::unflatten(flat, batch, polys, prm);
}

static RelinKey to_rlk(const std::vector<uint64_t>& flat, const BfvParamsPtr& prm) {
    const size_t Ln = prm->num_limbs() * prm->ring_degree;
    RelinKey k;
    k.params = prm;
    for (size_t g = 0; g * 2 * Ln < flat.size(); ++g) {
        RnsPoly a{prm->ring_degree, prm->num_limbs(), {}}, b = a;
        a.data.assign(flat.begin() + (long)(2 * g * Ln), flat.begin() + (long)((2 * g + 1) * Ln));
        b.data.assign(flat.begin() + (long)((2 * g + 1) * Ln), flat.begin() + (long)((2 * g + 2) * Ln));
        k.keys.push_back({a, b});
    }
    return k;
}

static bool same(const std::vector<BfvCiphertext>& got, const std::vector<uint64_t>& want) {
    std::vector<uint64_t> flat;
    for (auto& ct : got)
        for (auto& p : ct.c) flat.insert(flat.end(), p.data.begin(), p.data.end());
    return flat == want;
}

static int run_case(const std::string& dir, const std::string& name) {
    const Meta m = read_meta(dir + "/" + name + ".meta");
    auto prm = BfvParamsBuilder().ring_degree(m.n).plain_modulus(m.plain).ct_moduli(m.q).aux_moduli(m.aux)
                   .gadget_base(m.gbase).sigma(3.2).build();
    const size_t Ln = m.L * m.n;
    const RelinKey rlk = to_rlk(read_u64(dir + "/" + name + ".rlk.u64"), prm);
    if (m.d == 0) {
        const auto c1 = read_u64(dir + "/" + name + ".ct1.u64");
        const size_t B = c1.size() / (2 * Ln);
        auto a = to_cts(c1, B, 2, prm);
        auto b = to_cts(read_u64(dir + "/" + name + ".ct2.u64"), B, 2, prm);
        // eval.rs:73 bfv_mul_and_relin, batched and single
        const auto want = read_u64(dir + "/" + name + ".out.u64");
        if (!same(bfv_mul_and_relin(a, b, rlk), want)) return 1;
        auto one = bfv_mul_and_relin(a[0], b[0], rlk);
        if (!same({one}, std::vector<uint64_t>(want.begin(), want.begin() + (long)(2 * Ln)))) return 2;
        // eval.rs:89 bfv_mul_no_relin + keyswitch.rs:59 relinearize
        auto three = bfv_mul_no_relin(a, b);
        if (!same(three, read_u64(dir + "/" + name + ".out3.u64"))) return 3;
        if (!same(relinearize(three, rlk), read_u64(dir + "/" + name + ".out.u64"))) return 4;
    } else {
        auto dp = std::make_shared<DbfvParams>(DbfvParams{prm, m.base, m.d, m.dplain});
        const auto fa = read_u64(dir + "/" + name + ".a.u64");
        const auto fb = read_u64(dir + "/" + name + ".b.u64");
        const size_t per = m.d * 2 * Ln, B = fa.size() / per;
        std::vector<DbfvCiphertext> A(B), Bc(B);
        for (size_t i = 0; i < B; ++i) {
            A[i].limbs = to_cts(std::vector<uint64_t>(fa.begin() + (long)(i * per), fa.begin() + (long)((i + 1) * per)), m.d, 2, prm);
            Bc[i].limbs = to_cts(std::vector<uint64_t>(fb.begin() + (long)(i * per), fb.begin() + (long)((i + 1) * per)), m.d, 2, prm);
            A[i].degree = Bc[i].degree = m.d;
            A[i].params = Bc[i].params = dp;
        }
        auto r = dbfv_mul(A, Bc, rlk);
        std::vector<BfvCiphertext> limbs;
        for (auto& x : r) {
            if (x.mul_depth != 1 || x.degree != m.d) return 5;
            limbs.insert(limbs.end(), x.limbs.begin(), x.limbs.end());
        }
        const auto want = read_u64(dir + "/" + name + ".out.u64");
        if (!same(limbs, want)) return 6;
        // one GPU's share of a limb-split dbfv_mul: each limb, in reverse order, equals dbfv_mul's
        std::vector<uint32_t> rev;
        for (size_t k = m.d; k-- > 0;) rev.push_back((uint32_t)k);
        auto part = dbfv_mul_limbs(A, Bc, rlk, rev);
        for (size_t i = 0; i < B; ++i)
            for (size_t s = 0; s < rev.size(); ++s)
                if (part[i][s].c.size() != 2 || part[i][s].c[0].data != r[i].limbs[rev[s]].c[0].data ||
                    part[i][s].c[1].data != r[i].limbs[rev[s]].c[1].data)
                    return 44;
        // paper_repro.rs:203-236 chain: depth 1 is one dbfv_mul, depth 0 the input
        if (!same(dbfv_mul_chain(A[0], Bc[0], rlk, 1).limbs,
                  std::vector<uint64_t>(want.begin(), want.begin() + (long)per)))
            return 9;
        // dbfv/eval.rs:292-313: chained multiplication is rejected
        try {
            dbfv_mul(r[0], Bc[0], rlk);
            return 7;
        } catch (const ExactoError& e) {
            if (std::string(e.variant()) != "NotImplemented" ||
                std::string(e.what()).find("chained dBFV multiplication requires ciphertext-level lattice reduction") ==
                    std::string::npos)
                return 8;
        }
    }
    return 0;
}

static int error_cases() {
    // eval.rs:93-97 and keyswitch.rs:66-70 messages; params/mod.rs:82-90 builder errors
    try {
        BfvParamsBuilder().ring_degree(12).ct_moduli({65537}).build();
        return 10;
    } catch (const ExactoError& e) {
        if (std::string(e.variant()) != "InvalidRingDegree") return 11;
    }
    try {
        BfvParamsBuilder().ring_degree(16).build();
        return 12;
    } catch (const ExactoError& e) {
        if (std::string(e.what()) != "invalid parameter: must specify at least one ciphertext modulus") return 13;
    }
    auto prm = BfvParamsBuilder().ring_degree(16).plain_modulus(257).ct_moduli({65537, 1099509805057}).gadget_base(8).build();
    RnsPoly z{16, 2, std::vector<uint64_t>(32, 0)};
    BfvCiphertext c3{{z, z, z}, prm};
    RelinKey rlk{{}, prm};
    try {
        bfv_mul_and_relin(c3, c3, rlk);
        return 14;
    } catch (const ExactoError& e) {
        if (std::string(e.what()).find("multiplication requires degree-1 ciphertexts") == std::string::npos) return 15;
    }
    BfvCiphertext c4{{z, z, z, z}, prm};
    try {
        relinearize(c4, rlk);
        return 16;
    } catch (const ExactoError& e) {
        if (std::string(e.what()).find("relinearization only supports degree-2 ciphertexts") == std::string::npos) return 17;
    }
    // encrypt.rs:111-178 known answer: s = 0, c0 = Delta*m (constant, so every evaluation is
    // Delta*m), Delta = floor(q/p) = 255 for q = 65537, p = 257 -> decrypts to m, other coeffs 0
    {
        auto p1 = BfvParamsBuilder().ring_degree(16).plain_modulus(257).ct_moduli({65537}).build();
        RnsPoly c0{16, 1, std::vector<uint64_t>(16, 255 * 7)}, c1{16, 1, std::vector<uint64_t>(16, 12345)};
        SecretKey sk{RnsPoly{16, 1, std::vector<uint64_t>(16, 0)}, p1};
        auto m = decrypt(BfvCiphertext{{c0, c1}, p1}, sk);
        if (m.modulus != 257 || m.coeffs[0] != 7) return 18;
        for (size_t i = 1; i < 16; ++i)
            if (m.coeffs[i] != 0) return 19;
    }
    return 0;
}

// keygen.rs / encrypt.rs on the device through the C++ mirror: the reference's own round trips
// (encrypt.rs:262-285 sk/pk encrypt-decrypt of 42; eval.rs:883-899 3 * 7 = 21 with relinearisation)
static int keygen_case() {
    auto prm = BfvParamsBuilder().ring_degree(1024).plain_modulus(257).ct_moduli({1099509805057ull})
                   .aux_moduli({562949953443841ull}).sigma(3.2).build();
    ChaChaRng rng(42);
    auto sk = gen_secret_key_with_rng(prm, rng);
    auto pk = gen_public_key_with_rng(sk, rng);
    auto rlk = gen_relin_key_with_rng(sk, rng);
    if (rlk.keys.size() != prm->gadget_digits) return 20;
    if (decode_scalar(decrypt(encrypt_sk_with_rng(encode_scalar(42, prm), sk, prm, rng), sk)) != 42) return 21;
    if (decode_scalar(decrypt(encrypt_pk_with_rng(encode_scalar(42, prm), pk, prm, rng), sk)) != 42) return 22;
    auto c3 = encrypt_sk_with_rng(encode_scalar(3, prm), sk, prm, rng);
    auto c7 = encrypt_pk_with_rng(encode_scalar(7, prm), pk, prm, rng);
    if (decode_scalar(decrypt(bfv_mul_and_relin(c3, c7, rlk), sk)) != 21) return 23;
    // eval.rs:14-60: add / sub / neg, equal and mixed degrees (degree-2 product + degree-1 ct)
    if (decode_scalar(decrypt(bfv_add(c3, c7), sk)) != 10) return 25;
    if (decode_scalar(decrypt(bfv_sub(c3, c7), sk)) != 257 - 4) return 26;
    if (decode_scalar(decrypt(bfv_neg(c3), sk)) != 257 - 3) return 27;
    auto c21 = bfv_mul_no_relin(c3, c7);
    auto mixed = bfv_add(c21, c3);
    if (mixed.c.size() != 3 || decode_scalar(decrypt(mixed, sk)) != 24) return 28;
    auto mixed2 = bfv_sub(c3, c21);
    if (mixed2.c.size() != 3 || decode_scalar(decrypt(mixed2, sk)) != 257 - 18) return 29;
    // RCCL entry points over a one-rank communicator: the resident key broadcast in place (then the
    // product still decrypts), a device Galois-key buffer broadcast, an in-place all-gather
    {
        detail::load_key(rlk);
        RcclComm comm(1, RcclComm::unique_id(), 0, 0);
        broadcast_relin_key(*prm, comm, 0, rlk.keys.size());
        if (decode_scalar(decrypt(bfv_mul_and_relin(c3, c7, rlk), sk)) != 21) return 40;
        uint64_t* dev = exacto_ctx_relin_key_buffer(prm->ctx(), rlk.keys.size());
        if (!dev) return 41;
        detail::check(exacto_broadcast_galois_key(prm->ctx(), comm.handle(), 0, dev, rlk.keys.size()));
        detail::check(exacto_rccl_allgather_u64(prm->ctx(), comm.handle(), dev, dev, 1024));
        detail::check(exacto_synchronize(prm->ctx()));
        if (exacto_ctx_broadcast_relin_key(prm->ctx(), comm.handle(), 3, rlk.keys.size()) != EXACTO_ERR_INVALID_PARAM)
            return 42;
        if (decode_scalar(decrypt(bfv_mul_and_relin(c3, c7, rlk), sk)) != 21) return 43;
    }
    // eval.rs:954-976: sigma_3(1 + 2X) = 1 + 2X^3
    CoeffPoly m;
    m.coeffs.assign(prm->ring_degree, 0);
    m.coeffs[0] = 1;
    m.coeffs[1] = 2;
    m.modulus = prm->plain_modulus;
    auto gk = gen_galois_key_with_rng(sk, 3, rng);
    auto d = decrypt(bfv_apply_automorphism(encrypt_sk_with_rng(m, sk, prm, rng), gk), sk);
    if (d.coeffs[0] != 1 || d.coeffs[1] != 0 || d.coeffs[2] != 0 || d.coeffs[3] != 2) return 24;
    return 0;
}

// coeffs_to_slots.rs:221-318, digit_extract.rs:270-288, eval.rs:978-994, bfv_host.rs:430-476
// through the C++ mirror of the bootstrap API
static int bootstrap_case() {
    auto small = BfvParamsBuilder().ring_degree(16).plain_modulus(97).ct_moduli({1125899906842817ull}).sigma(3.2)
                     .gadget_base(8).build();
    ChaChaRng rng(42);
    auto sk = gen_secret_key_with_rng(small, rng);
    auto keys = gen_all_galois_keys(sk, rng);
    CoeffPoly m;
    m.modulus = 97;
    for (uint64_t i = 1; i <= 16; ++i) m.coeffs.push_back(i % 97);
    auto ct = encrypt_sk_with_rng(m, sk, small, rng);
    auto slots = coeffs_to_slots(ct, keys);
    for (size_t j = 0; j < 16; ++j)
        if (decode_scalar(decrypt(slots[j], sk)) != m.coeffs[j]) return 30;
    auto back = decrypt(slots_to_coeffs(slots), sk);
    if (back.coeffs != m.coeffs) return 31;
    if (decode_scalar(decrypt(extract_coefficient(ct, 2, keys), sk)) != 3) return 32;
    // regression: a batched extraction after a single one (scratch reuse across calls) is exact
    for (int rep = 0; rep < 3; ++rep)
        if (decode_scalar(decrypt(coeffs_to_slots(ct, keys)[2], sk)) != 3) return 39;
    if (required_trace_elements(64) != std::vector<size_t>{65, 33, 17, 9, 5, 3}) return 33;
    auto compact = BfvParamsBuilder().ring_degree(1024).plain_modulus(257).ct_moduli({1099509805057ull})
                       .aux_moduli({562949953443841ull}).sigma(3.2).build();
    auto skc = gen_secret_key_with_rng(compact, rng);
    for (uint64_t v : {0ull, 1ull, 42ull, 100ull, 256ull})
        if (decode_scalar(decrypt(trivial_encrypt(v, compact), skc)) != v) return 34;
    auto c10 = encrypt_sk_with_rng(encode_scalar(10, compact), skc, compact, rng);
    if (decode_scalar(decrypt(bfv_plain_add(c10, encode_scalar(5, compact)), skc)) != 15) return 35;
    if (decode_scalar(decrypt(bfv_plain_mul(c10, encode_scalar(7, compact)), skc)) != 70) return 36;
    // bfv_host.rs:430-476: trivial ciphertexts of m = 0..4 refreshed into the boot scheme
    auto orig = BfvParamsBuilder().ring_degree(16).plain_modulus(5).ct_moduli({65537ull}).sigma(3.2).build();
    auto boot = BfvParamsBuilder().ring_degree(16).plain_modulus(29).ct_moduli({1125899906842817ull}).sigma(3.2)
                    .gadget_base(8).build();
    auto sko = gen_secret_key_with_rng(orig, rng);
    auto bsk = gen_bootstrap_key(sko, boot, 25, 5, rng);
    for (uint64_t v = 0; v < 5; ++v) {
        const auto tin = trivial_encrypt(v, orig);
        uint64_t hin = 1469598103934665603ull;
        for (auto& p : tin.c)
            for (uint64_t w : p.data) hin = (hin ^ w) * 1099511628211ull;
        std::printf("boot v=%llu in=%016llx\n", (unsigned long long)v, (unsigned long long)hin);
        const auto out = bfv_bootstrap(tin, bsk);
        const uint64_t dec = decode_scalar(decrypt(out, bsk.boot_sk));
        uint64_t h = 1469598103934665603ull;   // FNV-1a of the output words: identical run to run
        for (auto& p : out.c)
            for (uint64_t w : p.data) h = (h ^ w) * 1099511628211ull;
        std::printf("boot v=%llu dec=%llu out=%016llx\n", (unsigned long long)v, (unsigned long long)dec,
                    (unsigned long long)h);
        if (dec % 5 != v) return 37;
    }
    if (lagrange_interpolate({0, 1, 4, 2}, 7) != std::vector<uint64_t>{0, 0, 1, 0}) return 38;
    return 0;
}

// diagnostic: the bootstrap of trivial ciphertexts repeated in one process; counts wrong decodes and
// outputs that differ from the first repetition (the computation is deterministic)
static int boot_repro(int reps) {
    auto orig = BfvParamsBuilder().ring_degree(16).plain_modulus(5).ct_moduli({65537ull}).sigma(3.2).build();
    auto boot = BfvParamsBuilder().ring_degree(16).plain_modulus(29).ct_moduli({1125899906842817ull}).sigma(3.2)
                    .gadget_base(8).build();
    ChaChaRng rng(42);
    auto sko = gen_secret_key_with_rng(orig, rng);
    auto bsk = gen_bootstrap_key(sko, boot, 25, 5, rng);
    std::vector<std::vector<uint64_t>> first(5);
    int wrong = 0, differ = 0;
    for (int r = 0; r < reps; ++r)
        for (uint64_t v = 0; v < 5; ++v) {
            auto out = bfv_bootstrap(trivial_encrypt(v, orig), bsk);
            std::vector<uint64_t> flat;
            for (auto& p : out.c) flat.insert(flat.end(), p.data.begin(), p.data.end());
            if (r == 0) first[v] = flat;
            else if (flat != first[v]) ++differ;
            if (decode_scalar(decrypt(out, bsk.boot_sk)) % 5 != v) ++wrong;
        }
    std::printf("boot_repro reps=%d wrong=%d differ=%d\n", reps, wrong, differ);
    return wrong || differ;
}

int main(int argc, char** argv) {
    if (argc == 3 && std::string(argv[1]) == "--boot-reps") return boot_repro(std::atoi(argv[2]));
    if (argc >= 3 && std::string(argv[1]) == "--seq") {   // diagnostic: named cases in the given order
        int bad = 0;
        for (int i = 2; i < argc; ++i) {
            const std::string c = argv[i];
            const int rc = c == "error" ? error_cases() : c == "keygen" ? keygen_case() : c == "boot" ? bootstrap_case() : 98;
            std::printf("%s %s (%d)\n", rc ? "FAIL" : "PASS", argv[i], rc);
            bad |= rc != 0;
        }
        return bad;
    }
    if (argc == 3 && std::string(argv[1]) == "--boot-case-reps") {   // the whole bootstrap case, repeated
        int fails = 0, first = 0;
        for (int r = 0; r < std::atoi(argv[2]); ++r) {
            const int rc = bootstrap_case();
            if (rc) {
                ++fails;
                if (!first) first = rc;
            }
        }
        std::printf("boot_case reps=%s fails=%d first_code=%d\n", argv[2], fails, first);
        return fails != 0;
    }
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <fixture-dir> <case>...\n", argv[0]);
        return 2;
    }
    int bad = 0;
    for (int i = 2; i < argc; ++i) {
        int rc;
        try {
            rc = run_case(argv[1], argv[i]);
        } catch (const std::exception& e) {
            std::printf("ERROR %s: %s\n", argv[i], e.what());
            rc = 99;
        }
        std::printf("%s %s (%d)\n", rc ? "FAIL" : "PASS", argv[i], rc);
        bad |= rc != 0;
    }
    const int e = error_cases();
    std::printf("%s error_cases (%d)\n", e ? "FAIL" : "PASS", e);
    bad |= e != 0;
    int k;
    try {
        k = keygen_case();
    } catch (const std::exception& ex) {
        std::printf("ERROR keygen: %s\n", ex.what());
        k = 99;
    }
    std::printf("%s keygen (%d)\n", k ? "FAIL" : "PASS", k);
    bad |= k != 0;
    try {
        k = bootstrap_case();
    } catch (const std::exception& ex) {
        std::printf("ERROR bootstrap: %s\n", ex.what());
        k = 99;
    }
    std::printf("%s bootstrap (%d)\n", k ? "FAIL" : "PASS", k);
    bad |= k != 0;
    if (!bad) std::printf("ALL OK\n");
    return bad;
}
