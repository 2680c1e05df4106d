// Host runtime and C ABI of libexacto_hip.so (see include/exacto_hip.h).
//
// Owns, per context: the prime set (ciphertext primes, then the auxiliary primes of
// the selected multiplication path), per-prime NTT twiddle tables and constants in
// HBM, the exact-CRT tables, the resident relinearisation key and a chunked
// workspace.  Every `_dev` entry point only enqueues kernels on the context stream.
#include <algorithm>
#include <cxxabi.h>
#include <dlfcn.h>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/exacto_hip.h"
#include "exacto_internal.hpp"

using namespace exacto;

thread_local const void* exacto::g_last_kernel = nullptr;

// ============================================================== errors

static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
static int invalid_param(const std::string& s) { return fail(EXACTO_ERR_INVALID_PARAM, "invalid parameter: " + s); }

#define HIP_TRY(x)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess)                                                                   \
            return fail(EXACTO_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(e_) +    \
                                            " (" #x ")");                                       \
    } while (0)

#define CHECK_LAUNCH()                                                                          \
    do {                                                                                        \
        hipError_t e_ = hipGetLastError();                                                      \
        if (e_ != hipSuccess)                                                                   \
            return fail(EXACTO_ERR_HIP, std::string("HIP launch error: ") + hipGetErrorString(e_)); \
    } while (0)

// ============================================================== host integer helpers

static u64 mulmod_h(u64 a, u64 b, u64 m) { return (u64)((u128)a * b % m); }

static u64 powmod_h(u64 b, u64 e, u64 m) {
    u64 r = 1 % m;
    b %= m;
    while (e) {
        if (e & 1) r = mulmod_h(r, b, m);
        b = mulmod_h(b, b, m);
        e >>= 1;
    }
    return r;
}

static bool is_prime_h(u64 n) {
    if (n < 2) return false;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : small)
        if (n % p == 0) return n == p;
    u64 d = n - 1;
    int s = 0;
    while ((d & 1) == 0) { d >>= 1; ++s; }
    for (u64 a : small) {
        u64 x = powmod_h(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s; ++r) {
            x = mulmod_h(x, x, n);
            if (x == n - 1) { comp = false; break; }
        }
        if (comp) return false;
    }
    return true;
}

// modular inverse via extended Euclid (returns 0 if not invertible)
static u64 invmod_h(u64 a, u64 m) {
    i128 t = 0, nt = 1, r = m, nr = a % m;
    while (nr != 0) {
        i128 q = r / nr;
        i128 tmp = t - q * nt; t = nt; nt = tmp;
        tmp = r - q * nr; r = nr; nr = tmp;
    }
    if (r != 1) return 0;
    if (t < 0) t += m;
    return (u64)t;
}

static u64 shoup_h(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
static int bitlen(u64 x) { return x ? 64 - __builtin_clzll(x) : 0; }

static int bitrev(int x, int bits) {
    int r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

// psi: smallest x >= 2 with (x^((q-1)/2n))^n == -1 (oracle/ring.py find_psi)
static u64 find_psi(u64 n, u64 q) {
    const u64 e = (q - 1) / (2 * n);
    for (u64 x = 2;; ++x) {
        const u64 psi = powmod_h(x, e, q);
        if (powmod_h(psi, n, q) == q - 1) return psi;
    }
}

// --- minimal unsigned big integer (little-endian 64-bit words) ---
struct Big {
    std::vector<u64> w;
    Big(u64 v = 0) { w.push_back(v); trim(); }
    void trim() { while (w.size() > 1 && w.back() == 0) w.pop_back(); }
    void mul(u64 m) {
        u64 c = 0;
        for (auto& x : w) { u128 t = (u128)x * m + c; x = (u64)t; c = (u64)(t >> 64); }
        if (c) w.push_back(c);
        trim();
    }
    void add(u64 a) {
        for (size_t i = 0; i < w.size() && a; ++i) { u64 s = w[i] + a; a = s < a; w[i] = s; }
        if (a) w.push_back(a);
    }
    void add(const Big& o) {
        u64 carry = 0;
        for (size_t i = 0; i < std::max(w.size(), o.w.size()) || carry; ++i) {
            if (i == w.size()) w.push_back(0);
            const u128 t = (u128)w[i] + (i < o.w.size() ? o.w[i] : 0) + carry;
            w[i] = (u64)t;
            carry = (u64)(t >> 64);
        }
        trim();
    }
    void shr1() {
        for (size_t i = 0; i < w.size(); ++i) w[i] = (w[i] >> 1) | (i + 1 < w.size() ? w[i + 1] << 63 : 0);
        trim();
    }
    u64 mod(u64 m) const {
        u128 r = 0;
        for (size_t i = w.size(); i-- > 0;) r = ((r << 64) | w[i]) % m;
        return (u64)r;
    }
    int cmp(const Big& o) const {
        if (w.size() != o.w.size()) return w.size() < o.w.size() ? -1 : 1;
        for (size_t i = w.size(); i-- > 0;)
            if (w[i] != o.w[i]) return w[i] < o.w[i] ? -1 : 1;
        return 0;
    }
};

// mixed-radix digits of X (given as residues mod primes[0..cnt)) — host Garner
static std::vector<u64> mixed_radix(const std::vector<u64>& res, const std::vector<u64>& pr) {
    std::vector<u64> v(pr.size());
    for (size_t i = 0; i < pr.size(); ++i) {
        u64 t = res[i];
        for (size_t k = 0; k < i; ++k) {
            const u64 vk = v[k] % pr[i];
            t = (t + pr[i] - vk) % pr[i];
            t = mulmod_h(t, invmod_h(pr[k] % pr[i], pr[i]), pr[i]);
        }
        v[i] = t;
    }
    return v;
}

// ============================================================== context

struct ProfRec {
    int kind;
    hipEvent_t a, b;
    u64 polys;
    double bytes;
    const void* kern;   // host handle of the last kernel launched inside the scope (EXACTO_LAUNCH)
};

// A 31-bit auxiliary basis of the ks32 key switch (ks32.hip) with its device tables and the
// relinearisation key converted to it.
struct Ks32Basis {
    int S = 0;
    int sum_max = 0;              // dBFV key-switch sums the basis lifts exactly
    int fpc_max = 0;              // ... and by the float-CRT lift (ks32_fpc_one's margin; S <= 3 or p < 2^32 / 3)
    int mac_form = 0;             // ks32_mac: 0 primes up to 2^31 (7 products per reduction),
                                  // 1 below 2^32 / 3 (12), 2 below 2^30 (12, lazy transforms)
    Big P;                        // product of the primes
    Prime32* d_p32 = nullptr;
    uint2* d_tw32 = nullptr;
    Ks32Tables* d_kst = nullptr;
    uint32_t* d_rs = nullptr;     // the relinearisation key in this basis
    size_t rs_cap = 0;
    bool rs_valid = false;
};

// Stream and per-chunk workspace of one extra pipeline lane (lane 0 is the context's own).
constexpr int EXACTO_MAX_LANES = 4;
struct LaneSet {
    hipStream_t stream = nullptr;
    hipEvent_t join = nullptr;
    size_t items = 0;
    u64 *coefQ = nullptr, *extP = nullptr, *T = nullptr, *D = nullptr;
    int16_t* D16 = nullptr;
    uint32_t *DS = nullptr, *U = nullptr;
};

struct exacto_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int n = 0, logn = 0, L = 0, K = 0;
    std::vector<u64> ctq, user_aux, int_aux, primes;  // primes = ctq ++ (path aux)
    u64 plain = 0, gbase = 0;
    int G = 0;
    int path = EXACTO_PATH_EXACT_RNS;
    int deferred_code = 0;  // error raised at multiplication time (reference semantics)
    std::string deferred_msg;
    PrimeConst* d_primes = nullptr;
    TwPair* d_tw = nullptr;
    CrtTables* d_crt = nullptr;
    CrtTables h_crt{};
    u64* d_scal = nullptr;
    u64* d_rlk = nullptr;
    u64* d_rlk_s = nullptr;  // Shoup companions of the key (limb-wise relinearisation MAC)
    size_t rlk_keys = 0, rlk_cap = 0, rlk_s_cap = 0;
    bool rlk_s_valid = false;
    // EXACTO_NTT_ASM=0: no special-prime (2^60 - d) asm rounds; those batches then take the generated
    // generic-prime asm rounds where their size has them (n = 1024 / 4096 / 8192, lazy primes), and the
    // compiler-scheduled C++ rounds only with EXACTO_NTT_GEN=0 as well (A/B switches)
    bool ntt_asm = true;
    bool ntt_asm_inv = true;  // EXACTO_NTT_ASM_INV=0: compiler-scheduled inverse NTT (A/B)
    // relinearisation MAC in an auxiliary basis of S 31-bit primes (ks32.hip; EXACTO_KS32=0: the
    // limb-wise 60-bit digit NTTs + relin_mac)
    bool ks32 = true;
    int S32 = 0;                 // 0: not eligible for these parameters
    int ks32_sum_max = 0;        // key-switch sums that may be added before one lift (prod p bound)
    int ks32_fpc_max = 0;        // ... that the active basis' float-CRT lift takes (Ks32Basis::fpc_max)
    bool ks_fpc = true;          // EXACTO_KS_FPC=0: the Garner lift in ks32_crt always (A/B)
    int ks32_mac_form = 0;       // ks32_mac's reduction form for the active basis (Ks32Basis::mac_form)
    Ks32Basis kw;                // wide basis (primes up to 2^31) for dBFV digit sums the primary cannot hold
    // The primary basis is one of two, chosen per relinearisation key (ensure_rs):
    //   kn: narrow primes below 2^32 / 3 bounding |sum_g d_g * r_g| by G n (B/2) (q/2) for ANY key;
    //   kz: lazy primes below 2^30 (cheaper 32-bit butterflies, ks32_dev.hpp), used when the resident
    //       key's own L1 norms bound the sum: |u_{c,l}| <= (B/2) sum_g ||r_{g,c,l}||_1 < prod p / 2
    //       (a uniform key has ||r||_1 ~ n q / 4: half the generic bound).  EXACTO_KS32_LAZY=0: kn only.
    // S32 / d_p32 / d_tw32 / d_kst / ks32_sum_max / ks32_mac_form describe the active one.
    Ks32Basis kn, kz;
    bool ks32_lazy_active = false;
    int ks32_need_m = 1;          // the most key-switch sums per output limb a dbfv_mul of this context asked for
    int last_dbfv_ks = -1;        // exacto_ctx_info.dbfv_key_switch
    // a dBFV pass with shared extensions: d and its products per item (0: plain BFV products), for
    // run_inv_tensor's algorithmic bytes and the tensor kernels' prime-major block order
    int tensor_share_d = 0, tensor_share_npairs = 0;
    // dBFV chain: the step that formed the output limbs in the coefficient domain also lifted them to
    // the auxiliary primes into ext_a and transformed both in one launch; the next step's extension of
    // its left operand is then already in ext_a (measured A/B: DESIGN.md §6.4)
    bool ext_a_ready = false;
    int16_t* ks_defer = nullptr;  // run_mul: int16 digits of product p to ks_defer + p G n, no key switch
    bool ks_defer8 = false;       // ... int8 digits instead (base <= 2^8; EXACTO_DIGIT8=0: int16)
    bool digit8_env = true;
    // dBFV psum (EXACTO_PSUM=0: off): an output limb's c0 / c1 scaled once from the sum of its
    // products' tensors in the auxiliary primes (run_mul, dbfv_mul_core); psum_max = the largest
    // product count m with m (p n Q + 2) < P, so that the summed rounding stays liftable from P
    bool psum_env = true;
    int psum_max = 0;
    int psum_fp_max = 0;         // ... and with |sum| < P / 4, the rounded-float CRT over P (kernels.hip fpc_lift)
    bool fp_crt = true;          // EXACTO_FP_CRT=0: Garner over P in the SP scale kernels (A/B)
    // the scale kernels' s = [p T]_Q by a rounded float sum (with fp_crt; kernels.hip fpq_y) wherever
    // |f - round(f)| <= fpq_lim.  EXACTO_FPQ=0: Garner over Q always; =2: a 1/4 band (half the
    // coefficients take Garner: the fallback's bit-exact variant)
    double fpq_lim = 0.5 - 0x1p-40;
    // HPS: the division-free scale (q > 2^32, p < min(q, 2^32); EXACTO_HPS_LITERAL=1: the literal i128
    // form, kept for the equivalence test) and, in dbfv_mul, the products' c0 / c1 and signed gadget
    // digits summed per output limb before ONE forward NTT + relinearisation MAC per limb
    // (EXACTO_HPS_SUM=0: per product)
    bool hps_fast = false;
    bool hps_sum_env = true;
    struct PsumPlan {
        bool on = false;
        int d = 0, npairs = 0;
        const int* term_start = nullptr;
        const CombineTerm* terms = nullptr;
        u64* out = nullptr;       // [B][d][2][L][n], coefficient domain
        bool fpc = false;         // its scale may take the rounded-float CRT over P (m <= psum_fp_max)
    } psum;
    u64* d_hdig = nullptr;       // dBFV over HPS: the summed digits' NTT residues [B][d][G][L][n]
    size_t hdig_cap = 0;
    int16_t* d_dall = nullptr;   // dBFV: per-product digits
    void* d_dk = nullptr;        // ... and their per-limb sums (int16, or int32 when m B/2 > 2^15 - 1)
    uint32_t *d_dsk = nullptr, *d_uk = nullptr;   // their residues and key-switch sums in the 31-bit basis
    size_t dall_cap = 0, dk_cap = 0, dsk_cap = 0, uk_cap = 0;
    Prime32* d_p32 = nullptr;
    uint2* d_tw32 = nullptr;
    Ks32Tables* d_kst = nullptr;
    uint32_t* d_rs = nullptr;    // key in the auxiliary basis [keys][2L][S][n], NTT domain mod p_s
    size_t rs_cap = 0;
    bool rs_valid = false;
    uint32_t *ws_DS = nullptr, *ws_U = nullptr;
    bool rlk_loaded = false;
    // workspace (per chunk)
    size_t chunk = 512;  // products per pipeline pass; throughput plateaus from ~512 (r1 sweep)
    size_t ws_items = 0;
    u64 *ws_coefQ = nullptr, *ws_extP = nullptr, *ws_T = nullptr, *ws_D = nullptr;
    // exact path with gadget base <= 2^16: the scale kernel writes each digit once as int16 and
    // the digit NTT converts it per limb on load (EXACTO_DIGIT16=0: u64 digits per limb)
    bool digit16 = true;
    int16_t* ws_D16 = nullptr;
    // further pipeline lanes: chunk i runs on lane i % lanes, each lane a stream with its own
    // workspace, so the kernels of consecutive chunks overlap (EXACTO_DUAL_STREAM=0: one lane;
    // EXACTO_LANES: lane count, 2 by default)
    bool dual = true;
    int lanes = 2;
    hipEvent_t ev_fork = nullptr;
    // dBFV chains of two or more items run as two halves on two streams (exacto_dbfv_mul_chain_dev):
    // the second half on a twin context (same parameters, its own stream and workspaces, a copy of
    // the relinearisation key), so each half's whole chain overlaps the other's
    static constexpr int MAX_TWINS = 3;
    exacto_ctx* twin[MAX_TWINS] = {};
    bool batch_split = true;         // EXACTO_CHAIN_SPLIT=0: one stream for the whole batch
    unsigned rlk_version = 0, twin_rlk_version[MAX_TWINS] = {~0u, ~0u, ~0u};
    hipEvent_t ev_twin_in = nullptr, ev_twin_out[MAX_TWINS] = {};
    LaneSet xl[EXACTO_MAX_LANES - 1];   // lanes 1 .. lanes-1
    // dBFV: per-ciphertext extensions shared by the products that use the ciphertext
    // (EXACTO_SHARE_EXT=0 recomputes them per product)
    bool share_ext = true;
    // keygen / encryption
    double* d_cdt = nullptr;
    size_t cdt_cap = 0;
    double cdt_sigma = 0.0;
    u64* d_gpow = nullptr;
    size_t gpow_cap = 0;
    u64* d_delta = nullptr;
    bool delta_ok = false;
    u64* enc_buf = nullptr;
    size_t enc_cap = 0;
    u64* gk_s = nullptr;  // Shoup companions of the Galois key of the last automorphism call
    size_t gk_s_cap = 0;
    uint32_t* d_gk_rs = nullptr;  // ks32: Galois key of the last automorphism call in the 31-bit basis
    size_t gk_rs_cap = 0;
    u64* pl_buf = nullptr;  // lifted plaintexts / monomial scratch
    size_t pl_cap = 0;
    u64 *ext_a = nullptr, *ext_b = nullptr;
    size_t ext_a_cap = 0, ext_b_cap = 0;
    u64* chain_buf = nullptr;  // dBFV chain ping-pong buffers
    size_t chain_bytes = 0;
    // dBFV chain, psum path: each step's relinearised limbs also in the coefficient domain (they are
    // there before the final forward NTT), so the next step's extension lifts them directly instead
    // of inverse-transforming its NTT-domain input (dbfv_mul_group, exacto_dbfv_mul_chain_dev)
    u64* chain_coef = nullptr;
    size_t chain_coef_bytes = 0;
    u64* coef_out = nullptr;        // where this step's coefficient form went (psum steps of a chain)
    int coef_slot = -1;             // set by the chain: chain_coef half for this step's coefficient form
    size_t coef_slot_words = 0;     // ... and the size of one half
    const u64* coef_in = nullptr;   // set by the chain: the coefficient form of this step's `a`
    bool coef_written = false;      // reported back: coef_out holds this step's results
    u64* dec_buf = nullptr;    // decryption phase [B][L][n]
    size_t dec_bytes = 0;
    u64* dig_buf = nullptr;    // dBFV decrypted digits [B][d][n]
    size_t dig_bytes = 0;
    // staging for host-pointer API and dBFV products
    u64* io = nullptr;
    size_t io_bytes = 0;
    u64* prod = nullptr;
    size_t prod_bytes = 0;
    // dBFV plan cache
    u64* d_off = nullptr;
    size_t off_cap = 0;
    size_t cached_B = 0, cached_d = 0;
    u64 cached_base = 0, cached_p = 0;
    int cached_npairs = 0;
    std::vector<int> cached_limbs;   // output limbs of the cached plan (all d, or a subset: exacto_dbfv_mul_limbs)
    int cached_sum_m = 0;        // max products per dBFV output limb when all combine terms are sums, else -1
    int* d_term_start = nullptr;
    CombineTerm* d_terms = nullptr;
    size_t terms_cap = 0;
    // per-call scratch: the context's own stream-ordered pool (Scratch)
    hipMemPool_t pool = nullptr;
    // the bootstrap's intermediates (coefficients, flags, the c0'/c1' rows, phase, slots): a persistent
    // buffer of the boot context, grown like the workspaces, never from the stream-ordered pool
    u64* boot_buf = nullptr;
    size_t boot_cap = 0;
    u64* boot_slots = nullptr;   // ... and the slots of the ring path, grown when an item takes it
    size_t boot_slots_cap = 0;
    bool debug_scratch = false;
    size_t dbfv_group_bytes = (size_t)16384 << 20;  // dbfv_mul item groups (EXACTO_DBFV_GROUP_MB)
    // profiling
    bool prof = false;
    std::vector<ProfRec> recs;
    std::map<int, std::map<const void*, std::pair<u64, double>>> prof_kern;   // kind -> kernel -> (launches, ms)
};

// EXACTO_DEBUG_ALLOC=1: every device allocation and release of the library is logged
// to stderr with its pointer, size, pool and stream; =2 adds the allocation range the runtime reports
// for it (hipMemGetAddressRange), so that the failing bootstrap call's blocks can be checked for
// overlap with any other live block.  (Round 5: with the range lookups the failure no longer showed.)
static int dbg_alloc_on() {
    static const int on = [] { const char* e = getenv("EXACTO_DEBUG_ALLOC"); return e ? atoi(e) : 0; }();
    return on;
}
static void dbg_alloc_log(const char* what, const void* p, size_t bytes, const void* pool, const void* stream,
                          bool range) {
    if (!dbg_alloc_on()) return;
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    if (range && p && dbg_alloc_on() > 1) {
        if (hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)p) != hipSuccess) base = nullptr;
        (void)hipGetLastError();   // a failed lookup must not reach the next CHECK_LAUNCH
    }
    std::fprintf(stderr, "alloc-dbg %s p=%p bytes=%zu pool=%p stream=%p range=%p+%zu\n", what, p, bytes, pool, stream,
                 (void*)base, sz);
}

static void free_dev(void* p) {
    if (p) {
        dbg_alloc_log("hipFree", p, 0, nullptr, nullptr, false);
        (void)hipFree(p);
    }
}

// Per-call scratch from the context's own stream-ordered pool (hipMallocFromPoolAsync / hipFreeAsync
// on the stream that uses it; no device-wide synchronisation).  The pool belongs to the context
// (hipMemPoolCreate), so its release threshold -- freed blocks stay mapped for the next call -- does
// not change the device's default pool that other libraries in the process use.
// EXACTO_DEBUG_SCRATCH=1 (read when a context is created) fills every block with 0xFF when it is
// handed out, so a kernel that reads scratch it never wrote gives wrong results at once instead of
// whatever the previous owner of the block left there.
struct Scratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    Scratch() = default;
    Scratch(const Scratch&) = delete;
    Scratch& operator=(const Scratch&) = delete;
    hipMemPool_t from = nullptr;
    ~Scratch() {
        if (p) {
            dbg_alloc_log("hipFreeAsync", p, 0, from, s, false);
            (void)hipFreeAsync(p, s);
        }
    }
    hipError_t alloc(size_t bytes, hipStream_t st, hipMemPool_t pool, bool debug) {
        s = st;
        from = pool;
        hipError_t e = pool ? hipMallocFromPoolAsync(&p, std::max<size_t>(bytes, 8), pool, st)
                            : hipMallocAsync(&p, std::max<size_t>(bytes, 8), st);
        if (e == hipSuccess) dbg_alloc_log(pool ? "hipMallocFromPoolAsync" : "hipMallocAsync", p, bytes, pool, st, true);
        if (e == hipSuccess && debug) e = hipMemsetAsync(p, 0xFF, std::max<size_t>(bytes, 8), st);
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Every device allocation of the library.  EXACTO_DEBUG_FILL=1 (read once): new blocks are filled
// with 0xA5 bytes, so that a kernel reading memory nothing wrote sees garbage at once instead of the
// zeros of fresh pages (a read of that kind passed in a fresh process and failed after other work
// had freed and re-used the memory).
static hipError_t dev_alloc(void** p, size_t bytes) {
    static const bool fill = [] { const char* e = getenv("EXACTO_DEBUG_FILL"); return e && e[0] == '1'; }();
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) dbg_alloc_log("hipMalloc", *p, bytes, nullptr, nullptr, true);
    if (e == hipSuccess && fill && bytes) {
        e = hipMemset(*p, 0xA5, bytes);
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    return e;
}

// Device -> device copies of the library, as a kernel (every size here is whole u64 words); device
// fills likewise (launch_fill_u32).  Round 3 replaced hipMemcpyAsync / hipMemsetAsync with these
// while chasing an intermittent stale bootstrap result; round 4 measured that the runtime's own
// device-to-device copy is a blit kernel on the same queue (__amd_rocclr_copyBuffer) and never read
// stale in 180k replays of the bootstrap's sequence (tools/d2d_repro.cpp), so the change is not a
// fix of a runtime fault.  It stays: every device-side operation of the library is a
// kernel of its own, one code path, visible by name in kernel traces.
static hipError_t dev_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    launch_copy_u64(static_cast<u64*>(dst), static_cast<const u64*>(src), (long)(bytes / 8), s);
    return hipGetLastError();
}

static int grow(u64** buf, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return 0;
    free_dev(*buf);
    *buf = nullptr;
    *cap = 0;
    HIP_TRY(dev_alloc((void**)buf, bytes));
    *cap = bytes;
    return 0;
}

// Host -> device copy ordered on the context stream.  The stream is non-blocking, so it does not
// wait for the legacy null stream that a plain hipMemcpy runs on: a kernel enqueued on it right
// after such a copy may read the destination before the copy has landed.  Returns once the copy
// is complete, so `src` may be reused at once.
static int upload(exacto_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!bytes) return 0;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

static int plan_check(size_t n, u64 q) {
    // make_plan (ntt.rs:19-29) via concrete-ntt Plan::try_new: prime q == 1 mod 2n, n >= 16.
    // This library additionally needs q < 2^62 (lazy butterflies keep 4q < 2^64).
    if (n < 16 || q < 2 || q >= (1ull << 62) || (q - 1) % (2 * n) != 0 || !is_prime_h(q))
        return invalid_param("cannot create NTT plan for n=" + std::to_string(n) + ", q=" + std::to_string(q) +
                             " (need prime q ≡ 1 mod " + std::to_string(2 * n));
    return 0;
}

static PrimeConst make_prime_const(u64 q, int n, int logn, TwPair* h_fwd, TwPair* h_inv) {
    PrimeConst P{};
    P.q = q;
    P.two_q = 2 * q;
    P.mu64 = (u64)((((u128)1) << 64) / q);
    P.bar_s = bitlen(q);
    P.bar_mu = (u64)((((u128)1) << (2 * P.bar_s)) / q);
    const u64 psi = find_psi(n, q);
    const u64 psi_inv = invmod_h(psi, q);
    for (int i = 0; i < n; ++i) {
        const int e = bitrev(i, logn);
        const u64 w = powmod_h(psi, e, q), wi = powmod_h(psi_inv, e, q);
        h_fwd[i] = {w, shoup_h(w, q)};
        h_inv[i] = {wi, shoup_h(wi, q)};
    }
    P.n_inv = invmod_h((u64)n % q, q);
    P.n_inv_s = shoup_h(P.n_inv, q);
    P.last_w = mulmod_h(h_inv[1].w, P.n_inv, q);
    P.last_ws = shoup_h(P.last_w, q);
    u64 qi = q;                                   // q^-1 mod 2^64 by Newton (q odd): 6 doublings
    for (int it = 0; it < 6; ++it) qi *= 2 - q * qi;
    P.qinv_neg = (u64)0 - qi;
    const u64 r = (u64)((((u128)1) << 64) % q);   // R = 2^64 mod q
    P.n_inv_r = mulmod_h(P.n_inv, r, q);
    P.n_inv_rs = shoup_h(P.n_inv_r, q);
    P.last_wr = mulmod_h(P.last_w, r, q);
    P.last_wrs = shoup_h(P.last_wr, q);
    return P;
}

static void set_shoup(u64& w, u64& ws, u64 v, u64 q) {
    w = v;
    ws = shoup_h(v, q);
}

// The largest m <= 64 with prod p > 2 m `one` + 1: the centred lift of a sum of m terms, each at most
// `one` in magnitude, is exact.  fpc: with the float-CRT lift's margin, prod p 2^20 > (2 m one + 1)
// (2^20 + 1), so |u| / P < 1/2 - 2^-21 against the float sum's error below 2^-48 (ks32_fpc_one).
static int sums_lifted(const Big& P, const Big& one, bool fpc) {
    Big pf = P;
    if (fpc) pf.mul(1ull << 20);
    int r = 0;
    for (u64 m = 1; m <= 64; ++m) {
        Big bm = one;
        bm.mul(2 * m);
        bm.add(1);
        if (fpc) bm.mul((1ull << 20) + 1);
        if (pf.cmp(bm) <= 0) break;
        r = (int)m;
    }
    return r;
}

// ks32.hip's auxiliary basis: the fewest primes p == 1 mod 2n in (2^30, 2^31), largest first, with
// prod p > 2 G n floor(B/2) floor(q_max/2) (the magnitude bound of sum_g d_g * r_g, digits balanced
// in [-B/2, B/2), key coefficients balanced).  Eligible: exact path, gadget base <= 2^16 (int16
// digits), every ciphertext prime 2^60 - d with d < 2^24 (ks32_crt reduces with reduce_near60),
// 1024 <= n <= 16384; S <= 4.
// One 31-bit basis for ks32: the fewest primes p == 1 mod 2n below pmax (largest first, all above
// 2^30) with prod p > `bound`, its twiddles, constants and Garner tables on the device.  sum_max:
// how many key-switch sums (dBFV products of one output limb) the basis lifts exactly when they
// are added first.  S = 0 when no basis of at most EXACTO_KS32_MAXS primes exists.
// fixedS > 0 (the lazy basis): exactly fixedS primes in (7 pmax / 8, pmax), no bound check here (the
// bound is the resident key's, checked when the key is converted: ensure_rs; ks32.hip's red_s64_lz
// needs p > 0.8 * 2^30).
static int build_ks32_basis_impl(exacto_ctx* c, u64 pmax, u64 qmax, const Big& bound, Ks32Basis* b,
                                 int fixedS = 0) {
    b->S = 0;
    std::vector<u64> ps;
    Big P(1);
    const u64 step = 2 * (u64)c->n;
    const u64 pmin = fixedS ? pmax - pmax / 8 : (1ull << 30);
    for (u64 p = (pmax - 1) / step * step + 1; p > pmin && ps.size() < EXACTO_KS32_MAXS; p -= step) {
        if (!is_prime_h(p)) continue;
        ps.push_back(p);
        P.mul(p);
        if (fixedS ? (int)ps.size() == fixedS : P.cmp(bound) > 0) break;
    }
    if (fixedS ? (int)ps.size() != fixedS : (P.cmp(bound) <= 0 || ps.size() < 2)) return 0;
    bool lazy = true, narrow = true;
    for (u64 p : ps) {
        lazy &= p < (1ull << 30);
        narrow &= p < (1ull << 32) / 3;
    }
    b->mac_form = lazy ? 2 : narrow ? 1 : 0;
    b->P = P;
    b->sum_max = b->fpc_max = 0;
    if (!fixedS) {   // the lazy basis' limits come from the resident key (ks32_select_basis)
        Big one((u64)c->G);
        one.mul((u64)c->n);
        one.mul(c->gbase / 2);
        one.mul(qmax / 2);
        b->sum_max = std::max(1, sums_lifted(P, one, false));   // P > bound was checked above
        b->fpc_max = ps.size() <= 3 || narrow ? sums_lifted(P, one, true) : 0;   // ks32_crt's condition
    }
    const int S = (int)ps.size(), n = c->n;
    std::vector<uint2> tw((size_t)S * 2 * n);
    std::vector<Prime32> pc(S);
    auto sh32 = [](u64 w, u64 p) { return (uint32_t)((w << 32) / p); };
    for (int s = 0; s < S; ++s) {
        const u64 p = ps[s];
        const u64 psi = find_psi(n, p), psi_inv = invmod_h(psi, p);
        for (int i = 0; i < n; ++i) {
            const int e = bitrev(i, c->logn);
            const u64 w = powmod_h(psi, e, p), wi = powmod_h(psi_inv, e, p);
            tw[(size_t)s * 2 * n + i] = make_uint2((uint32_t)w, sh32(w, p));
            tw[(size_t)s * 2 * n + n + i] = make_uint2((uint32_t)wi, sh32(wi, p));
        }
        Prime32& Q = pc[s];
        Q.p = (uint32_t)p;
        const u64 ninv = invmod_h((u64)n % p, p);
        Q.n_inv = (uint32_t)ninv;
        Q.n_inv_s = sh32(ninv, p);
        const u64 lw = mulmod_h(tw[(size_t)s * 2 * n + n + 1].x, ninv, p);
        Q.last_w = (uint32_t)lw;
        Q.last_ws = sh32(lw, p);
        const u64 c32 = (1ull << 32) % p;
        Q.c32 = (uint32_t)c32;
        Q.c32s = sh32(c32, p);
        const u64 m63 = (1ull << 63) % p;
        Q.k63 = (uint32_t)(m63 == 0 ? 0 : p - m63);
        // the float-CRT lift's factor pi = (P / p)^-1 mod p folded into the last inverse stage
        u64 pi = 1;
        for (int k = 0; k < (int)ps.size(); ++k)
            if (k != s) pi = mulmod_h(pi, ps[k] % p, p);
        pi = invmod_h(pi, p);
        const u64 fni = mulmod_h(ninv, pi, p), flw = mulmod_h(lw, pi, p);
        Q.fn_inv = (uint32_t)fni;
        Q.fn_inv_s = sh32(fni, p);
        Q.flast_w = (uint32_t)flw;
        Q.flast_ws = sh32(flw, p);
        Q.inv_p = 1.0 / (double)p;
    }
    HIP_TRY(dev_alloc((void**)&b->d_tw32, tw.size() * sizeof(uint2)));
    if (int e_ = upload(c, b->d_tw32, tw.data(), tw.size() * sizeof(uint2))) return e_;
    for (int s = 0; s < S; ++s) {
        pc[s].tw_fwd = b->d_tw32 + (size_t)s * 2 * n;
        pc[s].tw_inv = b->d_tw32 + (size_t)s * 2 * n + n;
    }
    HIP_TRY(dev_alloc((void**)&b->d_p32, S * sizeof(Prime32)));
    if (int e_ = upload(c, b->d_p32, pc.data(), S * sizeof(Prime32))) return e_;
    Ks32Tables T;
    std::memset(&T, 0, sizeof(T));
    for (int s = 0; s < S; ++s)
        for (int k = 0; k < s; ++k) {
            const u64 v = invmod_h(ps[k] % ps[s], ps[s]);
            T.ginv[s][k] = (uint32_t)v;
            T.ginv_s[s][k] = sh32(v, ps[s]);
        }
    Big H = P;
    H.shr1();
    {
        std::vector<u64> hr(S);
        for (int s = 0; s < S; ++s) hr[s] = H.mod(ps[s]);
        auto mr = mixed_radix(hr, ps);
        for (int s = 0; s < S; ++s) T.halfP[s] = (uint32_t)mr[s];
    }
    for (int l = 0; l < c->L; ++l) {
        const u64 q = c->ctq[l];
        u64 pref = 1;
        for (int s = 0; s < S; ++s) {
            T.pref_w[l][s] = pref;
            T.pref_ws[l][s] = shoup_h(pref, q);
            pref = mulmod_h(pref, ps[s] % q, q);
        }
        const u64 pm = P.mod(q);
        T.negP[l] = pm == 0 ? 0 : q - pm;
        constexpr u64 M30 = (1ull << 30) - 1;
        for (int s = 0; s < S; ++s) {
            u64 cs = 1;   // (P / p_s) mod q
            for (int k = 0; k < S; ++k)
                if (k != s) cs = mulmod_h(cs, ps[k] % q, q);
            T.fpc_c[l][s][0] = (uint32_t)(cs & M30);
            T.fpc_c[l][s][1] = (uint32_t)(cs >> 30);
        }
        T.fpc_n[l][0] = (uint32_t)(T.negP[l] & M30);
        T.fpc_n[l][1] = (uint32_t)(T.negP[l] >> 30);
    }
    HIP_TRY(dev_alloc((void**)&b->d_kst, sizeof(Ks32Tables)));
    if (int e_ = upload(c, b->d_kst, &T, sizeof(Ks32Tables))) return e_;
    b->S = S;
    return 0;
}

// the active primary basis (run_mul, dbfv_mul_group, bfv_apply_automorphism read these fields)
static void use_ks32_basis(exacto_ctx* c, const Ks32Basis& b) {
    c->S32 = b.S;
    c->d_p32 = b.d_p32;
    c->d_tw32 = b.d_tw32;
    c->d_kst = b.d_kst;
    c->ks32_sum_max = b.sum_max;
    c->ks32_fpc_max = b.fpc_max;
    c->ks32_mac_form = b.mac_form;
    c->ks32_lazy_active = &b == &c->kz;
}

static void free_basis(Ks32Basis* b) {
    free_dev(b->d_p32); free_dev(b->d_tw32); free_dev(b->d_kst); free_dev(b->d_rs);
    *b = Ks32Basis{};
}

// build_ks32_basis_impl, releasing whatever it allocated when a later step fails (the basis is not
// attached to the context yet, so exacto_ctx_destroy would not free it)
static int build_ks32_basis(exacto_ctx* c, u64 pmax, u64 qmax, const Big& bound, Ks32Basis* b, int fixedS = 0) {
    const int e = build_ks32_basis_impl(c, pmax, qmax, bound, b, fixedS);
    if (e) free_basis(b);
    return e;
}

// ks32.hip's auxiliary bases, bounding |sum_g d_g * r_g| <= G n floor(B/2) floor(q_max/2) (digits
// balanced in [-B/2, B/2), key coefficients balanced).  Eligible: exact path, gadget base <= 2^16
// (int16 digits), every ciphertext prime 2^60 - d with d < 2^24 (ks32_crt reduces with
// reduce_near60), 1024 <= n <= 16384; S <= 4.
//   primary: primes below 2^32 / 3, so that sums of three residues fit 32 bits and the MAC adds
//            twelve balanced products (< 2^58.9) per reduction;
//   wide:    primes up to 2^31 (seven products per reduction), kept only when it holds more
//            dBFV digit sums than the primary (cfg4: two products per limb).
// EXACTO_KS32_WIDE=0: no wide basis; =2: the wide basis as the primary too (A/B switch).
static int setup_ks32(exacto_ctx* c) {
    c->S32 = 0;
    if (c->path != EXACTO_PATH_EXACT_RNS || c->gbase > 65536 || c->logn < 10 || c->logn > 14 || c->L > 4)
        return 0;
    u64 qmax = 0;
    for (u64 q : c->ctq) {
        if (q >= (1ull << 60) || q <= (1ull << 60) - (1ull << 24)) return 0;
        qmax = std::max(qmax, q);
    }
    Big bound((u64)c->G);
    bound.mul((u64)c->n);
    bound.mul(c->gbase / 2);
    bound.mul(qmax / 2);
    bound.mul(2);
    bound.add(1);
    const char* wide_env = getenv("EXACTO_KS32_WIDE");
    const int wide_mode = wide_env ? atoi(wide_env) : 1;
    Ks32Basis prim;
    if (int e = build_ks32_basis(c, wide_mode == 2 ? (1ull << 31) : (1ull << 32) / 3, qmax, bound, &prim)) return e;
    if (wide_mode == 1) {
        if (int e = build_ks32_basis(c, 1ull << 31, qmax, bound, &c->kw)) {
            free_basis(&prim);
            return e;
        }
        if (prim.S == 0 && c->kw.S > 0) {   // only the wide range holds the bound: it is the primary
            prim = c->kw;
            c->kw = Ks32Basis{};
        } else if (c->kw.S > 0 && c->kw.sum_max <= prim.sum_max) {
            free_basis(&c->kw);
        }
    }
    if (prim.S == 0) return 0;
    c->kn = prim;
    // the lazy basis: as many primes below 2^30 as the primary has (the workspaces are sized by S)
    const char* lz = getenv("EXACTO_KS32_LAZY");
    if (!(lz && lz[0] == '0') && wide_mode != 2)
        if (int e = build_ks32_basis(c, 1ull << 30, qmax, bound, &c->kz, prim.S)) return e;
    use_ks32_basis(c, c->kn);
    return 0;
}

static int build_tables(exacto_ctx* c) {
    const int NP = (int)c->primes.size();
    std::vector<TwPair> tw((size_t)NP * 2 * c->n);
    std::vector<PrimeConst> pc(NP);
    for (int t = 0; t < NP; ++t)
        pc[t] = make_prime_const(c->primes[t], c->n, c->logn, &tw[(size_t)t * 2 * c->n],
                                 &tw[(size_t)t * 2 * c->n + c->n]);
    HIP_TRY(dev_alloc((void**)&c->d_tw, tw.size() * sizeof(TwPair)));
    if (int e_ = upload(c, c->d_tw, tw.data(), tw.size() * sizeof(TwPair))) return e_;
    for (int t = 0; t < NP; ++t) {
        pc[t].tw_fwd = c->d_tw + (size_t)t * 2 * c->n;
        pc[t].tw_inv = c->d_tw + (size_t)t * 2 * c->n + c->n;
    }
    HIP_TRY(dev_alloc((void**)&c->d_primes, NP * sizeof(PrimeConst)));
    if (int e_ = upload(c, c->d_primes, pc.data(), NP * sizeof(PrimeConst))) return e_;

    // ---- CRT tables
    CrtTables& C = c->h_crt;
    std::memset(&C, 0, sizeof(C));
    const int L = c->L, K = c->K;
    C.L = L;
    C.K = K;
    C.G = c->G;
    C.gbase = c->gbase;
    C.gshift = (c->gbase & (c->gbase - 1)) == 0 ? bitlen(c->gbase) - 1 : -1;
    C.plain = c->plain;
    const std::vector<u64> qv(c->primes.begin(), c->primes.begin() + L);
    const std::vector<u64> pv(c->primes.begin() + L, c->primes.end());
    for (int i = 0; i < L; ++i)
        for (int k = 0; k < i; ++k) set_shoup(C.gq_w[i][k], C.gq_ws[i][k], invmod_h(qv[k] % qv[i], qv[i]), qv[i]);
    Big Q(1);
    for (u64 q : qv) Q.mul(q);
    Big H = Q;
    H.shr1();
    {
        std::vector<u64> hr(L);
        for (int i = 0; i < L; ++i) hr[i] = H.mod(qv[i]);
        auto mr = mixed_radix(hr, qv);
        for (int i = 0; i < L; ++i) C.halfQ_mr[i] = mr[i];
    }
    for (int t = 0; t < NP; ++t) {
        const u64 pt = c->primes[t];
        u64 pref = 1 % pt;
        for (int k = 0; k <= L; ++k) {
            set_shoup(C.qpref_w[k][t], C.qpref_ws[k][t], pref, pt);
            if (k < L) pref = mulmod_h(pref, qv[k] % pt, pt);
        }
        set_shoup(C.pmod_w[t], C.pmod_ws[t], c->plain % pt, pt);
    }
    for (int i = 0; i < L && i < (int)Q.w.size(); ++i) C.Qwords[i] = Q.w[i];
    for (int t = 0; t < NP; ++t) C.hq[t] = H.mod(c->primes[t]);
    if (c->path == EXACTO_PATH_HPS) {
        const u64 q = qv[0];
        for (int a = 0; a < K && a < 2; ++a) {
            C.hps_qinv[a] = invmod_h(q % pv[a], pv[a]);
            C.hps_qinv_s[a] = shoup_h(C.hps_qinv[a], pv[a]);
        }
        if (c->plain < q) C.hps_pc = (u64)(((u128)c->plain << 64) / q);
        if (K == 2) {
            C.hps_p1_inv_p0 = invmod_h(pv[1] % pv[0], pv[0]);
            C.hps_p0_inv_p1 = invmod_h(pv[0] % pv[1], pv[1]);
            set_shoup(C.hps_t_w[0], C.hps_t_ws[0], mulmod_h(C.hps_qinv[0], C.hps_p1_inv_p0, pv[0]), pv[0]);
            set_shoup(C.hps_t_w[1], C.hps_t_ws[1], mulmod_h(C.hps_qinv[1], C.hps_p0_inv_p1, pv[1]), pv[1]);
            set_shoup(C.hps_pq_w[0], C.hps_pq_ws[0], pv[1] % q, q);
            set_shoup(C.hps_pq_w[1], C.hps_pq_ws[1], pv[0] % q, q);
            const u128 P = (u128)pv[0] * pv[1];
            const u64 Pq = (u64)(P % q);
            C.hps_kPq[0] = 0;
            C.hps_kPq[1] = Pq;
            C.hps_kPq[2] = (u64)(((u128)Pq * 2) % q);
            C.hps_P[0] = (u64)P; C.hps_P[1] = (u64)(P >> 64);
            C.hps_halfP[0] = (u64)(P >> 1); C.hps_halfP[1] = (u64)(P >> 65);
        }
    } else {
        for (int a = 0; a < K; ++a)
            for (int k = 0; k < a; ++k) set_shoup(C.gp_w[a][k], C.gp_ws[a][k], invmod_h(pv[k] % pv[a], pv[a]), pv[a]);
        Big P(1);
        for (u64 p : pv) P.mul(p);
        Big HP = P;
        HP.shr1();
        std::vector<u64> hr(K);
        for (int a = 0; a < K; ++a) hr[a] = HP.mod(pv[a]);
        auto mr = mixed_radix(hr, pv);
        for (int a = 0; a < K; ++a) C.halfP_mr[a] = mr[a];
        for (int i = 0; i < L; ++i) {
            u64 pref = 1 % qv[i];
            for (int k = 0; k <= K; ++k) {
                set_shoup(C.ppref_w[k][i], C.ppref_ws[k][i], pref, qv[i]);
                if (k < K) pref = mulmod_h(pref, pv[k] % qv[i], qv[i]);
            }
        }
        for (int a = 0; a < K; ++a) {
            const u64 pa = pv[a];
            const u64 qinv = invmod_h(Q.mod(pa), pa);
            set_shoup(C.qinvp_w[a], C.qinvp_ws[a], qinv, pa);
            set_shoup(C.pq_w[a], C.pq_ws[a], mulmod_h(c->plain % pa, qinv, pa), pa);
            for (int k = 0; k <= L; ++k)
                set_shoup(C.qpq_w[k][a], C.qpq_ws[k][a], mulmod_h(C.qpref_w[k][L + a], qinv, pa), pa);
        }
        for (int a = 0; a < K; ++a) {   // the FPC constants (see CrtTables)
            const u64 pa = pv[a];
            u64 others = 1;   // (P / p_a) mod p_a
            for (int b = 0; b < K; ++b)
                if (b != a) others = mulmod_h(others, pv[b] % pa, pa);
            const u64 pi = invmod_h(others, pa);
            C.fpc_pq[a] = mulmod_h(C.pq_w[a], pi, pa);
            for (int k = 0; k < L; ++k) C.fpc_qpq[k][a] = mulmod_h((pa - C.qpq_w[k][a]) % pa, pi, pa);
            C.fpc_neg[a] = pi;
            C.fpc_inv[a] = 1.0 / (double)pa;
            for (int i = 0; i < L; ++i) {
                u64 pm = 1 % qv[i];
                for (int b = 0; b < K; ++b)
                    if (b != a) pm = mulmod_h(pm, pv[b] % qv[i], qv[i]);
                C.fpc_pm[a][i] = pm;
            }
        }
        for (int i = 0; i < L; ++i) {
            const u64 pm = P.mod(qv[i]);
            C.fpc_negP[i] = pm == 0 ? 0 : qv[i] - pm;
        }
        for (int i = 0; i < L; ++i) {   // the FPQ constants (see CrtTables)
            const u64 q = qv[i];
            u64 qo = 1 % q;   // (Q / q_i) mod q_i
            for (int k = 0; k < L; ++k)
                if (k != i) qo = mulmod_h(qo, qv[k] % q, q);
            set_shoup(C.fpq_pz_w[i], C.fpq_pz_ws[i], mulmod_h(c->plain % q, invmod_h(qo, q), q), q);
            C.fpq_inv0[i] = 1.0 / (double)q;
            C.fpq_inv1[i] = (double)(1ull << 30) / (double)q;
            for (int a = 0; a < K; ++a) {
                const u64 pa = pv[a], qi = invmod_h(q % pa, pa);
                C.fpq_c[i][a] = mulmod_h((pa - qi) % pa, C.fpc_neg[a], pa);
            }
        }
    }
    {
        const u64 mx = *std::max_element(c->primes.begin(), c->primes.end());
        const u64 mn = *std::min_element(c->primes.begin(), c->primes.end());
        C.near = (u128)mx < 2 * (u128)mn;
        C.fast = C.near && mx < (1ull << 60);
        C.special = C.fast && mn > (1ull << 60) - (1ull << 24);
        C.digit_small = c->gbase <= *std::min_element(qv.begin(), qv.end());
    }
    HIP_TRY(dev_alloc((void**)&c->d_scal, EXACTO_MAX_L * sizeof(u64)));
    HIP_TRY(dev_alloc((void**)&c->d_crt, sizeof(CrtTables)));
    if (int e_ = upload(c, c->d_crt, &C, sizeof(CrtTables))) return e_;
    return 0;
}

extern "C" int exacto_ctx_create(exacto_ctx** out, size_t n, const uint64_t* ct_moduli, size_t L,
                                 const uint64_t* aux_moduli, size_t num_aux, uint64_t plain,
                                 uint64_t gadget_base, int device) {
    if (!out) return invalid_param("null context pointer");
    *out = nullptr;
    // BfvParamsBuilder::build order (params/mod.rs:81-98)
    if (n < 2 || (n & (n - 1)) != 0)
        return fail(EXACTO_ERR_INVALID_RING_DEGREE, "ring degree must be a power of 2, got " + std::to_string(n));
    if (L == 0 || !ct_moduli) return invalid_param("must specify at least one ciphertext modulus");
    if (plain < 2) return invalid_param("plaintext modulus must be >= 2");
    if (n > 16384) return invalid_param("ring degree " + std::to_string(n) + " exceeds the HIP NTT limit of 16384");
    if (L > EXACTO_MAX_L) return invalid_param("at most " + std::to_string(EXACTO_MAX_L) + " ciphertext moduli are supported");
    for (size_t i = 0; i < L; ++i)
        if (int e = plan_check(n, ct_moduli[i])) return e;
    for (size_t i = 0; i < L; ++i)
        for (size_t k = 0; k < i; ++k)
            if (ct_moduli[i] == ct_moduli[k]) return invalid_param("RNS moduli must be coprime");
    for (size_t i = 0; i < num_aux; ++i)
        if (int e = plan_check(n, aux_moduli[i])) return e;

    exacto_ctx* c = new exacto_ctx();
    c->device = device;
    c->n = (int)n;
    c->logn = bitlen(n) - 1;
    c->L = (int)L;
    c->ctq.assign(ct_moduli, ct_moduli + L);
    if (num_aux) c->user_aux.assign(aux_moduli, aux_moduli + num_aux);
    c->plain = plain;
    c->gbase = gadget_base == 0 ? (1ull << 16) : gadget_base;
    if (c->gbase < 2) { delete c; return invalid_param("gadget base must be >= 2"); }
    // compute_gadget_digits (params/mod.rs:126-140)
    {
        Big Q(1);
        for (u64 q : c->ctq) Q.mul(q);
        Big pw(1);
        int g = 0;
        while (pw.cmp(Q) < 0) { pw.mul(c->gbase); ++g; }
        c->G = std::max(g, 1);
    }
    if (c->G > EXACTO_MAX_G) { delete c; return invalid_param("gadget digit count exceeds " + std::to_string(EXACTO_MAX_G)); }
    // dispatcher (eval.rs:99-107)
    if (L > 1) {
        c->path = EXACTO_PATH_EXACT_RNS;
    } else if (num_aux > 0) {
        c->path = EXACTO_PATH_HPS;
        const u64 q = c->ctq[0];
        if (num_aux == 1) {
            const u128 min_required = ((u128)n * q) / 2;
            if ((u128)c->user_aux[0] <= min_required) {
                c->deferred_code = EXACTO_ERR_INVALID_PARAM;
                c->deferred_msg = "invalid parameter: single aux prime too small for HPS centering: P=" +
                                  std::to_string(c->user_aux[0]) + " <= n*Q/2=" + std::to_string((u64)min_required);
            }
        } else if (num_aux > 2) {
            c->deferred_code = EXACTO_ERR_INVALID_PARAM;
            c->deferred_msg = "invalid parameter: HPS scaling supports 1 or 2 aux primes, got " + std::to_string(num_aux);
        }
    } else {
        c->path = EXACTO_PATH_SCHOOLBOOK;
        // schoolbook_overflow_risk (eval.rs:457-464), u128 saturating
        const u128 maxc = c->ctq[0] / 2;
        const u128 sat = ~(u128)0;
        const u128 i128max = sat >> 1;
        auto smul = [&](u128 a, u128 b) -> u128 { return (b != 0 && a > sat / b) ? sat : a * b; };
        const u128 max_tensor = smul(smul((u128)n, maxc), maxc);
        const u128 max_scaled = smul(max_tensor, (u128)plain);
        if (max_tensor > i128max || max_scaled > i128max) {
            c->deferred_code = EXACTO_ERR_NOT_IMPLEMENTED;
            c->deferred_msg = "not yet implemented: schoolbook BFV multiplication can overflow i128 for these "
                              "parameters; use HPS auxiliary basis";
        }
    }
    c->primes = c->ctq;
    if (c->path == EXACTO_PATH_HPS) {
        if (num_aux <= 2) {
            c->K = (int)num_aux;
            for (u64 p : c->user_aux) c->primes.push_back(p);
        }
    } else {
        // internal auxiliary basis P > 4 * p * n * Q (exact tensor and exact rounding fit)
        Big need(4);
        need.mul(plain);
        need.mul(n);
        for (u64 q : c->ctq) need.mul(q);
        Big P(1);
        const u64 step = 2 * n;
        // below 2^60 so every prime of the exact path takes the lazy forward NTT (16q <= 2^64)
        u64 cand = ((1ull << 60) - 1) / step * step + 1;
        while (P.cmp(need) <= 0) {
            while (cand > step) {
                cand -= step;
                const bool used = std::find(c->ctq.begin(), c->ctq.end(), cand) != c->ctq.end();
                if (!used && is_prime_h(cand)) break;
            }
            c->int_aux.push_back(cand);
            P.mul(cand);
            if ((int)c->int_aux.size() > EXACTO_MAX_K) {
                delete c;
                return invalid_param("too many auxiliary primes required for exact multiplication");
            }
        }
        c->K = (int)c->int_aux.size();
        for (u64 p : c->int_aux) c->primes.push_back(p);
        // |r| <= p n Q / 2 + 1 for every scaled tensor component (|T| <= n Q^2 / 2), so a sum of m of
        // them is liftable from P (centred) when m (p n Q + 2) < P
        Big X(plain);
        X.mul(n);
        for (u64 q : c->ctq) X.mul(q);
        X.add(2);
        for (u64 m = 1; m <= 64; ++m) {
            Big Y = X;
            Y.mul(m);
            if (Y.cmp(P) >= 0) break;
            c->psum_max = (int)m;
        }
        // m (p n Q + 2) <= P / 2, i.e. |R| <= m (p n Q / 2 + 1) <= P / 4: the float CRT is exact
        for (u64 m = 1; m <= 64; ++m) {
            Big Y = X;
            Y.mul(2 * m);
            if (Y.cmp(P) >= 0) break;
            c->psum_fp_max = (int)m;
        }
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { delete c; return fail(EXACTO_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(e)); }
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return fail(EXACTO_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(e)); }
    c->own_stream = true;
    {
        // Per-call scratch (Scratch) comes from a stream-ordered pool created by the library, one per
        // device and shared by every context on it.  Its freed blocks stay mapped for reuse instead of
        // going back to the driver at every synchronisation (release threshold 0 is the default), and
        // the device's default pool keeps its settings for everything else in the process.
        // One pool per context instead (rounds 1-4; EXACTO_SCRATCH_POOL=own until round 5) made the
        // bootstrap's n = 16 scratch read back zeros written by no kernel of the library in 4 of 20 runs
        // of the C++ API test, 13 of 20 with destroyed contexts' pools kept alive, and 0 of 20 with one
        // pool for all contexts (tools/archive/r4_bootab.sh).  Round 6 removed that mode
        // ("own" now means the shared pool) and moved the bootstrap's intermediates off the pool.
        // The release threshold is read back after it is set: a pool that does not keep it is not used.
        // EXACTO_SCRATCH_POOL=default: the device's default pool (threshold raised there), for A/B
        const char* pe = getenv("EXACTO_SCRATCH_POOL");
        const std::string mode = pe ? pe : "shared";
        uint64_t thr = ~0ull;
        auto make_pool = [&](hipMemPool_t* p) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = device;
            if (hipMemPoolCreate(p, &props) != hipSuccess) return (*p = nullptr, false);
            dbg_alloc_log("hipMemPoolCreate", nullptr, 0, *p, nullptr, false);
            uint64_t back = 0;
            const bool set = hipMemPoolSetAttribute(*p, hipMemPoolAttrReleaseThreshold, &thr) == hipSuccess &&
                             hipMemPoolGetAttribute(*p, hipMemPoolAttrReleaseThreshold, &back) == hipSuccess;
            if (dbg_alloc_on())
                std::fprintf(stderr, "exacto-alloc pool %p device %d release threshold set %s, read back 0x%llx\n",
                             (void*)*p, device, set ? "ok" : "FAILED", (unsigned long long)back);
            if (set && back == thr) return true;
            (void)hipMemPoolDestroy(*p);
            return (*p = nullptr, false);
        };
        if (mode != "default") {
            static std::mutex mu;
            static std::map<int, hipMemPool_t> shared;   // never destroyed: lives as long as the process
            std::lock_guard<std::mutex> g(mu);
            auto it = shared.find(device);
            if (it == shared.end()) {
                hipMemPool_t p = nullptr;
                if (make_pool(&p)) it = shared.emplace(device, p).first;
            }
            if (it != shared.end()) c->pool = it->second;
        }
        if (!c->pool) {   // Scratch uses the device's default pool, kept mapped the same way
            hipMemPool_t dp;
            if (hipDeviceGetDefaultMemPool(&dp, device) == hipSuccess)
                (void)hipMemPoolSetAttribute(dp, hipMemPoolAttrReleaseThreshold, &thr);
        }
    }
    if (const char* e = getenv("EXACTO_DEBUG_SCRATCH")) c->debug_scratch = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_DBFV_GROUP_MB")) c->dbfv_group_bytes = (size_t)std::max(1, atoi(e)) << 20;
    if (const char* e = getenv("EXACTO_NTT_ASM")) c->ntt_asm = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_NTT_ASM_INV")) c->ntt_asm_inv = atoi(e) != 0;
    // products per pipeline chunk: 512 at cfg3's n (L + K) = 4096 x 7, more where a product is smaller,
    // so that every chunk's launches (and workspace, ~1.4 GB) stay about the same size (compact_bfv,
    // n = 1024 with L + K = 2: 7168 products per chunk instead of launches of a few blocks per CU)
    c->chunk = (size_t)std::min<long>(8192, std::max<long>(512, 512L * 4096 * 7 / ((long)n * (c->L + c->K)) / 64 * 64));
    if (const char* e = getenv("EXACTO_DUAL_STREAM")) c->dual = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_LANES")) c->lanes = std::max(1, std::min(EXACTO_MAX_LANES, atoi(e)));
    if (const char* e = getenv("EXACTO_SHARE_EXT")) c->share_ext = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_DIGIT16")) c->digit16 = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_KS32")) c->ks32 = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_PSUM")) c->psum_env = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_CHAIN_SPLIT")) c->batch_split = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_FP_CRT")) c->fp_crt = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_FPQ")) c->fpq_lim = atoi(e) == 0 ? 0.0 : atoi(e) == 2 ? 0.25 : c->fpq_lim;
    if (const char* e = getenv("EXACTO_KS_FPC")) c->ks_fpc = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_DIGIT8")) c->digit8_env = atoi(e) != 0;
    if (const char* e = getenv("EXACTO_HPS_SUM")) c->hps_sum_env = atoi(e) != 0;
    c->hps_fast = c->path == EXACTO_PATH_HPS && c->ctq[0] > (1ull << 32) && c->plain < c->ctq[0] &&
                  c->plain < (1ull << 32);
    if (const char* e = getenv("EXACTO_HPS_LITERAL")) c->hps_fast &= atoi(e) == 0;
    if (int rc = build_tables(c)) { exacto_ctx_destroy(c); return rc; }
    if (int rc = setup_ks32(c)) { exacto_ctx_destroy(c); return rc; }
    *out = c;
    return 0;
}

extern "C" void exacto_ctx_destroy(exacto_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    // EXACTO_LEAK_CTX=1 (diagnostic of DESIGN.md §3): keep every allocation of a destroyed context
    static const bool leak = [] { const char* e = getenv("EXACTO_LEAK_CTX"); return e && e[0] == '1'; }();
    if (leak) return;
    for (auto& r : c->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    free_dev(c->d_primes); free_dev(c->d_tw); free_dev(c->d_crt); free_dev(c->d_scal); free_dev(c->d_rlk); free_dev(c->d_rlk_s);
    free_dev(c->ws_coefQ); free_dev(c->ws_extP); free_dev(c->ws_T); free_dev(c->ws_D); free_dev(c->chain_buf); free_dev(c->chain_coef); free_dev(c->dec_buf); free_dev(c->dig_buf);
    for (LaneSet& l : c->xl) {
        if (l.stream) { (void)hipStreamSynchronize(l.stream); (void)hipStreamDestroy(l.stream); }
        if (l.join) (void)hipEventDestroy(l.join);
        free_dev(l.coefQ); free_dev(l.extP); free_dev(l.T); free_dev(l.D); free_dev(l.DS); free_dev(l.U);
        if (l.D16) (void)hipFree(l.D16);
    }
    free_dev(c->ext_a); free_dev(c->ext_b);
    free_dev((u64*)c->d_cdt); free_dev(c->d_gpow); free_dev(c->d_delta); free_dev(c->enc_buf); free_dev(c->gk_s); free_dev(c->d_gk_rs); free_dev(c->d_dall); free_dev(c->d_hdig); free_dev(c->d_dk); free_dev(c->d_dsk); free_dev(c->d_uk); free_dev(c->pl_buf);
    if (c->ws_D16) (void)hipFree(c->ws_D16);
    free_dev(c->d_rs);   // the active basis' tables belong to kn / kz
    free_dev(c->kn.d_p32); free_dev(c->kn.d_tw32); free_dev(c->kn.d_kst); free_dev(c->kn.d_rs);
    free_dev(c->kz.d_p32); free_dev(c->kz.d_tw32); free_dev(c->kz.d_kst); free_dev(c->kz.d_rs);
    free_dev(c->kw.d_p32); free_dev(c->kw.d_tw32); free_dev(c->kw.d_kst); free_dev(c->kw.d_rs);
    free_dev(c->ws_DS); free_dev(c->ws_U);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    for (int i = 0; i < exacto_ctx::MAX_TWINS; ++i) {
        if (c->twin[i]) exacto_ctx_destroy(c->twin[i]);
        if (c->ev_twin_out[i]) (void)hipEventDestroy(c->ev_twin_out[i]);
    }
    if (c->ev_twin_in) (void)hipEventDestroy(c->ev_twin_in);
    free_dev(c->io); free_dev(c->prod); free_dev(c->d_off); free_dev(c->d_term_start); free_dev(c->d_terms);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    free_dev(c->boot_buf); free_dev(c->boot_slots);
    delete c;
}

extern "C" int exacto_ctx_get_info(const exacto_ctx* c, exacto_ctx_info* info) {
    if (!c || !info) return invalid_param("null argument");
    info->ring_degree = c->n;
    info->num_ct_moduli = c->L;
    info->num_aux_moduli = c->user_aux.size();
    info->num_internal_aux = c->int_aux.size();
    info->gadget_digits = c->G;
    info->gadget_base = c->gbase;
    info->plain_modulus = c->plain;
    info->mul_path = c->path;
    info->device = c->device;
    info->ks32_primes = c->ks32 ? c->S32 : 0;
    info->psum_max = c->psum_env ? c->psum_max : 0;
    info->ks32_lazy = c->ks32 && c->ks32_lazy_active ? 1 : 0;
    info->ntt_order = EXACTO_NTT_ORDER;
    info->dbfv_key_switch = c->last_dbfv_ks;
    return 0;
}

extern "C" int exacto_ctx_set_stream(exacto_ctx* c, void* s) {
    // The handle is used as given; NULL is the device's default (null) stream, which is what
    // torch.cuda.current_stream().cuda_stream returns for the default torch stream.
    if (!c) return invalid_param("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->own_stream && c->stream) HIP_TRY(hipStreamDestroy(c->stream));
    c->stream = (hipStream_t)s;
    c->own_stream = false;
    return 0;
}

extern "C" int exacto_ctx_set_chunk(exacto_ctx* c, size_t chunk) {
    if (!c) return invalid_param("null context");
    c->chunk = chunk == 0 ? 128 : chunk;
    return 0;
}

extern "C" int exacto_synchronize(exacto_ctx* c) {
    if (!c) return invalid_param("null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

static size_t poly_bytes(const exacto_ctx* c) { return (size_t)c->n * sizeof(u64); }

extern "C" uint64_t* exacto_ctx_relin_key_buffer(exacto_ctx* c, size_t num_keys) {
    if (!c) return nullptr;
    const size_t bytes = num_keys * 2 * c->L * poly_bytes(c);
    if (hipSetDevice(c->device) != hipSuccess) return nullptr;
    if (grow(&c->d_rlk, &c->rlk_cap, std::max<size_t>(bytes, 8))) return nullptr;
    c->rlk_keys = num_keys;
    c->rlk_loaded = true;
    c->rlk_s_valid = false;  // contents change: companions recomputed before first use
    c->rs_valid = false; c->kw.rs_valid = false;     // and the auxiliary-basis key
    ++c->rlk_version;
    return c->d_rlk;
}

extern "C" int exacto_ctx_load_relin_key_dev(exacto_ctx* c, const uint64_t* rlk, size_t num_keys) {
    if (!c) return invalid_param("null context");
    if (num_keys && !rlk) return invalid_param("null relinearization key");
    u64* dst = exacto_ctx_relin_key_buffer(c, num_keys);
    if (!dst) return fail(EXACTO_ERR_HIP, "HIP error: relinearization key allocation failed");
    if (num_keys)
        HIP_TRY(dev_copy(dst, rlk, num_keys * 2 * c->L * poly_bytes(c), c->stream));
    return 0;
}

extern "C" int exacto_ctx_load_relin_key(exacto_ctx* c, const uint64_t* rlk, size_t num_keys) {
    if (!c) return invalid_param("null context");
    if (num_keys && !rlk) return invalid_param("null relinearization key");
    u64* dst = exacto_ctx_relin_key_buffer(c, num_keys);
    if (!dst) return fail(EXACTO_ERR_HIP, "HIP error: relinearization key allocation failed");
    if (num_keys) if (int e_ = upload(c, dst, rlk, num_keys * 2 * c->L * poly_bytes(c))) return e_;
    return 0;
}

// ============================================================== NTT helper (+ profiling)

// Kernel families timed by exacto_prof_enable (HIP events around each launch on the launching
// stream; the bench's roofline takes the family with the largest share of a profiled step).
// Bytes are ALGORITHMIC: each operand read once and each result written once.
enum ProfKind : int {
    PK_FWD = 0, PK_INV = 1, PK_TENSOR = 2, PK_POLYMUL = 3, PK_LIFT = 4, PK_SCALE = 5, PK_KS_DIGITS = 6,
    PK_KS_MAC = 7, PK_KS_CRT = 8, PK_PAIRSUM = 9, PK_PSUM_SCALE = 10, PK_TENSOR_C2 = 11, PK_DIGIT_SUM = 12,
    PK_COMBINE = 13, PK_HPS_EXT = 14, PK_RELIN_MAC = 15, PK_HPS_SCALE = 16, PK_COUNT = 17
};

struct ProfScope {
    exacto_ctx* c;
    ProfRec rec{};
    bool on;
    ProfScope(exacto_ctx* c_, int kind, u64 units, double bytes) : c(c_), on(c_->prof) {
        if (!on) return;
        rec.kind = kind; rec.polys = units; rec.bytes = bytes;
        g_last_kernel = nullptr;
        if (hipEventCreate(&rec.a) != hipSuccess || hipEventCreate(&rec.b) != hipSuccess ||
            hipEventRecord(rec.a, c->stream) != hipSuccess)
            on = false;
    }
    ~ProfScope() {
        if (!on) return;
        rec.kern = g_last_kernel;
        if (hipEventRecord(rec.b, c->stream) == hipSuccess) c->recs.push_back(rec);
    }
};

static int run_ntt(exacto_ctx* c, const NttBatch& nb, long count, bool inverse) {
    if (count <= 0) return 0;
    // algorithmic bytes: one read of the source (int16 digits: 2 B per coefficient) + one 8 B write
    ProfScope ps(c, inverse ? PK_INV : PK_FWD, (u64)count, ((nb.src16 ? 2.0 : 8.0) + 8.0) * c->n * (double)count);
    bool lazy = true, near60 = c->ntt_asm;
    int qbits = 0;   // bit length of the batch's largest prime
    for (int t = nb.prime_base; t < nb.prime_base + nb.period; ++t) {
        lazy &= c->primes[t] < (1ull << 60);
        near60 &= c->primes[t] < (1ull << 60) && c->primes[t] > (1ull << 60) - (1ull << 32);
        qbits = std::max(qbits, 64 - __builtin_clzll(c->primes[t]));
    }
    launch_ntt(nb, (int)count, c->logn, inverse, lazy, c->d_primes, c->stream, near60, near60 && c->ntt_asm_inv, qbits);
    CHECK_LAUNCH();
    return 0;
}

// two forward batches in one launch where both take the pinned rounds (every prime 2^60 - d, n = 4096
// / 8192), else two launches
static int run_ntt_fwd2(exacto_ctx* c, const NttBatch& nb1, long count1, const NttBatch& nb2, long count2) {
    bool near60 = c->ntt_asm && !nb1.src16 && !nb2.src16;
    for (u64 q : c->primes) near60 &= q < (1ull << 60) && q > (1ull << 60) - (1ull << 32);
    if (near60 && count1 > 0 && count2 > 0) {
        ProfScope ps(c, PK_FWD, (u64)(count1 + count2), 16.0 * c->n * (double)(count1 + count2));
        if (launch_ntt_fwd2(nb1, (int)count1, nb2, (int)count2, c->logn, c->d_primes, c->stream)) {
            CHECK_LAUNCH();
            return 0;
        }
    }
    if (int e = run_ntt(c, nb1, count1, false)) return e;
    return run_ntt(c, nb2, count2, false);
}

// the tensor runs the asm kernels (products by MulNear60*Asm, special-prime inverse rounds)
static bool tensor_asm(const exacto_ctx* c) {
    bool near60 = c->ntt_asm && c->ntt_asm_inv;
    for (int t = 0; t < c->L + c->K; ++t)   // the fused product needs d = 2^60 - q < 2^24
        near60 &= c->primes[t] < (1ull << 60) && c->primes[t] > (1ull << 60) - (1ull << 24);
    return near60;
}

static int run_inv_tensor(exacto_ctx* c, const Operands& o, int cnt, bool p2only = false) {
    const int NP = c->L + c->K;
    bool lazy = true;
    const bool near60 = tensor_asm(c);
    int qbits = 0;
    for (int t = 0; t < NP; ++t) {
        qbits = std::max(qbits, 64 - __builtin_clzll(c->primes[t]));
        lazy &= c->primes[t] < (1ull << 60);
    }
    // algorithmic bytes per (item, prime): the four operands a0, a1, b0, b1 in and the three
    // components out (7 polys); psum's auxiliary primes only c2 = a1 b1 (2 in, 1 out).  dBFV with
    // shared extensions (tensor_share_d > 0): the d^2 products of an item read only its 2d distinct
    // ciphertexts, so the inputs count once per ciphertext (the chunk's ceil(cnt / npairs) items),
    // not once per product (which overcounted: u64_dbfv's measured traffic was 0.95 of it)
    const double pb = 8.0 * c->n;
    double bytes;
    if (c->tensor_share_d > 0 && c->tensor_share_npairs > 0) {
        const double items = (double)((cnt + c->tensor_share_npairs - 1) / c->tensor_share_npairs);
        const double cts = items * 2.0 * c->tensor_share_d;
        bytes = pb * (c->L * (2.0 * cts + 3.0 * cnt) +
                      c->K * (p2only ? cts + (double)cnt : 2.0 * cts + 3.0 * cnt));
    } else {
        bytes = cnt * (p2only ? pb * (7.0 * c->L + 3.0 * c->K) : pb * 7.0 * NP);
    }
    ProfScope ps(c, PK_TENSOR, (u64)cnt * (p2only ? 3 * c->L + c->K : 3 * NP), bytes);
    // the exact path's scale kernels take T in [0, 2q) (shoup products, 30-bit-limb dot products with
    // headroom); the HPS scale subtracts residues as canonical
    launch_inv_tensor(o, c->ws_extP, c->ws_T, cnt, c->logn, c->L, c->K, lazy, c->d_primes, c->stream, near60, p2only,
                      qbits, c->tensor_share_npairs, near60 && c->path != EXACTO_PATH_HPS);
    CHECK_LAUNCH();
    return 0;
}

static NttBatch contiguous(u64* data, long count_items, long poly_per_item, int prime_base, int period,
                           int n) {
    (void)count_items;
    NttBatch nb{};
    nb.src = data;
    nb.src_off = nullptr;
    nb.src_item_stride = poly_per_item * n;
    nb.dst = data;
    nb.dst_item_stride = poly_per_item * n;
    nb.ppi = (int)poly_per_item;
    nb.prime_base = prime_base;
    nb.period = period;
    return nb;
}

// ============================================================== workspace

static int ensure_workspace(exacto_ctx* c, size_t items) {
    if (c->ws_items >= items) return 0;
    free_dev(c->ws_coefQ); free_dev(c->ws_extP); free_dev(c->ws_T); free_dev(c->ws_D);
    c->ws_coefQ = c->ws_extP = c->ws_T = c->ws_D = nullptr;
    c->ws_items = 0;
    const size_t pb = poly_bytes(c);
    const int NP = c->L + c->K;
    HIP_TRY(dev_alloc((void**)&c->ws_coefQ, items * 4 * c->L * pb));
    HIP_TRY(dev_alloc((void**)&c->ws_extP, items * 4 * std::max(c->K, 1) * pb));
    HIP_TRY(dev_alloc((void**)&c->ws_T, items * 3 * NP * pb));
    HIP_TRY(dev_alloc((void**)&c->ws_D, items * std::max(c->G, 1) * c->L * pb));
    if (c->ws_D16) (void)hipFree(c->ws_D16);
    HIP_TRY(dev_alloc((void**)&c->ws_D16, items * std::max(c->G, 1) * c->n * sizeof(int16_t)));
    free_dev(c->ws_DS); free_dev(c->ws_U);
    c->ws_DS = c->ws_U = nullptr;
    if (c->S32) {  // ks32: digit residues [item][G][S][n] and accumulators [item][2L][S][n]
        HIP_TRY(dev_alloc((void**)&c->ws_DS, items * std::max(c->G, 1) * c->S32 * c->n * sizeof(uint32_t)));
        HIP_TRY(dev_alloc((void**)&c->ws_U, items * 2 * c->L * c->S32 * c->n * sizeof(uint32_t)));
    }
    c->ws_items = items;
    return 0;
}

// Extra pipeline lane `idx` (1 ..): its stream, join event and workspace (allocated on first use).
static int ensure_lane(exacto_ctx* c, int idx, size_t items) {
    if (!c->ev_fork) HIP_TRY(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    LaneSet& l = c->xl[idx - 1];
    if (!l.stream) HIP_TRY(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
    if (!l.join) HIP_TRY(hipEventCreateWithFlags(&l.join, hipEventDisableTiming));
    if (l.items >= items) return 0;
    free_dev(l.coefQ); free_dev(l.extP); free_dev(l.T); free_dev(l.D); free_dev(l.DS); free_dev(l.U);
    if (l.D16) (void)hipFree(l.D16);
    l.coefQ = l.extP = l.T = l.D = nullptr;
    l.D16 = nullptr;
    l.DS = l.U = nullptr;
    l.items = 0;
    const size_t pb = poly_bytes(c);
    const int NP = c->L + c->K;
    HIP_TRY(dev_alloc((void**)&l.coefQ, items * 4 * c->L * pb));
    HIP_TRY(dev_alloc((void**)&l.extP, items * 4 * std::max(c->K, 1) * pb));
    HIP_TRY(dev_alloc((void**)&l.T, items * 3 * NP * pb));
    HIP_TRY(dev_alloc((void**)&l.D, items * std::max(c->G, 1) * c->L * pb));
    HIP_TRY(dev_alloc((void**)&l.D16, items * std::max(c->G, 1) * c->n * sizeof(int16_t)));
    if (c->S32) {
        HIP_TRY(dev_alloc((void**)&l.DS, items * std::max(c->G, 1) * c->S32 * c->n * sizeof(uint32_t)));
        HIP_TRY(dev_alloc((void**)&l.U, items * 2 * c->L * c->S32 * c->n * sizeof(uint32_t)));
    }
    l.items = items;
    return 0;
}

// Points the context's stream and workspace at lane idx (> 0) for the lifetime of the guard.
struct LaneGuard {
    exacto_ctx* c;
    int idx;
    LaneGuard(exacto_ctx* c_, int idx_) : c(c_), idx(idx_) { if (idx > 0) flip(); }
    ~LaneGuard() { if (idx > 0) flip(); }
    void flip() {
        LaneSet& l = c->xl[idx - 1];
        std::swap(c->stream, l.stream);
        std::swap(c->ws_coefQ, l.coefQ); std::swap(c->ws_extP, l.extP);
        std::swap(c->ws_T, l.T); std::swap(c->ws_D, l.D); std::swap(c->ws_D16, l.D16);
        std::swap(c->ws_DS, l.DS); std::swap(c->ws_U, l.U);
    }
};

// Lanes for a pass of nchunks chunks of C items: extra lanes forked off c->stream (their
// streams wait for everything enqueued so far); LaneJoin makes c->stream wait for them again.
static int fork_lanes(exacto_ctx* c, long nchunks, size_t C, int* nl) {
    *nl = (c->dual && !c->prof) ? (int)std::min<long>(c->lanes, nchunks) : 1;
    if (*nl <= 1) return 0;
    for (int i = 1; i < *nl; ++i)
        if (int e = ensure_lane(c, i, C)) return e;
    HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
    for (int i = 1; i < *nl; ++i) HIP_TRY(hipStreamWaitEvent(c->xl[i - 1].stream, c->ev_fork, 0));
    return 0;
}

struct LaneJoin {
    exacto_ctx* c;
    int nl;
    ~LaneJoin() {
        for (int i = 1; i < nl; ++i)
            if (hipEventRecord(c->xl[i - 1].join, c->xl[i - 1].stream) == hipSuccess)
                (void)hipStreamWaitEvent(c->stream, c->xl[i - 1].join, 0);
    }
};

static int ensure_rlk_companions(exacto_ctx* c) {
    if (c->rlk_s_valid) return 0;
    const size_t count = c->rlk_keys * 2 * c->L * (size_t)c->n;
    if (grow(&c->d_rlk_s, &c->rlk_s_cap, std::max<size_t>(count * sizeof(u64), 8))) return EXACTO_ERR_HIP;
    launch_shoup_companions(c->d_rlk, c->d_rlk_s, (long)count, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    c->rlk_s_valid = true;
    return 0;
}

// CRT kernel variant: 3 special-prime reductions, 2 lazy (fast), 1 near primes, 0 generic
static int crt_mode(const exacto_ctx* c) {
    return c->h_crt.special ? 3 : c->h_crt.fast ? 2 : c->h_crt.near ? 1 : 0;
}

// A key [keys][2][L][n] (NTT domain mod q_l) in ks32's auxiliary basis: INTT mod q_l
// (coefficient domain), balanced, reduced mod each p_s, forward NTT mod p_s -> dst [keys][2L][S][n]
// (grown as needed).
static int ks32_convert_key(exacto_ctx* c, const u64* key, size_t keys, uint32_t** dst, size_t* cap, int S = 0,
                            const Prime32* p32 = nullptr, int form = 0) {
    if (!S) { S = c->S32; p32 = c->d_p32; form = c->ks32_mac_form; }
    const long rows = (long)keys * 2 * c->L;
    if (grow((u64**)dst, cap, std::max<size_t>((size_t)rows * S * c->n * sizeof(uint32_t), 8)))
        return EXACTO_ERR_HIP;
    Scratch ks;
    HIP_TRY(ks.alloc((size_t)rows * c->n * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    NttBatch nb{};
    nb.src = key; nb.src_item_stride = 2L * c->L * c->n;
    nb.dst = ks.as<u64>(); nb.dst_item_stride = 2L * c->L * c->n;
    nb.ppi = 2 * c->L; nb.prime_base = 0; nb.period = c->L;
    if (int e = run_ntt(c, nb, rows, true)) return e;
    ks32_key(ks.as<u64>(), *dst, rows, c->L, S, c->logn, p32, c->d_primes, form, c->stream);
    CHECK_LAUNCH();
    return 0;
}

#ifndef EXACTO_KN_NORM
#define EXACTO_KN_NORM 1   // the narrow basis' digit-sum limit from the key's norms too (A/B build switch)
#endif
// The primary basis for the resident key: the lazy one (kz) when the key's own norms bound the key
// switch, |u_{c,l}| <= (B/2) sum_g ||r_{g,c,l}||_1 with ||r||_1 <= (sum floor(|r_j|/2^20) + n) 2^20
// (ks32_key_norm_kernel), for every (c, l): prod p > 2 m bound for m = 1 (and sum_max = the largest
// such m <= 64 for dBFV digit sums); otherwise the narrow one (kn), whose bound holds for any key.
static int ks32_select_basis(exacto_ctx* c) {
    use_ks32_basis(c, c->kn);
    if (c->kz.S == 0 || c->rlk_keys == 0) return 0;
    const long rows = (long)c->rlk_keys * 2 * c->L, CL = 2L * c->L;
    Scratch ks, nr;
    HIP_TRY(ks.alloc((size_t)rows * c->n * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    HIP_TRY(nr.alloc((size_t)rows * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    NttBatch nb{};
    nb.src = c->d_rlk; nb.src_item_stride = CL * c->n;
    nb.dst = ks.as<u64>(); nb.dst_item_stride = CL * c->n;
    nb.ppi = (int)CL; nb.prime_base = 0; nb.period = c->L;
    if (int e = run_ntt(c, nb, rows, true)) return e;
    ks32_key_norms(ks.as<u64>(), nr.as<u64>(), rows, c->L, c->n, c->d_primes, c->stream);
    CHECK_LAUNCH();
    std::vector<u64> h((size_t)rows);
    HIP_TRY(hipMemcpyAsync(h.data(), nr.as<u64>(), h.size() * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    Big worst(0);
    for (long cl = 0; cl < CL; ++cl) {
        Big acc(0);
        for (size_t g = 0; g < c->rlk_keys; ++g) {
            Big t(h[(size_t)g * CL + cl] + (u64)c->n);
            t.mul(1ull << 20);
            acc.add(t);
        }
        if (acc.cmp(worst) > 0) worst = acc;
    }
    worst.mul(c->gbase / 2);
    // sums the lazy / the narrow basis lift for this key (its norms, not the analytic bound), by the
    // Garner and by the float-CRT lift
    const int sm = sums_lifted(c->kz.P, worst, false);
    const int snm = EXACTO_KN_NORM ? sums_lifted(c->kn.P, worst, false) : 0;
    const int fsm = sums_lifted(c->kz.P, worst, true);   // lazy and narrow primes: any S (ks32_crt)
    const int fsnm = EXACTO_KN_NORM && (c->kn.S <= 3 || c->kn.mac_form != 0) ? sums_lifted(c->kn.P, worst, true) : 0;
    // the narrow basis with the key's own bound: cfg4's two-product digit sums (2^90.6) fit its 2^91.2,
    // which the analytic bound (2^91.6) refused -- they then take the narrow form instead of the wide one
    c->ks32_sum_max = std::max(c->kn.sum_max, snm);
    c->ks32_fpc_max = std::max(c->kn.fpc_max, fsnm);
    const int kn_sum = c->ks32_sum_max;
    // never a basis that lifts fewer sums than the narrow one where those sums are needed (a dBFV digit
    // sum the lazy basis cannot hold would otherwise drop to the per-product key switch)
    if (sm >= 1 && sm >= std::min(kn_sum, std::max(1, c->ks32_need_m))) {
        c->kz.sum_max = sm;
        c->kz.fpc_max = fsm;
        use_ks32_basis(c, c->kz);
    }
    return 0;
}

// The resident relinearisation key in ks32's basis (d_rs), the basis chosen for it first.  Once per key.
static int ensure_rs(exacto_ctx* c) {
    if (c->rs_valid) return 0;
    if (int e = ks32_select_basis(c)) return e;
    size_t cap = c->rs_cap;
    const int e = ks32_convert_key(c, c->d_rlk, c->rlk_keys, &c->d_rs, &cap);
    c->rs_cap = cap;
    if (e) return e;
    c->rs_valid = true;
    return 0;
}

// ... and in the wide basis (dBFV digit sums), on first use after each key load
static int ensure_rs_wide(exacto_ctx* c) {
    if (c->kw.rs_valid) return 0;
    size_t cap = c->kw.rs_cap;
    const int e = ks32_convert_key(c, c->d_rlk, c->rlk_keys, &c->kw.d_rs, &cap, c->kw.S, c->kw.d_p32, c->kw.mac_form);
    c->kw.rs_cap = cap;
    if (e) return e;
    c->kw.rs_valid = true;
    return 0;
}

// ============================================================== multiplication pipeline

// products [0, P): ct1 = op.a + off_a(p), ct2 = op.b + off_b(p) (each [2][L][n], NTT domain).
// relin: out[p] = [2][L][n] = relinearize(mul_no_relin); else out[p] = [3][L][n].
// coef (optional): when the key switch runs over the integers (ks32), the last forward NTT is left
// to the caller and *coef is set: out then holds the coefficient domain (a caller that first sums
// products, as dbfv_mul does, transforms the sums instead of every product).
static int run_mul(exacto_ctx* c, const Operands& op, long P, u64* out, long out_stride, bool relin,
                   bool* coef = nullptr) {
    if (coef) *coef = false;
    if (c->deferred_code) return fail(c->deferred_code, c->deferred_msg);
    if (relin && !c->rlk_loaded) return fail(EXACTO_ERR_MISSING_KEY, "key not available: relinearization key not loaded");
    if (P <= 0) return 0;
    const int n = c->n, L = c->L, K = c->K;
    const long Ln = (long)L * n;
    const int guse = relin ? (int)std::min<size_t>(c->G, c->rlk_keys) : 0;
    const exacto_ctx::PsumPlan& ps = c->psum;
    // psum: chunks hold whole dBFV items (their products are summed inside the chunk)
    size_t C = ps.on ? std::max<size_t>(ps.npairs, std::min<size_t>(c->chunk, (size_t)P) / ps.npairs * ps.npairs)
                     : std::min<size_t>(c->chunk, (size_t)P);
    // a batch that fits one chunk still takes two lanes when each half has work enough (>= 64
    // products): the halves fill each other's launch tails (cfg5, 288 products per dbfv_mul: 1837 ->
    // 1889 chains/s with two chunks of 144; four chunks of 72 measured 1800)
    if (c->dual && !c->prof && c->lanes > 1 && (size_t)P <= C && P >= 128) {
        size_t half = ((size_t)P + 1) / 2;
        if (ps.on) half = (half + ps.npairs - 1) / ps.npairs * ps.npairs;
        if (half < (size_t)P) C = half;
    }
    if (int e = ensure_workspace(c, C)) return e;
    // int16 gadget digits (base <= 2^16, exact path): the scale kernel writes each digit once
    const bool d16 = relin && guse > 0 && c->digit16 && c->path != EXACTO_PATH_HPS &&
                     c->gbase <= 65536;
    // ... and then the key switch runs over the integers in the 31-bit basis (ks32.hip)
    const bool k32 = d16 && c->ks32 && c->S32 > 0;
    // HPS in dbfv_mul (dbfv_mul_group): the scale writes each product's signed digits to ks_defer,
    // c0 / c1 stay in the coefficient domain; the caller sums both per output limb, then transforms
    // and relinearises once per limb
    const bool hps_defer = c->path == EXACTO_PATH_HPS && relin && guse > 0 && c->ks_defer && coef;
    const bool skip_fwd = coef && (k32 || hps_defer);
    if (skip_fwd) *coef = true;
    if (relin && guse > 0) {
        // both before the second lane forks: its kernels read these too
        // (a deferred key switch -- dbfv_mul_core's digit sums -- has already made the key for the basis
        // it uses, which may be the wide one: the primary form would be built and never read)
        if (int e = k32 ? (c->ks_defer ? 0 : ensure_rs(c)) : ensure_rlk_companions(c)) return e;
    }
    // two chunks or more: odd chunks on the second lane (profiling keeps one lane so its per-kernel
    // events time each kernel alone)
    int nl = 1;
    if (int e = fork_lanes(c, (P + (long)C - 1) / (long)C, C, &nl)) return e;
    LaneJoin join{c, nl};
    for (long s = 0; s < P; s += (long)C) {
        const int cnt = (int)std::min<long>((long)C, P - s);
        LaneGuard lane(c, (int)((s / (long)C) % nl));
        Operands o = op;
        if (o.a_off) o.a_off += s; else o.a += s * o.a_stride;
        if (o.b_off) o.b_off += s; else o.b += s * o.b_stride;
        if (!o.ea) {
            // 1. inputs -> coefficient domain (INTT), coefQ[item] = [c0, c1, d0, d1][L][n]
            NttBatch nb{};
            nb.src = o.a; nb.src_off = o.a_off; nb.src_item_stride = o.a_stride;
            nb.dst = c->ws_coefQ; nb.dst_item_stride = 4 * Ln;
            nb.ppi = 2 * L; nb.prime_base = 0; nb.period = L;
            if (int e = run_ntt(c, nb, (long)cnt * 2 * L, true)) return e;
            nb.src = o.b; nb.src_off = o.b_off; nb.src_item_stride = o.b_stride;
            nb.dst = c->ws_coefQ + 2 * Ln;
            if (int e = run_ntt(c, nb, (long)cnt * 2 * L, true)) return e;
            // 2. extension to the auxiliary primes
            if (c->path == EXACTO_PATH_HPS) {
                // per input poly: the q residues in, K auxiliary residues out
                ProfScope pl(c, PK_HPS_EXT, 4ull * cnt, 8.0 * (1 + K) * n * 4.0 * cnt);
                launch_hps_extend(c->ws_coefQ, c->ws_extP, 4L * cnt, n, c->d_primes, K, c->stream);
            } else {
                ProfScope pl(c, PK_LIFT, 4ull * cnt, 8.0 * (L + K) * n * 4.0 * cnt);
                launch_exact_lift(c->ws_coefQ, c->ws_extP, 4L * cnt, n, c->d_crt, c->d_primes, L, K,
                                  crt_mode(c), c->stream);
            }
            CHECK_LAUNCH();
            // 3. forward NTT of the extended polynomials (exact path with the asm tensor, its only
            // reader: outputs left in [0, 2q), which its products take)
            NttBatch eb = contiguous(c->ws_extP, cnt, 4L * K, L, K, n);
            eb.lazy_out = c->path != EXACTO_PATH_HPS && tensor_asm(c);
            if (int e = run_ntt(c, eb, (long)cnt * 4 * K, false)) return e;
        } else {
            o.ea_off += s;
            o.eb_off += s;
        }
        // 4+5. tensor product in every prime, fused into the inverse NTT of its components
        if (int e = run_inv_tensor(c, o, cnt, ps.on)) return e;
        if (ps.on) {
            // the output limbs' c0 / c1 auxiliary residues, summed over their products, then inverse-
            // transformed: [ib][k][c][a][n] in extP (unused: the extensions are shared, steps 1-3 skipped)
            const int ib_cnt = cnt / ps.npairs;
            {   // per (item, prime): the 2d input ciphertexts' two polys in, 2 sums per output limb out
                ProfScope pp(c, PK_PAIRSUM, (u64)ib_cnt * K * ps.d, 8.0 * n * K * ib_cnt * (4.0 * ps.d + 2.0 * ps.d));
                launch_dbfv_pairsum(o, c->ws_extP, ib_cnt, ps.d, ps.npairs, ps.term_start, ps.terms, L, K, n,
                                    c->d_primes, c->stream);
            }
            CHECK_LAUNCH();
            if (int e = run_ntt(c, contiguous(c->ws_extP, (long)ib_cnt * ps.d, 2L * K, L, K, n),
                                (long)ib_cnt * ps.d * 2 * K, true))
                return e;
        }
        // 6. scale-and-round (+ gadget digits of the third component)
        u64* R = out + s * out_stride;
        const int ncomp = relin ? 2 : 3;
        u64* D = relin ? c->ws_D : nullptr;
        // scale bytes per item: the three components' L+K residues in; c0, c1 (L residues each) out
        // (psum: c2 only), and the third component's digits (int16 / int8) or its L residues
        const double dig_b = (d16 || hps_defer) ? (c->ks_defer && c->ks_defer8 ? 1.0 : 2.0) * guse
                                                : 8.0 * L * (relin ? guse : 1);
        {   // (scoped: the events bracket the scale launch alone)
        ProfScope psc(c, c->path == EXACTO_PATH_HPS ? PK_HPS_SCALE : PK_SCALE, (u64)cnt, (double)n * cnt *
                      ((ps.on ? 1.0 : 3.0) * 8.0 * (L + K) + (ps.on ? 0.0 : 16.0 * L) + (relin ? dig_b : 8.0 * L)));
        if (c->path == EXACTO_PATH_HPS) {
            void* d16p = hps_defer ? (c->ks_defer8 ? (void*)((int8_t*)c->ks_defer + s * (long)guse * n)
                                                   : (void*)(c->ks_defer + s * (long)guse * n))
                                   : nullptr;
            launch_hps_scale(c->ws_T, R, out_stride, ncomp, hps_defer ? nullptr : D, d16p,
                             hps_defer && c->ks_defer8, guse, cnt, n, c->d_crt, c->d_primes, K, c->hps_fast,
                             c->stream);
        } else
            launch_exact_scale(c->ws_T, R, out_stride, ncomp, d16 ? nullptr : D,
                               d16 ? (c->ks_defer ? (c->ks_defer8
                                                         ? (int16_t*)((int8_t*)c->ks_defer + s * (long)guse * n)
                                                         : c->ks_defer + s * (long)guse * n)
                                                  : c->ws_D16)
                                   : nullptr,
                               guse, cnt, n, c->d_crt, c->d_primes, L, K, crt_mode(c),
                               c->stream, c->h_crt.gshift, ps.on, c->ks_defer && c->ks_defer8, c->fp_crt, c->fpq_lim);
        CHECK_LAUNCH();
        }
        if (ps.on) {   // ... and their scale: the output limbs' c0 / c1, coefficient domain
            const long item0 = s / ps.npairs;
            const double ib = (double)(cnt / ps.npairs);
            // per item: each limb's summed auxiliary residues (K) and its products' ciphertext-prime
            // residues (L each) in, the limb's L residues out, for c0 and c1
            ProfScope pq(c, PK_PSUM_SCALE, (u64)(cnt / ps.npairs) * ps.d,
                         ib * 2.0 * n * 8.0 * (ps.d * (double)(K + L) + (double)ps.npairs * L));
            if (!launch_psum_scale(c->ws_T, c->ws_extP, ps.out + item0 * ps.d * 2 * Ln, cnt / ps.npairs, ps.d, ps.npairs,
                                   ps.term_start, ps.terms, n, c->d_crt, c->d_primes, L, c->stream, ps.fpc,
                                   c->fpq_lim))
                return fail(EXACTO_ERR_HIP, "internal: psum scale not available for these limbs");
            CHECK_LAUNCH();
        }
        // 7. forward NTT of the results (and digits)
        NttBatch rb{};
        rb.src = R; rb.src_off = nullptr; rb.src_item_stride = out_stride;
        rb.dst = R; rb.dst_item_stride = out_stride;
        rb.ppi = ncomp * L; rb.prime_base = 0; rb.period = L;
        if (k32) {
            // 7'+8'. the key switch over the integers (ks32.hip): digits -> NTT mod p_s, MAC with the
            // key in the same basis, inverse NTT + centred lift, added to R mod q_l in the
            // coefficient domain; the forward NTT of R below then yields the relinearised result
            if (!c->ks_defer) {   // (deferred: the caller sums the digits of products first, dbfv_mul_core)
                {   // int16 digit in (2 B), 31-bit residue out (4 B) per coefficient and prime
                    ProfScope pd(c, PK_KS_DIGITS, (u64)cnt * guse * c->S32, 6.0 * n * cnt * guse * c->S32);
                    ks32_digits(c->ws_D16, c->ws_DS, cnt, guse, c->S32, c->logn, c->d_p32, c->ks32_mac_form, c->stream);
                }
                {   // per (item, prime, coefficient): G digit residues in, 2L sums out (the key slice from LDS)
                    ProfScope pm(c, PK_KS_MAC, (u64)cnt * c->S32, 4.0 * n * cnt * c->S32 * (guse + 2.0 * L));
                    ks32_mac(c->ws_DS, c->d_rs, c->ws_U, cnt, guse, L, c->S32, n, c->d_p32, c->ks32_mac_form, c->stream);
                }
                {   // per (item, component, limb): S 31-bit sums in, R in and out
                    ProfScope pc(c, PK_KS_CRT, (u64)cnt * 2 * L, (double)n * cnt * 2 * L * (4.0 * c->S32 + 16.0));
                    ks32_crt(c->ws_U, R, out_stride, cnt, L, c->S32, c->logn, c->d_kst, c->d_p32, c->d_primes, c->ks32_mac_form,
                             c->stream, c->ks_fpc && c->ks32_fpc_max >= 1);
                }
                CHECK_LAUNCH();
            }
        }
        if (skip_fwd) continue;   // (hps_defer: digits and c0 / c1 are the caller's now)
        if (int e = run_ntt(c, rb, (long)cnt * ncomp * L, false)) return e;
        if (relin && guse > 0 && !k32) {
            NttBatch db = contiguous(c->ws_D, cnt, (long)guse * L, 0, L, n);
            if (d16) {  // int16 digits [item][g][n] -> NTT residues [item][g][L][n]
                db.src16 = c->ws_D16;
                db.src16_item_stride = (long)guse * n;
            }
            if (int e = run_ntt(c, db, (long)cnt * guse * L, false)) return e;
            // 8. relinearisation MAC, in place on the output
            if (int e = ensure_rlk_companions(c)) return e;
            {   // per item: c0, c1 and the G digit residues in, c0, c1 out (the key from LDS)
                ProfScope pm(c, PK_RELIN_MAC, (u64)cnt, 8.0 * n * L * cnt * (4.0 + guse));
                launch_relin_mac(R, out_stride, c->ws_D, c->d_rlk, c->d_rlk_s, guse, R, out_stride, cnt, n, L,
                                 c->d_primes, c->stream);
            }
            CHECK_LAUNCH();
        }
    }
    return 0;
}

// ============================================================== C ABI: NTT / RNS

static int check_ctx(exacto_ctx* c) {
    if (!c) return invalid_param("null context");
    HIP_TRY(hipSetDevice(c->device));
    return 0;
}

static int ntt_dev(exacto_ctx* c, uint64_t* polys, size_t count, size_t limb, bool inverse) {
    if (int e = check_ctx(c)) return e;
    if (limb >= (size_t)c->L)
        // the reference's Display text ("expected {expected}, got {got}", error.rs:8-9): the context's
        // limb count and the limb index asked for
        return fail(EXACTO_ERR_DIMENSION_MISMATCH, "dimension mismatch: expected " + std::to_string(c->L) + ", got " +
                                                       std::to_string(limb));
    return run_ntt(c, contiguous(polys, count, 1, (int)limb, 1, c->n), (long)count, inverse);
}

extern "C" int exacto_ntt_fwd_dev(exacto_ctx* c, uint64_t* p, size_t count, size_t limb) { return ntt_dev(c, p, count, limb, false); }
extern "C" int exacto_ntt_inv_dev(exacto_ctx* c, uint64_t* p, size_t count, size_t limb) { return ntt_dev(c, p, count, limb, true); }

extern "C" int exacto_rns_fwd_dev(exacto_ctx* c, uint64_t* p, size_t count) {
    if (int e = check_ctx(c)) return e;
    return run_ntt(c, contiguous(p, count, c->L, 0, c->L, c->n), (long)count * c->L, false);
}
extern "C" int exacto_rns_inv_dev(exacto_ctx* c, uint64_t* p, size_t count) {
    if (int e = check_ctx(c)) return e;
    return run_ntt(c, contiguous(p, count, c->L, 0, c->L, c->n), (long)count * c->L, true);
}

static int stage(exacto_ctx* c, size_t bytes) {
    if (grow(&c->io, &c->io_bytes, bytes)) return EXACTO_ERR_HIP;
    return 0;
}

static int ntt_host(exacto_ctx* c, uint64_t* polys, size_t count, size_t limb, bool inverse) {
    if (int e = check_ctx(c)) return e;
    const size_t bytes = count * poly_bytes(c);
    if (int e = stage(c, std::max<size_t>(bytes, 8))) return e;
    if (int e_ = upload(c, c->io, polys, bytes)) return e_;
    if (int e = ntt_dev(c, c->io, count, limb, inverse)) return e;
    HIP_TRY(hipMemcpyAsync(polys, c->io, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}
extern "C" int exacto_ntt_fwd(exacto_ctx* c, uint64_t* p, size_t count, size_t limb) { return ntt_host(c, p, count, limb, false); }
extern "C" int exacto_ntt_inv(exacto_ctx* c, uint64_t* p, size_t count, size_t limb) { return ntt_host(c, p, count, limb, true); }

static int pw(exacto_ctx* c, PwOp op, const u64* a, const u64* b, u64* out, long polys, const u64* scal) {
    if (int e = check_ctx(c)) return e;
    launch_pointwise(op, a, b, out, polys, c->n, c->L, scal, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_rns_add_dev(exacto_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* o, size_t n) {
    return pw(c, PwOp::Add, a, b, o, (long)n * (c ? c->L : 0), nullptr);
}
extern "C" int exacto_rns_sub_dev(exacto_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* o, size_t n) {
    return pw(c, PwOp::Sub, a, b, o, (long)n * (c ? c->L : 0), nullptr);
}
extern "C" int exacto_rns_neg_dev(exacto_ctx* c, const uint64_t* a, uint64_t* o, size_t n) {
    return pw(c, PwOp::Neg, a, nullptr, o, (long)n * (c ? c->L : 0), nullptr);
}
extern "C" int exacto_rns_mul_dev(exacto_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* o, size_t n) {
    return pw(c, PwOp::Mul, a, b, o, (long)n * (c ? c->L : 0), nullptr);
}
// INTT(a (.) b): RnsPoly::mul then to_coeff_poly per limb, fused (one pass instead of a
// pointwise pass and an inverse transform); [count][L][n], out may alias a or b.
extern "C" int exacto_rns_mul_inv_dev(exacto_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* o, size_t count) {
    if (int e = check_ctx(c)) return e;
    if (count == 0) return 0;
    if (!a || !b || !o) return invalid_param("null buffer");
    bool lazy = true, near60 = c->ntt_asm && c->ntt_asm_inv;
    for (int t = 0; t < c->L; ++t) {
        lazy &= c->ctq[t] < (1ull << 60);
        near60 &= c->ctq[t] < (1ull << 60) && c->ctq[t] > (1ull << 60) - (1ull << 24);
    }
    launch_mul_inv(a, b, o, (long)count * c->L, c->L, c->logn, lazy, near60, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}
// Negacyclic products of coefficient-domain RnsPolys: to_coeff_poly(from_coeff_poly(a) (.)
// from_coeff_poly(b)) per limb (ntt.rs:181-195 composed).  n = 4096 / 8192 with special primes:
// one fused kernel; otherwise the forward transforms into scratch and the fused product + inverse.
// [count][L][n]; out may alias a or b.
extern "C" int exacto_rns_polymul_dev(exacto_ctx* c, const uint64_t* a, const uint64_t* b, uint64_t* o, size_t count) {
    if (int e = check_ctx(c)) return e;
    if (count == 0) return 0;
    if (!a || !b || !o) return invalid_param("null buffer");
    bool near60 = c->ntt_asm && c->ntt_asm_inv, lazy = true;
    for (int t = 0; t < c->L; ++t) {
        lazy &= c->ctq[t] < (1ull << 60);
        near60 &= c->ctq[t] < (1ull << 60) && c->ctq[t] > (1ull << 60) - (1ull << 24);
    }
    const long rows = (long)count * c->L;
    if (near60 && (c->logn == 12 || c->logn == 13)) {
        // fused product: 3 transforms, algorithmic bytes a + b in, product out
        ProfScope pp(c, PK_POLYMUL, (u64)rows, 24.0 * c->n * (double)rows);
        launch_polymul(a, b, o, rows, c->L, c->logn, c->d_primes, c->stream);
        CHECK_LAUNCH();
        return 0;
    }
    Scratch sa, sb;
    HIP_TRY(sa.alloc((size_t)rows * poly_bytes(c), c->stream, c->pool, c->debug_scratch));
    HIP_TRY(sb.alloc((size_t)rows * poly_bytes(c), c->stream, c->pool, c->debug_scratch));
    NttBatch nb = contiguous(sa.as<u64>(), count, c->L, 0, c->L, c->n);
    nb.src = a;
    if (int e = run_ntt(c, nb, rows, false)) return e;
    nb = contiguous(sb.as<u64>(), count, c->L, 0, c->L, c->n);
    nb.src = b;
    if (int e = run_ntt(c, nb, rows, false)) return e;
    launch_mul_inv(sa.as<u64>(), sb.as<u64>(), o, rows, c->L, c->logn, lazy, false, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_rns_scalar_mul_dev(exacto_ctx* c, const uint64_t* a, uint64_t scalar, uint64_t* o, size_t n) {
    if (int e = check_ctx(c)) return e;
    // s = scalar % q_i per limb (ntt.rs:136); tiny synchronous upload into the context's table
    u64 sm[EXACTO_MAX_L];
    for (int i = 0; i < c->L; ++i) sm[i] = scalar % c->ctq[i];
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int e_ = upload(c, c->d_scal, sm, c->L * sizeof(u64))) return e_;
    return pw(c, PwOp::ScalarMul, a, nullptr, o, (long)n * c->L, c->d_scal);
}

// bfv_add / bfv_sub / bfv_neg (eval.rs:14-60), batched: ct1 [B][p1][L][n], ct2 [B][p2][L][n] ->
// out [B][max(p1, p2)][L][n].  Components beyond the shorter operand pass through from the longer
// one, negated when they are ct2's under subtraction (eval.rs:21-22, 41-42).
static int bfv_addsub(exacto_ctx* c, bool sub, const u64* x, size_t p1, const u64* y, size_t p2, u64* o, size_t B) {
    if (int e = check_ctx(c)) return e;
    const size_t pm = std::max(p1, p2);
    if (!B || !pm) return 0;
    if ((p1 && !x) || (p2 && !y) || !o) return invalid_param("null ciphertext pointer");
    // in place only over an operand laid out like the output; any other overlap is rejected
    const size_t pw = (size_t)c->L * c->n;
    auto overlaps = [&](const u64* in, size_t polys) {
        return in && polys && in < o + B * pm * pw && o < in + B * polys * pw;
    };
    if ((overlaps(x, p1) && (o != x || p1 != pm)) || (overlaps(y, p2) && (o != y || p2 != pm)))
        return invalid_param("output may alias an input only when it has as many components as the output");
    launch_bfv_addsub(sub, x, (int)p1, y, (int)p2, o, (long)B, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}
extern "C" int exacto_bfv_add_dev(exacto_ctx* c, const uint64_t* x, size_t p1, const uint64_t* y, size_t p2, uint64_t* o,
                                  size_t B) {
    return bfv_addsub(c, false, x, p1, y, p2, o, B);
}
extern "C" int exacto_bfv_sub_dev(exacto_ctx* c, const uint64_t* x, size_t p1, const uint64_t* y, size_t p2, uint64_t* o,
                                  size_t B) {
    return bfv_addsub(c, true, x, p1, y, p2, o, B);
}
extern "C" int exacto_bfv_neg_dev(exacto_ctx* c, const uint64_t* x, size_t polys, uint64_t* o, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!B || !polys) return 0;
    if (!x || !o) return invalid_param("null ciphertext pointer");
    return pw(c, PwOp::Neg, x, nullptr, o, (long)B * polys * c->L, nullptr);
}

// ============================================================== C ABI: BFV

static Operands plain_operands(const exacto_ctx* c, const u64* a, const u64* b) {
    Operands op{};
    op.a = a; op.a_off = nullptr; op.a_stride = 2L * c->L * c->n;
    op.b = b; op.b_off = nullptr; op.b_stride = 2L * c->L * c->n;
    return op;
}

extern "C" int exacto_bfv_mul_no_relin_dev(exacto_ctx* c, const uint64_t* ct1, size_t polys1,
                                           const uint64_t* ct2, size_t polys2, uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (polys1 != 2 || polys2 != 2) return invalid_param("multiplication requires degree-1 ciphertexts");
    return run_mul(c, plain_operands(c, ct1, ct2), (long)B, out, 3L * c->L * c->n, false);
}

extern "C" int exacto_bfv_mul_and_relin_dev(exacto_ctx* c, const uint64_t* ct1, const uint64_t* ct2,
                                            uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    return run_mul(c, plain_operands(c, ct1, ct2), (long)B, out, 2L * c->L * c->n, true);
}

extern "C" int exacto_relinearize_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    const long Ln = (long)c->L * c->n;
    if (polys < 3) {  // keyswitch.rs:63-65: already degree-1, cloned: out = [B][polys][L][n]
        if (B * polys)
            HIP_TRY(dev_copy(out, ct, B * polys * Ln * sizeof(u64), c->stream));
        return 0;
    }
    if (polys > 3) return invalid_param("relinearization only supports degree-2 ciphertexts");
    if (!c->rlk_loaded) return fail(EXACTO_ERR_MISSING_KEY, "key not available: relinearization key not loaded");
    const int guse = (int)std::min<size_t>(c->G, c->rlk_keys);
    const size_t C = std::min<size_t>(c->chunk, std::max<size_t>(B, 1));
    if (int e = ensure_workspace(c, C)) return e;
    for (size_t s = 0; s < B; s += C) {
        const int cnt = (int)std::min(C, B - s);
        const u64* src = ct + s * 3 * Ln;
        u64* dst = out + s * 2 * Ln;
        // c0, c1 copied, then accumulated in place
        launch_rows(dst, 2 * Ln, src, 3 * Ln, 2 * Ln, cnt, c->stream);
        CHECK_LAUNCH();
        if (guse == 0) continue;
        NttBatch nb{};
        nb.src = src + 2 * Ln; nb.src_off = nullptr; nb.src_item_stride = 3 * Ln;
        nb.dst = c->ws_coefQ; nb.dst_item_stride = Ln;
        nb.ppi = c->L; nb.prime_base = 0; nb.period = c->L;
        if (int e = run_ntt(c, nb, (long)cnt * c->L, true)) return e;
        const bool d16 = c->digit16 && c->gbase <= 65536;  // int16 digits, as in run_mul
        launch_decompose(c->ws_coefQ, Ln, c->ws_D, guse, cnt, c->n, c->d_crt, c->d_primes, c->L, c->stream,
                         d16 ? c->ws_D16 : nullptr);
        CHECK_LAUNCH();
        NttBatch db = contiguous(c->ws_D, cnt, (long)guse * c->L, 0, c->L, c->n);
        if (d16) {
            db.src16 = c->ws_D16;
            db.src16_item_stride = (long)guse * c->n;
        }
        if (int e = run_ntt(c, db, (long)cnt * guse * c->L, false)) return e;
        if (int e = ensure_rlk_companions(c)) return e;
        launch_relin_mac(dst, 2 * Ln, c->ws_D, c->d_rlk, c->d_rlk_s, guse, dst, 2 * Ln, cnt, c->n, c->L,
                         c->d_primes, c->stream);
        CHECK_LAUNCH();
    }
    return 0;
}

extern "C" int exacto_gadget_decompose_dev(exacto_ctx* c, const uint64_t* coeffs, uint64_t* digits, size_t B,
                                           size_t num_digits) {
    if (int e = check_ctx(c)) return e;
    const int guse = (int)std::min<size_t>(c->G, num_digits);
    launch_decompose(coeffs, (long)c->L * c->n, digits, guse, (int)B, c->n, c->d_crt, c->d_primes, c->L, c->stream);
    CHECK_LAUNCH();
    return 0;
}

// host-pointer wrappers: stage inputs in the context's io buffer, run the _dev entry, copy back
static int host_call(exacto_ctx* c, const std::vector<std::pair<const void*, size_t>>& ins, size_t out_bytes,
                     void* host_out, const std::function<int(std::vector<u64*>&, u64*)>& fn) {
    if (int e = check_ctx(c)) return e;
    size_t total = out_bytes;
    for (auto& in : ins) total += (in.second + 255) / 256 * 256;
    if (int e = stage(c, std::max<size_t>(total, 8))) return e;
    std::vector<u64*> dins;
    char* p = (char*)c->io;
    for (auto& in : ins) {
        // stream-ordered on the context stream (see upload)
        if (in.second) HIP_TRY(hipMemcpyAsync(p, in.first, in.second, hipMemcpyHostToDevice, c->stream));
        dins.push_back((u64*)p);
        p += (in.second + 255) / 256 * 256;
    }
    // landed before fn runs: fn may read the inputs on another context's stream (bootstrap)
    HIP_TRY(hipStreamSynchronize(c->stream));
    u64* dout = (u64*)p;
    if (int e = fn(dins, dout)) return e;
    HIP_TRY(hipMemcpyAsync(host_out, dout, out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    static const bool dbg = [] { const char* e = getenv("EXACTO_DEBUG_BOOT"); return e && e[0] == '1'; }();
    if (dbg && host_out && out_bytes >= 8 && out_bytes <= 64 * 8) {   // (the bootstrap diagnostic: what the host received)
        u64 hsh = 1469598103934665603ull;
        const u64* ho = static_cast<const u64*>(host_out);
        for (size_t k = 0; k < out_bytes / 8; ++k) hsh = (hsh ^ ho[k]) * 1099511628211ull;
        std::fprintf(stderr, "boot-dbg host_out       %016llx [%llu %llu %llu %llu]\n", (unsigned long long)hsh,
                     (unsigned long long)ho[0], (unsigned long long)(out_bytes > 8 ? ho[1] : 0),
                     (unsigned long long)(out_bytes > 16 ? ho[2] : 0), (unsigned long long)(out_bytes > 24 ? ho[3] : 0));
    }
    return 0;
}

extern "C" int exacto_bfv_mul_no_relin(exacto_ctx* c, const uint64_t* ct1, size_t p1, const uint64_t* ct2, size_t p2,
                                       uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * 2 * c->L * poly_bytes(c);
    return host_call(c, {{ct1, ctb}, {ct2, ctb}}, B * 3 * c->L * poly_bytes(c), out,
                     [&](std::vector<u64*>& d, u64* o) { return exacto_bfv_mul_no_relin_dev(c, d[0], p1, d[1], p2, o, B); });
}

extern "C" int exacto_bfv_mul_and_relin(exacto_ctx* c, const uint64_t* ct1, const uint64_t* ct2, uint64_t* out,
                                        size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * 2 * c->L * poly_bytes(c);
    return host_call(c, {{ct1, ctb}, {ct2, ctb}}, ctb, out,
                     [&](std::vector<u64*>& d, u64* o) { return exacto_bfv_mul_and_relin_dev(c, d[0], d[1], o, B); });
}

extern "C" int exacto_relinearize(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t inb = B * polys * c->L * poly_bytes(c);
    const size_t outp = polys < 3 ? polys : 2;
    return host_call(c, {{ct, inb}}, B * outp * c->L * poly_bytes(c), out,
                     [&](std::vector<u64*>& d, u64* o) { return exacto_relinearize_dev(c, d[0], polys, o, B); });
}

// ============================================================== C ABI: dBFV

// lattice.rs:104-122 compute_simple + decomposition.rs:8-16 digit_decompose
extern "C" int exacto_bfv_add(exacto_ctx* c, const uint64_t* ct1, size_t p1, const uint64_t* ct2, size_t p2,
                              uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t pb = c->L * poly_bytes(c);
    return host_call(c, {{ct1, B * p1 * pb}, {ct2, B * p2 * pb}}, B * std::max(p1, p2) * pb, out,
                     [&](std::vector<u64*>& in, u64* o) { return exacto_bfv_add_dev(c, in[0], p1, in[1], p2, o, B); });
}
extern "C" int exacto_bfv_sub(exacto_ctx* c, const uint64_t* ct1, size_t p1, const uint64_t* ct2, size_t p2,
                              uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t pb = c->L * poly_bytes(c);
    return host_call(c, {{ct1, B * p1 * pb}, {ct2, B * p2 * pb}}, B * std::max(p1, p2) * pb, out,
                     [&](std::vector<u64*>& in, u64* o) { return exacto_bfv_sub_dev(c, in[0], p1, in[1], p2, o, B); });
}
extern "C" int exacto_bfv_neg(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t bytes = B * polys * c->L * poly_bytes(c);
    return host_call(c, {{ct, bytes}}, bytes, out,
                     [&](std::vector<u64*>& in, u64* o) { return exacto_bfv_neg_dev(c, in[0], polys, o, B); });
}

static std::vector<std::vector<i64>> small_reps(u64 base, size_t d, u64 p) {
    std::vector<std::vector<i64>> reps;
    for (size_t j = d; j + 1 < 2 * d; ++j) {
        u64 val;
        if (p == 0) {
            val = 1;
            for (size_t e = 0; e < j; ++e) val *= base;  // wrapping_pow
        } else {
            val = powmod_h(base, j, p);
        }
        std::vector<i64> dg;
        u64 rem = val;
        for (size_t k = 0; k < d; ++k) { dg.push_back((i64)(rem % base)); rem /= base; }
        reps.push_back(dg);
    }
    return reps;
}

// The product list and combine terms of a dbfv_mul batch (dbfv/eval.rs:109-132 + reduce,
// reduction.rs:34-52) for the output limbs `limbs` (all of 0..d-1, or the subset one GPU computes
// when the limbs of one dbfv_mul are split across GPUs): output slot s = limb limbs[s] gets the sum
// over pairs (i, j) with i + j == limbs[s] plus the reps folding of the high limbs i + j >= d.  Only
// the pairs some listed limb uses are multiplied.
static int dbfv_plan(exacto_ctx* c, size_t B, size_t d, u64 base, u64 plain, const std::vector<int>& limbs) {
    if (c->cached_B == B && c->cached_d == d && c->cached_base == base && c->cached_p == plain && c->d_off &&
        c->cached_limbs == limbs)
        return 0;
    const auto reps = small_reps(base, d, plain);
    const size_t dout = limbs.size();
    auto coef_of = [&](size_t i, size_t j, size_t ko) -> i64 {
        const size_t k = i + j;
        return k == ko ? 1 : k >= d ? reps[k - d][ko] : 0;
    };
    std::vector<std::pair<int, int>> pairs;
    for (size_t i = 0; i < d; ++i)
        for (size_t j = 0; j < d; ++j) {
            bool needed = false;
            for (int ko : limbs) needed |= coef_of(i, j, (size_t)ko) != 0;
            if (needed) pairs.push_back({(int)i, (int)j});
        }
    const int npairs = (int)pairs.size();
    std::vector<int> start(dout + 1, 0);
    std::vector<CombineTerm> terms;
    for (size_t so = 0; so < dout; ++so) {
        start[so] = (int)terms.size();
        for (int pi = 0; pi < npairs; ++pi) {
            const i64 coef = coef_of(pairs[pi].first, pairs[pi].second, (size_t)limbs[so]);
            if (coef != 0) terms.push_back({pi, 0, coef});
        }
    }
    start[dout] = (int)terms.size();
    // ks32 sums before the lift: every combine term a plain sum (zero reps), at most this many per limb
    int sum_m = 0;
    for (const CombineTerm& t : terms) if (t.coef != 1) sum_m = -1;
    for (size_t so = 0; so < dout && sum_m >= 0; ++so) sum_m = std::max(sum_m, start[so + 1] - start[so]);
    const long Ln2 = 2L * c->L * c->n, Kn2 = 2L * c->K * c->n;
    // [0, BP): a offsets, [BP, 2BP): b offsets (ciphertexts), [2BP, 4BP): the same into the
    // per-ciphertext extension buffers
    const size_t BP = B * npairs;
    std::vector<u64> off(4 * BP);
    for (size_t b = 0; b < B; ++b)
        for (int pi = 0; pi < npairs; ++pi) {
            off[b * npairs + pi] = (u64)((b * d + pairs[pi].first) * Ln2);
            off[BP + b * npairs + pi] = (u64)((b * d + pairs[pi].second) * Ln2);
            off[2 * BP + b * npairs + pi] = (u64)((b * d + pairs[pi].first) * Kn2);
            off[3 * BP + b * npairs + pi] = (u64)((b * d + pairs[pi].second) * Kn2);
        }
    size_t cap = c->off_cap;
    if (grow(&c->d_off, &cap, off.size() * sizeof(u64) + 8)) return EXACTO_ERR_HIP;
    c->off_cap = cap;
    if (int e_ = upload(c, c->d_off, off.data(), off.size() * sizeof(u64))) return e_;
    free_dev(c->d_term_start);
    free_dev(c->d_terms);
    HIP_TRY(dev_alloc((void**)&c->d_term_start, start.size() * sizeof(int)));
    if (int e_ = upload(c, c->d_term_start, start.data(), start.size() * sizeof(int))) return e_;
    HIP_TRY(dev_alloc((void**)&c->d_terms, std::max<size_t>(terms.size(), 1) * sizeof(CombineTerm)));
    if (!terms.empty())
        if (int e_ = upload(c, c->d_terms, terms.data(), terms.size() * sizeof(CombineTerm))) return e_;
    c->cached_B = B; c->cached_d = d; c->cached_base = base; c->cached_p = plain;
    c->cached_npairs = npairs;
    c->cached_limbs = limbs;
    c->cached_sum_m = sum_m;
    return 0;
}

// DbfvParams::new checks (params/mod.rs:168-184)
static int dbfv_params_check(size_t d, uint64_t base, uint64_t plain) {
    if (base < 2) return invalid_param("base must be >= 2");
    if (d < 1) return invalid_param("num_digits must be >= 1");
    u128 bd = 1;
    const u128 sat = ~(u128)0;
    for (size_t i = 0; i < d; ++i) bd = (bd > sat / base) ? sat : bd * base;
    const u128 p128 = plain == 0 ? ((u128)1 << 64) : (u128)plain;
    if (bd < p128) {
        auto u128s = [](u128 v) { std::string s; do { s.insert(s.begin(), char('0' + (int)(v % 10))); v /= 10; } while (v); return s; };
        return invalid_param("base^digits = " + u128s(bd) + " < plain_modulus = " + u128s(p128));
    }
    return 0;
}

// Every input ciphertext of a dBFV product batch enters d products (dbfv/eval.rs:109-122): its
// inverse NTT, its exact (or HPS) extension to the auxiliary primes and their forward NTT
// (pipeline steps 1-3) are computed here once per ciphertext, ext = [ct][2][K][n], instead of
// once per product.  The results are identical: steps 1-3 depend on the ciphertext alone.
// coef: the same ciphertexts already in the coefficient domain (a dBFV chain's previous step,
// [ct][2][L][n]), or nullptr: the inverse NTT is skipped and the lift reads them directly.
static int extend_cts(exacto_ctx* c, const u64* cts, size_t ncts, u64* ext, const u64* coef = nullptr) {
    const int n = c->n, L = c->L, K = c->K;
    const long Ln2 = 2L * L * n, Kn2 = 2L * K * n;
    if (int e = ensure_workspace(c, std::min<size_t>(c->chunk, (ncts + 1) / 2))) return e;
    const size_t G = coef ? ncts : 2 * c->ws_items;  // ciphertexts per pass: coefQ holds 4 polys x L per item
    for (size_t g0 = 0; g0 < ncts; g0 += G) {
        const long cnt = (long)std::min(G, ncts - g0);
        const u64* cq = coef ? coef + g0 * Ln2 : c->ws_coefQ;
        if (!coef) {
            NttBatch nb{};
            nb.src = cts + g0 * Ln2; nb.src_off = nullptr; nb.src_item_stride = Ln2;
            nb.dst = c->ws_coefQ; nb.dst_item_stride = Ln2;
            nb.ppi = 2 * L; nb.prime_base = 0; nb.period = L;
            if (int e = run_ntt(c, nb, cnt * 2 * L, true)) return e;
        }
        u64* eo = ext + g0 * Kn2;
        if (c->path == EXACTO_PATH_HPS) {
            ProfScope pl(c, PK_HPS_EXT, 2ull * cnt, 8.0 * (1 + K) * n * 2.0 * cnt);
            launch_hps_extend(cq, eo, 2 * cnt, n, c->d_primes, K, c->stream);
        } else {
            ProfScope pl(c, PK_LIFT, 2ull * cnt, 8.0 * (L + K) * n * 2.0 * cnt);
            launch_exact_lift(cq, eo, 2 * cnt, n, c->d_crt, c->d_primes, L, K,
                              crt_mode(c), c->stream);
        }
        CHECK_LAUNCH();
        if (int e = run_ntt(c, contiguous(eo, cnt, 2L * K, L, K, n), cnt * 2 * K, false)) return e;
    }
    return 0;
}

// b_extended: c->ext_b already holds the extensions of b (a chain's constant right operand)
// out = [B][dout][2][L][n] for the output limbs `limbs` (dout = limbs.size()), one group of items
static int dbfv_mul_group(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                          const uint64_t* b, uint64_t* out, size_t B, bool b_extended,
                          const std::vector<int>* limbs) {
    const size_t dout = limbs->size();
    if (int e = dbfv_plan(c, B, d, base, plain, *limbs)) return e;
    const int npairs = c->cached_npairs;
    const long Ln2 = 2L * c->L * c->n;
    const long P = (long)B * npairs;
    size_t cap = c->prod_bytes;
    if (grow(&c->prod, &cap, (size_t)P * Ln2 * sizeof(u64))) return EXACTO_ERR_HIP;
    c->prod_bytes = cap;
    Operands op{};
    const size_t BP = (size_t)B * npairs;
    op.a = a; op.a_off = c->d_off; op.a_stride = 0;
    op.b = b; op.b_off = c->d_off + BP; op.b_stride = 0;
    if (c->share_ext && c->K > 0 && !c->deferred_code) {
        const size_t nct = B * d, bytes = nct * 2 * c->K * poly_bytes(c);
        if (c->ext_a_ready) {   // made by the previous chain step (same ciphertexts, same buffer size)
            if (c->ext_a_cap < bytes) return fail(EXACTO_ERR_HIP, "internal: pre-extended operand buffer too small");
        } else {
            if (grow(&c->ext_a, &c->ext_a_cap, bytes)) return EXACTO_ERR_HIP;
            if (int e = extend_cts(c, a, nct, c->ext_a, c->coef_in)) return e;
        }
        c->ext_a_ready = false;
        if (!b_extended) {
            if (grow(&c->ext_b, &c->ext_b_cap, bytes)) return EXACTO_ERR_HIP;
            if (int e = extend_cts(c, b, nct, c->ext_b)) return e;
        }
        op.ea = c->ext_a; op.ea_off = c->d_off + 2 * BP;
        op.eb = c->ext_b; op.eb_off = c->d_off + 3 * BP;
    }
    // the per-limb sums (dbfv/eval.rs:124-132) and the degree reduction are linear, so with ks32 they
    // run on the products' coefficient-domain results and only the d output limbs are transformed
    // (B d 2L forward NTTs instead of B npairs 2L)
    // ... and when the 31-bit basis holds the sum of a limb's key switches, the key switch is
    // linear in the digits, so the products' int16 digits are summed per output limb (still int16)
    // and transformed, multiplied with the key and lifted once per limb instead of once per product
    // (cfg5: 8 instead of 36 products' worth of digit NTTs, MACs and lifts per dbfv_mul)
    // The primary 31-bit basis when it holds the sums, else the wide one (primes up to 2^31).
    const size_t gu = std::min<size_t>(c->G, c->rlk_keys);
    const int m = c->cached_sum_m;
    // the primary basis (narrow or lazy) and its sum_max depend on the resident key: decide first
    if (m > c->ks32_need_m) {
        c->ks32_need_m = m;
        // a key already on the lazy basis that cannot lift these sums while the narrow one can: re-select
        if (c->rs_valid && c->ks32_lazy_active && m > c->ks32_sum_max) c->rs_valid = false;
    }
    if (c->S32 > 0 && c->ks32 && c->rlk_loaded && gu > 0)
        if (int e = ensure_rs(c)) return e;
    const bool on = c->S32 > 0 && c->ks32 && m > 0 && c->digit16 && c->gbase <= 65536 &&
                    c->rlk_loaded && gu > 0;
    const bool use_prim = on && m <= c->ks32_sum_max;
    const bool use_wide = on && !use_prim && c->kw.S > 0 && m <= c->kw.sum_max;
    const bool sum_ks = use_prim || use_wide;
    c->last_dbfv_ks = use_prim ? 1 : use_wide ? 2 : 0;
    const int S = use_wide ? c->kw.S : c->S32;
    const Prime32* p32 = use_wide ? c->kw.d_p32 : c->d_p32;
    const Ks32Tables* kst = use_wide ? c->kw.d_kst : c->d_kst;
    const int mac_form = use_wide ? c->kw.mac_form : c->ks32_mac_form;
    const bool wide = (u64)m * (c->gbase / 2) > 32767;   // digit sums beyond int16
    const size_t Bd = B * dout, Sn = (size_t)S * c->n;
    // HPS (u64_dbfv): with the products' c0 / c1 kept in the coefficient domain, relinearize is linear
    // mod q in the gadget digits and so are the per-limb sums and the NTT: limb k = NTT(sum c0) +
    // sum_g NTT(sum_p d_pg) (.) rlk_g.  The scale writes every product's signed digits (int8 when the
    // base is at most 2^8), ks32_digit_sum adds them per output limb as int16 (|sum| <= m B / 2), and
    // the forward NTTs and the MAC run once per output limb instead of once per product (u64_dbfv:
    // 8 instead of 36 products' worth of 10 forward NTTs and one MAC per dbfv_mul).
    const bool hps_sum = c->path == EXACTO_PATH_HPS && c->hps_sum_env && m > 0 && c->gbase <= 65536 &&
                         (u64)m * (c->gbase / 2) <= 32767 && c->rlk_loaded && gu > 0 && c->n >= 1024 &&
                         !c->deferred_code;
    if (hps_sum) {
        if (grow((u64**)&c->d_dall, &c->dall_cap, std::max<size_t>((size_t)P * gu * c->n * sizeof(int16_t), 8)) ||
            grow((u64**)&c->d_dk, &c->dk_cap, std::max<size_t>(Bd * gu * c->n * 2, 8)) ||
            grow(&c->d_hdig, &c->hdig_cap, std::max<size_t>(Bd * gu * c->L * c->n * sizeof(u64), 8)))
            return EXACTO_ERR_HIP;
        if (int e = ensure_rlk_companions(c)) return e;
        c->ks_defer = c->d_dall;
        c->ks_defer8 = c->digit8_env && c->gbase <= 256;
    }
    if (sum_ks) {
        if (grow((u64**)&c->d_dall, &c->dall_cap, std::max<size_t>((size_t)P * gu * c->n * sizeof(int16_t), 8)) ||
            grow((u64**)&c->d_dk, &c->dk_cap, std::max<size_t>(Bd * gu * c->n * (wide ? 4 : 2), 8)) ||
            grow((u64**)&c->d_dsk, &c->dsk_cap, std::max<size_t>(Bd * gu * Sn * sizeof(uint32_t), 8)) ||
            grow((u64**)&c->d_uk, &c->uk_cap, std::max<size_t>(Bd * 2 * c->L * Sn * sizeof(uint32_t), 8)))
            return EXACTO_ERR_HIP;
        if (int e = use_wide ? ensure_rs_wide(c) : ensure_rs(c)) return e;
        c->ks_defer = c->d_dall;
        // base <= 2^8: every balanced digit fits int8 (half the digit bytes written and summed)
        const int sh = c->h_crt.gshift;
        c->ks_defer8 = c->digit8_env && sh > 0 && sh <= 8 && 32 % sh == 0 &&
                       exact_scale_sp_ok(c->L, c->K, crt_mode(c));
    }
    // psum: each output limb's c0 / c1 from one scale of its products' summed tensors (the
    // auxiliary-prime residues summed in the NTT domain and inverse-transformed once per limb, the
    // per-product corrections from the ciphertext-prime residues; exact_psum_sp_kernel), written
    // straight to out: no per-product c0 / c1 and no dbfv_combine pass.  Needs the summed digits
    // (so the third component is per product only for its digits), shared extensions, special
    // primes with K = L + 1 (30-bit-limb scale) and the asm tensor kernels.
    bool near60 = c->ntt_asm && c->ntt_asm_inv;
    for (u64 q : c->primes) near60 &= q < (1ull << 60) && q > (1ull << 60) - (1ull << 24);
    const bool psum = sum_ks && c->psum_env && m <= c->psum_max && op.ea != nullptr && near60 &&
                      (c->logn == 12 || c->logn == 13) && exact_scale_sp_ok(c->L, c->K, crt_mode(c));
    // chain (psum): the limbs are formed in the coefficient domain in coef_out and forward-transformed
    // from there into out, so coef_out keeps them for the next step's extension.  The buffer is grown
    // only here, where psum is known to be on (HPS or non-psum chains never allocate it).
    c->coef_out = nullptr;
    if (psum && c->coef_slot >= 0) {
        size_t ccap = c->chain_coef_bytes;
        if (grow(&c->chain_coef, &ccap, 2 * c->coef_slot_words * sizeof(u64))) return EXACTO_ERR_HIP;
        c->chain_coef_bytes = ccap;
        c->coef_out = c->chain_coef + (size_t)c->coef_slot * c->coef_slot_words;
    }
    u64* cf = psum && c->coef_out ? c->coef_out : out;
    c->coef_written = false;
    if (psum) {
        c->psum.on = true;
        c->psum.d = (int)dout;
        c->psum.npairs = npairs;
        c->psum.term_start = c->d_term_start;
        c->psum.terms = c->d_terms;
        c->psum.out = cf;
        c->psum.fpc = c->fp_crt && m <= c->psum_fp_max;
    }
    bool coef = false;
    if (op.ea) {
        c->tensor_share_d = (int)d;
        c->tensor_share_npairs = npairs;
    }
    const int rc = run_mul(c, op, P, c->prod, Ln2, true, &coef);
    c->tensor_share_d = c->tensor_share_npairs = 0;
    c->ks_defer = nullptr;
    const bool in8 = c->ks_defer8;
    c->ks_defer8 = false;
    c->psum.on = false;
    if (rc) return rc;
    if ((sum_ks || hps_sum) && !coef) return fail(EXACTO_ERR_HIP, "internal: digit sums without a deferred key switch");
    if (!psum) {
        ProfScope pk(c, PK_COMBINE, (u64)B * dout, 8.0 * c->n * B * 2 * c->L * (double)(npairs + dout));
        launch_dbfv_combine(c->prod, npairs, c->d_term_start, c->d_terms, out, (int)B, (int)dout, c->n, c->L,
                            c->d_primes, c->stream);
        CHECK_LAUNCH();
    }
    if (sum_ks) {
        const double nn = c->n, ds = wide ? 4.0 : 2.0;
        {   // every product's digits in (1 or 2 B), one sum per (limb, digit) out
            ProfScope pd(c, PK_DIGIT_SUM, (u64)Bd, nn * gu * ((double)B * npairs * (in8 ? 1.0 : 2.0) + (double)Bd * ds));
            ks32_digit_sum(c->d_dall, in8, npairs, c->d_term_start, c->d_terms, c->d_dk, wide, (int)B, (int)dout, (int)gu,
                           c->n, c->stream);
        }
        {
            ProfScope pn(c, PK_KS_DIGITS, (u64)Bd * gu * S, nn * Bd * gu * S * (ds + 4.0));
            if (wide) ks32_digits32((const int32_t*)c->d_dk, c->d_dsk, (int)Bd, (int)gu, S, c->logn, p32, mac_form, c->stream);
            else ks32_digits((const int16_t*)c->d_dk, c->d_dsk, (int)Bd, (int)gu, S, c->logn, p32, mac_form, c->stream);
        }
        {
            ProfScope pm(c, PK_KS_MAC, (u64)Bd * S, 4.0 * nn * Bd * S * (gu + 2.0 * c->L));
            ks32_mac(c->d_dsk, use_wide ? c->kw.d_rs : c->d_rs, c->d_uk, (int)Bd, (int)gu, c->L, S, c->n, p32,
                     mac_form, c->stream);
        }
        {
            ProfScope pc(c, PK_KS_CRT, (u64)Bd * 2 * c->L, nn * Bd * 2 * c->L * (4.0 * S + 16.0));
            const bool fpc = c->ks_fpc && m <= (use_wide ? c->kw.fpc_max : c->ks32_fpc_max);
            ks32_crt(c->d_uk, cf, 2L * c->L * c->n, (int)Bd, c->L, S, c->logn, kst, p32, c->d_primes, mac_form, c->stream,
                     fpc);
        }
        CHECK_LAUNCH();
    }
    if (hps_sum) {
        const double nn = c->n;
        {   // every product's digits in (1 or 2 B), one int16 sum per (limb, digit) out
            ProfScope pd(c, PK_DIGIT_SUM, (u64)Bd, nn * gu * ((double)B * npairs * (in8 ? 1.0 : 2.0) + 2.0 * Bd));
            ks32_digit_sum(c->d_dall, in8, npairs, c->d_term_start, c->d_terms, c->d_dk, false, (int)B, (int)dout,
                           (int)gu, c->n, c->stream);
        }
        CHECK_LAUNCH();
        NttBatch db = contiguous(c->d_hdig, (long)Bd, (long)gu * c->L, 0, c->L, c->n);
        db.src16 = (const int16_t*)c->d_dk;
        db.src16_item_stride = (long)gu * c->n;
        if (int e = run_ntt(c, db, (long)Bd * gu * c->L, false)) return e;
    }
    if (coef) {
        NttBatch ob = contiguous(out, (long)B * dout, 2L * c->L, 0, c->L, c->n);
        ob.src = cf;   // (== out unless a chain keeps the coefficient form)
        // a chain step whose limbs stay in the coefficient domain (cf) for the next step: that step's
        // extension of its left operand (exact lift of cf to the auxiliary primes, then their forward
        // transform: extend_cts with coef = cf) is made here, and the two forward batches go in one
        // launch (cfg5: 512 + 640 polynomials instead of two launches that each fill about one
        // generation of the 512 resident workgroups)
        const bool pre = cf != out && op.ea != nullptr && dout == d && !c->deferred_code &&
                         c->path != EXACTO_PATH_HPS && c->ext_a_cap >= (size_t)B * d * 2 * c->K * poly_bytes(c);
        if (pre) {
            const long cts = (long)B * d;
            {
                ProfScope pl(c, PK_LIFT, 2ull * cts, 8.0 * (c->L + c->K) * c->n * 2.0 * cts);
                launch_exact_lift(cf, c->ext_a, 2 * cts, c->n, c->d_crt, c->d_primes, c->L, c->K, crt_mode(c),
                                  c->stream);
                CHECK_LAUNCH();
            }
            const NttBatch eb = contiguous(c->ext_a, cts, 2L * c->K, c->L, c->K, c->n);
            if (int e = run_ntt_fwd2(c, ob, cts * 2 * c->L, eb, cts * 2 * c->K)) return e;
            c->ext_a_ready = true;
        } else {
            if (int e = run_ntt(c, ob, (long)B * dout * 2 * c->L, false)) return e;
        }
        c->coef_written = cf != out;
    }
    if (hps_sum) {
        ProfScope pm(c, PK_RELIN_MAC, (u64)Bd, 8.0 * c->n * c->L * Bd * (4.0 + gu));
        launch_relin_mac(out, 2L * c->L * c->n, c->d_hdig, c->d_rlk, c->d_rlk_s, (int)gu, out, 2L * c->L * c->n,
                         (int)Bd, c->n, c->L, c->d_primes, c->stream);
        CHECK_LAUNCH();
    }
    return 0;
}

// Every buffer of a dbfv_mul pass grows with its item count (the products' results and digits, their
// per-limb digit sums and 31-bit residues, the shared extensions: per_item below, 4.4 MB at cfg4 and
// 113 MB at cfg5), so a batch runs in groups of whole items whose buffers stay within
// EXACTO_DBFV_GROUP_MB (default 16 GiB of the 288 GB HBM: the BASELINE batches, 4.5 GB at cfg4 and
// 0.9 GB at cfg5, are one group -- a 4 GiB default split cfg4's 1024 items into 932 + 92 and cost 5 %).
// Items are independent: the groups give the same results as one pass.  out = [B][dout][2][L][n] for
// the output limbs `limbs` (nullptr: all d).
static int dbfv_mul_core(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                         const uint64_t* b, uint64_t* out, size_t B, bool b_extended,
                         const std::vector<int>* limbs = nullptr) {
    std::vector<int> all;
    if (!limbs) {
        for (size_t k = 0; k < d; ++k) all.push_back((int)k);
        limbs = &all;
    }
    const size_t dout = limbs->size();
    const size_t budget = c->dbfv_group_bytes;
    const size_t n = c->n, L = c->L, K = c->K, G = c->G, S = std::max(c->S32, c->kw.S);
    const size_t per_item = 8 * n * (d * d * 2 * L + 2 * d * 2 * K) +       // products, both extensions
                            n * G * (d * d * 2 + d * (4 + 4 * S)) +         // digits, sums, residues
                            4 * n * d * 2 * L * S;                          // key-switch sums
    const size_t Bg = std::max<size_t>(1, budget / std::max<size_t>(per_item, 1));
    if (B <= Bg) return dbfv_mul_group(c, d, base, plain, a, b, out, B, b_extended, limbs);
    // several groups: no coefficient-form carry between chain steps (its buffers are whole-batch)
    c->coef_in = nullptr;
    c->coef_slot = -1;
    const size_t ctw = 2 * L * n;
    for (size_t g0 = 0; g0 < B; g0 += Bg) {
        const size_t cnt = std::min(Bg, B - g0);
        // b's extensions are per group here (a chain recomputes them for each group)
        if (int e = dbfv_mul_group(c, d, base, plain, a + g0 * d * ctw, b + g0 * d * ctw, out + g0 * dout * ctw, cnt,
                                   false, limbs))
            return e;
    }
    return 0;
}

static int ensure_twin(exacto_ctx* c, int i);

// A batch of independent items in `parts` near-equal parts on the context and its twins (each on its own
// stream, overlapping), or whole on the context: f(ctx, first item, items) per part.  The context's
// stream waits for every twin's part.  Parts measured: a depth-4 cfg5 chain batch 2 /
// 3 / 4 parts 2558 / 2575 / 2586 chains/s; dbfv_mul batches: cfg4 188.7k / 187.0k / 186.7k/s,
// u64_dbfv 57.5k / 56.2k / 55.1k/s -- so four parts for chains, two for single dbfv_mul batches.
template <class F>
static int split_run(exacto_ctx* c, size_t B, int want, F f) {
    const int parts = c->batch_split ? (int)std::min<size_t>(B, (size_t)std::min(want, exacto_ctx::MAX_TWINS + 1)) : 1;
    if (parts < 2 || !c->dual || c->prof || !c->rlk_loaded || c->deferred_code) return f(c, 0, B);
    const size_t per = (B + parts - 1) / parts;
    int rc = 0;
    for (int i = 1; i < parts; ++i) {
        const size_t i0 = per * i;
        if (i0 >= B) break;
        if (int e = ensure_twin(c, i - 1)) return e;
        const int r = f(c->twin[i - 1], i0, std::min(per, B - i0));
        if (!rc) rc = r;
    }
    const int r0 = f(c, 0, std::min(per, B));
    for (int i = 1; i < parts && per * i < B; ++i) {
        HIP_TRY(hipEventRecord(c->ev_twin_out[i - 1], c->twin[i - 1]->stream));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_twin_out[i - 1], 0));
    }
    return r0 ? r0 : rc;   // (the last error message is the failing call's)
}

extern "C" int exacto_dbfv_mul_dev(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                                   const uint64_t* b, uint64_t* out, size_t B, const uint32_t* depth_a,
                                   const uint32_t* depth_b, uint32_t* depth_out) {
    if (int e = check_ctx(c)) return e;
    if (int e = dbfv_params_check(d, base, plain)) return e;
    // depth guard (dbfv/eval.rs:96-102)
    for (size_t i = 0; i < B; ++i) {
        const uint32_t da = depth_a ? depth_a[i] : 0, db = depth_b ? depth_b[i] : 0;
        if (std::max(da, db) + 1 > 1)
            return fail(EXACTO_ERR_NOT_IMPLEMENTED, "not yet implemented: chained dBFV multiplication requires "
                                                    "ciphertext-level lattice reduction (paper §4.6.2)");
    }
    if (B == 0) return 0;
    const size_t w = d * 2 * c->L * (size_t)c->n;
    if (int e = split_run(c, B, 2, [&](exacto_ctx* x, size_t i0, size_t cnt) {
            return dbfv_mul_core(x, d, base, plain, a + i0 * w, b + i0 * w, out + i0 * w, cnt, false);
        }))
        return e;
    if (depth_out)
        for (size_t i = 0; i < B; ++i) depth_out[i] = 1;
    return 0;
}

// One GPU's share of a dbfv_mul whose output limbs are split across GPUs (dbfv/eval.rs:109-132): the
// output limbs limbs[0..nlimbs) only, out = [B][nlimbs][2][L][n] (slot s = limb limbs[s]), each exactly
// as exacto_dbfv_mul computes it (its pairs i + j = k, relinearised and summed, and the reduce
// folding of the high limbs).  Distinct limbs need no cross-GPU sum: the caller gathers the slots.
extern "C" int exacto_dbfv_mul_limbs_dev(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                                         const uint64_t* b, uint64_t* out, size_t B, const uint32_t* limbs,
                                         size_t nlimbs) {
    if (int e = check_ctx(c)) return e;
    if (int e = dbfv_params_check(d, base, plain)) return e;
    if (nlimbs && !limbs) return invalid_param("null limb list");
    std::vector<int> ls;
    for (size_t s = 0; s < nlimbs; ++s) {
        if (limbs[s] >= d) return invalid_param("output limb " + std::to_string(limbs[s]) + " >= d = " + std::to_string(d));
        if (std::find(ls.begin(), ls.end(), (int)limbs[s]) != ls.end()) return invalid_param("repeated output limb");
        ls.push_back((int)limbs[s]);
    }
    if (B == 0 || ls.empty()) return 0;
    return dbfv_mul_core(c, d, base, plain, a, b, out, B, false, &ls);
}

extern "C" int exacto_dbfv_mul_limbs(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                                     const uint64_t* b, uint64_t* out, size_t B, const uint32_t* limbs, size_t nlimbs) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * d * 2 * c->L * poly_bytes(c);
    return host_call(c, {{a, ctb}, {b, ctb}}, B * nlimbs * 2 * c->L * poly_bytes(c), out,
                     [&](std::vector<u64*>& in, u64* o) {
                         return exacto_dbfv_mul_limbs_dev(c, d, base, plain, in[0], in[1], o, B, limbs, nlimbs);
                     });
}

// ============================================================== decryption

// bfv/encrypt.rs:111-178 for a batch: phase = sum_k c_k s^k (NTT domain), INTT, exact rounding.
// ct = [B][polys][L][n] (stride ct_stride words per ciphertext), sk = [L][n] NTT domain.
static int decrypt_batch(exacto_ctx* c, const u64* ct, size_t polys, long ct_stride, const u64* sk, u64* out,
                         size_t B) {
    if (polys < 1) return invalid_param("ciphertext has no polynomials");
    if (B == 0) return 0;
    const int L = c->L, n = c->n;
    if (L >= 2 && (c->K < 1 || c->plain >= c->primes[L]))
        return fail(EXACTO_ERR_NOT_IMPLEMENTED, "not yet implemented: GPU decryption needs plain_modulus below the "
                                                "first internal auxiliary prime");
    size_t cap = c->dec_bytes;
    if (grow(&c->dec_buf, &cap, B * L * poly_bytes(c))) return EXACTO_ERR_HIP;
    c->dec_bytes = cap;
    launch_phase(ct, (int)polys, ct_stride, sk, c->dec_buf, (int)B, n, L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = run_ntt(c, contiguous(c->dec_buf, (long)B, L, 0, L, n), (long)B * L, true)) return e;
    launch_decrypt_round(c->dec_buf, out, (int)B, n, L, c->d_crt, c->d_primes, c->plain, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_bfv_decrypt_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* sk,
                                      uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    return decrypt_batch(c, ct, polys, (long)polys * c->L * c->n, sk, out, B);
}

extern "C" int exacto_bfv_decrypt(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* sk,
                                  uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{ct, B * polys * c->L * poly_bytes(c)}, {sk, c->L * poly_bytes(c)}}, B * poly_bytes(c), out,
                     [&](std::vector<u64*>& dv, u64* o) { return exacto_bfv_decrypt_dev(c, dv[0], polys, dv[1], o, B); });
}

// dbfv/decrypt.rs:20-79: every limb decrypted with the BFV plaintext modulus t, then signed
// recomposition mod p coefficient-wise (poly) or of coefficient 0 (scalar).
static int dbfv_decrypt_common(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* ct,
                               const uint64_t* sk, uint64_t* out, size_t B, bool scalar) {
    if (int e = check_ctx(c)) return e;
    if (int e = dbfv_params_check(d, base, plain)) return e;
    if (!scalar && plain == 0)
        return invalid_param("polynomial dBFV decrypt requires finite plain_modulus (plain_modulus=0 is scalar-only)");
    if (B == 0) return 0;
    const size_t nd = B * d;
    size_t cap = c->dig_bytes;
    if (grow(&c->dig_buf, &cap, nd * poly_bytes(c))) return EXACTO_ERR_HIP;
    c->dig_bytes = cap;
    if (int e = decrypt_batch(c, ct, 2, 2L * c->L * c->n, sk, c->dig_buf, nd)) return e;
    launch_dbfv_recompose(c->dig_buf, out, (int)B, c->n, (int)d, base, plain, c->plain, scalar, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_dbfv_decrypt_dev(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* ct,
                                       const uint64_t* sk, uint64_t* out, size_t B) {
    return dbfv_decrypt_common(c, d, base, plain, ct, sk, out, B, true);
}

extern "C" int exacto_dbfv_decrypt_poly_dev(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain,
                                            const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t B) {
    return dbfv_decrypt_common(c, d, base, plain, ct, sk, out, B, false);
}

extern "C" int exacto_dbfv_decrypt(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* ct,
                                   const uint64_t* sk, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{ct, B * d * 2 * c->L * poly_bytes(c)}, {sk, c->L * poly_bytes(c)}}, B * sizeof(u64), out,
                     [&](std::vector<u64*>& dv, u64* o) {
                         return exacto_dbfv_decrypt_dev(c, d, base, plain, dv[0], dv[1], o, B);
                     });
}

extern "C" int exacto_dbfv_decrypt_poly(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain,
                                        const uint64_t* ct, const uint64_t* sk, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{ct, B * d * 2 * c->L * poly_bytes(c)}, {sk, c->L * poly_bytes(c)}}, B * poly_bytes(c), out,
                     [&](std::vector<u64*>& dv, u64* o) {
                         return exacto_dbfv_decrypt_poly_dev(c, d, base, plain, dv[0], dv[1], o, B);
                     });
}

// dBFV multiplication chain with the guard-bypass semantics of paper_repro.rs:203-236 (and the
// chain of bfv_host.rs:258-288 without its bootstrap): acc <- dbfv_mul(acc, y) `depth` times,
// both mul_depth reset to 0 before every step; intermediates ping-pong between two
// context-owned device buffers and never leave HBM.
// The twin of a context (its second chain stream): created on first use with the same parameters
// and chunking, its own stream, workspaces and scratch; the relinearisation key is copied from the
// context whenever it changed since (rlk_version), ordered after everything on the context's stream.
static int ensure_twin(exacto_ctx* c, int i) {
    if (!c->twin[i]) {
        exacto_ctx* t = nullptr;
        if (int e = exacto_ctx_create(&t, c->n, c->ctq.data(), c->L, c->user_aux.empty() ? nullptr : c->user_aux.data(),
                                      c->user_aux.size(), c->plain, c->gbase, c->device))
            return e;
        t->batch_split = false;
        c->twin[i] = t;
        if (!c->ev_twin_in) HIP_TRY(hipEventCreateWithFlags(&c->ev_twin_in, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_twin_out[i], hipEventDisableTiming));
    }
    exacto_ctx* t = c->twin[i];
    t->chunk = c->chunk;
    HIP_TRY(hipEventRecord(c->ev_twin_in, c->stream));
    HIP_TRY(hipStreamWaitEvent(t->stream, c->ev_twin_in, 0));
    if (c->twin_rlk_version[i] != c->rlk_version) {
        if (int e = exacto_ctx_load_relin_key_dev(t, c->d_rlk, c->rlk_keys)) return e;
        c->twin_rlk_version[i] = c->rlk_version;
    }
    return 0;
}

static int dbfv_chain_one(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* x,
                          const uint64_t* y, uint64_t* out, size_t B, size_t depth);

extern "C" int exacto_dbfv_mul_chain_dev(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain,
                                         const uint64_t* x, const uint64_t* y, uint64_t* out, size_t B,
                                         size_t depth) {
    if (int e = check_ctx(c)) return e;
    // two halves on two streams: items are independent, so each half's chain is the chain of those
    // items (bit-identical: tests/test_gpu_chain.py against EXACTO_CHAIN_SPLIT=0)
    if (depth >= 1)
        if (int e = dbfv_params_check(d, base, plain)) return e;
    const size_t w = d * 2 * c->L * (size_t)c->n;
    if (depth == 0) return dbfv_chain_one(c, d, base, plain, x, y, out, B, depth);
    return split_run(c, B, 4, [&](exacto_ctx* t, size_t i0, size_t cnt) {
        return dbfv_chain_one(t, d, base, plain, x + i0 * w, y + i0 * w, out + i0 * w, cnt, depth);
    });
}

static int dbfv_chain_one(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* x,
                          const uint64_t* y, uint64_t* out, size_t B, size_t depth) {
    const size_t bytes = B * d * 2 * c->L * poly_bytes(c);
    if (depth == 0) {
        if (B && out != x) HIP_TRY(dev_copy(out, x, bytes, c->stream));
        return 0;
    }
    if (depth > 1 && B) {
        size_t cap = c->chain_bytes;
        if (grow(&c->chain_buf, &cap, 2 * bytes)) return EXACTO_ERR_HIP;
        c->chain_bytes = cap;
    }
    if (int e = dbfv_params_check(d, base, plain)) return e;
    if (B == 0) return 0;
    // the coefficient form of each step's result (psum path, one item group) goes to chain_coef, and
    // the next step lifts it directly: one batched inverse NTT of its input less per step
    // (dbfv_mul_group allocates chain_coef, two halves of `bytes`, only when the step runs psum)
    const bool carry = depth > 1 && c->share_ext && c->K > 0;
    c->ext_a_ready = false;
    const uint64_t* src = x;
    const u64* src_coef = nullptr;
    int rc = 0;
    for (size_t k = 0; k < depth && rc == 0; ++k) {
        uint64_t* dst = (k + 1 == depth) ? out : c->chain_buf + (k % 2) * (bytes / sizeof(u64));
        c->coef_in = src_coef;
        c->coef_slot = carry && k + 1 < depth ? (int)(k % 2) : -1;
        c->coef_slot_words = bytes / sizeof(u64);
        c->coef_out = nullptr;
        c->coef_written = false;
        // y's extensions are computed by the first step and reused by the others
        rc = dbfv_mul_core(c, d, base, plain, src, y, dst, B, k > 0);
        src_coef = c->coef_out && c->coef_written ? c->coef_out : nullptr;
        src = dst;
    }
    c->coef_in = nullptr;
    c->coef_out = nullptr;
    c->coef_slot = -1;
    c->coef_written = false;
    c->ext_a_ready = false;
    return rc;
}

extern "C" int exacto_dbfv_mul_chain(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* x,
                                     const uint64_t* y, uint64_t* out, size_t B, size_t depth) {
    if (!c) return invalid_param("null context");
    const size_t bytes = B * d * 2 * c->L * poly_bytes(c);
    return host_call(c, {{x, bytes}, {y, bytes}}, bytes, out, [&](std::vector<u64*>& dv, u64* o) {
        return exacto_dbfv_mul_chain_dev(c, d, base, plain, dv[0], dv[1], o, B, depth);
    });
}

extern "C" int exacto_dbfv_mul(exacto_ctx* c, size_t d, uint64_t base, uint64_t plain, const uint64_t* a,
                               const uint64_t* b, uint64_t* out, size_t B, const uint32_t* depth_a,
                               const uint32_t* depth_b, uint32_t* depth_out) {
    if (!c) return invalid_param("null context");
    const size_t bytes = B * d * 2 * c->L * poly_bytes(c);
    return host_call(c, {{a, bytes}, {b, bytes}}, bytes, out, [&](std::vector<u64*>& dv, u64* o) {
        return exacto_dbfv_mul_dev(c, d, base, plain, dv[0], dv[1], o, B, depth_a, depth_b, depth_out);
    });
}

// ============================================================== keygen / encryption

// Gaussian CDT of sampling/gaussian.rs:18-33 (unnormalised cumulative weights over
// [-ceil(6 sigma), ceil(6 sigma)]), cached on the device per sigma.
static int gaussian_table(exacto_ctx* c, double sigma, int* tail, int* len, double* total) {
    if (!(sigma > 0.0) || sigma > 1e6) return invalid_param("sigma must be positive");
    const int t = (int)std::ceil(6.0 * sigma);
    std::vector<double> cdf;
    double cum = 0.0;
    const double two_s2 = 2.0 * sigma * sigma;
    for (long x = -t; x <= t; ++x) {
        cum += std::exp(-(double)(x * x) / two_s2);
        cdf.push_back(cum);
    }
    if (c->cdt_sigma != sigma || !c->d_cdt) {
        size_t cap = c->cdt_cap;
        if (grow((u64**)&c->d_cdt, &cap, cdf.size() * sizeof(double))) return EXACTO_ERR_HIP;
        c->cdt_cap = cap;
        HIP_TRY(hipStreamSynchronize(c->stream));  // in-flight samplers may still read the old table
        if (int e_ = upload(c, c->d_cdt, cdf.data(), cdf.size() * sizeof(double))) return e_;
        c->cdt_sigma = sigma;
    }
    *tail = t;
    *len = (int)cdf.size();
    *total = cum;
    return 0;
}

static ChaChaKey chacha_key(const uint64_t* key) {
    ChaChaKey k{};
    for (int i = 0; i < 4; ++i) k.w[i] = key ? key[i] : 0;
    return k;
}

// Sample `polys` polynomials ([L][n] residues each, at out + p * stride) with indices base + p * step.
static int sample_polys(exacto_ctx* c, int kind, const ChaChaKey& key, u64 stream, u64* out, long stride, u64 base,
                        u64 step, long polys, double sigma) {
    int tail = 0, len = 0;
    double total = 0.0;
    if (kind == KG_GAUSSIAN)
        if (int e = gaussian_table(c, sigma, &tail, &len, &total)) return e;
    launch_sample(kind, key, stream, out, stride, base, step, polys, c->n, c->L, c->d_primes, c->d_cdt, len, tail,
                  total, c->stream);
    CHECK_LAUNCH();
    return 0;
}

// Forward NTT of `items` groups of `polys_per_item` [L][n] blocks spaced `stride` words apart.
static int ntt_items(exacto_ctx* c, u64* data, long items, long stride, long polys_per_item) {
    NttBatch nb{};
    nb.src = data; nb.src_item_stride = stride;
    nb.dst = data; nb.dst_item_stride = stride;
    nb.ppi = (int)polys_per_item; nb.prime_base = 0; nb.period = c->L;
    return run_ntt(c, nb, items * polys_per_item, false);
}

extern "C" int exacto_gen_secret_key_dev(exacto_ctx* c, const uint64_t* key, uint64_t stream, uint64_t* sk) {
    if (int e = check_ctx(c)) return e;
    if (!key || !sk) return invalid_param("null argument");
    // keygen.rs:69-79: ternary s mod q0 -> RnsPoly::from_coeff_poly
    if (int e = sample_polys(c, KG_TERNARY, chacha_key(key), stream, sk, 0, 0, 1, 1, 0.0)) return e;
    return ntt_items(c, sk, 1, 0, c->L);
}

extern "C" int exacto_gen_public_key_dev(exacto_ctx* c, const uint64_t* sk, double sigma, const uint64_t* key,
                                         uint64_t stream, uint64_t* pk) {
    if (int e = check_ctx(c)) return e;
    if (!key || !sk || !pk) return invalid_param("null argument");
    const long Ln = (long)c->L * c->n;
    const ChaChaKey k = chacha_key(key);
    // keygen.rs:90-110: a (-> pk1), e (-> pk0 slot), pk0 = -(a s + e)
    if (int e = sample_polys(c, KG_UNIFORM, k, stream, pk + Ln, 0, 0, 1, 1, sigma)) return e;
    if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, pk, 0, 1, 1, 1, sigma)) return e;
    if (int e = ntt_items(c, pk, 1, 0, 2L * c->L)) return e;
    launch_combine(KG_PK, pk, 1, 0, Ln, sk, nullptr, nullptr, nullptr, nullptr, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_gen_relin_key_dev(exacto_ctx* c, const uint64_t* sk, double sigma, const uint64_t* key,
                                        uint64_t stream, size_t num_keys, uint64_t* rlk) {
    if (int e = check_ctx(c)) return e;
    if (!key || !sk) return invalid_param("null argument");
    const long Ln = (long)c->L * c->n;
    const bool resident = rlk == nullptr;
    if (resident) {  // generate straight into the context's resident key (no host build, no upload)
        rlk = exacto_ctx_relin_key_buffer(c, num_keys);
        if (!rlk && num_keys) return fail(EXACTO_ERR_HIP, "HIP error: relinearization key allocation failed");
    }
    if (num_keys == 0) return 0;
    // g_i = base^i mod q_l (keygen.rs:133-158: gadget_s_sq scaled by base after every key)
    std::vector<u64> gpow(num_keys * c->L);
    for (int l = 0; l < c->L; ++l) {
        const u64 q = c->primes[l];
        u64 g = 1 % q;
        const u64 b = c->gbase % q;
        for (size_t i = 0; i < num_keys; ++i) {
            gpow[i * c->L + l] = g;
            g = (u64)((u128)g * b % q);
        }
    }
    size_t cap = c->gpow_cap;
    if (grow(&c->d_gpow, &cap, gpow.size() * sizeof(u64))) return EXACTO_ERR_HIP;
    c->gpow_cap = cap;
    // the table is host-pageable and d_gpow may still be read by a previous call's kernels
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int e_ = upload(c, c->d_gpow, gpow.data(), gpow.size() * sizeof(u64))) return e_;
    const ChaChaKey k = chacha_key(key);
    // key i: a_i (index 2i) into the rlk1 slot, e_i (index 2i+1) into the rlk0 slot
    if (int e = sample_polys(c, KG_UNIFORM, k, stream, rlk + Ln, 2 * Ln, 0, 2, (long)num_keys, sigma)) return e;
    if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, rlk, 2 * Ln, 1, 2, (long)num_keys, sigma)) return e;
    if (int e = ntt_items(c, rlk, (long)num_keys, 2 * Ln, 2L * c->L)) return e;
    launch_combine(KG_RLK, rlk, (long)num_keys, 2 * Ln, Ln, sk, nullptr, nullptr, nullptr, c->d_gpow, c->n, c->L,
                   c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (resident) {
        HIP_TRY(hipStreamSynchronize(c->stream));  // the key must be complete before it is marked loaded
        c->rlk_keys = num_keys;
        c->rlk_loaded = true;
        c->rlk_s_valid = false;
        c->rs_valid = false; c->kw.rs_valid = false;
        ++c->rlk_version;
    }
    return 0;
}

// Delta_i = floor(Q / p) mod q_i (encrypt.rs:205-229), device copy in c->d_delta.
static int delta_residues(exacto_ctx* c) {
    if (c->delta_ok) return 0;
    // Q as little-endian 64-bit words, then floor(Q / p) by long division, then mod each q_i
    std::vector<u64> Qw(1, 1);
    for (int i = 0; i < c->L; ++i) {
        u128 carry = 0;
        for (auto& w : Qw) {
            const u128 t = (u128)w * c->primes[i] + carry;
            w = (u64)t;
            carry = t >> 64;
        }
        if (carry) Qw.push_back((u64)carry);
    }
    std::vector<u64> D(Qw.size());
    u128 rem = 0;
    for (size_t w = Qw.size(); w-- > 0;) {
        const u128 cur = (rem << 64) | Qw[w];
        D[w] = (u64)(cur / c->plain);
        rem = cur % c->plain;
    }
    bool zero = true;
    for (u64 w : D) zero &= (w == 0);
    if (zero) return invalid_param("ciphertext modulus product Q must be >= plaintext modulus p");
    std::vector<u64> dr(c->L);
    for (int i = 0; i < c->L; ++i) {
        u128 r = 0;
        for (size_t w = D.size(); w-- > 0;) r = ((r << 64) | D[w]) % c->primes[i];
        dr[i] = (u64)r;
    }
    if (!c->d_delta) HIP_TRY(dev_alloc((void**)&c->d_delta, EXACTO_MAX_L * sizeof(u64)));
    if (int e_ = upload(c, c->d_delta, dr.data(), dr.size() * sizeof(u64))) return e_;
    c->delta_ok = true;
    return 0;
}

// encrypt.rs:29-106 for a batch: pt = [B][n] plaintext coefficients, ct = [B][2][L][n] (NTT domain).
// pk == nullptr: secret-key encryption with sk; otherwise public-key encryption with pk [2][L][n].
static int encrypt_batch(exacto_ctx* c, const u64* pt, const u64* sk, const u64* pk, double sigma,
                         const uint64_t* key, u64 stream, u64* ct, size_t B) {
    if (!key || !pt || !ct || (!sk && !pk)) return invalid_param("null argument");
    if (B == 0) return 0;
    if (int e = delta_residues(c)) return e;
    const long Ln = (long)c->L * c->n;
    const ChaChaKey k = chacha_key(key);
    // scratch: Delta m [B][L][n], and u [B][L][n] for pk-encryption
    size_t cap = c->enc_cap;
    if (grow(&c->enc_buf, &cap, (size_t)B * (pk ? 2 : 1) * Ln * sizeof(u64))) return EXACTO_ERR_HIP;
    c->enc_cap = cap;
    u64* dm = c->enc_buf;
    u64* u = c->enc_buf + (size_t)B * Ln;
    launch_scale_plain(pt, c->d_delta, dm, (long)B, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = ntt_items(c, dm, (long)B, Ln, c->L)) return e;
    if (!pk) {
        // encrypt.rs:79-106, item b: a (index 2b) -> c1, e (index 2b+1) -> c0 slot
        if (int e = sample_polys(c, KG_UNIFORM, k, stream, ct + Ln, 2 * Ln, 0, 2, (long)B, sigma)) return e;
        if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, ct, 2 * Ln, 1, 2, (long)B, sigma)) return e;
        if (int e = ntt_items(c, ct, (long)B, 2 * Ln, 2L * c->L)) return e;
        launch_combine(KG_ENC_SK, ct, (long)B, 2 * Ln, Ln, sk, dm, nullptr, nullptr, nullptr, c->n, c->L, c->d_primes,
                       c->stream);
    } else {
        // encrypt.rs:29-69, item b: u binary (3b), e1 (3b+1) -> c0 slot, e2 (3b+2) -> c1 slot
        if (int e = sample_polys(c, KG_BINARY, k, stream, u, Ln, 0, 3, (long)B, sigma)) return e;
        if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, ct, 2 * Ln, 1, 3, (long)B, sigma)) return e;
        if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, ct + Ln, 2 * Ln, 2, 3, (long)B, sigma)) return e;
        if (int e = ntt_items(c, u, (long)B, Ln, c->L)) return e;
        if (int e = ntt_items(c, ct, (long)B, 2 * Ln, 2L * c->L)) return e;
        launch_combine(KG_ENC_PK, ct, (long)B, 2 * Ln, Ln, nullptr, u, dm, pk, nullptr, c->n, c->L, c->d_primes,
                       c->stream);
    }
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_encrypt_sk_dev(exacto_ctx* c, const uint64_t* pt, const uint64_t* sk, double sigma,
                                     const uint64_t* key, uint64_t stream, uint64_t* ct, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!sk) return invalid_param("null argument");
    return encrypt_batch(c, pt, sk, nullptr, sigma, key, stream, ct, B);
}

extern "C" int exacto_encrypt_pk_dev(exacto_ctx* c, const uint64_t* pt, const uint64_t* pk, double sigma,
                                     const uint64_t* key, uint64_t stream, uint64_t* ct, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!pk) return invalid_param("null argument");
    return encrypt_batch(c, pt, nullptr, pk, sigma, key, stream, ct, B);
}

// ---- Galois automorphisms (eval.rs:512-561, keygen.rs:171-262)

// gen_galois_key_with_rng (keygen.rs:171-209).  s(X^k) is formed as the reference does: limb 0 of s
// in the coefficient domain (mod q0), sigma_k mod q0, then reduced modulo every q_i (keygen.rs:179-182).
extern "C" int exacto_gen_galois_key_dev(exacto_ctx* c, const uint64_t* sk, uint64_t element, double sigma,
                                         const uint64_t* key, uint64_t stream, size_t num_keys, uint64_t* gk) {
    if (int e = check_ctx(c)) return e;
    if (!key || !sk || !gk) return invalid_param("null argument");
    if (num_keys == 0) return 0;
    const int n = c->n, L = c->L;
    const long Ln = (long)L * n;
    size_t cap = c->enc_cap;
    if (grow(&c->enc_buf, &cap, (size_t)(2 * n + Ln) * sizeof(u64))) return EXACTO_ERR_HIP;
    c->enc_cap = cap;
    u64 *t0 = c->enc_buf, *t1 = t0 + n, *s_auto = t1 + n;
    HIP_TRY(dev_copy(t0, sk, n * sizeof(u64), c->stream));
    if (int e = run_ntt(c, contiguous(t0, 1, 1, 0, 1, n), 1, true)) return e;
    launch_automorph(t0, n, t1, n, 1, 1, n, 1, element, c->d_primes, 0, c->stream);
    launch_lift_q0(t1, s_auto, 1, n, L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = ntt_items(c, s_auto, 1, 0, L)) return e;
    std::vector<u64> gpow(num_keys * L);
    for (int l = 0; l < L; ++l) {
        const u64 q = c->primes[l];
        u64 g = 1 % q;
        const u64 b = c->gbase % q;
        for (size_t i = 0; i < num_keys; ++i) {
            gpow[i * L + l] = g;
            g = (u64)((u128)g * b % q);
        }
    }
    cap = c->gpow_cap;
    if (grow(&c->d_gpow, &cap, gpow.size() * sizeof(u64))) return EXACTO_ERR_HIP;
    c->gpow_cap = cap;
    // the table is host-pageable and d_gpow may still be read by a previous call's kernels
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int e_ = upload(c, c->d_gpow, gpow.data(), gpow.size() * sizeof(u64))) return e_;
    const ChaChaKey k = chacha_key(key);
    if (int e = sample_polys(c, KG_UNIFORM, k, stream, gk + Ln, 2 * Ln, 0, 2, (long)num_keys, sigma)) return e;
    if (int e = sample_polys(c, KG_GAUSSIAN, k, stream, gk, 2 * Ln, 1, 2, (long)num_keys, sigma)) return e;
    if (int e = ntt_items(c, gk, (long)num_keys, 2 * Ln, 2L * L)) return e;
    launch_combine(KG_GALOIS, gk, (long)num_keys, 2 * Ln, Ln, sk, s_auto, nullptr, nullptr, c->d_gpow, n, L,
                   c->d_primes, c->stream);
    CHECK_LAUNCH();
    // gpow / s_auto scratch is reused by the next call: finish this one first
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// bfv_apply_automorphism (eval.rs:512-561), batched: sigma_k(c0) + sum_i d_i (.) gk_i0, sum_i d_i (.) gk_i1
// with d = gadget digits of sigma_k(c1) (exact CRT: extension semantics for Q >= 2^64, as relinearize).
extern "C" int exacto_bfv_apply_automorphism_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t element,
                                                 const uint64_t* gk, size_t num_keys, uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (polys != 2) return invalid_param("automorphism requires degree-1 ciphertext");
    if (num_keys == 0 || !gk) return invalid_param("galois key is empty");
    if (B == 0) return 0;
    const int n = c->n, L = c->L;
    const long Ln = (long)L * n;
    const int guse = (int)std::min<size_t>(c->G, num_keys);
    const size_t count = (size_t)guse * 2 * Ln;
    const bool d16 = c->digit16 && c->gbase <= 65536;  // int16 digits, as in run_mul
    // ks32 key switch (as run_mul): the key converted to the 31-bit basis on every call (the
    // caller may pass a different key in the same buffer), G L (2L) 60-bit (32-bit) transforms
    // The narrow basis (kn) always: its bound holds for any key, and this key's norms are not
    // examined (the lazy basis is chosen per resident relinearisation key only).
    const Ks32Basis& kb = c->kn;
    const bool k32 = d16 && c->ks32 && kb.S > 0 && c->path == EXACTO_PATH_EXACT_RNS;
    if (k32) {
        size_t cap = c->gk_rs_cap;
        const int e = ks32_convert_key(c, gk, (size_t)guse, &c->d_gk_rs, &cap, kb.S, kb.d_p32, kb.mac_form);
        c->gk_rs_cap = cap;
        if (e) return e;
    } else {
        size_t cap = c->gk_s_cap;
        if (grow(&c->gk_s, &cap, count * sizeof(u64))) return EXACTO_ERR_HIP;
        c->gk_s_cap = cap;
        launch_shoup_companions(gk, c->gk_s, (long)count, n, L, c->d_primes, c->stream);
        CHECK_LAUNCH();
    }
    const size_t C = std::min<size_t>(c->chunk, B);
    if (int e = ensure_workspace(c, C)) return e;
    // chunks alternate over the pipeline lanes as in run_mul (the key tables above are made on
    // the main stream before the fork)
    int nl = 1;
    if (int e = fork_lanes(c, (long)((B + C - 1) / C), C, &nl)) return e;
    LaneJoin join{c, nl};
    for (size_t s0 = 0; s0 < B; s0 += C) {
        const int cnt = (int)std::min(C, B - s0);
        LaneGuard lane(c, (int)((s0 / C) % (size_t)nl));
        const u64* src = ct + s0 * 2 * Ln;
        u64* dst = out + s0 * 2 * Ln;
        NttBatch nb{};
        nb.src = src; nb.src_item_stride = 2 * Ln;
        nb.dst = c->ws_coefQ; nb.dst_item_stride = 2 * Ln;
        nb.ppi = 2 * L; nb.prime_base = 0; nb.period = L;
        if (int e = run_ntt(c, nb, (long)cnt * 2 * L, true)) return e;
        launch_automorph(c->ws_coefQ, 2 * Ln, c->ws_T, 2 * Ln, cnt, 2, n, L, element, c->d_primes, -1, c->stream);
        CHECK_LAUNCH();
        if (k32) {
            // digits of sigma(c1); sum_g d_g * r_g over the integers added to (sigma(c0), 0) in the
            // coefficient domain; then both components forward
            launch_decompose(c->ws_T + Ln, 2 * Ln, c->ws_D, guse, cnt, n, c->d_crt, c->d_primes, L, c->stream,
                             c->ws_D16);
            CHECK_LAUNCH();
            launch_rows(c->ws_T + Ln, 2 * Ln, nullptr, 0, Ln, cnt, c->stream);
            CHECK_LAUNCH();
            ks32_digits(c->ws_D16, c->ws_DS, cnt, guse, kb.S, c->logn, kb.d_p32, kb.mac_form, c->stream);
            ks32_mac(c->ws_DS, c->d_gk_rs, c->ws_U, cnt, guse, L, kb.S, n, kb.d_p32, kb.mac_form, c->stream);
            ks32_crt(c->ws_U, c->ws_T, 2 * Ln, cnt, L, kb.S, c->logn, kb.d_kst, kb.d_p32, c->d_primes, kb.mac_form, c->stream,
                     c->ks_fpc && kb.fpc_max >= 1);
            CHECK_LAUNCH();
            NttBatch rb{};
            rb.src = c->ws_T; rb.src_item_stride = 2 * Ln;
            rb.dst = dst; rb.dst_item_stride = 2 * Ln;
            rb.ppi = 2 * L; rb.prime_base = 0; rb.period = L;
            if (int e = run_ntt(c, rb, (long)cnt * 2 * L, false)) return e;
            continue;
        }
        NttBatch c0{};
        c0.src = c->ws_T; c0.src_item_stride = 2 * Ln;
        c0.dst = dst; c0.dst_item_stride = 2 * Ln;
        c0.ppi = L; c0.prime_base = 0; c0.period = L;
        if (int e = run_ntt(c, c0, (long)cnt * L, false)) return e;
        launch_rows(dst + Ln, 2 * Ln, nullptr, 0, Ln, cnt, c->stream);
        launch_decompose(c->ws_T + Ln, 2 * Ln, c->ws_D, guse, cnt, n, c->d_crt, c->d_primes, L, c->stream,
                         d16 ? c->ws_D16 : nullptr);
        CHECK_LAUNCH();
        NttBatch db = contiguous(c->ws_D, cnt, (long)guse * L, 0, L, n);
        if (d16) {
            db.src16 = c->ws_D16;
            db.src16_item_stride = (long)guse * n;
        }
        if (int e = run_ntt(c, db, (long)cnt * guse * L, false)) return e;
        launch_relin_mac(dst, 2 * Ln, c->ws_D, gk, c->gk_s, guse, dst, 2 * Ln, cnt, n, L, c->d_primes, c->stream);
        CHECK_LAUNCH();
    }
    return 0;
}

extern "C" int exacto_gen_galois_key(exacto_ctx* c, const uint64_t* sk, uint64_t element, double sigma,
                                     const uint64_t* key, uint64_t stream, size_t num_keys, uint64_t* gk) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{sk, c->L * poly_bytes(c)}}, num_keys * 2 * c->L * poly_bytes(c), gk,
                     [&](std::vector<u64*>& d, u64* o) {
                         return exacto_gen_galois_key_dev(c, d[0], element, sigma, key, stream, num_keys, o);
                     });
}

extern "C" int exacto_bfv_apply_automorphism(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t element,
                                             const uint64_t* gk, size_t num_keys, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    if (polys != 2) return invalid_param("automorphism requires degree-1 ciphertext");
    return host_call(c, {{ct, B * 2 * c->L * poly_bytes(c)}, {gk, num_keys * 2 * c->L * poly_bytes(c)}},
                     B * 2 * c->L * poly_bytes(c), out, [&](std::vector<u64*>& d, u64* o) {
                         return exacto_bfv_apply_automorphism_dev(c, d[0], polys, element, d[1], num_keys, o, B);
                     });
}

// ---- plaintext-ciphertext operations and the trace (bfv/eval.rs:468-503, 572-652) ----

static int pl_scratch(exacto_ctx* c, size_t words) {
    size_t cap = c->pl_cap;
    if (grow(&c->pl_buf, &cap, words * sizeof(u64))) return EXACTO_ERR_HIP;
    c->pl_cap = cap;
    return 0;
}

// pt [items][n] (any u64) -> NTT(pt mod q_i [* Delta_i]) as [items][L][n] in c->pl_buf
static int lift_plain(exacto_ctx* c, const u64* pt, long items, bool delta) {
    const long Ln = (long)c->L * c->n;
    if (delta)
        if (int e = delta_residues(c)) return e;
    if (int e = pl_scratch(c, (size_t)items * Ln)) return e;
    launch_scale_plain(pt, delta ? c->d_delta : nullptr, c->pl_buf, items, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return ntt_items(c, c->pl_buf, items, Ln, c->L);
}

extern "C" int exacto_bfv_plain_mul_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* pt,
                                        uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!ct || !pt || !out) return invalid_param("null argument");
    if (polys == 0) return invalid_param("ciphertext has no components");
    if (B == 0) return 0;
    if (int e = lift_plain(c, pt, (long)B, false)) return e;
    const long Ln = (long)c->L * c->n;
    launch_plain_apply(PLAIN_MUL, ct, (long)polys * Ln, out, (long)B, (int)polys, c->pl_buf, Ln, c->n, c->L, c->d_primes,
                       c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_bfv_plain_add_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* pt,
                                        uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!ct || !pt || !out) return invalid_param("null argument");
    if (polys == 0) return invalid_param("ciphertext has no components");
    if (B == 0) return 0;
    if (int e = lift_plain(c, pt, (long)B, true)) return e;
    const long Ln = (long)c->L * c->n;
    launch_plain_apply(PLAIN_ADD, ct, (long)polys * Ln, out, (long)B, (int)polys, c->pl_buf, Ln, c->n, c->L, c->d_primes,
                       c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_bfv_inner_product_dev(exacto_ctx* c, const uint64_t* cts, const uint64_t* pts, size_t K,
                                            size_t polys, uint64_t* out) {
    if (int e = check_ctx(c)) return e;
    if (K == 0) return invalid_param("mismatched ct/pt lengths");
    if (!cts || !pts || !out) return invalid_param("null argument");
    if (polys == 0) return invalid_param("ciphertext has no components");
    if (int e = lift_plain(c, pts, (long)K, false)) return e;
    launch_inner_product(cts, c->pl_buf, out, (int)K, (int)polys, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_bfv_monomial_mul_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t j,
                                           uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!ct || !out) return invalid_param("null argument");
    if (B == 0 || polys == 0) return 0;
    const long Ln = (long)c->L * c->n;
    j %= 2 * (u64)c->n;
    if (j == 0) {  // eval.rs:619-621: a clone
        if (out != ct)
            HIP_TRY(dev_copy(out, ct, B * polys * Ln * sizeof(u64), c->stream));
        return 0;
    }
    if (int e = pl_scratch(c, (size_t)Ln)) return e;
    launch_monomials(c->pl_buf, 1, j, false, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = ntt_items(c, c->pl_buf, 1, 0, c->L)) return e;
    launch_plain_apply(PLAIN_MUL, ct, polys * Ln, out, (long)B, (int)polys, c->pl_buf, 0, c->n, c->L, c->d_primes,
                       c->stream);
    CHECK_LAUNCH();
    return 0;
}

// Trace accumulation over [B][2][L][n] in r: chain (src == nullptr): r += sigma_k(r) for each k in
// order (eval.rs:572-586, coeffs_to_slots.rs:65-75); naive: r += sigma_k(src) (coeffs_to_slots.rs:79-95).
// key e of ks lives at gks + kidx[e] * num_keys * 2Ln.
static int trace_core(exacto_ctx* c, const u64* src, u64* r, const std::vector<u64>& ks,
                      const std::vector<size_t>& kidx, const u64* gks, size_t num_keys, size_t B) {
    if (ks.empty()) return 0;
    const long Ln = (long)c->L * c->n;
    Scratch rs;
    HIP_TRY(rs.alloc(B * 2 * Ln * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    u64* rot = rs.as<u64>();
    int rc = 0;
    for (size_t e = 0; e < ks.size() && rc == 0; ++e) {
        rc = exacto_bfv_apply_automorphism_dev(c, src ? src : r, 2, ks[e], gks + kidx[e] * num_keys * 2 * Ln,
                                               num_keys, rot, B);
        if (rc == 0) {
            launch_pointwise(PwOp::Add, r, rot, r, (long)B * 2 * c->L, c->n, c->L, nullptr, c->d_primes, c->stream);
            if (hipGetLastError() != hipSuccess) rc = fail(EXACTO_ERR_HIP, "HIP error: trace add launch");
        }
    }
    return rc;
}

// eval.rs:572-586 batched: result = ct; for k in elements: result += sigma_k(result).
// elements is a host array [E]; gks = [E][num_keys][2][L][n], the key of elements[e] at index e.
extern "C" int exacto_bfv_trace_dev(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* elements,
                                    size_t E, const uint64_t* gks, size_t num_keys, uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!ct || !out || (E && (!elements || !gks))) return invalid_param("null argument");
    if (B == 0) return 0;
    const long Ln = (long)c->L * c->n;
    if (out != ct) HIP_TRY(dev_copy(out, ct, B * polys * Ln * sizeof(u64), c->stream));
    if (E == 0) return 0;
    if (polys != 2) return invalid_param("automorphism requires degree-1 ciphertext");
    std::vector<u64> ks(elements, elements + E);
    std::vector<size_t> kidx(E);
    for (size_t e = 0; e < E; ++e) kidx[e] = e;
    return trace_core(c, nullptr, out, ks, kidx, gks, num_keys, B);
}

// coeffs_to_slots.rs:168-183
extern "C" size_t exacto_required_trace_elements(size_t n, uint64_t* out, size_t cap) {
    std::vector<u64> v;
    if (n <= 32 || (n & (n - 1))) {
        for (u64 k = 3; k < 2 * (u64)n; k += 2) v.push_back(k);
    } else {
        for (u64 step = n; step >= 2; step >>= 1) v.push_back(step + 1);
    }
    for (size_t i = 0; i < v.size() && i < cap && out; ++i) out[i] = v[i];
    return v.size();
}

// coeffs_to_slots.rs:21-49 for the coefficients j0 .. j0+J-1 of one ciphertext at once:
// out[t] = n^-1 * Tr(X^(2n-j) ct), j = j0 + t; the J shifted copies share every trace step.
extern "C" int exacto_extract_coefficients_dev(exacto_ctx* c, const uint64_t* ct, uint64_t j0, size_t J,
                                               const uint64_t* elements, size_t E, const uint64_t* gks,
                                               size_t num_keys, uint64_t* out) {
    if (int e = check_ctx(c)) return e;
    if (!ct || !out || (E && (!elements || !gks))) return invalid_param("null argument");
    if (J == 0) return 0;
    const int n = c->n;
    if (j0 + J - 1 > 2 * (u64)n) return invalid_param("coefficient index out of range");
    // resolve every key the trace needs first (HashMap lookups, coeffs_to_slots.rs:67-69, 87-89)
    std::vector<u64> ks(exacto_required_trace_elements(n, nullptr, 0));
    exacto_required_trace_elements(n, ks.data(), ks.size());
    std::vector<size_t> kidx(ks.size());
    for (size_t e = 0; e < ks.size(); ++e) {
        size_t f = 0;
        while (f < E && elements[f] != ks[e]) ++f;
        if (f == E) return invalid_param("missing Galois key for element " + std::to_string(ks[e]));
        kidx[e] = f;
    }
    // n^-1 mod t (coeffs_to_slots.rs:40-42)
    const u64 n_inv = invmod_h((u64)n % c->plain, c->plain);
    if (!n_inv) return invalid_param("n not invertible mod t");
    const long Ln = (long)c->L * n;
    const bool naive = n <= 32 || (n & (n - 1));
    // shifted copies X^(2n-j) ct: the monomial table [J][L][n] in the NTT domain, one broadcast product
    if (int e = pl_scratch(c, J * Ln)) return e;
    launch_monomials(c->pl_buf, (long)J, j0, true, n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = ntt_items(c, c->pl_buf, (long)J, Ln, c->L)) return e;
    Scratch ss;
    if (naive) HIP_TRY(ss.alloc(J * 2 * Ln * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    u64* shifted = naive ? ss.as<u64>() : out;
    launch_plain_apply(PLAIN_MUL, ct, 0, shifted, (long)J, 2, c->pl_buf, Ln, n, c->L, c->d_primes, c->stream);
    int rc = hipGetLastError() == hipSuccess ? 0 : fail(EXACTO_ERR_HIP, "HIP error: monomial launch");
    if (rc == 0 && naive)
        rc = dev_copy(out, shifted, J * 2 * Ln * sizeof(u64), c->stream) == hipSuccess
                 ? 0 : fail(EXACTO_ERR_HIP, "HIP error: copy");
    if (rc == 0) rc = trace_core(c, naive ? shifted : nullptr, out, ks, kidx, gks, num_keys, J);
    if (rc) return rc;
    // times the constant plaintext n^-1: NTT(constant) is that constant in every slot
    return exacto_rns_scalar_mul_dev(c, out, n_inv, out, J * 2);
}

// coeffs_to_slots.rs:121-145: sum_j X^j slots[j], as one inner product against the monomial table
extern "C" int exacto_slots_to_coeffs_dev(exacto_ctx* c, const uint64_t* slots, size_t S, size_t polys,
                                          uint64_t* out) {
    if (int e = check_ctx(c)) return e;
    if (S == 0) return invalid_param("empty slots");
    if (S != (size_t)c->n)
        return invalid_param("expected " + std::to_string(c->n) + " slots, got " + std::to_string(S));
    if (!slots || !out) return invalid_param("null argument");
    if (polys == 0) return invalid_param("ciphertext has no components");
    const long Ln = (long)c->L * c->n;
    if (int e = pl_scratch(c, S * Ln)) return e;
    launch_monomials(c->pl_buf, (long)S, 0, false, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    if (int e = ntt_items(c, c->pl_buf, (long)S, Ln, c->L)) return e;
    launch_inner_product(slots, c->pl_buf, out, (int)S, (int)polys, c->n, c->L, c->d_primes, c->stream);
    CHECK_LAUNCH();
    return 0;
}

extern "C" int exacto_extract_coefficients(exacto_ctx* c, const uint64_t* ct, uint64_t j0, size_t J,
                                           const uint64_t* elements, size_t E, const uint64_t* gks, size_t num_keys,
                                           uint64_t* out) {
    if (!c) return invalid_param("null context");
    const size_t ctb = 2 * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}, {gks, E * num_keys * ctb}}, J * ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_extract_coefficients_dev(c, d[0], j0, J, elements, E, d[1], num_keys, o);
    });
}

extern "C" int exacto_slots_to_coeffs(exacto_ctx* c, const uint64_t* slots, size_t S, size_t polys, uint64_t* out) {
    if (!c) return invalid_param("null context");
    const size_t ctb = polys * c->L * poly_bytes(c);
    return host_call(c, {{slots, S * ctb}}, ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_slots_to_coeffs_dev(c, d[0], S, polys, o);
    });
}

extern "C" int exacto_bfv_plain_mul(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* pt,
                                    uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * polys * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}, {pt, B * poly_bytes(c)}}, ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_bfv_plain_mul_dev(c, d[0], polys, d[1], o, B);
    });
}

extern "C" int exacto_bfv_plain_add(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* pt,
                                    uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * polys * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}, {pt, B * poly_bytes(c)}}, ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_bfv_plain_add_dev(c, d[0], polys, d[1], o, B);
    });
}

extern "C" int exacto_bfv_inner_product(exacto_ctx* c, const uint64_t* cts, const uint64_t* pts, size_t K,
                                        size_t polys, uint64_t* out) {
    if (!c) return invalid_param("null context");
    if (K == 0) return invalid_param("mismatched ct/pt lengths");
    const size_t ctb = polys * c->L * poly_bytes(c);
    return host_call(c, {{cts, K * ctb}, {pts, K * poly_bytes(c)}}, ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_bfv_inner_product_dev(c, d[0], d[1], K, polys, o);
    });
}

extern "C" int exacto_bfv_monomial_mul(exacto_ctx* c, const uint64_t* ct, size_t polys, uint64_t j, uint64_t* out,
                                       size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * polys * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}}, ctb, out, [&](std::vector<u64*>& d, u64* o) {
        return exacto_bfv_monomial_mul_dev(c, d[0], polys, j, o, B);
    });
}

extern "C" int exacto_bfv_trace(exacto_ctx* c, const uint64_t* ct, size_t polys, const uint64_t* elements, size_t E,
                                const uint64_t* gks, size_t num_keys, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * polys * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}, {gks, E * num_keys * 2 * c->L * poly_bytes(c)}}, ctb, out,
                     [&](std::vector<u64*>& d, u64* o) {
                         return exacto_bfv_trace_dev(c, d[0], polys, elements, E, d[1], num_keys, o, B);
                     });
}

// ---- digit extraction pieces (bootstrap/digit_extract.rs) ----

// lagrange_interpolate (digit_extract.rs:37-90): the Lagrange formula at the points 0..n-1 over Z_p.
// The numerator prod_{k != j} (x - k) is the master polynomial prod_k (x - k) divided by the monic
// (x - j) -- exact over Z, so reducing mod p commutes -- which makes it O(n^2) instead of O(n^3)
// with the same coefficients; the denominators prod_{k != j} (j - k) are the reference's.
extern "C" int exacto_lagrange_interpolate(const uint64_t* values, size_t n, uint64_t p, uint64_t* out) {
    if (n == 0) return 0;
    if (!values || !out) return invalid_param("null argument");
    if (p == 0) return invalid_param("modulus must be nonzero");
    if (n == 1) { out[0] = values[0] % p; return 0; }
    auto mulm = [p](u64 a, u64 b) { return (u64)((u128)a * b % p); };
    auto addm = [p](u64 a, u64 b) { return (u64)(((u128)a + b) % p); };
    // master[d], degree n: prod_{k=0}^{n-1} (x - k)
    std::vector<u64> master(n + 1, 0), num(n), res(n, 0);
    master[0] = 1 % p;
    for (size_t k = 0; k < n; ++k) {
        const u64 neg_k = (p - (u64)k % p) % p;
        for (size_t d = k + 2; d-- > 0;) {  // d = k+1 .. 0
            const u64 lower = d ? master[d - 1] : 0;
            master[d] = addm(lower, mulm(master[d], neg_k));
        }
    }
    for (size_t j = 0; j < n; ++j) {
        if (values[j] % p == 0) continue;
        // synthetic division of master by (x - j): num[n-1] = master[n], num[d-1] = master[d] + j num[d]
        const u64 jm = (u64)j % p;
        num[n - 1] = master[n];
        for (size_t d = n - 1; d >= 1; --d) num[d - 1] = addm(master[d], mulm(jm, num[d]));
        u64 denom = 1 % p;
        for (size_t k = 0; k < n; ++k) {
            if (k == j) continue;
            const u64 diff = j >= k ? (u64)(j - k) % p : (p - (u64)(k - j) % p) % p;
            denom = mulm(denom, diff);
        }
        const u64 dinv = invmod_h(denom, p);
        if (!dinv) return invalid_param("points must be distinct mod p");
        const u64 scale = mulm(values[j] % p, dinv);
        for (size_t d = 0; d < n; ++d) res[d] = addm(res[d], mulm(num[d], scale));
    }
    std::copy(res.begin(), res.end(), out);
    return 0;
}

// compute_rounding_poly (digit_extract.rs:19-30): g(x) = round(t_orig (x mod q') / q') mod t_orig
// on x in [0, t_boot), interpolated over Z_{t_boot}; out has t_boot coefficients.
extern "C" int exacto_compute_rounding_poly(uint64_t t_orig, uint64_t q_prime, uint64_t t_boot, uint64_t* out) {
    if (!out) return invalid_param("null argument");
    if (q_prime == 0 || t_orig == 0) return invalid_param("moduli must be nonzero");
    std::vector<u64> v(t_boot);
    for (u64 x = 0; x < t_boot; ++x) {
        const u128 reduced = x % q_prime;
        v[x] = (u64)(((u128)t_orig * reduced + q_prime / 2) / q_prime % t_orig);
    }
    return exacto_lagrange_interpolate(v.data(), t_boot, t_boot, out);
}

// trivial_encrypt_poly (digit_extract.rs:179-189): (Delta m, 0), m = pt [B][n] as given
extern "C" int exacto_trivial_encrypt_dev(exacto_ctx* c, const uint64_t* pt, uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (!pt || !out) return invalid_param("null argument");
    if (B == 0) return 0;
    const long Ln = (long)c->L * c->n;
    if (int e = lift_plain(c, pt, (long)B, true)) return e;
    launch_rows(out, 2 * Ln, c->pl_buf, Ln, Ln, (long)B, c->stream);
    launch_rows(out + Ln, 2 * Ln, nullptr, 0, Ln, (long)B, c->stream);
    CHECK_LAUNCH();
    return 0;
}

// eval_poly_homomorphic (digit_extract.rs:101-157), batched: the same polynomial on B ciphertexts.
// Paterson-Stockmeyer with the reference's schedule: baby steps x^i = x^(i/2) * x^(i - i/2) for
// i = 2..k, k = max(2, ceil(sqrt(d + 1))); groups g_i = sum_j a_{ik+j} x^j (trivial(0) + scalar
// multiples, coefficients reduced mod t as bfv_scalar_mul does); Horner in x^k.  Uses the context's
// resident relinearisation key for every bfv_mul_and_relin.
extern "C" int exacto_eval_poly_dev(exacto_ctx* c, const uint64_t* ct, const uint64_t* coeffs, size_t m,
                                    uint64_t* out, size_t B) {
    if (int e = check_ctx(c)) return e;
    if (m == 0) return invalid_param("empty polynomial");
    if (!ct || !out || !coeffs) return invalid_param("null argument");
    if (B == 0) return 0;
    if (int e = delta_residues(c)) return e;
    const long Ln = (long)c->L * c->n;
    const size_t words = B * 2 * Ln;
    const size_t d = m - 1;
    const u64 t = c->plain;
    if (d == 0) {  // digit_extract.rs:109-111: trivial_encrypt(a_0)
        launch_trivial_const(out, (long)B, coeffs[0] % t, c->d_delta, c->n, c->L, c->d_primes, c->stream);
        CHECK_LAUNCH();
        return 0;
    }
    if (!c->rlk_loaded) return fail(EXACTO_ERR_MISSING_KEY, "key not available: relinearization key not loaded");
    const size_t k = std::max<size_t>(2, (size_t)std::ceil(std::sqrt((double)d + 1.0)));
    const size_t groups = (d + k) / k;
    // workspace: baby[0], baby[2..k] (baby[1] is ct), one group accumulator, a Horner ping buffer
    const size_t nbuf = k + 3;
    Scratch wss;
    HIP_TRY(wss.alloc(nbuf * words * sizeof(u64), c->stream, c->pool, c->debug_scratch));
    u64* ws = wss.as<u64>();
    std::vector<const u64*> baby(k + 1);
    auto slot = [&](size_t i) { return ws + i * words; };
    baby[0] = slot(0);
    baby[1] = ct;
    u64* acc = slot(k + 1);
    u64* ping = slot(k + 2);
    int rc = 0;
    launch_trivial_const(slot(0), (long)B, 1 % t, c->d_delta, c->n, c->L, c->d_primes, c->stream);
    if (hipGetLastError() != hipSuccess) rc = fail(EXACTO_ERR_HIP, "HIP error: trivial launch");
    for (size_t i = 2; i <= k && rc == 0; ++i) {
        const size_t half = i / 2;
        rc = exacto_bfv_mul_and_relin_dev(c, baby[half], baby[i - half], slot(i), B);
        baby[i] = slot(i);
    }
    // group g_i into `dst`: trivial(0) + sum_j (a mod t) x^j
    auto group = [&](size_t gi, u64* dst) -> int {
        launch_fill_u32(reinterpret_cast<uint32_t*>(dst), 0, (long)(2 * words), c->stream);   // (see dev_copy)
        HIP_TRY(hipGetLastError());
        for (size_t j = 0; j < k; ++j) {
            const size_t idx = gi * k + j;
            if (idx >= m) break;
            if (coeffs[idx] == 0) continue;
            launch_axpy(dst, baby[j], coeffs[idx] % t, (long)B * 2 * c->L, c->n, c->L, c->d_primes, c->stream);
            CHECK_LAUNCH();
        }
        return 0;
    };
    // Horner from the last group; the running result alternates between out and ping
    u64* res = ((groups - 1) % 2 == 0) ? out : ping;  // so that the final result lands in out
    u64* other = res == out ? ping : out;
    if (rc == 0) rc = group(groups - 1, res);
    for (size_t gi = groups - 1; gi-- > 0 && rc == 0;) {
        rc = exacto_bfv_mul_and_relin_dev(c, res, baby[k], other, B);
        if (rc == 0) rc = group(gi, acc);
        if (rc == 0) {
            launch_pointwise(PwOp::Add, other, acc, other, (long)B * 2 * c->L, c->n, c->L, nullptr, c->d_primes,
                             c->stream);
            if (hipGetLastError() != hipSuccess) rc = fail(EXACTO_ERR_HIP, "HIP error: add launch");
        }
        std::swap(res, other);
    }
    return rc;
}

// ---- bootstrap composition (bootstrap/bfv_host.rs) ----

static int boot_pair_check(exacto_ctx* o, exacto_ctx* b) {
    if (int e = check_ctx(o)) return e;
    if (int e = check_ctx(b)) return e;
    if (o->n != b->n) return invalid_param("boot params must have same ring degree");
    if (o->device != b->device) return invalid_param("both contexts must be on one device");
    // the reference switches from q = moduli[0] after to_coeff_poly, which only holds one residue
    // system when L = 1 (bfv_host.rs:149-157): multi-prime originals are not supported
    if (o->L != 1) return invalid_param("bootstrap requires a single-prime ciphertext modulus");
    return 0;
}

// The bootstrap functions work on two contexts.  They run every step of both on ONE stream (the
// boot context's): o's stream is rebound to b's for the call, so that every hand-off between the
// contexts (the inputs uploaded on b's stream and copied on o's, the modulus-switched rows written on
// o's and read on b's) is ordered by the runtime instead of by host-side synchronisation alone.
// (Made while chasing an intermittent failure of the C++ test's bootstrap case)
struct StreamRebind {
    exacto_ctx* c;
    hipStream_t saved;
    StreamRebind(exacto_ctx* c_, hipStream_t s) : c(c_), saved(c_->stream) {
        if (saved != s) (void)hipStreamSynchronize(saved);
        c->stream = s;
    }
    ~StreamRebind() {
        if (c->stream != saved) (void)hipStreamSynchronize(c->stream);
        c->stream = saved;
    }
};

// gen_bootstrap_key's key material (bfv_host.rs:57-100, 289-330): the boot scheme's secret key
// boot_sk [Lb][n] (NTT domain, create_boot_sk) and the plaintext s_pt [n] that bsk encrypts.
extern "C" int exacto_bootstrap_key_material_dev(exacto_ctx* o, exacto_ctx* b, const uint64_t* sk, uint64_t* boot_sk,
                                                 uint64_t* s_pt) {
    if (int e = boot_pair_check(o, b)) return e;
    if (!sk || !boot_sk || !s_pt) return invalid_param("null argument");
    const int n = o->n;
    StreamRebind one(o, b->stream);   // before the scratch: its block is freed on b's stream
    Scratch ts;
    HIP_TRY(ts.alloc(2 * n * sizeof(u64), o->stream, o->pool, o->debug_scratch));
    u64* tmp = ts.as<u64>();
    HIP_TRY(dev_copy(tmp, sk, n * sizeof(u64), o->stream));
    int rc = run_ntt(o, contiguous(tmp, 1, 1, 0, 1, n), 1, true);  // sk.poly.components[0].to_coeff_poly()
    if (rc == 0) {
        launch_boot_key_map(tmp, tmp + n, s_pt, n, o->primes[0], b->primes[0], b->plain, o->stream);
        rc = hipGetLastError() == hipSuccess ? 0 : fail(EXACTO_ERR_HIP, "HIP error: key map launch");
    }
    if (rc == 0) rc = hipStreamSynchronize(o->stream) == hipSuccess ? 0 : fail(EXACTO_ERR_HIP, "HIP error: sync");
    if (rc == 0) {  // RnsPoly::from_coeff_poly over the boot basis, then its NTT
        launch_scale_plain(tmp + n, nullptr, boot_sk, 1, n, b->L, b->d_primes, b->stream);
        rc = hipGetLastError() == hipSuccess ? 0 : fail(EXACTO_ERR_HIP, "HIP error: lift launch");
    }
    if (rc == 0) rc = ntt_items(b, boot_sk, 1, 0, b->L);
    // tmp + n was read on b's stream: both streams drain before the block returns to o's pool
    const hipError_t sb = hipStreamSynchronize(b->stream), so = hipStreamSynchronize(o->stream);
    if (rc == 0 && (sb != hipSuccess || so != hipSuccess)) rc = fail(EXACTO_ERR_HIP, "HIP error: sync");
    return rc;
}

// EXACTO_DEBUG_BOOT=1: the diagnostic of DESIGN.md §3's intermittent bootstrap result.  snap()
// copies the first words of an intermediate into a debug buffer on the stream as the call runs;
// xsnap() reads a block from 16 workgroups spread over the XCDs, each recording its XCD; dump()
// prints both to stderr after the call's final synchronisation.  Off: every call is a no-op.
struct BootDebug {
    static constexpr int DW = 64, DN = 16, XB = 16, XN = 4;
    hipStream_t s;
    bool on;
    u64* dbuf = nullptr;
    u64* xbuf = nullptr;
    uint32_t* xcc = nullptr;
    uint32_t* whit = nullptr;   // write-watch flags (kernels.hip DbgWatch)
    std::vector<std::pair<std::string, size_t>> names;
    std::vector<std::string> xnames;
    explicit BootDebug(hipStream_t st) : s(st) {
        static const bool env = [] { const char* e = getenv("EXACTO_DEBUG_BOOT"); return e && e[0] == '1'; }();
        on = env && hipMalloc((void**)&dbuf, DN * DW * sizeof(u64)) == hipSuccess &&
             hipMalloc((void**)&xbuf, XN * XB * 4 * sizeof(u64)) == hipSuccess &&
             hipMalloc((void**)&xcc, XN * XB * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc((void**)&whit, 8 * sizeof(uint32_t)) == hipSuccess;
        if (on) launch_fill_u32(whit, 0, 8, s);
    }
    ~BootDebug() {
        if (dbuf || xbuf || xcc || whit) (void)hipStreamSynchronize(s);
        free_dev(dbuf); free_dev(xbuf); free_dev(xcc); free_dev(whit);
    }
    // null source (an earlier allocation failed; the call's rc carries the real error): skipped, so the
    // diagnostic never faults the GPU and hides that error
    void snap(const std::string& name, const u64* p, size_t words) {
        if (!on || !p || names.size() >= (size_t)DN) return;
        const size_t w = std::min<size_t>(words, DW);
        launch_copy_u64(dbuf + names.size() * DW, p, (long)w, s);
        names.emplace_back(name, w);
    }
    void xsnap(const std::string& name, const u64* p) {
        if (!on || !p || xnames.size() >= (size_t)XN) return;
        launch_xcd_probe(p, xbuf + xnames.size() * XB * 4, 4, xcc + xnames.size() * XB, XB, s);
        xnames.push_back(name);
    }
    void dump() {
        if (!on) return;
        std::vector<u64> h(DN * DW), hx(XN * XB * 4);
        std::vector<uint32_t> hc(XN * XB);
        (void)hipMemcpyAsync(h.data(), dbuf, h.size() * sizeof(u64), hipMemcpyDeviceToHost, s);
        (void)hipMemcpyAsync(hx.data(), xbuf, hx.size() * sizeof(u64), hipMemcpyDeviceToHost, s);
        (void)hipMemcpyAsync(hc.data(), xcc, hc.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        for (size_t i = 0; i < xnames.size(); ++i) {
            std::string line = "boot-dbg xcd " + xnames[i] + ":";
            for (int k = 0; k < XB; ++k)
                line += " x" + std::to_string(hc[i * XB + k]) + "=" + std::to_string(hx[(i * XB + k) * 4]);
            std::fprintf(stderr, "%s\n", line.c_str());
        }
        for (size_t i = 0; i < names.size(); ++i) {
            u64 hsh = 1469598103934665603ull;   // FNV-1a of the snapshot
            for (size_t k = 0; k < names[i].second; ++k) hsh = (hsh ^ h[i * DW + k]) * 1099511628211ull;
            std::fprintf(stderr, "boot-dbg %-14s %016llx [%llu %llu %llu %llu]\n", names[i].first.c_str(),
                         (unsigned long long)hsh, (unsigned long long)h[i * DW], (unsigned long long)h[i * DW + 1],
                         (unsigned long long)h[i * DW + 2], (unsigned long long)h[i * DW + 3]);
        }
    }
};

// bfv_bootstrap (bfv_host.rs:131-205) on B ciphertexts of the original scheme (ct [B][2][1][n] on
// o) -> out [B][2][Lb][n] on b.  bsk [2][Lb][n] is the encryption of s under b; the boot
// relinearisation key must be resident in b; (elements, gks) are the trace keys as in
// exacto_extract_coefficients; rpoly [m] (host) the rounding polynomial.  Items whose c1 is zero
// take the reference's trivial fast path, the others the full ring path.
extern "C" int exacto_bfv_bootstrap_dev(exacto_ctx* o, exacto_ctx* b, const uint64_t* ct, size_t polys,
                                        const uint64_t* bsk, const uint64_t* rpoly, size_t m, uint64_t q_prime,
                                        const uint64_t* elements, size_t E, const uint64_t* gks, size_t num_keys,
                                        uint64_t* out, size_t B) {
    if (int e = boot_pair_check(o, b)) return e;
    if (polys != 2) return invalid_param("bootstrap requires degree-1 ciphertext");
    if (!ct || !bsk || !out || !rpoly) return invalid_param("null argument");
    if (q_prime == 0) return invalid_param("q_prime must be nonzero");
    if (B == 0) return 0;
    const int n = o->n;
    const long Lbn = (long)b->L * n;
    StreamRebind one(o, b->stream);
    // The call's intermediates live in b's persistent buffers (boot_buf: coefficients, flags, the
    // c0'/c1' rows, phase; boot_slots: the ring path's slots), grown like the workspaces and never
    // taken from the stream-ordered pool (round 4-5's zeros appeared in pool blocks).
    // Both streams drain before the call returns (`drain`, on every return path; the normal path calls
    // finish() to fold a failed synchronisation, e.g. a kernel fault, into the return code).
    const size_t ctw = 2 * Lbn;
    const size_t w_coef = 2 * B * 2 * n, w_flags = (B + 1) / 2, w_c0pt = 2 * B * n;
    {
        size_t cap = b->boot_cap;
        if (grow(&b->boot_buf, &cap, (w_coef + w_flags + w_c0pt + ctw) * sizeof(u64))) return EXACTO_ERR_HIP;
        b->boot_cap = cap;
    }
    int rc = 0;
    struct Drain {
        exacto_ctx *o, *b;
        bool done = false;
        int finish(int code) {
            done = true;
            const hipError_t sb = hipStreamSynchronize(b->stream), so = hipStreamSynchronize(o->stream);
            if (code == 0 && (sb != hipSuccess || so != hipSuccess)) return fail(EXACTO_ERR_HIP, "HIP error: sync");
            return code;
        }
        ~Drain() {
            if (!done) finish(1);
        }
    } drain{o, b};
    auto ok = [&](hipError_t e, const char* what) {
        if (rc == 0 && e != hipSuccess) rc = fail(EXACTO_ERR_HIP, std::string("HIP error: ") + what);
    };
    BootDebug dbg(b->stream);
    // 1. to coefficients (o), modulus switch to q' and reduce mod t_boot; c1 == 0 flags
    u64* coef = b->boot_buf;
    int* flags = reinterpret_cast<int*>(coef + w_coef);
    u64* small = coef + B * 2 * n;
    dbg.snap("ct", ct, B * 2 * n);
    ok(dev_copy(coef, ct, B * 2 * n * sizeof(u64), o->stream), "copy");
    launch_fill_u32(reinterpret_cast<uint32_t*>(flags), 0, (long)B, o->stream);   // (see dev_copy)
    ok(hipGetLastError(), "flags fill");
    dbg.snap("coef", coef, B * 2 * n);
    if (rc == 0) rc = exacto_rns_inv_dev(o, coef, B * 2);
    dbg.snap("coef_inv", coef, B * 2 * n);
    if (rc == 0) {
        launch_modswitch(coef, small, flags, (long)B, n, o->primes[0], q_prime, b->plain, o->stream);
        ok(hipGetLastError(), "modswitch launch");
    }
    dbg.snap("small", small, B * 2 * n);
    std::vector<int> hflags(B);
    if (rc == 0) ok(hipMemcpyAsync(hflags.data(), flags, B * sizeof(int), hipMemcpyDeviceToHost, o->stream), "flags");
    if (rc == 0) ok(hipStreamSynchronize(o->stream), "sync");
    // 2. phase = TrivialEnc(c0') + bsk * c1' (b), written into out
    // [B][n] copies of c0' and c1' rows in the plaintext layout
    u64* c0pt = coef + w_coef + w_flags;
    u64* c1pt = c0pt + B * n;
    // debug: the library's generic writers (rows / copy / fill kernels) report writes into c0pt and
    // c1pt from here to the end of the call (the rows copies below are the expected ones, kind 0)
    // EXACTO_DEBUG_WATCH=1: the watch alone, its flag buffer allocated once per process (the least
    // perturbing diagnostic: the snapshots' per-call allocations made the failure disappear in round 5)
    static uint32_t* watch_hit = [] {
        uint32_t* p = nullptr;
        const char* e = getenv("EXACTO_DEBUG_WATCH");
        if (e && e[0] == '1' && hipMalloc((void**)&p, 8 * sizeof(uint32_t)) == hipSuccess &&
            hipMemset(p, 0, 8 * sizeof(uint32_t)) == hipSuccess && hipDeviceSynchronize() == hipSuccess)
            return p;
        return (uint32_t*)nullptr;
    }();
    uint32_t* whit = dbg.on ? dbg.whit : watch_hit;
    if (whit && rc == 0) debug_watch_set(c0pt, c0pt + 2 * B * n, whit, b->stream);
    dbg.snap("small_again", small, B * 2 * n);
    dbg.xsnap("small", small);
    dbg.xsnap("c0pt_before", c0pt);
    if (rc == 0) {
        launch_rows(c0pt, n, small, 2 * n, n, (long)B, b->stream);
        launch_rows(c1pt, n, small + n, 2 * n, n, (long)B, b->stream);
        ok(hipGetLastError(), "copy c0/c1");
    }
    dbg.snap("c0pt_copied", c0pt, B * n);
    dbg.xsnap("c0pt_after", c0pt);
    if (rc == 0) rc = lift_plain(b, c1pt, (long)B, false);
    dbg.snap("c0pt_lift1", c0pt, B * n);
    if (rc == 0) {
        launch_plain_apply(PLAIN_MUL, bsk, 0, out, (long)B, 2, b->pl_buf, Lbn, n, b->L, b->d_primes, b->stream);
        ok(hipGetLastError(), "plain_mul launch");
    }
    if (rc == 0) rc = lift_plain(b, c0pt, (long)B, true);
    if (rc == 0) {
        launch_plain_apply(PLAIN_ADD, out, 2 * Lbn, out, (long)B, 2, b->pl_buf, Lbn, n, b->L, b->d_primes,
                           b->stream);
        ok(hipGetLastError(), "plain_add launch");
    }
    dbg.snap("c0pt", c0pt, B * n);
    dbg.snap("phase_out", out, B * 2 * Lbn);
    // 3. per item: rounding polynomial directly (trivial) or CoeffsToSlots -> g -> SlotsToCoeffs
    u64* phase = c0pt + w_c0pt;
    u64 *slots = nullptr, *rounded = nullptr;
    for (size_t i = 0; i < B && rc == 0; ++i) {
        u64* oi = out + i * ctw;
        ok(dev_copy(phase, oi, ctw * sizeof(u64), b->stream), "copy");
        if (rc) break;
        dbg.snap("phase" + std::to_string(i), phase, ctw);
        if (!hflags[i]) {  // bfv_host.rs:180-186
            rc = exacto_eval_poly_dev(b, phase, rpoly, m, oi, 1);
            dbg.snap("result" + std::to_string(i), oi, ctw);
            continue;
        }
        if (!slots) {  // once per call, on the first item that takes the ring path
            size_t cap = b->boot_slots_cap;
            if (b->boot_slots_cap < 2 * (size_t)n * ctw * sizeof(u64)) ok(hipStreamSynchronize(b->stream), "sync");
            if (rc == 0 && grow(&b->boot_slots, &cap, 2 * (size_t)n * ctw * sizeof(u64))) rc = EXACTO_ERR_HIP;
            b->boot_slots_cap = cap;
            if (rc) break;
            slots = b->boot_slots;
            rounded = slots + (size_t)n * ctw;
        }
        rc = exacto_extract_coefficients_dev(b, phase, 0, n, elements, E, gks, num_keys, slots);
        if (rc == 0) rc = exacto_eval_poly_dev(b, slots, rpoly, m, rounded, n);
        if (rc == 0) rc = exacto_slots_to_coeffs_dev(b, rounded, n, 2, oi);
    }
    rc = drain.finish(rc);
    dbg.dump();
    if (whit) {
        debug_watch_set(nullptr, nullptr, nullptr);
        uint32_t hh[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpy(hh, whit, sizeof(hh), hipMemcpyDeviceToHost);
        (void)hipMemset(whit, 0, sizeof(hh));
        uint32_t hits = 0;
        for (int k = 0; k < 8; ++k) hits |= hh[k] ? (1u << k) : 0;
        std::fprintf(stderr, "boot-dbg watch c0pt=%p..%p hits=0x%x (bit k: 0 rows copy, 1 rows zero, 2 copy_u64, "
                     "3 fill 0, 4 fill other)\n", (void*)c0pt, (void*)(c0pt + 2 * B * n), hits);
    }
    if (dbg.on) {
        std::fprintf(stderr, "boot-dbg ptrs coef=%p small=%p flags=%p c0pt=%p out=%p o.pool=%p b.pool=%p o.stream=%p "
                     "b.stream=%p\n", (void*)coef, (void*)small, (void*)flags, (void*)c0pt, (void*)out, (void*)o->pool,
                     (void*)b->pool, (void*)o->stream, (void*)b->stream);
    }
    return rc;
}

extern "C" int exacto_bootstrap_key_material(exacto_ctx* o, exacto_ctx* b, const uint64_t* sk, uint64_t* boot_sk,
                                             uint64_t* s_pt) {
    if (!o || !b) return invalid_param("null context");
    if (int e = boot_pair_check(o, b)) return e;
    const size_t n = o->n;
    u64* d = nullptr;
    HIP_TRY(dev_alloc((void**)&d, (n + b->L * n + n) * sizeof(u64)));
    int rc = upload(o, d, sk, n * sizeof(u64));
    if (rc == 0) rc = exacto_bootstrap_key_material_dev(o, b, d, d + n, d + n + b->L * n);
    if (rc == 0 && (hipMemcpyAsync(boot_sk, d + n, b->L * n * sizeof(u64), hipMemcpyDeviceToHost, o->stream) != hipSuccess ||
                    hipMemcpyAsync(s_pt, d + n + b->L * n, n * sizeof(u64), hipMemcpyDeviceToHost, o->stream) != hipSuccess ||
                    hipStreamSynchronize(o->stream) != hipSuccess))
        rc = fail(EXACTO_ERR_HIP, "HIP error: copy back");
    (void)hipFree(d);
    return rc;
}

extern "C" int exacto_bfv_bootstrap(exacto_ctx* o, exacto_ctx* b, const uint64_t* ct, size_t polys,
                                    const uint64_t* bsk, const uint64_t* rpoly, size_t m, uint64_t q_prime,
                                    const uint64_t* elements, size_t E, const uint64_t* gks, size_t num_keys,
                                    uint64_t* out, size_t B) {
    if (!o || !b) return invalid_param("null context");
    if (int e = boot_pair_check(o, b)) return e;
    if (polys != 2) return invalid_param("bootstrap requires degree-1 ciphertext");
    const size_t ctb = 2 * b->L * poly_bytes(b);
    return host_call(b, {{ct, B * 2 * o->L * poly_bytes(o)}, {bsk, ctb}, {gks, E * num_keys * ctb}}, B * ctb, out,
                     [&](std::vector<u64*>& d, u64* dout) {
                         return exacto_bfv_bootstrap_dev(o, b, d[0], polys, d[1], rpoly, m, q_prime, elements, E,
                                                         d[2], num_keys, dout, B);
                     });
}

extern "C" int exacto_trivial_encrypt(exacto_ctx* c, const uint64_t* pt, uint64_t* out, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{pt, B * poly_bytes(c)}}, B * 2 * c->L * poly_bytes(c), out,
                     [&](std::vector<u64*>& d, u64* o) { return exacto_trivial_encrypt_dev(c, d[0], o, B); });
}

extern "C" int exacto_eval_poly(exacto_ctx* c, const uint64_t* ct, const uint64_t* coeffs, size_t m, uint64_t* out,
                                size_t B) {
    if (!c) return invalid_param("null context");
    const size_t ctb = B * 2 * c->L * poly_bytes(c);
    return host_call(c, {{ct, ctb}}, ctb, out,
                     [&](std::vector<u64*>& d, u64* o) { return exacto_eval_poly_dev(c, d[0], coeffs, m, o, B); });
}

// Host-pointer variants (synchronous); `key` is always a host pointer to 4 words.
extern "C" int exacto_gen_secret_key(exacto_ctx* c, const uint64_t* key, uint64_t stream, uint64_t* sk) {
    if (!c) return invalid_param("null context");
    return host_call(c, {}, c->L * poly_bytes(c), sk,
                     [&](std::vector<u64*>&, u64* o) { return exacto_gen_secret_key_dev(c, key, stream, o); });
}

extern "C" int exacto_gen_public_key(exacto_ctx* c, const uint64_t* sk, double sigma, const uint64_t* key,
                                     uint64_t stream, uint64_t* pk) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{sk, c->L * poly_bytes(c)}}, 2 * c->L * poly_bytes(c), pk, [&](std::vector<u64*>& d, u64* o) {
        return exacto_gen_public_key_dev(c, d[0], sigma, key, stream, o);
    });
}

extern "C" int exacto_gen_relin_key(exacto_ctx* c, const uint64_t* sk, double sigma, const uint64_t* key,
                                    uint64_t stream, size_t num_keys, uint64_t* rlk) {
    if (!c) return invalid_param("null context");
    if (!rlk) {  // resident key only: stage the secret key, generate in place
        return host_call(c, {{sk, c->L * poly_bytes(c)}}, 0, nullptr, [&](std::vector<u64*>& d, u64*) {
            return exacto_gen_relin_key_dev(c, d[0], sigma, key, stream, num_keys, nullptr);
        });
    }
    return host_call(c, {{sk, c->L * poly_bytes(c)}}, num_keys * 2 * c->L * poly_bytes(c), rlk,
                     [&](std::vector<u64*>& d, u64* o) {
                         return exacto_gen_relin_key_dev(c, d[0], sigma, key, stream, num_keys, o);
                     });
}

extern "C" int exacto_encrypt_sk(exacto_ctx* c, const uint64_t* pt, const uint64_t* sk, double sigma,
                                 const uint64_t* key, uint64_t stream, uint64_t* ct, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{pt, B * poly_bytes(c)}, {sk, c->L * poly_bytes(c)}}, B * 2 * c->L * poly_bytes(c), ct,
                     [&](std::vector<u64*>& d, u64* o) {
                         return exacto_encrypt_sk_dev(c, d[0], d[1], sigma, key, stream, o, B);
                     });
}

extern "C" int exacto_encrypt_pk(exacto_ctx* c, const uint64_t* pt, const uint64_t* pk, double sigma,
                                 const uint64_t* key, uint64_t stream, uint64_t* ct, size_t B) {
    if (!c) return invalid_param("null context");
    return host_call(c, {{pt, B * poly_bytes(c)}, {pk, 2 * c->L * poly_bytes(c)}}, B * 2 * c->L * poly_bytes(c), ct,
                     [&](std::vector<u64*>& d, u64* o) {
                         return exacto_encrypt_pk_dev(c, d[0], d[1], sigma, key, stream, o, B);
                     });
}

// ============================================================== diagnostics

extern "C" size_t exacto_last_error(char* buf, size_t len) {
    if (buf && len) {
        const size_t m = std::min(len - 1, g_last_error.size());
        std::memcpy(buf, g_last_error.data(), m);
        buf[m] = 0;
    }
    return g_last_error.size();
}

extern "C" int exacto_prof_enable(exacto_ctx* c, int enable) {
    if (!c) return invalid_param("null context");
    c->prof = enable != 0;
    return 0;
}

extern "C" int exacto_prof_read(exacto_ctx* c, int kind, uint64_t* launches, double* total_ms, double* total_bytes,
                                uint64_t* polys) {
    if (!c) return invalid_param("null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    u64 nl = 0, np = 0;
    double ms = 0, by = 0;
    std::vector<ProfRec> keep;
    std::vector<double> rate;   // bytes per ms of each launch
    for (auto& r : c->recs) {
        if (r.kind != kind) { keep.push_back(r); continue; }
        float t = 0;
        HIP_TRY(hipEventElapsedTime(&t, r.a, r.b));
        ms += t; by += r.bytes; np += r.polys; ++nl;
        if (t > 0) rate.push_back(r.bytes / t);
        if (r.kern) {
            auto& k = c->prof_kern[kind][r.kern];
            k.first += 1;
            k.second += t;
        }
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    c->recs.swap(keep);
    // Robust total: the family's bytes at the MEDIAN per-launch rate.  An event pair can also span a
    // host-side gap before its launch reaches an idle stream (seen once: a cfg5 inverse family at 3x
    // its rocprofv3 durations in one run); the median ignores such a launch.  EXACTO_PROF_RAW=1 sums
    // the raw intervals.
    static const bool raw = [] { const char* e = getenv("EXACTO_PROF_RAW"); return e && atoi(e) != 0; }();
    if (!raw && !rate.empty()) {
        std::sort(rate.begin(), rate.end());
        const size_t m = rate.size();
        const double med = m % 2 ? rate[m / 2] : 0.5 * (rate[m / 2 - 1] + rate[m / 2]);
        if (med > 0) ms = by / med;
    }
    if (launches) *launches = nl;
    if (total_ms) *total_ms = ms;
    if (total_bytes) *total_bytes = by;
    if (polys) *polys = np;
    return 0;
}

// The kernels behind one profiled family in the records exacto_prof_read consumed since the last
// exacto_prof_kernels call for it, as rocprofv3 names them (the demangled kernel symbol without its
// "void " and parameter list), by descending event time: "name (launches, ms); name (...)".  Returns
// the length of the full text (like snprintf); buf may be NULL (a size query).  A call with a buffer
// clears the list.
static std::string kernel_symbol_name(const void* handle) {
    Dl_info info{};
    if (!dladdr(handle, &info) || !info.dli_sname) return "?";
    int st = 0;
    char* dm = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &st);
    std::string nm = (st == 0 && dm) ? dm : info.dli_sname;
    free(dm);
    if (nm.rfind("void ", 0) == 0) nm = nm.substr(5);
    int depth = 0;   // cut the parameter list: the first '(' outside template brackets
    for (size_t i = 0; i < nm.size(); ++i) {
        if (nm[i] == '<') ++depth;
        else if (nm[i] == '>') --depth;
        else if (nm[i] == '(' && depth == 0) { nm.resize(i); break; }
    }
    return nm;
}

extern "C" size_t exacto_prof_kernels(exacto_ctx* c, int kind, char* buf, size_t len) {
    if (!c) return 0;
    std::vector<std::pair<double, std::string>> v;
    for (auto& kv : c->prof_kern[kind]) {
        char tail[64];
        snprintf(tail, sizeof tail, " (%llu, %.3f ms)", (unsigned long long)kv.second.first, kv.second.second);
        v.emplace_back(kv.second.second, kernel_symbol_name(kv.first) + tail);
    }
    if (buf && len) c->prof_kern.erase(kind);   // a size query (buf NULL) keeps the list
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    std::string out;
    for (auto& e : v) out += (out.empty() ? "" : "; ") + e.second;
    if (buf && len) {
        const size_t k = std::min(len - 1, out.size());
        std::memcpy(buf, out.data(), k);
        buf[k] = 0;
    }
    return out.size();
}

// ============================================================== RCCL collectives
//
// Keys are made once and broadcast over xGMI to every GPU (the reference builds them on one host,
// keygen.rs:123-209); the limbs of a split dbfv_mul are gathered (never summed: an RCCL sum of
// residues would overflow mod q).  librccl is opened at first use (dlopen of librccl.so.1, or
// EXACTO_RCCL_LIB), so a process that already loaded RCCL (torch) shares that instance and the
// library has no link-time dependency on it.  Communicators are plain ncclComm_t handles, passed as
// void*: made here (exacto_rccl_comm_init) or by the caller's own RCCL.

#include <rccl/rccl.h>

namespace {
struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    // optional (deadline handling): a communicator whose collective missed its deadline is aborted
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        const char* env = getenv("EXACTO_RCCL_LIB");
        void* h = dlopen(env ? env : "librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { x.why = std::string("cannot open RCCL: ") + dlerror(); return x; }
        bool all = true;
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            all &= f != nullptr;
        };
        sym(x.get_unique_id, "ncclGetUniqueId");
        sym(x.comm_init_rank, "ncclCommInitRank");
        sym(x.comm_destroy, "ncclCommDestroy");
        sym(x.comm_count, "ncclCommCount");
        sym(x.comm_user_rank, "ncclCommUserRank");
        sym(x.broadcast, "ncclBroadcast");
        sym(x.all_gather, "ncclAllGather");
        sym(x.error_string, "ncclGetErrorString");
        x.ok = all;
        x.comm_abort = reinterpret_cast<decltype(x.comm_abort)>(dlsym(h, "ncclCommAbort"));
        x.async_error = reinterpret_cast<decltype(x.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
        if (!all) x.why = "RCCL library lacks a required symbol";
        return x;
    }();
    return r;
}
}  // namespace

#define RCCL_TRY(x)                                                                                      \
    do {                                                                                                 \
        const ncclResult_t r_ = (x);                                                                     \
        if (r_ != ncclSuccess)                                                                           \
            return fail(EXACTO_ERR_HIP, std::string("RCCL error: ") + rccl().error_string(r_) + " (" #x ")"); \
    } while (0)

static int rccl_ready() {
    if (!rccl().ok) return fail(EXACTO_ERR_HIP, "RCCL error: " + rccl().why);
    return 0;
}

extern "C" int exacto_rccl_unique_id(uint8_t* id) {
    if (!id) return invalid_param("null id buffer");
    if (int e = rccl_ready()) return e;
    ncclUniqueId u;
    RCCL_TRY(rccl().get_unique_id(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

// Deadline of the blocking RCCL steps (communicator init, the agreement all-gather, exacto_rccl_sync):
// $EXACTO_RCCL_TIMEOUT_S seconds (default 300; 0 = wait forever).  A rank that never joins makes the
// others fail with EXACTO_ERR_HIP "RCCL error: ... timed out" instead of blocking their process for
// good (the driver's 8-GPU run has one time limit for everything).
static double rccl_timeout_s() {
    const char* e = getenv("EXACTO_RCCL_TIMEOUT_S");
    return e ? atof(e) : 300.0;
}

// Communicators aborted after a missed deadline: RCCL has freed them, so destroy must not touch them.
static std::mutex g_aborted_mu;
static std::set<void*> g_aborted;

static int rccl_abort_timeout(void* comm, const std::string& what, double secs) {
    if (rccl().comm_abort) {
        (void)rccl().comm_abort((ncclComm_t)comm);
        std::lock_guard<std::mutex> g(g_aborted_mu);
        g_aborted.insert(comm);
    }
    return fail(EXACTO_ERR_HIP, "RCCL error: " + what + " timed out after " + std::to_string((int)secs) +
                                    " s (a rank did not join); communicator aborted");
}

// Waits for the context stream (the collectives enqueued on it) with the deadline: polls hipStreamQuery
// and the communicator's asynchronous error.  On expiry the communicator is aborted (RCCL then stops its
// kernels) and the call fails; it never returns with a collective still blocking the stream silently.
static int rccl_stream_wait(exacto_ctx* c, void* comm, const char* what) {
    const double lim = rccl_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return 0;
        if (q != hipErrorNotReady) return fail(EXACTO_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(q) + " (" + what + ")");
        if (rccl().async_error) {
            ncclResult_t ae = ncclSuccess;
            if (rccl().async_error((ncclComm_t)comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
                return fail(EXACTO_ERR_HIP, std::string("RCCL error: ") + rccl().error_string(ae) + " (" + what + ")");
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (lim > 0 && el > lim) return rccl_abort_timeout(comm, what, lim);
        std::this_thread::sleep_for(std::chrono::microseconds(it < 100 ? 20 : 1000));
    }
}

extern "C" int exacto_rccl_comm_init(void** comm, int nranks, const uint8_t* id, int rank, int device) {
    if (!comm || !id) return invalid_param("null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return invalid_param("rank out of range");
    if (int e = rccl_ready()) return e;
    HIP_TRY(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    // ncclCommInitRank blocks until every rank has joined: it runs on a helper thread so that the
    // caller's wait has a deadline.  On expiry the helper is left behind (it holds only its own copy
    // of the arguments) and the call fails; the caller is expected to end the process.
    struct InitState {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false;
        ncclResult_t r = ncclSuccess;
        ncclComm_t cm = nullptr;
    };
    auto st = std::make_shared<InitState>();
    std::thread([st, nranks, u, rank, device] {
        (void)hipSetDevice(device);
        ncclComm_t cm = nullptr;
        const ncclResult_t r = rccl().comm_init_rank(&cm, nranks, u, rank);
        std::lock_guard<std::mutex> g(st->mu);
        st->r = r;
        st->cm = cm;
        st->done = true;
        st->cv.notify_all();
    }).detach();
    const double lim = rccl_timeout_s();
    std::unique_lock<std::mutex> lk(st->mu);
    if (lim > 0) {
        if (!st->cv.wait_for(lk, std::chrono::duration<double>(lim), [&] { return st->done; }))
            return fail(EXACTO_ERR_HIP, "RCCL error: ncclCommInitRank timed out after " + std::to_string((int)lim) +
                                            " s (a rank did not join)");
    } else {
        st->cv.wait(lk, [&] { return st->done; });
    }
    if (st->r != ncclSuccess)
        return fail(EXACTO_ERR_HIP, std::string("RCCL error: ") + rccl().error_string(st->r) + " (ncclCommInitRank)");
    *comm = st->cm;
    return 0;
}

extern "C" int exacto_rccl_comm_destroy(void* comm) {
    if (!comm) return 0;
    if (int e = rccl_ready()) return e;
    {
        std::lock_guard<std::mutex> g(g_aborted_mu);
        if (g_aborted.erase(comm)) return 0;   // freed by ncclCommAbort
    }
    RCCL_TRY(rccl().comm_destroy((ncclComm_t)comm));
    return 0;
}

extern "C" int exacto_rccl_sync(exacto_ctx* c, void* comm) {
    if (int e = check_ctx(c)) return e;
    if (!comm) return invalid_param("null communicator");
    if (int e = rccl_ready()) return e;
    return rccl_stream_wait(c, comm, "collective on the context stream");
}

extern "C" int exacto_rccl_comm_count(void* comm, int* nranks) {
    if (!comm || !nranks) return invalid_param("null argument");
    if (int e = rccl_ready()) return e;
    RCCL_TRY(rccl().comm_count((ncclComm_t)comm, nranks));
    return 0;
}

// In-place broadcast of `words` u64 at buf from root's buffer, enqueued on the context stream.
// Checks the communicator and the root first; *my_rank (optional) receives this rank.
static int rccl_check(void* comm, int root, int* my_rank) {
    if (!comm) return invalid_param("null communicator");
    if (int e = rccl_ready()) return e;
    int nr = 0;
    RCCL_TRY(rccl().comm_count((ncclComm_t)comm, &nr));
    if (root < 0 || root >= nr) return invalid_param("root out of range");
    if (my_rank) RCCL_TRY(rccl().comm_user_rank((ncclComm_t)comm, my_rank));
    return 0;
}

static int rccl_bcast(exacto_ctx* c, void* comm, int root, u64* buf, size_t words) {
    if (int e = rccl_check(comm, root, nullptr)) return e;
    if (!words) return 0;
    RCCL_TRY(rccl().broadcast(buf, buf, words, ncclUint64, root, (ncclComm_t)comm, c->stream));
    return 0;
}

// Agreement step of a collective call: every rank contributes {its num_keys, its own verdict} and
// all-gathers everyone's, so that every rank takes the same decision (proceed or InvalidParam)
// before any rank resizes its key or enqueues the key broadcast.  A mismatch therefore fails on all
// ranks instead of leaving the others blocked in a broadcast the failing rank never joins.
static int rccl_agree(exacto_ctx* c, void* comm, u64 mine, u64 ok, bool* agreed, std::string* why) {
    *agreed = false;
    int nr = 0;
    RCCL_TRY(rccl().comm_count((ncclComm_t)comm, &nr));
    u64* dev = nullptr;
    HIP_TRY(hipMalloc((void**)&dev, sizeof(u64) * 2 * (nr + 1)));
    std::vector<u64> host(2 * (size_t)(nr + 1));
    host[0] = mine;
    host[1] = ok;
    int rc = 0;
    if (hipMemcpyAsync(dev, host.data(), 2 * sizeof(u64), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        rc = fail(EXACTO_ERR_HIP, "HIP error: hipMemcpyAsync (agreement header)");
    else {
        const ncclResult_t r = rccl().all_gather(dev, dev + 2, 2, ncclUint64, (ncclComm_t)comm, c->stream);
        if (r != ncclSuccess)
            rc = fail(EXACTO_ERR_HIP, std::string("RCCL error: ") + rccl().error_string(r) + " (ncclAllGather)");
        else if (hipMemcpyAsync(host.data() + 2, dev + 2, 2 * sizeof(u64) * nr, hipMemcpyDeviceToHost, c->stream) !=
                     hipSuccess ||
                 (rc = rccl_stream_wait(c, comm, "agreement all-gather")) != 0) {
            if (!rc) rc = fail(EXACTO_ERR_HIP, "HIP error: agreement header read-back");
        }
    }
    if (rc) return rc;   // a timed-out all-gather may still own `dev`: leave it (the process is ending)
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(dev);
    for (int r = 0; r < nr; ++r) {
        if (!host[2 + 2 * r + 1]) {
            *why = "rank " + std::to_string(r) + " rejected the call";
            return 0;
        }
        if (host[2 + 2 * r] != host[2]) {
            *why = "ranks disagree on num_keys (rank 0: " + std::to_string(host[2]) + ", rank " + std::to_string(r) +
                   ": " + std::to_string(host[2 + 2 * r]) + ")";
            return 0;
        }
    }
    *agreed = true;
    return 0;
}

// Every check runs before the resident key is touched: a failed call (bad root, no RCCL, a root
// without a loaded key of that size, ranks passing different num_keys) leaves every rank's key
// exactly as it was and returns InvalidParam on every rank (rccl_agree).  The root broadcasts its
// resident key as loaded (never resized); a receiving rank's buffer is (re)sized and marked loaded
// only once the broadcast into it has been enqueued.
extern "C" int exacto_ctx_broadcast_relin_key(exacto_ctx* c, void* comm, int root, size_t num_keys) {
    if (int e = check_ctx(c)) return e;
    int me = -1;
    if (int e = rccl_check(comm, root, &me)) return e;
    const size_t words = num_keys * 2 * c->L * (size_t)c->n;
    const bool root_ok = c->rlk_loaded && c->rlk_keys == num_keys;
    std::string why;
    bool agreed = false;
    if (int e = rccl_agree(c, comm, num_keys, me == root ? root_ok : 1, &agreed, &why)) return e;
    if (!agreed) {
        if (me == root && !root_ok)
            why = "broadcast root has no resident relinearization key of " + std::to_string(num_keys) + " rows";
        return invalid_param(why);
    }
    if (me == root) {
        if (!words) return 0;
        RCCL_TRY(rccl().broadcast(c->d_rlk, c->d_rlk, words, ncclUint64, root, (ncclComm_t)comm, c->stream));
        return 0;
    }
    u64* dst = exacto_ctx_relin_key_buffer(c, num_keys);
    if (!dst) return fail(EXACTO_ERR_HIP, "HIP error: relinearization key allocation failed");
    if (words) {
        const ncclResult_t r = rccl().broadcast(dst, dst, words, ncclUint64, root, (ncclComm_t)comm, c->stream);
        if (r != ncclSuccess) {
            c->rlk_loaded = false;   // the buffer's contents are undefined now
            return fail(EXACTO_ERR_HIP, std::string("RCCL error: ") + rccl().error_string(r) + " (ncclBroadcast)");
        }
    }
    return 0;
}

extern "C" int exacto_broadcast_galois_key(exacto_ctx* c, void* comm, int root, uint64_t* gk, size_t num_keys) {
    if (int e = check_ctx(c)) return e;
    if (num_keys && !gk) return invalid_param("null Galois key");
    return rccl_bcast(c, comm, root, gk, num_keys * 2 * c->L * (size_t)c->n);
}

extern "C" int exacto_rccl_allgather_u64(exacto_ctx* c, void* comm, const uint64_t* send, uint64_t* recv, size_t count) {
    if (int e = check_ctx(c)) return e;
    if (!comm) return invalid_param("null communicator");
    if (count && (!send || !recv)) return invalid_param("null buffer");
    if (int e = rccl_ready()) return e;
    if (!count) return 0;
    RCCL_TRY(rccl().all_gather(send, recv, count, ncclUint64, (ncclComm_t)comm, c->stream));
    return 0;
}

extern "C" const char* exacto_version(void) { return "exacto-hip 0.4.0 (gfx950)"; }
