// Compute-only / memory-only probes of the two NTT kernels the J2 roofline is about:
// the pinned forward transform (ntt_fwd_pin_kernel<12>) and cfg3's tensor + inverse
// (ntt_inv_tensor_kernel<12, true, true>), each in the library's own form (PROBE = 0) and with its
// global memory traffic removed (PROBE = 1: synthetic operands, stores skipped at run time) or, for
// the forward transform, its arithmetic removed (PROBE = 2: loads, LDS exchanges, stores).  The
// kernels are the library's (ntt.hip is included; the probes are compile-time template modes the
// library never instantiates).  The instruction stream is data-independent (branch-free rounds), so
// random twiddles and residues time exactly what the product runs.
//
// If the compute-only form takes nearly as long as the full kernel, the kernel is bound by its
// instructions, not by HBM: its HBM fraction can only rise with fewer instructions per byte.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ntt_probe.hip -o build/ntt_probe
// Run:   build/ntt_probe [reps]   -> one JSON line
#include "../exacto_amd/csrc/ntt.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace exacto;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

static u64 shoup_c(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    constexpr int LOGN = 12, N = 1 << LOGN;
    const u64 q = 1152921504606830593ull;   // cfg3's first prime (2^60 - d)
    std::mt19937_64 rng(7);
    std::vector<TwPair> tw(N);
    for (auto& t : tw) {
        t.w = rng() % q;
        t.ws = shoup_c(t.w, q);
    }
    TwPair* d_tw = nullptr;
    CK(hipMalloc(&d_tw, N * sizeof(TwPair)));
    CK(hipMemcpy(d_tw, tw.data(), N * sizeof(TwPair), hipMemcpyHostToDevice));
    constexpr int NP = 7;   // cfg3: L = 3 ciphertext + K = 4 auxiliary primes (same q here: timing only)
    std::vector<PrimeConst> pc(NP);
    for (auto& P : pc) {
        P = PrimeConst{};
        P.q = q; P.two_q = 2 * q; P.mu64 = (u64)(~(u128)0 / q); P.bar_s = 60;
        P.n_inv = rng() % q; P.n_inv_s = shoup_c(P.n_inv, q);
        P.last_w = rng() % q; P.last_ws = shoup_c(P.last_w, q);
        P.tw_fwd = d_tw; P.tw_inv = d_tw;
    }
    PrimeConst* d_pc = nullptr;
    CK(hipMalloc(&d_pc, NP * sizeof(PrimeConst)));
    CK(hipMemcpy(d_pc, pc.data(), NP * sizeof(PrimeConst), hipMemcpyHostToDevice));

    // forward: one cfg3 extension launch (8192 polynomials)
    const long polys = 8192;
    u64 *src = nullptr, *dst = nullptr;
    CK(hipMalloc(&src, polys * N * sizeof(u64)));
    CK(hipMalloc(&dst, polys * N * sizeof(u64)));
    CK(hipMemset(src, 0x11, polys * N * sizeof(u64)));   // < q in every word
    NttBatch nb{};
    nb.src = src; nb.src_item_stride = N; nb.dst = dst; nb.dst_item_stride = N;
    nb.ppi = 1; nb.prime_base = 0; nb.period = 1;
    // tensor: one cfg3 chunk (512 products x 3 components x 7 primes)
    const long items = 512;
    u64 *A = nullptr, *B = nullptr, *E = nullptr, *Tt = nullptr;
    CK(hipMalloc(&A, items * 2 * 3 * N * sizeof(u64)));
    CK(hipMalloc(&B, items * 2 * 3 * N * sizeof(u64)));
    CK(hipMalloc(&E, items * 4 * 4 * N * sizeof(u64)));
    CK(hipMalloc(&Tt, items * 3 * NP * N * sizeof(u64)));
    CK(hipMemset(A, 0x11, items * 2 * 3 * N * sizeof(u64)));
    CK(hipMemset(B, 0x22, items * 2 * 3 * N * sizeof(u64)));
    CK(hipMemset(E, 0x33, items * 4 * 4 * N * sizeof(u64)));
    Operands op{};
    op.a = A; op.a_stride = 2 * 3 * N; op.b = B; op.b_stride = 2 * 3 * N;
    const long tblocks = items * 3 * NP;

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1000.0 * ms / reps;   // us per launch
    };
    const double f_full = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<LOGN, 0>), dim3(polys), dim3(256), 0, 0, nb, d_pc); });
    const double f_comp = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<LOGN, 1>), dim3(polys), dim3(256), 0, 0, nb, d_pc); });
    const double f_mem = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<LOGN, 2>), dim3(polys), dim3(256), 0, 0, nb, d_pc); });
    const double f_stag = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<LOGN, 3>), dim3(polys), dim3(256), 0, 0, nb, d_pc); });
    const double t_full = timed([&] {
        hipLaunchKernelGGL((ntt_inv_tensor_kernel<LOGN, true, true, 0>), dim3(tblocks), dim3(256), 0, 0, op, E, Tt, 3, 4, d_pc, 1, 0);
    });
    const double t_comp = timed([&] {
        hipLaunchKernelGGL((ntt_inv_tensor_kernel<LOGN, true, true, 1>), dim3(tblocks), dim3(256), 0, 0, op, E, Tt, 3, 4, d_pc, 1, 0);
    });
    const double t_mem = timed([&] {
        hipLaunchKernelGGL((ntt_inv_tensor_kernel<LOGN, true, true, 2>), dim3(tblocks), dim3(256), 0, 0, op, E, Tt, 3, 4, d_pc, 1, 0);
    });
    const double t_stag = timed([&] {
        hipLaunchKernelGGL((ntt_inv_tensor_kernel<LOGN, true, true, 3>), dim3(tblocks), dim3(256), 0, 0, op, E, Tt, 3, 4, d_pc, 1, 0);
    });
    const double fbytes = 16.0 * N * polys, tbytes = 7.0 * 8 * N * items * NP;
    // n = 8192 forward (cfg5's launches hold 512-640 polynomials against 512 resident blocks): full,
    // compute only, memory only, and the second block of each CU started late by a swept delay
    constexpr int N13 = 1 << 13;
    std::vector<TwPair> tw13(N13);
    for (auto& t : tw13) {
        t.w = rng() % q;
        t.ws = shoup_c(t.w, q);
    }
    TwPair* d_tw13 = nullptr;
    CK(hipMalloc(&d_tw13, N13 * sizeof(TwPair)));
    CK(hipMemcpy(d_tw13, tw13.data(), N13 * sizeof(TwPair), hipMemcpyHostToDevice));
    for (auto& P : pc) P.tw_fwd = P.tw_inv = d_tw13;
    CK(hipMemcpy(d_pc, pc.data(), NP * sizeof(PrimeConst), hipMemcpyHostToDevice));
    std::printf("{\"n8192\": [");
    for (long p13 : {512L, 576L, 1024L}) {
        nb.src_item_stride = N13; nb.dst_item_stride = N13;
        const double a = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<13, 0>), dim3(p13), dim3(512), 0, 0, nb, d_pc); });
        const double c = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<13, 1>), dim3(p13), dim3(512), 0, 0, nb, d_pc); });
        const double m = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<13, 2>), dim3(p13), dim3(512), 0, 0, nb, d_pc); });
        std::printf("%s{\"polys\": %ld, \"full_us\": %.2f, \"frac\": %.3f, \"compute_only_us\": %.2f, \"memory_only_us\": %.2f, \"stagger\": {",
                    p13 == 512 ? "" : ", ", p13, a, 16.0 * N13 * p13 / (a * 1e3) / 8000.0, c, m);
        for (int sl : {0, 2, 4, 6, 8, 12, 16}) {
            CK(hipMemcpyToSymbol(HIP_SYMBOL(exacto_probe_sleeps), &sl, sizeof(int)));
            const double t = timed([&] { hipLaunchKernelGGL((ntt_fwd_pin_kernel<13, 3>), dim3(p13), dim3(512), 0, 0, nb, d_pc); });
            std::printf("%s\"%d\": %.2f", sl ? ", " : "", sl, t);
        }
        std::printf("}}");
        const int off = -1;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(exacto_probe_sleeps), &off, sizeof(int)));
    }
    std::printf("]}\n");
    std::printf("{\"fwd_pin_polys\": %ld, \"fwd_full_us\": %.2f, \"fwd_compute_only_us\": %.2f, \"fwd_memory_only_us\": %.2f, "
                "\"fwd_staggered_us\": %.2f, \"fwd_full_GBs\": %.1f, \"fwd_compute_over_full\": %.3f, "
                "\"tensor12_blocks\": %ld, \"tensor_full_us\": %.2f, \"tensor_compute_only_us\": %.2f, "
                "\"tensor_no_transform_us\": %.2f, \"tensor_staggered_us\": %.2f, "
                "\"tensor_full_GBs\": %.1f, \"tensor_compute_over_full\": %.3f, \"reps\": %d}\n",
                polys, f_full, f_comp, f_mem, f_stag, fbytes / (f_full * 1e3), f_comp / f_full, tblocks, t_full, t_comp,
                t_mem, t_stag, tbytes / (t_full * 1e3), t_comp / t_full, reps);
    return 0;
}
