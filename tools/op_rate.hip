// Microbenchmark: issue cost of the gfx950 VALU instructions an NTT butterfly can be built from.
// Each wave runs 8 independent chains of one instruction, 8 waves per SIMD; the result is wave
// instructions per ns per CU and, from it, cycles per wave-instruction per SIMD at the clock the
// caller names (default 2.4 GHz; pass the clock measured alongside to get true cycles).
// Build: hipcc --offload-arch=gfx950 -O3 tools/op_rate.hip -o tools/op_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define ITERS 2048
typedef uint64_t u64;
typedef uint32_t u32;

// one instruction on chain i: 32-bit state a[i], 64-bit state w[i], constants b (VGPR), s (SGPR)
#define OPS(X)                                                                                          \
    X(0, "v_mad_u64_u32 (vcc)", asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(b)))  \
    X(1, "v_mad_u64_u32 (s sdst)", asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(b) : "s40", "s41")) \
    X(2, "v_mul_lo_u32", asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))               \
    X(3, "v_mul_hi_u32", asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))               \
    X(4, "v_add_u32", asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))                     \
    X(5, "v_add3_u32", asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))               \
    X(6, "v_lshl_add_u64", asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[i]) : "v"((u64)b)))   \
    X(7, "v_add_co_u32 (vcc)", asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b)))    \
    X(8, "v_add_co_u32_e64 s", asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %1" : "+v"(a[i]) : "v"(b) : "s40", "s41")) \
    X(9, "v_addc_co_u32_e64 s", asm volatile("v_addc_co_u32_e64 %0, s[40:41], %0, %1, s[40:41]" : "+v"(a[i]) : "v"(b) : "s40", "s41")) \
    X(10, "v_cndmask_b32_e64 s", asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a[i]) : "v"(b) : "s40", "s41")) \
    X(11, "v_cndmask_b32 vcc", asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b)))   \
    X(12, "v_cmp_le_u64_e64 s", asm volatile("v_cmp_le_u64_e64 s[40:41], %0, %1" :: "v"(w[i]), "v"((u64)b) : "s40", "s41")) \
    X(13, "v_cmp_le_u32_e64 s", asm volatile("v_cmp_le_u32_e64 s[40:41], %0, %1" :: "v"(a[i]), "v"(b) : "s40", "s41")) \
    X(14, "v_mov_b32", asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(b)))                       \
    X(15, "v_lshrrev_b32", asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])))                     \
    X(16, "v_alignbit_b32", asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b)))        \
    X(17, "v_lshlrev_b64", asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(w[i])))                      \
    X(18, "v_mov_b64", asm volatile("v_mov_b64 %0, %1" : "=v"(w[i]) : "v"((u64)b)))                   \
    X(19, "v_mad_u32_u24", asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))        \
    X(20, "v_mad_i64_i32", asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(b))) \
    X(21, "v_sub_co_u32_e64 s", asm volatile("v_sub_co_u32_e64 %0, s[40:41], %0, %1" : "+v"(a[i]) : "v"(b) : "s40", "s41")) \
    X(22, "v_and_b32", asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))                    \
    X(23, "v_bfi_b32", asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))                \
    X(24, "v_pk_mov_b32", asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(w[i]) : "v"((u64)b))) \
    X(25, "v_mul_hi_u32_u24", asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b)))      \
    X(26, "v_lshl_or_b32", asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b)))         \
    X(27, "v_sub_u32", asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))                    \
    X(28, "v_max_u32", asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))                    \
    X(29, "v_min_u32", asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))                    \
    X(30, "v_mul_u32_u24", asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b)))            \
    X(31, "v_fma_f64", asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(w[i]) : "v"((u64)b)))           \
    X(32, "v_mul_f64", asm volatile("v_mul_f64 %0, %0, %1" : "+v"(w[i]) : "v"((u64)b)))               \
    X(33, "v_cvt_f64_u32", asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(w[i]) : "v"(a[i])))             \
    X(34, "v_cvt_u32_f64", asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(a[i]) : "v"(w[i])))             \
    X(35, "v_fma_f32", asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))                \
    X(36, "v_pk_fma_f32", asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(w[i]) : "v"((u64)b)))     \
    X(37, "v_mul_lo_u16", asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))             \
    X(38, "v_pk_mul_lo_u16", asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))        \
    X(39, "v_dot2_u32_u16", asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b)))      \
    X(40, "PAIR cmp+cndmask vcc", asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc")) \
    X(41, "PAIR cmp+cndmask s", asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a[i]) : "v"(b) : "s40", "s41")) \
    X(42, "PAIR sub+min", asm volatile("v_sub_u32 %0, %0, %1\n\tv_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b))) \
    X(43, "v_cndmask_b32 vcc (set)", asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b)))     \
    X(44, "PAIR sub_co+subb vcc", asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_subb_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc")) \
    X(45, "PAIR sub_co+subb s", asm volatile("v_sub_co_u32_e64 %0, s[40:41], %0, %1\n\tv_subb_co_u32_e64 %0, s[40:41], %0, %1, s[40:41]" : "+v"(a[i]) : "v"(b) : "s40", "s41"))

template <int OP>
__global__ void __launch_bounds__(256) k(u32* out, u32 seed) {
    u32 a[8], b = seed + threadIdx.x;
    u64 w[8];
    for (int i = 0; i < 8; ++i) { a[i] = seed * (i + 3) + threadIdx.x; w[i] = a[i]; }
    if (OP == 43) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a[0]), "v"(b) : "vcc");
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#define CASE(n, name, stmt) if (OP == n) { stmt; }
            OPS(CASE)
#undef CASE
        }
    }
    u64 s = 0;
    for (int i = 0; i < 8; ++i) s += w[i] + a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (u32)s;
}

template <int OP>
void run(const char* name, u32* d, int cus, double ghz) {
    const int blocks = cus * 8, threads = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = 5.0 * blocks * (threads / 64) * ITERS * 8.0;
    const double per_cu_per_ns = wave_instr / (ms * 1e6) / cus;
    printf("%-24s %8.3f ms  %.3f wave-instr/ns/CU  %.2f cycles/wave-instr/SIMD @%.2fGHz\n", name, ms,
           per_cu_per_ns, 4.0 * ghz / per_cu_per_ns, ghz);
}

int main(int argc, char** argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("%s CUs=%d clock=%d kHz\n", p.gcnArchName, cus, p.clockRate);
    u32* d;
    hipMalloc(&d, sizeof(u32) * cus * 8 * 256);
#define RUN(n, name, stmt) run<n>(name, d, cus, ghz);
    OPS(RUN)
#undef RUN
    return 0;
}
