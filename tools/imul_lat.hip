// Microbenchmark: dependent-chain latency (one wave per CU, one chain) of the integer ops the
// NTT butterfly is built from, and of a VALU->SGPR carry handoff (gfx950).  Cycles via s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 1024
template <int OP>
__global__ void k(uint64_t* out, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = seed * 3 + 1;
    uint64_t acc = a;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s40", "s41");
            if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
            if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b));
            if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
            if (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc) : "v"((uint64_t)b));
            if (OP == 5) asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %1\n\ts_nop 1\n\tv_addc_co_u32_e64 %0, s[40:41], %0, %1, s[40:41]\n\ts_nop 1" : "+v"(a) : "v"(b) : "s40", "s41");
            if (OP == 6) asm volatile("s_nop 1\n\ts_nop 1" ::);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (acc == 12345 && a == 7) out[0] = 1;
}

template <int OP>
void run(const char* name, uint64_t* d, int cus) {
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(64), 0, 0, d, 1u);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<OP>, dim3(cus), dim3(64), 0, 0, d, 1u);
    uint64_t h[4];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-26s %.2f memtime-cycles per dependent op\n", name, (double)h[1] / (ITERS * 8.0));
}

int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    uint64_t* d; hipMalloc(&d, sizeof(uint64_t) * cus);
    run<0>("v_mad_u64_u32", d, cus);
    run<1>("v_mul_lo_u32", d, cus);
    run<2>("v_mul_hi_u32", d, cus);
    run<3>("v_add_u32", d, cus);
    run<4>("v_lshl_add_u64", d, cus);
    run<5>("add_co+nop1+addc+nop1 (pair)", d, cus);
    run<6>("s_nop1 x2 (pair)", d, cus);
    return 0;
}
