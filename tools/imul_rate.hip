// Microbenchmark: issue rate of the integer ops the NTT butterfly is built from (gfx950).
// Each wave runs 8 independent chains of one instruction; rate = instr / (time * CUs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
template <int OP>
__global__ void k(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b = seed + threadIdx.x;
    uint64_t acc[8];
    for (int i = 0; i < 8; ++i) { a[i] = seed * (i + 3) + threadIdx.x; acc[i] = a[i]; }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a[i]), "v"(b));
            if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"((uint64_t)b));
            if (OP == 5) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 6) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[i]) : "v"((uint64_t)b));
            if (OP == 7) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b));
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i] + a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

template <int OP>
void run(const char* name, uint32_t* d, int cus) {
    const int blocks = cus * 8, threads = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double wave_instr = 5.0 * blocks * (threads / 64) * ITERS * 8.0;
    double per_cu_per_ns = wave_instr / (ms * 1e6) / cus;
    // cycles per wave-instruction per SIMD at 2.4 GHz: 4 SIMDs per CU
    printf("%-18s %8.3f ms  %.3f wave-instr/ns/CU  => %.2f cycles per wave-instr per SIMD @2.4GHz\n", name, ms,
           per_cu_per_ns, 4.0 * 2.4 / per_cu_per_ns);
}

int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    printf("%s CUs=%d clock=%d kHz\n", p.gcnArchName, cus, p.clockRate);
    uint32_t* d; hipMalloc(&d, sizeof(uint32_t) * cus * 8 * 256);
    run<0>("v_mad_u64_u32", d, cus);
    run<1>("v_mul_lo_u32", d, cus);
    run<2>("v_mul_hi_u32", d, cus);
    run<3>("v_add_u32", d, cus);
    run<4>("v_lshl_add_u64", d, cus);
    run<5>("v_mul_u32_u24", d, cus);
    run<6>("v_fma_f64", d, cus);
    run<7>("v_sub_co_u32", d, cus);
    return 0;
}
