// Single-purpose reproducer for DESIGN.md §3: can a kernel that reads a buffer through the SCALAR
// data cache (s_load: hipcc emits it when every lane reads the same address) see an older value of
// a block that a previous kernel on the same stream rewrote with vector stores?
//
// Round 1's n = 16 NTT kernels loaded their polynomial with s_load_dwordx16 and returned a pool
// block's previous contents; round 3's n = 16 bootstrap returned the previous call's result.  This
// replays the pattern on one non-blocking stream, per iteration it:
//   1. writer<<<8 blocks>>>: every lane stores tag(it) into the 32-word block B (vector stores)
//   2. reader<<<8 blocks>>>: reads B through scalar loads (mode "scalar": the address is uniform,
//      s_load_dwordx16 x2) or through vector loads (mode "vector": the lane index is opaque to the
//      compiler) and stores, per block, whether all 32 words equal tag(it) (vector stores)
//   3. a 32-byte D2H copy of the verdicts + hipStreamSynchronize
// B is either a fixed hipMalloc block or a block of a stream-ordered pool (hipMallocFromPoolAsync /
// hipFreeAsync every iteration: the same address comes back), as the library's Scratch.
// Output: one line per (mode, memory): iterations, stale reads (a block saw tag(it - 1)), other
// mismatches.  Build: hipcc --offload-arch=gfx950 -O2 tools/kcache_repro.cpp -o build/kcache_repro
// (tools/r4_d2d.sh also checks that the scalar reader really issues s_load).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int WORDS = 32;

__device__ __forceinline__ uint64_t tag(uint64_t it) { return it * 0x9E3779B97F4A7C15ull; }

__global__ void writer(uint64_t* blk, uint64_t it) {
    if (threadIdx.x < WORDS) blk[threadIdx.x] = tag(it) ^ threadIdx.x;
}

// every lane reads the same 32 words: uniform addresses, so hipcc uses scalar loads
__global__ void reader_scalar(const uint64_t* __restrict__ blk, uint64_t it, uint32_t* verdict) {
    uint32_t ok = 1, prev = 1;
#pragma unroll
    for (int k = 0; k < WORDS; ++k) {
        const uint64_t w = blk[k];
        ok &= w == (tag(it) ^ (uint64_t)k);
        prev &= w == (tag(it - 1) ^ (uint64_t)k);
    }
    if (threadIdx.x == 0) verdict[blockIdx.x] = ok ? 1u : (prev ? 2u : 3u);
}

// the same reads through vector loads (a lane index hipcc cannot prove uniform)
__global__ void reader_vector(const uint64_t* __restrict__ blk, uint64_t it, uint32_t* verdict) {
    int z = 0;
    asm volatile("" : "+v"(z));
    uint32_t ok = 1, prev = 1;
#pragma unroll
    for (int k = 0; k < WORDS; ++k) {
        const uint64_t w = blk[k + z];
        ok &= w == (tag(it) ^ (uint64_t)k);
        prev &= w == (tag(it - 1) ^ (uint64_t)k);
    }
    if (threadIdx.x == 0) verdict[blockIdx.x] = ok ? 1u : (prev ? 2u : 3u);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = 0;
    hipMemPool_t pool;
    CK(hipMemPoolCreate(&pool, &props));
    uint64_t thr = ~0ull;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    uint32_t* verdict = nullptr;
    CK(hipMalloc(&verdict, 8 * sizeof(uint32_t)));
    uint64_t* fixed = nullptr;
    CK(hipMalloc(&fixed, WORDS * sizeof(uint64_t)));
    long total_bad = 0;
    for (const char* mode : {"scalar", "vector"}) {
        for (const char* mem : {"fixed", "pool"}) {
            const bool sc = std::strcmp(mode, "scalar") == 0, pl = std::strcmp(mem, "pool") == 0;
            long stale = 0, other = 0;
            int first = -1;
            for (int it = 1; it <= iters; ++it) {
                uint64_t* blk = fixed;
                if (pl) CK(hipMallocFromPoolAsync((void**)&blk, WORDS * sizeof(uint64_t), pool, s));
                hipLaunchKernelGGL(writer, dim3(8), dim3(64), 0, s, blk, (uint64_t)it);
                if (sc) hipLaunchKernelGGL(reader_scalar, dim3(8), dim3(64), 0, s, blk, (uint64_t)it, verdict);
                else hipLaunchKernelGGL(reader_vector, dim3(8), dim3(64), 0, s, blk, (uint64_t)it, verdict);
                CK(hipGetLastError());
                uint32_t h[8];
                CK(hipMemcpyAsync(h, verdict, sizeof(h), hipMemcpyDeviceToHost, s));
                if (pl) CK(hipFreeAsync(blk, s));
                CK(hipStreamSynchronize(s));
                for (int b = 0; b < 8; ++b) {
                    if (h[b] == 1) continue;
                    if (h[b] == 2) ++stale; else ++other;
                    if (first < 0) first = it;
                }
            }
            std::printf("mode=%s mem=%s iters=%d stale_blocks=%ld other_bad_blocks=%ld first=%d\n", mode, mem, iters,
                        stale, other, first);
            std::fflush(stdout);
            total_bad += stale + other;
        }
    }
    std::printf("total_bad=%ld\n", total_bad);
    CK(hipFree(verdict));
    CK(hipFree(fixed));
    CK(hipMemPoolDestroy(pool));
    CK(hipStreamDestroy(s));
    return 0;
}
