// Single-purpose reproducer for DESIGN.md §3/§6: is a same-stream runtime device-to-device copy
// (hipMemcpyAsync) into a block of a stream-ordered memory pool always seen by the next kernel on
// that stream?  Round 3 replaced every such copy in the library with a copy kernel after the C++
// host-API test's n = 16 bootstrap returned the previous call's output about one suite run in three.
//
// Each iteration replays the failing call's sequence on one non-blocking stream, as
// exacto_bfv_bootstrap did it (host_call -> exacto_bfv_bootstrap_dev):
//   1. H2D upload of the iteration's input (pageable host memory) into a hipMalloc staging buffer,
//      hipStreamSynchronize                                           (host_call)
//   2. a block from the context's own pool (hipMemPoolCreate, release threshold UINT64_MAX),
//      hipMallocFromPoolAsync on the stream                           (Scratch::alloc)
//   3. the copy staging -> block: hipMemcpyAsync D2D (mode "memcpy"), a copy kernel ("kernel"), or
//      hipMemcpyAsync into a hipMalloc block instead of a pool block ("memcpy_nopool")
//   4. a kernel that reads the block and records whether it saw this iteration's input
//   5. a 4-byte D2H hipMemcpyAsync + hipStreamSynchronize             (the bootstrap's flags read)
//   6. hipFreeAsync of the block, hipStreamSynchronize                (Scratch dtor, Drain)
// Every block is handed out again at the same address (the pool keeps it mapped), so a copy that the
// kernel does not see leaves the PREVIOUS iteration's input in place, exactly the recorded symptom.
//
// Output: one line per (mode, size): iterations, mismatches, first mismatching iteration.
// Build: hipcc --offload-arch=gfx950 -O2 tools/d2d_repro.cpp -o build/d2d_repro
// Run:   build/d2d_repro [iterations]      (default 20000 per case; a few seconds on one GPU)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void copy_kernel(uint64_t* dst, const uint64_t* src, long words) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// one block: every thread checks a strided part of the block against the expected pattern, the
// block's verdict (plain vector stores, no atomics) goes to seen[0..1]
__global__ void check_kernel(const uint64_t* blk, long words, uint64_t tag, uint32_t* seen) {
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    int mine = 0;
    for (long i = threadIdx.x; i < words; i += blockDim.x)
        mine |= blk[i] != (tag * 0x9E3779B97F4A7C15ull ^ (uint64_t)i);
    if (mine) bad = 1;   // benign race: every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) {
        seen[0] = bad ? 0u : 1u;
        seen[1] = (uint32_t)(blk[0] == ((tag - 1) * 0x9E3779B97F4A7C15ull));   // previous iteration's value
    }
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
    uint32_t* seen = nullptr;
    CK(hipMalloc(&seen, 64));
    const char* modes[] = {"memcpy", "kernel", "memcpy_nopool"};
    const size_t sizes[] = {256, 4096, 1 << 20};   // 256 B: the n = 16 trivial ciphertext [2][1][16]
    int total_bad = 0;
    for (const char* mode : modes) {
        for (size_t bytes : sizes) {
            const long words = (long)(bytes / 8);
            uint64_t* stage = nullptr;
            CK(hipMalloc(&stage, bytes));
            uint64_t* fixed = nullptr;
            if (std::strcmp(mode, "memcpy_nopool") == 0) CK(hipMalloc(&fixed, bytes));
            std::vector<uint64_t> host(words);
            int bad = 0, stale = 0, first = -1;
            void* prev_addr = nullptr;
            int moved = 0;
            for (int it = 1; it <= iters; ++it) {
                for (long i = 0; i < words; ++i) host[i] = (uint64_t)it * 0x9E3779B97F4A7C15ull ^ (uint64_t)i;
                CK(hipMemcpyAsync(stage, host.data(), bytes, hipMemcpyHostToDevice, s));   // 1
                CK(hipStreamSynchronize(s));
                uint64_t* blk = fixed;
                if (!blk) CK(hipMallocFromPoolAsync((void**)&blk, bytes, pool, s));          // 2
                if (prev_addr && prev_addr != blk) ++moved;
                prev_addr = blk;
                if (std::strcmp(mode, "kernel") == 0)                                      // 3
                    hipLaunchKernelGGL(copy_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, blk, stage,
                                       words);
                else
                    CK(hipMemcpyAsync(blk, stage, bytes, hipMemcpyDeviceToDevice, s));
                hipLaunchKernelGGL(check_kernel, dim3(1), dim3(256), 0, s, blk, words, (uint64_t)it, seen);   // 4
                CK(hipGetLastError());
                uint32_t h[2] = {0, 0};
                CK(hipMemcpyAsync(h, seen, 8, hipMemcpyDeviceToHost, s));                 // 5
                CK(hipStreamSynchronize(s));
                if (!fixed) CK(hipFreeAsync(blk, s));                                       // 6
                CK(hipStreamSynchronize(s));
                if (!h[0]) {
                    ++bad;
                    stale += h[1];
                    if (first < 0) first = it;
                }
            }
            std::printf("mode=%-14s bytes=%-8zu iters=%d mismatches=%d stale_previous=%d first=%d block_moved=%d\n",
                        mode, bytes, iters, bad, stale, first, moved);
            std::fflush(stdout);
            total_bad += bad;
            CK(hipFree(stage));
            if (fixed) CK(hipFree(fixed));
        }
    }
    CK(hipFree(seen));
    CK(hipMemPoolDestroy(pool));
    CK(hipStreamDestroy(s));
    std::printf("total_mismatches=%d\n", total_bad);
    return 0;
}
