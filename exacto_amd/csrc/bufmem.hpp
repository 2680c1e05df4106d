// Polynomial loads and stores through a buffer resource (one residue polynomial per workgroup).
// The transforms move their 16 values per thread at positions tid + k n/16: with a 64-bit flat
// address per access hipcc spends a 64-bit add (2 VALU) on every pair of them once the constant
// offset k n/16 * 8 outgrows the instruction's 12-bit immediate.  A buffer access takes a 32-bit
// per-lane offset (tid * elem, one VGPR for all 16) and the constant part in an SGPR, so the
// addressing costs no VALU at all.  The descriptor is built from wave-uniform values (the block's
// polynomial base); num_records bounds every access to that polynomial.
#pragma once
#include "arith.hpp"

namespace exacto {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// base must be the same in every lane of the wave (the block's polynomial).  The readfirstlane
// makes that provable to hipcc where its uniformity analysis gives up (values computed after a
// divergent early return): otherwise it wraps every access in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t poly_rsrc(const void* base, int bytes) {
    const unsigned long long a = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    void* p = (void*)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, bytes, 0x00020000);
}

__device__ __forceinline__ u64 buf_ld64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

__device__ __forceinline__ void buf_st64(__amdgpu_buffer_rsrc_t r, u64 x, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, x), r, voff, soff, 0);
}

__device__ __forceinline__ uint32_t buf_ld32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}

__device__ __forceinline__ void buf_st32(__amdgpu_buffer_rsrc_t r, uint32_t x, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32(x, r, voff, soff, 0);
}

}  // namespace exacto

namespace exacto {

// One polynomial's 64-bit accesses at byte offsets voff (per lane) + soff (uniform): buffer
// instructions (BUF) or flat ones at base + voff + soff (the A/B form, tools/build_variants.sh)
template <bool BUF>
struct PolyIO {
    char* p;
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ PolyIO(const void* base, int bytes)
        : p((char*)const_cast<void*>(base)), r(poly_rsrc(base, bytes)) {}
    __device__ __forceinline__ u64 ld64(int voff, int soff) const {
        if constexpr (BUF) return buf_ld64(r, voff, soff);
        else return *reinterpret_cast<const u64*>(p + voff + soff);
    }
    __device__ __forceinline__ void st64(u64 x, int voff, int soff) const {
        if constexpr (BUF) buf_st64(r, x, voff, soff);
        else *reinterpret_cast<u64*>(p + voff + soff) = x;
    }
};

}  // namespace exacto
