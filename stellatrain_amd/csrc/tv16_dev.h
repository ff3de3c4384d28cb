// tv16_dev.h -- device helpers shared by the thresholdv16 scan (tv16.hip) and
// its regime-B heap fill (tv16fill.hip).  gfx950 only.
#pragma once

#include <algorithm>

#include "ws.h"
#include "wire_dev.h"

namespace stg {
namespace tv16 {

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

using ::stg::spin_expired;  // common.h: every bounded wait gives up after 200 ms

__device__ __forceinline__ uint32_t bitlen(uint32_t x) { return x ? 32u - __clz(x) : 0u; }

// Wave-uniform values read from memory or LDS: move them to SGPRs.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ float uni(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

// lane id, opaque to the compiler (not hoisted into a live register)
__device__ __forceinline__ uint32_t flane() {
    uint32_t x;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
    return x;
}
__device__ __forceinline__ uint64_t below_mask(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// LDS hand-offs between the waves of one workgroup: the writer drains its
// LDS operations before the flag; LDS executes one wave's operations in order.
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Tree sum of one 16-float line held as a float4 by each lane of a quad
// (lanes 0,1: floats 0..7; lanes 2,3: floats 8..15): p = |x_i| + |x_{i+4}|,
// h = (p0+p1)+(p2+p3) per half, S = h_lo + h_hi  (thresholdv16.cpp:57-73,143).
__device__ __forceinline__ float quad_line_sum(const float4 v) {
    const float ax = fabsf(v.x), ay = fabsf(v.y), az = fabsf(v.z), aw = fabsf(v.w);
    const float px = ax + dpp_f<QP_XOR1>(ax);
    const float py = ay + dpp_f<QP_XOR1>(ay);
    const float pz = az + dpp_f<QP_XOR1>(az);
    const float pw = aw + dpp_f<QP_XOR1>(aw);
    const float h = (px + py) + (pz + pw);
    return h + dpp_f<QP_XOR2>(h);
}

// The same sum by one lane from memory (bit-identical: the same adds in the
// same order; IEEE addition is commutative).
__device__ __forceinline__ float lane_line_sum(const float *p) {
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    const float4 a = p4[0], b = p4[1], c = p4[2], e = p4[3];
    const float lo = ((fabsf(a.x) + fabsf(b.x)) + (fabsf(a.y) + fabsf(b.y))) +
                     ((fabsf(a.z) + fabsf(b.z)) + (fabsf(a.w) + fabsf(b.w)));
    const float hi = ((fabsf(c.x) + fabsf(e.x)) + (fabsf(c.y) + fabsf(e.y))) +
                     ((fabsf(c.z) + fabsf(e.z)) + (fabsf(c.w) + fabsf(e.w)));
    return lo + hi;
}

// One lane writes `len` (<= 16) pairs of the line at `pos` to slot `off`.
template <typename D>
__device__ __forceinline__ void emit_line(const D &d, bool vec, uint32_t pos, uint32_t off, uint32_t len) {
    if (vec && len == 16) {
        const float4 *s4 = reinterpret_cast<const float4 *>(d.src + pos);
        const uint32_t b = pos + (uint32_t)d.idx_offset;
        const float4 x0 = s4[0], x1 = s4[1], x2 = s4[2], x3 = s4[3];
        put_pair4(d, off, b, x0);
        put_pair4(d, off + 4, b + 4, x1);
        put_pair4(d, off + 8, b + 8, x2);
        put_pair4(d, off + 12, b + 12, x3);
    } else {
        for (uint32_t i = 0; i < len; ++i) {
            put_pair(d, off + i, pos + i + (uint32_t)d.idx_offset, d.src[(size_t)pos + i]);
        }
    }
}

template <typename D>
__device__ __forceinline__ bool aligned16(const D &d) {
    return ((reinterpret_cast<uintptr_t>(d.src) | reinterpret_cast<uintptr_t>(d.idx) |
             reinterpret_cast<uintptr_t>(d.val)) & 15u) == 0;
}

// `n16` 16-byte words from global memory (read through to L2: sc1) into LDS
// at `dst`, in chunks of 64 (the destination must hold whole chunks); waits.
__device__ __forceinline__ void gather16(const void *src, uint32_t n16, void *dst) {
    const uint32_t lane = flane();
    for (uint32_t c = 0; c * 64 < n16; ++c) {
        const uint32_t v = std::min(c * 64 + lane, n16 - 1);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char *>(src) + (size_t)v * 16,
                                         reinterpret_cast<char *>(dst) + c * 1024, 16, 0, 16 /* sc1 */);
    }
    vm_drain();
}

// Heap positions of libstdc++'s make_heap (node q = pos + 1 >= 1).
__device__ __forceinline__ uint32_t depth_of(uint32_t q) { return 31u - __clz(q); }
// right-first pre-order key of heap position pos (< 2^20 - 1): ancestors
// first, then the right subtree before the left one
__device__ __forceinline__ uint32_t rf_key(uint32_t pos) {
    const uint32_t q = pos + 1, d = depth_of(q);
    const uint32_t path = q - (1u << d);
    const uint32_t inv = ~path & ((1u << d) - 1u);
    return ((inv << (19u - d)) << 5) | d;
}
__device__ __forceinline__ bool is_desc(uint32_t q, uint32_t qt) {  // heap node q (pos + 1) below node qt
    const uint32_t dp = depth_of(q), dt = depth_of(qt);
    return dp > dt && (q >> (dp - dt)) == qt;
}

}  // namespace tv16
}  // namespace stg
