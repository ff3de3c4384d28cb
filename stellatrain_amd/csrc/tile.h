// tile.h -- 8192-element streaming tiles with in-order compaction ranks.
//
// A tile is 256 threads x 8 float4 (32 KiB).  Float4 f of the tile is
// f = u * 256 + threadIdx.x, so each wave-instruction reads 1 KiB contiguous
// (fully coalesced) and element order inside the tile is (u, wave, lane, j).
#pragma once

#include "ws.h"

namespace stg {

constexpr uint32_t TILE_U = 8;  // float4 per thread per tile

template <bool VEC>
__device__ __forceinline__ void load_tile(const float *__restrict__ a, size_t m, size_t base, uint32_t last_mask,
                                          float4 (&v)[TILE_U]) {
    // a whole, aligned tile with no partial float: all TILE_U loads issued
    // before any is used (a per-load bounds test makes the compiler wait for
    // each load in turn: TILE_U serial HBM round trips)
    if (VEC && base + TV_TILE <= m && (last_mask == 0xffffffffu || base + TV_TILE < m)) {
        const float4 *p = reinterpret_cast<const float4 *>(a + base) + threadIdx.x;
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) v[u] = p[u * STG_WG];
        return;
    }
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
        if (VEC && e + 3 < m) {
            v[u] = *reinterpret_cast<const float4 *>(a + e);
        } else {
            float x[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = (e + j < m) ? a[e + j] : 0.f;
            v[u] = make_float4(x[0], x[1], x[2], x[3]);
        }
        if (last_mask != 0xffffffffu) {
            // partial last float (top-k's byte-count memcpy): keep only its low bytes
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (e + j == m - 1) {
                    float *c = reinterpret_cast<float *>(&v[u]) + j;
                    *c = u2f(f2u(*c) & last_mask);
                }
        }
    }
}

__device__ __forceinline__ float comp(const float4 &v, int j) {
    return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// In-order ranks of the flagged elements of a tile.  `q` holds one bit per
// (u, j) (bit u*4+j).  Returns the tile-local slot of each flagged element
// in `slot` (same bit layout) and the tile total.  s_wt: TILE_U*STG_WAVES+1 words.
__device__ __forceinline__ void tile_ranks(uint32_t q, uint32_t (&slot)[TILE_U * 4], uint32_t *s_wt,
                                           uint32_t *total) {
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t below[TILE_U];
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        uint32_t bl = 0, wt = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint64_t b = __ballot((q >> (u * 4 + j)) & 1u);
            bl += (uint32_t)__popcll(b & lt);
            wt += (uint32_t)__popcll(b);
        }
        below[u] = bl;
        if (lane == 0) s_wt[u * STG_WAVES + wave] = wt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t i = 0; i < TILE_U * STG_WAVES; ++i) { const uint32_t x = s_wt[i]; s_wt[i] = acc; acc += x; }
        s_wt[TILE_U * STG_WAVES] = acc;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        uint32_t r = s_wt[u * STG_WAVES + wave] + below[u];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            slot[u * 4 + j] = r;
            r += (q >> (u * 4 + j)) & 1u;
        }
    }
    *total = s_wt[TILE_U * STG_WAVES];
    __syncthreads();
}

}  // namespace stg
