// select.h -- the radix select's per-level pick, run by the last workgroup
// of whichever pass filled the level's histogram (select.hip, topk.hip).
#pragma once

#include "ws.h"

namespace stg {

// The bin holding the rank, counting from the top bin, by one workgroup of NT
// threads: each thread sums its (top-down) bins, a workgroup scan finds the
// thread whose range holds the rank, that thread walks its bins.  It also
// zeroes the histogram for the next level (and the next select: the table is
// zero at allocation and after every complete select).  The first level
// (SHIFT + NBITS == 31) takes the rank from the argument and starts the prefix
// afresh.  Run by the last workgroup of the pass that filled the histogram
// (the other workgroups' bin atomics are device-visible: they fenced before
// counting themselves done), so a level costs no launch of its own.
template <int SHIFT, int NBITS, uint32_t NT, uint32_t NSH>
__device__ void pick_level(RSel *st, uint64_t extra_zeros, uint32_t rank_arg) {
    static_assert(NSH >= 1 && NSH <= RS_SHARDS, "shards the feeding pass added into");
    constexpr bool FIRST = SHIFT + NBITS == 31;
    constexpr uint32_t NB = 1u << NBITS;
    constexpr uint32_t PER = (NB + NT - 1) / NT;
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t s_bin, s_before, s_cnt;
    const uint32_t t = threadIdx.x, lane = __lane_id(), wave = t >> 6;
    const uint32_t prefix = FIRST ? 0u : ld_sc1(&st->prefix);
    const uint32_t rank = FIRST ? rank_arg : ld_sc1(&st->rank);
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t td = PER * t + j;  // top-down bin index
        c[j] = 0;
        if (td < NB) {
            const uint32_t b = NB - 1 - td;
            c[j] = 0;
#pragma unroll
            for (uint32_t h = 0; h < NSH; ++h) c[j] += ld_sc1(&st->hist[h][b]);
            if (b == 0 && prefix == 0) c[j] += (uint32_t)extra_zeros;  // implicit zero keys
        }
        sum += c[j];
    }
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) wsum[wave] = incl;
    if (t == 0) { s_bin = 0xffffffffu; s_before = 0; }
    __syncthreads();
    uint32_t before = incl - sum;
    for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
    if (sum && rank >= before && rank - before < sum) {
        uint32_t acc = before;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            if (rank - acc < c[j]) { s_bin = NB - 1 - (PER * t + j); s_before = acc; s_cnt = c[j]; break; }
            acc += c[j];
        }
    }
    __syncthreads();
    // zero the shards' bins read above, 16 bytes per store (sc1: straight to
    // the device-coherent level, where the next pass's atomics land)
    static_assert(NB % 4 == 0, "whole 16-byte groups");
    for (uint32_t i = t; i < NSH * (NB / 4); i += NT) {
        const uint32_t h = i / (NB / 4), g = i % (NB / 4);
        st_sc1_zero16(&st->hist[0][0], NSH * RS_BINS * 4u, (h * RS_BINS + 4 * g) * 4u);
    }
    if (t == 0) {
        const bool hit = s_bin != 0xffffffffu;
        const uint32_t b = hit ? s_bin : 0u;  // rank out of range: degenerate
        const uint32_t bb = hit ? s_before : 0u;
        st_sc1(&st->rank, rank - bb);
        st_sc1(&st->pad[1], hit ? s_cnt : 0u);  // the chosen bin's keys (top-k's level-2 list)
        st_sc1(&st->cnt_gt, (FIRST ? 0u : ld_sc1(&st->cnt_gt)) + bb);
        st_sc1(&st->prefix, prefix | (b << SHIFT));
        st_sc1(&st->mask, (FIRST ? 0u : ld_sc1(&st->mask)) | ((NB - 1) << SHIFT));
    }
}

// True in exactly one workgroup of the grid: the last to finish this pass.
// What the last one reads was written with agent-scope atomics or stores
// (coherent across the XCDs' L2s), and every thread's memory operations have
// completed before its workgroup counts itself done.  Counting is two-level --
// the workgroups of each residue class of blockIdx.x mod 64 on their own word,
// the last of each class on the shared one -- so no word takes more than
// gridDim.x / 64 returning atomics (one word serialises them at ~90 per us).
__device__ inline bool last_workgroup(RSel *st) {
    __shared__ uint32_t s_last;
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt / lgkmcnt / expcnt all 0: this thread's memory ops are done
    __syncthreads();
    if (threadIdx.x == 0) {
        constexpr uint32_t NC = 64;
        const uint32_t G = gridDim.x, c = blockIdx.x % NC;
        const uint32_t in_c = G / NC + (c < G % NC ? 1u : 0u);  // workgroups of this class
        uint32_t last = 0;
        if (g_add(&st->done64[c], 1u) == in_c - 1) {
            st_sc1(&st->done64[c], 0u);
            const uint32_t classes = G < NC ? G : NC;
            if (g_add(&st->done, 1u) == classes - 1) {
                st_sc1(&st->done, 0u);
                last = 1;
            }
        }
        s_last = last;
    }
    __syncthreads();
    return s_last != 0;
}

}  // namespace stg
