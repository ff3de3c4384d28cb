// select.hip -- exact radix select on fp32 magnitudes (gfx950).
//
// Finds the key of a given descending rank among |x| bit patterns, as the
// reference's std::nth_element calls do for the first thresholds
// (thresholdv16.cpp:36-54, thresholdv.cpp:27-37) and for top-k
// (topk.cpp:36-38).  The order statistic is unique, so the result is
// bit-identical to nth_element's whatever the partition order.
//
// Three histogram levels over the 31 magnitude bits (11 + 11 + 9 bits).  Each
// level is one streaming pass: an LDS histogram per workgroup in four copies
// (lane & 3 picks the copy, so lanes whose keys share a bin -- magnitudes
// cluster in a few exponents -- rarely hit one LDS address together) and one
// global atomic per non-empty bin; then one 1024-thread workgroup picks the
// bin holding the rank and zeroes the table.
#include "select.h"

namespace stg {

namespace {

constexpr uint32_t kRsGridmul = 1;  // histogram workgroups per CU (fewer global bin atomics; 2: +7 us on top-k)
constexpr uint32_t kRsNcopy = 4;
constexpr uint32_t NCOPY = kRsNcopy;
constexpr uint32_t HWG = 1024;  // rs_hist workgroup: one fat workgroup per CU, few global bin atomics

#ifndef STG_RS_STAMPS
#define STG_RS_STAMPS 0  // diagnostics: level-1 phase times (100 MHz clock) into dbg[24..31]
#endif

template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(HWG) rs_hist(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                               RSel *st, uint64_t extra_zeros, uint32_t rank, uint32_t *dbg) {
    constexpr bool STAMPS = STG_RS_STAMPS && SHIFT == 20;
    auto now = [] { return (uint32_t)__builtin_amdgcn_s_memrealtime(); };
    if (STAMPS && threadIdx.x == 0) { const uint32_t t = now(); atomicMax(&dbg[24], ~t); atomicMax(&dbg[25], t); }
    constexpr bool FIRST = SHIFT + NBITS == 31;
    constexpr uint32_t NB = 1u << NBITS;
    // copies one word apart in the bank order (a stride of NB words would put
    // every copy of a bin in the same bank)
    constexpr uint32_t NBP = NB + 1;
    __shared__ uint32_t h[NCOPY][NBP];
    for (uint32_t i = threadIdx.x; i < NCOPY * NBP; i += HWG) (&h[0][0])[i] = 0;
    // the first level counts every key (its prefix and mask are still those of
    // the previous select)
    const uint32_t prefix = FIRST ? 0u : st->prefix;
    const uint32_t mask = FIRST ? 0u : st->mask;
    __syncthreads();

    uint32_t *hc = h[threadIdx.x & (NCOPY - 1)];
    const size_t m4 = m / 4;
    const float4 *a4 = reinterpret_cast<const float4 *>(a);
    const size_t stride = (size_t)gridDim.x * HWG;
    auto add = [&](uint32_t key) {
        if ((key & mask) == prefix) atomicAdd(&hc[(key >> SHIFT) & (NB - 1)], 1u);
    };
    // UF float4 loads per thread per step, double-buffered: the next step's
    // loads are issued before this step's keys are counted, so 2 x UF x 16 B
    // per thread stay in flight (128 KiB per CU; one step's worth, 64 KiB, is
    // under what hides an HBM miss)
    constexpr uint32_t UF = 4;
    // unconditional loads (a clamped index past the end; those keys are not
    // counted): a load under a branch makes the compiler wait for every load
    // at the join
    auto load_step = [&](size_t i0, float4 (&v)[UF]) {
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) v[u] = a4[std::min(i0 + u * stride, m4 - 1)];
    };
    auto count_step = [&](size_t i0, const float4 (&v)[UF]) {
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) {
            const size_t i = i0 + u * stride;
            if (i >= m4) break;
            uint32_t k0 = f2u(v[u].x) & 0x7fffffffu, k1 = f2u(v[u].y) & 0x7fffffffu;
            uint32_t k2 = f2u(v[u].z) & 0x7fffffffu, k3 = f2u(v[u].w) & 0x7fffffffu;
            if (4 * i + 3 == m - 1) k3 &= last_mask;
            add(k0); add(k1); add(k2); add(k3);
        }
    };
    // ping-pong over two register sets (no copies between them, so counting
    // one set waits only for its own loads)
    const size_t step = UF * stride;
    size_t i0 = (size_t)blockIdx.x * HWG + threadIdx.x;
    float4 va[UF], vb[UF];
    if (m4) {
        load_step(i0, va);
        for (; i0 < m4; i0 += 2 * step) {
            load_step(i0 + step, vb);
            count_step(i0, va);
            load_step(i0 + 2 * step, va);
            count_step(i0 + step, vb);
        }
    }
    if (blockIdx.x == 0) {
        for (size_t i = m4 * 4 + threadIdx.x; i < m; i += HWG) {
            uint32_t k = f2u(a[i]) & 0x7fffffffu;
            if (i == m - 1) k &= last_mask;
            add(k);
        }
    }
    __syncthreads();
    if (STAMPS && threadIdx.x == 0) atomicMax(&dbg[26], now());  // streaming done
    for (uint32_t i = threadIdx.x; i < NB; i += HWG) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t q = 0; q < NCOPY; ++q) c += h[q][i];
        if (c) g_add(&st->hist[blockIdx.x % RS_SH_HIST][i], c);
    }
    if (STAMPS) { __syncthreads(); if (threadIdx.x == 0) atomicMax(&dbg[27], now()); }  // flushed
    if (last_workgroup(st)) {
        const uint32_t t0 = now();
        pick_level<SHIFT, NBITS, HWG, RS_SH_HIST>(st, extra_zeros, rank);
        if (STAMPS) {
            __syncthreads();
            if (threadIdx.x == 0) {  // this call's record at [32..37], accumulators reset
                dbg[32] = ~atomicExch(&dbg[24], 0u);
                dbg[33] = atomicExch(&dbg[25], 0u);
                dbg[34] = atomicExch(&dbg[26], 0u);
                dbg[35] = atomicExch(&dbg[27], 0u);
                dbg[36] = t0;
                dbg[37] = now();
            }
        }
    }
}

}  // namespace

hipError_t launch_radix_select(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros, uint32_t rank,
                               const DevWS &ws, int num_cu, hipStream_t s) {
    const size_t work = (m / 4 + HWG - 1) / HWG;
    const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(work, (size_t)num_cu * kRsGridmul));
    rs_hist<20, 11><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros, rank, ws.misc);
    rs_hist<9, 11><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros, rank, ws.misc);
    rs_hist<0, 9><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros, rank, ws.misc);
    return hipGetLastError();
}

// The select's first level alone (top 11 bits; the histogram table is zero
// afterwards) -- top-k's superset passes take it from there.
hipError_t launch_radix_level1(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros, uint32_t rank,
                               const DevWS &ws, int num_cu, hipStream_t s) {
    const size_t work = (m / 4 + HWG - 1) / HWG;
    const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(work, (size_t)num_cu * kRsGridmul));
    rs_hist<20, 11><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros, rank, ws.misc);
    return hipGetLastError();
}

}  // namespace stg
