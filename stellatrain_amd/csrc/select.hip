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
// cluster in a few exponents -- rarely hit one LDS address together), one
// global atomic per non-empty bin, and the last workgroup to finish picks the
// bin holding the rank (no separate launch).
#include "ws.h"

namespace stg {

namespace {

#ifndef STG_RS_LASTBLOCK
#define STG_RS_LASTBLOCK 0  // 1: the last histogram workgroup picks; 0: one 64-thread pick launch per level
#endif
#ifndef STG_RS_NCOPY
#define STG_RS_NCOPY 4
#endif
constexpr uint32_t NCOPY = STG_RS_NCOPY;
constexpr uint32_t HWG = 1024;  // rs_hist workgroup: one fat workgroup per CU, few global bin atomics

__global__ void __launch_bounds__(STG_WG) rs_init(RSel *st, const uint32_t *d_rank, uint32_t rank) {
    for (uint32_t i = threadIdx.x; i < RS_BINS; i += STG_WG) st->hist[i] = 0;
    if (threadIdx.x == 0) {
        st->prefix = 0;
        st->mask = 0;
        st->rank = d_rank ? *d_rank : rank;
        st->cnt_gt = 0;
        st->done = 0;
    }
}

// The bin holding st->rank, counting from the top bin; run by one wave of the
// level's last workgroup (every other workgroup's bin atomics are complete).
template <int SHIFT, int NBITS>
__device__ __forceinline__ void pick(RSel *st, uint64_t extra_zeros) {
    constexpr uint32_t NB = 1u << NBITS;
    constexpr uint32_t PER = NB / 64;  // bins per lane, lane l owns top-down bins [PER l, PER l + PER)
    const uint32_t lane = __lane_id();
    const uint32_t prefix = st->prefix;
    const uint32_t rank = st->rank;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t b = NB - 1 - (PER * lane + j);
        uint32_t c = ld_acq_relaxed(&st->hist[b]);
        if (b == 0 && prefix == 0) c += (uint32_t)extra_zeros;  // implicit zero keys
        sum += c;
    }
    const uint32_t incl = wave_incl_scan(sum);
    const uint32_t before = incl - sum;
    const uint64_t hit = __ballot(rank >= before && rank < incl);
    uint32_t bin = 0xffffffffu, bbefore = 0;
    if (hit) {
        const uint32_t src = (uint32_t)__ffsll((long long)hit) - 1u;
        if (lane == src) {
            uint32_t acc = before;
            for (uint32_t j = 0; j < PER; ++j) {
                const uint32_t b = NB - 1 - (PER * lane + j);
                uint32_t c = ld_acq_relaxed(&st->hist[b]);
                if (b == 0 && prefix == 0) c += (uint32_t)extra_zeros;
                if (rank < acc + c) { bin = b; bbefore = acc; break; }
                acc += c;
            }
        }
        bin = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)src);
        bbefore = (uint32_t)__builtin_amdgcn_readlane((int)bbefore, (int)src);
    }
    for (uint32_t i = lane; i < RS_BINS; i += 64) st->hist[i] = 0;  // for the next level
    if (lane == 0) {
        const uint32_t b = bin == 0xffffffffu ? 0 : bin;  // rank out of range: degenerate
        st->rank = rank - bbefore;
        st->cnt_gt += bbefore;
        st->prefix = prefix | (b << SHIFT);
        st->mask |= (NB - 1) << SHIFT;
        st->done = 0;
    }
}

template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(HWG) rs_hist(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                               RSel *st, uint64_t extra_zeros) {
    constexpr uint32_t NB = 1u << NBITS;
    __shared__ uint32_t h[NCOPY][NB];
    __shared__ uint32_t s_last;
    for (uint32_t i = threadIdx.x; i < NCOPY * NB; i += HWG) (&h[0][0])[i] = 0;
    const uint32_t prefix = st->prefix;
    const uint32_t mask = st->mask;
    __syncthreads();

    uint32_t *hc = h[threadIdx.x & (NCOPY - 1)];
    const size_t m4 = m / 4;
    const float4 *a4 = reinterpret_cast<const float4 *>(a);
    const size_t stride = (size_t)gridDim.x * HWG;
    auto add = [&](uint32_t key) {
        if ((key & mask) == prefix) atomicAdd(&hc[(key >> SHIFT) & (NB - 1)], 1u);
    };
    // UF float4 loads per thread in flight before any is used
    constexpr uint32_t UF = 4;
    for (size_t i0 = (size_t)blockIdx.x * HWG + threadIdx.x; i0 < m4; i0 += UF * stride) {
        float4 v[UF];
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) {
            const size_t i = i0 + u * stride;
            v[u] = i < m4 ? a4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) {
            const size_t i = i0 + u * stride;
            if (i >= m4) break;
            uint32_t k0 = f2u(v[u].x) & 0x7fffffffu, k1 = f2u(v[u].y) & 0x7fffffffu;
            uint32_t k2 = f2u(v[u].z) & 0x7fffffffu, k3 = f2u(v[u].w) & 0x7fffffffu;
            if (4 * i + 3 == m - 1) k3 &= last_mask;
            add(k0); add(k1); add(k2); add(k3);
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
    for (uint32_t i = threadIdx.x; i < NB; i += HWG) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t q = 0; q < NCOPY; ++q) c += h[q][i];
        if (c) atomicAdd(&st->hist[i], c);
    }
    // The last workgroup to finish picks the bin.  Agent-scope atomics are
    // coherent across the XCDs without fences (an agent-scope release fence
    // would write back the whole L2): every thread waits for its atomics to
    // complete, then one relaxed atomic counts the workgroup done; the picker
    // reads the bins with agent-scope loads.
    if (!STG_RS_LASTBLOCK) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(&st->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (s_last && threadIdx.x < 64) pick<SHIFT, NBITS>(st, extra_zeros);
}

template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(64) rs_pick(RSel *st, uint64_t extra_zeros) {
    pick<SHIFT, NBITS>(st, extra_zeros);
}

}  // namespace

hipError_t launch_radix_select(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros,
                               const uint32_t *d_rank, uint32_t rank, const DevWS &ws, int num_cu,
                               hipStream_t s) {
    const size_t work = (m / 4 + HWG - 1) / HWG;
    const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(work, (size_t)num_cu * 2));
    rs_init<<<1, STG_WG, 0, s>>>(ws.rsel, d_rank, rank);
    rs_hist<20, 11><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros);
    if (!STG_RS_LASTBLOCK) rs_pick<20, 11><<<1, 64, 0, s>>>(ws.rsel, extra_zeros);
    rs_hist<9, 11><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros);
    if (!STG_RS_LASTBLOCK) rs_pick<9, 11><<<1, 64, 0, s>>>(ws.rsel, extra_zeros);
    rs_hist<0, 9><<<grid, HWG, 0, s>>>(a, m, last_mask, ws.rsel, extra_zeros);
    if (!STG_RS_LASTBLOCK) rs_pick<0, 9><<<1, 64, 0, s>>>(ws.rsel, extra_zeros);
    return hipGetLastError();
}

}  // namespace stg
