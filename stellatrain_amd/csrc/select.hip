// select.hip -- exact radix select on fp32 magnitudes (gfx950).
//
// Finds the key of a given descending rank among |x| bit patterns, as the
// reference's std::nth_element calls do for the first thresholds
// (thresholdv16.cpp:36-54, thresholdv.cpp:27-37) and for top-k
// (topk.cpp:36-38).  The order statistic is unique, so the result is
// bit-identical to nth_element's whatever the partition order.
//
// Three histogram levels over the 31 magnitude bits (11 + 11 + 9 bits).  Each
// level is one streaming pass (LDS histogram per workgroup, one global atomic
// per non-empty bin) plus a one-workgroup pick of the bin holding the rank.
#include "ws.h"

namespace stg {

namespace {

__global__ void __launch_bounds__(STG_WG) rs_init(RSel *st, const uint32_t *d_rank, uint32_t rank) {
    for (uint32_t i = threadIdx.x; i < RS_BINS; i += STG_WG) st->hist[i] = 0;
    if (threadIdx.x == 0) {
        st->prefix = 0;
        st->mask = 0;
        st->rank = d_rank ? *d_rank : rank;
        st->cnt_gt = 0;
    }
}

template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(STG_WG) rs_hist(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                  RSel *st) {
    constexpr uint32_t NB = 1u << NBITS;
    __shared__ uint32_t h[NB];
    for (uint32_t i = threadIdx.x; i < NB; i += STG_WG) h[i] = 0;
    const uint32_t prefix = st->prefix;
    const uint32_t mask = st->mask;
    __syncthreads();

    const size_t m4 = m / 4;
    const float4 *a4 = reinterpret_cast<const float4 *>(a);
    const size_t stride = (size_t)gridDim.x * STG_WG;
    auto add = [&](uint32_t key) {
        if ((key & mask) == prefix) atomicAdd(&h[(key >> SHIFT) & (NB - 1)], 1u);
    };
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < m4; i += stride) {
        const float4 v = a4[i];
        uint32_t k0 = f2u(v.x) & 0x7fffffffu, k1 = f2u(v.y) & 0x7fffffffu;
        uint32_t k2 = f2u(v.z) & 0x7fffffffu, k3 = f2u(v.w) & 0x7fffffffu;
        if (4 * i + 3 == m - 1) k3 &= last_mask;
        add(k0); add(k1); add(k2); add(k3);
    }
    if (blockIdx.x == 0) {
        for (size_t i = m4 * 4 + threadIdx.x; i < m; i += STG_WG) {
            uint32_t k = f2u(a[i]) & 0x7fffffffu;
            if (i == m - 1) k &= last_mask;
            add(k);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NB; i += STG_WG)
        if (h[i]) atomicAdd(&st->hist[i], h[i]);
}

// One workgroup: locate the bin holding st->rank, counting from the top bin.
template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(STG_WG) rs_pick(RSel *st, uint64_t extra_zeros) {
    constexpr uint32_t NB = 1u << NBITS;
    constexpr uint32_t PER = NB / STG_WG;  // bins per thread
    __shared__ uint32_t sh[STG_WAVES + 1];
    __shared__ uint32_t s_bin, s_before;
    const uint32_t prefix = st->prefix;
    const uint32_t rank = st->rank;
    if (threadIdx.x == 0) { s_bin = 0xffffffffu; s_before = 0; }
    // thread t owns bins [NB-1-PER*t-(PER-1), NB-1-PER*t], scanned top-down
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t b = NB - 1 - (PER * threadIdx.x + j);
        uint32_t c = st->hist[b];
        if (b == 0 && prefix == 0) c += (uint32_t)extra_zeros;  // implicit zero keys
        loc[j] = c;
        sum += c;
    }
    uint32_t total;
    const uint32_t before = wg_excl_scan(sum, sh, &total);
    if (rank >= before && rank < before + sum) {
        uint32_t acc = before;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            if (rank < acc + loc[j]) {
                s_bin = NB - 1 - (PER * threadIdx.x + j);
                s_before = acc;
                break;
            }
            acc += loc[j];
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < RS_BINS; i += STG_WG) st->hist[i] = 0;
    if (threadIdx.x == 0) {
        const uint32_t b = s_bin == 0xffffffffu ? 0 : s_bin;  // rank out of range: degenerate
        st->rank = rank - s_before;
        st->cnt_gt += s_before;
        st->prefix = prefix | (b << SHIFT);
        st->mask |= (NB - 1) << SHIFT;
    }
}

}  // namespace

hipError_t launch_radix_select(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros,
                               const uint32_t *d_rank, uint32_t rank, const DevWS &ws, int num_cu,
                               hipStream_t s) {
    const size_t work = (m / 4 + STG_WG - 1) / STG_WG;
    const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(work, (size_t)num_cu * 8));
    rs_init<<<1, STG_WG, 0, s>>>(ws.rsel, d_rank, rank);
    rs_hist<20, 11><<<grid, STG_WG, 0, s>>>(a, m, last_mask, ws.rsel);
    rs_pick<20, 11><<<1, STG_WG, 0, s>>>(ws.rsel, extra_zeros);
    rs_hist<9, 11><<<grid, STG_WG, 0, s>>>(a, m, last_mask, ws.rsel);
    rs_pick<9, 11><<<1, STG_WG, 0, s>>>(ws.rsel, extra_zeros);
    rs_hist<0, 9><<<grid, STG_WG, 0, s>>>(a, m, last_mask, ws.rsel);
    rs_pick<0, 9><<<1, STG_WG, 0, s>>>(ws.rsel, extra_zeros);
    return hipGetLastError();
}

}  // namespace stg
