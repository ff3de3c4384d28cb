// topk.hip -- Top-k by |x| on gfx950.
//
// Reference: TopkCompressor::impl_nth_element (compress/topk.cpp:28-46), the
// default method (topk.h:30).  As shipped it has two defects that the
// "topk" method reproduces:
//   * memcpy(clone, src, n) copies n *bytes*: only floats [0, n/4) survive,
//     float n/4 keeps its low n%4 bytes, the rest of the clone is +0.0;
//   * idx[i] = i for i < k (idx_offset is not forwarded), val[i] = clone[i]
//     after nth_element, i.e. the k largest |clone| in partition order.
// "topk_exact" is the intended operator: the k largest |x| of the whole
// bucket with their real indices (+ idx_offset).
// Both emit the winners in index order (the reference's partition order is an
// artefact of libstdc++ introselect); ties at the k-th magnitude are taken in
// index order.  compress() returns the capacity (topk.cpp:25) and throws when
// capacity < k (topk.cpp:33-34).
//
// GPU structure: exact radix select of the k-th magnitude (select.hip), then
// a per-tile count of (> T, == T) and an ordered emission pass.
#include <algorithm>

#include "tile.h"

namespace stg {

namespace {

template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_count(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                   const RSel *__restrict__ rs, uint32_t *__restrict__ tile_gt,
                                                   uint32_t *__restrict__ tile_eq) {
    __shared__ uint32_t s_c[2 * STG_WAVES];
    const uint32_t T = rs->prefix;
    const size_t base = (size_t)blockIdx.x * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(a, m, base, last_mask, v);
    uint32_t gt = 0, eq = 0;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = f2u(comp(v[u], j)) & 0x7fffffffu;
            const bool valid = e + j < m;
            gt += valid && key > T;
            eq += valid && key == T;
        }
    }
    gt = wave_sum(gt);
    eq = wave_sum(eq);
    if (__lane_id() == 0) { s_c[threadIdx.x >> 6] = gt; s_c[STG_WAVES + (threadIdx.x >> 6)] = eq; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t g = 0, q = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) { g += s_c[w]; q += s_c[STG_WAVES + w]; }
        tile_gt[blockIdx.x] = g;
        tile_eq[blockIdx.x] = q;
    }
}

struct TkArgs {
    const float *a;
    uint64_t m;          // elements actually present
    uint64_t zeros;      // implicit +0.0 elements after them (bug-compat)
    uint32_t last_mask;
    uint32_t ntiles, k, cap;
    int32_t idx_offset;
    bool bug_compat;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    const RSel *rs;
    const uint32_t *tile_gt;
    const uint32_t *tile_eq;
};

template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_emit(TkArgs a) {
    __shared__ uint64_t sh64[STG_WAVES];
    __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
    const uint32_t G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const uint32_t t_begin = (uint32_t)((uint64_t)w * a.ntiles / G);
    const uint32_t t_end = (uint32_t)((uint64_t)(w + 1) * a.ntiles / G);
    const uint32_t T = a.rs->prefix;
    const uint64_t need_eq = (uint64_t)a.k - a.rs->cnt_gt;  // ties to take, in index order

    uint64_t bg = 0, be = 0, tg = 0, te = 0;
    for (uint32_t i = tid; i < a.ntiles; i += STG_WG) {
        const uint32_t g = a.tile_gt[i], q = a.tile_eq[i];
        tg += g;
        te += q;
        if (i < t_begin) { bg += g; be += q; }
    }
    uint64_t gt_before = wg_sum64(bg, sh64);
    uint64_t eq_before = wg_sum64(be, sh64);
    const uint64_t gt_total = wg_sum64(tg, sh64);
    const uint64_t eq_total = wg_sum64(te, sh64);

    for (uint32_t tile = t_begin; tile < t_end; ++tile) {
        const uint32_t cg = a.tile_gt[tile], ce = a.tile_eq[tile];
        if (cg || (ce && eq_before < need_eq)) {  // uniform per workgroup
            float4 v[TILE_U];
            const size_t base = (size_t)tile * TV_TILE;
            load_tile<VEC>(a.a, a.m, base, a.last_mask, v);
            uint32_t qg = 0, qe = 0;
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) {
                const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t key = f2u(comp(v[u], j)) & 0x7fffffffu;
                    if (e + j < a.m) {
                        if (key > T) qg |= 1u << (u * 4 + j);
                        else if (key == T) qe |= 1u << (u * 4 + j);
                    }
                }
            }
            uint32_t se[TILE_U * 4], sw[TILE_U * 4], tot;
            tile_ranks(qe, se, s_wt, &tot);
            uint32_t qw = qg;
#pragma unroll
            for (uint32_t b = 0; b < TILE_U * 4; ++b)
                if (((qe >> b) & 1u) && eq_before + se[b] < need_eq) qw |= 1u << b;
            tile_ranks(qw, sw, s_wt, &tot);
            const uint64_t win_before = gt_before + std::min(eq_before, need_eq);
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) {
                const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t b = u * 4 + j;
                    if ((qw >> b) & 1u) {
                        const uint64_t slot = win_before + sw[b];
                        a.idx[slot] = a.bug_compat ? (uint32_t)slot : (uint32_t)(e + j) + (uint32_t)a.idx_offset;
                        a.val[slot] = comp(v[u], j);
                    }
                }
            }
        }
        gt_before += cg;
        eq_before += ce;
    }
    // implicit +0.0 elements past the copied bytes (bug-compat only): they tie
    // at T == 0 after every real element
    if (w == 0 && a.zeros && T == 0) {
        const uint64_t first = gt_total + std::min(eq_total, need_eq);
        for (uint64_t s = first + tid; s < a.k; s += STG_WG) {
            a.idx[s] = (uint32_t)s;
            a.val[s] = 0.f;
        }
    }
    if (w == 0 && tid == 0) *a.count_out = a.cap;
}

__global__ void tk_empty(uint32_t *count_out, uint32_t cap) { *count_out = cap; }

}  // namespace

hipError_t launch_topk(const TopkLaunch &a, const DevWS &ws, hipStream_t s) {
    if (a.k == 0 || a.n == 0) {
        tk_empty<<<1, 1, 0, s>>>(a.count_out, a.cap);
        return hipGetLastError();
    }
    uint64_t m = a.n, zeros = 0;
    uint32_t last_mask = 0xffffffffu;
    if (a.bug_compat) {
        // memcpy(clone, src, n) copies n bytes (topk.cpp:31)
        m = a.n / 4 + (a.n % 4 ? 1 : 0);
        if (a.n % 4) last_mask = (1u << (8 * (a.n % 4))) - 1u;
        zeros = a.n - m;
    }
    const uint32_t kk = (uint32_t)std::min<uint64_t>(a.k, a.n);
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    hipError_t e = launch_radix_select(a.src, m, last_mask, zeros, nullptr, kk - 1, ws, a.num_cu, s);
    if (e != hipSuccess) return e;
    const uint32_t ntiles = (uint32_t)((m + TV_TILE - 1) / TV_TILE);
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
    if (vec) tk_count<true><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, ws.tile_cnt, ws.tile_aux);
    else tk_count<false><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, ws.tile_cnt, ws.tile_aux);
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    TkArgs t;
    t.a = a.src;
    t.m = m;
    t.zeros = zeros;
    t.last_mask = last_mask;
    t.ntiles = ntiles;
    t.k = kk;
    t.cap = a.cap;
    t.idx_offset = a.idx_offset;
    t.bug_compat = a.bug_compat;
    t.idx = a.idx;
    t.val = a.val;
    t.count_out = a.count_out;
    t.rs = ws.rsel;
    t.tile_gt = ws.tile_cnt;
    t.tile_eq = ws.tile_aux;
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)a.num_cu * 2, ntiles));
    if (vec) tk_emit<true><<<G, STG_WG, 0, s>>>(t);
    else tk_emit<false><<<G, STG_WG, 0, s>>>(t);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
