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

// Per tile: elements > T and == T.
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

// One workgroup: the tile counts' exclusive prefixes at [ntiles + t], the
// totals at [2 ntiles] (a done-counter in tk_count would have 2048 workgroups
// contend on one atomic).  2048 tiles per round, 8 consecutive per thread,
// all loads issued before the scan.
__global__ void __launch_bounds__(STG_WG) tk_scan(uint32_t *__restrict__ tile_gt, uint32_t *__restrict__ tile_eq,
                                                  uint32_t ntiles) {
    __shared__ uint32_t sh[STG_WAVES + 1];
    uint32_t cg = 0, ce = 0;  // running prefixes
    constexpr uint32_t PT = 8;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += PT * STG_WG) {
        const uint32_t tb = t0 + PT * threadIdx.x;
        uint32_t g[PT], q[PT], sg = 0, sq = 0;
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) {
            g[i] = tb + i < ntiles ? tile_gt[tb + i] : 0u;
            q[i] = tb + i < ntiles ? tile_eq[tb + i] : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) { sg += g[i]; sq += q[i]; }
        uint32_t tg, tq;
        uint32_t pg = cg + wg_excl_scan(sg, sh, &tg);
        uint32_t pq = ce + wg_excl_scan(sq, sh, &tq);
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) {
            if (tb + i < ntiles) {
                tile_gt[ntiles + tb + i] = pg;
                tile_eq[ntiles + tb + i] = pq;
            }
            pg += g[i];
            pq += q[i];
        }
        cg += tg;
        ce += tq;
    }
    if (threadIdx.x == 0) {
        tile_gt[2 * ntiles] = cg;
        tile_eq[2 * ntiles] = ce;
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

// One workgroup per tile: the winners (> T, then == T in index order until
// k) at their prefix offsets.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_emit(TkArgs a) {
    __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
    const uint32_t tile = blockIdx.x, tid = threadIdx.x, nt = a.ntiles;
    const uint32_t T = a.rs->prefix;
    const uint64_t need_eq = (uint64_t)a.k - a.rs->cnt_gt;  // ties to take, in index order
    const uint32_t cg = a.tile_gt[tile], ce = a.tile_eq[tile];
    const uint64_t gt_before = a.tile_gt[nt + tile], eq_before = a.tile_eq[nt + tile];
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
    // implicit +0.0 elements past the copied bytes (bug-compat only): they tie
    // at T == 0 after every real element
    if (tile == 0 && a.zeros && T == 0) {
        const uint64_t first = (uint64_t)a.tile_gt[2 * nt] + std::min<uint64_t>(a.tile_eq[2 * nt], need_eq);
        for (uint64_t s = first + tid; s < a.k; s += STG_WG) {
            a.idx[s] = (uint32_t)s;
            a.val[s] = 0.f;
        }
    }
    if (tile == 0 && tid == 0) *a.count_out = a.cap;
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
    tk_scan<<<1, STG_WG, 0, s>>>(ws.tile_cnt, ws.tile_aux, ntiles);
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
    if (vec) tk_emit<true><<<ntiles, STG_WG, 0, s>>>(t);
    else tk_emit<false><<<ntiles, STG_WG, 0, s>>>(t);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
