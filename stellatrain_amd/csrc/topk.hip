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
// GPU structure: two passes over the bucket, the rest over a ~3 % superset:
//   rs_hist level 1 (select.hip; its last workgroup picks): the top 11 bits
//     of the k-th magnitude T;
//   tk_pass: every element at or above that bin goes, in index order, to its
//     tile's superset region (an overflowing tile keeps only a count and is
//     re-read later); the bin's elements fill the level-2 histogram;
//   tk_pick level 2: bits 19..9 of T (and how many keys share that bin);
//   buckets of <= TOPK_LIST_TILES tiles: tk_resolve lists the keys of T's
//     level-2 bin (~100 at 64 MiB) and counts each tile's keys above it;
//     tk_final (one workgroup) takes T from the list, fixes the per-tile
//     (> T, == T) counts and scans them.  A bin holding more keys than the
//     list (ties) falls back inside the same two launches: tk_resolve fills
//     the level-3 histogram and tk_final picks T and recounts the bin's keys
//     per tile itself (slow, ties only);
//   larger buckets: tk_hist3 + tk_pick level 3, tk_count2 + tk_scan;
//   tk_emit2: the ordered emission from the supersets.
#include <algorithm>

#include "select.h"
#include "tile.h"

namespace stg {

namespace {

// The tile counts' exclusive prefixes at [ntiles + t], the totals at
// [2 ntiles], by the last workgroup of tk_count2 (coherent loads: the other
// workgroups wrote the counts in this launch).  8 consecutive tiles per
// thread, all loads issued before the scan.
__device__ void scan_tiles(uint32_t *__restrict__ tile_gt, uint32_t *__restrict__ tile_eq, uint32_t ntiles) {
    __shared__ uint32_t sh[STG_WAVES + 1];
    uint32_t cg = 0, ce = 0;  // running prefixes
    constexpr uint32_t PT = 8;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += PT * STG_WG) {
        const uint32_t tb = t0 + PT * threadIdx.x;
        uint32_t g[PT], q[PT], sg = 0, sq = 0;
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) {
            g[i] = tb + i < ntiles ? ld_sc1(&tile_gt[tb + i]) : 0u;
            q[i] = tb + i < ntiles ? ld_sc1(&tile_eq[tb + i]) : 0u;
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

constexpr uint32_t SUP_CAP = TOPK_SUP_CAP;  // superset entries kept per tile (4 per thread); more: re-read the tile
static_assert(SUP_CAP == 4 * STG_WG, "four superset entries per thread");

__device__ __forceinline__ uint32_t mag(uint32_t bits) { return bits & 0x7fffffffu; }

// Pass 2: the tile's superset (|x| bits >= lo, the level-1 bin's low edge) in
// index order as {element, raw bits}, its count, and the level-2 histogram
// (next 11 bits) of the level-1 bin's elements.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_pass(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                  RSel *__restrict__ rs, uint2 *__restrict__ sup,
                                                  uint32_t *__restrict__ sup_n) {
    constexpr uint32_t NB2 = 2048;
    __shared__ uint32_t h2[NB2];
    __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
    for (uint32_t i = threadIdx.x; i < NB2; i += STG_WG) h2[i] = 0;
    const uint32_t lo = rs->prefix;  // level 1: bits 30..20 of T, the rest 0
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        rs->pad[0] = lo;  // for the later passes
        rs->pad[2] = 0;   // the level-2 bin's list (tk_resolve)
    }
    __syncthreads();
    const uint32_t tile = blockIdx.x, lane = __lane_id(), wave = threadIdx.x >> 6;
    const size_t base = (size_t)tile * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(a, m, base, last_mask, v);
    // flags, the level-2 histogram, and each lane's place among the flagged
    // elements of its wave for each u (element order is (u, wave, lane, j));
    // slots are rebuilt from these when written, so no per-element registers
    uint32_t q = 0, pre[TILE_U];
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag(f2u(comp(v[u], j)));
            if (e + j < m && key >= lo) {
                q |= 1u << (u * 4 + j);
                if ((key >> 20) == (lo >> 20)) atomicAdd(&h2[(key >> 9) & (NB2 - 1)], 1u);
            }
        }
        const uint32_t c = (uint32_t)__popc((q >> (4 * u)) & 0xfu);
        const uint32_t incl = wave_incl_scan(c);
        pre[u] = incl - c;
        if (lane == 63) s_wt[u * STG_WAVES + wave] = incl;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // (u, wave) offsets: one wave scans the 32 counts
        constexpr uint32_t NW = TILE_U * STG_WAVES;
        static_assert(NW <= 64, "one wave scans the wave counts");
        const uint32_t x = threadIdx.x < NW ? s_wt[threadIdx.x] : 0u;
        const uint32_t inc = wave_incl_scan(x);
        if (threadIdx.x < NW) s_wt[threadIdx.x] = inc - x;
        if (threadIdx.x == NW - 1) s_wt[NW] = inc;
    }
    __syncthreads();
    const uint32_t tot = s_wt[TILE_U * STG_WAVES];
    if (tot <= SUP_CAP) {
        uint2 *dst = sup + (size_t)tile * SUP_CAP;
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
            uint32_t slot = s_wt[u * STG_WAVES + wave] + pre[u];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((q >> (u * 4 + j)) & 1u) dst[slot++] = make_uint2((uint32_t)(e + j), f2u(comp(v[u], j)));
        }
    }
    if (threadIdx.x == 0) sup_n[tile] = tot;
    for (uint32_t i = threadIdx.x; i < NB2; i += STG_WG)
        if (h2[i]) g_add(&rs->hist[blockIdx.x % RS_SHARDS][i], h2[i]);
}

// The tile's superset entries (or, for a tile that overflowed, its elements
// re-read with the same keys) handed one at a time to f(element, raw bits)
// in index order per thread: thread t takes entries 4t .. 4t+3.
template <bool VEC, typename F>
__device__ __forceinline__ void for_tile(const float *__restrict__ a, size_t m, uint32_t last_mask, uint32_t lo,
                                         const uint2 *__restrict__ sup, uint32_t n, F f) {
    const uint32_t tile = blockIdx.x;
    if (n <= SUP_CAP) {
        const uint2 *src = sup + (size_t)tile * SUP_CAP;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t j = 4 * threadIdx.x + r;
            if (j < n) {
                const uint2 x = src[j];
                f(x.x, x.y);
            }
        }
        return;
    }
    const size_t base = (size_t)tile * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(a, m, base, last_mask, v);
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (e + j < m && mag(f2u(comp(v[u], j))) >= lo) f((uint32_t)(e + j), f2u(comp(v[u], j)));
    }
}

// Level 3 over the supersets: the low 9 bits of the keys in the level-2 bin.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_hist3(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                   RSel *__restrict__ rs, const uint2 *__restrict__ sup,
                                                   const uint32_t *__restrict__ sup_n) {
    __shared__ uint32_t h3[512];
    for (uint32_t i = threadIdx.x; i < 512; i += STG_WG) h3[i] = 0;
    const uint32_t prefix = rs->prefix, mask = rs->mask, lo = rs->pad[0];  // bits 30..9
    const uint32_t n = sup_n[blockIdx.x];
    __syncthreads();
    for_tile<VEC>(a, m, last_mask, lo, sup, n, [&](uint32_t, uint32_t bits) {
        const uint32_t key = mag(bits);
        if ((key & mask) == prefix) atomicAdd(&h3[key & 511u], 1u);
    });
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 512; i += STG_WG)
        if (h3[i]) g_add(&rs->hist[blockIdx.x % RS_SHARDS][i], h3[i]);
}

// A level's pick as its own launch (the per-tile passes have too many
// workgroups for a last-workgroup pick to pay).
template <int SHIFT, int NBITS>
__global__ void __launch_bounds__(1024) tk_pick(RSel *rs, uint64_t zeros) {
    pick_level<SHIFT, NBITS, 1024, RS_SHARDS>(rs, zeros, 0);
}

__global__ void __launch_bounds__(STG_WG) tk_scan(uint32_t *tile_gt, uint32_t *tile_eq, uint32_t ntiles) {
    scan_tiles(tile_gt, tile_eq, ntiles);
}

// Per tile: elements > T and == T.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_count2(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                    const RSel *__restrict__ rs,
                                                    const uint2 *__restrict__ sup, const uint32_t *__restrict__ sup_n,
                                                    uint32_t *__restrict__ tile_gt, uint32_t *__restrict__ tile_eq) {
    __shared__ uint32_t s_c[2 * STG_WAVES];
    const uint32_t T = rs->prefix, lo = rs->pad[0];
    uint32_t gt = 0, eq = 0;
    for_tile<VEC>(a, m, last_mask, lo, sup, sup_n[blockIdx.x], [&](uint32_t, uint32_t bits) {
        const uint32_t key = mag(bits);
        gt += key > T;
        eq += key == T;
    });
    gt = wave_sum(gt);
    eq = wave_sum(eq);
    if (__lane_id() == 0) { s_c[threadIdx.x >> 6] = gt; s_c[STG_WAVES + (threadIdx.x >> 6)] = eq; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t g = 0, e = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) { g += s_c[w]; e += s_c[STG_WAVES + w]; }
        tile_gt[blockIdx.x] = g;
        tile_eq[blockIdx.x] = e;
    }
}

// ---------------------------------------------------------------------------
// Level 3 without a histogram pass (buckets of <= TOPK_LIST_TILES tiles): T's
// level-2 bin spans 2^9 ulps and holds ~100 keys at 64 MiB, so they are listed
// and one workgroup finishes the select, the per-tile counts and their scan.
// ---------------------------------------------------------------------------
struct TkList {
    uint2 *list;       // {element, key} of the level-2 bin's keys, TOPK_LIST_CAP
    uint32_t ntiles;
    uint64_t zeros;    // implicit +0.0 keys (bug-compat)
};

// Per tile: the superset's keys above T's level-2 bin (count) and those in it
// (listed); with a crowded bin (ties: more than the list holds) the level-3
// histogram instead.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_resolve(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                     RSel *__restrict__ rs, const uint2 *__restrict__ sup,
                                                     const uint32_t *__restrict__ sup_n, uint32_t *__restrict__ tile_gt,
                                                     TkList L) {
    __shared__ uint32_t h3[512];
    __shared__ uint2 s_list[TOPK_LIST_CAP];  // this tile's keys in the bin, then one global append
    __shared__ uint32_t s_c[STG_WAVES], s_ln, s_base;
    const uint32_t prefix = rs->prefix, mask = rs->mask, lo = rs->pad[0];  // bits 30..9 of T
    const uint32_t real = rs->pad[1] - (prefix == 0 ? (uint32_t)L.zeros : 0u);  // listed keys
    const bool listed = real <= TOPK_LIST_CAP;
    if (threadIdx.x == 0) s_ln = 0;
    if (!listed)
        for (uint32_t i = threadIdx.x; i < 512; i += STG_WG) h3[i] = 0;
    __syncthreads();
    uint32_t above = 0;
    for_tile<VEC>(a, m, last_mask, lo, sup, sup_n[blockIdx.x], [&](uint32_t e, uint32_t bits) {
        const uint32_t key = mag(bits), top = key & mask;
        above += top > prefix;
        if (top == prefix) {
            if (listed) {
                const uint32_t j = atomicAdd(&s_ln, 1u);
                if (j < TOPK_LIST_CAP) s_list[j] = make_uint2(e, key);
            } else {
                atomicAdd(&h3[key & 511u], 1u);
            }
        }
    });
    above = wave_sum(above);
    if (__lane_id() == 0) s_c[threadIdx.x >> 6] = above;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t g = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) g += s_c[w];
        tile_gt[blockIdx.x] = g;
        // one device atomic per tile with keys in the bin (a word takes ~90 per us)
        s_base = s_ln ? g_add(&rs->pad[2], s_ln) : 0u;
    }
    __syncthreads();
    if (listed) {
        const uint32_t n = std::min(s_ln, TOPK_LIST_CAP);
        for (uint32_t i = threadIdx.x; i < n; i += STG_WG)
            if (s_base + i < TOPK_LIST_CAP) L.list[s_base + i] = s_list[i];
    }
    if (!listed)
        for (uint32_t i = threadIdx.x; i < 512; i += STG_WG)
            if (h3[i]) g_add(&rs->hist[blockIdx.x % RS_SHARDS][i], h3[i]);
}

constexpr uint32_t FWGT = 1024;  // tk_final: one workgroup
constexpr uint32_t FNWT = FWGT / 64;

// One workgroup: T from the list (or the level-3 histogram), the per-tile
// (> T, == T) counts and their exclusive prefixes -- what tk_count2 + tk_scan
// leave for the emission.
template <bool VEC>
__global__ void __launch_bounds__(FWGT) tk_final(const float *__restrict__ a, size_t m, uint32_t last_mask,
                                                 RSel *__restrict__ rs, const uint2 *__restrict__ sup,
                                                 const uint32_t *__restrict__ sup_n, uint32_t *__restrict__ tile_gt,
                                                 uint32_t *__restrict__ tile_eq, TkList L) {
    __shared__ uint32_t g[TOPK_LIST_TILES], q[TOPK_LIST_TILES];
    __shared__ uint32_t h[512];
    __shared__ uint32_t sh[FNWT + 1];
    __shared__ uint32_t s_T, s_above;
    const uint32_t tid = threadIdx.x, nt = L.ntiles;
    const uint32_t prefix = rs->prefix, lo = rs->pad[0];
    const uint32_t rank = rs->rank, cnt_gt = rs->cnt_gt;
    const uint32_t real = rs->pad[1] - (prefix == 0 ? (uint32_t)L.zeros : 0u);
    const bool listed = real <= TOPK_LIST_CAP;
    const uint32_t nl = listed ? std::min(rs->pad[2], TOPK_LIST_CAP) : 0u;
    for (uint32_t i = tid; i < 512; i += FWGT) h[i] = 0;
    for (uint32_t t = tid; t < nt; t += FWGT) { g[t] = tile_gt[t]; q[t] = 0; }
    __syncthreads();
    uint32_t T;
    if (listed) {
        // the low 9 bits of the listed keys (+ the implicit zeros in the bin of 0)
        for (uint32_t i = tid; i < nl; i += FWGT) atomicAdd(&h[L.list[i].y & 511u], 1u);
        if (tid == 0 && prefix == 0 && L.zeros) atomicAdd(&h[0], (uint32_t)L.zeros);
        __syncthreads();
        {   // the bin of descending rank `rank`: thread i holds bin 511 - i, a
            // workgroup scan gives the keys above it (a serial walk over 512 LDS
            // words cost ~15 us)
            const uint32_t c = tid < 512 ? h[511 - tid] : 0u;
            uint32_t tot;
            const uint32_t above = blk_excl_scan<FNWT>(c, sh, &tot);
            if (tid < 512 && c && rank >= above && rank - above < c) {
                s_T = prefix | (511u - tid);
                s_above = above;
            }
            if (tid == 0 && rank >= tot) { s_T = prefix; s_above = tot; }  // rank out of range: degenerate
        }
        __syncthreads();
        T = s_T;
        for (uint32_t i = tid; i < nl; i += FWGT) {  // the listed keys' tiles
            const uint2 x = L.list[i];
            const uint32_t t = x.x / TV_TILE;
            if (x.y > T) atomicAdd(&g[t], 1u);
            else if (x.y == T) atomicAdd(&q[t], 1u);
        }
    } else {
        // a crowded bin: tk_resolve filled the level-3 histogram; then every
        // tile's keys in the bin again (slow, one workgroup; ties only)
        pick_level<0, 9, FWGT, RS_SHARDS>(rs, L.zeros, 0);
        if (tid == 0) __builtin_amdgcn_s_waitcnt(0);  // its stores done before the others read them
        __syncthreads();
        T = ld_sc1(&rs->prefix);
        const uint32_t mask2 = 0x7ffffe00u;
        for (uint32_t t = 0; t < nt; ++t) {
            uint32_t cg = 0, ce = 0;
            const uint32_t n = sup_n[t];
            if (n <= SUP_CAP) {
                for (uint32_t j = tid; j < n; j += FWGT) {
                    const uint32_t key = mag(sup[(size_t)t * SUP_CAP + j].y);
                    if ((key & mask2) == prefix) { cg += key > T; ce += key == T; }
                }
            } else {
                const size_t base = (size_t)t * TV_TILE, end = std::min<size_t>(m, base + TV_TILE);
                for (size_t e = base + tid; e < end; e += FWGT) {
                    uint32_t key = mag(f2u(a[e]));
                    if (e == m - 1) key &= last_mask;
                    if (key >= lo && (key & mask2) == prefix) { cg += key > T; ce += key == T; }
                }
            }
            cg = wave_sum(cg);
            ce = wave_sum(ce);
            if (__lane_id() == 0) { if (cg) atomicAdd(&g[t], cg); if (ce) atomicAdd(&q[t], ce); }
        }
        if (tid == 0) s_above = ld_sc1(&rs->cnt_gt) - cnt_gt;
    }
    __syncthreads();
    // exclusive prefixes over the tiles, 8 consecutive tiles per thread
    uint32_t cg = 0, ce = 0;
    constexpr uint32_t PT8 = 8;
    for (uint32_t t0 = 0; t0 < nt; t0 += PT8 * FWGT) {
        const uint32_t tb = t0 + PT8 * tid;
        uint32_t sg = 0, sq = 0;
#pragma unroll
        for (uint32_t i = 0; i < PT8; ++i)
            if (tb + i < nt) { sg += g[tb + i]; sq += q[tb + i]; }
        uint32_t tg, tq;
        uint32_t pg = cg + blk_excl_scan<FNWT>(sg, sh, &tg);
        uint32_t pq = ce + blk_excl_scan<FNWT>(sq, sh, &tq);
#pragma unroll
        for (uint32_t i = 0; i < PT8; ++i) {
            if (tb + i < nt) {
                tile_gt[tb + i] = g[tb + i];
                tile_eq[tb + i] = q[tb + i];
                tile_gt[nt + tb + i] = pg;
                tile_eq[nt + tb + i] = pq;
                pg += g[tb + i];
                pq += q[tb + i];
            }
        }
        cg += tg;
        ce += tq;
    }
    if (tid == 0) {
        tile_gt[2 * nt] = cg;
        tile_eq[2 * nt] = ce;
        if (listed) {  // the select's result, as the histogram levels leave it
            rs->prefix = T;
            rs->cnt_gt = cnt_gt + s_above;
            rs->rank = rank - s_above;
        }
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
    uint32_t *fail;      // the workspace's sticky failure word
    const RSel *rs;
    const uint32_t *tile_gt;
    const uint32_t *tile_eq;
    const uint2 *sup;
    const uint32_t *sup_n;
};

// A winner ranked past k: the select's counts and the tiles disagree (never
// with a consistent select).  The write is dropped (kept in bounds), the
// sticky failure word gets FAIL_SELECT and the count is poisoned, so the call
// fails loudly (stg_codec_check, compress_host) instead of returning a short
// stream with STG_OK.
__device__ __forceinline__ void select_broken(const TkArgs &a) {
    g_or(a.fail, FAIL_SELECT);
    __hip_atomic_fetch_max(gp(a.count_out), POISON_COUNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One workgroup per tile: the winners (> T, then == T in index order until
// k) at their prefix offsets, from the tile's superset.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tk_emit2(TkArgs a) {
    __shared__ uint32_t sh[STG_WAVES + 1];
    const uint32_t tile = blockIdx.x, tid = threadIdx.x, nt = a.ntiles;
    const uint32_t T = a.rs->prefix;
    const uint64_t need_eq = (uint64_t)a.k - a.rs->cnt_gt;  // ties to take, in index order
    const uint32_t cg = a.tile_gt[tile], ce = a.tile_eq[tile];
    const uint64_t gt_before = a.tile_gt[nt + tile], eq_before = a.tile_eq[nt + tile];
    if (cg || (ce && eq_before < need_eq)) {  // uniform per workgroup
        const uint32_t n = a.sup_n[tile];
        if (n <= SUP_CAP) {
            // four consecutive entries per thread: ranks by two workgroup scans
            const uint2 *src = a.sup + (size_t)tile * SUP_CAP;
            uint2 x[4];
            uint32_t qe = 0, qg = 0;
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                const uint32_t j = 4 * tid + r;
                x[r] = j < n ? src[j] : make_uint2(0u, 0u);
                const uint32_t key = mag(x[r].y);
                if (j < n && key > T) qg |= 1u << r;
                if (j < n && key == T) qe |= 1u << r;
            }
            uint32_t tot;
            uint32_t er = wg_excl_scan((uint32_t)__popc(qe), sh, &tot);
            uint32_t qw = qg;
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r)
                if ((qe >> r) & 1u) { if (eq_before + er < need_eq) qw |= 1u << r; ++er; }
            uint32_t wr = wg_excl_scan((uint32_t)__popc(qw), sh, &tot);
            const uint64_t win_before = gt_before + std::min(eq_before, need_eq);
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                if ((qw >> r) & 1u) {
                    const uint64_t slot = win_before + wr++;
                    if (slot >= a.k) { select_broken(a); continue; }  // an inconsistent select: surfaced
                    a.idx[slot] = a.bug_compat ? (uint32_t)slot : x[r].x + (uint32_t)a.idx_offset;
                    a.val[slot] = u2f(x[r].y);
                }
            }
        } else {  // the tile overflowed its superset: from the bucket itself
            __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
            float4 v[TILE_U];
            const size_t base = (size_t)tile * TV_TILE;
            load_tile<VEC>(a.a, a.m, base, a.last_mask, v);
            uint32_t qg = 0, qe = 0;
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) {
                const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t key = mag(f2u(comp(v[u], j)));
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
                        if (slot >= a.k) { select_broken(a); continue; }  // an inconsistent select: surfaced
                        a.idx[slot] = a.bug_compat ? (uint32_t)slot : (uint32_t)(e + j) + (uint32_t)a.idx_offset;
                        a.val[slot] = comp(v[u], j);
                    }
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
    // the count, then the failure word again: a tile whose select_broken (fail
    // bit, then POISON_COUNT) came before that second read is seen there and
    // poisoned here; one that came after it stores its poison after ours
    if (tile == 0 && tid == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        if (!(ld_sc1(a.fail) & FAIL_SELECT)) {
            st_sc1(a.count_out, a.cap);
            __builtin_amdgcn_s_waitcnt(0);
            if (ld_sc1(a.fail) & FAIL_SELECT)  // (POISON_COUNT is the largest value: whichever store lands last, it stays)
                __hip_atomic_fetch_max(gp(a.count_out), POISON_COUNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
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
    const uint32_t ntiles = (uint32_t)((m + TV_TILE - 1) / TV_TILE);
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
    uint2 *sup = reinterpret_cast<uint2 *>(ws.sums);          // ntiles x SUP_CAP entries
    uint32_t *sup_n = ws.tile_cnt + 2 * (size_t)ntiles + 1;  // after the > T counts and their prefixes
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    hipError_t e = launch_radix_level1(a.src, m, last_mask, zeros, kk - 1, ws, a.num_cu, s);
    if (e != hipSuccess) return e;
    if (vec) tk_pass<true><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n);
    else tk_pass<false><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n);
    tk_pick<9, 11><<<1, 1024, 0, s>>>(ws.rsel, zeros);
    if (ntiles <= TOPK_LIST_TILES) {  // level 3 from the level-2 bin's list: two launches
        TkList L{reinterpret_cast<uint2 *>(ws.sums) + (size_t)ntiles * SUP_CAP, ntiles, zeros};
        if (vec) tk_resolve<true><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, L);
        else tk_resolve<false><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, L);
        if (vec) tk_final<true><<<1, FWGT, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, ws.tile_aux, L);
        else tk_final<false><<<1, FWGT, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, ws.tile_aux, L);
    } else {
        if (vec) tk_hist3<true><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n);
        else tk_hist3<false><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n);
        tk_pick<0, 9><<<1, 1024, 0, s>>>(ws.rsel, zeros);
        if (vec) tk_count2<true><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, ws.tile_aux);
        else tk_count2<false><<<ntiles, STG_WG, 0, s>>>(a.src, m, last_mask, ws.rsel, sup, sup_n, ws.tile_cnt, ws.tile_aux);
        tk_scan<<<1, STG_WG, 0, s>>>(ws.tile_cnt, ws.tile_aux, ntiles);
    }
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
    t.fail = ws.fail;
    t.rs = ws.rsel;
    t.tile_gt = ws.tile_cnt;
    t.tile_eq = ws.tile_aux;
    t.sup = sup;
    t.sup_n = sup_n;
    if (vec) tk_emit2<true><<<ntiles, STG_WG, 0, s>>>(t);
    else tk_emit2<false><<<ntiles, STG_WG, 0, s>>>(t);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
