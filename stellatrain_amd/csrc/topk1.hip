// topk1.hip -- Top-k by |x| in one launch, steered by the key's previous k-th
// magnitude (gfx950).
//
// Reference: TopkCompressor::impl_nth_element (compress/topk.cpp:28-46); the
// two modes and their semantics are topk.hip's (the shipped byte-count memcpy
// and slot indices, or the intended operator), emitted in index order with
// ties at the k-th magnitude T taken in index order.
//
// compress() carries the tensor's name (compressor.h:30), and a gradient's
// magnitude distribution moves little from one iteration to the next, so the
// key's last T (KeyState.t; the band's relative half width in KeyState.inc)
// fixes a band [F, H) = T_prev (1 -/+ d) that almost always holds this call's
// T.  Then one pass over the bucket replaces the select's passes:
//   STREAM  per 32 KiB tile: its superset {|x| >= F} in index order, its count
//           of keys >= H, the band's keys in a fine histogram (8,192 bins);
//   PICK    (one workgroup) T's band bin and its rank inside the bin, from the
//           histogram and the count above H -- or a miss;
//   COUNT   per tile, from its superset: keys above T's bin; the bin's keys
//           listed (a few per call);
//   EXACT   (one workgroup) T from the list, the bin's keys into the per-tile
//           (> T, == T) counts, their prefixes, the key's next hint;
//   EMIT    per tile: the winners from its superset at their prefix offsets.
// A band that misses T (or a key's first call) takes the select's way inside
// the same launch -- three radix levels over the bucket (H1/P1, H2/P2,
// H3/P3), per-tile counts (CNT, SCAN), EMIT re-reading the tiles -- and the
// band doubles for the next call.
//
// Work goes by tickets, so no unit is waited on before a running workgroup
// holds it: a multi-unit phase's tiles in 8 shards (tile % 8, each counter on
// a line of its own), a workgroup draining its home shard (blockIdx % 8: one
// XCD) and then the others; the workgroup whose unit completes a phase (the
// last shard's last unit) runs the single-unit phase after it, the rest wait
// for its flag, bounded.  Hand-offs are sc1 stores and loads, or device atomics.
#include <algorithm>

#include "select.h"
#include "tile.h"
#include "tv16_dev.h"

namespace stg {

namespace {

using tv16::bitlen;
using tv16::spin_expired;
using tv16::vm_drain;

#ifndef STG_TK1_STAMPS
#define STG_TK1_STAMPS 0  // diagnostics: phase times (100 MHz clock) into debug words 40..47
#endif
#define TK1_STAMP(w)                                                                                  \
    do {                                                                                              \
        if (STG_TK1_STAMPS && threadIdx.x == 0) A.dbg[w] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

constexpr uint32_t SUP_CAP1 = TOPK_SUP_CAP;
constexpr uint32_t NB_BAND = TK1_FINE;
constexpr uint32_t BINL = TK1_BINL;

enum : uint32_t {
    P_STREAM = 0, P_PICK, P_COUNT, P_EXACT,
    M_H1, M_P1, M_H2, M_P2, M_H3, M_P3, M_CNT, M_SCAN,
    P_EMIT, NPH
};
static_assert(NPH == TK1_NPH, "phases");

__device__ __forceinline__ uint32_t mag1(uint32_t bits) { return bits & 0x7fffffffu; }

struct T1Args {
    const float *a;
    uint64_t m, zeros;
    uint32_t last_mask, nt, k, cap;
    int32_t idx_offset;
    bool bug_compat;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    uint32_t *fail;
    KeyState *state;       // t: the previous call's T, inc: the band's relative half width, init: valid
    bool hinted;           // the key has a T from an earlier call (its first call takes the select's way)
    TopkCtl *ctl, *ctl_next;
    uint32_t tag;          // >= 1
    RSel *rs;              // the select's way
    uint2 *sup;            // per tile: superset {element, bits}, SUP_CAP1 entries
    uint32_t *sup_n;       // per tile: superset size
    uint32_t *sup_hi;      // per tile: keys >= H
    uint32_t *tile_gt, *tile_eq;  // scan_tiles layout: counts [0, nt), prefixes [nt, 2nt), totals [2nt]
    uint32_t *fine;        // band histogram (zero between calls)
    uint32_t *dbg;         // ws.misc: [38] calls resolved in the band, [39] calls that took the select's way
};

struct T1Lds {
    uint32_t s_wt[TILE_U * STG_WAVES + 1];
    uint32_t sh[STG_WAVES + 1];
    union {
        uint32_t h[2048];  // a select level's tile histogram
        uint2 bl[BINL];    // EXACT: T's bin
    } u;
    uint32_t v[16];
};

// shard s of a phase with U units holds units s, s + 8, ...
__device__ __forceinline__ uint32_t shard_units(uint32_t U, uint32_t s) { return U > s ? (U - s + TK1_SH - 1) / TK1_SH : 0u; }

// The band of this call from the key's hint.
struct Band {
    uint32_t F, H, sh;  // key bits: [F, H); fine bin = (key - F) >> sh
};
__device__ __forceinline__ Band band_of(const KeyState *st) {
    const float t = st->t, d = st->inc;
    Band b;
    b.F = mag1(f2u(t * (1.0f - d)));
    b.H = mag1(f2u(t * (1.0f + d)));
    if (b.H <= b.F) b.H = b.F + 1u;
    const uint32_t span = b.H - b.F;
    b.sh = bitlen(span - 1u) > 13u ? bitlen(span - 1u) - 13u : 0u;
    return b;
}

// ---------------------------------------------------------------------------
// multi-unit phase bodies (one tile each)
// ---------------------------------------------------------------------------
// STREAM: the tile's superset {|x| >= F} in index order (tk_pass's ranks), its
// count of keys >= H, the band's keys into the fine histogram
template <bool VEC>
__device__ __noinline__ void unit_stream(const T1Args &A, T1Lds &L, uint32_t tile, const Band B) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const size_t base = (size_t)tile * TV_TILE;
    const size_t m = A.m;
    float4 v[TILE_U];
    load_tile<VEC>(A.a, m, base, A.last_mask, v);
    uint32_t q = 0, pre[TILE_U], nhi = 0;
    uint32_t *const fine = A.fine;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag1(f2u(comp(v[u], j)));
            if (e + j < m && key >= B.F) {
                q |= 1u << (u * 4 + j);
                if (key >= B.H) ++nhi;
                else __hip_atomic_fetch_add(gp(&fine[(key - B.F) >> B.sh]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const uint32_t c = (uint32_t)__popc((q >> (4 * u)) & 0xfu);
        const uint32_t incl = wave_incl_scan(c);
        pre[u] = incl - c;
        if (lane == 63) L.s_wt[u * STG_WAVES + wave] = incl;
    }
    nhi = wave_sum(nhi);
    if (lane == 0) atomicAdd(&L.v[1], nhi);  // zeroed by the caller
    __syncthreads();
    if (tid < 64) {  // (u, wave) offsets: one wave scans the 32 counts
        constexpr uint32_t NW = TILE_U * STG_WAVES;
        static_assert(NW <= 64, "one wave scans the wave counts");
        const uint32_t x = tid < NW ? L.s_wt[tid] : 0u;
        const uint32_t inc = wave_incl_scan(x);
        if (tid < NW) L.s_wt[tid] = inc - x;
        if (tid == NW - 1) L.s_wt[NW] = inc;
    }
    __syncthreads();
    const uint32_t nsup = L.s_wt[TILE_U * STG_WAVES];
    if (nsup <= SUP_CAP1) {
        uint64_t *const dst = reinterpret_cast<uint64_t *>(A.sup + (size_t)tile * SUP_CAP1);
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
            uint32_t slot = L.s_wt[u * STG_WAVES + wave] + pre[u];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((q >> (u * 4 + j)) & 1u)
                    st_sc1(dst + slot++, ((uint64_t)f2u(comp(v[u], j)) << 32) | (uint32_t)(e + j));
        }
    }
    if (tid == 0) {
        st_sc1(&A.sup_n[tile], nsup);
        st_sc1(&A.sup_hi[tile], L.v[1]);
    }
}

// The tile's keys (superset entries, or the tile re-read when it overflowed
// its superset) >= lo, one at a time: f(element, bits).
template <bool VEC, typename F>
__device__ __forceinline__ void tile_keys(const T1Args &A, uint32_t tile, uint32_t lo, bool from_sup, F f) {
    const uint32_t n = from_sup ? ld_sc1(&A.sup_n[tile]) : SUP_CAP1 + 1u;
    if (n <= SUP_CAP1) {
        const uint64_t *src = reinterpret_cast<const uint64_t *>(A.sup + (size_t)tile * SUP_CAP1);
        uint64_t w[4];
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t j = 4 * threadIdx.x + r;
            w[r] = j < n ? ld_sc1(&src[j]) : 0ull;
        }
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r)
            if (4 * threadIdx.x + r < n) f((uint32_t)w[r], (uint32_t)(w[r] >> 32));
        return;
    }
    const size_t base = (size_t)tile * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(A.a, A.m, base, A.last_mask, v);
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (e + j < A.m && mag1(f2u(comp(v[u], j))) >= lo) f((uint32_t)(e + j), f2u(comp(v[u], j)));
    }
}

// COUNT: the tile's keys above T's band bin [blo, bhi); the bin's keys listed
template <bool VEC>
__device__ __noinline__ void unit_countband(const T1Args &A, T1Lds &L, uint32_t tile, uint32_t blo, uint32_t bhi) {
    const uint32_t tid = threadIdx.x;
    uint32_t above = 0;
    if (tid == 0) L.v[2] = 0;
    __syncthreads();
    tile_keys<VEC>(A, tile, blo, true, [&](uint32_t e, uint32_t bits) {
        const uint32_t key = mag1(bits);
        if (key >= bhi) ++above;
        else if (key >= blo) {
            const uint32_t x = atomicAdd(&L.v[2], 1u);
            if (x < BINL) L.u.bl[x] = make_uint2(e, key);
        }
    });
    uint32_t tot;
    (void)blk_excl_scan<STG_WAVES>(above, L.sh, &tot);
    const uint32_t nb = min(L.v[2], BINL);
    if (tid == 0) {
        st_sc1(&A.tile_gt[tile], tot);
        st_sc1(&A.tile_eq[tile], 0u);
        L.v[3] = nb ? g_add(&A.ctl->nbin_list, nb) : 0u;
        if (L.v[2] > BINL) g_add(&A.ctl->nbin_list, BINL + 1u);  // a crowded bin: EXACT gives up
    }
    __syncthreads();
    const uint32_t b0 = L.v[3];
    for (uint32_t i = tid; i < nb; i += STG_WG)
        if (b0 + i < BINL) {
            const uint2 x = L.u.bl[i];
            st_sc1(reinterpret_cast<uint64_t *>(A.ctl->binl) + b0 + i, ((uint64_t)x.y << 32) | x.x);
        }
}

// A select level's histogram over one tile (the keys under the prefix).
template <bool VEC, int SHIFT, int NBITS>
__device__ __noinline__ void unit_hist(const T1Args &A, T1Lds &L, uint32_t tile) {
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t NB = 1u << NBITS;
    for (uint32_t i = tid; i < NB; i += STG_WG) L.u.h[i] = 0;
    const uint32_t prefix = SHIFT == 20 ? 0u : ld_sc1(&A.rs->prefix), mask = SHIFT == 20 ? 0u : ld_sc1(&A.rs->mask);
    __syncthreads();
    const size_t base = (size_t)tile * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(A.a, A.m, base, A.last_mask, v);
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag1(f2u(comp(v[u], j)));
            if (e + j < A.m && (key & mask) == prefix) atomicAdd(&L.u.h[(key >> SHIFT) & (NB - 1u)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < NB; i += STG_WG)
        if (L.u.h[i]) g_add(&A.rs->hist[tile % RS_SHARDS][i], L.u.h[i]);
}

// CNT: the tile's keys > T and == T (the select's way)
template <bool VEC>
__device__ __noinline__ void unit_count(const T1Args &A, T1Lds &L, uint32_t tile) {
    const uint32_t tid = threadIdx.x, T = ld_sc1(&A.rs->prefix);
    const size_t base = (size_t)tile * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(A.a, A.m, base, A.last_mask, v);
    uint32_t gt = 0, eq = 0;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag1(f2u(comp(v[u], j)));
            if (e + j < A.m) { gt += key > T; eq += key == T; }
        }
    }
    uint32_t tg, tq;
    (void)blk_excl_scan<STG_WAVES>(gt, L.sh, &tg);
    (void)blk_excl_scan<STG_WAVES>(eq, L.sh, &tq);
    if (tid == 0) {
        st_sc1(&A.tile_gt[tile], tg);
        st_sc1(&A.tile_eq[tile], tq);
    }
}

__device__ __forceinline__ void t1_broken(const T1Args &A) {
    g_or(A.fail, FAIL_SELECT);
    st_sc1(A.count_out, POISON_COUNT);
}

// EMIT: the tile's winners (> T, then == T in index order until k) at their
// prefix offsets: from the superset, or from the tile itself.
template <bool VEC>
__device__ __noinline__ void unit_emit(const T1Args &A, T1Lds &L, uint32_t tile, uint32_t T, uint64_t need_eq,
                                       bool from_sup) {
    const uint32_t tid = threadIdx.x, nt = A.nt;
    const uint32_t cg = ld_sc1(&A.tile_gt[tile]), ce = ld_sc1(&A.tile_eq[tile]);
    const uint64_t gt_before = ld_sc1(&A.tile_gt[nt + tile]), eq_before = ld_sc1(&A.tile_eq[nt + tile]);
    if (!(cg || (ce && eq_before < need_eq))) return;
    const uint64_t win_before = gt_before + std::min(eq_before, need_eq);
    const uint32_t n = from_sup ? ld_sc1(&A.sup_n[tile]) : SUP_CAP1 + 1u;
    if (n <= SUP_CAP1) {
        const uint64_t *src = reinterpret_cast<const uint64_t *>(A.sup + (size_t)tile * SUP_CAP1);
        uint2 x[4];
        uint32_t qe = 0, qg = 0;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t j = 4 * tid + r;
            const uint64_t w = j < n ? ld_sc1(&src[j]) : 0ull;
            x[r] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
            const uint32_t key = mag1(x[r].y);
            if (j < n && key > T) qg |= 1u << r;
            if (j < n && key == T) qe |= 1u << r;
        }
        uint32_t tot;
        uint32_t er = blk_excl_scan<STG_WAVES>((uint32_t)__popc(qe), L.sh, &tot);
        uint32_t qw = qg;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r)
            if ((qe >> r) & 1u) { if (eq_before + er < need_eq) qw |= 1u << r; ++er; }
        uint32_t wr = blk_excl_scan<STG_WAVES>((uint32_t)__popc(qw), L.sh, &tot);
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            if ((qw >> r) & 1u) {
                const uint64_t slot = win_before + wr++;
                if (slot >= A.k) { t1_broken(A); continue; }
                A.idx[slot] = A.bug_compat ? (uint32_t)slot : x[r].x + (uint32_t)A.idx_offset;
                A.val[slot] = u2f(x[r].y);
            }
        }
        return;
    }
    float4 v[TILE_U];
    const size_t base = (size_t)tile * TV_TILE;
    load_tile<VEC>(A.a, A.m, base, A.last_mask, v);
    uint32_t qg = 0, qe = 0;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag1(f2u(comp(v[u], j)));
            if (e + j < A.m) {
                if (key > T) qg |= 1u << (u * 4 + j);
                else if (key == T) qe |= 1u << (u * 4 + j);
            }
        }
    }
    uint32_t se[TILE_U * 4], sw[TILE_U * 4], tot;
    tile_ranks(qe, se, L.s_wt, &tot);
    uint32_t qw = qg;
#pragma unroll
    for (uint32_t b = 0; b < TILE_U * 4; ++b)
        if (((qe >> b) & 1u) && eq_before + se[b] < need_eq) qw |= 1u << b;
    tile_ranks(qw, sw, L.s_wt, &tot);
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t b = u * 4 + j;
            if ((qw >> b) & 1u) {
                const uint64_t slot = win_before + sw[b];
                if (slot >= A.k) { t1_broken(A); continue; }
                A.idx[slot] = A.bug_compat ? (uint32_t)slot : (uint32_t)(e + j) + (uint32_t)A.idx_offset;
                A.val[slot] = comp(v[u], j);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// single-unit phases (the workgroup that completed the phase before)
// ---------------------------------------------------------------------------
// topk.hip's scan_tiles with sc1 stores: its prefixes are read by other
// workgroups of this launch (sc1 loads), not after a kernel boundary.
__device__ __noinline__ void scan_tiles1(uint32_t *tile_gt, uint32_t *tile_eq, uint32_t nt, uint32_t *sh) {
    uint32_t cg = 0, ce = 0;
    constexpr uint32_t PT = 8;
    for (uint32_t t0 = 0; t0 < nt; t0 += PT * STG_WG) {
        const uint32_t tb = t0 + PT * threadIdx.x;
        uint32_t g[PT], q[PT], sg = 0, sq = 0;
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) {
            g[i] = tb + i < nt ? ld_sc1(&tile_gt[tb + i]) : 0u;
            q[i] = tb + i < nt ? ld_sc1(&tile_eq[tb + i]) : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) { sg += g[i]; sq += q[i]; }
        uint32_t tg, tq;
        uint32_t pg = cg + blk_excl_scan<STG_WAVES>(sg, sh, &tg);
        uint32_t pq = ce + blk_excl_scan<STG_WAVES>(sq, sh, &tq);
#pragma unroll
        for (uint32_t i = 0; i < PT; ++i) {
            if (tb + i < nt) {
                st_sc1(&tile_gt[nt + tb + i], pg);
                st_sc1(&tile_eq[nt + tb + i], pq);
            }
            pg += g[i];
            pq += q[i];
        }
        cg += tg;
        ce += tq;
    }
    if (threadIdx.x == 0) {
        st_sc1(&tile_gt[2 * nt], cg);
        st_sc1(&tile_eq[2 * nt], ce);
    }
}

// PICK: T's band bin from the fine histogram and the keys >= H, or a miss
__device__ __noinline__ void pick_band(const T1Args &A, T1Lds &L) {
    const uint32_t tid = threadIdx.x, nt = A.nt;
    const uint32_t r = A.k - 1u;  // T's descending rank
    uint32_t hi = 0;
    for (uint32_t t = tid; t < nt; t += STG_WG) hi += ld_sc1(&A.sup_hi[t]);
    constexpr uint32_t PER = NB_BAND / STG_WG;
    uint32_t c[PER], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        c[j] = ld_sc1(&A.fine[NB_BAND - 1u - (PER * tid + j)]);
        s += c[j];
    }
    uint32_t th, tband;
    (void)blk_excl_scan<STG_WAVES>(hi, L.sh, &th);
    if (tid == 0) L.v[2] = 0xffffffffu;
    uint32_t above = blk_excl_scan<STG_WAVES>(s, L.sh, &tband);
    const bool hit = th <= r && r < th + tband;
    const uint32_t rr = r - th;
    if (hit) {
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            if (above <= rr && rr < above + c[j]) { L.v[2] = NB_BAND - 1u - (PER * tid + j); L.v[3] = rr - above; }
            above += c[j];
        }
    }
    // the histogram back to zero for the next call (16-byte sc1 stores)
    for (uint32_t i = tid; i < NB_BAND / 4u; i += STG_WG) st_sc1_zero16(A.fine, NB_BAND * 4u, 16u * i);
    __syncthreads();
    if (tid == 0) {
        const bool ok = hit && L.v[2] != 0xffffffffu;
        st_sc1(&A.ctl->miss, ok ? 0u : 1u);
        st_sc1(&A.ctl->pick_bin, ok ? L.v[2] : 0u);
        st_sc1(&A.ctl->pick_rin, ok ? L.v[3] : 0u);
        if (!ok) A.state->inc = fminf(2.0f * A.state->inc, 0.5f);
    }
}

// EXACT: T from the bin's list, its keys into the per-tile counts, the
// prefixes, the next hint -- or a miss (a crowded bin)
__device__ __noinline__ void exact_band(const T1Args &A, T1Lds &L) {
    const uint32_t tid = threadIdx.x;
    const uint32_t nb = ld_sc1(&A.ctl->nbin_list), rin = ld_sc1(&A.ctl->pick_rin);
    if (nb > BINL || rin >= nb) {
        if (tid == 0) {
            st_sc1(&A.ctl->miss, 1u);
            A.state->inc = fminf(2.0f * A.state->inc, 0.5f);
        }
        return;
    }
    for (uint32_t i = tid; i < nb; i += STG_WG) {
        const uint64_t w = ld_sc1(reinterpret_cast<const uint64_t *>(A.ctl->binl) + i);
        L.u.bl[i] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
    }
    __syncthreads();
    for (uint32_t i = tid; i < nb; i += STG_WG) {  // T: the key of descending rank rin in the bin
        const uint32_t key = L.u.bl[i].y;
        uint32_t gt = 0, eq = 0;
        for (uint32_t x = 0; x < nb; ++x) { gt += L.u.bl[x].y > key; eq += L.u.bl[x].y == key; }
        if (gt <= rin && rin < gt + eq) L.v[4] = key;
    }
    __syncthreads();
    const uint32_t T = L.v[4];
    for (uint32_t i = tid; i < nb; i += STG_WG) {
        const uint2 x = L.u.bl[i];
        if (x.y > T) g_add(&A.tile_gt[x.x / TV_TILE], 1u);
        else if (x.y == T) g_add(&A.tile_eq[x.x / TV_TILE], 1u);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    scan_tiles1(A.tile_gt, A.tile_eq, A.nt, L.sh);
    if (tid == 0) {
        const float Tp = A.state->t, d = A.state->inc, Tf = u2f(T);
        A.state->t = Tf;  // the next call's hint; the band narrows while T keeps landing near its middle
        A.state->inc = fabsf(Tf - Tp) < 0.25f * d * Tp ? fmaxf(0.75f * d, 1.0f / 512.0f) : d;
        st_sc1(&A.ctl->res_T, T);
        st_sc1(&A.ctl->miss, 0u);
        atomicAdd(&A.dbg[38], 1u);
    }
}

// ---------------------------------------------------------------------------
// the launch
// ---------------------------------------------------------------------------
// 2 workgroups per CU at least (<= 128 VGPRs); each phase body is its own
// function within that budget
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) __attribute__((amdgpu_waves_per_eu(4, 8))) tk_one(T1Args Ak) {
    __shared__ T1Lds L;
    // the arguments in LDS: the phase bodies take them by reference (a
    // reference to the kernel's argument block would be copied to scratch)
    __shared__ T1Args A;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) A = Ak;
    __syncthreads();
    TopkCtl *const C = A.ctl;
    if (blockIdx.x == 0) TK1_STAMP(40);
    if (blockIdx.x == 0) {  // the next call's control block (this call never touches it)
        constexpr uint32_t W4 = (uint32_t)(offsetof(TopkCtl, binl) / 16);
        for (uint32_t i = tid; i < W4; i += STG_WG)
            st_sc1_zero16(reinterpret_cast<uint32_t *>(A.ctl_next), (uint32_t)offsetof(TopkCtl, binl), 16u * i);
    }
    const Band B = band_of(A.state);
    const uint32_t home = blockIdx.x % TK1_SH;
    auto poison = [&]() {
        if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(A.count_out, POISON_COUNT); }
    };
    // wait for the single-unit phase p's flag (one lane polls, sparsely)
    auto wait_flag = [&](uint32_t p) -> bool {
        if (tid == 0) {
            uint32_t ok = 1;
            uint64_t st = 0;
            for (uint32_t sp = 0; ld_sc1(&C->flag[p]) != A.tag; ++sp) {
                __builtin_amdgcn_s_sleep(24);
                if (spin_expired(sp, st)) { ok = 0; break; }
            }
            L.v[8] = ok;
        }
        __syncthreads();
        const bool ok = L.v[8] != 0;
        __syncthreads();
        return ok;
    };
    // the single-unit phase p + 1 after multi-unit phase p
    auto run_single = [&](uint32_t p) {
        if (p == P_STREAM) TK1_STAMP(41);
        if (p == P_COUNT) TK1_STAMP(43);
        if (p == P_STREAM) {
            pick_band(A, L);
        } else if (p == P_COUNT) {
            exact_band(A, L);
        } else if (p == M_H1) {
            pick_level<20, 11, STG_WG, RS_SHARDS>(A.rs, A.zeros, A.k - 1u);
        } else if (p == M_H2) {
            pick_level<9, 11, STG_WG, RS_SHARDS>(A.rs, A.zeros, 0);
        } else if (p == M_H3) {
            pick_level<0, 9, STG_WG, RS_SHARDS>(A.rs, A.zeros, 0);
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            if (tid == 0) {
                const uint32_t T = ld_sc1(&A.rs->prefix);
                st_sc1(&C->res_T, T);
                atomicAdd(&A.dbg[39], 1u);
                A.state->t = u2f(T);
                if (!A.state->init) A.state->inc = 1.0f / 64.0f;
                A.state->init = 1;
            }
        } else if (p == M_CNT) {
            scan_tiles1(A.tile_gt, A.tile_eq, A.nt, L.sh);
        }
        vm_drain();
        __syncthreads();
        if (p == P_STREAM) TK1_STAMP(42);
        if (p == P_COUNT) TK1_STAMP(44);
        if (tid == 0) st_sc1(&C->flag[p + 1], A.tag);
    };
    // one multi-unit phase: take units until every shard is empty; the
    // workgroup completing the phase also runs the single-unit phase after it
    uint32_t blo = 0, bhi = 0;
    auto run_multi = [&](uint32_t p, uint32_t T, uint64_t need_eq, bool from_sup) {
        const uint32_t U = A.nt, nsh = min(U, TK1_SH);
        for (uint32_t si = 0; si < TK1_SH; ++si) {
            const uint32_t s = (home + si) % TK1_SH, su = shard_units(U, s);
            for (;;) {
                if (tid == 0) {  // a plain look first: an empty shard costs no atomic
                    L.v[9] = ld_sc1(&C->tk[p][s][0]) >= su ? su : g_add(&C->tk[p][s][0], 1u);
                    L.v[1] = 0;
                }
                __syncthreads();
                const uint32_t c = L.v[9];
                if (c >= su) { __syncthreads(); break; }
                const uint32_t tile = s + TK1_SH * c;
                if (p == P_STREAM) unit_stream<VEC>(A, L, tile, B);
                else if (p == P_COUNT) unit_countband<VEC>(A, L, tile, blo, bhi);
                else if (p == M_H1) unit_hist<VEC, 20, 11>(A, L, tile);
                else if (p == M_H2) unit_hist<VEC, 9, 11>(A, L, tile);
                else if (p == M_H3) unit_hist<VEC, 0, 9>(A, L, tile);
                else if (p == M_CNT) unit_count<VEC>(A, L, tile);
                else unit_emit<VEC>(A, L, tile, T, need_eq, from_sup);
                vm_drain();
                __syncthreads();
                if (tid == 0) {
                    uint32_t last = 0;
                    if (g_add(&C->done[p][s][0], 1u) + 1u == su && g_add(&C->sdone[p][0], 1u) + 1u == nsh) last = 1;
                    L.v[10] = last;
                }
                __syncthreads();
                if (L.v[10]) {
                    if (p == P_EMIT) {  // the count, then the failure word again (see topk.hip)
                        TK1_STAMP(45);
                        if (tid == 0) {
                            __builtin_amdgcn_s_waitcnt(0);
                            if (!(ld_sc1(A.fail) & FAIL_SELECT)) {
                                st_sc1(A.count_out, A.cap);
                                __builtin_amdgcn_s_waitcnt(0);
                                if (ld_sc1(A.fail) & FAIL_SELECT) st_sc1(A.count_out, POISON_COUNT);
                            }
                        }
                    } else {
                        run_single(p);
                    }
                }
                __syncthreads();
            }
        }
    };
    bool miss = !A.hinted;
    if (!miss) {
        run_multi(P_STREAM, 0, 0, false);
        if (!wait_flag(P_PICK)) { poison(); return; }
        miss = ld_sc1(&C->miss) != 0;
        if (!miss) {
            const uint32_t b = ld_sc1(&C->pick_bin);
            blo = B.F + (b << B.sh);
            bhi = min(B.H, blo + (1u << B.sh));
            run_multi(P_COUNT, 0, 0, false);
            if (!wait_flag(P_EXACT)) { poison(); return; }
            miss = ld_sc1(&C->miss) != 0;
        }
    }
    if (miss) {
        const uint32_t seq[4] = {M_H1, M_H2, M_H3, M_CNT};
        for (uint32_t i = 0; i < 4; ++i) {
            run_multi(seq[i], 0, 0, false);
            if (!wait_flag(seq[i] + 1u)) { poison(); return; }
        }
    }
    const uint32_t T = ld_sc1(&C->res_T);
    const uint64_t tgt = ld_sc1(&A.tile_gt[2 * A.nt]), teq = ld_sc1(&A.tile_eq[2 * A.nt]);
    const uint64_t need_eq = (uint64_t)A.k - tgt;
    // implicit +0.0 elements past the copied bytes (bug-compat only): they tie at T == 0 after every real element
    if (blockIdx.x == 0 && A.zeros && T == 0) {
        const uint64_t first = tgt + std::min<uint64_t>(teq, need_eq);
        for (uint64_t s = first + tid; s < A.k; s += STG_WG) {
            A.idx[s] = (uint32_t)s;
            A.val[s] = 0.f;
        }
    }
    if (blockIdx.x == 0) TK1_STAMP(46);  // workgroup 0 reaches the emission
    run_multi(P_EMIT, T, need_eq, !miss);
}

}  // namespace

hipError_t launch_topk1(const TopkLaunch &a, const DevWS &ws, KeyState *state, bool hinted, uint32_t tag,
                        hipStream_t s) {
    if (a.k == 0 || a.n == 0 || !tag) return hipErrorInvalidValue;
    uint64_t m = a.n, zeros = 0;
    uint32_t last_mask = 0xffffffffu;
    if (a.bug_compat) {  // memcpy(clone, src, n) copies n bytes (topk.cpp:31)
        m = a.n / 4 + (a.n % 4 ? 1 : 0);
        if (a.n % 4) last_mask = (1u << (8 * (a.n % 4))) - 1u;
        zeros = a.n - m;
    }
    const uint32_t nt = (uint32_t)((m + TV_TILE - 1) / TV_TILE);
    if (nt > TOPK_LIST_TILES) return hipErrorInvalidValue;
    T1Args A{};
    A.a = a.src;
    A.m = m;
    A.zeros = zeros;
    A.last_mask = last_mask;
    A.nt = nt;
    A.k = (uint32_t)std::min<uint64_t>(a.k, a.n);
    A.cap = a.cap;
    A.idx_offset = a.idx_offset;
    A.bug_compat = a.bug_compat;
    A.idx = a.idx;
    A.val = a.val;
    A.count_out = a.count_out;
    A.fail = ws.fail;
    A.state = state;
    A.hinted = hinted;
    A.ctl = ws.tkctl + (tag & 1u);
    A.ctl_next = ws.tkctl + ((tag + 1u) & 1u);
    A.tag = tag;
    A.rs = ws.rsel;
    A.sup = reinterpret_cast<uint2 *>(ws.sums);
    A.tile_gt = ws.tile_cnt;
    A.tile_eq = ws.tile_aux;
    A.sup_n = ws.tile_cnt + 2 * (size_t)nt + 1;
    A.sup_hi = ws.tile_aux + 2 * (size_t)nt + 1;
    A.fine = ws.tkfine;
    A.dbg = ws.misc;
    const uint32_t G = std::min<uint32_t>(nt, (uint32_t)a.num_cu * 2u);
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
    if (vec) tk_one<true><<<G, STG_WG, 0, s>>>(A);
    else tk_one<false><<<G, STG_WG, 0, s>>>(A);
    if (a.ev) { (void)hipEventRecord(a.ev[1], s); (void)hipEventRecord(a.ev[2], s); }
    return hipGetLastError();
}

}  // namespace stg
