// tv16wide.h -- thresholdv16's regime-B fill when the window cannot order it:
// the leader (an exact ordering of the pops over a candidate list in global
// memory) and the crew (a window-miss bucket's top candidates found again by
// many workgroups).  Included by tv16fill.hip in its anonymous namespace,
// after tv16lfin.h.
//
// Reference: thresholdv16.cpp:261-293 (the priority_queue fill), :243-259
// (AIMD: t decays by only 1 % per regime-B call, so after a drop of the
// gradient scale a key stays many calls in regime B with every line sum far
// below the window the scan lists).
//
// Why the pop order is computable without the heap (tv16fill.hip (1)-(3)):
//  * distinct sums pop in sum order, whatever the heap looks like;
//  * a run of equal sums s pops in right-first pre-order of its members'
//    positions once every member has had its own sift (an element moves down
//    only as the value of its own sift, inside its start subtree; afterwards it
//    moves up only, a node takes the larger child entry -- the right one on
//    equal sums -- so of two members in disjoint subtrees the right one passes
//    their common ancestor first, and a member above another pops first),
//    provided no element >= s is ever re-inserted by pop_heap (checked: no such
//    element ends make_heap in the last P + 1 positions);
//  * make_heap moves an element of R_s = {sum >= s} only through comparisons
//    with elements of R_s (tv16fill.hip (1)), so a subtree's make_heap can be
//    replayed with every other candidate as -inf.
// So the leader sorts R by (sum desc, right-first key of the start position),
// and only where a run has a member whose start is above another member's, or a
// late line of R_s has an R_s line at its parent or sibling, it replays the
// make_heap of that small subtree exactly (libstdc++'s __adjust_heap, dense, in
// LDS) and orders the run by the replayed positions.  Anything it cannot bound
// (NaN sums, a subtree above height 12, a run of more than 512 equal sums, R
// past its scratch) goes to the literal heap, exactly as before.
//
// The crew: a window-miss bucket (regime B with fewer than M lines in the
// window just below t) has its top candidates nowhere, so extra workgroups of
// the fill launch, each taking units in ticket order, find them again:
//   Z  zero the bucket's level-1 histogram                              (1 unit)
//   A  stream la lines (la: the bucket over the crew): line sums in the
//      scan's AVX tree order, the ordered key of each line (0 for a
//      qualifying line) into the scratch, the candidates' histogram of the
//      key's top 13 bits                                                 (nb / la)
//   C  pick the bin holding the (min(P0 + 1, N - 1) + 1)-th largest key
//      (every unit, from the histogram), list every candidate in that bin
//      or above, in scan order, with its candidate index (look-back over
//      the units' tagged counts)                                         (nb / 16384)
//   D  the leader over the list                                          (1 unit)
//   E  emit the pops                                                     (32 units)
// A unit waits only for units with smaller tickets (the previous phase of its
// bucket; the same phase of the bucket before), every wait bounded.
#pragma once

constexpr uint32_t WBINS = 8192;  // crew level-1 bins: the ordered key's top 13 bits (1/16 octave)
constexpr uint32_t WSH = 19;
constexpr uint32_t WTILE = 4096;  // leader: entries ranked per LDS tile (a bin never spans two)
constexpr uint32_t WHMAX = 12;    // leader: the largest subtree replayed (8,191 nodes)
constexpr uint32_t WSIM = (2u << WHMAX) - 1;
constexpr uint32_t WHL = 6;       // a late line's subtree: its ancestor 6 levels up
constexpr uint32_t WROOTS = 64;   // replayed subtrees at most
constexpr uint32_t WRUN = 512;    // equal sums re-ordered after a replay at most
constexpr uint32_t WRFD = 27;     // rf32: heap positions < 2^28 - 1
constexpr uint32_t CW_LA = 2048;  // crew phase A: lines per unit at least (128 KiB)
constexpr uint32_t CW_LC = 8192;  // crew phase C: keys per unit (16 per thread)
constexpr uint32_t CW_NE = 32;    // crew phase E: emission units
constexpr uint32_t CW_DA = 6;     // crew phase A: float4 loads in flight per lane (batched fill launches)
constexpr uint32_t CW_DA_LONE = 12;  // ... one-bucket launches
constexpr uint32_t CW_PH = 5;     // phases Z A C D E
constexpr uint32_t LNONE = 0x7fffffffu;
#ifndef STG_CREW_STAMPS
#define STG_CREW_STAMPS 0  // diagnostics: crew phase completion times (100 MHz clock), debug words 16..23
#endif
static_assert(CW_LC == 16 * FILL_WG && CW_LC <= 0xffffu, "phase C: 16 keys per thread; 16-bit unit counts");

// A window-miss bucket as the crew sees it.
struct CrewBk {
    Tv16FillBucket d;
    uint32_t slot, cnt, rem, N, tbits, tail, tail_bits;
    uint32_t la, nA, nC;  // A: lines per unit, units; C: units
};

// LDS of the leader and the crew (a view of the fill launch's dynamic LDS):
// WT entries of R ranked per tile, NBH bins while sorting.  The batched fill
// launch shares its CU with two scan workgroups (WideLds: 4,096 / 8,192); the
// one-bucket (lfin) launch has the CU to itself, so its crew ranks 11,264
// entries per tile (the 10.5 k pops of a 64 MiB bucket in one pass over the
// list) with 4,096 bins (WideLdsBig, ~153 KB).
template <uint32_t WT_, uint32_t NBH_>
struct WideLdsT {
    static constexpr uint32_t WT = WT_, NBH = NBH_;
    static_assert(NBH >= 2048 && (NBH & (NBH - 1u)) == 0 && NBH <= WBINS, "sort bins");
    static_assert(WT <= 2u * (WSIM + 1u), "the late-line list fits the replay's LDS");
    union {
        uint32_t hist8[WBINS];     // the crew's phases: level-1 bins, the emission shares' positions
        struct {
            uint32_t hist[NBH];    // bins (select, sort)
            uint64_t tk[WT];       // ranking tile: composite keys (the run reorder: two words of each entry)
            uint32_t ti[WT];       // ... their list entries
        } s;
        uint2 sim[WSIM + 1];       // a replayed subtree: {ordered key (0: -inf), list entry}
    } u;
    uint32_t sh[32];
    uint32_t roots[WROOTS];
    uint32_t lvl[2 * (WHMAX + 2)];  // replay gather: first list entry / prefix per level
    uint32_t v[16];                 // scalars
    CrewBk bk[MAX_BATCH];
    uint32_t tb[MAX_BATCH + 1];             // first ticket of each requested bucket
    uint32_t cp[CW_PH][MAX_BATCH + 1];      // units of phase p in the requested buckets before j
    uint32_t nreq;
};

using WideLds = WideLdsT<WTILE, WBINS>;
using WideLdsBig = WideLdsT<11264, 4096>;
static_assert(sizeof(WideLds) <= sizeof(FillLds), "the wide views fit the fill's LDS");
static_assert(sizeof(WideLdsBig) <= 160 * 1024, "one lfin workgroup per CU");

// canonical ordered key of a sum: -0 -> +0 (the reference's float compare ties them)
__device__ __forceinline__ uint32_t okey(uint32_t b) {
    if (!(b & 0x7fffffffu)) b = 0u;
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ bool nan_bits(uint32_t b) { return (b & 0x7fffffffu) > 0x7f800000u; }
// right-first pre-order key of heap position pos (< 2^28 - 1): ancestors first,
// then the right subtree before the left one
__device__ __forceinline__ uint32_t rf32(uint32_t pos) {
    const uint32_t q = pos + 1, d = depth_of(q);
    const uint32_t inv = ~(q - (1u << d)) & ((1u << d) - 1u);
    return ((inv << (WRFD - d)) << 5) | d;
}

struct LeadIn {
    const uint32_t *lk, *lp, *lc;  // the list in scan order: sum bits (>= +0), element position, candidate index
    uint32_t n;
    uint32_t tail, tail_bits;      // tail = 1: the ragged tail is entry n (candidate N - 1, position nb * 16)
    uint32_t N, nb, rem, tl;
    uint32_t *g;                   // scratch words (8-byte aligned)
    uint32_t gcap;
    uint32_t *dbg;                 // stamp builds: the leader's step times, words 24..28
    uint32_t lvl1, r1;             // lvl1 != NONE: the key at rank sel has top 13 bits lvl1, rank r1 among them
    bool positions;                // also resolve the pops' element positions (ordpos); the crew's
                                   // emission units resolve them from `order` themselves
};
struct LeadOut {
    bool ok;
    uint32_t P, tail_rank;
    const uint32_t *ordpos;  // element position of each pop (I.positions)
    const uint32_t *order;   // list entry of each pop (| 2^31 when tied)
    uint32_t why;            // failure: 1 NaN, 2 scratch, 3 crowded bin / rank not found, 4 short list, 5 roots, 6 height, 7 late, 8 run
};

// Bounded poll by thread 0 until *w >= target; every thread gets the verdict.
__device__ __forceinline__ bool wide_wait(uint32_t *w, uint32_t target, uint32_t *flag) {
    if (threadIdx.x == 0) {
        uint32_t ok = 1;
        uint64_t st = 0;
        uint32_t nap = 1;  // backing off: many waiters on one line slow everyone's memory path
        for (uint32_t sp = 0; ld_sc1(w) < target; ++sp) {
            for (uint32_t k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(4);
            nap = min(2u * nap, 16u);
            if (spin_expired(sp, st)) { ok = 0; break; }
        }
        *flag = ok;
    }
    __syncthreads();
    const bool r = *flag != 0;
    __syncthreads();
    return r;
}

// Batched loops: each thread loads B entries (all in flight), then uses them
// -- a loop whose every iteration waits for its own load runs at one L2 round
// trip per iteration.  The loads are unconditional (an index past the end
// loads entry n - 1 again): a load under a branch gets a wait for it at the
// branch's join, which serialises the batch again.  ld must not branch either.
constexpr uint32_t WB = 8;
template <typename V, uint32_t B = WB, typename Ld, typename Use>
__device__ __forceinline__ void each_b(uint32_t n, Ld ld, Use use) {
    for (uint32_t i0 = 0; i0 < n; i0 += B * FILL_WG) {
        V v[B];
#pragma unroll
        for (uint32_t b = 0; b < B; ++b) v[b] = ld(min(i0 + b * FILL_WG + threadIdx.x, n - 1u));
#pragma unroll
        for (uint32_t b = 0; b < B; ++b) {
            const uint32_t i = i0 + b * FILL_WG + threadIdx.x;
            if (i < n) use(i, v[b]);
        }
    }
}
// ... with a second load that depends on the first (two round trips per batch)
template <typename V1, typename V2, typename Ld1, typename Ld2, typename Use>
__device__ __forceinline__ void each_b2(uint32_t n, Ld1 ld1, Ld2 ld2, Use use) {
    for (uint32_t i0 = 0; i0 < n; i0 += WB * FILL_WG) {
        V1 a[WB];
        V2 v[WB];
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) a[b] = ld1(min(i0 + b * FILL_WG + threadIdx.x, n - 1u));
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) v[b] = ld2(min(i0 + b * FILL_WG + threadIdx.x, n - 1u), a[b]);
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) {
            const uint32_t i = i0 + b * FILL_WG + threadIdx.x;
            if (i < n) use(i, a[b], v[b]);
        }
    }
}
struct KC4 {
    u4v k, c;  // four list entries: sum bits, candidate indices
};
struct Adj {
    uint32_t o, o2;  // two neighbours of R: entries (with the tie bit)
    uint64_t s, s2;  // ... their composite keys
};
// the heap position of a right-first key (the inverse of rf32)
__device__ __forceinline__ uint32_t rf_pos(uint32_t r) {
    const uint32_t d = r & 31u, inv = (r >> 5) >> (WRFD - d), mk = (1u << d) - 1u;
    return ((1u << d) | (~inv & mk)) - 1u;
}

// plain loads (see the leader)
__device__ __forceinline__ uint32_t ldc(const uint32_t *p) { return *p; }
__device__ __forceinline__ uint64_t ldc(const uint64_t *p) { return *p; }

#define LEAD_STAMP(i)                                                                                       \
    do {                                                                                                    \
        if (STG_CREW_STAMPS && threadIdx.x == 0) I.dbg[24 + (i)] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
// finer steps (stamp builds): words 8..15, and the list / R sizes in 6, 7
#define LEAD_SUB(i)                                                                                         \
    do {                                                                                                    \
        if (STG_CREW_STAMPS && threadIdx.x == 0) I.dbg[8 + (i)] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

// The leader: the pops of a regime-B fill over a candidate list that holds
// every candidate of the top min(P0 + 2, N) (P0 = ceil(rem / 16)); candidates
// not listed have smaller sums than every listed one of R.  One workgroup;
// every pass over global data keeps WB loads per thread in flight (the list as
// 16-byte loads), and lookups by candidate index go through an LDS sample.
template <class WL>
__device__ __noinline__ LeadOut leader(WL &W, const LeadIn I) {
    constexpr uint32_t WT = WL::WT, NBH = WL::NBH, NBL = 31u - __builtin_clz(NBH);
    LeadOut O;
    O.ok = false;
    O.P = 0;
    O.tail_rank = NONE;
    O.why = 0;
    const uint32_t tid = threadIdx.x;
    // Loads go through this XCD's L2 (cached: the list and the scratch are
    // read many times); the acquire drops lines other XCDs have since written.
    // The scratch only this workgroup reads is stored plain (its L2): on this
    // chip vmcnt counts stores with loads, in order, so a load issued after an
    // sc1 store (written through to HBM) waits for that store.  What other
    // workgroups read (the pops' order, their positions) is stored sc1.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t n = uni(I.n), tail = uni(I.tail), tbits = uni(I.tail_bits), NN = uni(I.N);
    const uint32_t m = n + tail;
    const uint32_t *const lk = uni_ptr(I.lk), *const lp = uni_ptr(I.lp), *const lc = uni_ptr(I.lc);
    if (!m) { O.ok = true; return O; }
    // entry i (i == n: the tail); branch-free (see each_b)
    const uint32_t nl = n ? n - 1u : 0u, tpos = uni(I.nb) * 16u;
    auto kb = [&](uint32_t i) -> uint32_t { const uint32_t x = ldc(&lk[min(i, nl)]); return i < n ? x : tbits; };
    auto cx = [&](uint32_t i) -> uint32_t { const uint32_t x = ldc(&lc[min(i, nl)]); return i < n ? x : NN - 1u; };
    auto ps = [&](uint32_t i) -> uint32_t { const uint32_t x = ldc(&lp[min(i, nl)]); return i < n ? x : tpos; };
    if ((size_t)6 * m + 8 > uni(I.gcap) || NN >= (1u << 28)) { O.why = 2; return O; }
    uint32_t *const g = uni_ptr(I.g);
    // R in order: entries (with the tie bit), composite keys; positions; the pops' positions
    uint32_t *const go = g, *const gp = go + m, *const op = gp + m;
    uint64_t *const gs = reinterpret_cast<uint64_t *>(g + 4 * (size_t)m);
    const uint32_t *const gs32 = reinterpret_cast<const uint32_t *>(gs);
    const uint32_t P0 = (uni(I.rem) + 15u) / 16u;
    const uint32_t sel = min(P0 + 1u, m - 1u);
    uint32_t *const hist = W.u.s.hist;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(lk), 0, n * 4u, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(lc), 0, n * 4u, 0x00020000);
    const uint32_t nq = (n + 3u) / 4u;
    auto ld4 = [&](__amdgpu_buffer_rsrc_t r, uint32_t q) -> u4v {
        return __builtin_amdgcn_raw_buffer_load_b128(r, q * 16u, 0, 0);
    };
    auto keys4 = [&](auto use) {  // use(entry, sum bits) for every entry
        each_b<u4v>(nq, [&](uint32_t q) { return ld4(rk, q); }, [&](uint32_t q, u4v x) {
            const uint32_t i = 4u * q;
            use(i, x.x);
            if (i + 1u < n) use(i + 1u, x.y);
            if (i + 2u < n) use(i + 2u, x.z);
            if (i + 3u < n) use(i + 3u, x.w);
        });
        if (tail && tid == 0) use(n, tbits);
    };

    // ---- 1. the key at descending rank sel: radix levels of 11, 11 and 10
    //      bits, the first skipped when the caller knows the top 13 bits ----
    uint32_t pre = 0, pm = 0, r = sel, p0 = 0;
    if (uni(I.lvl1) != NONE) {
        pre = uni(I.lvl1) << WSH;
        pm = ~((1u << WSH) - 1u);
        r = uni(I.r1);
        p0 = 1;
    }
    if (tid == 0) { W.v[0] = 0; W.v[1] = 0; }
    for (uint32_t pass = p0; pass < 3; ++pass) {
        const uint32_t sh = pass == 0 ? 21u : pass == 1 ? 10u : 0u, nbin = pass == 2 ? 1024u : 2048u;
        const bool first = pass == p0;
        for (uint32_t b = tid; b < nbin; b += FILL_WG) hist[b] = 0;
        if (tid == 0) W.v[2] = NONE;
        __syncthreads();
        uint32_t kmx = 0, nanf = 0;
        keys4([&](uint32_t, uint32_t b) {
            const uint32_t k = okey(b);
            if (first) {
                nanf |= nan_bits(b) ? 1u : 0u;
                kmx = max(kmx, k);
            }
            if ((k & pm) == pre) atomicAdd(&hist[(k >> sh) & (nbin - 1u)], 1u);
        });
        if (first) {
            kmx = wave_max(kmx);
            if ((tid & 63u) == 0) atomicMax(&W.v[1], kmx);
            if (nanf) W.v[0] = 1;
        }
        __syncthreads();
        const uint32_t per = nbin / FILL_WG;  // 4 or 2 bins per thread, highest first
        uint32_t c[8], s = 0;
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            c[u] = u < per ? hist[nbin - 1u - (per * tid + u)] : 0u;
            s += c[u];
        }
        uint32_t tot;
        uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            if (u < per && a <= r && r < a + c[u]) { W.v[2] = nbin - 1u - (per * tid + u); W.v[3] = r - a; }
            a += c[u];
        }
        __syncthreads();
        if (W.v[0]) { O.why = 1; return O; }
        if (W.v[2] == NONE) { O.why = 3; return O; }
        pre |= uni(W.v[2]) << sh;
        pm |= (nbin - 1u) << sh;
        r = uni(W.v[3]);
        __syncthreads();
    }
    const uint32_t okS = uni(pre), kmax = uni(W.v[1]);
    LEAD_STAMP(0);

    // ---- 2. R = {key >= okS} by (key desc, rf32(start) asc): counting sort
    //      into bins of the key's distance below the maximum, then ranks
    //      inside each bin, one LDS tile of whole bins at a time ----
    const uint32_t D = kmax - okS, shb = bitlen(D) > NBL ? bitlen(D) - NBL : 0u, nbin = (D >> shb) + 1u;
    for (uint32_t b = tid; b < nbin; b += FILL_WG) hist[b] = 0;
    if (tid == 0) { W.v[4] = 0; W.v[5] = 0; }
    __syncthreads();
    uint32_t nr = 0;
    keys4([&](uint32_t, uint32_t b) {
        const uint32_t k = okey(b);
        if (k >= okS) { atomicAdd(&hist[(kmax - k) >> shb], 1u); ++nr; }
    });
    nr = wave_sum(nr);
    if ((tid & 63u) == 0) atomicAdd(&W.v[4], nr);
    __syncthreads();
    nr = uni(W.v[4]);
    LEAD_SUB(0);
    if (STG_CREW_STAMPS && tid == 0) { I.dbg[6] = m; I.dbg[7] = nr; }
    {   // exclusive scan of the bins (NBH / FILL_WG per thread), and the largest bin
        constexpr uint32_t PB = NBH / FILL_WG;
        uint32_t c[PB], s = 0, mx = 0;
#pragma unroll
        for (uint32_t u = 0; u < PB; ++u) {
            const uint32_t b = PB * tid + u;
            c[u] = b < nbin ? hist[b] : 0u;
            s += c[u];
            mx = max(mx, c[u]);
        }
        uint32_t tot;
        uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
        for (uint32_t u = 0; u < PB; ++u) {
            const uint32_t b = PB * tid + u;
            if (b < nbin) hist[b] = a;
            a += c[u];
        }
        mx = wave_max(mx);
        if ((tid & 63u) == 0) atomicMax(&W.v[5], mx);
        __syncthreads();
    }
    if (W.v[5] > WT) { O.why = 3; return O; }
    LEAD_SUB(1);
    // hist[b]: the start of bin b.  Tiles of whole bins: one pass over the
    // list (cached loads) places the tile's entries in LDS, where they are
    // ranked; only the ranked entries are stored (no load waits behind them).
    uint32_t tie_any = 0;
    for (uint32_t s0 = 0, b0 = 0; s0 < nr;) {
        if (tid == 0) {  // the largest b1 <= nbin with start(b1) <= s0 + WT (start(nbin) = nr)
            uint32_t lo = b0 + 1u, hi = nbin;
            while (lo < hi) {
                const uint32_t md = (lo + hi + 1u) >> 1;
                if ((md < nbin ? hist[md] : nr) <= s0 + WT) lo = md; else hi = md - 1u;
            }
            W.v[6] = lo;
        }
        __syncthreads();
        const uint32_t b1 = uni(W.v[6]), s1 = uni(b1 < nbin ? hist[b1] : nr);
        auto put = [&](uint32_t i, uint32_t bits, uint32_t c) {
            const uint32_t k = okey(bits);
            const uint32_t b = (kmax - k) >> shb;
            if (k < okS || b < b0 || b >= b1) return;
            const uint32_t slot = atomicAdd(&hist[b], 1u) - s0;
            W.u.s.tk[slot] = ((uint64_t)(kmax - k) << 32) | rf32(c);
            W.u.s.ti[slot] = i;
        };
        each_b<KC4, 4>(nq, [&](uint32_t q) { KC4 x; x.k = ld4(rk, q); x.c = ld4(rc, q); return x; }, [&](uint32_t q, KC4 x) {
            const uint32_t i = 4u * q;
            put(i, x.k.x, x.c.x);
            if (i + 1u < n) put(i + 1u, x.k.y, x.c.y);
            if (i + 2u < n) put(i + 2u, x.k.z, x.c.z);
            if (i + 3u < n) put(i + 3u, x.k.w, x.c.w);
        });
        if (tail && tid == 0) put(n, tbits, NN - 1u);
        __syncthreads();  // hist[b], b0 <= b < b1: the end of bin b
        if (s0 == 0) LEAD_SUB(6);
        const uint32_t nt = s1 - s0;
        for (uint32_t j = tid; j < nt; j += FILL_WG) {
            const uint64_t key = W.u.s.tk[j];
            const uint32_t b = (uint32_t)(key >> 32) >> shb;
            const uint32_t lo = (b > b0 ? hist[b - 1u] : s0) - s0, hi = hist[b] - s0;
            uint32_t rk = s0 + lo;
            bool tie = false;
            for (uint32_t x = lo; x < hi; ++x) {
                const uint64_t kx = W.u.s.tk[x];
                rk += kx < key;
                tie |= x != j && (uint32_t)(kx >> 32) == (uint32_t)(key >> 32);
            }
            tie_any |= tie ? 1u : 0u;
            go[rk] = W.u.s.ti[j] | (tie ? 0x80000000u : 0u);
            gs[rk] = key;
        }
        __syncthreads();
        if (s0 == 0) LEAD_SUB(7);
        s0 = s1;
        b0 = b1;
    }
    vm_drain();
    const bool ties = __syncthreads_or((int)tie_any);
    LEAD_STAMP(2);

    // ---- 3. runs of equal sums: start positions one above the other, or a
    //      late line of R_s with an R_s line beside it -> replay those subtrees ----
    const uint32_t late_lo = NN > sel + 2u ? NN - (sel + 2u) : 0u;
    if (ties) {
        uint32_t dmx = 0;  // the lowest tied key (largest distance below kmax)
        each_b<uint2>(nr, [&](uint32_t rr) { return make_uint2(ldc(&go[rr]), ldc(&gs32[2u * rr + 1u])); },
                      [&](uint32_t, uint2 x) { if (x.x >> 31) dmx = max(dmx, x.y); });
        dmx = wave_max(dmx);
        if (tid == 0) { W.v[7] = 0; W.v[8] = 0; }
        __syncthreads();
        if ((tid & 63u) == 0) atomicMax(&W.v[7], dmx);
        __syncthreads();
        dmx = uni(W.v[7]);
        LEAD_SUB(2);
        const uint32_t ksm = kmax - dmx;  // R_smin = {key >= ksm} = R's entries at distance <= dmx
        auto add_root = [&](uint32_t a) {
            const uint32_t x = atomicAdd(&W.v[8], 1u);
            if (x < WROOTS) W.roots[x] = a;
        };
        // (a) adjacent members of a run (rf32 order): the second below the first
        each_b<Adj>(nr ? nr - 1u : 0u,
                    [&](uint32_t rr) {
                        Adj a;
                        a.o = ldc(&go[rr]);
                        a.o2 = ldc(&go[rr + 1u]);
                        a.s = ldc(&gs[rr]);
                        a.s2 = ldc(&gs[rr + 1u]);
                        return a;
                    },
                    [&](uint32_t, Adj a) {
                        if (!(a.o >> 31) || !(a.o2 >> 31) || (uint32_t)(a.s >> 32) != (uint32_t)(a.s2 >> 32)) return;
                        const uint32_t ce = rf_pos((uint32_t)a.s), cf = rf_pos((uint32_t)a.s2);
                        if (is_desc(cf + 1u, ce + 1u)) add_root(ce);
                    });
        // lookups by candidate index: the list is in candidate order; smp[j] = cx(j S)
        const uint32_t S = (m + WT - 1u) / WT, ns = (m + S - 1u) / S;
        LEAD_SUB(3);
        uint32_t *const smp = W.u.s.ti;  // (past the replay's LDS)
        each_b<uint32_t>(ns, [&](uint32_t j) { return cx(j * S); }, [&](uint32_t j, uint32_t c) { smp[j] = c; });
        __syncthreads();
        auto lower = [&](uint32_t c) -> uint2 {  // the first entry with candidate index >= c, and that index
            uint32_t lo = 0, hi = ns;
            while (lo < hi) {
                const uint32_t md = (lo + hi) >> 1;
                if (smp[md] < c) lo = md + 1u; else hi = md;
            }
            if (lo == 0) return make_uint2(0u, smp[0]);
            const uint32_t base = (lo - 1u) * S, end = min(lo * S, m);  // cx(base) < c <= cx(end)
            uint32_t rr = end, rcx = lo < ns ? smp[lo] : NONE;
            for (uint32_t i0 = base + 1u; i0 < end && rr == end; i0 += 8u) {
                uint32_t v[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u) {
                    const uint32_t x = cx(min(i0 + u, end - 1u));
                    v[u] = i0 + u < end ? x : NONE;
                }
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u)
                    if (rr == end && v[u] != NONE && v[u] >= c) { rr = i0 + u; rcx = v[u]; }
            }
            return make_uint2(rr, rcx);
        };
        auto member = [&](uint32_t c) {
            const uint2 f = lower(c);
            return f.x < m && f.y == c && okey(kb(f.x)) >= ksm;
        };
        // (b) late lines of R_smin (start >= late_lo) with an R_smin line at
        //     the parent or sibling: the late lines listed first (in the
        //     replay's LDS, free here), then one lookup pair per thread
        uint32_t *const late = reinterpret_cast<uint32_t *>(W.u.sim);
        constexpr uint32_t LATE_CAP = WT;
        if (tid == 0) W.v[9] = 0;
        __syncthreads();
        each_b<uint64_t>(nr, [&](uint32_t rr) { return ldc(&gs[rr]); }, [&](uint32_t, uint64_t s) {
            const uint32_t c = rf_pos((uint32_t)s);
            if ((uint32_t)(s >> 32) > dmx || !c || c < late_lo) return;
            const uint32_t x = atomicAdd(&W.v[9], 1u);
            if (x < LATE_CAP) late[x] = c;
        });
        __syncthreads();
        const uint32_t nlate = uni(W.v[9]);
        if (nlate > LATE_CAP) { O.why = 7; return O; }
        for (uint32_t x = tid; x < nlate; x += FILL_WG) {
            const uint32_t c = late[x];
            const uint32_t par = (c - 1u) / 2u, sib = ((c - 1u) ^ 1u) + 1u;
            if (member(par) || (sib < NN && member(sib))) {
                const uint32_t q = c + 1u, dq = depth_of(q);
                add_root(dq >= WHL ? (q >> WHL) - 1u : 0u);
            }
        }
        __syncthreads();
        LEAD_SUB(4);
        const uint32_t nroot = uni(W.v[8]);
        if (STG_CREW_STAMPS && tid == 0) I.dbg[5] = nroot;
        if (nroot > WROOTS) { O.why = 5; return O; }
        if (nroot) {
            const uint32_t Dm = depth_of(NN);  // depth of the last position N - 1
            // maximal roots only (drop one with an ancestor, or an equal one before it, in the list)
            bool keep = false;
            uint32_t my = 0;
            if (tid < nroot) {
                my = W.roots[tid];
                keep = true;
                for (uint32_t x = 0; x < nroot; ++x) {
                    const uint32_t o = W.roots[x];
                    if (x == tid) continue;
                    if (o == my ? x < tid : is_desc(my + 1u, o + 1u)) keep = false;
                }
            }
            const bool too_high = keep && Dm - depth_of(my + 1u) > WHMAX;
            if (__syncthreads_or((int)too_high)) { O.why = 6; return O; }
            if (tid == 0) W.v[10] = 0;
            __syncthreads();
            if (keep) W.roots[WROOTS - 1u - atomicAdd(&W.v[10], 1u)] = my;  // kept roots at the end
            __syncthreads();
            const uint32_t nk = uni(W.v[10]);
            // positions: starts, then replays
            each_b<u4v>(nq, [&](uint32_t q) { return ld4(rc, q); }, [&](uint32_t q, u4v x) {
                const uint32_t i = 4u * q;
                gp[i] = x.x;
                if (i + 1u < n) gp[i + 1u] = x.y;
                if (i + 2u < n) gp[i + 2u] = x.z;
                if (i + 3u < n) gp[i + 3u] = x.w;
            });
            if (tail && tid == 0) gp[n] = NN - 1u;
            vm_drain();
            __syncthreads();
            uint32_t late_bad = 0;
            for (uint32_t ri = 0; ri < nk; ++ri) {
                const uint32_t a = W.roots[WROOTS - 1u - ri], qa = a + 1u, d0 = depth_of(qa), h = Dm - d0;
                const uint32_t nn = (2u << h) - 1u;
                uint2 *const sim = W.u.sim;
                for (uint32_t l = tid; l < nn; l += FILL_WG) sim[l] = make_uint2(0u, NONE);
                if (tid <= h) {  // the list entries at each depth of the subtree
                    const uint32_t lo = (qa << tid) - 1u, hi = min(lo + (1u << tid), NN);
                    const uint32_t f = lo < NN ? lower(lo).x : m, e = lo < NN ? lower(hi).x : m;
                    W.lvl[tid] = f;
                    W.lvl[WHMAX + 2u + tid] = e - f;
                }
                __syncthreads();
                if (tid == 0) {  // per-level prefix over the counts
                    uint32_t acc = 0;
                    for (uint32_t t = 0; t <= h; ++t) { const uint32_t c = W.lvl[WHMAX + 2u + t]; W.lvl[WHMAX + 2u + t] = acc; acc += c; }
                    W.v[11] = acc;
                }
                __syncthreads();
                const uint32_t tot = uni(W.v[11]);
                auto entry = [&](uint32_t f, uint32_t &t) {
                    t = 0;
                    while (t < h && W.lvl[WHMAX + 3u + t] <= f) ++t;
                    return W.lvl[t] + (f - W.lvl[WHMAX + 2u + t]);
                };
                each_b<uint2>(tot, [&](uint32_t f) { uint32_t t; const uint32_t i = entry(f, t); return make_uint2(kb(i), cx(i)); },
                              [&](uint32_t f, uint2 x) {
                                  uint32_t t;
                                  const uint32_t i = entry(f, t), k = okey(x.x);
                                  if (k >= ksm) sim[(1u << t) - 1u + (x.y + 1u - (qa << t))] = make_uint2(k, i);
                              });
                __syncthreads();
                // make_heap on the subtree: every node p <= (N - 2) / 2, deepest first,
                // libstdc++'s __adjust_heap / __push_heap with len = N (non-R_smin: -inf = 0)
                for (int t = (int)h - 1; t >= 0; --t) {
                    const uint32_t l0 = (1u << t) - 1u, w = 1u << t;
                    for (uint32_t o = tid; o < w; o += FILL_WG) {
                        const uint32_t top = (qa << t) - 1u + o;
                        if (NN < 2u || top > (NN - 2u) / 2u) continue;
                        const uint2 value = sim[l0 + o];
                        uint32_t hp = top, hl = l0 + o, sc = top;
                        while (sc < (NN - 1u) / 2u) {
                            sc = 2u * (sc + 1u);
                            uint32_t cl = 2u * hl + 2u;
                            if (sim[cl].x < sim[cl - 1u].x) { --sc; --cl; }
                            sim[hl] = sim[cl];
                            hp = sc;
                            hl = cl;
                        }
                        if ((NN & 1u) == 0 && sc == (NN - 2u) / 2u) {
                            sc = 2u * (sc + 1u);
                            sim[hl] = sim[2u * hl + 1u];
                            hp = sc - 1u;
                            hl = 2u * hl + 1u;
                        }
                        while (hp > top && sim[(hl - 1u) / 2u].x < value.x) {
                            sim[hl] = sim[(hl - 1u) / 2u];
                            hp = (hp - 1u) / 2u;
                            hl = (hl - 1u) / 2u;
                        }
                        sim[hl] = value;
                    }
                    __syncthreads();
                }
                for (uint32_t l = tid; l < nn; l += FILL_WG) {
                    const uint2 x = sim[l];
                    if (x.y == NONE) continue;
                    const uint32_t t = depth_of(l + 1u), p = (qa << t) - 1u + (l - ((1u << t) - 1u));
                    gp[x.y] = p;
                    if (p >= late_lo) late_bad = 1;  // an R_smin line stays where pop_heap re-inserts
                }
                vm_drain();
                __syncthreads();
            }
            if (__syncthreads_or((int)late_bad)) { O.why = 7; return O; }
            LEAD_SUB(5);
            // re-order every run by the replayed positions (rf32), one LDS tile
            // of whole runs at a time
            uint32_t *const dd = reinterpret_cast<uint32_t *>(W.u.s.tk), *const rfk = dd + WT, *const oo = W.u.s.ti;
            for (uint32_t s0 = 0; s0 < nr;) {
                const uint32_t nt = min(WT, nr - s0), ext = s0 + nt < nr ? 1u : 0u;
                each_b<uint2>(nt, [&](uint32_t j) { return make_uint2(ldc(&go[s0 + j]), ldc(&gs32[2u * (s0 + j) + 1u])); },
                              [&](uint32_t j, uint2 x) { oo[j] = x.x; dd[j] = x.y; });
                if (tid == 0) W.v[11] = ext ? ldc(&gs32[2u * (s0 + nt) + 1u]) : NONE;
                __syncthreads();
                each_b<uint32_t>(nt, [&](uint32_t j) { return ldc(&gp[oo[j] & LNONE]); },
                                 [&](uint32_t j, uint32_t p) { rfk[j] = rf32(p); });
                if (tid == 0) {  // the tile ends where a run ends
                    uint32_t c = nt;
                    if (ext) while (c > 0 && dd[c - 1u] == W.v[11]) --c;
                    W.v[12] = c;
                }
                __syncthreads();
                const uint32_t cut = uni(W.v[12]);
                uint32_t big = cut == 0 ? 1u : 0u;
                for (uint32_t j = tid; j < cut; j += FILL_WG) {
                    const uint32_t o = oo[j];
                    if (!(o >> 31)) continue;
                    const uint32_t dj = dd[j], kj = rfk[j];
                    uint32_t g0 = j, g1 = j + 1u;
                    while (g0 > 0 && j - g0 < WRUN && dd[g0 - 1u] == dj) --g0;
                    while (g1 < cut && g1 - j < WRUN && dd[g1] == dj) ++g1;
                    if (g1 - g0 >= WRUN) { big = 1; continue; }
                    uint32_t rk = g0;
                    for (uint32_t x = g0; x < g1; ++x) rk += rfk[x] < kj;
                    go[s0 + rk] = o;
                }
                vm_drain();
                if (__syncthreads_or((int)big)) { O.why = 8; return O; }
                s0 += cut;
            }
        }
    }

    // ---- 4. the pops: P and the ragged tail's rank; the order's positions ----
    LEAD_STAMP(3);
    if (tid == 0) W.v[12] = NONE;
    __syncthreads();
    if (tail)
        each_b<uint32_t>(nr, [&](uint32_t rr) { return ldc(&go[rr]); }, [&](uint32_t rr, uint32_t o) {
            if ((o & LNONE) == n) W.v[12] = rr;
        });
    __syncthreads();
    const uint32_t tr = uni(W.v[12]);
    uint32_t P = P0;
    if (tr < P0) P = (uni(I.rem) + (16u - uni(I.tl)) + 15u) / 16u;
    if (P > nr) { O.why = 4; return O; }
    // go was stored plain: the order for other workgroups (the crew's
    // emission units) is written through here, sc1 and coalesced
    for (uint32_t i0 = 0; i0 < P; i0 += WB * FILL_WG) {
        uint32_t x[WB];
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) x[b] = ldc(&go[min(i0 + b * FILL_WG + tid, P - 1u)]);
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b)
            if (i0 + b * FILL_WG + tid < P) st_sc1(&go[i0 + b * FILL_WG + tid], x[b]);
    }
    if (I.positions) {
        each_b2<uint32_t, uint32_t>(P, [&](uint32_t i) { return ldc(&go[i]) & LNONE; }, [&](uint32_t, uint32_t e) { return ps(e); },
                                    [&](uint32_t i, uint32_t, uint32_t p) { st_sc1(&op[i], p); });
        vm_drain();
        __syncthreads();
    }
    vm_drain();
    __syncthreads();
    LEAD_STAMP(4);
    O.P = P;
    O.tail_rank = tr;
    O.ordpos = op;
    O.order = go;
    O.ok = true;
    return O;
}

// ---------------------------------------------------------------------------
// the crew
// ---------------------------------------------------------------------------
// regime B with lines (or the tail) to fill, and the window does not hold them
__device__ __forceinline__ bool crew_wants(uint32_t flags, uint32_t M, uint32_t mode) {
    return (flags & TV16_DEC_B) && (M || (flags & TV16_DEC_TAIL)) && (!(flags & TV16_DEC_WIN) || mode == 4u) &&
           mode != 2u;  // mode 2 (tests): the literal heap for every regime-B bucket
}

// scratch layout of a crew bucket (words of d.heap: 2 (nb + 64) of them)
struct CrewMap {
    uint32_t *keys, *lk, *lp, *lc;
    uint64_t *cdesc;
    uint32_t kwords, lcap;
};
// (values read from LDS are moved to SGPRs: a buffer descriptor built from
// VGPRs would make every load a waterfall loop)
__device__ __forceinline__ CrewMap crew_map(const CrewBk &B) {
    CrewMap c;
    uint32_t *const g = uni_ptr(reinterpret_cast<uint32_t *>(B.d.heap));
    const uint32_t nb = uni(B.d.nb), nC = uni(B.nC);
    const uint32_t total = 2u * (nb + 64u);
    c.kwords = (nb + 16u + 3u) & ~3u;
    c.keys = g;
    const uint32_t co = c.kwords;
    c.cdesc = reinterpret_cast<uint64_t *>(g + co);
    const uint32_t lo = (co + 2u * nC + 3u) & ~3u;
    c.lcap = total > lo ? (total - lo) / 3u : 0u;
    c.lk = g + lo;
    c.lp = c.lk + c.lcap;
    c.lc = c.lp + c.lcap;
    return c;
}

// A: one unit of la lines.
template <uint32_t DA, class WL>
__device__ __noinline__ void crew_a(WL &W, const CrewBk &B, CrewCtl *ctl, uint32_t u) {
    u = uni(u);  // (a callee's arguments arrive in VGPRs)
    ctl = uni_ptr(ctl);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uni(tid >> 6), q = lane & 3u;
    const CrewMap cm = crew_map(B);
    uint32_t *const hist = W.u.hist8;
    for (uint32_t b = tid; b < WBINS; b += FILL_WG) hist[b] = 0;
    __syncthreads();
    const uint32_t nb = uni(B.d.nb);
    const uint32_t la = uni(B.la), L0 = u * la, nl = nb > L0 ? min(la, nb - L0) : 0u;
    const float *const src = uni_ptr(B.d.src);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src + (size_t)L0 * 16), 0, nl * 64u, 0x00020000);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(cm.keys, 0, cm.kwords * 4u, 0x00020000);
    const float t = u2f(uni(B.tbits));
    const uint32_t steps = (nl + 15u) / 16u;
    const uint32_t mine = steps > wave ? (steps - wave + FNW_F - 1u) / FNW_F : 0u;
    auto load = [&](uint32_t mm) -> float4 {
        uint32_t voff = ((wave + mm * FNW_F) * 16u + (lane >> 2)) * 64u + q * 16u;
        asm volatile("" : "+v"(voff));
        const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 2 /* nt */);
        return make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w));
    };
    float4 v[DA];
#pragma unroll
    for (uint32_t j = 0; j < DA; ++j) v[j] = load(j);
    for (uint32_t m0 = 0; m0 < mine; m0 += DA) {
#pragma unroll
        for (uint32_t j = 0; j < DA; ++j) {
            const float4 x = v[j];
            v[j] = load(m0 + j + DA);
            if (m0 + j >= mine) continue;
            const uint32_t s = wave + (m0 + j) * FNW_F, line = s * 16u + (lane >> 2);
            const float S = quad_line_sum(x);
            const bool valid = line < nl;
            const bool qual = S >= t;
            const uint32_t k = qual ? 0u : okey(f2u(S));
            if (STG_CREW_STAMPS != 4 && valid && !qual && q == 0) atomicAdd(&hist[k >> WSH], 1u);
            // lane 16 j stores the keys of lines 4 j .. 4 j + 3 of the step (one 16-byte sc1 store)
            const uint32_t k1 = __shfl_down(k, 4, 64), k2 = __shfl_down(k, 8, 64), k3 = __shfl_down(k, 12, 64);
            if (STG_CREW_STAMPS != 3 && (lane & 15u) == 0 && valid) {
                u4v kv;
                kv.x = k; kv.y = k1; kv.z = k2; kv.w = k3;
                __builtin_amdgcn_raw_buffer_store_b128(kv, rk, (L0 + s * 16u + (lane >> 2)) * 4u, 0, 16 /* sc1 */);
            }
        }
    }
    if (u + 1u == uni(B.nA) && B.tail && tid == 0) atomicAdd(&hist[okey(B.tail_bits) >> WSH], 1u);
    __syncthreads();
    for (uint32_t b = tid; b < WBINS; b += FILL_WG) {
        const uint32_t c = hist[b];
        if (c) __hip_atomic_fetch_add(gp(&ctl->hist[b]), c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// C: the level-1 bin beta of the (sel + 1)-th largest candidate key (every
// unit picks it from the bucket's histogram), then the candidates of bins >=
// beta in keys [c * LC, ...), listed in scan order.
template <class WL>
__device__ __noinline__ bool crew_c(WL &W, const CrewBk &B, CrewCtl *ctl, uint32_t c, uint32_t epoch) {
    c = uni(c);
    epoch = uni(epoch);
    ctl = uni_ptr(ctl);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const CrewMap cm = crew_map(B);
    const uint32_t nb = uni(B.d.nb);
    const uint32_t K0 = c * CW_LC + 16u * tid;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(cm.keys, 0, nb * 4u, 0x00020000);
    u4v kv[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) kv[j] = __builtin_amdgcn_raw_buffer_load_b128(rk, (K0 + 4u * j) * 4u, 0, 16 /* sc1 */);
    {   // the histogram into LDS beside them (8,192 words: 32 chunks of 64 lanes x 16 bytes)
        const char *const src = reinterpret_cast<const char *>(ctl->hist);
        char *const dst = reinterpret_cast<char *>(W.u.hist8);
        for (uint32_t ch = wave; ch < WBINS / 256u; ch += FNW_F)
            __builtin_amdgcn_global_load_lds(src + (size_t)(ch * 64u + lane) * 16u, dst + ch * 1024u, 16, 0, 16 /* sc1 */);
    }
    vm_drain();
    __syncthreads();
    uint32_t beta, r1;
    {   // descending bins, 16 per thread
        const uint32_t P0 = (B.rem + 15u) / 16u, sel = min(P0 + 1u, B.N - 1u);
        constexpr uint32_t PER = WBINS / FILL_WG;
        uint32_t hc[PER], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            hc[j] = W.u.hist8[WBINS - 1u - (PER * tid + j)];
            s += hc[j];
        }
        if (tid == 0) { W.v[0] = 0; W.v[1] = 0; }
        uint32_t tot;
        uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            if (a <= sel && sel < a + hc[j]) { W.v[0] = WBINS - 1u - (PER * tid + j); W.v[1] = sel - a; }
            a += hc[j];
        }
        __syncthreads();
        beta = uni(W.v[0]);
        r1 = uni(W.v[1]);
    }
    if (c == 0 && tid == 0) {
        st_sc1(&ctl->beta, beta);
        st_sc1(&ctl->pad[0], r1);  // its rank inside the bin (the leader starts there)
    }
    auto key = [&](uint32_t j) -> uint32_t {
        const u4v x = kv[j >> 2];
        const uint32_t w = j & 3u;
        return w == 0 ? x.x : w == 1 ? x.y : w == 2 ? x.z : x.w;
    };
    uint32_t nl = 0, nq = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t k = key(j);
        const bool in = K0 + j < nb;
        nq += (in && k == 0) ? 1u : 0u;
        nl += (in && k && (k >> WSH) >= beta) ? 1u : 0u;
    }
    uint32_t NL, NQ;
    const uint32_t lo = blk_excl_scan<FNW_F>(nl, W.sh, &NL);
    const uint32_t qo = blk_excl_scan<FNW_F>(nq, W.sh, &NQ);
    // {tag | qualifying lines : 16 | listed : 16} of this unit
    if (tid == 0) st_sc1(&cm.cdesc[c], ((uint64_t)epoch << 32) | (NQ << 16) | NL);
    if (tid < 64) {  // earlier units' counts (tagged, look-back)
        uint32_t sl = 0, sq = 0, ok = 1;
        for (uint32_t i = lane; i < c; i += 64u) {
            uint64_t x = ld_sc1(&cm.cdesc[i]);
            uint64_t st = 0;
            for (uint32_t sp = 0; (uint32_t)(x >> 32) != epoch; ++sp) {
                __builtin_amdgcn_s_sleep(2);
                x = ld_sc1(&cm.cdesc[i]);
                if (spin_expired(sp, st)) { ok = 0; break; }
            }
            sl += (uint32_t)x & 0xffffu;
            sq += ((uint32_t)x >> 16) & 0xffffu;
        }
        sl = wave_sum(sl);
        sq = wave_sum(sq);
        ok = __ballot(!ok) ? 0u : 1u;
        if (lane == 0) { W.v[2] = sl; W.v[3] = sq; W.v[4] = ok; }
    }
    __syncthreads();
    if (!W.v[4]) return false;
    uint32_t off = W.v[2] + lo, qb = W.v[3] + qo, ovf = 0;
    // (buffer stores: a base in SGPRs and 32-bit offsets, sc1)
    const __amdgpu_buffer_rsrc_t rlk = __builtin_amdgcn_make_buffer_rsrc(cm.lk, 0, cm.lcap * 4u, 0x00020000);
    const __amdgpu_buffer_rsrc_t rlp = __builtin_amdgcn_make_buffer_rsrc(cm.lp, 0, cm.lcap * 4u, 0x00020000);
    const __amdgpu_buffer_rsrc_t rlc = __builtin_amdgcn_make_buffer_rsrc(cm.lc, 0, cm.lcap * 4u, 0x00020000);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t k = key(j), line = K0 + j;
        const bool in = line < nb;
        if (in && k == 0) ++qb;
        if (in && k && (k >> WSH) >= beta) {
            if (off < cm.lcap) {
                // sums are >= +0: the ordered key is bits | 2^31
                __builtin_amdgcn_raw_buffer_store_b32(k & 0x7fffffffu, rlk, off * 4u, 0, 16 /* sc1 */);
                __builtin_amdgcn_raw_buffer_store_b32(line * 16u, rlp, off * 4u, 0, 16 /* sc1 */);
                __builtin_amdgcn_raw_buffer_store_b32(line - qb, rlc, off * 4u, 0, 16 /* sc1 */);
            } else {
                ovf = 1;
            }
            ++off;
        }
    }
    if (__syncthreads_or((int)ovf) && tid == 0) st_sc1(&ctl->status, 1u);
    if (c + 1u == B.nC && tid == 0) st_sc1(&ctl->nL, W.v[2] + NL);
    return true;
}

// What the crew takes from the launch's arguments (by value: a reference to the
// kernel's argument block would make the compiler copy the block to scratch).
struct CrewArgs {
    CallCtl *cc;
    uint32_t *fail;
    uint32_t *dbg;
    CrewCtl *crew_ctl;
    uint32_t epoch;
};
__device__ __forceinline__ uint32_t phase_units(const CrewBk &B, uint32_t p) {
    return p == 1 ? B.nA : p == 2 ? B.nC : p == 4 ? CW_NE : 1u;
}

// LONE: a one-bucket fill launch (one workgroup per CU, the kernel's register
// budget is not shared with scans): phase A keeps twice the loads in flight
template <bool LONE, class WL>
__device__ __noinline__ void crew_loop(WL &W, FillLds &S, const CrewArgs A) {
    const uint32_t tid = threadIdx.x;
    CallCtl *const cc = A.cc;
    uint32_t *const ticket = &cc->crew_ticket[0], *const done = &cc->crew_done[0];  // zeroed for each call by the scan
    const uint32_t nreq = W.nreq;
    auto poison = [&]() {
        if (tid == 0) {
            g_or(A.fail, FAIL_SPIN_TIMEOUT);
            for (uint32_t j = 0; j < nreq; ++j) st_sc1(W.bk[j].d.count_out, POISON_COUNT);
        }
    };
    if (STG_CREW_STAMPS && tid == 0) atomicMax(&A.dbg[23], (uint32_t)__builtin_amdgcn_s_memrealtime());  // the last crew start
    for (;;) {
        if (tid == 0) W.v[15] = g_add(ticket, 1u);
        __syncthreads();
        const uint32_t tk = W.v[15];
        __syncthreads();
        if (tk >= W.tb[nreq]) return;
        if (STG_CREW_STAMPS && tk == 0 && tid == 0) A.dbg[22] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        uint32_t j = 0;
        while (tk >= W.tb[j + 1]) ++j;
        const CrewBk &B = W.bk[j];
        uint32_t rel = tk - W.tb[j], p = 0;
        while (rel >= phase_units(B, p)) { rel -= phase_units(B, p); ++p; }
        // the previous phase of this bucket, and this phase of the buckets before it
        if (p && !wide_wait(&done[p - 1], W.cp[p - 1][j] + phase_units(B, p - 1), &W.v[14])) { poison(); return; }
        if (j && !wide_wait(&done[p], W.cp[p][j], &W.v[14])) { poison(); return; }
        CrewCtl *const ctl = A.crew_ctl + B.slot;
        if (p == 0) {  // Z
            for (uint32_t i = tid; i < WBINS / 4u; i += FILL_WG)
                st_sc1_zero16(ctl->hist, WBINS * 4u, 16u * i);
            if (tid == 0) st_sc1(&ctl->status, 0u);
        } else if (p == 1) {  // A
            crew_a<LONE ? CW_DA_LONE : CW_DA>(W, B, ctl, rel);
        } else if (p == 2) {  // C
            if (!crew_c(W, B, ctl, rel, A.epoch)) { poison(); return; }
        } else if (p == 3) {  // D: the leader, or the literal heap (uniform: p from the ticket in LDS)
            const CrewMap cm = crew_map(B);
            const uint32_t nL = ld_sc1(&ctl->nL), ovf = ld_sc1(&ctl->status), beta = ld_sc1(&ctl->beta);
            LeadIn I;
            I.lk = cm.lk;
            I.lp = cm.lp;
            I.lc = cm.lc;
            I.n = nL;
            I.tail = B.tail && (okey(B.tail_bits) >> WSH) >= beta ? 1u : 0u;
            I.tail_bits = B.tail_bits;
            I.N = B.N;
            I.nb = B.d.nb;
            I.rem = B.rem;
            I.tl = B.d.tl;
            I.g = cm.keys;  // the keys are dead once the list is built
            I.gcap = cm.kwords;
            I.dbg = A.dbg;
            I.lvl1 = beta;
            I.r1 = ld_sc1(&ctl->pad[0]);
            I.positions = false;
            if (STG_CREW_STAMPS && tid == 0) A.dbg[29] = (uint32_t)__builtin_amdgcn_s_memrealtime();
            LeadOut O;
            O.ok = false;
            O.tail_rank = NONE;
            O.ordpos = cm.keys;
            O.order = cm.keys;
            if (STG_CREW_STAMPS >= 2 && !ovf) {  // diagnostics: a first run warms the caches (uniform: a final word)
                (void)leader(W, I);
                __syncthreads();
                if (tid == 0) A.dbg[29] = (uint32_t)__builtin_amdgcn_s_memrealtime();
            }
            if (!ovf) O = leader(W, I);
            const bool ok = O.ok;
            if (tid == 0) {
                atomicAdd(&A.dbg[53], 1u);
                if (!ok) atomicAdd(&A.dbg[55], 1u);
                st_sc1(&ctl->P, ok ? O.P : 0u);
                st_sc1(&ctl->tail_rank, O.tail_rank);
                st_sc1(&ctl->op, ok ? (uint32_t)(O.order - cm.keys) : 0u);
            }
            if (!ok) {  // exact, slow; its LDS view covers this workgroup's plan, so it takes no more units (uniform: the leader's result)
                const CrewBk Bl = B;
                __syncthreads();
                full_path(S, Bl.d, Bl.cnt, Bl.N, u2f(Bl.tbits), Bl.tail != 0, u2f(Bl.tail_bits), A.fail);
                vm_drain();
                __syncthreads();
                if (tid == 0) g_add(&done[p], 1u);
                return;
            }
        } else {  // E: emission share `rel`: the pops' list entries -> element positions (LDS), then the lines
            const uint32_t P = ld_sc1(&ctl->P), tr = ld_sc1(&ctl->tail_rank), nL = ld_sc1(&ctl->nL);
            const CrewMap cm = crew_map(B);
            const uint32_t *const go = cm.keys + ld_sc1(&ctl->op);
            const uint32_t *const lp = cm.lp;
            const uint32_t tpos = uni(B.d.nb) * 16u, nl1 = nL ? nL - 1u : 0u;
            const uint32_t per = (P + CW_NE - 1u) / CW_NE;
            uint32_t *const posl = W.u.hist8;  // WBINS words
            for (uint32_t i0 = rel * per, i1 = min(P, (rel + 1u) * per); i0 < i1; i0 += WBINS) {
                const uint32_t ie = min(i1, i0 + WBINS);
                each_b2<uint32_t, uint32_t>(ie - i0, [&](uint32_t j) { return ld_sc1(&go[i0 + j]) & LNONE; },
                                            [&](uint32_t, uint32_t e) { const uint32_t x = ld_sc1(&lp[min(e, nl1)]); return e < nL ? x : tpos; },
                                            [&](uint32_t j, uint32_t, uint32_t p) { posl[j] = p; });
                __syncthreads();
                emit_order(B.d, B.cnt, B.rem, P, tr, [&](uint32_t i) { return posl[i - i0]; }, i0, ie);
                __syncthreads();
            }
        }
        vm_drain();
        __syncthreads();
        if (tid == 0) g_add(&done[p], 1u);
        if (STG_CREW_STAMPS && tid == 0) atomicMax(&A.dbg[16 + p], (uint32_t)__builtin_amdgcn_s_memrealtime());
    }
}

// Units and tickets of the requested buckets (W.bk[0 .. nreq) filled).
// A's units: the bucket's lines over the crew (at least CW_LA lines each).
template <class WL>
__device__ __forceinline__ void crew_plan(WL &W, uint32_t ncrew) {
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t j = 0; j < W.nreq; ++j) {
            CrewBk &B = W.bk[j];
            B.la = max(CW_LA, ((B.d.nb + ncrew - 1u) / max(ncrew, 1u) + 255u) & ~255u);
            B.nA = max(1u, (B.d.nb + B.la - 1u) / B.la);
            B.nC = max(1u, (B.d.nb + CW_LC - 1u) / CW_LC);
            W.tb[j] = t;
            for (uint32_t p = 0; p < CW_PH; ++p) {
                W.cp[p][j] = j ? W.cp[p][j - 1] + phase_units(W.bk[j - 1], p) : 0u;
                t += phase_units(B, p);
            }
        }
        W.tb[W.nreq] = t;
    }
    __syncthreads();
}

// A crew workgroup of a batched launch (or a lone one with helpers): the
// launch's window-miss buckets, from the scan's decisions (final: the scan
// launch has ended).
template <bool LONE>
__device__ __forceinline__ void crew_from_decisions(WideLds &W, FillLds &S, const Tv16FillArgs &A) {
    if (threadIdx.x == 0) {
        uint32_t nr = 0;
        const uint32_t failed = ld_sc1(A.fail);
        for (uint32_t b = 0; b < A.nbk && !failed; ++b) {
            const Decision &Dc = A.dec[b];
            const uint64_t w0 = ld_sc1(&Dc.w[0]);
            if ((uint32_t)(w0 >> 32) != ((A.epoch << 8) | TV16_TAG_DEC)) continue;
            const uint64_t w1 = ld_sc1(&Dc.w[1]), w2 = ld_sc1(&Dc.w[2]), w3 = ld_sc1(&Dc.w[3]);
            const uint32_t flags = (uint32_t)w0;
            if (!crew_wants(flags, (uint32_t)w1, A.mode)) continue;
            CrewBk &B = W.bk[nr++];
            B.d = A.bk[b];
            B.slot = b;
            B.cnt = (uint32_t)(w1 >> 32);
            B.rem = B.d.dst_len - B.cnt;
            B.tail = (flags & TV16_DEC_TAIL) ? 1u : 0u;
            B.N = B.d.nb - (uint32_t)(w3 >> 32) + B.tail;
            B.tbits = (uint32_t)w3;
            B.tail_bits = (uint32_t)w2;
        }
        W.nreq = nr;
    }
    __syncthreads();
    if (!W.nreq) return;
    crew_plan(W, A.crew);
    crew_loop<LONE>(W, S, CrewArgs{A.cc, A.fail, A.dbg, A.crew_ctl, A.epoch});
}

// A crew workgroup of a one-bucket (lfin) launch: the decision every lfin role
// takes (tv16lfin.h lfin_prefix).
__device__ __forceinline__ void crew_lfin(LfinLds &Lf, const Tv16FillArgs &A) {
    LfinDec D;
    lfin_prefix(Lf, Lf.args, D);
    const uint32_t flags =
        D.regimeB ? (TV16_DEC_B | (D.tail_cand ? TV16_DEC_TAIL : 0u) | (D.listw ? TV16_DEC_WIN : 0u)) : 0u;
    const bool want = crew_wants(flags, D.M, A.mode) && !ld_sc1(A.fail);
    __syncthreads();  // every read of the lfin view is done
    WideLdsBig &W = *reinterpret_cast<WideLdsBig *>(&Lf);
    if (threadIdx.x == 0) {
        W.nreq = want ? 1u : 0u;
        if (want) {
            CrewBk &B = W.bk[0];
            B.d = A.bk[0];
            B.slot = 0;
            B.cnt = D.cnt;
            B.rem = B.d.dst_len - D.cnt;
            B.N = D.N;
            B.tbits = f2u(D.t);
            B.tail = D.tail_cand ? 1u : 0u;
            B.tail_bits = f2u(D.tail_key);
        }
    }
    __syncthreads();
    if (!W.nreq) return;
    crew_plan(W, A.crew);
    crew_loop<true>(W, *reinterpret_cast<FillLds *>(&Lf), CrewArgs{A.cc, A.fail, A.dbg, A.crew_ctl, A.epoch});
}
