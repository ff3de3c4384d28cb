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
//   A  stream 4,096 lines: line sums in the scan's AVX tree order, the ordered
//      key of each line (0 for a qualifying line) into the scratch, the
//      candidates' histogram of the key's top 13 bits, qualifying count  (nb / 4096)
//   B  pick the bin holding the (min(P0 + 1, N - 1) + 1)-th largest key  (1 unit)
//   C  list every candidate in that bin or above, in scan order, with its
//      candidate index (look-back over the units' tagged counts)          (nb / 16384)
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
constexpr uint32_t CW_LA = 4096;  // crew phase A: lines per unit (256 KiB)
constexpr uint32_t CW_LC = 16384; // crew phase C: keys per unit (32 per thread)
constexpr uint32_t CW_NE = 32;    // crew phase E: emission units
constexpr uint32_t CW_DA = 6;     // crew phase A: float4 loads in flight per lane
constexpr uint32_t CW_PH = 6;     // phases Z A B C D E
constexpr uint32_t LNONE = 0x7fffffffu;
#ifndef STG_CREW_STAMPS
#define STG_CREW_STAMPS 0  // diagnostics: crew phase completion times (100 MHz clock), debug words 16..22
#endif
static_assert(CW_LC == 32 * FILL_WG && CW_LC % CW_LA == 0, "phase C: 32 keys per thread, whole A units");

// A window-miss bucket as the crew sees it.
struct CrewBk {
    Tv16FillBucket d;
    uint32_t slot, cnt, rem, N, tbits, tail, tail_bits;
    uint32_t nA, nC;
};

// LDS of the leader and the crew (a view of the fill launch's dynamic LDS).
struct WideLds {
    union {
        struct {
            uint32_t hist[WBINS];  // bins (select, sort, crew phase A)
            uint64_t tk[WTILE];    // ranking tile: composite keys
            uint32_t ti[WTILE];    // ... their list entries
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
static_assert(sizeof(WideLds) <= sizeof(FillLds), "the wide views fit the fill's LDS");

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
};
struct LeadOut {
    bool ok;
    uint32_t P, tail_rank;
    const uint32_t *ordpos;  // element position of each pop
    uint32_t why;            // failure: 1 NaN, 2 scratch, 3 crowded bin, 4 short list, 5 roots, 6 height, 7 late, 8 run
};

// Bounded poll by thread 0 until *w >= target; every thread gets the verdict.
__device__ __forceinline__ bool wide_wait(uint32_t *w, uint32_t target, uint32_t *flag) {
    if (threadIdx.x == 0) {
        uint32_t ok = 1;
        uint64_t st = 0;
        for (uint32_t sp = 0; ld_sc1(w) < target; ++sp) {
            __builtin_amdgcn_s_sleep(4);
            if (spin_expired(sp, st)) { ok = 0; break; }
        }
        *flag = ok;
    }
    __syncthreads();
    const bool r = *flag != 0;
    __syncthreads();
    return r;
}

// Batched loops: each thread loads WB entries (all in flight), then uses them
// -- a loop whose every iteration waits for its own load runs at one L2 round
// trip per iteration.
constexpr uint32_t WB = 8;
template <typename V, typename Ld, typename Use>
__device__ __forceinline__ void each_b(uint32_t n, Ld ld, Use use) {
    for (uint32_t i0 = 0; i0 < n; i0 += WB * FILL_WG) {
        V v[WB];
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) {
            const uint32_t i = i0 + b * FILL_WG + threadIdx.x;
            if (i < n) v[b] = ld(i);
        }
#pragma unroll
        for (uint32_t b = 0; b < WB; ++b) {
            const uint32_t i = i0 + b * FILL_WG + threadIdx.x;
            if (i < n) use(i, v[b]);
        }
    }
}

// The leader: the pops of a regime-B fill over a candidate list that holds
// every candidate of the top min(P0 + 2, N) (P0 = ceil(rem / 16)); candidates
// not listed have smaller sums than every listed one of R.  One workgroup.
__device__ __noinline__ LeadOut leader(WideLds &W, const LeadIn I) {
    LeadOut O;
    O.ok = false;
    const uint32_t tid = threadIdx.x;
    const uint32_t m = I.n + I.tail;
    auto kb = [&](uint32_t i) -> uint32_t { return i < I.n ? ld_sc1(&I.lk[i]) : I.tail_bits; };
    auto cx = [&](uint32_t i) -> uint32_t { return i < I.n ? ld_sc1(&I.lc[i]) : I.N - 1u; };
    auto ps = [&](uint32_t i) -> uint32_t { return i < I.n ? ld_sc1(&I.lp[i]) : I.nb * 16u; };
    O.P = 0;
    O.tail_rank = NONE;
    O.why = 0;
    if (!m) { O.ok = true; return O; }
    if ((size_t)6 * m + 8 > I.gcap || I.N >= (1u << 28)) { O.why = 2; return O; }
    uint64_t *const gk = reinterpret_cast<uint64_t *>(I.g);
    uint32_t *const gi = I.g + 2 * (size_t)m, *const go = gi + m, *const gp = go + m, *const op = gp + m;
    const uint32_t P0 = (I.rem + 15u) / 16u;
    const uint32_t sel = min(P0 + 1u, m - 1u);
    uint32_t *const hist = W.u.s.hist;

    // ---- 1. the key at descending rank sel: three radix levels (11, 11, 10 bits) ----
    if (tid == 0) { W.v[0] = 0; W.v[1] = 0; }
    uint32_t pre = 0, pm = 0, r = sel;
    for (uint32_t pass = 0; pass < 3; ++pass) {
        const uint32_t sh = pass == 0 ? 21u : pass == 1 ? 10u : 0u, nbin = pass == 2 ? 1024u : 2048u;
        for (uint32_t b = tid; b < nbin; b += FILL_WG) hist[b] = 0;
        __syncthreads();
        uint32_t kmx = 0, nanf = 0;
        each_b<uint32_t>(m, kb, [&](uint32_t, uint32_t b) {
            const uint32_t k = okey(b);
            nanf |= nan_bits(b) ? 1u : 0u;
            kmx = max(kmx, k);
            if ((k & pm) == pre) atomicAdd(&hist[(k >> sh) & (nbin - 1u)], 1u);
        });
        if (pass == 0) {
            kmx = wave_max(kmx);
            if ((tid & 63u) == 0) atomicMax(&W.v[1], kmx);
            if (nanf) W.v[0] = 1;
        }
        __syncthreads();
        const uint32_t per = nbin / FILL_WG;  // 4 or 2 bins per thread, highest first
        uint32_t c[4], s = 0;
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            c[u] = u < per ? hist[nbin - 1u - (per * tid + u)] : 0u;
            s += c[u];
        }
        uint32_t tot;
        uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            if (u < per && a <= r && r < a + c[u]) { W.v[2] = nbin - 1u - (per * tid + u); W.v[3] = r - a; }
            a += c[u];
        }
        __syncthreads();
        pre |= W.v[2] << sh;
        pm |= (nbin - 1u) << sh;
        r = W.v[3];
        __syncthreads();
    }
    if (W.v[0]) { O.why = 1; return O; }
    const uint32_t okS = pre, kmax = W.v[1];

    // ---- 2. R = {key >= okS} by (key desc, rf32(start) asc): counting sort
    //      into bins of the key's distance below the maximum, then ranks
    //      inside each bin, one LDS tile of whole bins at a time ----
    const uint32_t D = kmax - okS, shb = bitlen(D) > 13u ? bitlen(D) - 13u : 0u, nbin = (D >> shb) + 1u;
    for (uint32_t b = tid; b < nbin; b += FILL_WG) hist[b] = 0;
    if (tid == 0) { W.v[4] = 0; W.v[5] = 0; }
    __syncthreads();
    uint32_t nr = 0;
    each_b<uint32_t>(m, kb, [&](uint32_t, uint32_t b) {
        const uint32_t k = okey(b);
        if (k >= okS) { atomicAdd(&hist[(kmax - k) >> shb], 1u); ++nr; }
    });
    nr = wave_sum(nr);
    if ((tid & 63u) == 0) atomicAdd(&W.v[4], nr);
    __syncthreads();
    nr = W.v[4];
    {   // exclusive scan of the bins (16 per thread), and the largest bin
        uint32_t c[16], s = 0, mx = 0;
#pragma unroll
        for (uint32_t u = 0; u < 16; ++u) {
            const uint32_t b = 16u * tid + u;
            c[u] = b < nbin ? hist[b] : 0u;
            s += c[u];
            mx = max(mx, c[u]);
        }
        uint32_t tot;
        uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
        for (uint32_t u = 0; u < 16; ++u) {
            const uint32_t b = 16u * tid + u;
            if (b < nbin) hist[b] = a;
            a += c[u];
        }
        mx = wave_max(mx);
        if ((tid & 63u) == 0) atomicMax(&W.v[5], mx);
        __syncthreads();
    }
    if (W.v[5] > WTILE) { O.why = 3; return O; }
    each_b<uint2>(m, [&](uint32_t i) { return make_uint2(kb(i), cx(i)); }, [&](uint32_t i, uint2 x) {
        const uint32_t k = okey(x.x);
        if (k < okS) return;
        const uint32_t slot = atomicAdd(&hist[(kmax - k) >> shb], 1u);
        st_sc1(&gk[slot], ((uint64_t)(kmax - k) << 32) | rf32(x.y));
        st_sc1(&gi[slot], i);
    });
    vm_drain();
    __syncthreads();  // hist[b]: the end of bin b
    uint32_t tie_any = 0;
    for (uint32_t s0 = 0, b0 = 0; s0 < nr;) {
        if (tid == 0) {  // the last bin b1 - 1 with end <= s0 + WTILE
            uint32_t lo = b0 + 1u, hi = nbin;
            while (lo < hi) {
                const uint32_t md = (lo + hi + 1u) >> 1;
                if (hist[md - 1u] <= s0 + WTILE) lo = md; else hi = md - 1u;
            }
            W.v[6] = lo;
        }
        __syncthreads();
        const uint32_t b1 = W.v[6], s1 = hist[b1 - 1u], nt = s1 - s0;
        each_b<uint64_t>(nt, [&](uint32_t j) { return ld_sc1(&gk[s0 + j]); }, [&](uint32_t j, uint64_t x) { W.u.s.tk[j] = x; });
        each_b<uint32_t>(nt, [&](uint32_t j) { return ld_sc1(&gi[s0 + j]); }, [&](uint32_t j, uint32_t x) { W.u.s.ti[j] = x; });
        __syncthreads();
        for (uint32_t j = tid; j < nt; j += FILL_WG) {
            const uint64_t key = W.u.s.tk[j];
            const uint32_t b = (uint32_t)(key >> 32) >> shb;
            const uint32_t lo = (b ? hist[b - 1u] : 0u) - s0, hi = hist[b] - s0;
            uint32_t rk = s0 + lo;
            bool tie = false;
            for (uint32_t x = lo; x < hi; ++x) {
                const uint64_t kx = W.u.s.tk[x];
                rk += kx < key;
                tie |= x != j && (uint32_t)(kx >> 32) == (uint32_t)(key >> 32);
            }
            tie_any |= tie ? 1u : 0u;
            st_sc1(&go[rk], W.u.s.ti[j] | (tie ? 0x80000000u : 0u));
        }
        __syncthreads();
        s0 = s1;
        b0 = b1;
    }
    vm_drain();
    const bool ties = __syncthreads_or((int)tie_any);

    // ---- 3. runs of equal sums: start positions one above the other, or a
    //      late line of R_s with an R_s line beside it -> replay those subtrees ----
    const uint32_t late_lo = I.N > sel + 2u ? I.N - (sel + 2u) : 0u;
    if (ties) {
        uint32_t dmx = 0;  // the lowest tied key (largest distance below kmax)
        each_b<uint32_t>(nr, [&](uint32_t rr) { return ld_sc1(&go[rr]); }, [&](uint32_t, uint32_t o) {
            if (o >> 31) dmx = max(dmx, kmax - okey(kb(o & LNONE)));
        });
        dmx = wave_max(dmx);
        if (tid == 0) { W.v[7] = 0; W.v[8] = 0; }
        __syncthreads();
        if ((tid & 63u) == 0) atomicMax(&W.v[7], dmx);
        __syncthreads();
        const uint32_t ksm = kmax - W.v[7];  // R_smin = {key >= ksm}
        auto add_root = [&](uint32_t a) {
            const uint32_t x = atomicAdd(&W.v[8], 1u);
            if (x < WROOTS) W.roots[x] = a;
        };
        // (a) adjacent members of a run (rf32 order): the second below the first
        for (uint32_t rr = tid; rr + 1u < nr; rr += FILL_WG) {
            const uint32_t o = ld_sc1(&go[rr]), o2 = ld_sc1(&go[rr + 1u]);
            if (!(o >> 31) || !(o2 >> 31)) continue;
            const uint32_t e = o & LNONE, f = o2 & LNONE;
            if (okey(kb(e)) != okey(kb(f))) continue;
            const uint32_t ce = cx(e), cf = cx(f);
            if (is_desc(cf + 1u, ce + 1u)) add_root(ce);
        }
        // (b) late lines of R_smin (start >= late_lo) with an R_smin line at the parent or sibling
        auto lower = [&](uint32_t c) {  // first entry with candidate index >= c
            uint32_t lo = 0, hi = m;
            while (lo < hi) {
                const uint32_t md = (lo + hi) >> 1;
                if (cx(md) < c) lo = md + 1u; else hi = md;
            }
            return lo;
        };
        auto member = [&](uint32_t c) {
            const uint32_t i = lower(c);
            return i < m && cx(i) == c && okey(kb(i)) >= ksm;
        };
        if (tid == 0) W.v[9] = lower(late_lo);
        __syncthreads();
        for (uint32_t i = W.v[9] + tid; i < m; i += FILL_WG) {
            const uint32_t c = cx(i);
            if (!c || okey(kb(i)) < ksm) continue;
            const uint32_t par = (c - 1u) / 2u, sib = ((c - 1u) ^ 1u) + 1u;
            if (member(par) || (sib < I.N && member(sib))) {
                const uint32_t q = c + 1u, dq = depth_of(q);
                add_root(dq >= WHL ? (q >> WHL) - 1u : 0u);
            }
        }
        __syncthreads();
        const uint32_t nroot = W.v[8];
        if (nroot > WROOTS) { O.why = 5; return O; }
        if (nroot) {
            const uint32_t Dm = depth_of(I.N);  // depth of the last position N - 1
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
            const uint32_t nk = W.v[10];
            each_b<uint32_t>(m, cx, [&](uint32_t i, uint32_t c) { st_sc1(&gp[i], c); });  // positions: starts, then replays
            vm_drain();
            __syncthreads();
            uint32_t late_bad = 0;
            for (uint32_t ri = 0; ri < nk; ++ri) {
                const uint32_t a = W.roots[WROOTS - 1u - ri], qa = a + 1u, d0 = depth_of(qa), h = Dm - d0;
                const uint32_t nn = (2u << h) - 1u;
                uint2 *const sim = W.u.sim;
                for (uint32_t l = tid; l < nn; l += FILL_WG) sim[l] = make_uint2(0u, NONE);
                if (tid <= h) {  // the list entries at each depth of the subtree
                    const uint32_t lo = (qa << tid) - 1u, hi = min(lo + (1u << tid), I.N);
                    const uint32_t f = lo < I.N ? lower(lo) : m, e = lo < I.N ? lower(hi) : m;
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
                const uint32_t tot = W.v[11];
                for (uint32_t f = tid; f < tot; f += FILL_WG) {
                    uint32_t t = 0;
                    while (t < h && W.lvl[WHMAX + 3u + t] <= f) ++t;
                    const uint32_t i = W.lvl[t] + (f - W.lvl[WHMAX + 2u + t]);
                    const uint32_t k = okey(kb(i));
                    if (k >= ksm) sim[(1u << t) - 1u + (cx(i) + 1u - (qa << t))] = make_uint2(k, i);
                }
                __syncthreads();
                // make_heap on the subtree: every node p <= (N - 2) / 2, deepest first,
                // libstdc++'s __adjust_heap / __push_heap with len = N (non-R_smin: -inf = 0)
                for (int t = (int)h - 1; t >= 0; --t) {
                    const uint32_t l0 = (1u << t) - 1u, w = 1u << t;
                    for (uint32_t o = tid; o < w; o += FILL_WG) {
                        const uint32_t top = (qa << t) - 1u + o;
                        if (I.N < 2u || top > (I.N - 2u) / 2u) continue;
                        const uint2 value = sim[l0 + o];
                        uint32_t hp = top, hl = l0 + o, sc = top;
                        while (sc < (I.N - 1u) / 2u) {
                            sc = 2u * (sc + 1u);
                            uint32_t cl = 2u * hl + 2u;
                            if (sim[cl].x < sim[cl - 1u].x) { --sc; --cl; }
                            sim[hl] = sim[cl];
                            hp = sc;
                            hl = cl;
                        }
                        if ((I.N & 1u) == 0 && sc == (I.N - 2u) / 2u) {
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
                    st_sc1(&gp[x.y], p);
                    if (p >= late_lo) late_bad = 1;  // an R_smin line stays where pop_heap re-inserts
                }
                vm_drain();
                __syncthreads();
            }
            if (__syncthreads_or((int)late_bad)) { O.why = 7; return O; }
            // re-order every run by the replayed positions (rf32), through op
            uint32_t big = 0;
            for (uint32_t rr = tid; rr < nr; rr += FILL_WG) {
                const uint32_t o = ld_sc1(&go[rr]);
                if (!(o >> 31)) continue;
                const uint32_t e = o & LNONE, k = okey(kb(e)), ke = rf32(ld_sc1(&gp[e]));
                uint32_t g0 = rr, g1 = rr + 1u;
                while (g0 > 0 && rr - g0 < WRUN && okey(kb(ld_sc1(&go[g0 - 1u]) & LNONE)) == k) --g0;
                while (g1 < nr && g1 - rr < WRUN && okey(kb(ld_sc1(&go[g1]) & LNONE)) == k) ++g1;
                if (g1 - g0 >= WRUN) { big = 1; continue; }
                uint32_t rk = g0;
                for (uint32_t x = g0; x < g1; ++x) rk += rf32(ld_sc1(&gp[ld_sc1(&go[x]) & LNONE])) < ke;
                st_sc1(&op[rk], o);
            }
            vm_drain();
            if (__syncthreads_or((int)big)) { O.why = 8; return O; }
            for (uint32_t rr = tid; rr < nr; rr += FILL_WG) {
                const uint32_t o = ld_sc1(&go[rr]);
                if (o >> 31) st_sc1(&go[rr], ld_sc1(&op[rr]));
            }
            vm_drain();
            __syncthreads();
        }
    }

    // ---- 4. the pops: P and the ragged tail's rank; the order's positions ----
    if (tid == 0) W.v[12] = NONE;
    __syncthreads();
    if (I.tail)
        each_b<uint32_t>(nr, [&](uint32_t rr) { return ld_sc1(&go[rr]); }, [&](uint32_t rr, uint32_t o) {
            if ((o & LNONE) == I.n) W.v[12] = rr;
        });
    __syncthreads();
    const uint32_t tr = W.v[12];
    uint32_t P = P0;
    if (tr < P0) P = (I.rem + (16u - I.tl) + 15u) / 16u;
    if (P > nr) { O.why = 4; return O; }
    each_b<uint32_t>(P, [&](uint32_t i) { return ld_sc1(&go[i]) & LNONE; }, [&](uint32_t i, uint32_t o) {
        op[i] = o;  // the entries first (one round trip), their positions below
    });
    vm_drain();
    __syncthreads();
    each_b<uint32_t>(P, [&](uint32_t i) { return ps(op[i]); }, [&](uint32_t i, uint32_t x) { st_sc1(&op[i], x); });
    vm_drain();
    __syncthreads();
    O.P = P;
    O.tail_rank = tr;
    O.ordpos = op;
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
    uint32_t *keys, *qual, *lk, *lp, *lc;
    uint64_t *cdesc;
    uint32_t kwords, lcap;
};
// (values read from LDS are moved to SGPRs: a buffer descriptor built from
// VGPRs would make every load a waterfall loop)
__device__ __forceinline__ CrewMap crew_map(const CrewBk &B) {
    CrewMap c;
    uint32_t *const g = uni_ptr(reinterpret_cast<uint32_t *>(B.d.heap));
    const uint32_t nb = uni(B.d.nb), nA = uni(B.nA), nC = uni(B.nC);
    const uint32_t total = 2u * (nb + 64u);
    c.kwords = (nb + 16u + 3u) & ~3u;
    c.keys = g;
    c.qual = g + c.kwords;
    const uint32_t co = (c.kwords + nA + 1u) & ~1u;
    c.cdesc = reinterpret_cast<uint64_t *>(g + co);
    const uint32_t lo = co + 2u * nC;
    c.lcap = total > lo ? (total - lo) / 3u : 0u;
    c.lk = g + lo;
    c.lp = c.lk + c.lcap;
    c.lc = c.lp + c.lcap;
    return c;
}

// A: one unit of 4,096 lines.
__device__ __noinline__ void crew_a(WideLds &W, const CrewBk &B, CrewCtl *ctl, uint32_t u) {
    u = uni(u);  // (a callee's arguments arrive in VGPRs)
    ctl = uni_ptr(ctl);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uni(tid >> 6), q = lane & 3u;
    const CrewMap cm = crew_map(B);
    uint32_t *const hist = W.u.s.hist;
    for (uint32_t b = tid; b < WBINS; b += FILL_WG) hist[b] = 0;
    __syncthreads();
    const uint32_t nb = uni(B.d.nb);
    const uint32_t L0 = u * CW_LA, nl = nb > L0 ? min(CW_LA, nb - L0) : 0u;
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
    float4 v[CW_DA];
#pragma unroll
    for (uint32_t j = 0; j < CW_DA; ++j) v[j] = load(j);
    uint32_t nq = 0;
    for (uint32_t m0 = 0; m0 < mine; m0 += CW_DA) {
#pragma unroll
        for (uint32_t j = 0; j < CW_DA; ++j) {
            const float4 x = v[j];
            v[j] = load(m0 + j + CW_DA);
            if (m0 + j >= mine) continue;
            const uint32_t s = wave + (m0 + j) * FNW_F, line = s * 16u + (lane >> 2);
            const float S = quad_line_sum(x);
            const bool valid = line < nl;
            const bool qual = S >= t;
            const uint32_t k = qual ? 0u : okey(f2u(S));
            if (valid && !qual && q == 0) atomicAdd(&hist[k >> WSH], 1u);
            nq += (valid && qual && q == 0) ? 1u : 0u;
            // lane 16 j stores the keys of lines 4 j .. 4 j + 3 of the step (one 16-byte sc1 store)
            const uint32_t k1 = __shfl_down(k, 4, 64), k2 = __shfl_down(k, 8, 64), k3 = __shfl_down(k, 12, 64);
            if ((lane & 15u) == 0 && valid) {
                u4v kv;
                kv.x = k; kv.y = k1; kv.z = k2; kv.w = k3;
                __builtin_amdgcn_raw_buffer_store_b128(kv, rk, (L0 + s * 16u + (lane >> 2)) * 4u, 0, 16 /* sc1 */);
            }
        }
    }
    nq = wave_sum(nq);
    if (lane == 0) atomicAdd(&W.v[13], nq);  // zeroed by the caller
    if (u + 1u == uni(B.nA) && B.tail && tid == 0) atomicAdd(&hist[okey(B.tail_bits) >> WSH], 1u);
    __syncthreads();
    for (uint32_t b = tid; b < WBINS; b += FILL_WG) {
        const uint32_t c = hist[b];
        if (c) __hip_atomic_fetch_add(gp(&ctl->hist[b]), c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) st_sc1(&cm.qual[u], W.v[13]);
}

// B: the level-1 bin of the (sel + 1)-th largest candidate key.
__device__ __noinline__ void crew_b(WideLds &W, const CrewBk &B, CrewCtl *ctl) {
    ctl = uni_ptr(ctl);
    const uint32_t tid = threadIdx.x;
    const uint32_t P0 = (B.rem + 15u) / 16u, sel = min(P0 + 1u, B.N - 1u);
    constexpr uint32_t PER = WBINS / FILL_WG;
    uint32_t c[PER], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        c[j] = ld_sc1(&ctl->hist[WBINS - 1u - (PER * tid + j)]);
        s += c[j];
    }
    if (tid == 0) W.v[0] = 0;
    uint32_t tot;
    uint32_t a = blk_excl_scan<FNW_F>(s, W.sh, &tot);
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (a <= sel && sel < a + c[j]) W.v[0] = WBINS - 1u - (PER * tid + j);
        a += c[j];
    }
    __syncthreads();
    if (tid == 0) st_sc1(&ctl->beta, W.v[0]);
}

// C: list the candidates of bins >= beta in keys [c * LC, ...), in scan order.
__device__ __noinline__ bool crew_c(WideLds &W, const CrewBk &B, CrewCtl *ctl, uint32_t c, uint32_t epoch) {
    c = uni(c);
    epoch = uni(epoch);
    ctl = uni_ptr(ctl);
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const CrewMap cm = crew_map(B);
    const uint32_t beta = uni(ld_sc1(&ctl->beta)), nb = uni(B.d.nb);
    const uint32_t K0 = c * CW_LC + 32u * tid;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(cm.keys, 0, nb * 4u, 0x00020000);
    u4v kv[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) kv[j] = __builtin_amdgcn_raw_buffer_load_b128(rk, (K0 + 4u * j) * 4u, 0, 16 /* sc1 */);
    auto key = [&](uint32_t j) -> uint32_t {
        const u4v x = kv[j >> 2];
        const uint32_t w = j & 3u;
        return w == 0 ? x.x : w == 1 ? x.y : w == 2 ? x.z : x.w;
    };
    uint32_t nl = 0, nq = 0;
#pragma unroll
    for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t k = key(j);
        const bool in = K0 + j < nb;
        nq += (in && k == 0) ? 1u : 0u;
        nl += (in && k && (k >> WSH) >= beta) ? 1u : 0u;
    }
    uint32_t NL, NQ;
    const uint32_t lo = blk_excl_scan<FNW_F>(nl, W.sh, &NL);
    const uint32_t qo = blk_excl_scan<FNW_F>(nq, W.sh, &NQ);
    if (tid == 0) st_sc1(&cm.cdesc[c], ((uint64_t)epoch << 32) | NL);
    if (tid < 64) {  // earlier units' counts (tagged, look-back) and the A units' qualifying lines before this unit
        uint32_t sl = 0, sq = 0, ok = 1;
        for (uint32_t i = lane; i < c; i += 64u) {
            uint64_t x = ld_sc1(&cm.cdesc[i]);
            uint64_t st = 0;
            for (uint32_t sp = 0; (uint32_t)(x >> 32) != epoch; ++sp) {
                __builtin_amdgcn_s_sleep(2);
                x = ld_sc1(&cm.cdesc[i]);
                if (spin_expired(sp, st)) { ok = 0; break; }
            }
            sl += (uint32_t)x;
        }
        const uint32_t na = c * (CW_LC / CW_LA);
        for (uint32_t i = lane; i < na; i += 64u) sq += ld_sc1(&cm.qual[i]);
        sl = wave_sum(sl);
        sq = wave_sum(sq);
        ok = __ballot(!ok) ? 0u : 1u;
        if (lane == 0) { W.v[0] = sl; W.v[1] = sq; W.v[2] = ok; }
    }
    __syncthreads();
    if (!W.v[2]) return false;
    uint32_t off = W.v[0] + lo, qb = W.v[1] + qo, ovf = 0;
#pragma unroll
    for (uint32_t j = 0; j < 32; ++j) {
        const uint32_t k = key(j), line = K0 + j;
        const bool in = line < nb;
        if (in && k == 0) ++qb;
        if (in && k && (k >> WSH) >= beta) {
            if (off < cm.lcap) {
                st_sc1(&cm.lk[off], k & 0x7fffffffu);  // sums are >= +0: the ordered key is bits | 2^31
                st_sc1(&cm.lp[off], line * 16u);
                st_sc1(&cm.lc[off], line - qb);
            } else {
                ovf = 1;
            }
            ++off;
        }
    }
    if (__syncthreads_or((int)ovf) && tid == 0) st_sc1(&ctl->status, 1u);
    if (c + 1u == B.nC && tid == 0) st_sc1(&ctl->nL, W.v[0] + NL);
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
    return p == 1 ? B.nA : p == 3 ? B.nC : p == 5 ? CW_NE : 1u;
}

__device__ __noinline__ void crew_loop(WideLds &W, FillLds &S, const CrewArgs A) {
    const uint32_t tid = threadIdx.x;
    CallCtl *const cc = A.cc;
    uint32_t *const ticket = &cc->pad[6], *const done = &cc->pad[7];  // zeroed for each call by the scan
    const uint32_t nreq = W.nreq;
    auto poison = [&]() {
        if (tid == 0) {
            g_or(A.fail, FAIL_SPIN_TIMEOUT);
            for (uint32_t j = 0; j < nreq; ++j) st_sc1(W.bk[j].d.count_out, POISON_COUNT);
        }
    };
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
            if (tid == 0) W.v[13] = 0;
            __syncthreads();
            crew_a(W, B, ctl, rel);
        } else if (p == 2) {  // B
            crew_b(W, B, ctl);
        } else if (p == 3) {  // C
            if (!crew_c(W, B, ctl, rel, A.epoch)) { poison(); return; }
        } else if (p == 4) {  // D: the leader, or the literal heap
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
            LeadOut O;
            O.ok = false;
            O.tail_rank = NONE;
            O.ordpos = cm.keys;
            if (!ovf) O = leader(W, I);
            const bool ok = O.ok;
            if (tid == 0) {
                atomicAdd(&A.dbg[53], 1u);
                if (!ok) atomicAdd(&A.dbg[55], 1u);
                st_sc1(&ctl->P, ok ? O.P : 0u);
                st_sc1(&ctl->tail_rank, O.tail_rank);
                st_sc1(&ctl->op, ok ? (uint32_t)(O.ordpos - cm.keys) : 0u);
            }
            if (!ok) {  // exact, slow; its LDS view covers this workgroup's plan, so it takes no more units
                const CrewBk Bl = B;
                __syncthreads();
                full_path(S, Bl.d, Bl.cnt, Bl.N, u2f(Bl.tbits), Bl.tail != 0, u2f(Bl.tail_bits), A.fail);
                vm_drain();
                __syncthreads();
                if (tid == 0) g_add(&done[p], 1u);
                return;
            }
        } else {  // E: emission share `rel`
            const uint32_t P = ld_sc1(&ctl->P), tr = ld_sc1(&ctl->tail_rank);
            const uint32_t *const op = crew_map(B).keys + ld_sc1(&ctl->op);
            const uint32_t per = (P + CW_NE - 1u) / CW_NE;
            if (P && rel * per < P)
                emit_order(B.d, B.cnt, B.rem, P, tr, [&](uint32_t i) { return ld_sc1(&op[i]); }, rel * per, (rel + 1u) * per);
        }
        vm_drain();
        __syncthreads();
        if (tid == 0) g_add(&done[p], 1u);
        if (STG_CREW_STAMPS && tid == 0) atomicMax(&A.dbg[16 + p], (uint32_t)__builtin_amdgcn_s_memrealtime());
    }
}

// Units and tickets of the requested buckets (W.bk[0 .. nreq) filled).
__device__ __forceinline__ void crew_plan(WideLds &W) {
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t j = 0; j < W.nreq; ++j) {
            CrewBk &B = W.bk[j];
            B.nA = max(1u, (B.d.nb + CW_LA - 1u) / CW_LA);
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
    crew_plan(W);
    crew_loop(W, S, CrewArgs{A.cc, A.fail, A.dbg, A.crew_ctl, A.epoch});
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
    WideLds &W = *reinterpret_cast<WideLds *>(&Lf);
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
    crew_plan(W);
    crew_loop(W, *reinterpret_cast<FillLds *>(&Lf), CrewArgs{A.cc, A.fail, A.dbg, A.crew_ctl, A.epoch});
}
