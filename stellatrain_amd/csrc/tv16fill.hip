// tv16fill.hip -- thresholdv16's regime-B heap fill, in libstdc++ pop order.
//
// Reference: thresholdv16.cpp:261-293.  When the ordered scan leaves the
// output short (regime B), the reference builds
//     std::priority_queue<pair<float,uint32_t>, vector<...>, Compare> q(Compare(), cand)
// (Compare: lhs.first < rhs.first, i.e. the line sums only) over the vector
// of every non-qualifying line in scan order plus the ragged tail, and pops
// until the output is full.  Lines with equal sums -- which D1 gradients
// produce in most regime-B calls -- come out in the order GCC's make_heap /
// pop_heap leave them in, so the index *stream* (and, when the tie sits at
// the cut, the index *set*) depends on that order.  This launch reproduces it
// exactly, one workgroup per bucket, after the scan launch (tv16.hip) has
// decided the regime and listed the window just below the threshold.
//
// Fast path (the window holds the top M lines: every regime-B call of a
// steady AIMD run).  Call the window's lines plus a competing tail R; every
// other candidate has a smaller sum.  Two facts, both checked against
// libstdc++ by tests/test_gpu_codecs.py (and a CPU model in DESIGN.md):
//  (1) Shadow heap: make_heap / pop_heap move an element of R only by
//      comparisons with elements of R -- a candidate below R's smallest sum
//      only ever loses -- so running make_heap with every non-R candidate
//      replaced by -inf gives every R element its real final position.
//      Only the nodes whose subtree holds two or more R elements ("U") need
//      processing; an element alone in its subtree just rises to the subtree's
//      top.  |U| is a few thousand, processed level by level.
//  (2) Pops: while position len-1 never holds an R element (checked: every R
//      position after make_heap < N - P), pop_heap's reinserted value is -inf
//      for R, and the pop sequence of a heap is root, then the merge of its
//      subtrees' sequences with ties going to the right subtree -- i.e. R in
//      (sum desc, right-first pre-order of its make_heap position) order.
// Full path (otherwise: the window missed the top M, > 4096 entries, or a
// bucket of 2^20+ lines): the candidate vector is built in global memory and
// make_heap / pop_heap run literally (make_heap level-parallel: subtrees of
// one level are disjoint).  Slow (milliseconds at 64 MiB), exact, rare.
#include <algorithm>
#include <cstddef>

#include "tv16_dev.h"

namespace stg {

namespace {

using namespace tv16;

constexpr uint32_t FILL_WG = 1024;
constexpr uint32_t EMAX = CAND_CAP;            // R: window entries + the ragged tail
constexpr uint32_t VCAP = 6144;                // shadow-heap nodes held (more: full path)
constexpr uint32_t DMAX = 20;                  // depths 0..19: positions < 2^20 - 1
constexpr uint32_t POS_LIM = (1u << 20) - 1;   // fast path: N <= POS_LIM (20-bit paths)
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint16_t NONE16 = 0xffffu;
constexpr uint32_t NBIN = 2048;                // counting-sort bins

// A heap node as a DFS key: its path from the root left-aligned to depth 19
// (20 bits) << 5 | its depth.  Ascending keys = pre-order, left subtree first;
// ancestors come before their descendants.
__device__ __forceinline__ uint32_t depth_of(uint32_t q) { return 31u - __clz(q); }  // q = pos + 1 >= 1
__device__ __forceinline__ uint32_t dkey_of_pos(uint32_t pos) {
    const uint32_t q = pos + 1, d = depth_of(q);
    return ((q << (19u - d)) << 5) | d;
}
__device__ __forceinline__ uint32_t dk_depth(uint32_t k) { return k & 31u; }
__device__ __forceinline__ uint32_t dk_pos(uint32_t k) { return ((k >> 5) >> (19u - (k & 31u))) - 1u; }
__device__ __forceinline__ uint32_t dk_anc(uint32_t k, uint32_t d) {  // the ancestor at depth d <= depth(k)
    return (((k >> 5) >> (19u - d)) << (19u - d) << 5) | d;
}
__device__ __forceinline__ uint32_t dk_left(uint32_t k) { return (k & ~31u) | (dk_depth(k) + 1); }
__device__ __forceinline__ uint32_t dk_right(uint32_t k) {
    return (((k >> 5) | (1u << (18u - dk_depth(k)))) << 5) | (dk_depth(k) + 1);
}
__device__ __forceinline__ uint32_t dk_parent(uint32_t k) {
    const uint32_t d = dk_depth(k);
    return (((k >> 5) & ~(1u << (19u - d))) << 5) | (d - 1);
}
// depth of the lowest common ancestor of two nodes (DFS keys)
__device__ __forceinline__ int dk_lca(uint32_t a, uint32_t b) {
    const uint32_t m = min(dk_depth(a), dk_depth(b));
    const uint32_t x = ((a >> 5) ^ (b >> 5)) >> (19u - m);  // path bits down to depth m
    return x ? (int)m - (int)(32u - __clz(x)) : (int)m;
}

struct SortScratch {
    uint32_t bin[NBIN];  // counts -> starts
    uint32_t cur[NBIN];  // scatter cursors
    uint16_t tmp[VCAP];  // items grouped by bin
    uint16_t ord[VCAP];  // the sorted order
};

// LDS of a fill workgroup (< 124 KiB: it shares a CU with one scan workgroup).
struct FillLds {
    uint32_t key[EMAX];   // line-sum bits (the tail: its signed key's bits)
    uint32_t cix[EMAX];   // candidate index -> start node (DFS key) -> final position
    union {
        struct {                   // element DFS order, then shadow-heap node construction
            uint32_t vlist[VCAP];  // nodes (DFS keys), unsorted
            SortScratch s;         // element order, then node order
        } a;
        struct {                   // the shadow heap: nodes in DFS order
            uint16_t vc[VCAP];     // element at the node (NONE16: -inf)
            uint16_t vr[VCAP];     // right child's node index (NONE16: -inf)
            uint32_t vk[VCAP];     // the node's DFS key
            uint16_t ord_spare[VCAP];
            uint16_t ulist[VCAP];  // nodes with a child in the heap, by depth
        } h;
        SortScratch o;             // output order
    } r;
    uint32_t uoff[DMAX + 2];
    uint32_t sh[32];      // block-scan scratch
    uint32_t flag, nv, maxpos, npop;
};
static_assert(sizeof(FillLds) <= 120 * 1024, "a fill workgroup beside one scan workgroup per CU");
static_assert(offsetof(FillLds, r) + offsetof(decltype(FillLds::r), h.vk) >=
              offsetof(FillLds, r) + offsetof(decltype(FillLds::r), a.s.bin), "vk is written over the node sort's bins");

__device__ __forceinline__ float kf(const FillLds &S, uint32_t e) { return e == NONE ? -INFINITY : u2f(S.key[e]); }

// Counting sort of items 0..n-1 by (bin(i), full(i)) ascending into X.ord:
// bins of a few items each; inside a bin, an item's rank is the number of
// bin members with a smaller full key.
template <typename Bin, typename Full>
__device__ void counting_sort(SortScratch &X, uint32_t *sh, uint32_t n, Bin bin_of, Full full_of) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < NBIN; i += FILL_WG) X.bin[i] = 0;
    __syncthreads();
    for (uint32_t e = tid; e < n; e += FILL_WG) atomicAdd(&X.bin[bin_of(e)], 1u);
    __syncthreads();
    {  // exclusive scan of the bins, NBIN / FILL_WG per thread
        constexpr uint32_t PER = NBIN / FILL_WG;
        uint32_t c0 = X.bin[PER * tid], c1 = X.bin[PER * tid + 1];
        static_assert(PER == 2, "two bins per thread");
        uint32_t tot;
        const uint32_t run = blk_excl_scan<FILL_WG / 64>(c0 + c1, sh, &tot);
        X.bin[PER * tid] = X.cur[PER * tid] = run;
        X.bin[PER * tid + 1] = X.cur[PER * tid + 1] = run + c0;
    }
    __syncthreads();
    for (uint32_t e = tid; e < n; e += FILL_WG) X.tmp[atomicAdd(&X.cur[bin_of(e)], 1u)] = (uint16_t)e;
    __syncthreads();
    for (uint32_t e = tid; e < n; e += FILL_WG) {
        const uint32_t b = bin_of(e), lo = X.bin[b], hi = X.cur[b];
        const uint64_t k = full_of(e);
        uint32_t r = lo;
        for (uint32_t x = lo; x < hi; ++x) r += full_of(X.tmp[x]) < k;
        X.ord[r] = (uint16_t)e;
    }
    __syncthreads();
}

// index of DFS key k among the sorted node keys vk[0..nv), or NONE16
__device__ __forceinline__ uint32_t vfind(const FillLds &S, uint32_t nv, uint32_t k) {
    uint32_t lo = 0, hi = nv;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (S.r.h.vk[m] < k) lo = m + 1; else hi = m;
    }
    return lo < nv && S.r.h.vk[lo] == k ? lo : NONE16;
}
__device__ __forceinline__ uint32_t vleft(const FillLds &S, uint32_t nv, uint32_t v) {
    return v + 1 < nv && S.r.h.vk[v + 1] == dk_left(S.r.h.vk[v]) ? v + 1 : NONE16;
}
__device__ __forceinline__ uint32_t velem(const FillLds &S, uint32_t v) {
    if (v == NONE16) return NONE;
    const uint32_t e = S.r.h.vc[v];
    return e == NONE16 ? NONE : e;
}

// libstdc++ __adjust_heap (heap length N) at shadow-heap node v; the descent
// stops where both children are -inf (nothing below moves an element of R).
__device__ void shadow_sift(FillLds &S, uint32_t nv, uint32_t v, uint32_t N) {
    const uint32_t x = velem(S, v);
    uint32_t hole = v, hpos = dk_pos(S.r.h.vk[v]);
    bool entered = false;
    const uint32_t half = (N - 1) / 2;
    while (hpos < half) {  // while (secondChild < (len - 1) / 2), secondChild == the hole
        const uint32_t r = S.r.h.vr[hole], l = vleft(S, nv, hole);
        uint32_t er = velem(S, r == NONE16 ? NONE16 : r);
        const uint32_t el = velem(S, l);
        uint32_t c = r, cpos = 2 * (hpos + 1);
        if (kf(S, er) < kf(S, el)) { c = l; er = el; --cpos; }
        if (er == NONE) { entered = true; break; }
        S.r.h.vc[hole] = (uint16_t)er;
        hole = c;
        hpos = cpos;
    }
    if (!entered && (N & 1u) == 0 && hpos == (N - 2) / 2) {
        const uint32_t l = vleft(S, nv, hole);
        const uint32_t el = velem(S, l);
        if (el != NONE) { S.r.h.vc[hole] = (uint16_t)el; hole = l; }
    }
    if (x == NONE) {  // -inf value: it stays below; the hole's stale copy goes
        if (hole != v) S.r.h.vc[hole] = NONE16;
        return;
    }
    const float xk = kf(S, x);
    while (hole != v) {  // __push_heap up to the top index v
        const uint32_t par = vfind(S, nv, dk_parent(S.r.h.vk[hole]));
        const uint32_t ep = velem(S, par);
        if (!(kf(S, ep) < xk)) break;
        S.r.h.vc[hole] = (uint16_t)ep;
        hole = par;
    }
    S.r.h.vc[hole] = (uint16_t)x;
}

// right-first pre-order key of heap position pos (< 2^20 - 1): ancestors
// first, then the right subtree before the left one
__device__ __forceinline__ uint32_t rf_key(uint32_t pos) {
    const uint32_t q = pos + 1, d = depth_of(q);
    const uint32_t path = q - (1u << d);
    const uint32_t inv = ~path & ((1u << d) - 1u);
    return ((inv << (19u - d)) << 5) | d;
}

// Emit the lines / tail of the output order: element i of the order goes to
// offset cnt + 16 i (less 16 - tl after the tail), at most rem elements.  Four
// lanes per line (a float4 each), 256 lines per round, loads of four rounds
// issued before their stores.
struct EmitEnt {
    float4 x;
    uint32_t pos, off, len;
    bool v4;
};

template <typename GetPos>
__device__ __forceinline__ void emit_load(const Tv16FillBucket &d, uint32_t i, uint32_t np, uint32_t rem,
                                          uint32_t tail_rank, bool vec, GetPos &pos_of, EmitEnt &E) {
    const uint32_t q = threadIdx.x & 3u;
    E.len = 0;
    if (i >= np) return;
    const bool is_tail = i == tail_rank;
    E.off = 16u * i - (tail_rank < i ? 16u - d.tl : 0u);
    if (E.off >= rem) return;
    E.len = min(is_tail ? d.tl : 16u, rem - E.off);
    E.pos = pos_of(i);
    E.v4 = vec && E.len == 16 && (E.off & 3u) == 0;
    if (E.v4) E.x = *reinterpret_cast<const float4 *>(d.src + (size_t)E.pos + 4 * q);
}

__device__ __forceinline__ void emit_store(const Tv16FillBucket &d, uint32_t cnt, const EmitEnt &E) {
    const uint32_t q = threadIdx.x & 3u;
    if (!E.len) return;
    const uint32_t o = cnt + E.off + 4 * q, bi = E.pos + 4 * q + (uint32_t)d.idx_offset;
    if (E.v4) {
        *reinterpret_cast<float4 *>(d.val + o) = E.x;
        *reinterpret_cast<uint4 *>(d.idx + o) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
        return;
    }
    for (uint32_t c = 0; c < 4; ++c) {
        if (4 * q + c < E.len) {
            d.val[o + c] = d.src[(size_t)E.pos + 4 * q + c];
            d.idx[o + c] = bi + c;
        }
    }
}

// Emit the lines / tail of the output order: element i of the order goes to
// offset cnt + 16 i (less 16 - tl after the tail), at most rem elements.  Four
// lanes per line (a float4 each), 256 lines per round, the loads of four
// rounds issued before their stores.
template <typename GetPos>
__device__ void emit_order(const Tv16FillBucket &d, uint32_t cnt, uint32_t rem, uint32_t np, uint32_t tail_rank,
                           GetPos pos_of) {
    const bool vec = aligned16(d) && (cnt & 3u) == 0;
    constexpr uint32_t PER = FILL_WG / 4;
    for (uint32_t i0 = threadIdx.x >> 2; i0 < np; i0 += 4 * PER) {
        EmitEnt e0, e1, e2, e3;
        emit_load(d, i0, np, rem, tail_rank, vec, pos_of, e0);
        emit_load(d, i0 + PER, np, rem, tail_rank, vec, pos_of, e1);
        emit_load(d, i0 + 2 * PER, np, rem, tail_rank, vec, pos_of, e2);
        emit_load(d, i0 + 3 * PER, np, rem, tail_rank, vec, pos_of, e3);
        emit_store(d, cnt, e0);
        emit_store(d, cnt, e1);
        emit_store(d, cnt, e2);
        emit_store(d, cnt, e3);
    }
}

// ---------------------------------------------------------------------------
// full path: the literal algorithm on the whole candidate vector
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint2 hld(const uint2 *h, uint32_t i) {
    const uint64_t v = ld_sc1(reinterpret_cast<const uint64_t *>(h) + i);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ void hst(uint2 *h, uint32_t i, uint2 v) {
    st_sc1(reinterpret_cast<uint64_t *>(h) + i, ((uint64_t)v.y << 32) | v.x);
}
// std::__adjust_heap(first, hole, len, value, Compare) with Compare = key <
__device__ void adjust_heap(uint2 *H, uint32_t hole, uint32_t len, uint2 value) {
    const uint32_t top = hole;
    uint32_t sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if (u2f(hld(H, sc).x) < u2f(hld(H, sc - 1).x)) --sc;
        hst(H, hole, hld(H, sc));
        hole = sc;
    }
    if ((len & 1u) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        hst(H, hole, hld(H, sc - 1));
        hole = sc - 1;
    }
    uint32_t par = (hole - 1) / 2;  // std::__push_heap
    while (hole > top && u2f(hld(H, par).x) < u2f(value.x)) {
        hst(H, hole, hld(H, par));
        hole = par;
        par = (hole - 1) / 2;
    }
    hst(H, hole, value);
}

__device__ void full_path(FillLds &S, const Tv16FillBucket &d, uint32_t cnt, uint32_t N, float t, bool tail,
                          float tail_key, uint32_t *fail) {
    uint2 *H = d.heap;
    const uint32_t tid = threadIdx.x;
    // the candidate vector: every line with !(S >= t) in scan order, then the tail
    uint32_t base = 0;
    for (uint32_t l0 = 0; l0 < d.nb; l0 += FILL_WG) {
        const uint32_t l = l0 + tid;
        float s = 0.f;
        bool f = false;
        if (l < d.nb) {
            s = lane_line_sum(d.src + (size_t)l * 16);
            f = !(s >= t);
        }
        uint32_t tot;
        const uint32_t r = blk_excl_scan<FILL_WG / 64>(f ? 1u : 0u, S.sh, &tot);
        if (f) hst(H, base + r, make_uint2(f2u(s), l * 16));
        base += tot;
    }
    if (tail) {
        if (tid == 0) hst(H, base, make_uint2(f2u(tail_key), d.nb * 16));
        ++base;
    }
    if (base != N) {  // the scan and this pass disagree: never emit from it
        if (tid == 0) { g_or(fail, FAIL_LEVELS); st_sc1(d.count_out, POISON_COUNT); }
        return;
    }
    vm_drain();
    __syncthreads();
    // make_heap: parents (N-2)/2 .. 0, one level at a time (disjoint subtrees)
    if (N >= 2) {
        const uint32_t last = (N - 2) / 2;
        for (int dd = (int)depth_of(last + 1); dd >= 0; --dd) {
            const uint32_t lo = (1u << dd) - 1, hi = min((2u << dd) - 2, last);
            for (uint32_t p = lo + tid; p <= hi; p += FILL_WG) adjust_heap(H, p, N, hld(H, p));
            vm_drain();
            __syncthreads();
        }
    }
    // pops (one lane): pop_heap moves the top to the end, so the popped
    // candidates end up at H[N-1], H[N-2], ...
    const uint32_t rem = d.dst_len - cnt;
    if (tid == 0) {
        uint32_t len = N, acc = 0, np = 0;
        while (acc < rem && len > 0) {
            const uint2 top = hld(H, 0);
            const uint32_t n_el = min(16u, min(d.nb * 16 + d.tl - top.y, rem - acc));
            acc += n_el;
            ++np;
            if (len > 1) {
                const uint2 v = hld(H, len - 1);
                hst(H, len - 1, top);
                adjust_heap(H, 0, len - 1, v);
            }
            --len;
        }
        S.npop = np;
    }
    vm_drain();
    __syncthreads();
    const uint32_t np = S.npop;
    uint32_t tail_rank = NONE;
    for (uint32_t i = tid; i < np; i += FILL_WG)
        if (hld(H, N - 1 - i).y == d.nb * 16 && tail) atomicMin(&S.flag, i);
    __syncthreads();
    tail_rank = S.flag;
    emit_order(d, cnt, rem, np, tail_rank, [&](uint32_t i) { return hld(H, N - 1 - i).y; });
}

#ifndef STG_FILL_STAMPS
#define STG_FILL_STAMPS 0
#endif
__global__ void __launch_bounds__(FILL_WG) tv16_fill(Tv16FillArgs A) {
    __shared__ FillLds S;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    uint32_t nst = 0;
    auto stamp = [&](uint32_t v) {
        if (STG_FILL_STAMPS && tid == 0 && b == 0 && nst < 32)
            A.dbg[nst] = v ? v : (uint32_t)__builtin_amdgcn_s_memrealtime();
        ++nst;
    };
    stamp(0);
    const Tv16FillBucket &d = A.bk[b];
    const Decision &D = A.dec[b];
    const uint64_t w0 = ld_sc1(&D.w[0]);
    if ((uint32_t)(w0 >> 32) != ((A.epoch << 8) | TV16_TAG_DEC)) {  // the scan never decided this bucket
        if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(d.count_out, POISON_COUNT); }
        return;
    }
    const uint32_t flags = (uint32_t)w0;
    if (!(flags & TV16_DEC_B) || ld_sc1(A.fail)) return;  // regime A, or the launch already failed
    const uint64_t w1 = ld_sc1(&D.w[1]), w2 = ld_sc1(&D.w[2]), w3 = ld_sc1(&D.w[3]);
    const uint32_t cnt = (uint32_t)(w1 >> 32), M = (uint32_t)w1;
    const uint32_t Wtot = (uint32_t)(w2 >> 32);
    const float tail_key = u2f((uint32_t)w2);
    const uint32_t Qtot = (uint32_t)(w3 >> 32);
    const float t = u2f((uint32_t)w3);
    const bool tail = (flags & TV16_DEC_TAIL) != 0;
    const uint32_t N = d.nb - Qtot + (tail ? 1u : 0u);  // candidate vector length
    const uint32_t rem = d.dst_len - cnt;
    if (!M && !tail) return;
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;
    const bool tail_in = tail && tail_key >= u2f(wlo);
    const uint32_t W = Wtot + (tail_in ? 1u : 0u);
    bool fast = (flags & TV16_DEC_WIN) && N <= POS_LIM && W <= EMAX && W > 0;
    // output-order bins over the window below t (sum descending)
    auto obin = [&](uint32_t e) -> uint32_t {
        const float k = u2f(S.key[e]);
        if (k >= t) return 0u;
        if (!(k > 0.f)) return NBIN - 1;
        return min((tb - 1u - S.key[e]) >> 6, NBIN - 1);
    };
    auto okey = [&](uint32_t e) -> uint64_t { return (uint64_t)(~ford(u2f(S.key[e]))) << 32; };
    if (tid == 0) { S.flag = NONE; S.nv = 0; S.maxpos = 0; S.npop = 0; }
    __syncthreads();
    if (fast) {
        const uint32_t *cu = d.cand, *ci = d.cand + 2 * CAND_CAP;
        for (uint32_t e = tid; e < Wtot; e += FILL_WG) {
            S.key[e] = ld_sc1(&cu[e]);
            S.cix[e] = ld_sc1(&ci[e]);
        }
        if (tail_in && tid == 0) { S.key[Wtot] = f2u(tail_key); S.cix[Wtot] = N - 1; }
        __syncthreads();
        stamp(0);
        // (sum desc, position asc): the output order when no two emitted
        // lines tie; also decides whether the exact heap order is needed
        counting_sort(S.r.o, S.sh, W, obin, [&](uint32_t e) { return okey(e) | S.cix[e]; });
        stamp(0);
        // pops needed (entries with an output offset < rem), the tail's rank,
        // and whether two of the popped lines (or the last popped and the
        // next) have equal sums
        uint32_t np_l = 0, tie_l = 0;
        for (uint32_t i = tid; i < W; i += FILL_WG) {
            if (tail_in && S.r.o.ord[i] == Wtot) S.flag = i;
        }
        __syncthreads();
        const uint32_t tail_rank0 = S.flag;
        for (uint32_t i = tid; i < W; i += FILL_WG) {
            const uint32_t off = 16u * i - (tail_rank0 < i ? 16u - d.tl : 0u);
            if (off < rem) {
                np_l = max(np_l, i + 1);
                if (i + 1 < W && S.key[S.r.o.ord[i]] == S.key[S.r.o.ord[i + 1]]) tie_l = 1;
            }
        }
        np_l = wave_max(np_l);
        tie_l = wave_max(tie_l);
        if ((tid & 63u) == 0) { atomicMax(&S.npop, np_l); if (tie_l) S.nv = 1; }
        __syncthreads();
        const uint32_t P0 = S.npop;
        const bool ties = S.nv != 0;
        const uint32_t covered = 16u * W - (tail_in ? 16u - d.tl : 0u);
        fast = covered >= rem;
        if (fast && !ties) {  // distinct sums: the heap pops them in sum order
            emit_order(d, cnt, rem, P0, tail_rank0, [&](uint32_t i) {
                const uint32_t e = S.r.o.ord[i];
                return e == Wtot ? d.nb * 16 : ld_sc1(&d.cand[CAND_CAP + e]);
            });
            stamp(5);
            return;
        }
        __syncthreads();
        if (tid == 0) { S.flag = NONE; S.npop = 0; S.nv = 0; }
        __syncthreads();
    }
    if (fast) {
        // ---- the shadow heap (see (1) above) ----
        // DFS order of the initial positions
        for (uint32_t e = tid; e < W; e += FILL_WG) S.cix[e] = dkey_of_pos(S.cix[e]);
        __syncthreads();
        counting_sort(S.r.a.s, S.sh, W, [&](uint32_t e) { return S.cix[e] >> 14; },
                      [&](uint32_t e) { return (uint64_t)S.cix[e]; });
        stamp(0);
        // nodes: U = the common ancestors of DFS-adjacent elements (pair i owns
        // those deeper than pair i-1's lowest common ancestor: each node once),
        // S = each element's start when alone in its subtree: the top of the
        // largest subtree holding no other element
        const uint16_t *eo = S.r.a.s.ord;
        auto L = [&](uint32_t i) -> int { return dk_lca(S.cix[eo[i]], S.cix[eo[i + 1]]); };
        constexpr uint32_t PT = EMAX / FILL_WG;  // pairs / elements per thread
        uint32_t nmine = 0;
        for (uint32_t u = 0; u < PT; ++u) {
            const uint32_t i = PT * tid + u;
            if (i + 1 < W) nmine += (uint32_t)max(0, L(i) - (i ? L(i - 1) : -1));
            if (i < W) {
                int sh = -1;
                if (i) sh = max(sh, L(i - 1));
                if (i + 1 < W) sh = max(sh, L(i));
                nmine += sh < (int)dk_depth(S.cix[eo[i]]);
            }
        }
        uint32_t nv;
        uint32_t vo = blk_excl_scan<FILL_WG / 64>(nmine, S.sh, &nv);
        fast = nv <= VCAP;
        if (fast) {
            for (uint32_t u = 0; u < PT; ++u) {
                const uint32_t i = PT * tid + u;
                if (i + 1 < W) {
                    const int hi = L(i), lo = i ? L(i - 1) : -1;
                    const uint32_t k = S.cix[eo[i]];
                    for (int dd = lo + 1; dd <= hi; ++dd) S.r.a.vlist[vo++] = dk_anc(k, (uint32_t)dd);
                }
            }
            // starts (held in registers until every thread has read the keys)
            uint32_t st0 = NONE, st1 = NONE, st2 = NONE, st3 = NONE;
            static_assert(PT == 4, "four elements per thread");
            auto start_of = [&](uint32_t i, uint32_t &vo_, uint32_t &st) {
                if (i >= W) return;
                int sh = -1;
                if (i) sh = max(sh, L(i - 1));
                if (i + 1 < W) sh = max(sh, L(i));
                const uint32_t k = S.cix[eo[i]];
                if (sh < (int)dk_depth(k)) {
                    st = dk_anc(k, (uint32_t)(sh + 1));
                    S.r.a.vlist[vo_++] = st;
                } else {
                    st = k;  // its own node holds others: a U node
                }
            };
            start_of(PT * tid + 0, vo, st0);
            start_of(PT * tid + 1, vo, st1);
            start_of(PT * tid + 2, vo, st2);
            start_of(PT * tid + 3, vo, st3);
            __syncthreads();
            if (st0 != NONE) S.cix[eo[PT * tid + 0]] = st0;
            if (st1 != NONE) S.cix[eo[PT * tid + 1]] = st1;
            if (st2 != NONE) S.cix[eo[PT * tid + 2]] = st2;
            if (st3 != NONE) S.cix[eo[PT * tid + 3]] = st3;
            __syncthreads();
            stamp(0);
            // the nodes in DFS order
            counting_sort(S.r.a.s, S.sh, nv, [&](uint32_t i) { return S.r.a.vlist[i] >> 14; },
                          [&](uint32_t i) { return (uint64_t)S.r.a.vlist[i]; });
            for (uint32_t i = tid; i < nv; i += FILL_WG) S.r.h.vk[i] = S.r.a.vlist[S.r.a.s.ord[i]];
            __syncthreads();
            // links and contents
            for (uint32_t v = tid; v < nv; v += FILL_WG) {
                S.r.h.vr[v] = (uint16_t)vfind(S, nv, dk_right(S.r.h.vk[v]));
                S.r.h.vc[v] = NONE16;
            }
            __syncthreads();
            for (uint32_t e = tid; e < W; e += FILL_WG) S.r.h.vc[vfind(S, nv, S.cix[e])] = (uint16_t)e;
            // internal nodes (a child among the nodes) by depth
            if (tid <= DMAX + 1) S.uoff[tid] = 0;
            __syncthreads();
            for (uint32_t v = tid; v < nv; v += FILL_WG)
                if (S.r.h.vr[v] != NONE16 || vleft(S, nv, v) != NONE16) atomicAdd(&S.uoff[dk_depth(S.r.h.vk[v]) + 1], 1u);
            __syncthreads();
            if (tid == 0) {
                for (uint32_t dd = 1; dd <= DMAX + 1; ++dd) S.uoff[dd] += S.uoff[dd - 1];
                for (uint32_t dd = 0; dd <= DMAX; ++dd) S.sh[dd] = S.uoff[dd];
            }
            __syncthreads();
            for (uint32_t v = tid; v < nv; v += FILL_WG)
                if (S.r.h.vr[v] != NONE16 || vleft(S, nv, v) != NONE16)
                    S.r.h.ulist[atomicAdd(&S.sh[dk_depth(S.r.h.vk[v])], 1u)] = (uint16_t)v;
            __syncthreads();
            stamp(0);
            // make_heap, deepest level first (a level's subtrees are disjoint)
            for (int dd = DMAX - 1; dd >= 0; --dd) {
                const uint32_t o0 = S.uoff[dd], o1 = S.uoff[dd + 1];
                for (uint32_t i = o0 + tid; i < o1; i += FILL_WG) shadow_sift(S, nv, S.r.h.ulist[i], N);
                if (o1 > o0) __syncthreads();
                if (STG_FILL_STAMPS && tid == 0 && b == 0) {
                    A.dbg[32 + dd] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                    A.dbg[52 + dd / 2] = 0;
                }
            }
            if (STG_FILL_STAMPS && tid == 0 && b == 0) {
                A.dbg[54] = nv;
                for (int dd = 0; dd < 8; ++dd) A.dbg[55 + dd] = S.uoff[10 + dd + 1] - S.uoff[10 + dd];
            }
            stamp(0);
            // final positions
            uint32_t mp = 0;
            for (uint32_t v = tid; v < nv; v += FILL_WG) {
                const uint32_t e = S.r.h.vc[v];
                if (e != NONE16) {
                    const uint32_t pos = dk_pos(S.r.h.vk[v]);
                    S.cix[e] = pos;
                    mp = max(mp, pos);
                }
            }
            mp = wave_max(mp);
            if ((tid & 63u) == 0) atomicMax(&S.maxpos, mp);
            __syncthreads();
            // output order: sum desc, then right-first pre-order of the position
            counting_sort(S.r.o, S.sh, W, obin, [&](uint32_t e) { return okey(e) | rf_key(S.cix[e]); });
            for (uint32_t i = tid; i < W; i += FILL_WG)
                if (tail_in && S.r.o.ord[i] == Wtot) S.flag = i;
            __syncthreads();
            const uint32_t tail_rank = S.flag;
            uint32_t npl = 0;
            for (uint32_t i = tid; i < W; i += FILL_WG) {
                const uint32_t off = 16u * i - (tail_rank < i ? 16u - d.tl : 0u);
                if (off < rem) npl = max(npl, i + 1);
            }
            npl = wave_max(npl);
            if ((tid & 63u) == 0) atomicMax(&S.npop, npl);
            __syncthreads();
            const uint32_t P = S.npop;
            stamp(0);
            // the pops never reinsert an element of R (see (2) above)
            if (S.maxpos + P < N) {
                emit_order(d, cnt, rem, P, tail_rank, [&](uint32_t i) {
                    const uint32_t e = S.r.o.ord[i];
                    return e == Wtot ? d.nb * 16 : ld_sc1(&d.cand[CAND_CAP + e]);
                });
                stamp(1);
                return;
            }
            fast = false;
        }
        __syncthreads();
        if (tid == 0) { S.flag = NONE; S.npop = 0; }
        __syncthreads();
    }
    stamp(3);
    full_path(S, d, cnt, N, t, tail, tail_key, A.fail);
    stamp(0);
}

}  // namespace

hipError_t launch_tv16_fill(const Tv16FillArgs &a, hipStream_t s) {
    if (!a.nbk) return hipSuccess;
    tv16_fill<<<a.nbk, FILL_WG, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace stg
