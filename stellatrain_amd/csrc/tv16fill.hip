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
//  (3) Without the heap: an element leaves the subtree of its start node
//      only upwards, through its ancestors (it moves down only as the value
//      of its own sift, inside that subtree), and a node takes the larger of
//      its children's entries, the right one on equal sums, from subtrees
//      that are heaps by then.  So of two equal sums a, b whose start nodes
//      are not one above the other, the one on the right side of their
//      lowest common ancestor passes it first (the other side's entry is
//      >= the other element), and they keep that order above it, through
//      the pops.  Hence when no two equal sums among the pops start one
//      above the other, they pop in right-first pre-order of their START
//      positions; and when no element of R starting in the last P + 1
//      positions has an R element at its parent or sibling, each of them
//      has moved up before the pops begin, so (2) holds.  Both are checked
//      (a few thousand comparisons); almost every regime-B call ends here.
// Full path (otherwise: the window missed the top M, > 4096 entries, or a
// bucket of 2^20+ lines): the candidate vector is built in global memory and
// make_heap / pop_heap run literally (make_heap level-parallel: subtrees of
// one level are disjoint).  Slow (milliseconds at 64 MiB), exact, rare.
//
// Built twice (Makefile): tv16fill.o with STG_WIRE_EMIT=0 writes the codec's
// u32 / f32 stream, with the registers of a fill that has no wire stores;
// tv16fillw.o (STG_WIRE_EMIT=1) also writes the wire form (wire_dev.h) and is
// launched when a bucket of the call asks for it.
#ifndef STG_WIRE_EMIT
#define STG_WIRE_EMIT 0
#endif
#include <algorithm>
#include <cstddef>

#include "tv16_dev.h"

namespace stg {

namespace {

using namespace tv16;

constexpr uint32_t FILL_WG = 512;              // 8 waves: beside two 12-wave scan workgroups
constexpr uint32_t FNW_F = FILL_WG / 64;
constexpr uint32_t EMAX = 4096;                // window entries kept (+ the ragged tail)
constexpr uint32_t VCAP = 6144;                // shadow-heap nodes held (more: full path)
constexpr uint32_t POS_LIM = (1u << 20) - 1;   // fast path: N <= POS_LIM (20-bit paths)
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t NONE13 = 0x1fffu;           // no node (13-bit node index)
constexpr uint32_t CNONE = 0xffffffu;          // content -inf (24-bit content field)
constexpr uint32_t NBIN = 1024;                // counting-sort bins
constexpr uint32_t NDEP = 20;                  // depths 0..19
constexpr uint32_t PT = EMAX / FILL_WG;        // ranks / DFS slots per thread
constexpr uint32_t NJ = VCAP / FILL_WG;        // nodes per thread
constexpr uint32_t TCAP = 256;                 // tied ranks checked without the heap (more: the heap)
constexpr uint32_t ECAP = 64;                  // late start positions checked (more: the heap)
static_assert(VCAP < NONE13, "13-bit node indices");
static_assert(NBIN << 8 == TV16_WIN, "output-sort bins of 256 ulps cover the window");

// A heap node as a DFS key: its path from the root left-aligned to depth 19
// (20 bits) << 5 | its depth.  Ascending keys = pre-order, left subtree first;
// ancestors come before their descendants.
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
// depth of the lowest common ancestor of two nodes (DFS keys)
__device__ __forceinline__ int dk_lca(uint32_t a, uint32_t b) {
    const uint32_t m = min(dk_depth(a), dk_depth(b));
    const uint32_t x = ((a >> 5) ^ (b >> 5)) >> (19u - m);  // path bits down to depth m
    return x ? (int)m - (int)(32u - __clz(x)) : (int)m;
}

// A shadow-heap node record (8 bytes, one ds_read_b64):
//   .x = content (grp << 12 | rank; CNONE: -inf) | pos[7:0] << 24
//   .y = pos[19:8] | right child << 12 | has left << 25 | has right << 26 | U << 27
// The left child, when present, is the next node in pre-order.
__device__ __forceinline__ uint32_t r_content(uint2 r) { return r.x & CNONE; }
__device__ __forceinline__ uint32_t r_pos(uint2 r) { return (r.x >> 24) | ((r.y & 0xfffu) << 8); }
__device__ __forceinline__ uint32_t r_right(uint2 r) { return (r.y >> 12) & NONE13; }
__device__ __forceinline__ bool r_hasl(uint2 r) { return (r.y >> 25) & 1u; }
__device__ __forceinline__ bool r_hasr(uint2 r) { return (r.y >> 26) & 1u; }
__device__ __forceinline__ bool r_isu(uint2 r) { return (r.y >> 27) & 1u; }
__device__ __forceinline__ uint2 r_make(uint32_t content, uint32_t pos, bool isu) {
    return make_uint2(content | (pos << 24), (pos >> 8) | (isu ? 1u << 27 : 0u));
}

struct SortScratch {
    uint32_t bin[NBIN];  // counts -> starts
    uint32_t cur[NBIN];  // scatter cursors
    uint16_t tmp[EMAX];  // items grouped by bin
};

// LDS of a fill workgroup: it runs beside two scan workgroups on one CU.
// Elements are window entries (ids < W); ranks are positions in the output
// order `ord`; R, the shadow heap's elements, are the ranks [0, rn).  The
// union's views follow the phases; each is written only after a barrier that
// ends every read of what it covers.
struct FillLds {
    uint16_t ord[EMAX];  // rank -> element: (sum desc, position asc), then ties in heap order
    uint16_t grp[EMAX];  // rank -> first rank of its equal-sum run
    union {
        struct {  // load and output sort
            uint32_t key[EMAX];   // element -> line-sum bits (the tail: its signed key's bits)
            uint32_t cix[EMAX];   // element -> candidate index (= start heap position)
            SortScratch s;
            uint32_t line[EMAX];  // element -> first element of its line (the emission; V goes over it)
        } a;
        struct {  // DFS sort of R
            uint32_t dk[EMAX];  // rank -> DFS key of its start position (over key)
            uint16_t eo[EMAX];  // ranks in DFS order (over cix)
            uint16_t pad[EMAX];
            SortScratch s;
        } b;
        struct {  // the nodes V in pre-order (over dk / eo: built from registers)
            uint32_t vk[VCAP];    // DFS key
            uint2 rec[VCAP + 1];  // [VCAP]: a -inf leaf, read in place of a missing node
        } v;
        struct {  // the sift
            uint16_t ul[VCAP];  // U nodes by depth, deepest first (over vk)
            uint16_t pad[VCAP];
            uint2 rec[VCAP + 1];
        } w;
        struct {  // the tie order
            uint32_t fpos[EMAX];  // rank -> final heap position (over ul)
            uint16_t ord2[EMAX];
        } f;
    } u;
    uint32_t sh[32];  // block-scan scratch
    uint32_t cnt[NDEP + 1], uoff[NDEP + 1];
    uint16_t tl[TCAP];  // tied ranks among the pops
    uint32_t el[ECAP];  // start positions of R among the last P + 1
    uint32_t flag, nv, maxpos, npop, dmax, rn, nc, nu, ntl, nel, flag2, et;
};
static_assert(sizeof(FillLds) + 2 * TV16_SCAN_LDS <= 160 * 1024, "a fill workgroup beside two scan workgroups");
static_assert(EMAX <= 4096, "ranks fit the 12-bit content fields");
static_assert(sizeof(uint32_t) * EMAX + sizeof(uint16_t) * EMAX <= sizeof(uint32_t) * VCAP,
              "the tie order stays clear of the node records");

// Counting sort of items 0..n-1 by (bin(i), full(i)) ascending into out:
// bins of a few items each; inside a bin, an item's rank is the number of
// bin members with a smaller full key.
template <typename Bin, typename Full>
__device__ void counting_sort(SortScratch &X, uint16_t *out, uint32_t *sh, uint32_t n, Bin bin_of, Full full_of) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < NBIN; i += FILL_WG) X.bin[i] = 0;
    __syncthreads();
    for (uint32_t e = tid; e < n; e += FILL_WG) atomicAdd(&X.bin[bin_of(e)], 1u);
    __syncthreads();
    {  // exclusive scan of the bins, NBIN / FILL_WG per thread
        constexpr uint32_t PER = NBIN / FILL_WG;
        static_assert(PER == 2, "two bins per thread");
        const uint32_t c0 = X.bin[PER * tid], c1 = X.bin[PER * tid + 1];
        uint32_t tot;
        const uint32_t run = blk_excl_scan<FNW_F>(c0 + c1, sh, &tot);
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
        out[r] = (uint16_t)e;
    }
    __syncthreads();
}


// Emit the lines / tail of the output order: entry i of the order goes to
// offset cnt + 16 i (less 16 - tl after the tail), at most rem elements.  Four
// lanes per line (a float4 each: one 64-byte request per line), eight rounds
// of loads in flight before their stores.
// W: the stream's wire form (one instance per form, so that the plain one's
// registers are those of a kernel without the wire stores).
template <uint32_t K, bool W, typename GetPos>
__device__ __forceinline__ void emit_order_w(const Tv16FillBucket &d, uint32_t cnt, uint32_t rem, uint32_t np,
                                             uint32_t tail_rank, GetPos pos_of, uint32_t i_lo, uint32_t i_hi) {
    np = min(np, i_hi);  // ranks [i_lo, min(np, i_hi)) of the order
    constexpr uint32_t LPR = FILL_WG / 4;  // lines per round; K rounds of loads in flight
    const bool vec = aligned16(d) && (cnt & 3u) == 0;
    const uint32_t q = threadIdx.x & 3u;
    auto span = [&](uint32_t i, uint32_t &off, uint32_t &len) {  // output offset and length of entry i
        len = 0;
        off = 16u * i - (tail_rank < i ? 16u - d.tl : 0u);
        if (i < np && off < rem) len = min(i == tail_rank ? d.tl : 16u, rem - off);
    };
    for (uint32_t i0 = i_lo + (threadIdx.x >> 2); i0 < np; i0 += K * LPR) {
        float4 x[K];
#pragma unroll
        for (uint32_t r = 0; r < K; ++r) {
            uint32_t off, len;
            const uint32_t i = i0 + r * LPR;
            span(i, off, len);
            x[r] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (vec && len == 16 && (off & 3u) == 0)
                x[r] = reinterpret_cast<const float4 *>(d.src + (size_t)pos_of(i))[q];
        }
#pragma unroll
        for (uint32_t r = 0; r < K; ++r) {
            uint32_t off, len;
            const uint32_t i = i0 + r * LPR;
            span(i, off, len);
            if (!len) continue;
            const uint32_t pos = pos_of(i), o = cnt + off + 4 * q, bi = pos + 4 * q + (uint32_t)d.idx_offset;
            if (vec && len == 16 && (off & 3u) == 0) {
                put_pair4_w<W>(d, o, bi, x[r]);
            } else {
                for (uint32_t c = 0; c < 4; ++c) {
                    if (4 * q + c < len) {
                        put_pair_w<W>(d, o + c, bi + c, d.src[(size_t)pos + 4 * q + c]);
                    }
                }
            }
        }
    }
}
template <uint32_t K = 5, typename GetPos>
__device__ __forceinline__ void emit_order(const Tv16FillBucket &d, uint32_t cnt, uint32_t rem, uint32_t np, uint32_t tail_rank,
                           GetPos pos_of, uint32_t i_lo = 0, uint32_t i_hi = 0xffffffffu) {
    if (STG_WIRE_EMIT && d.wflag) emit_order_w<K, true>(d, cnt, rem, np, tail_rank, pos_of, i_lo, i_hi);
    else emit_order_w<K, false>(d, cnt, rem, np, tail_rank, pos_of, i_lo, i_hi);
}

// The orderer's emission of the pops' order: with helper workgroups (a lone
// bucket), publish the order's line positions and the pop count, then emit
// share 0; the helpers emit the other shares.
template <uint32_t KE, bool LONE, typename GetPos>
__device__ __forceinline__ void emit_all(const Tv16FillBucket &d, uint32_t cnt, uint32_t rem, uint32_t P,
                                         uint32_t tail_rank, GetPos pos_of, uint32_t nhelp, CallCtl *ccp,
                                         uint32_t *order_g, uint32_t ready_tag) {
    if (LONE && nhelp) {
        for (uint32_t i = threadIdx.x; i < P; i += FILL_WG) st_sc1(&order_g[i], pos_of(i));
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (threadIdx.x == 0) {
            st_sc1(&ccp->pad[2], P);
            st_sc1(&ccp->pad[3], tail_rank);
            __builtin_amdgcn_s_waitcnt(0);
            st_sc1(&ccp->pad[1], ready_tag);
        }
        emit_order<KE>(d, cnt, rem, P, tail_rank, pos_of, 0, (P + nhelp) / (nhelp + 1));
    } else {
        emit_order<KE>(d, cnt, rem, P, tail_rank, pos_of);
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

// The pops of the literal heap, by one wave.  Each pop is GCC's pop_heap /
// __adjust_heap / __push_heap exactly (the element moves are the same); only
// where the nodes are read differs:
//  * positions < HC (depths 0..12) are held in LDS (Hl);
//  * the descent reads its nodes a batch at a time: every node of the next
//    4 or 8 levels below the hole in one round of loads (batch roots at depths
//    0, 4, 12, 20, ...), then walks those levels with readlane.  The depths
//    13..20 of a 2^20-line bucket are one round of global loads per pop
//    instead of eight dependent ones.
//  * every global position p is loaded and stored only by lane hl_lane(p)
//    (its lane in the one batch that holds its depth), so a lane re-reads what
//    it wrote itself;
//  * __push_heap climbs the descent path, whose new contents are kept in pv.
constexpr uint32_t HC = 8191;  // heap positions held in LDS by the pops
static_assert(sizeof(uint2) * (HC + 32) <= sizeof(decltype(FillLds::u)), "the LDS heap fits the union");
__device__ __forceinline__ uint32_t hl_rootdepth(uint32_t dd) { return dd <= 4 ? 0u : 4u + ((dd - 5u) >> 3) * 8u; }
__device__ __forceinline__ uint32_t hl_lane(uint32_t p) {
    const uint32_t dd = depth_of(p + 1), j = dd - hl_rootdepth(dd);
    return (p + 1) & ((1u << min(j, 6u)) - 1u);
}
__device__ __forceinline__ uint2 rl2(uint2 v, uint32_t l) {
    return make_uint2(__builtin_amdgcn_readlane(v.x, l), __builtin_amdgcn_readlane(v.y, l));
}
__device__ __forceinline__ void hl_put(uint2 *Hl, uint2 *H, uint32_t p, uint2 v, uint32_t lane) {
    if (p < HC) Hl[p] = v;  // every lane writes the same value
    else if (lane == hl_lane(p)) hst(H, p, v);
}
// level j (1..8) of a batch: offset o in slot (j <= 6 ? j - 1 : j == 7 ? 6 + o / 64 : 8 + o / 64), lane o % 64.
// A batch is all in LDS (roots at depths 0, 4) or all in global memory (roots
// at depths 12, 20, ...).  The loads carry no branches (a node past the heap
// reads a clamped LDS slot or 0 from the bounded buffer and is never walked
// to), so a batch's loads are all in flight together.
__device__ __forceinline__ uint2 hb_gld(__amdgpu_buffer_rsrc_t r, uint64_t p, uint32_t L) {
    typedef unsigned int u2v __attribute__((ext_vector_type(2)));
    const uint32_t off = p < L ? (uint32_t)p * 8u : 0xfffffff0u;
    const u2v v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16 /* sc1 */);
    return make_uint2(v.x, v.y);
}
template <int D, bool GLB>
__device__ __forceinline__ void hb_load(uint2 (&b)[12], const uint2 *Hl, __amdgpu_buffer_rsrc_t r, uint32_t root,
                                        uint32_t L, uint32_t lane) {
#pragma unroll
    for (int j = 1; j <= D; ++j) {
        const int ns = j <= 6 ? 1 : (1 << (j - 6)), s0 = j <= 6 ? j - 1 : (j == 7 ? 6 : 8);
#pragma unroll
        for (int q = 0; q < ns; ++q) {
            const uint64_t p = (((uint64_t)root + 1) << j) - 1 + (uint32_t)q * 64u + lane;
            b[s0 + q] = GLB ? hb_gld(r, p, L) : Hl[min(p, (uint64_t)HC - 1)];
        }
    }
}
template <int J>
__device__ __forceinline__ uint2 hb_node(const uint2 (&b)[12], uint32_t o) {
    if constexpr (J <= 6) return rl2(b[J - 1], o);
    else if constexpr (J == 7) return (o >> 6) ? rl2(b[7], o & 63u) : rl2(b[6], o & 63u);
    const uint32_t g = o >> 6, l = o & 63u;
    const uint2 a0 = rl2(b[8], l), a1 = rl2(b[9], l), a2 = rl2(b[10], l), a3 = rl2(b[11], l);
    return g == 0 ? a0 : g == 1 ? a1 : g == 2 ? a2 : a3;
}
// Level J of the walk below a batch root (the hole at offset o of level J - 1).
// Returns false when the descent has ended.
template <int J, int D>
__device__ __forceinline__ bool hb_steps(const uint2 (&b)[12], uint2 *Hl, uint2 *H, uint2 *pv, uint32_t &hole,
                                         uint32_t o, uint32_t L, uint32_t lane) {
    if constexpr (J > D) {
        return true;
    } else {
        const uint32_t dh = depth_of(hole + 1);
        if (hole < (L - 1) / 2) {
            const uint2 cl = hb_node<J>(b, 2 * o), cr = hb_node<J>(b, 2 * o + 1);
            const bool left = u2f(cr.x) < u2f(cl.x);
            const uint2 c = left ? cl : cr;
            hl_put(Hl, H, hole, c, lane);
            pv[dh] = c;
            hole = 2 * hole + (left ? 1u : 2u);
            return hb_steps<J + 1, D>(b, Hl, H, pv, hole, 2 * o + (left ? 0u : 1u), L, lane);
        }
        if ((L & 1u) == 0 && hole == (L - 2) / 2) {  // a left child only
            const uint2 c = hb_node<J>(b, 2 * o);
            hl_put(Hl, H, hole, c, lane);
            pv[dh] = c;
            hole = 2 * hole + 1;
        }
        return false;
    }
}
// Walk up to D levels below `hole` (a batch root) for a heap of length L.
template <int D, bool GLB>
__device__ __forceinline__ bool hb_walk(uint2 *Hl, uint2 *H, __amdgpu_buffer_rsrc_t r, uint2 *pv, uint32_t &hole,
                                        uint32_t L, uint32_t lane) {
    uint2 b[12];
    hb_load<D, GLB>(b, Hl, r, hole, L, lane);
    return hb_steps<1, D>(b, Hl, H, pv, hole, 0u, L, lane);
}
template <typename T>
__device__ __forceinline__ T *uni_ptr(T *p) {  // a wave-uniform pointer, in SGPRs
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    return reinterpret_cast<T *>(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a));
}
// (noinline: the kernel keeps its own register budget; the arguments are
// made wave-uniform again here, so the walk's branches and readlanes are scalar)
__device__ __attribute__((noinline)) uint32_t wave_pops(uint2 *Hl, uint2 *pv, uint2 *H, uint32_t N, uint32_t rem,
                                                        uint32_t end, uint32_t lane) {
    Hl = uni_ptr(Hl);
    pv = uni_ptr(pv);
    H = uni_ptr(H);
    N = __builtin_amdgcn_readfirstlane(N);
    rem = __builtin_amdgcn_readfirstlane(rem);
    end = __builtin_amdgcn_readfirstlane(end);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(H, 0, N * 8u, 0x00020000);
    uint32_t len = N, acc = 0, np = 0;
    while (acc < rem && len > 0) {
        const uint2 top = Hl[0];
        const uint32_t n_el = min(16u, min(end - top.y, rem - acc));
        acc += n_el;
        ++np;
        if (len > 1) {
            const uint32_t L = len - 1, lv = hl_lane(L);
            // the last element: its global load is read only at the climb
            const uint2 vl = Hl[min(L, HC - 1)], vg = hb_gld(r, L, L + 1);
            hl_put(Hl, H, L, top, lane);
            // __adjust_heap(first, 0, L, v): batches at depths 0 (4 levels), 4 (8), 12, 20, ... (8)
            uint32_t hole = 0;
            if (hb_walk<4, false>(Hl, H, r, pv, hole, L, lane) && hb_walk<8, false>(Hl, H, r, pv, hole, L, lane))
                while (hb_walk<8, true>(Hl, H, r, pv, hole, L, lane)) {
                }
            // __push_heap: the path above the hole holds pv[0 .. depth - 1]
            const uint2 v = L < HC ? vl : rl2(vg, lv);
            uint32_t dh = depth_of(hole + 1);
            while (hole > 0) {
                const uint2 pc = pv[dh - 1];
                if (!(u2f(pc.x) < u2f(v.x))) break;
                hl_put(Hl, H, hole, pc, lane);
                hole = (hole - 1) / 2;
                --dh;
            }
            hl_put(Hl, H, hole, v, lane);
        }
        --len;
    }
    return np;
}

__device__ void full_path(FillLds &S, const Tv16FillBucket d, uint32_t cnt, uint32_t N, float t, bool tail,
                          float tail_key, uint32_t *fail) {
    uint2 *H = d.heap;
    const uint32_t tid = threadIdx.x;
    __syncthreads();
    if (tid == 0) { S.flag = NONE; S.npop = 0; }  // the tail's rank below starts from NONE (any caller)
    __syncthreads();
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
    // pops (wave 0): pop_heap moves the top to the end, so the popped
    // candidates end up at H[N-1], H[N-2], ...  The top HC positions live in
    // LDS meanwhile (written back below).
    const uint32_t rem = d.dst_len - cnt;
    uint2 *Hl = reinterpret_cast<uint2 *>(&S.u);
    const uint32_t nl = min(N, HC);
    for (uint32_t p = tid; p < nl; p += FILL_WG) Hl[p] = hld(H, p);
    __syncthreads();
    if (tid < 64) {
        const uint32_t np = wave_pops(Hl, Hl + HC, H, N, rem, d.nb * 16 + d.tl, tid);
        if (tid == 0) S.npop = np;
    }
    __syncthreads();
    for (uint32_t p = tid; p < nl; p += FILL_WG) hst(H, p, Hl[p]);
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

#include "tv16lfin.h"
#include "tv16wide.h"

// Registers for 8 waves per SIMD (<= 64 VGPRs): the workgroup's two waves per
// SIMD run beside the six of two scan workgroups.  The LDS is dynamic: the
// compiler derives the occupancy it aims for from static LDS and would widen
// the register budget to the one workgroup per CU that 88 KiB alone allows.
// LONE: the launch's only bucket(s), nothing co-resident to share the CU
// with: 4 waves per SIMD (128 VGPRs), the whole window prefetched (no second
// round trip for its tail) and twice the emission loads in flight.
template <bool LONE>
__global__ void __launch_bounds__(FILL_WG) __attribute__((amdgpu_waves_per_eu(LONE ? 4 : 8, 8)))
tv16_fill(Tv16FillArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fill_lds[];
    FillLds &S = *reinterpret_cast<FillLds *>(fill_lds);
    // LONE with helpers: one bucket, 1 + A.helpers workgroups; the first to
    // start (ticket 0) orders the lines, the others wait for its order and
    // emit a share of it (each waits only on a workgroup already running)
    __shared__ uint32_t s_role, s_last;
    const uint32_t tid = threadIdx.x;
    // a one-bucket call its scan launch finished (tv16lf2.h): nothing to do
    if (LONE && A.fin && !__syncthreads_or(tid < A.fin && A.fin_done[tid] != A.fin_tag)) return;
    if (!LONE && blockIdx.x >= A.nbk) {  // the crew (tv16wide.h)
        crew_from_decisions<LONE>(*reinterpret_cast<WideLds *>(fill_lds), S, A);
        return;
    }
    uint32_t role = 0;
    if (LONE && (A.helpers || A.lfin || A.crew)) {
        if (tid == 0) s_role = g_add(&A.cc->pad[0], 1u);
        __syncthreads();
        role = s_role;
    }
    if (LONE && !A.lfin && role > A.helpers) {  // the crew of a lone launch with helpers
        crew_from_decisions<LONE>(*reinterpret_cast<WideLds *>(fill_lds), S, A);
        return;
    }
    // lfin (tv16lfin.h): tickets [0, workers) finish the scan, the next
    // `rankers` order the regime-B fill in parallel; the last workgroup to
    // finish runs the exact orderer below only when the rankers could not
    // prove their order.  No helpers in this mode.
    const uint32_t first_helper = A.lfin ? 0xffffffffu : 1u;
    if (LONE && A.lfin) {
        LfinLds &Lf = *reinterpret_cast<LfinLds *>(fill_lds);
        if (tid == 0) {
            LfinArgs &W = Lf.args;
            W.d = A.bk[0];
            W.nc = A.nc;
            W.workers = A.workers;
            W.rankers = A.rankers;
            W.epoch = A.epoch;
            W.mode = A.mode;
            W.ldesc = A.ldesc;
            W.lq = A.lq;
            W.lw = A.lw;
            W.lv = A.lv;
            W.whist = A.whist;
            W.went = A.went;
            W.state = A.state;
            W.cp = A.cp;
            W.resid = A.resid;
            W.fail = A.fail;
            W.dec = const_cast<Decision *>(A.dec);
            W.cc = A.cc;
            W.dbg = A.dbg;
        }
        __syncthreads();
        if (role < A.workers) lfin_worker(Lf, role);
        else if (role < A.workers + A.rankers) lfin_ranker(Lf, role - A.workers);
        else {  // the crew (tv16wide.h): not counted among the roles below
            crew_lfin(Lf, A);
            return;
        }
        vm_drain();  // every wave's stores drained, then one add for the workgroup
        __syncthreads();
        if (tid == 0) s_last = g_add(&A.cc->pad[4], 1u) == A.workers + A.rankers - 1;
        __syncthreads();
        if (STG_FILL_STAMPS && tid == 0) {  // diagnostics: each role's arrival (words 24..27: worker 0, ranker 0, last)
            if (role == 0) A.dbg[24] = (uint32_t)__builtin_amdgcn_s_memrealtime();
            if (role == A.workers) A.dbg[25] = (uint32_t)__builtin_amdgcn_s_memrealtime();
            if (s_last) { A.dbg[26] = (uint32_t)__builtin_amdgcn_s_memrealtime(); A.dbg[27] = role; }
        }
        if (!s_last) return;
        // every role is done with the binned window: zero its counts for the next call
        for (uint32_t i = tid; i < LNBIN; i += FILL_WG) st_sc1(&A.whist[i], 0u);
        const uint32_t rep = ld_sc1(&A.cc->pad[5]);
        // how the call's fill was ordered (debug words 48..51: rankers without
        // ties, rankers with ties, the orderer after a violation, the orderer
        // for a call the rankers could not take; tests read them)
        const bool ranked = A.rankers && !(rep & LF_FALLBACK) && !((rep & LF_TIES) && (rep & LF_VIOL));
        if (tid == 0 && (rep & (LF_RANKED | LF_FALLBACK)))
            atomicAdd(&A.dbg[48 + (ranked ? ((rep & LF_TIES) ? 1 : 0) : ((rep & LF_FALLBACK) ? 3 : 2))], 1u);
        if (ranked) return;
        lfin_list(Lf);  // the orderer's input (its LDS view then goes over the lfin view)
    }
    const uint32_t b = LONE ? 0u : blockIdx.x;  // a lone launch has one bucket
    uint32_t nst = 0;
    auto stamp = [&](uint32_t v) {
        if (STG_FILL_STAMPS && tid == 0 && b == 0 && nst < 32)
            A.dbg[nst] = v ? v : (uint32_t)__builtin_amdgcn_s_memrealtime();
        ++nst;
    };
    // which way each regime-B bucket was ordered (debug words 56..59: no
    // ties, ties by start position, shadow heap, literal heap; tests read them)
    auto count_path = [&](uint32_t path) {
        if (tid == 0) atomicAdd(&A.dbg[56 + path], 1u);
    };
    stamp(0);
    const Tv16FillBucket &d = A.bk[b];
    const Decision &D = A.dec[b];
    uint32_t *const order_g = const_cast<uint32_t *>(d.cand) + 3 * CAND_CAP;  // the spare window array: the order
    const uint32_t ready_tag = (A.epoch << 8) | 0x5au;
    if (LONE && role >= first_helper) {  // a helper: wait for the orderer's pop order, emit share `role` of it
        const uint32_t share = role - first_helper + 1;
        uint64_t h0 = ld_sc1(&D.w[0]);
        if (A.lfin) {  // the decision comes from worker 0 of this launch (ticket 0: running)
            uint64_t st1 = 0;
            for (uint32_t spins = 0; (uint32_t)(h0 >> 32) != ((A.epoch << 8) | TV16_TAG_DEC); ++spins) {
                __builtin_amdgcn_s_sleep(4);
                h0 = ld_sc1(&D.w[0]);
                if (spin_expired(spins, st1)) {
                    if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(d.count_out, POISON_COUNT); }
                    return;
                }
            }
        }
        const uint64_t h1 = ld_sc1(&D.w[1]);
        if ((uint32_t)(h0 >> 32) != ((A.epoch << 8) | TV16_TAG_DEC) || !((uint32_t)h0 & TV16_DEC_B) ||
            ld_sc1(A.fail) || share > A.helpers || (A.crew && crew_wants((uint32_t)h0, (uint32_t)h1, A.mode)))
            return;  // no regime-B fill (or the scan failed, or the crew orders it): nothing to emit
        if (!(uint32_t)h1 && !((uint32_t)h0 & TV16_DEC_TAIL)) return;  // nothing missing (the orderer returns too)
        uint64_t st0 = 0;
        for (uint32_t spins = 0; ld_sc1(&A.cc->pad[1]) != ready_tag; ++spins) {
            __builtin_amdgcn_s_sleep(4);
            if (spin_expired(spins, st0)) {
                if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(d.count_out, POISON_COUNT); }
                return;
            }
        }
        const uint32_t P = ld_sc1(&A.cc->pad[2]), tail_rank = ld_sc1(&A.cc->pad[3]);
        const uint32_t nsh = A.helpers + 1u, chunk = (P + nsh - 1) / nsh;
        const uint32_t cnt = (uint32_t)(h1 >> 32), rem = d.dst_len - cnt;
        // the share [i0, i1) of the order, as emit_order writes it (scalars
        // taken out of the argument block first: emitting through a reference
        // to it here made the compiler copy the whole block to scratch)
        const float *src = d.src;
        uint32_t *oidx = d.idx;
        float *oval = d.val;
        const uint32_t tl = d.tl, ioff = (uint32_t)d.idx_offset, wflag = d.wflag, wend = d.wend;
        const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(oidx) |
                           reinterpret_cast<uintptr_t>(oval)) & 15u) == 0 && (cnt & 3u) == 0;
        const uint32_t i1 = min(P, (share + 1) * chunk), q = tid & 3u;
        for (uint32_t i = share * chunk + (tid >> 2); i < i1; i += FILL_WG / 4) {
            const uint32_t o16 = 16u * i - (tail_rank < i ? 16u - tl : 0u);
            if (o16 >= rem) continue;
            const uint32_t len = min(i == tail_rank ? tl : 16u, rem - o16);
            const uint32_t pos = ld_sc1(&order_g[i]), o = cnt + o16 + 4 * q, bi = pos + 4 * q + ioff;
            if (vec && len == 16 && (o16 & 3u) == 0) {
                wire_put4(oidx, oval, STG_WIRE_EMIT ? wflag : 0u, wend, o, bi,
                          reinterpret_cast<const float4 *>(src + (size_t)pos)[q]);
            } else {
                for (uint32_t c = 0; c < 4; ++c) {
                    if (4 * q + c < len) {
                        wire_put(oidx, oval, STG_WIRE_EMIT ? wflag : 0u, wend, o + c, bi + c, src[(size_t)pos + 4 * q + c]);
                    }
                }
            }
        }
        return;
    }
    // the scan launch has finished: every word is final, read them together,
    // with the first PRE window entries (most buckets have fewer) ahead of
    // knowing how many there are
    constexpr uint32_t PRE = LONE ? 10 : 8, PREX = PRE;  // keys / lines and indices prefetched per thread
    constexpr uint32_t KE = LONE ? 10 : 5;                 // emission rounds in flight (> 10: the compiler spills x[])
    const uint32_t *cu = d.cand, *cl = d.cand + CAND_CAP, *ci = d.cand + 2 * CAND_CAP;
    uint32_t pk[PRE], pl[PREX], pc[PREX];
#pragma unroll
    for (uint32_t u = 0; u < PRE; ++u) {
        const uint32_t e = tid + u * FILL_WG;
        pk[u] = ld_sc1(&cu[e]);
        if (u < PREX) {
            pl[u] = ld_sc1(&cl[e]);
            pc[u] = ld_sc1(&ci[e]);
        }
    }
    static_assert(PRE * FILL_WG <= CAND_CAP, "prefetch inside the window buffer");
    const uint64_t w0 = ld_sc1(&D.w[0]), w1 = ld_sc1(&D.w[1]), w2 = ld_sc1(&D.w[2]), w3 = ld_sc1(&D.w[3]);
    const uint32_t failed = ld_sc1(A.fail);
    if ((uint32_t)(w0 >> 32) != ((A.epoch << 8) | TV16_TAG_DEC)) {  // the scan never decided this bucket
        if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(d.count_out, POISON_COUNT); }
        return;
    }
    const uint32_t flags = (uint32_t)w0;
    if (!(flags & TV16_DEC_B) || failed) return;  // regime A, or the launch already failed
    const uint32_t cnt = (uint32_t)(w1 >> 32), M = (uint32_t)w1;
    const uint32_t Wtot = (uint32_t)(w2 >> 32);
    const float tail_key = u2f((uint32_t)w2);
    const uint32_t Qtot = (uint32_t)(w3 >> 32);
    const float t = u2f((uint32_t)w3);
    const bool tail = (flags & TV16_DEC_TAIL) != 0;
    const uint32_t N = d.nb - Qtot + (tail ? 1u : 0u);  // candidate vector length
    const uint32_t rem = d.dst_len - cnt;
    if (!M && !tail) return;
    if (A.crew && crew_wants(flags, M, A.mode)) return;  // a window miss: the crew orders it (tv16wide.h)
    const uint32_t nhelp = LONE ? A.helpers : 0u;
    CallCtl *const ccp = A.cc;
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;
    const bool tail_in = tail && tail_key >= u2f(wlo);
    bool fast = (flags & TV16_DEC_WIN) && N <= POS_LIM && Wtot + (tail_in ? 1u : 0u) > 0 && A.mode != 2u &&
                A.mode != 3u;
    if (!fast && tid == 0) {  // why the literal heap (debug words 60..63)
        if (!(flags & TV16_DEC_WIN)) atomicAdd(&A.dbg[60], 1u);
        if (N > POS_LIM) atomicAdd(&A.dbg[61], 1u);
    }
    uint32_t *const key = S.u.a.key, *const cix = S.u.a.cix;
    // output-order bins over the window below t (sum descending)
    auto kbin = [&](uint32_t kb) -> uint32_t {
        const float k = u2f(kb);
        if (k >= t) return 0u;
        if (!(k > 0.f)) return NBIN - 1;
        return min((tb - 1u - kb) >> 8, NBIN - 1);
    };
    auto okey = [&](uint32_t e) -> uint64_t { return (uint64_t)(~ford(u2f(key[e]))) << 32; };
    auto ksum = [&](uint32_t r) -> float { return u2f(key[S.ord[r]]); };  // sum at rank r
    uint32_t W = 0, Et = NONE;  // entries kept, the ragged tail's element id
    uint32_t *const lines_g = reinterpret_cast<uint32_t *>(d.heap);  // element -> line, for the shadow path
    auto line_of = [&](uint32_t i) { return ld_sc1(&lines_g[S.ord[i]]); };  // after V went over S.u.a.line
    auto line_lds = [&](uint32_t i) { return S.u.a.line[S.ord[i]]; };
    // pops needed for the order in S.ord (entries with an output offset < rem) and the tail's rank
    auto pops = [&](uint32_t &P, uint32_t &tail_rank) {
        for (uint32_t i = tid; i < W; i += FILL_WG)
            if (S.ord[i] == Et) S.flag = i;
        __syncthreads();
        tail_rank = S.flag;
        uint32_t npl = 0;
        for (uint32_t i = tid; i < W; i += FILL_WG) {
            const uint32_t off = 16u * i - (tail_rank < i ? 16u - d.tl : 0u);
            if (off < rem) npl = max(npl, i + 1);
        }
        npl = wave_max(npl);
        if ((tid & 63u) == 0) atomicMax(&S.npop, npl);
        __syncthreads();
        P = S.npop;
    };
    if (tid == 0) { S.flag = NONE; S.nv = 0; S.maxpos = 0; S.npop = 0; S.dmax = 0; S.rn = 0; S.nc = 0; S.nu = 0; S.et = NONE; }
    __syncthreads();
    uint32_t P0 = 0, tail_rank0 = NONE;
    if (fast) {
        // ---- the output order of the top of the window, in one counting
        // sort: bins of 256 ulps below t (sum descending), cut after the first
        // bins that hold M + 2 entries (every pop, the first entry past them
        // and its ties: a bin never splits equal sums), at most EMAX; the
        // window lists up to CAND_CAP.  An entry's id is its slot in the
        // bin-grouped arrays; inside a bin, (sum desc, position asc). ----
        SortScratch &X = S.u.a.s;
        stamp(0);
        for (uint32_t i = tid; i < NBIN; i += FILL_WG) X.bin[i] = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < PRE; ++u)
            if (tid + u * FILL_WG < Wtot) atomicAdd(&X.bin[kbin(pk[u])], 1u);
        for (uint32_t e = tid + PRE * FILL_WG; e < Wtot; e += FILL_WG) atomicAdd(&X.bin[kbin(ld_sc1(&cu[e]))], 1u);
        if (tail_in && tid == 0) atomicAdd(&X.bin[kbin(f2u(tail_key))], 1u);
        __syncthreads();
        stamp(0);
        {
            constexpr uint32_t PER = NBIN / FILL_WG;
            static_assert(PER == 2, "two bins per thread");
            const uint32_t c0 = X.bin[PER * tid], c1 = X.bin[PER * tid + 1], need = M + 2;
            uint32_t tot;
            const uint32_t run = blk_excl_scan<FNW_F>(c0 + c1, S.sh, &tot);
            X.bin[PER * tid] = X.cur[PER * tid] = run;
            X.bin[PER * tid + 1] = X.cur[PER * tid + 1] = run + c0;
            if (run < need && run + c0 >= need) { S.flag = PER * tid + 1; S.nv = run + c0; }
            else if (run + c0 < need && run + c0 + c1 >= need) { S.flag = PER * tid + 2; S.nv = run + c0 + c1; }
            if (tid == 0 && tot < need) { S.flag = NBIN; S.nv = tot; }
            __syncthreads();
        }
        const uint32_t cut = S.flag;  // bins [0, cut) are kept
        W = S.nv;
        fast = W <= EMAX;
        if (!fast && tid == 0) atomicAdd(&A.dbg[62], 1u);
        if (fast) {
            auto keep = [&](uint32_t kb, uint32_t line, uint32_t cx, bool is_tail) {
                const uint32_t e = atomicAdd(&X.cur[kbin(kb)], 1u);
                key[e] = kb;
                S.u.a.line[e] = line;
                cix[e] = cx;
                st_sc1(&lines_g[e], line);
                if (is_tail) S.et = e;
            };
#pragma unroll
            for (uint32_t u = 0; u < PRE; ++u) {
                const uint32_t e = tid + u * FILL_WG;
                if (e >= Wtot || kbin(pk[u]) >= cut) continue;
                if (u < PREX) keep(pk[u], pl[u], pc[u], false);
                else keep(pk[u], ld_sc1(&cl[e]), ld_sc1(&ci[e]), false);
            }
            for (uint32_t e = tid + PRE * FILL_WG; e < Wtot; e += FILL_WG) {
                const uint32_t kb = ld_sc1(&cu[e]);
                if (kbin(kb) < cut) keep(kb, ld_sc1(&cl[e]), ld_sc1(&ci[e]), false);
            }
            if (tail_in && tid == 0 && kbin(f2u(tail_key)) < cut) keep(f2u(tail_key), d.nb * 16, N - 1, true);
            __syncthreads();
            stamp(0);
            for (uint32_t e = tid; e < W; e += FILL_WG) {
                const uint32_t bb = kbin(key[e]), lo = X.bin[bb], hi = X.cur[bb];
                const uint64_t k = okey(e) | cix[e];
                uint32_t r = lo;
                for (uint32_t x = lo; x < hi; ++x) r += (okey(x) | cix[x]) < k;
                S.ord[r] = (uint16_t)e;
            }
        }
        Et = S.et;
        __syncthreads();
        if (tid == 0) { S.flag = NONE; S.nv = 0; }
        __syncthreads();
    }
    if (fast) {
        stamp(0);
        pops(P0, tail_rank0);
        // two of the popped lines (or the last popped and the next) with equal sums?
        uint32_t tie_l = 0;
        for (uint32_t i = tid; i < P0; i += FILL_WG)
            if (i + 1 < W && ksum(i) == ksum(i + 1)) tie_l = 1;
        tie_l = wave_max(tie_l);
        if ((tid & 63u) == 0 && tie_l) S.nv = 1;
        __syncthreads();
        const bool ties = S.nv != 0;
        const uint32_t covered = 16u * W - (Et != NONE ? 16u - d.tl : 0u);
        fast = covered >= rem;
        if (!fast && tid == 0) atomicAdd(&A.dbg[63], 1u);
        if (fast && !ties) {  // distinct sums: the heap pops them in sum order
            emit_all<KE, LONE>(d, cnt, rem, P0, tail_rank0, line_lds, nhelp, ccp, order_g, ready_tag);
            count_path(0);
            stamp(5);
            return;
        }
    }
    if (fast) {
        // ---- the shadow heap (see (1) above) over R = ranks [0, rn): every
        // rank through the first one past the pops, and all that tie with it
        // (reordering a tie can move the tail, and with it the pop count, by one)
        const uint32_t pc = min(P0, W - 1);
        const float kc = ksum(pc);
        for (uint32_t r = tid; r < W; r += FILL_WG)
            if (ksum(r) == kc && (r + 1 == W || ksum(r + 1) != kc)) S.rn = r + 1;
        __syncthreads();
        fast = S.rn < EMAX;  // ranks <= 4094: no content equals CNONE
    }
    if (fast) {
        const uint32_t Rn = S.rn;
        const uint32_t i0 = PT * tid;  // this thread's ranks, then DFS slots
        {   // grp: the first rank of each equal-sum run (run starts listed in order)
            uint32_t stm = 0, nsm = 0;
#pragma unroll
            for (uint32_t u = 0; u < PT; ++u) {
                const uint32_t r = i0 + u;
                if (r < Rn && (r == 0 || ksum(r - 1) != ksum(r))) { stm |= 1u << u; ++nsm; }
            }
            uint32_t tot;
            const uint32_t so = blk_excl_scan<FNW_F>(nsm, S.sh, &tot);
            uint16_t *const starts = S.u.a.s.tmp;
            uint32_t o = so;
#pragma unroll
            for (uint32_t u = 0; u < PT; ++u)
                if (stm >> u & 1u) starts[o++] = (uint16_t)(i0 + u);
            __syncthreads();
            uint32_t c = so;
#pragma unroll
            for (uint32_t u = 0; u < PT; ++u) {
                c += stm >> u & 1u;
                if (i0 + u < Rn) S.grp[i0 + u] = starts[c - 1];
            }
            __syncthreads();  // every sum read is done: dk goes over key
        }
        stamp(0);
        {   // ---- ties without the heap (see (3) above) ----
            if (tid == 0) { S.ntl = 0; S.nel = 0; S.flag2 = 0; }
            __syncthreads();
            const uint32_t lim = N > P0 + 1 ? N - (P0 + 1) : 0u;
            for (uint32_t r = tid; r < Rn; r += FILL_WG) {
                const uint32_t g = S.grp[r];
                if (g <= P0 && (g != r || (r + 1 < Rn && S.grp[r + 1] == g))) {  // tied, and among the pops
                    const uint32_t i = atomicAdd(&S.ntl, 1u);
                    if (i < TCAP) S.tl[i] = (uint16_t)r;
                }
                const uint32_t p = cix[S.ord[r]];
                if (p >= lim) {  // starts among the last P + 1 positions
                    const uint32_t i = atomicAdd(&S.nel, 1u);
                    if (i < ECAP) S.el[i] = p;
                }
            }
            __syncthreads();
            const uint32_t ntl = S.ntl, nel = S.nel;
            stamp(0);
            if (STG_FILL_STAMPS && tid == 0 && b == 0) { A.dbg[40] = W; A.dbg[41] = Rn; A.dbg[42] = ntl; A.dbg[43] = nel; A.dbg[44] = P0; }
            bool bad = ntl > TCAP || nel > ECAP;
            if (!bad) {
                for (uint32_t j = tid; j < ntl; j += FILL_WG) {  // a tied line starting above one of its run
                    const uint32_t tr = S.tl[j], g = S.grp[tr];
                    const uint32_t qt = cix[S.ord[tr]] + 1, dt = depth_of(qt);
                    for (uint32_t x = g; x < Rn && S.grp[x] == g; ++x) {
                        const uint32_t q = cix[S.ord[x]] + 1, dp = depth_of(q);
                        if (x != tr && dp > dt && (q >> (dp - dt)) == qt) bad = true;
                    }
                }
                if (nel) {  // a line of R at the parent or sibling of a late one
                    for (uint32_t r = tid; r < Rn; r += FILL_WG) {
                        const uint32_t p = cix[S.ord[r]];
                        for (uint32_t j = 0; j < nel; ++j) {
                            const uint32_t e = S.el[j];
                            if (e && (p == (e - 1) / 2 || p == (((e - 1) ^ 1u) + 1))) bad = true;
                        }
                    }
                }
            }
            if ((__any(bad) || A.mode == 1u) && (tid & 63u) == 0) S.flag2 = 1;
            __syncthreads();
            stamp(0);
            if (!S.flag2) {
                // each run of equal sums in right-first pre-order of its start positions
                uint16_t *const ord2 = S.u.a.s.tmp;
                for (uint32_t r = tid; r < Rn; r += FILL_WG) {
                    const uint32_t g = S.grp[r], kr = rf_key(cix[S.ord[r]]);
                    uint32_t o = g;
                    for (uint32_t x = g; x < Rn && S.grp[x] == g; ++x) o += rf_key(cix[S.ord[x]]) < kr;
                    ord2[o] = S.ord[r];
                }
                __syncthreads();
                for (uint32_t r = tid; r < Rn; r += FILL_WG) S.ord[r] = ord2[r];
                if (tid == 0) { S.flag = NONE; S.npop = 0; }
                __syncthreads();
                uint32_t P, tail_rank;
                pops(P, tail_rank);
                stamp(0);
                emit_all<KE, LONE>(d, cnt, rem, P, tail_rank, line_lds, nhelp, ccp, order_g, ready_tag);
                count_path(1);
                stamp(0);
                stamp(2);
                return;
            }
        }
        for (uint32_t r = tid; r < Rn; r += FILL_WG) S.u.b.dk[r] = dkey_of_pos(cix[S.ord[r]]);
        __syncthreads();  // cix free: eo goes over it
        // R in DFS order of the start positions
        counting_sort(S.u.b.s, S.u.b.eo, S.sh, Rn, [&](uint32_t r) { return S.u.b.dk[r] >> 15; },
                      [&](uint32_t r) { return (uint64_t)S.u.b.dk[r]; });
        stamp(0);
        // V in pre-order, built by one scan: DFS slot i emits the ancestors of
        // its start at depths L(i-1)+1 .. L(i) (L(i): depth of the lowest common
        // ancestor of slots i and i+1 -- the U nodes, each once), then, when no
        // other element shares its subtree below max(L(i-1), L(i)), its start
        // S_i: the ancestor one deeper, where the element sits after its own
        // subtree's make_heap.  Keys and ranks go to registers first: V is
        // written over dk / eo.
        uint32_t kq[PT + 1], rq[PT];
#pragma unroll
        for (uint32_t u = 0; u <= PT; ++u) kq[u] = i0 + u < Rn ? S.u.b.dk[S.u.b.eo[i0 + u]] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < PT; ++u) rq[u] = i0 + u < Rn ? S.u.b.eo[i0 + u] : 0u;
        const uint32_t kp = (i0 >= 1 && i0 - 1 < Rn) ? S.u.b.dk[S.u.b.eo[i0 - 1]] : 0u;
        auto Lof = [&](uint32_t u) -> int {  // L(i0 + u - 1)
            const uint32_t i = i0 + u;
            return (i >= 1 && i < Rn) ? dk_lca(u ? kq[u - 1] : kp, kq[u]) : -1;
        };
        uint32_t nmine = 0;
#pragma unroll
        for (uint32_t u = 0; u < PT; ++u) {
            if (i0 + u >= Rn) continue;
            const int lo = Lof(u), hi = Lof(u + 1);
            nmine += (uint32_t)max(0, hi - lo) + (max(lo, hi) < (int)dk_depth(kq[u]));
        }
        uint32_t nv;
        uint32_t vo = blk_excl_scan<FNW_F>(nmine, S.sh, &nv);
        fast = nv <= VCAP;
        if (fast) {
            uint32_t *const vk = S.u.v.vk;
            uint2 *const rec = S.u.v.rec;
#pragma unroll
            for (uint32_t u = 0; u < PT; ++u) {
                if (i0 + u >= Rn) continue;
                const int lo = Lof(u), hi = Lof(u + 1);
                const uint32_t k = kq[u], r = rq[u];
                const uint32_t ck = ((uint32_t)S.grp[r] << 12) | r;
                for (int dd = lo + 1; dd <= hi; ++dd, ++vo) {
                    const uint32_t nk = dk_anc(k, (uint32_t)dd);
                    vk[vo] = nk;
                    rec[vo] = r_make(dd == (int)dk_depth(k) ? ck : CNONE, dk_pos(nk), true);
                }
                const int sh = max(lo, hi);
                if (sh < (int)dk_depth(k)) {
                    const uint32_t nk = dk_anc(k, (uint32_t)(sh + 1));
                    vk[vo] = nk;
                    rec[vo] = r_make(ck, dk_pos(nk), false);
                    ++vo;
                }
            }
            if (tid <= NDEP) S.cnt[tid] = 0;
            if (tid == 0) rec[VCAP] = make_uint2(CNONE, 0u);
            __syncthreads();
            // links of the U nodes: the left child follows in pre-order, the
            // right one is found by binary search (four nodes in lockstep, their
            // reads in flight together); U nodes per depth; the deepest U depth
            uint32_t dm = 0;
#pragma unroll
            for (uint32_t g = 0; g < NJ; g += 4) {
                uint32_t lo[4], hi[4], kr[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t v = tid + (g + q) * FILL_WG;
                    lo[q] = hi[q] = kr[q] = 0;
                    if (v < nv && r_isu(rec[v])) {
                        const uint32_t k = vk[v];
                        kr[q] = dk_right(k);
                        lo[q] = v + 1;
                        hi[q] = nv;
                        dm = max(dm, dk_depth(k) + 1);
                        atomicAdd(&S.cnt[dk_depth(k)], 1u);
                    }
                }
                if (!__any(kr[0] | kr[1] | kr[2] | kr[3])) continue;  // no U node of this wave here
                for (uint32_t it = 0; it < 13; ++it) {  // 2^13 > VCAP
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q) {
                        if (lo[q] < hi[q]) {
                            const uint32_t m = (lo[q] + hi[q]) >> 1;
                            if (vk[m] < kr[q]) lo[q] = m + 1; else hi[q] = m;
                        }
                    }
                }
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t v = tid + (g + q) * FILL_WG;
                    if (kr[q]) {
                        const uint32_t k = vk[v];
                        const bool hl = v + 1 < nv && vk[v + 1] == dk_left(k);
                        const bool hr = lo[q] < nv && vk[lo[q]] == kr[q];
                        rec[v].y |= (hr ? lo[q] << 12 : 0u) | (hl ? 1u << 25 : 0u) | (hr ? 1u << 26 : 0u);
                    }
                }
            }
            dm = wave_max(dm);
            if ((tid & 63u) == 0) atomicMax(&S.dmax, dm);
            __syncthreads();
            if (tid == 0) {  // U nodes by depth, deepest first
                uint32_t acc = 0;
                for (int dd = NDEP - 1; dd >= 0; --dd) { S.uoff[dd] = acc; acc += S.cnt[dd]; }
                S.nu = acc;
            }
            __syncthreads();
            if (tid < NDEP) S.cnt[tid] = S.uoff[tid];
            __syncthreads();
            for (uint32_t j = 0; j < NJ; ++j) {  // over vk: every search is done
                const uint32_t v = tid + j * FILL_WG;
                if (v < nv) {
                    const uint2 rc = rec[v];
                    if (r_isu(rc)) S.u.w.ul[atomicAdd(&S.cnt[depth_of(r_pos(rc) + 1)], 1u)] = (uint16_t)v;
                }
            }
            __syncthreads();
            stamp(0);
            // make_heap on V, top-down and pipelined.  __adjust_heap walks the
            // larger-child path (right on ties) to the bottom and pushes the
            // value back up past smaller entries; the path is non-increasing,
            // so that equals swapping the value down while the larger child is
            // >= it.  A U node at depth d starts at step Dm - d: its children's
            // sifts are then one step ahead, their holes two levels below its
            // own, so every node it reads is final and no two sifts of a step
            // touch the same node.  Content order: a smaller grp is a larger
            // sum; CNONE (-inf) has the largest.
            const uint32_t D1 = S.dmax, nU = S.nu;
            if (STG_FILL_STAMPS && tid == 0 && b == 0) {
                A.dbg[40] = W; A.dbg[41] = Rn; A.dbg[42] = nv; A.dbg[43] = D1; A.dbg[44] = P0; A.dbg[46] = nU;
            }
            if (D1) {
                const uint32_t Dm = D1 - 1;
                uint32_t st[NJ];  // hole | start step << 16 (hole NONE13: done)
#pragma unroll
                for (uint32_t j = 0; j < NJ; ++j) {
                    const uint32_t p = tid + j * FILL_WG;
                    st[j] = NONE13;
                    if (p < nU) {
                        const uint32_t v = S.u.w.ul[p];
                        st[j] = v | (Dm - depth_of(r_pos(rec[v]) + 1)) << 16;
                    }
                }
                for (uint32_t tau = 0; tau <= 2 * Dm + 1; ++tau) {
                    // groups of four of this thread's nodes: a group no lane
                    // of the wave has a live sift in is skipped; otherwise
                    // every read of the group is issued at once (missing
                    // nodes read the -inf leaf), then the moves
#pragma unroll
                    for (uint32_t g = 0; g < NJ; g += 4) {
                        bool on[4];
                        uint32_t hs[4];
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q) {
                            on[q] = (st[g + q] & NONE13) != NONE13 && (st[g + q] >> 16) <= tau;
                            hs[q] = on[q] ? (st[g + q] & NONE13) : VCAP;
                        }
                        if (!__any(on[0] || on[1] || on[2] || on[3])) continue;
                        uint2 H[4], La[4], Rb[4];
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q) H[q] = rec[hs[q]];
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q) {
                            La[q] = rec[r_hasl(H[q]) ? hs[q] + 1 : VCAP];
                            Rb[q] = rec[r_hasr(H[q]) ? r_right(H[q]) : VCAP];
                        }
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q) {
                            if (!on[q]) continue;
                            const uint32_t h = hs[q], x = r_content(H[q]);
                            const uint32_t cl = r_content(La[q]), cr = r_content(Rb[q]);
                            const bool left = (cr >> 12) > (cl >> 12);  // right < left
                            const uint32_t cm = left ? cl : cr;
                            if (cm == CNONE || (cm >> 12) > (x >> 12)) {  // the value stays here
                                st[g + q] = NONE13;
                            } else {
                                const uint32_t c = left ? h + 1 : r_right(H[q]);
                                const uint32_t mx = left ? La[q].x : Rb[q].x;
                                rec[h].x = cm | (H[q].x & ~CNONE);
                                rec[c].x = x | (mx & ~CNONE);
                                st[g + q] = (st[g + q] & ~NONE13) | c;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
            stamp(0);
            // final positions (by rank, over ul), the deepest one, and a count of R
            uint32_t mp = 0, nc = 0;
            for (uint32_t j = 0; j < NJ; ++j) {
                const uint32_t v = tid + j * FILL_WG;
                if (v < nv) {
                    const uint2 rc = rec[v];
                    const uint32_t c = r_content(rc);
                    if (c != CNONE) {
                        const uint32_t pos = r_pos(rc);
                        S.u.f.fpos[c & 0xfffu] = pos;
                        mp = max(mp, pos);
                        ++nc;
                    }
                }
            }
            mp = wave_max(mp);
            nc = wave_sum(nc);
            if ((tid & 63u) == 0) { atomicMax(&S.maxpos, mp); atomicAdd(&S.nc, nc); }
            __syncthreads();
            fast = S.nc == Rn;
        }
        if (fast) {
            // equal sums pop in right-first pre-order of their positions (see (2))
            for (uint32_t r = tid; r < Rn; r += FILL_WG) {
                const uint32_t g = S.grp[r], kr = rf_key(S.u.f.fpos[r]);
                uint32_t o = g;
                for (uint32_t x = g; x < Rn && S.grp[x] == g; ++x) o += rf_key(S.u.f.fpos[x]) < kr;
                S.u.f.ord2[o] = S.ord[r];
            }
            __syncthreads();
            for (uint32_t r = tid; r < Rn; r += FILL_WG) S.ord[r] = S.u.f.ord2[r];
            if (tid == 0) { S.flag = NONE; S.npop = 0; }
            __syncthreads();
            uint32_t P, tail_rank;
            pops(P, tail_rank);
            stamp(0);
            if (STG_FILL_STAMPS && tid == 0 && b == 0) A.dbg[45] = P;
            // the pops never reinsert an element of R (see (2) above)
            if (S.maxpos + P < N && P <= Rn) {
                emit_all<KE, LONE>(d, cnt, rem, P, tail_rank, line_of, nhelp, ccp, order_g, ready_tag);
                count_path(2);
                stamp(1);
                return;
            }
            fast = false;
        }
    }
    __syncthreads();
    // the leader (tv16wide.h) over the window list, when the window holds the
    // top min(P0 + 2, N) candidates (the ragged tail joins as an entry)
    if ((flags & TV16_DEC_WIN) && A.mode != 2u) {
        const uint32_t P0 = (rem + 15u) / 16u, seln = min(P0 + 1u, N - 1u);
        if (Wtot >= seln + 1u || Wtot + (tail ? 1u : 0u) == N) {
            WideLds &Wl = *reinterpret_cast<WideLds *>(fill_lds);
            LeadIn I;
            I.lk = cu;
            I.lp = cl;
            I.lc = ci;
            I.n = Wtot;
            I.tail = tail ? 1u : 0u;
            I.tail_bits = f2u(tail_key);
            I.N = N;
            I.nb = d.nb;
            I.rem = rem;
            I.tl = d.tl;
            I.g = reinterpret_cast<uint32_t *>(d.heap);
            I.dbg = A.dbg;
            I.lvl1 = NONE;
            I.r1 = 0;
            I.gcap = 2u * (d.nb + 64u);
            I.positions = true;
            const LeadOut O = leader(Wl, I);
            if (O.ok) {
                const uint32_t *const opos = O.ordpos;
                emit_all<KE, LONE>(d, cnt, rem, O.P, O.tail_rank, [&](uint32_t i) { return ld_sc1(&opos[i]); }, nhelp,
                                   ccp, order_g, ready_tag);
                if (tid == 0) atomicAdd(&A.dbg[52], 1u);
                return;
            }
            if (tid == 0) atomicAdd(&A.dbg[54], 1u);
            __syncthreads();
        }
    }
    if (tid == 0) { S.flag = NONE; S.npop = 0; }
    __syncthreads();
    stamp(3);
    count_path(3);
    // the literal heap emits everything itself: release the helpers before it
    // runs (an empty share each), so none of them waits out its length
    if (LONE && A.helpers && tid == 0) {
        st_sc1(&A.cc->pad[2], 0u);
        __builtin_amdgcn_s_waitcnt(0);
        st_sc1(&A.cc->pad[1], ready_tag);
    }
    full_path(S, d, cnt, N, t, tail, tail_key, A.fail);
    stamp(0);
}

}  // namespace

constexpr size_t LFIN_LDS = std::max(std::max(sizeof(FillLds), sizeof(LfinLds)), sizeof(WideLdsBig));
static_assert(LFIN_LDS <= 160 * 1024, "one lfin workgroup per CU");

#if STG_WIRE_EMIT
hipError_t launch_tv16_fill_wire(const Tv16FillArgs &a, hipStream_t s) {
#else
hipError_t launch_tv16_fill(const Tv16FillArgs &a, hipStream_t s) {
#endif
    if (!a.nbk) return hipSuccess;
    static const hipError_t attr0 =
        hipFuncSetAttribute(reinterpret_cast<const void *>(&tv16_fill<false>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(FillLds));
    static const hipError_t attr1 =
        hipFuncSetAttribute(reinterpret_cast<const void *>(&tv16_fill<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)LFIN_LDS);
    if (attr0 != hipSuccess) return attr0;
    if (attr1 != hipSuccess) return attr1;
    if (a.lfin) tv16_fill<true><<<a.workers + a.rankers + a.crew, FILL_WG, LFIN_LDS, s>>>(a);
    else if (a.lone) tv16_fill<true><<<a.nbk + a.helpers + a.crew, FILL_WG, sizeof(FillLds), s>>>(a);
    else tv16_fill<false><<<a.nbk + a.crew, FILL_WG, sizeof(FillLds), s>>>(a);
    return hipGetLastError();
}

}  // namespace stg
