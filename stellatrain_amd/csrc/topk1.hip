// topk1.hip -- Top-k by |x| in one pass over the bucket, steered by the key's
// previous k-th magnitude (gfx950).
//
// Reference: TopkCompressor::impl_nth_element (compress/topk.cpp:28-46); the
// two modes and their semantics are topk.hip's (the shipped byte-count memcpy
// and slot indices, or the intended operator), emitted in index order with
// ties at the k-th magnitude T taken in index order.
//
// compress() carries the tensor's name (compressor.h:30), and a gradient's
// magnitude distribution moves little from one call to the next, so the key's
// last T (KeyState.t; the band's relative half width d in KeyState.inc) fixes
// a band [F, H) = T_prev (1 -/+ d), at most TK2_FINE ulps wide, that almost
// always holds this call's T.  Two launches:
//   tk2_stream  one workgroup per 32 KiB tile: the tile's superset
//               {|x| >= F} (in index order) into region tile % 32 at an offset
//               taken by one atomic; its count of keys >= H; every band key
//               into the band histogram, one bin per ulp (and a coarse one per
//               256 ulps).  One read of the bucket.
//   tk_one      every workgroup finds T exactly from the histograms (the
//               count above H, the coarse bins, one coarse bin's 256 ulps: T
//               is a bin), then as one of the NU emission units (up to 16
//               tiles, units in ticket order) counts its supersets' (> T,
//               == T) keys, publishes them, sums the earlier units' (look-back)
//               and writes its winners in order.
// (The same finish inside the stream launch, by its first NU workgroups,
// measured 26.5 / 37.5 us per shipped / exact C2 call against 24.4 / 35.0 and
// was removed in round 6.)
// A band that misses T, or a superset region that overflowed, takes the
// select's way inside tk_one (three radix levels over the bucket, per-tile
// counts, emission re-reading the tiles; units by sharded tickets, every
// single-unit phase run by the workgroup that completes the phase before it)
// and the band widens for the next call.  A key's first call runs topk.hip's
// launches and seeds the hint (tk2_seed).
//
// No unit is waited on before a running workgroup holds it (tickets), and
// every wait is bounded: a wait that gives up sets the failure word and
// poisons the count.
#include <algorithm>
#include <cstdlib>

#include "select.h"
#include "tile.h"
#include "tv16_dev.h"

namespace stg {

namespace {

using tv16::spin_expired;
using tv16::vm_drain;

#ifndef STG_TK1_STAMPS
#define STG_TK1_STAMPS 0  // diagnostics: phase times (100 MHz clock) into debug words 40..47
#endif
#define TK1_STAMP(w)                                                                                  \
    do {                                                                                              \
        if (STG_TK1_STAMPS && threadIdx.x == 0) A.dbg[w] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
// ... the latest over the workgroups
#define TK1_STAMP_MAX(w)                                                                              \
    do {                                                                                              \
        if (STG_TK1_STAMPS && threadIdx.x == 0)                                                       \
            atomicMax(&A.dbg[w], (uint32_t)__builtin_amdgcn_s_memrealtime());                         \
    } while (0)

enum : uint32_t { M_H1 = 0, M_P1, M_H2, M_P2, M_H3, M_P3, M_CNT, M_SCAN, P_EMIT, NPH };
static_assert(NPH == TK1_NPH, "phases");

constexpr float D_MIN = 1.0f / 1024.0f;  // the band's relative half width d: narrowest
constexpr float D_MAX = 1.0f / 128.0f;   // ... widest (2 d T_prev < TK2_FINE ulps)
constexpr float D_SEED = 1.0f / 256.0f;  // ... after a key's first call

__device__ __forceinline__ uint32_t mag1(uint32_t bits) { return bits & 0x7fffffffu; }

// Coarse bin c's word: bins interleaved over 64 lines of 16 words (c mod 64
// picks the line), so the few dozen bins a narrow band covers sit on as many
// lines -- consecutive bins on one 128-byte line serialise every tile's band
// atomics at that line.
__device__ __forceinline__ uint32_t coarse_word(uint32_t c) { return (c & 63u) * 16u + (c >> 6); }
static_assert(TK2_COARSE == 1024, "64 lines x 16 words");

// The band of this call from the key's hint: [F, H) in key bits, at most
// TK2_FINE wide (centred on T_prev when d T_prev spans more ulps); ok = false
// for a hint that cannot steer (zero, denormal, inf or NaN).
struct Band {
    uint32_t F, H;
    bool ok;
};
__device__ __forceinline__ Band band_of(const KeyState *st) {
    const float t = st->t, d = st->inc;
    const uint32_t tb = mag1(f2u(t));
    Band b;
    b.ok = st->init && tb >= 0x00800000u && tb < 0x7f800000u;
    b.F = mag1(f2u(t * (1.0f - d)));
    b.H = mag1(f2u(t * (1.0f + d)));
    if (b.H <= b.F) b.H = b.F + 1u;
    if (b.H - b.F > TK2_FINE) {
        b.F = tb - TK2_FINE / 2u;
        b.H = b.F + TK2_FINE;
    }
    return b;
}

// ---------------------------------------------------------------------------
// the emission launch
// ---------------------------------------------------------------------------
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
    TopkCtl *ctl, *ctl_next;
    uint32_t tag;          // >= 1
    RSel *rs;              // the select's way
    uint2 *sup;            // the stream launch's superset regions
    uint32_t shard_cap;
    uint32_t *sup_n, *sup_off;
    uint32_t *tile_gt, *tile_eq;  // the select's way: counts [0, nt), prefixes [nt, 2nt), totals [2nt]
    uint32_t *fine;        // this call's band histogram
    uint32_t *fine_next;   // the other parity's (the stream launch zeroes what the previous call touched)
    uint32_t *dbg;         // ws.misc: [38] calls resolved in the band, [39] calls that took the select's way
    uint32_t ut;           // tiles per emission unit (<= TK2_UT): about ER STG_WG superset entries
    bool withhold;         // tests (STG_DEBUG_TK_WITHHOLD=1): unit 0 never publishes its counts, so every
                           // later unit's look-back runs out its bound: the failure path end to end
    bool fixed;            // tile t's superset at slot t / TK2_REG of its region (no offset atomic)
};

constexpr uint32_t ER = 8;  // superset entries per thread per emission round

struct T1Ldf {  // the band's way (pick and emission units)
    uint32_t s_wt[TILE_U * STG_WAVES + 1];
    uint32_t sh[STG_WAVES + 1];
    uint64_t sh64[STG_WAVES];
    uint32_t uc[TK2_UT], uo[TK2_UT], up[TK2_UT + 1], ub[TK2_UT];  // emission unit: per tile count, offset, flat start, base
    uint32_t v[16];
};
struct T1Lds : T1Ldf {
    uint32_t h[2048];       // a select level's tile histogram
};

// Loads of what the stream launch wrote: plain after the kernel boundary
// (tk_one), sc1 inside the stream launch (its finish: the writers stored sc1)
template <bool COH>
__device__ __forceinline__ uint32_t ldw(const uint32_t *p) {
    if constexpr (COH) return ld_sc1(p);
    else return *p;
}
template <bool COH>
__device__ __forceinline__ uint2 ldw(const uint2 *p) {
    if constexpr (COH) {
        const uint64_t w = ld_sc1(reinterpret_cast<const uint64_t *>(p));
        return make_uint2((uint32_t)w, (uint32_t)(w >> 32));
    } else {
        return *p;
    }
}

// shard s of a phase with U units holds units s, s + 8, ...
__device__ __forceinline__ uint32_t shard_units(uint32_t U, uint32_t s) { return U > s ? (U - s + TK1_SH - 1) / TK1_SH : 0u; }

__device__ __forceinline__ void t1_broken(const T1Args &A) {
    g_or(A.fail, FAIL_SELECT);
    __hip_atomic_fetch_max(gp(A.count_out), POISON_COUNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// T exactly from the stream launch's histograms, by every workgroup (a few
// KiB from L2; no workgroup waits for another): the count above H, the coarse
// bins top-down, then the 256 one-ulp bins of T's coarse bin.  Returns hit.
struct Pick {
    uint32_t T, gt;  // T; keys > T
};
// (COH: inlined into the stream launch, which makes no calls -- a kernel that
// calls a function is also given the LDS of every kernel whose variables a
// called function might reach: tk_one's 17 KiB; tk_one calls the plain copies)
template <bool COH>
__device__ __forceinline__ bool pick_exact(const T1Args &A, T1Ldf &L, Pick &P) {
    const uint32_t tid = threadIdx.x;
    const TopkCtl *const C = A.ctl;
    // tk_one: plain loads (written by the stream launch, a kernel boundary,
    // read by every workgroup -- cached in each XCD's L2, where coherent loads
    // of the same few lines by 512 workgroups queue at the memory side)
    const uint32_t ok = ldw<COH>(&C->band_ok), ovf = ldw<COH>(&C->ovf), F = ldw<COH>(&C->band_F);
    constexpr uint32_t PER = TK2_COARSE / STG_WG;
    uint32_t c[PER], s = 0, hi = tid < TK2_HI ? ldw<COH>(&C->hi[tid][0]) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {  // top-down: thread tid holds coarse bins 1023 - (PER tid + j)
        const uint32_t cw = coarse_word(TK2_COARSE - 1u - (PER * tid + j));
        c[j] = 0;
#pragma unroll
        for (uint32_t sh = 0; sh < TK2_CSHARDS; ++sh) c[j] += ldw<COH>(&C->coarse[sh][cw]);
        s += c[j];
    }
    uint32_t th, tband;
    (void)blk_excl_scan<STG_WAVES>(hi, L.sh, &th);
    if (tid == 0) L.v[2] = 0xffffffffu;
    uint32_t above = blk_excl_scan<STG_WAVES>(s, L.sh, &tband);
    const uint32_t r = A.k - 1u;  // T's descending rank
    const bool hit = ok && !ovf && th <= r && r - th < tband;
    if (!__syncthreads_or((int)hit)) return false;  // (uniform)
    const uint32_t rr = r - th;
    // the emission unit's tile counts and offsets (emit_unit), loaded beside
    // the fine bins: the ticket (L.v[9], taken before the pick) is back by now
    const uint32_t u = L.v[9], t0 = u * A.ut;
    const bool pre = t0 < A.nt && tid < std::min(A.ut, A.nt - t0);
    uint32_t pc = 0, po = 0;
    if (pre) {
        pc = ldw<COH>(&A.sup_n[t0 + tid]);
        po = ldw<COH>(&A.sup_off[t0 + tid]);
    }
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (above <= rr && rr < above + c[j]) { L.v[2] = TK2_COARSE - 1u - (PER * tid + j); L.v[3] = rr - above; }
        above += c[j];
    }
    __syncthreads();
    const uint32_t cb = L.v[2], rc = L.v[3];
    const uint32_t f = ldw<COH>(&A.fine[(cb << TK2_CSH) + (1u << TK2_CSH) - 1u - tid]);  // top-down
    static_assert((1u << TK2_CSH) == STG_WG, "one fine bin per thread");
    if (pre) {  // (after the fine load is issued: its round trip overlaps theirs)
        L.uc[tid] = pc;
        L.uo[tid] = po;
    }
    if (tid == 0) L.v[4] = 0xffffffffu;
    uint32_t tot;
    const uint32_t fa = blk_excl_scan<STG_WAVES>(f, L.sh, &tot);
    if (f && fa <= rc && rc < fa + f) { L.v[4] = (1u << TK2_CSH) - 1u - tid; L.v[5] = fa; }
    __syncthreads();
    if (L.v[4] == 0xffffffffu) return false;  // the bins disagree (cannot happen): the select's way
    P.T = F + (cb << TK2_CSH) + L.v[4];
    P.gt = th + (r - th - rc) + L.v[5];  // above H, the coarse bins above T's, T's bin's ulps above T
    __syncthreads();
    return true;
}

// One emission unit: tiles [u UT, u UT + UT).  Counts the (> T, == T) keys of
// their supersets, publishes them, sums the earlier units' (look-back: units
// are taken in ticket order, so each is held by a running or finished
// workgroup) and writes the winners at their offsets.  Returns false when a
// wait gave up.  `pre`: the tiles' counts and offsets are in L.uc / L.uo
// already (pick_exact loads them).  `get(T, need_eq)` supplies T once the
// unit's first round of entries is in flight (the stream launch's finishers
// wait for the pick there): > 0 go on, 0 skip the unit, < 0 a wait gave up.
// Returns 1 emitted, 0 skipped, -1 a wait gave up.
template <bool COH, class GetT>
__device__ __forceinline__ int emit_unit(const T1Args &A, T1Ldf &L, uint32_t u, GetT get, bool pre) {
    const uint32_t tid = threadIdx.x, nt = A.nt;
    const uint32_t UT = A.ut, t0 = u * UT, nT = std::min(UT, nt - t0);
    if (!pre) {
        if (tid < nT) {
            L.uc[tid] = ldw<COH>(&A.sup_n[t0 + tid]);
            L.uo[tid] = ldw<COH>(&A.sup_off[t0 + tid]);
        }
        __syncthreads();
    }
    if (tid < 64) {  // the tiles' flat starts: one wave scans the counts
        const uint32_t c = tid < nT ? L.uc[tid] : 0u, o = tid < nT ? L.uo[tid] : 0u;
        const uint32_t incl = wave_incl_scan(c), ex = incl - c;
        const bool bad = tid < nT && (c > TV_TILE || o + c > A.shard_cap);
        if (tid <= TK2_UT) L.up[tid] = tid < nT ? ex : 0xffffffffu;
        // entry f of tile j is at sup[ub[j] + f] (mod 2^32: the true index is < 2^32)
        if (tid < nT) L.ub[tid] = ((t0 + tid) % TK2_REG) * A.shard_cap + o - ex;
        const uint32_t tot = __shfl(incl, (int)nT - 1, 64);
        if (tid == nT) L.up[tid] = tot;
        const uint64_t b = __ballot(bad);
        if (tid == 0) L.v[11] = b ? 1u : 0u;
    }
    __syncthreads();
    // A bad count or offset cannot follow a pick that hit (the stream launch
    // wrote every tile's; an overflowing tile marks the call ovf, a miss).
    // The stream launch's finishers get here before they know the pick, so
    // the verdict waits for it.
    const bool broken = L.v[11] != 0;
    const uint32_t N = broken ? 0u : L.up[nT];
    // the tiles' flat starts in scalar registers: entry f's tile is the count of
    // starts (after the first) at or below f -- no branch, so a round's loads
    // are all issued before any is waited for
    uint32_t st1[TK2_UT - 1];
#pragma unroll
    for (uint32_t t = 1; t < TK2_UT; ++t) st1[t - 1] = tv16::uni(t < nT ? L.up[t] : 0xffffffffu);
    auto ld = [&](uint32_t f) -> uint2 {
        uint32_t j = 0;
#pragma unroll
        for (uint32_t t = 0; t + 1 < TK2_UT; ++t) j += st1[t] <= f ? 1u : 0u;
        return ldw<COH>(&A.sup[L.ub[j] + f]);
    };
    uint2 e[ER];
    auto load_round = [&](uint32_t b0) {
#pragma unroll
        for (uint32_t r = 0; r < ER; ++r) {
            const uint32_t f = b0 + ER * tid + r;
            e[r] = ld(std::min(f, N ? N - 1u : 0u));
        }
    };
    if (N) load_round(0);
    uint32_t T;
    uint64_t need_eq;
    const int g = get(T, need_eq);  // (uniform)
    if (g <= 0) return g;
    if (broken) {
        if (tid == 0) t1_broken(A);
        return 1;
    }
    // counts
    uint32_t gt = 0, eq = 0;
    for (uint32_t b0 = 0; b0 < N; b0 += ER * STG_WG) {
        if (b0) load_round(b0);
#pragma unroll
        for (uint32_t r = 0; r < ER; ++r) {
            const uint32_t key = mag1(e[r].y);
            const bool in = b0 + ER * tid + r < N;
            gt += in && key > T;
            eq += in && key == T;
        }
    }
    uint32_t GT, EQ;
    (void)blk_excl_scan<STG_WAVES>(gt, L.sh, &GT);
    (void)blk_excl_scan<STG_WAVES>(eq, L.sh, &EQ);
    TopkCtl *const C = A.ctl;
    TK1_STAMP_MAX(46);  // the last unit counted
    if (tid == 0 && !(A.withhold && u == 0)) st_sc1(&C->udesc[u], ((uint64_t)(GT | 0x80000000u) << 32) | EQ);
    // look-back: the earlier units' counts, one thread per unit
    uint64_t pg = 0, pe = 0;
    uint32_t bad = 0;
    for (uint32_t i = tid; i < u; i += STG_WG) {
        uint64_t w = ld_sc1(&C->udesc[i]);
        uint64_t st = 0;
        for (uint32_t sp = 0; !(w >> 63); ++sp) {
            __builtin_amdgcn_s_sleep(2);
            w = ld_sc1(&C->udesc[i]);
            if (spin_expired(sp, st)) { bad = 1; break; }
        }
        pg += (w >> 32) & 0x7fffffffu;
        pe += (uint32_t)w;
    }
    if (__syncthreads_or((int)bad)) return -1;
    TK1_STAMP_MAX(47);  // the last look-back done
    const uint64_t gt_before = blk_sum64<STG_WAVES>(pg, L.sh64), eq_before = blk_sum64<STG_WAVES>(pe, L.sh64);
    if (!(GT || (EQ && eq_before < need_eq))) return 1;
    // emission: > T always, == T in index order while fewer than need_eq came before
    uint64_t wbase = gt_before + std::min(eq_before, need_eq), ebase = eq_before;
    for (uint32_t b0 = 0; b0 < N; b0 += ER * STG_WG) {
        if (N > ER * STG_WG) load_round(b0);  // (one round: still in registers)
        uint32_t qg = 0, qe = 0;
#pragma unroll
        for (uint32_t r = 0; r < ER; ++r) {
            const uint32_t key = mag1(e[r].y);
            const bool in = b0 + ER * tid + r < N;
            qg |= (in && key > T) ? 1u << r : 0u;
            qe |= (in && key == T) ? 1u << r : 0u;
        }
        uint32_t te, tw;
        uint32_t er = blk_excl_scan<STG_WAVES>((uint32_t)__popc(qe), L.sh, &te);
        uint32_t qw = qg;
#pragma unroll
        for (uint32_t r = 0; r < ER; ++r)
            if ((qe >> r) & 1u) { if (ebase + er < need_eq) qw |= 1u << r; ++er; }
        uint32_t wr = blk_excl_scan<STG_WAVES>((uint32_t)__popc(qw), L.sh, &tw);
#pragma unroll
        for (uint32_t r = 0; r < ER; ++r) {
            if ((qw >> r) & 1u) {
                const uint64_t slot = wbase + wr++;
                if (slot >= A.k) { t1_broken(A); continue; }
                A.idx[slot] = A.bug_compat ? (uint32_t)slot : e[r].x + (uint32_t)A.idx_offset;
                A.val[slot] = u2f(e[r].y);
            }
        }
        wbase += tw;
        ebase += te;
    }
    return 1;
}

__device__ __noinline__ bool pick_exact_call(const T1Args &A, T1Ldf &L, Pick &P) { return pick_exact<false>(A, L, P); }
// false: a wait gave up
__device__ __noinline__ bool emit_unit_call(const T1Args &A, T1Ldf &L, uint32_t u, uint32_t T, uint64_t need_eq) {
    auto known = [&](uint32_t &t, uint64_t &ne) -> int { t = T; ne = need_eq; return 1; };
    return emit_unit<false>(A, L, u, known, true) >= 0;
}

// ---------------------------------------------------------------------------
// the stream launch
// ---------------------------------------------------------------------------

// One workgroup per tile.  Before its tile, each zeroes its share of the
// previous hinted call's control block (from its second line on) and of the
// fine bins that call's band touched (ctl_next keeps the band: [0, H - F)).
// Seven waves per SIMD (eight: 64 VGPRs with spills, measured slower in round 4).
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) __attribute__((amdgpu_waves_per_eu(7, 8))) tk2_stream(const T1Args A) {
    __shared__ T1Ldf L;
    __shared__ uint32_t s_off, s_hi;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, tile = blockIdx.x, nt = A.nt;
    const Band B = band_of(A.state);
    const size_t base = (size_t)tile * TV_TILE, m = A.m;
    float4 v[TILE_U];
    if (B.ok) load_tile<VEC>(A.a, m, base, A.last_mask, v);
    auto zero_prev = [&]() {
        const TopkCtl *const cn = A.ctl_next;
        const uint32_t span = cn->band_ok ? std::min(cn->band_H - cn->band_F, TK2_FINE) : 0u;
        constexpr uint32_t CW = (uint32_t)((sizeof(TopkCtl) - 4u * TK1_LINE) / 16u);
        uint4 *const c4 = reinterpret_cast<uint4 *>(reinterpret_cast<char *>(A.ctl_next) + 4u * TK1_LINE);
        uint4 *const f4 = reinterpret_cast<uint4 *>(A.fine_next);
        for (uint32_t i = tile * STG_WG + tid, n = CW + (span + 3u) / 4u; i < n; i += nt * STG_WG) {
            if (i < CW) c4[i] = make_uint4(0u, 0u, 0u, 0u);
            else f4[i - CW] = make_uint4(0u, 0u, 0u, 0u);
        }
    };
    zero_prev();
    if (!B.ok) {  // tk_one takes the select's way: this call's block says so
        // (its first line is never zeroed, so it would still hold the band of
        // the hinted call two calls back)
        if (tile == 0 && tid == 0) st_sc1(&A.ctl->band_ok, 0u);
        return;
    }
    if (tile == 0) TK1_STAMP(40);  // the stream launch's first workgroup starts
    TopkCtl *const C = A.ctl;
    if (tile == 0 && tid == 0) {
        st_sc1(A.count_out, A.cap);  // the band's way fills every slot; a failure poisons it (atomicMax)
        st_sc1(&C->band_F, B.F);
        st_sc1(&C->band_H, B.H);
        st_sc1(&C->band_ok, 1u);
    }
    if (tid == 0) s_hi = 0;
    uint32_t q = 0, pre[TILE_U], nhi = 0;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t key = mag1(f2u(comp(v[u], j)));
            if (e + j < m && key >= B.F) {
                q |= 1u << (u * 4 + j);
                if (key >= B.H) {
                    ++nhi;
                } else {
                    const uint32_t f = key - B.F;
                    __hip_atomic_fetch_add(gp(&A.fine[f]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    // (TK2_CSHARDS copies: every tile's band atomics on 64 lines serialised there)
                    __hip_atomic_fetch_add(gp(&C->coarse[tile % TK2_CSHARDS][coarse_word(f >> TK2_CSH)]), 1u,
                                           __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        const uint32_t c = (uint32_t)__popc((q >> (4 * u)) & 0xfu);
        const uint32_t incl = wave_incl_scan(c);
        pre[u] = incl - c;
        if (lane == 63) L.s_wt[u * STG_WAVES + wave] = incl;
    }
    nhi = wave_sum(nhi);
    __syncthreads();
    if (lane == 0 && nhi) atomicAdd(&s_hi, nhi);
    if (tid < 64) {  // (u, wave) offsets: one wave scans the 32 counts
        constexpr uint32_t NW = TILE_U * STG_WAVES;
        static_assert(NW <= 64, "one wave scans the wave counts");
        const uint32_t x = tid < NW ? L.s_wt[tid] : 0u;
        const uint32_t inc = wave_incl_scan(x);
        if (tid < NW) L.s_wt[tid] = inc - x;
        if (tid == NW - 1) L.s_wt[NW] = inc;
    }
    __syncthreads();
    const uint32_t nsup = L.s_wt[TILE_U * STG_WAVES], sh = tile % TK2_REG;
    // sc1 stores throughout: the finishing workgroups of this launch read them
    if (tid == 0) {
        uint32_t off = 0;
        if (nsup && A.fixed) {  // TOPK_SUP_CAP entries of the region per tile; more: the select's way
            off = tile / TK2_REG * TOPK_SUP_CAP;
            if (nsup > TOPK_SUP_CAP) st_sc1(&C->ovf, 1u);
        } else if (nsup) {
            off = g_add(&C->shn[sh][0], nsup);
            if (off + nsup > A.shard_cap) st_sc1(&C->ovf, 1u);
        }
        s_off = off;
        st_sc1(&A.sup_n[tile], nsup);
        st_sc1(&A.sup_off[tile], off);
        if (s_hi) g_add(&C->hi[tile % TK2_HI][0], s_hi);
    }
    __syncthreads();
    const uint32_t off = s_off;
    if (nsup && off + nsup <= A.shard_cap && !(A.fixed && nsup > TOPK_SUP_CAP)) {
        uint64_t *const dst = reinterpret_cast<uint64_t *>(A.sup) + (size_t)sh * A.shard_cap + off;
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
            uint32_t slot = L.s_wt[u * STG_WAVES + wave] + pre[u];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((q >> (u * 4 + j)) & 1u) {
                    const uint64_t w = (uint64_t)f2u(comp(v[u], j)) << 32 | (uint32_t)(e + j);
                    // sc1 (write-through) stores even without the finish in this
                    // launch: plain ones measured 29.5 / 49.7 us per shipped / exact
                    // call and 15 / 55 MB written per call, against 24.5 / 35.3 us and
                    // 7.1 / 8.1 MB (profiles/r05_pmc_topk*_hinted.json)
                    st_sc1(&dst[slot++], w);
                }
        }
    }
}

// A key's first call ran topk.hip's launches: T (rs->prefix) seeds the hint.
__global__ void tk2_seed(KeyState *st, const RSel *rs, uint32_t *dbg) {
    st->t = u2f(rs->prefix);
    st->inc = D_SEED;
    st->init = 1;
    atomicAdd(&dbg[39], 1u);  // a call that took the select's way
}

// A select level's histogram over one tile (the keys under the prefix).
template <bool VEC, int SHIFT, int NBITS>
__device__ __noinline__ void unit_hist(const T1Args &A, T1Lds &L, uint32_t tile) {
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t NB = 1u << NBITS;
    for (uint32_t i = tid; i < NB; i += STG_WG) L.h[i] = 0;
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
            if (e + j < A.m && (key & mask) == prefix) atomicAdd(&L.h[(key >> SHIFT) & (NB - 1u)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < NB; i += STG_WG)
        if (L.h[i]) g_add(&A.rs->hist[tile % RS_SHARDS][i], L.h[i]);
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

// EMIT (the select's way): the tile's winners (> T, then == T in index order
// until k) at their prefix offsets, from the tile itself.
template <bool VEC>
__device__ __noinline__ void unit_emit(const T1Args &A, T1Lds &L, uint32_t tile, uint32_t T, uint64_t need_eq) {
    const uint32_t tid = threadIdx.x, nt = A.nt;
    const uint32_t cg = ld_sc1(&A.tile_gt[tile]), ce = ld_sc1(&A.tile_eq[tile]);
    const uint64_t gt_before = ld_sc1(&A.tile_gt[nt + tile]), eq_before = ld_sc1(&A.tile_eq[nt + tile]);
    if (!(cg || (ce && eq_before < need_eq))) return;
    const uint64_t win_before = gt_before + std::min(eq_before, need_eq);
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

// the count, then the failure word again: a select_broken (fail bit, then
// POISON_COUNT) that came before the second read is seen there and poisoned
// here; one that came after it stores its poison after ours
__device__ __forceinline__ void write_count(const T1Args &A) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        if (!(ld_sc1(A.fail) & FAIL_SELECT)) {
            st_sc1(A.count_out, A.cap);
            __builtin_amdgcn_s_waitcnt(0);
            if (ld_sc1(A.fail) & FAIL_SELECT) st_sc1(A.count_out, POISON_COUNT);
        }
    }
}

// 2 workgroups per CU at least (<= 128 VGPRs); each phase body is its own
// function within that budget
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) __attribute__((amdgpu_waves_per_eu(4, 8))) tk_one(T1Args Ak) {
    __shared__ T1Lds L;
    // the arguments in LDS: the phase bodies take them by reference (a
    // reference to the kernel's argument block would be copied to scratch)
    __shared__ T1Args A;
    const uint32_t tid = threadIdx.x;
    // the argument block into LDS field by field: `A = Ak` compiled to a private
    // copy of the whole block, stored to scratch by every thread of every
    // workgroup before anything else (~10 MB a launch, ~15 us)
    if (tid == 0) {
        A.a = Ak.a; A.m = Ak.m; A.zeros = Ak.zeros; A.last_mask = Ak.last_mask; A.nt = Ak.nt; A.k = Ak.k;
        A.cap = Ak.cap; A.idx_offset = Ak.idx_offset; A.bug_compat = Ak.bug_compat; A.idx = Ak.idx; A.val = Ak.val;
        A.count_out = Ak.count_out; A.fail = Ak.fail; A.state = Ak.state; A.ctl = Ak.ctl; A.ctl_next = Ak.ctl_next;
        A.tag = Ak.tag; A.rs = Ak.rs; A.sup = Ak.sup; A.shard_cap = Ak.shard_cap; A.sup_n = Ak.sup_n;
        A.sup_off = Ak.sup_off; A.tile_gt = Ak.tile_gt; A.tile_eq = Ak.tile_eq; A.fine = Ak.fine;
        A.fine_next = Ak.fine_next; A.dbg = Ak.dbg; A.ut = Ak.ut;
        A.withhold = Ak.withhold; A.fixed = Ak.fixed;
    }
    __syncthreads();
    TopkCtl *const C = A.ctl;
    if (blockIdx.x == 0) TK1_STAMP(40);
    const uint32_t home = blockIdx.x % TK1_SH;
    auto poison = [&]() {
        if (tid == 0) {
            g_or(A.fail, FAIL_SPIN_TIMEOUT);
            __hip_atomic_fetch_max(gp(A.count_out), POISON_COUNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // the band's way
    Pick P;
    // the hit path's NU emission units: the first NU workgroups take one
    // ticket each (units in ticket order), issued before the pick so its
    // round trip overlaps the pick's loads
    const uint32_t NU = (A.nt + A.ut - 1u) / A.ut;
    if (tid == 0) L.v[9] = blockIdx.x < NU ? g_add(&C->utk[0], 1u) : NU;
    const bool hit = pick_exact_call(A, L, P);
    if (blockIdx.x == 0) TK1_STAMP(42);  // workgroup 0: pick done
    TK1_STAMP_MAX(43);                   // every workgroup's pick done
    if (hit) {
        if (blockIdx.x == 0 && tid == 0) {  // the next call's hint; the band narrows while T keeps landing near T_prev
            const float Tp = A.state->t, d = A.state->inc, Tf = u2f(P.T);
            A.state->t = Tf;
            A.state->inc = fabsf(Tf - Tp) < 0.25f * d * Tp ? fmaxf(0.75f * d, D_MIN) : fminf(d, D_MAX);
            atomicAdd(&A.dbg[38], 1u);
        }
        const uint64_t need_eq = (uint64_t)A.k - P.gt;
        __syncthreads();
        const uint32_t u = L.v[9];
        __syncthreads();
        if (u < NU) {
            TK1_STAMP_MAX(48);  // the last unit taken
            if (!emit_unit_call(A, L, u, P.T, need_eq)) { poison(); return; }
            TK1_STAMP_MAX(44);  // the last unit done
        }
        TK1_STAMP_MAX(45);      // the last workgroup out
        return;
    }
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
        if (p == M_H1) {
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
                if (!A.state->init) {
                    A.state->inc = D_SEED;
                } else if (ld_sc1(&C->band_ok)) {
                    // a hinted call missed.  T outside [F, H): widen the band.
                    // T inside it, but a superset overflowed its slots
                    // (magnitudes dense near F): narrow it, since a wider band
                    // would only admit more entries next call
                    const bool in = ld_sc1(&C->band_F) <= T && T < ld_sc1(&C->band_H);
                    A.state->inc = in ? fmaxf(0.5f * A.state->inc, D_MIN) : fminf(2.0f * A.state->inc, D_MAX);
                }
                A.state->init = 1;
            }
        } else if (p == M_CNT) {
            scan_tiles1(A.tile_gt, A.tile_eq, A.nt, L.sh);
        }
        vm_drain();
        __syncthreads();
        if (tid == 0) st_sc1(&C->flag[p + 1], A.tag);
    };
    // one multi-unit phase: take units until every shard is empty; the
    // workgroup completing the phase also runs the single-unit phase after it
    auto run_multi = [&](uint32_t p, uint32_t T, uint64_t need_eq) {
        const uint32_t U = A.nt, nsh = min(U, TK1_SH);
        for (uint32_t si = 0; si < TK1_SH; ++si) {
            const uint32_t s = (home + si) % TK1_SH, su = shard_units(U, s);
            for (;;) {
                if (tid == 0)  // a plain look first: an empty shard costs no atomic
                    L.v[9] = ld_sc1(&C->tk[p][s][0]) >= su ? su : g_add(&C->tk[p][s][0], 1u);
                __syncthreads();
                const uint32_t c = L.v[9];
                if (c >= su) { __syncthreads(); break; }  // uniform: c is read from LDS after a barrier
                const uint32_t tile = s + TK1_SH * c;
                if (p == M_H1) unit_hist<VEC, 20, 11>(A, L, tile);
                else if (p == M_H2) unit_hist<VEC, 9, 11>(A, L, tile);
                else if (p == M_H3) unit_hist<VEC, 0, 9>(A, L, tile);
                else if (p == M_CNT) unit_count<VEC>(A, L, tile);
                else unit_emit<VEC>(A, L, tile, T, need_eq);
                vm_drain();
                __syncthreads();
                if (tid == 0) {
                    uint32_t last = 0;
                    if (g_add(&C->done[p][s][0], 1u) + 1u == su && g_add(&C->sdone[p][0], 1u) + 1u == nsh) last = 1;
                    L.v[10] = last;
                }
                __syncthreads();
                if (L.v[10]) {
                    if (p == P_EMIT) write_count(A);
                    else run_single(p);
                }
                __syncthreads();
            }
        }
    };
    const uint32_t seq[4] = {M_H1, M_H2, M_H3, M_CNT};
    for (uint32_t i = 0; i < 4; ++i) {
        run_multi(seq[i], 0, 0);
        if (!wait_flag(seq[i] + 1u)) { poison(); return; }
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
    run_multi(P_EMIT, T, need_eq);
}

}  // namespace

hipError_t launch_topk1(const TopkLaunch &a, const DevWS &ws, KeyState *state, bool hinted, uint32_t *tagp,
                        hipStream_t s) {
    // k == 0 (topk.cpp accepts it: nothing selected, returns cap) takes the
    // select's launcher, which writes the count alone; no hint is seeded
    if (a.k == 0 || a.n == 0) return launch_topk(a, ws, s);
    uint64_t m = a.n, zeros = 0;
    uint32_t last_mask = 0xffffffffu;
    if (a.bug_compat) {  // memcpy(clone, src, n) copies n bytes (topk.cpp:31)
        m = a.n / 4 + (a.n % 4 ? 1 : 0);
        if (a.n % 4) last_mask = (1u << (8 * (a.n % 4))) - 1u;
        zeros = a.n - m;
    }
    const uint32_t nt = (uint32_t)((m + TV_TILE - 1) / TV_TILE);
    if (nt > TOPK_LIST_TILES) return hipErrorInvalidValue;
    if (!hinted) {  // a key's first call: the select's launches, then the hint
        hipError_t e = launch_topk(a, ws, s);
        if (e != hipSuccess) return e;
        tk2_seed<<<1, 1, 0, s>>>(state, ws.rsel, ws.misc);
        return hipGetLastError();
    }
    // The control block and band histogram alternate by the tag's parity: each
    // stream launch zeroes what the previous hinted call used of the other
    // parity's copies.  So the tag moves only here, and always to the other parity
    // (0 is never a tag: 0xffffffff is followed by 2).  A launch error leaves
    // both copies in an unknown state; they are zeroed on the stream.
    const uint32_t tag = *tagp + 1u == 0u ? 2u : *tagp + 1u;
    *tagp = tag;
    auto reset_ctl = [&](hipError_t e) {
        (void)hipMemsetAsync(ws.tkctl, 0, 2 * sizeof(TopkCtl), s);
        (void)hipMemsetAsync(ws.tkfine, 0, 2 * (size_t)TK2_FINE * sizeof(uint32_t), s);
        return e;
    };
    TopkCtl *const ctl = ws.tkctl + (tag & 1u);
    uint32_t *const fine = ws.tkfine + (size_t)(tag & 1u) * TK2_FINE;
    // superset regions: the bucket's share of TOPK_SUP_CAP entries per tile, in TK2_REG regions
    // Fixed slots when k is at most 1/16 of the keys (a tile's superset, ~k / nt
    // entries plus the band, stays well under TOPK_SUP_CAP = TV_TILE / 8);
    // denser calls take region offsets by atomics, so that a region's 32
    // tiles share its space.  Fixed: C2 33.6 -> 33.1 us.
    const bool fixed = (uint64_t)std::min<uint64_t>(a.k, m) * 16u <= m;
    const uint32_t shard_cap = fixed ? (nt + TK2_REG - 1) / TK2_REG * TOPK_SUP_CAP
                                     : (uint32_t)((size_t)nt * TOPK_SUP_CAP / TK2_REG);
    uint32_t *const sup_n = ws.tile_cnt + 2 * (size_t)nt + 1, *const sup_off = ws.tile_aux + 2 * (size_t)nt + 1;
    uint2 *const sup = reinterpret_cast<uint2 *>(ws.sums);
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
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
    A.ctl = ctl;
    A.ctl_next = ws.tkctl + ((tag + 1u) & 1u);
    A.tag = tag;
    A.rs = ws.rsel;
    A.sup = sup;
    A.shard_cap = shard_cap;
    A.sup_n = sup_n;
    A.sup_off = sup_off;
    A.tile_gt = ws.tile_cnt;
    A.tile_eq = ws.tile_aux;
    A.fine = fine;
    // a unit's superset (~ k / nt entries per tile): about `per_unit` entries,
    // so that the units spread over the CUs
    constexpr uint64_t per_unit = (uint64_t)ER * STG_WG * 3 / 4;
    A.ut = (uint32_t)std::max<uint64_t>((nt + TK2_UNITS - 1) / TK2_UNITS,
                                        std::min<uint64_t>(TK2_UT, per_unit * nt / std::max<uint64_t>(A.k, 1)));
    A.ut = std::max(1u, std::min(A.ut, TK2_UT));
    A.fine_next = ws.tkfine + (size_t)((tag + 1u) & 1u) * TK2_FINE;
    A.dbg = ws.misc;
    A.fixed = fixed;
    const uint32_t NU = (nt + A.ut - 1u) / A.ut;
    static const bool withhold = getenv("STG_DEBUG_TK_WITHHOLD") && atoi(getenv("STG_DEBUG_TK_WITHHOLD")) == 1;
    A.withhold = withhold;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    if (vec) tk2_stream<true><<<nt, STG_WG, 0, s>>>(A);
    else tk2_stream<false><<<nt, STG_WG, 0, s>>>(A);
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    // every emission unit has a workgroup of its own (NU <= TK2_UNITS)
    const uint32_t G = std::max<uint32_t>(std::min<uint32_t>(nt, (uint32_t)a.num_cu * 2u), NU);
    if (vec) tk_one<true><<<G, STG_WG, 0, s>>>(A);
    else tk_one<false><<<G, STG_WG, 0, s>>>(A);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? e : reset_ctl(e);
}

}  // namespace stg
